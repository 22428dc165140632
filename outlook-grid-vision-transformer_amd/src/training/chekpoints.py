"""Drop-in for src/training/chekpoints.py:1-40 — the same checkpoint dict
{"model", "optimizer", "scheduler", "scaler", "epoch", "best_top1", "extra"}, so files written by
the reference load here and vice versa (parameter/buffer names match the reference state_dict).

Loading uses torch.load(weights_only=True): a checkpoint holds tensors, numbers, strings and
containers only, and nothing in it is executed.  Tensors are mapped to `map_location` and then
copied into the (device-resident) modules by load_state_dict.  The optimizer state goes through
ogv.train.load_optimizer_state: a fused / capturable AdamW keeps its flags and its device lr
tensors (a saved float lr is copied into them), and existing moment tensors are overwritten in
place, so a hipGraph recorded over the optimizer stays valid after a resume.
"""
import torch


def save_checkpoint(path: str, model, optimizer, scheduler, scaler, epoch: int, best_top1: float,
                    extra: dict | None = None):
    core = model.module if hasattr(model, "module") else model
    # cloned: the Outlooker's v / attn tensors are views into one padded buffer (_AliasedConcat), and
    # torch.save of shared-storage views writes that whole buffer
    ckpt = {
        "model": {k: v.detach().clone() for k, v in core.state_dict().items()},
        "optimizer": optimizer.state_dict() if optimizer is not None else None,
        "scheduler": scheduler.state_dict() if scheduler is not None else None,
        "scaler": scaler.state_dict() if scaler is not None else None,
        "epoch": epoch,
        "best_top1": best_top1,
        "extra": extra or {},
    }
    torch.save(ckpt, path)


def load_checkpoint(path: str, model, optimizer=None, scheduler=None, scaler=None, map_location="cpu",
                    strict: bool = True):
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    core = model.module if hasattr(model, "module") else model
    core.load_state_dict(ckpt["model"], strict=strict)
    if optimizer is not None and ckpt.get("optimizer") is not None:
        from ogv.train import load_optimizer_state
        load_optimizer_state(optimizer, ckpt["optimizer"])
    if scheduler is not None and ckpt.get("scheduler") is not None:
        scheduler.load_state_dict(ckpt["scheduler"])
    if scaler is not None and ckpt.get("scaler") is not None:
        scaler.load_state_dict(ckpt["scaler"])
    return ckpt
