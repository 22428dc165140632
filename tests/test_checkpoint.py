"""Checkpoint format (src/training/chekpoints.py:1-40): the drop-in writes the reference's dict and
reads one written the reference's way (same keys, same state_dict names).  CPU only: modules are
constructed on the host, no kernel runs."""
import torch

import _fixtures as fx
import gen_params as gp


def _model_b():
    import test_gpu_parity as tg
    meta, _ = fx.load("model_b_eval_b2")
    m = tg._module(meta)
    gp.fill_module(m, meta["seed"])
    return m


def test_roundtrip_and_reference_layout(tmp_path):
    from src.training.chekpoints import load_checkpoint, save_checkpoint
    m = _model_b()
    opt = torch.optim.AdamW(m.parameters(), lr=5e-4)
    for p in m.parameters():
        p.grad = torch.ones_like(p)
    opt.step()
    sched = torch.optim.lr_scheduler.StepLR(opt, 10)
    path = tmp_path / "last.pt"
    save_checkpoint(str(path), m, opt, sched, None, epoch=3, best_top1=41.5, extra={"note": "x"})
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert set(ck) == {"model", "optimizer", "scheduler", "scaler", "epoch", "best_top1", "extra"}
    assert list(ck["model"]) == [k for k, _ in _model_b().state_dict().items()]
    assert list(ck["model"]) == list(fx.shapes_for(fx.load("model_b_eval_b2")[0]))   # the reference's names

    m2 = _model_b()
    with torch.no_grad():
        for p in m2.parameters():
            p.zero_()
    opt2 = torch.optim.AdamW(m2.parameters(), lr=5e-4)
    sched2 = torch.optim.lr_scheduler.StepLR(opt2, 10)
    got = load_checkpoint(str(path), m2, opt2, sched2, None)
    assert got["epoch"] == 3 and got["best_top1"] == 41.5 and got["extra"] == {"note": "x"}
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
    assert opt2.state_dict()["state"][0]["step"] == opt.state_dict()["state"][0]["step"]


def test_reads_a_reference_style_checkpoint(tmp_path):
    """A dict saved exactly as the reference's save_checkpoint builds it (plain torch.save)."""
    from src.training.chekpoints import load_checkpoint
    m = _model_b()
    path = tmp_path / "best.pt"
    torch.save({"model": m.state_dict(), "optimizer": None, "scheduler": None, "scaler": None, "epoch": 7,
                "best_top1": 12.0, "extra": {}}, path)
    m2 = _model_b()
    with torch.no_grad():
        for p in m2.parameters():
            p.add_(1.0)
    ck = load_checkpoint(str(path), m2)
    assert ck["epoch"] == 7
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
