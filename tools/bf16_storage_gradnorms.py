"""Where a bf16 training step's per-parameter gradient-norm deviations come from (CPU, test infrastructure):
the oracle's Model-B / Model-A fixture step (fp32 restatement of the reference) three ways against the fixture's
fp32 gradient norms --
  storage   every activation AND gradient an op produces rounded to bf16 (tests/_fixtures.Bf16Storage: what any
            bf16-storage implementation, ours included, does -- parameters unrounded, fp32 arithmetic);
  autocast  torch.autocast("cpu", bf16) -- the reference's own bf16 path: matmul / conv outputs bf16, while
            LayerNorm / BatchNorm outputs and every residual sum x + branch are promoted back to fp32;
  recorded  the reference's own CPU-autocast run recorded in the fixture (make_golden.py r3).
Prints the relative deviation of the listed parameters and the worst / RMS over all parameters.
    python tools/bf16_storage_gradnorms.py [model_b_train_b16] [param ...]"""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in (ROOT / "tests", ROOT / "tests" / "golden", ROOT / "oracle"):
    sys.path.insert(0, str(p))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import _fixtures as fx  # noqa: E402
import gen_params as gp  # noqa: E402
import ogv_oracle as orc  # noqa: E402


class _Except(fx.Bf16Storage):
    """Bf16Storage, except the outputs of the listed aten ops stay fp32."""
    def __init__(self, keep):
        super().__init__()
        self.keep = keep

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        if any(k in str(func) for k in self.keep):
            return func(*args, **(kwargs or {}))
        return super().__torch_dispatch__(func, types, args, kwargs)


class _Logits32(fx.Bf16Storage):
    """Bf16Storage, except the Outlooker logits stay fp32 (the attn 1x1 conv's [B, 9h, H, W] output and the
    [B, L, h, 9] tensors of its softmax): what a kernel keeping the logit columns of cat in fp32 would do."""
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))

        def rnd(t):
            if isinstance(t, torch.Tensor) and t.dtype == torch.float32 and t.ndim >= 1 and t.numel() > 1:
                if t.shape[-1] == 9 or ("convolution.default" in str(func) and t.ndim == 4 and t.shape[1] % 9 == 0
                                        and t.shape[1] <= 72):
                    return t
                return t.to(torch.bfloat16).to(torch.float32)
            return t
        return torch.utils._pytree.tree_map(rnd, out)


VARIANTS = {  # storage variants: aten ops whose outputs stay fp32
    "st_add32": ("aten.add.",),                                  # residual sums (and other adds)
    "st_norm32": ("native_layer_norm", "native_batch_norm"),     # normalisation outputs (+ their backward)
    "st_conv32": ("convolution", "aten.addmm", "aten.mm", "aten.bmm"),   # GEMM / conv outputs and their gradients
    "st_cfwd32": ("aten.convolution.default", "aten.addmm"),    # conv / Linear forward outputs only
    "st_cbwd32": ("convolution_backward", "aten.mm"),           # conv / Linear gradient outputs only
}


def grad_norms(meta, arr, mode):
    st = meta["stages"]
    if meta["kind"] == "model_b":
        shapes = orc.model_b_shapes(st, meta["num_classes"], 3, meta["stem_dim"], meta["outlooker_front_depth"])
        fwd = lambda x, p: orc.model_b(x, p, st, meta["outlooker_front_depth"], train=meta["mode"] == "train")  # noqa: E731
    else:
        shapes = orc.model_a_shapes(st, meta["num_classes"], 3, meta["stem_dim"])
        fwd = lambda x, p: orc.model_a(x, p, st, train=meta["mode"] == "train")  # noqa: E731
    p = orc.make_params(shapes, lambda k, s: gp.param_value(k, s, meta["seed"]))
    x = torch.from_numpy(gp.input_from_spec(meta["x"]))
    y = torch.from_numpy(arr["targets"])
    if mode in ("storage", "st_logits32") or mode in VARIANTS:
        with (fx.Bf16Storage() if mode == "storage" else _Logits32() if mode == "st_logits32" else _Except(VARIANTS[mode])):
            logits = fwd(x.to(torch.bfloat16).float(), p)
            loss = F.cross_entropy(logits.float(), y, label_smoothing=0.1)
            loss.backward()
    elif mode == "autocast":
        with torch.autocast("cpu", dtype=torch.bfloat16):
            logits = fwd(x, p)
        loss = F.cross_entropy(logits.float(), y, label_smoothing=0.1)
        loss.backward()
    else:
        logits = fwd(x, p)
        loss = F.cross_entropy(logits.float(), y, label_smoothing=0.1)
        loss.backward()
    return {k: (float(v.grad.norm()) if v.grad is not None else 0.0) for k, v in p.items()
            if torch.is_tensor(v) and v.is_floating_point() and v.requires_grad}


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "model_b_train_b16"
    focus = sys.argv[2:] or ["front.2.attn.attn.bias", "front.1.attn.attn.bias", "front.0.attn.attn.bias"]
    meta, arr = fx.load(name)
    names = meta["param_names"]
    ref = np.asarray(arr["grad_norms"], dtype=np.float64)
    floor = 1e-3 * np.abs(ref).max()
    cols = {"recorded": np.asarray(arr["grad_norms_cpu_bf16_autocast"], dtype=np.float64)}
    torch.set_num_threads(8)
    for mode in ("fp32", "storage", "autocast") + tuple(VARIANTS) + ("st_logits32",):
        g = grad_norms(meta, arr, mode)
        cols[mode] = np.array([g[k] for k in names])
    print(f"{name}: relative grad-norm deviation from the fixture's fp32 norms")
    print(f"{'parameter':40s} " + " ".join(f"{m:>10s}" for m in cols))
    rel = {m: np.abs(v - ref) / (np.abs(ref) + floor) for m, v in cols.items()}
    for k in focus:
        i = names.index(k)
        print(f"{k:40s} " + " ".join(f"{rel[m][i]:10.4f}" for m in cols))
    for m in cols:
        w = int(np.argmax(rel[m]))
        print(f"{m:10s} worst {rel[m][w]:.4f} ({names[w]}), RMS {float(np.sqrt(np.mean(rel[m] ** 2))):.4f}")


if __name__ == "__main__":
    main()
