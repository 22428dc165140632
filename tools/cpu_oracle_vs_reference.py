"""CPU baseline fairness check (build container only: it imports the reference from /root/reference):
the oracle's training step (oracle/ogv_oracle.py train_step, what bench.py's cpu_baseline times) against
the REFERENCE'S OWN step (src/training/one_epoch_train.py train_one_epoch on one batch, fp32, with the
AdamW / param groups of src/training/train_full_model.py:56-66 and its WarmupCosineLR) on the same cores,
same model (Model-A-7M), same batch size, interleaved samples.
    python tools/cpu_oracle_vs_reference.py [--threads 8] [--bs 64] [--seconds 6] [--reps 3]"""
import argparse
import os
import pathlib
import statistics
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
REF = pathlib.Path(os.environ.get("OGV_REFERENCE", "/root/reference"))
for p in (ROOT / "oracle", ROOT / "tests" / "golden"):
    sys.path.insert(0, str(p))
sys.path.insert(0, str(REF))     # the reference's src/ (this repo's package also has a src/: not on the path here)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--bs", type=int, default=64)
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    import gen_params as gp
    import ogv_oracle as orc
    from make_golden import STAGES_7M
    cfg = dict(stages=STAGES_7M, num_classes=100, stem_dim=64, dpr_max=0.07)   # configs/cifar100_model_a_7m.yaml
    from src.Model_A_OutGridNet import MaxOutNet
    from src.stage_config import StageCfg
    from src.training.one_epoch_train import train_one_epoch
    from src.training.warmup import WarmupCosineLR, build_param_groups_no_wd

    g = torch.Generator().manual_seed(7)
    x = torch.randn(a.bs, 3, 32, 32, generator=g)
    y = torch.randint(0, 100, (a.bs,), generator=g)
    # the oracle, as bench.py cpu_baseline runs it
    p = orc.make_params(orc.model_a_shapes(cfg["stages"], cfg["num_classes"], 3, cfg["stem_dim"]),
                        lambda k, s: gp.param_value(k, s, 7))
    opt_o = orc.make_optimizer(p)
    oracle_step = lambda: orc.train_step(x, y, p, cfg["stages"], opt_o)  # noqa: E731
    # the reference's own step (dpr 0.07 as configs/cifar100_model_a_7m.yaml; DropPath active in train mode)
    m = MaxOutNet(num_classes=100, stages=[StageCfg(**s) for s in cfg["stages"]], in_ch=3, stem_dim=64,
                  dpr_max=cfg["dpr_max"])
    gp.fill_module(m, 7)
    opt_r = torch.optim.AdamW(build_param_groups_no_wd(m, weight_decay=0.05), lr=5e-4, betas=(0.9, 0.999), eps=1e-8)
    sched = WarmupCosineLR(opt_r, total_steps=10_000, warmup_steps=500, min_lr=1e-6)
    ref_step = lambda: train_one_epoch(m, [(x, y)], opt_r, sched, device="cpu", use_amp=False,  # noqa: E731
                                       grad_clip_norm=1.0, label_smoothing=0.1, num_classes=100, print_every=0)
    res = {"oracle": [], "reference": []}
    for fn in (oracle_step, ref_step):
        for _ in range(2):
            fn()
    for _ in range(a.reps):
        for name, fn in (("oracle", oracle_step), ("reference", ref_step)):
            n, t0 = 0, time.perf_counter()
            while True:
                fn()
                n += 1
                if time.perf_counter() - t0 > a.seconds:
                    break
            res[name].append(n * a.bs / (time.perf_counter() - t0))
    med = {k: statistics.median(v) for k, v in res.items()}
    print(f"threads {a.threads} (host CPUs {os.cpu_count()}), bs {a.bs}, {a.reps} interleaved samples of ~{a.seconds:.0f} s:")
    for k, v in res.items():
        print(f"  {k:9s} median {med[k]:7.2f} imgs/s  samples {[round(s, 2) for s in v]}")
    print(f"  oracle / reference = {med['oracle'] / med['reference']:.3f}")


if __name__ == "__main__":
    main()
