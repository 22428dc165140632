"""Diagnostic (GPU box): graph-mode DP with the bucketed overlapped collectives (Trainer dp_overlap) vs the
single-process Trainer on a world-size-1 RCCL group -- per step, which gradients / parameters differ.
    python tools/diag_dp_overlap.py"""
import os
import pathlib
import socket
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "outlook-grid-vision-transformer_amd"))
with socket.socket() as sk:
    sk.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    import ogv
    from ogv.train import MODEL_CONFIGS, Trainer, build_model
    ogv.load()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    cfg = MODEL_CONFIGS["model_a_7m"]
    batches = []
    for i in range(4):
        g = torch.Generator(device="cuda").manual_seed(90 + i)
        batches.append((torch.randn(16, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last),
                        torch.randint(0, 100, (16,), device="cuda", generator=g)))
    tr = {}
    for mode in ("plain", "dp"):
        torch.manual_seed(31)
        m = build_model(dict(type="model_a", num_classes=100, stem_dim=64, dpr_max=0.0, stages=cfg["stages"]))
        m = m.cuda().to(memory_format=torch.channels_last)
        tr[mode] = (m, Trainer(m, total_steps=50, warmup_ratio=0.1, graphs=True, capture_warmup=1, force_dp=mode == "dp"))
    names = [n for n, _ in tr["plain"][0].named_parameters()]
    for step, b in enumerate(batches):
        for mode in ("plain", "dp"):
            tr[mode][1].step(*b)
        torch.cuda.synchronize()
        tp, td = tr["plain"][1], tr["dp"][1]
        gp = tp.graph_grads if tp._g is not None else [p.grad for p in tp.params]
        gd = [p.grad for p in td.params]
        worst = []
        for n, a, c, pa, pd in zip(names, gp, gd, tp.params, td.params):
            dg = (a.double() - c.double()).abs().max().item() if a is not None and c is not None else -1
            dpp = (pa.double() - pd.double()).abs().max().item()
            if dg or dpp:
                worst.append((n, dg, dpp, tuple(a.stride()) if a is not None else None,
                              tuple(c.stride()) if c is not None else None, tuple(pa.stride())))
        print(f"step {step}: {len(worst)} params differ; graph={td._g is not None} overlap={td.dp_overlap}")
        for w in worst[:12]:
            print("   ", w)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
