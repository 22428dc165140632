"""Child process of tests/test_gpu_train.py::test_rccl_world1_dp_path_matches_single_process (GPU box
only): a world-size-1 RCCL ("nccl") process group and the Trainer's data-parallel path on it, against
the single-process Trainer.  Prints one JSON line per mode; the parent asserts on them."""
import json
import os
import pathlib
import socket
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in (ROOT / "outlook-grid-vision-transformer_amd", ROOT / "tests", ROOT / "tests" / "golden"):
    sys.path.insert(0, str(p))

with socket.socket() as sk:     # env rendezvous on 127.0.0.1, set before anything touches the GPU
    sk.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    import ogv
    from ogv.train import MODEL_CONFIGS, Trainer, build_model
    ogv.load()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    print(json.dumps({"stage": "init", "backend": dist.get_backend()}), flush=True)
    cfg = MODEL_CONFIGS["model_a_7m"]
    batches = []
    for i in range(4):
        g = torch.Generator(device="cuda").manual_seed(90 + i)
        batches.append((torch.randn(16, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last),
                        torch.randint(0, 100, (16,), device="cuda", generator=g)))
    runs = {}
    for mode in ("plain", "dp_graph", "dp_graph_flat", "dp_capture", "plain_eager", "dp_eager", "dp_graph_fallback",
                 "dp_graph_other_error"):
        torch.backends.cudnn.benchmark = False
        torch.manual_seed(31)
        m = build_model(dict(type="model_a", num_classes=100, stem_dim=64, dpr_max=0.0, stages=cfg["stages"]))
        m = m.cuda().to(memory_format=torch.channels_last)
        dp = mode.startswith("dp")
        t = Trainer(m, total_steps=50, warmup_ratio=0.1, graphs=not mode.endswith("eager"), capture_warmup=1,
                    force_dp=dp, dp_capture_collective=mode == "dp_capture", dp_overlap=mode != "dp_graph_flat")
        assert t.dp == dp and t.dp_capture_collective == (mode == "dp_capture")
        assert t.dp_overlap == (mode in ("dp_graph", "dp_graph_fallback", "dp_graph_other_error")), (mode, t.dp_overlap)
        if mode == "dp_graph_fallback":   # a runtime that refuses to record the collectives: the capture raises
            def refuse(*a, **k):
                raise RuntimeError("simulated: operation not permitted when stream is capturing")
            t._fwd_bwd_overlap = refuse
        if mode == "dp_graph_other_error":   # any other failure (here: OOM) is re-raised on every rank, no fallback
            def oom(*a, **k):
                raise RuntimeError("simulated: HIP out of memory")
            t._fwd_bwd_overlap = oom
            try:
                for b in batches:
                    t.step(*b)
                raised = ""
            except RuntimeError as e:
                raised = str(e)
            print(json.dumps({"mode": mode, "backend": t.backend, "raised": raised, "dp_overlap": t.dp_overlap}),
                  flush=True)
            del t
            continue
        warned = []
        import warnings
        with warnings.catch_warnings(record=True) as wl:
            warnings.simplefilter("always")
            losses = [t.step(*b).float().item() for b in batches]     # eager, capture, replay, replay
            warned = [str(w.message) for w in wl if "bucketed all-reduces failed" in str(w.message)]
        torch.cuda.synchronize()
        state = [p.detach().clone() for p in m.parameters()] + [b.detach().clone() for b in m.buffers()]
        runs[mode] = (losses, state)
        out = {"mode": mode, "backend": t.backend, "losses": losses, "graphs": t.graphs, "dp_overlap": t.dp_overlap,
               "fallback_warned": len(warned)}
        if t.dp_overlap:     # the reduced gradients the optimizer read are the parameters' .grad
            out["buckets"] = len(t._gbuckets)
            out["grad_is_view"] = all(p.grad.data_ptr() == v.data_ptr() for p, v in zip(t.params, t._gviews))
        for ref in ("plain", "plain_eager"):
            if ref in runs and ref != mode:
                out["max_param_diff_vs_" + ref] = max(float((a.double() - b.double()).abs().max())
                                                      for a, b in zip(state, runs[ref][1]) if a.is_floating_point())
        print(json.dumps(out), flush=True)
        del t
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print(json.dumps({"stage": "done"}), flush=True)


if __name__ == "__main__":
    main()
