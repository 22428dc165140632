"""Data-parallel step (ogv.train.Trainer, world_size 2, gloo on CPU).

The DP path is model-agnostic: rank-0 broadcast of parameters/buffers at start, fwd+bwd per rank,
one all_reduce of a flat gradient bucket pre-divided by world size, then clip + AdamW.  With equal
per-rank batches that is exactly one single-process step on the concatenated batch, which is what
these tests check (on a small CPU model: the OutGridBlock kernels themselves are HIP-only).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from ogv.train import Trainer

STEPS = 3


def _model(seed):
    torch.manual_seed(seed)
    m = nn.Sequential(nn.Linear(8, 16), nn.BatchNorm1d(16), nn.GELU(), nn.Linear(16, 5))
    return m


def _data():
    g = torch.Generator().manual_seed(123)
    return torch.randn(STEPS, 8, 8, generator=g), torch.randint(0, 5, (STEPS, 8), generator=g)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = _model(seed=0 if rank == 0 else 99)   # rank 1 starts different: broadcast must fix it
        tr = Trainer(model, amp_dtype=None, total_steps=10, warmup_ratio=0.0)
        assert tr.world == world
        X, Y = _data()
        per = X.shape[1] // world
        for t in range(STEPS):
            # BatchNorm in eval: per-rank batch statistics would otherwise (legitimately) differ from
            # the full-batch ones; the DP contract under test is the gradient exchange
            model.eval()
            tr.step(X[t, rank * per:(rank + 1) * per], Y[t, rank * per:(rank + 1) * per])
        torch.save([p.detach().clone() for p in model.parameters()], os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _single():
    model = _model(seed=0)
    tr = Trainer(model, amp_dtype=None, total_steps=10, warmup_ratio=0.0)
    assert tr.world == 1
    X, Y = _data()
    for t in range(STEPS):
        model.eval()
        tr.step(X[t], Y[t])
    return [p.detach().clone() for p in model.parameters()]


@pytest.mark.timeout(300)
def test_dp_world2_matches_single_process(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    ref = _single()
    for a, b, c in zip(r0, r1, ref):
        assert torch.equal(a, b), "ranks diverged"
        torch.testing.assert_close(a, c, rtol=1e-5, atol=1e-6)


def test_flat_bucket_roundtrip():
    """_flatten / _unflatten are exact inverses (world 1 arithmetic, no process group)."""
    model = _model(seed=3)
    tr = Trainer(model, amp_dtype=None)
    tr.world = 2
    tr._sizes = [p.numel() for p in tr.params]
    tr.flat = torch.zeros(sum(tr._sizes))
    g0 = [torch.randn_like(p) for p in tr.params]
    for p, g in zip(tr.params, g0):
        p.grad = g.clone()
    tr._flatten()
    assert tr.flat.numel() == sum(p.numel() for p in tr.params)
    tr.flat.mul_(2.0)           # what a 2-rank all_reduce of identical buckets would give
    tr._unflatten()
    for p, g in zip(tr.params, g0):
        torch.testing.assert_close(p.grad, g, rtol=0, atol=0)
