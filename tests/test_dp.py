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


def _worker(rank, world, port, out_dir, bucket_mb=8.0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = _model(seed=0 if rank == 0 else 99)   # rank 1 starts different: broadcast must fix it
        tr = Trainer(model, amp_dtype=None, total_steps=10, warmup_ratio=0.0, bucket_mb=bucket_mb)
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
@pytest.mark.parametrize("bucket_mb", [8.0, 0.0, 1e-4])
def test_dp_world2_matches_single_process(tmp_path, bucket_mb):
    """One bucket (8 MB), the single flat bucket (0), and ~1 parameter per bucket (1e-4 MB: the
    asynchronous all_reduces overlap the rest of backward) all equal the single-process step."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), bucket_mb), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    ref = _single()
    for a, b, c in zip(r0, r1, ref):
        assert torch.equal(a, b), "ranks diverged"
        torch.testing.assert_close(a, c, rtol=1e-5, atol=1e-6)


def _bn_worker(rank, world, port, out_dir, bucket_mb):
    """Train-mode BatchNorm on different per-rank shards: after every step each rank holds rank 0's
    running statistics (DDP broadcast_buffers), and rank 0's equal a lone process on its shard."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = _model(seed=0)
        tr = Trainer(model, amp_dtype=None, total_steps=10, warmup_ratio=0.0, bucket_mb=bucket_mb)
        X, Y = _data()
        per = X.shape[1] // world
        rms = []
        for t in range(STEPS):
            model.train()
            tr.step(X[t, rank * per:(rank + 1) * per], Y[t, rank * per:(rank + 1) * per])
            rms.append(model[1].running_mean.clone())
        torch.save(rms, os.path.join(out_dir, f"bn{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bucket_mb", [8.0, 0.0])
def test_dp_broadcasts_bn_buffers_from_rank0(tmp_path, bucket_mb):
    world = 2
    mp.spawn(_bn_worker, args=(world, _free_port(), str(tmp_path), bucket_mb), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "bn0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "bn1.pt", weights_only=True)
    for a, b in zip(r0, r1):
        assert torch.equal(a, b), "running statistics differ across ranks"
    # step 1 starts from identical (zero) running means, so rank 0's value is its own shard's update
    model = _model(seed=0).train()
    X, _ = _data()
    with torch.no_grad():
        model(X[0, :X.shape[1] // world])
    torch.testing.assert_close(r0[0], model[1].running_mean, rtol=1e-6, atol=1e-7)
    assert not torch.equal(r0[0], r0[1])


def _nan_worker(rank, world, port, out_dir):
    """A non-finite loss on ONE rank makes every rank skip the step (the flag rides in the
    all_reduce), leaving parameters and optimizer state unchanged on both."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = _model(seed=0)
        tr = Trainer(model, amp_dtype=None, total_steps=10, warmup_ratio=0.0)
        X, Y = _data()
        model.eval()
        tr.step(X[0, rank * 4:(rank + 1) * 4], Y[0, rank * 4:(rank + 1) * 4])
        before = [p.detach().clone() for p in model.parameters()]
        st = [v.clone() for p in tr.params for v in tr.opt.state[p].values()]
        x = X[1, rank * 4:(rank + 1) * 4].clone()
        if rank == 1:
            x[0, 0] = float("nan")
        tr.step(x, Y[1, rank * 4:(rank + 1) * 4])
        same = all(torch.equal(a, b) for a, b in zip(before, model.parameters()))
        same_st = all(torch.equal(a, b) for a, b in zip(st, [v for p in tr.params for v in tr.opt.state[p].values()]))
        torch.save({"same": same, "same_st": same_st, "nonfinite": tr.nonfinite_steps, "sched": tr.sched.step_num},
                   os.path.join(out_dir, f"nan{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_nonfinite_loss_on_one_rank_skips_everywhere(tmp_path):
    mp.spawn(_nan_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"nan{r}.pt", weights_only=True)
        assert d["same"] and d["same_st"], d
        assert d["nonfinite"] == 1 and d["sched"] == 1, d


def _nan_train_worker(rank, world, port, out_dir, bucket_mb):
    """Train-mode BatchNorm with a NaN batch on rank 1: rank 1's running statistics go NaN in its
    forward, the step is skipped everywhere, and the buffer exchange (rank 0 contributes its values,
    the others zeros -- not b * 0) leaves every rank holding rank 0's finite statistics."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = _model(seed=0)
        tr = Trainer(model, amp_dtype=None, total_steps=10, warmup_ratio=0.0, bucket_mb=bucket_mb)
        X, Y = _data()
        model.train()
        tr.step(X[0, rank * 4:(rank + 1) * 4], Y[0, rank * 4:(rank + 1) * 4])
        before = [p.detach().clone() for p in model.parameters()]
        x = X[1, rank * 4:(rank + 1) * 4].clone()
        if rank == 1:
            x[0, 0] = float("nan")
        tr.step(x, Y[1, rank * 4:(rank + 1) * 4])
        bufs = [b.clone() for b in model.buffers() if b.is_floating_point()]
        torch.save({"same": all(torch.equal(a, b) for a, b in zip(before, model.parameters())), "bufs": bufs,
                    "nonfinite": tr.nonfinite_steps}, os.path.join(out_dir, f"nant{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bucket_mb", [8.0, 0.0])
def test_dp_nonfinite_train_mode_keeps_bn_buffers_finite(tmp_path, bucket_mb):
    mp.spawn(_nan_train_worker, args=(2, _free_port(), str(tmp_path), bucket_mb), nprocs=2, join=True)
    d0 = torch.load(tmp_path / "nant0.pt", weights_only=True)
    d1 = torch.load(tmp_path / "nant1.pt", weights_only=True)
    for d in (d0, d1):
        assert d["same"] and d["nonfinite"] == 1
        assert all(torch.isfinite(b).all() for b in d["bufs"]), "a NaN rank poisoned the running statistics"
    for a, b in zip(d0["bufs"], d1["bufs"]):
        assert torch.equal(a, b)


def test_nonfinite_loss_skips_step_host():
    """one_epoch_train.py:98-108: a non-finite loss skips the update and the schedule step."""
    model = _model(seed=0).eval()
    tr = Trainer(model, amp_dtype=None, total_steps=10, warmup_ratio=0.2)
    X, Y = _data()
    tr.step(X[0], Y[0])
    before = [p.detach().clone() for p in model.parameters()]
    lr_before = [g["lr"] for g in tr.opt.param_groups]
    x = X[1].clone()
    x[3, 2] = float("inf")
    tr.step(x, Y[1])
    assert all(torch.equal(a, b) for a, b in zip(before, model.parameters()))
    assert tr.nonfinite_steps == 1 and tr.sched.step_num == 1
    assert [g["lr"] for g in tr.opt.param_groups] == lr_before
    tr.step(X[2], Y[2])
    assert tr.sched.step_num == 2 and not all(torch.equal(a, b) for a, b in zip(before, model.parameters()))


def test_flat_bucket_roundtrip():
    """_flatten / _unflatten are exact inverses (world 1 arithmetic, no process group)."""
    model = _model(seed=3)
    tr = Trainer(model, amp_dtype=None)
    tr.world, tr.rank = 2, 0
    tr._bufs = [b for b in model.buffers() if b.is_floating_point()]
    tr._sizes = [p.numel() for p in tr.params]
    tr._bsizes = [b.numel() for b in tr._bufs]
    tr._ng, tr._nb = sum(tr._sizes), sum(tr._bsizes)
    tr.flat = torch.zeros(tr._ng + tr._nb + 1)
    g0 = [torch.randn_like(p) for p in tr.params]
    b0 = [b.clone() for b in tr._bufs]
    for p, g in zip(tr.params, g0):
        p.grad = g.clone()
    tr._flatten(torch.tensor(1.0))
    assert tr.flat.numel() == sum(p.numel() for p in tr.params) + tr._nb + 1
    tr.flat[:tr._ng].mul_(2.0)           # what a 2-rank all_reduce of identical buckets would give
    for b in tr._bufs:
        b.add_(5.0)
    flag = tr._unflatten()
    assert float(flag) == 0.0
    for p, g in zip(tr.params, g0):
        torch.testing.assert_close(p.grad, g, rtol=0, atol=0)
    for b, r in zip(tr._bufs, b0):
        torch.testing.assert_close(b, r, rtol=0, atol=0)


def test_load_optimizer_state_keeps_device_lr_and_tensors():
    """Resume into a (capturable) optimizer whose lr is a tensor: the saved float lr is copied into
    the existing lr tensor and moment tensors are overwritten in place (a recorded graph keeps
    reading the same storage)."""
    from ogv.train import load_optimizer_state
    m = _model(seed=1)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    for p in m.parameters():
        p.grad = torch.ones_like(p)
    opt.step()
    opt.param_groups[0]["lr"] = 2.5e-4
    sd = opt.state_dict()
    m2 = _model(seed=1)
    lr_t = torch.tensor(9.0)
    opt2 = torch.optim.AdamW(m2.parameters(), lr=lr_t, foreach=False)
    for p in m2.parameters():
        p.grad = torch.zeros_like(p)
    opt2.step()
    old = {id(p): opt2.state[p]["exp_avg"] for p in m2.parameters()}
    load_optimizer_state(opt2, sd)
    assert opt2.param_groups[0]["lr"] is lr_t and abs(float(lr_t) - 2.5e-4) < 1e-10
    assert opt2.param_groups[0]["foreach"] is False
    for p, q in zip(m2.parameters(), m.parameters()):
        assert opt2.state[p]["exp_avg"] is old[id(p)]
        torch.testing.assert_close(opt2.state[p]["exp_avg"], opt.state[q]["exp_avg"], rtol=0, atol=0)


def _agree_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ogv.train import agree_status
        # only rank 1 fails its capture: every rank must see the failure
        got = [agree_status(s, torch.device("cpu")) for s in ((0, 1, 0) if rank == 0 else (1, 2, 0))]
        torch.save(got, os.path.join(out_dir, f"a{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_capture_decision_agreed_over_ranks(tmp_path):
    """Trainer._capture's fallback decision is the MAX of the per-rank capture statuses (0 ok, 1 capture
    unsupported -> flat form, 2 other error -> raise), one all_reduce, so no rank replays the bucketed
    graph while another records the flat one; the error classifier sends only capture refusals to the
    fallback."""
    from ogv.train import _capture_unsupported
    mp.spawn(_agree_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert torch.load(tmp_path / f"a{r}.pt") == [1, 2, 0]
    assert _capture_unsupported(RuntimeError("operation not permitted when stream is capturing"))
    assert _capture_unsupported(RuntimeError("hipErrorStreamCaptureUnsupported"))
    assert not _capture_unsupported(RuntimeError("HIP out of memory. Tried to allocate 2.00 GiB"))
    assert not _capture_unsupported(RuntimeError("ogv_gemm_fwd: bad shape"))
