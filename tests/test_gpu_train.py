"""Training step on the MI355X: hipGraph replay (bench.py's execution mode) vs eager launches.

Replay must reproduce the eager trajectory: same losses and parameters after several steps
(DropPath off so both paths draw no random numbers; all ogv kernels are deterministic).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

# Every layer of the model, stem / downsample / head included, runs on the ogv kernels
# (ogv_convbn_*, ogv_bn_act_*: no atomics), so replay and eager are held to 1e-3 everywhere.
GRAD_TOL = 1e-3


@pytest.fixture(autouse=True, scope="module")
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ogv
    ogv.load()


def _model(seed):
    from ogv.train import MODEL_CONFIGS, build_model
    cfg = MODEL_CONFIGS["model_a_7m"]
    torch.manual_seed(seed)
    m = build_model(dict(type="model_a", num_classes=cfg["num_classes"], stem_dim=cfg["stem_dim"], dpr_max=0.0,
                         stages=cfg["stages"]))
    return m.cuda().to(memory_format=torch.channels_last)


def _snapshot(model, opt):
    st = [t.detach().clone() for t in list(model.parameters()) + list(model.buffers())]
    ost = [{k: v.clone() for k, v in opt.state[p].items()} for g in opt.param_groups for p in g["params"]]
    lrs = [g["lr"].clone() for g in opt.param_groups]
    return st, ost, lrs


def _restore(model, opt, snap):
    st, ost, lrs = snap
    with torch.no_grad():
        for t, s in zip(list(model.parameters()) + list(model.buffers()), st):
            t.copy_(s)
        for (p, d) in zip([p for g in opt.param_groups for p in g["params"]], ost):
            for k, v in d.items():
                opt.state[p][k].copy_(v)
        for g, l in zip(opt.param_groups, lrs):
            g["lr"].copy_(l)


def _batch(B, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(B, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 100, (B,), device="cuda", generator=g)
    return x, y


def test_graph_replay_matches_eager_step():
    """Each replayed step == an eager step taken from the identical training state (params,
    BatchNorm buffers, AdamW moments, device lr), for several consecutive replays: same loss,
    same clipped gradients, same update."""
    from ogv.train import Trainer
    torch.backends.cudnn.benchmark = False
    x, y = _batch(16, 3)
    m = _model(11)
    t = Trainer(m, total_steps=50, warmup_ratio=0.1, graphs=True, capture_warmup=1)
    l0 = t.step(x, y).float().item()      # eager
    t.step(x, y)                          # eager on the side stream + capture
    assert t._g is not None, "graph was not captured"
    names = [n for n, _ in m.named_parameters()]
    losses = []
    for k in range(3):
        snap = _snapshot(m, t.opt)
        loss_r = t.step(x, y).float().item()  # replay
        g_r = [g.detach().clone() for g in t.graph_grads]
        p_r = [p.detach().clone() for p in m.parameters()]
        b_r = [b.detach().clone() for b in m.buffers()]
        _restore(m, t.opt, snap)
        loss_e = t._eager(x, y).float().item()
        losses.append(loss_e)
        assert abs(loss_r - loss_e) <= 1e-6 * max(1.0, abs(loss_e)), (k, loss_r, loss_e)
        for n, gr, p in zip(names, g_r, m.parameters()):
            ge = p.grad.detach()
            scale = max(float(ge.abs().max()), 1e-12)
            err = float((gr - ge).abs().max())
            assert err <= GRAD_TOL * scale, f"replay {k}: grad {n} max|d|={err:.3e} scale={scale:.3e}"
        for n, pr, p in zip(names, p_r, m.parameters()):
            # Adam turns last-bit gradient noise on near-zero gradients into sign flips: bound by
            # one lr step either way
            err = float((pr - p.detach()).abs().max())
            assert err <= 2 * float(t.opt.param_groups[0]["lr"]) + 1e-7, f"replay {k}: param {n} max|d|={err:.3e}"
        for (n, b), br in zip(m.named_buffers(), b_r):
            torch.testing.assert_close(br.float(), b.detach().float(), rtol=1e-5, atol=1e-6,
                                       msg=lambda s: f"replay {k}: {n}: {s}")
    assert losses[-1] < l0, (l0, losses)


def test_graph_replay_takes_new_inputs():
    """A captured step records trainer-owned copies of the batch: each later call copies ITS batch
    in, so the replayed loss equals the eager forward loss of that batch at the same parameters,
    and the caller's tensors are never written.  Returned losses are distinct tensors."""
    import torch.nn.functional as F
    from ogv.train import Trainer
    m = _model(2)
    t = Trainer(m, total_steps=50, graphs=True, capture_warmup=0)
    x0, y0 = _batch(8, 5)
    x0_keep = x0.clone()
    t.step(x0, y0)                        # capture with batch 0
    kept = []
    for i in (6, 5, 6):
        x, y = _batch(8, i)               # a fresh tensor every call
        # (grad mode on: the training forward's kernels -- under no_grad the Outlooker takes the
        # fused inference kernel, equal only to bf16 rounding)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            ref = F.cross_entropy(m(x).float(), y, label_smoothing=0.1).item()
        loss = t.step(x, y)
        kept.append(loss)
        got = loss.float().item()
        assert abs(got - ref) <= 1e-5 * max(1.0, abs(ref)), (i, got, ref)
    assert torch.equal(x0, x0_keep), "the capture batch was overwritten"
    assert len({k.data_ptr() for k in kept}) == len(kept)
    assert kept[0].item() != kept[1].item()


def test_graph_ragged_batch_runs_eager():
    """A batch whose shape differs from the recorded one (ragged last batch) is not copied into
    the graph's inputs: it runs as an eager step on the same state."""
    import torch.nn.functional as F
    from ogv.train import Trainer
    m = _model(4)
    t = Trainer(m, total_steps=50, graphs=True, capture_warmup=0)
    t.step(*_batch(8, 1))
    t.step(*_batch(8, 2))
    x, y = _batch(5, 3)
    with torch.autocast("cuda", dtype=torch.bfloat16):     # the training forward's kernels
        ref = F.cross_entropy(m(x).float(), y, label_smoothing=0.1).item()
    got = t.step(x, y).item()
    assert t.eager_fallbacks == 1 and abs(got - ref) <= 1e-5 * max(1.0, abs(ref))
    t.step(*_batch(8, 4))                 # back to replay
    assert t.eager_fallbacks == 1


def test_release_graphs_then_recapture_continues_bit_identically():
    """Trainer.release_graphs() (bench.py drops the recorded graph before its eager diagnostic steps so they
    never allocate beside the graph's pool): the next step records the graph again and the run continues
    as one that never released it (losses, parameters) -- and the pool's memory is returned to the device by
    empty_cache."""
    from ogv.train import Trainer
    runs = []
    for release in (False, True):
        m = _model(12)
        t = Trainer(m, total_steps=50, warmup_ratio=0.1, graphs=True, capture_warmup=1)
        losses = [t.step(*_batch(8, 40 + i)).item() for i in range(3)]      # eager, capture, replay
        if release:
            torch.cuda.synchronize()
            before = torch.cuda.memory_reserved()
            t.release_graphs()
            torch.cuda.empty_cache()
            assert t._g is None and torch.cuda.memory_reserved() < before
        losses += [t.step(*_batch(8, 43 + i)).item() for i in range(3)]     # (re-)capture, replay, replay
        assert t._g is not None
        torch.cuda.synchronize()
        runs.append((losses, [p.detach().clone() for p in m.parameters()],
                     [v.detach().clone() for p in t.params for v in t.opt.state[p].values()]))
        del t
    # steps 1-3 identical; the released run takes step 4 as the capture step's eager update, which equals a
    # replay to the tolerances of test_graph_replay_matches_eager_step (Adam sign flips: <= 2 lr per step)
    assert runs[0][0][:3] == runs[1][0][:3]
    for a, b in zip(runs[0][0][3:], runs[1][0][3:]):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(a)), (runs[0][0], runs[1][0])
    lr = 5e-4
    for a, b in zip(runs[0][1], runs[1][1]):
        assert float((a - b).abs().max()) <= 3 * 2 * lr + 1e-6


@pytest.mark.parametrize("graphs", [True, False])
def test_nonfinite_loss_skips_update_without_sync(graphs):
    """one_epoch_train.py:98-108 on the device: a NaN batch leaves parameters, BN-free optimizer
    state (moments, step counts), lr and the schedule counter unchanged -- in a replayed graph
    and in eager launches -- and the next finite batch trains normally."""
    from ogv.train import Trainer
    m = _model(8)
    t = Trainer(m, total_steps=50, warmup_ratio=0.1, graphs=graphs, capture_warmup=1)
    for i in range(3):                    # eager, capture, replay
        t.step(*_batch(8, 20 + i))
    torch.cuda.synchronize()
    params = [p.detach().clone() for p in m.parameters()]
    state = [v.detach().clone() for p in t.params for v in t.opt.state[p].values()]
    lrs = [g["lr"].detach().clone() for g in t.opt.param_groups]
    sched0 = t.sched.step_num
    x, y = _batch(8, 30)
    x[2, 1, 5, 7] = float("nan")
    loss = t.step(x, y)
    assert not torch.isfinite(loss).item()
    for a, b in zip(params, m.parameters()):
        assert torch.equal(a, b), "parameters changed on a non-finite step"
    for a, b in zip(state, [v for p in t.params for v in t.opt.state[p].values()]):
        assert torch.equal(a, b), "optimizer state changed on a non-finite step"
    for a, g in zip(lrs, t.opt.param_groups):
        assert torch.equal(a, g["lr"])
    assert t.sched.step_num == sched0 and t.nonfinite_steps == 1
    loss = t.step(*_batch(8, 31))
    assert torch.isfinite(loss).item() and t.sched.step_num == sched0 + 1
    assert any(not torch.equal(a, b) for a, b in zip(params, m.parameters()))


def test_resume_into_graph_trainer_follows_schedule(tmp_path):
    """Checkpoint -> resume into a graphs=True Trainer (src/training/chekpoints.py dict): the lr the
    replays use keeps following the warmup-cosine schedule from the saved step, and the resumed
    trajectory equals the uninterrupted one."""
    from ogv.train import Trainer
    from src.training.chekpoints import load_checkpoint, save_checkpoint
    torch.backends.cudnn.benchmark = False
    batches = [_batch(8, 50 + i) for i in range(8)]
    ma = _model(9)
    ta = Trainer(ma, total_steps=20, warmup_ratio=0.2, graphs=True, capture_warmup=1)
    for i in range(4):
        ta.step(*batches[i])
    save_checkpoint(str(tmp_path / "last.pt"), ma, ta.opt, ta.sched, None, epoch=0, best_top1=0.0)
    lr_a = []
    for i in range(4, 8):
        ta.step(*batches[i])
        lr_a.append(float(ta.opt.param_groups[0]["lr"]))
    mb = _model(10)
    tb = Trainer(mb, total_steps=20, warmup_ratio=0.2, graphs=True, capture_warmup=0)
    load_checkpoint(str(tmp_path / "last.pt"), mb, tb.opt, tb.sched, None)
    assert tb.sched.step_num == 4
    lr_b = []
    for i in range(4, 8):
        tb.step(*batches[i])              # capture (eager on a side stream), then replays
        lr_b.append(float(tb.opt.param_groups[0]["lr"]))
    assert lr_b == lr_a, (lr_a, lr_b)
    expect = [ta.sched.lr_at(s, 5e-4) for s in range(5, 9)]
    assert all(abs(a - e) <= 1e-6 * e for a, e in zip(lr_a, expect)), (lr_a, expect)
    for (n, a), b in zip(ma.named_parameters(), mb.parameters()):
        err = float((a - b).abs().max())
        assert err <= 2 * 5e-4 + 1e-7, (n, err)


def _dp_worker(rank, world, port, out):
    import os
    import torch.distributed as dist
    from ogv.train import Trainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import ogv
    ogv.load()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.backends.cudnn.benchmark = False
        m = _model(11 + rank)                 # different init: the rank-0 broadcast must fix it
        t = Trainer(m, total_steps=50, graphs=True, capture_warmup=1)
        assert t.world == world
        x, y = _batch(8, 40 + rank)           # per-rank shard
        losses = [t.step(x, y).float().item() for _ in range(4)]   # eager, capture, replay, replay
        torch.save({"params": [p.detach().cpu() for p in m.parameters()], "losses": losses}, f"{out}/r{rank}.pt")
    finally:
        dist.destroy_process_group()


def test_graph_dp_world2_ranks_agree(tmp_path):
    """world_size 2 on one GPU (gloo carries the all_reduce; RCCL needs one GPU per rank): graph A
    (fwd+bwd+flatten), all_reduce of the flat bucket, graph B (unflatten+clip+AdamW) keep the two
    ranks' parameters identical while each rank trains on its own shard."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_dp_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert r0["losses"] != r1["losses"], "ranks saw the same data"
    assert all(l == l for l in r0["losses"] + r1["losses"]), "non-finite loss"
    for a, b in zip(r0["params"], r1["params"]):
        assert torch.equal(a, b), "ranks diverged"


def test_model_b_step_with_cutmix_soft_targets():
    """Model B (OutlookerFrontGridNet) through the Trainer, fed a CutMix batch from the native mix
    kernels (soft targets -> soft_target_cross_entropy, one_epoch_train.py:77-92): graph replay
    reproduces the eager loss on the same batch and the parameters move."""
    import random
    from ogv.mix import apply_mixup_cutmix
    from ogv.train import MODEL_CONFIGS, Trainer, build_model

    cfg = dict(MODEL_CONFIGS["model_b_cifar100"])
    cfg.pop("img")
    cfg["dpr_max"] = 0.0
    torch.manual_seed(1)
    m = build_model(cfg).cuda().to(memory_format=torch.channels_last)
    x, y = _batch(64, 5)
    random.seed(0)
    xm, ys = apply_mixup_cutmix(x, y, 100, cutmix_alpha=1.0, prob=1.0)
    assert ys.shape == (64, 100) and torch.allclose(ys.sum(1), torch.ones(64, device="cuda"))
    before = [p.detach().clone() for p in m.parameters()]
    tr = Trainer(m, total_steps=100, graphs=True, capture_warmup=1)
    snap = _snapshot(m, tr.opt)
    l_eager = tr.step(xm, ys).item()                 # eager
    _restore(m, tr.opt, snap)
    tr.step(xm, ys)                                  # capture (eager on a side stream)
    _restore(m, tr.opt, snap)
    l_replay = tr.step(xm, ys).item()                # replay
    assert torch.isfinite(torch.tensor(l_eager)) and abs(l_replay - l_eager) <= 1e-3 * max(1.0, abs(l_eager))
    moved = sum(int(not torch.equal(a, b)) for a, b in zip(before, m.parameters()))
    assert moved > 0.9 * len(before)


def test_resume_from_plain_adamw_checkpoint(tmp_path):
    """A checkpoint written with the reference's optimizer -- a plain torch.optim.AdamW (not fused,
    not capturable: src/training/train_full_model.py:56-57) -- resumes into a fresh graphs=True
    Trainer: every state['step'] lands on the device as fp32 (torch leaves them as CPU scalars for
    such a checkpoint), and the captured / replayed steps keep advancing them."""
    import torch.nn.functional as F
    from ogv.train import Trainer, param_groups_no_wd
    from src.training.chekpoints import load_checkpoint, save_checkpoint
    m0 = _model(12)
    plain = torch.optim.AdamW(param_groups_no_wd(m0, 0.05), lr=5e-4)
    for i in range(2):
        x, y = _batch(8, 60 + i)
        plain.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m0(x).float(), y, label_smoothing=0.1)
        loss.backward()
        plain.step()
    save_checkpoint(str(tmp_path / "plain.pt"), m0, plain, None, None, epoch=0, best_top1=0.0)
    m1 = _model(13)
    t = Trainer(m1, total_steps=20, warmup_ratio=0.1, graphs=True, capture_warmup=0)
    load_checkpoint(str(tmp_path / "plain.pt"), m1, t.opt, None, None)
    steps = [t.opt.state[p]["step"] for p in t.params]
    assert all(s.device.type == "cuda" and s.dtype == torch.float32 and float(s) == 2.0 for s in steps)
    for i in range(3):                               # capture (eager on a side stream), replay, replay
        loss = t.step(*_batch(8, 70 + i))
        assert torch.isfinite(loss).item()
    torch.cuda.synchronize()
    assert all(float(t.opt.state[p]["step"]) == 5.0 for p in t.params)


def _dp_eval_worker(rank, world, port, out):
    import os
    import torch.distributed as dist
    from ogv.train import Trainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import ogv
    ogv.load()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.backends.cudnn.benchmark = False
        m = _model(21 + rank).eval()          # BN on running statistics: the shards then see the same model
        t = Trainer(m, total_steps=50, warmup_ratio=0.1, graphs=True, capture_warmup=1)
        for i in range(3):                    # eager, capture, replay
            x, y = _batch(16, 80 + i)
            t.step(x[rank * 8:(rank + 1) * 8].contiguous(memory_format=torch.channels_last), y[rank * 8:(rank + 1) * 8])
        torch.save([p.detach().cpu() for p in m.parameters()], f"{out}/e{rank}.pt")
    finally:
        dist.destroy_process_group()


def test_graph_dp_world2_matches_single_process(tmp_path):
    """Graph-mode DP (graph A, all_reduce of the flat bucket, graph B) on two 8-image shards equals a
    single-process graph-mode Trainer on the concatenated 16-image batch (BatchNorm in eval mode so
    per-rank batch statistics do not enter): parameters within one AdamW step of lr per step (Adam
    turns last-bit differences of near-zero gradients -- the row sums are split differently -- into
    sign flips)."""
    import socket
    import torch.multiprocessing as mp
    from ogv.train import Trainer
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_dp_eval_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "e0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "e1.pt", weights_only=True)
    m = _model(21).eval()
    t = Trainer(m, total_steps=50, warmup_ratio=0.1, graphs=True, capture_warmup=1)
    for i in range(3):
        t.step(*_batch(16, 80 + i))
    init = [p.detach().cpu() for p in _model(21).parameters()]
    lr_sum = 3 * 2 * 5e-4
    d_dp = d_move = 0.0
    for a, b, p, p0 in zip(r0, r1, m.parameters(), init):
        assert torch.equal(a, b), "ranks diverged"
        err = float((a - p.detach().cpu()).abs().max())
        assert err <= lr_sum + 1e-6, err
        d_dp += float((a - p.detach().cpu()).double().norm() ** 2)
        d_move += float((p.detach().cpu() - p0).double().norm() ** 2)
    # the DP trajectory differs from the single-process one by far less than the training moved
    assert d_dp ** 0.5 <= 0.25 * d_move ** 0.5, (d_dp ** 0.5, d_move ** 0.5)


DEFER_CASES = [("model_a_7m", 64, 0.0), ("model_a_7m", 32, 0.07), ("model_a_14m_tin64", 8, 0.08),
               ("model_a_22m_224", 2, 0.11), ("model_b_cifar100", 16, 0.1)]


@pytest.mark.parametrize("cfg_name,B,dpr", DEFER_CASES, ids=[f"{c}_b{b}_dpr{d}" for c, b, d in DEFER_CASES])
def test_deferred_param_reductions_match_immediate(cfg_name, B, dpr):
    """The Trainer's backward records the parameter-gradient column reductions (Linear weight / bias
    gradients, LayerNorm gamma / beta, the fused MBConv's weight gradients) and runs them as one batched
    launch at its end (functional.deferred_param_reductions): every gradient equals the immediate path's
    (same single-pass arithmetic where that path used it, fp32 rounding of a different split otherwise),
    and the deferral really took the reductions (dozens pending before the flush) -- on every model
    configuration, with DropPath on (its per-row scales enter the weight-gradient prologues; the same
    seed draws the same masks in both runs)."""
    from ogv import functional as OF
    from ogv._lib import load
    from ogv.train import MODEL_CONFIGS, Trainer, build_model
    cfg = dict(MODEL_CONFIGS[cfg_name])
    img = cfg.pop("img")
    cfg["dpr_max"] = dpr
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(B, 3, img, img, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, cfg["num_classes"], (B,), device="cuda", generator=g)
    grads, pending = [], []
    for defer in (False, True):
        torch.manual_seed(13)
        m = build_model(cfg).cuda().to(memory_format=torch.channels_last)
        t = Trainer(m, total_steps=50, graphs=False, defer_reductions=False)
        t.opt.zero_grad(set_to_none=True)
        torch.manual_seed(99)                  # the same DropPath draws in both runs
        with OF.deferred_param_reductions(defer):
            loss, _ = t._loss(x, y)
            loss.backward()
            pending.append(load().ogv_reduce_defer(1 if defer else 0))
        torch.cuda.synchronize()
        grads.append([p.grad.detach().clone() for p in m.parameters()])
        # every parameter received a distinct gradient tensor (a deferred destination written twice or
        # into a stolen / cloned buffer would alias or leave one unwritten)
        ptrs = [p.grad.data_ptr() for p in m.parameters()]
        assert len(set(ptrs)) == len(ptrs)
    assert pending[0] == 0 and pending[1] >= 20, pending
    same = 0
    for a, b in zip(*grads):
        assert torch.isfinite(b).all()
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-7)
        same += bool(torch.equal(a, b))
    assert same >= len(grads[0]) // 2, (same, len(grads[0]))


class _ParamBag(torch.nn.Module):
    """> 64 parameter tensors (several ogv_clip_adamw launches), odd sizes, > 8192-element tensors
    (several chunks), channels_last 4-D weights and both weight-decay groups."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(3)
        self.ws = torch.nn.ParameterList(
            [torch.nn.Parameter(torch.randn(n, generator=g)) for n in (1, 3, 5, 17, 63, 64, 65, 8191, 8192, 8193, 40000)]
            + [torch.nn.Parameter(torch.randn(7, 13, generator=g)) for _ in range(60)])
        self.conv = torch.nn.Parameter(torch.randn(32, 16, 3, 3, generator=g).contiguous(memory_format=torch.channels_last))
        self.norm_w = torch.nn.Parameter(torch.randn(96, generator=g))
        self.bias = torch.nn.Parameter(torch.randn(130, generator=g))


@pytest.mark.parametrize("clip", [1.0, None, 1e6, 0.0])
def test_native_clip_adamw_matches_torch(clip):
    """ogv_clip_adamw (the Trainer's default) against torch's clip_grad_norm_(foreach) + AdamW(fused,
    capturable).step() on the same parameters, gradients and schedule, over 4 steps with a skipped
    (found_inf) one: parameters, moments, step counters and the clipped gradients (on applied steps:
    on a skipped one torch's clip_grad_norm_ still scales .grad, the native path leaves it as is --
    the skipped step's gradients are discarded either way)."""
    from ogv.train import Trainer
    dev = "cuda"
    mods = [_ParamBag().to(dev) for _ in range(2)]
    trs = [Trainer(m, lr=3e-3, weight_decay=0.05, clip=clip, native_optimizer=nat, total_steps=50)
           for m, nat in zip(mods, (True, False))]
    g = torch.Generator(device=dev).manual_seed(11)
    for step in range(4):
        grads = [torch.randn(p.shape, device=dev, generator=g) * (0.5 + step) for p in mods[0].parameters()]
        for tr, m in zip(trs, mods):
            for p, gr in zip(m.parameters(), grads):
                p.grad = gr.clone().contiguous(memory_format=torch.channels_last) if p.dim() == 4 else gr.clone()
            tr._found.fill_(1.0 if step == 2 else 0.0)
            tr._update()
        torch.cuda.synchronize()
        assert trs[0].native_optimizer_fallbacks == 0
        for (n0, p0), p1 in zip(mods[0].named_parameters(), mods[1].parameters()):
            if step != 2:
                torch.testing.assert_close(p0.grad, p1.grad, rtol=1e-5, atol=1e-7, msg=f"{n0} grad step {step}")
            torch.testing.assert_close(p0, p1, rtol=1e-5, atol=1e-6, msg=f"{n0} param step {step}")
            s0, s1 = trs[0].opt.state[p0], trs[1].opt.state[p1]
            assert float(s0["step"]) == float(s1["step"]) == (step + 1 if step < 2 else step)
            torch.testing.assert_close(s0["exp_avg"], s1["exp_avg"], rtol=1e-5, atol=1e-7)
            torch.testing.assert_close(s0["exp_avg_sq"], s1["exp_avg_sq"], rtol=1e-5, atol=1e-9)


def test_state_dict_tensors_do_not_share_storage(tmp_path):
    """the Outlooker's v / attn parameters are views into one padded [ld, C] buffer after the
    first forward; Trainer.state_dict() and save_checkpoint write independent, unpadded tensors (the file
    holds the parameters' bytes, not the padded buffer's)."""
    from ogv.train import Trainer
    from src.training.chekpoints import save_checkpoint
    m = _model(3)
    t = Trainer(m, total_steps=10, graphs=False)
    t.step(*_batch(8, 1))
    live = dict(m.state_dict())
    shared = [k for k, v in live.items() if v.untyped_storage().nbytes() > v.numel() * v.element_size()]
    assert shared, "expected the Outlooker's aliased parameter buffer"
    for k, v in t.state_dict()["model"].items():
        assert v.untyped_storage().nbytes() == v.numel() * v.element_size(), k
        assert torch.equal(v, live[k])
    save_checkpoint(str(tmp_path / "c.pt"), m, None, None, None, epoch=0, best_top1=0.0)
    ck = torch.load(tmp_path / "c.pt", map_location="cpu", weights_only=True)
    for k, v in ck["model"].items():
        assert v.untyped_storage().nbytes() == v.numel() * v.element_size(), k


def test_native_optimizer_after_contiguous_moment_resume(tmp_path):
    """a checkpoint whose AdamW moments are contiguous (the reference's layout) resumed into a
    channels_last model: load_optimizer_state re-lays them like their parameters, so the native clip +
    AdamW keeps running (no silent per-step torch fallback)."""
    from ogv.train import Trainer
    from src.training.chekpoints import load_checkpoint, save_checkpoint
    m0 = _model(4)
    t0 = Trainer(m0, total_steps=10, graphs=False)
    t0.step(*_batch(8, 2))
    sd = t0.opt.state_dict()
    for st in sd["state"].values():
        for k in ("exp_avg", "exp_avg_sq"):
            st[k] = st[k].contiguous()
    torch.save({"model": m0.state_dict(), "optimizer": sd, "scheduler": t0.sched.state_dict(), "scaler": None,
                "epoch": 0, "best_top1": 0.0, "extra": {}}, tmp_path / "r.pt")
    m1 = _model(5)
    t1 = Trainer(m1, total_steps=10, graphs=False)
    load_checkpoint(str(tmp_path / "r.pt"), m1, t1.opt, t1.sched, None)
    t1.step(*_batch(8, 3))
    assert t1.native_optimizer_fallbacks == 0


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_rccl_world1_dp_path_matches_single_process():
    """The RCCL branch executed: a world-size-1 "nccl" (= RCCL) process group, the Trainer's data-parallel
    path forced on (force_dp: rank-0 broadcast, gradient + buffer + non-finite-flag bucket, all_reduce), in
    graph mode with the bucketed all_reduces captured on a side stream as backward completes each bucket
    (dp_overlap, the RCCL default), with the flat path (graph A -> RCCL all_reduce -> graph B), with the
    all_reduce captured at the end of the step's graph (dp_capture_collective), and eagerly with the bucketed asynchronous all_reduces during backward: every
    loss and parameter equals the single-process Trainer's (the all_reduce of one rank is the identity; the
    eager bucket path runs its parameter-gradient reductions immediately instead of deferred, so it is held
    to one lr step per element, Adam's sign flips of near-zero gradients).  Runs tests/_rccl_world1.py as a
    child process (its own process group and HIP context; an RCCL abort cannot take the test runner down).
    dp_graph_fallback: the overlapped capture made to raise (a runtime that refuses to record collectives)
    -- the Trainer warns once and records the flat two-graph form instead, with the same result."""
    import json
    import pathlib
    import subprocess
    import sys
    here = pathlib.Path(__file__).resolve().parent
    r = subprocess.run([sys.executable, str(here / "_rccl_world1.py")], capture_output=True, text=True, timeout=240)
    print(r.stdout[-4000:], r.stderr[-4000:])
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    res = {d["mode"]: d for d in lines if "mode" in d}
    assert set(res) >= {"plain", "dp_graph", "dp_graph_flat", "dp_capture", "plain_eager", "dp_eager",
                        "dp_graph_fallback", "dp_graph_other_error"}, \
        (r.returncode, list(res))
    for mode in ("dp_graph", "dp_graph_flat", "dp_capture", "dp_eager"):
        assert res[mode]["backend"] == "nccl", res[mode]
    assert res["dp_graph"]["dp_overlap"] and res["dp_graph"]["buckets"] >= 2 and res["dp_graph"]["grad_is_view"]
    # the overlapped capture refused (simulated): one warning, the flat two-graph form, same result
    assert not res["dp_graph_fallback"]["dp_overlap"] and res["dp_graph_fallback"]["fallback_warned"] == 1
    assert "out of memory" in res["dp_graph_other_error"]["raised"], res["dp_graph_other_error"]
    assert res["dp_graph"]["fallback_warned"] == 0
    for mode, ref in (("dp_graph", "plain"), ("dp_graph_flat", "plain"), ("dp_capture", "plain"),
                      ("dp_graph_fallback", "plain")):
        assert res[mode]["losses"] == res[ref]["losses"], (mode, res[mode]["losses"], res[ref]["losses"])
        assert res[mode]["max_param_diff_vs_" + ref] == 0.0, res[mode]
    la, lb = res["dp_eager"]["losses"], res["plain_eager"]["losses"]
    assert all(abs(a - b) <= 1e-3 * max(1.0, abs(b)) for a, b in zip(la, lb)), (la, lb)
    assert res["dp_eager"]["max_param_diff_vs_plain_eager"] <= 4 * 2 * 5e-4 + 1e-6
    assert r.returncode == 0, r.returncode


def _ddp_worker(rank, world, port, out):
    import os
    import torch.distributed as dist
    from ogv.train import Trainer, wrap_ddp
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import ogv
    ogv.load()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.backends.cudnn.benchmark = False
        res = {}
        for kind in ("ddp", "bare"):
            m = _model(41).eval()                 # running-statistics BN: the shards see the same model
            model = wrap_ddp(m, torch.device("cuda", 0)) if kind == "ddp" else m
            t = Trainer(model, total_steps=50, warmup_ratio=0.1, graphs=False)
            assert t.ddp == (kind == "ddp")
            assert not (t.ddp and t.defer_reductions), "deferral must be off under DDP"
            for i in range(2):
                x, y = _batch(16, 100 + i)
                t.step(x[rank * 8:(rank + 1) * 8].contiguous(memory_format=torch.channels_last), y[rank * 8:(rank + 1) * 8])
            res[kind] = [p.detach().cpu() for p in m.parameters()]
        torch.save(res, f"{out}/d{rank}.pt")
    finally:
        dist.destroy_process_group()


def test_ddp_wrapped_model_world2(tmp_path):
    """a DDP-wrapped model handed to the Trainer.  DDP's reducer copies each gradient
    into its bucket when AccumulateGrad fires, so the deferred parameter-gradient reductions must be off
    (they would be all-reduced before being written).  Two gloo ranks on one GPU, eval-mode BatchNorm:
    the DDP run equals the Trainer's own DP path on the same shards (one lr step per element: Adam sign
    flips of near-zero gradients) and both ranks agree."""
    import torch.multiprocessing as mp
    mp.spawn(_ddp_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "d0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "d1.pt", weights_only=True)
    for a, b in zip(r0["ddp"], r1["ddp"]):
        assert torch.equal(a, b), "DDP ranks diverged"
    init = [p.detach().cpu() for p in _model(41).parameters()]
    move = sum(float((a - p0).double().norm() ** 2) for a, p0 in zip(r0["bare"], init)) ** 0.5
    diff = 0.0
    for a, b in zip(r0["ddp"], r0["bare"]):
        assert float((a - b).abs().max()) <= 2 * 2 * 5e-4 + 1e-6
        diff += float((a - b).double().norm() ** 2)
    assert diff ** 0.5 <= 0.25 * move, (diff ** 0.5, move)
