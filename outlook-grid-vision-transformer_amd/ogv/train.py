"""Model-A training harness on MI355X: builder, optimizer/schedule, one-process-per-GPU data
parallelism, and the per-step function the benchmark times.

Restates the reference's training semantics (not its host-side logging):
  build_model            scripts/train.py:29-60 (StageCfg(**s) per stage -> MaxOutNet)
  param_groups_no_wd     src/training/warmup.py:4-26
  WarmupCosineLR         src/training/warmup.py:29-59 (step-based, state_dict = step_num)
  train step             src/training/one_epoch_train.py:85-153: autocast fwd, CE(label
                         smoothing) in fp32, backward, clip_grad_norm_(1.0), AdamW, scheduler
The reference loop syncs the host ~5x per step (isfinite, float(gnorm), .item()s); this step has
no host syncs: the grad-norm stays on device (clip_grad_norm_ foreach path) and the loss is
returned as a device tensor.

Execution: the whole step is captured once as a hipGraph (torch.cuda.CUDAGraph) and replayed,
so ~1200 kernel launches per step cost one graph launch instead of ~1200 Python/HIP launches.
The learning rate lives in a device tensor the schedule updates before each replay.

Data parallelism (the reference has none): one process per GPU, torch.distributed with the
"nccl" backend (= RCCL on ROCm) over xGMI.  Graph mode on RCCL (the default, Trainer(dp_overlap)):
ONE graph per step, the fp32 gradients all-reduced (pre-divided by world size) in ~bucket_mb buckets
recorded inside it, each launched as soon as backward has produced its last gradient so it overlaps
the rest of the backward, the optimizer reading the reduced gradients in place.  Alternatives:
graph A (fwd + bwd + flatten into one bucket) -> one all_reduce -> graph B (unflatten + clip +
AdamW) -- the form gloo groups (whose collectives cannot be recorded) and dp_overlap=False use, and
the fallback when a runtime refuses to record collectives -- or that flat all_reduce recorded at
the end of the one graph (dp_capture_collective).  Parameters and buffers are broadcast from rank 0
once at start; the BatchNorm running buffers then ride in the collectives every step (rank 0's
values, the others contribute zeros: DDP's broadcast_buffers), and each rank normalises with its
own batch statistics.  Eager mode all-reduces 8 MB buckets asynchronously as backward
produces them.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

# Stage layouts of the reference configs (configs/cifar100_model_a_7m.yaml:7-27,
# configs/cifar100_model_a_14m.yaml:7-27, configs/tinyimagenet200_model_a.yaml:7-27).
MODEL_CONFIGS = {
    "model_a_7m": dict(num_classes=100, stem_dim=64, dpr_max=0.07, img=32, stages=[
        dict(dim=48, depth=1, num_heads=2, grid_size=8, outlook_heads=2),
        dict(dim=96, depth=2, num_heads=3, grid_size=8, outlook_heads=3),
        dict(dim=192, depth=3, num_heads=6, grid_size=4, outlook_heads=6),
        dict(dim=256, depth=1, num_heads=8, grid_size=2, outlook_heads=8)]),
    "model_a_14m_tin64": dict(num_classes=200, stem_dim=64, dpr_max=0.08, img=64, stages=[
        dict(dim=64, depth=2, num_heads=2, grid_size=8, outlook_heads=2),
        dict(dim=128, depth=2, num_heads=4, grid_size=8, outlook_heads=4),
        dict(dim=256, depth=3, num_heads=8, grid_size=4, outlook_heads=8),
        dict(dim=384, depth=1, num_heads=6, grid_size=2, outlook_heads=6)]),
    "model_a_22m_224": dict(num_classes=1000, stem_dim=64, dpr_max=0.11, img=224, stages=[
        dict(dim=64, depth=2, num_heads=2, grid_size=8, outlook_heads=2),
        dict(dim=128, depth=3, num_heads=4, grid_size=8, outlook_heads=4),
        dict(dim=256, depth=4, num_heads=8, grid_size=4, outlook_heads=8),
        dict(dim=384, depth=2, num_heads=6, grid_size=2, outlook_heads=6)]),
    # Model B (OutlookerFrontGridNet), configs/cifar100_model_b.yaml:1-29
    "model_b_cifar100": dict(type="model_b", num_classes=100, stem_dim=64, dpr_max=0.1, img=32,
                             outlooker_front_depth=3, stages=[
        dict(dim=64, depth=2, num_heads=2, grid_size=8, outlook_heads=2),
        dict(dim=128, depth=2, num_heads=4, grid_size=8, outlook_heads=4),
        dict(dim=256, depth=3, num_heads=8, grid_size=4, outlook_heads=8),
        dict(dim=384, depth=1, num_heads=6, grid_size=2, outlook_heads=6)]),
}


def build_model(model_cfg: dict) -> nn.Module:
    """YAML `model:` section -> MaxOutNet (Model A) or OutlookerFrontGridNet (Model B), the
    dispatch of scripts/train.py:33-60 (same type aliases, same errors)."""
    from src.Model_A_OutGridNet import MaxOutNet
    from src.Model_B_OutGridNet import OutlookerFrontGridNet
    from src.model.downsampling import DownsampleConfig
    from src.stage_config import StageCfg

    kind = str(model_cfg.get("type", "model_a")).lower()
    stages = [StageCfg(**s) for s in model_cfg.get("stages", [])]
    if not stages:
        raise ValueError("model.stages must have at least one stage config")
    common = dict(num_classes=int(model_cfg.get("num_classes", 100)), stages=stages,
                  in_ch=int(model_cfg.get("in_ch", 3)), stem_dim=int(model_cfg.get("stem_dim", 64)),
                  dpr_max=float(model_cfg.get("dpr_max", 0.1)),
                  down_cfg=DownsampleConfig(**model_cfg.get("downsample", {})))
    if kind in ("a", "model_a", "maxout", "outgrid"):
        return MaxOutNet(**common)
    if kind in ("b", "model_b", "outlooker_front", "front"):
        return OutlookerFrontGridNet(outlooker_front_depth=int(model_cfg.get("outlooker_front_depth", 2)), **common)
    raise ValueError(f"Unknown model.type '{kind}'. Use 'model_a' (MaxOutNet) or 'model_b' (OutlookerFrontGridNet)")


def _dense_like(t: torch.Tensor, p: torch.Tensor) -> bool:
    """t is an fp32 CUDA tensor of p's shape, dense (contiguous or channels_last) and in p's memory
    order: strides equal wherever the size is > 1 (a [C, K, 1, 1] weight is both contiguous and
    channels_last with different strides on its size-1 dims, same bytes)."""
    if t.dtype != torch.float32 or not t.is_cuda or t.shape != p.shape:
        return False
    if not (t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))):
        return False
    return all(a == b for a, b, n in zip(t.stride(), p.stride(), p.shape) if n > 1)


def param_groups_no_wd(model: nn.Module, weight_decay: float):
    decay, no_decay = [], []
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        low = name.lower()
        skip = name.endswith(".bias") or any(tag in low for tag in ("norm", "bn", "ln", "pos", "cls_token"))
        (no_decay if skip else decay).append(p)
    return [{"params": decay, "weight_decay": weight_decay}, {"params": no_decay, "weight_decay": 0.0}]


class WarmupCosineLR:
    """Linear warmup for warmup_steps, then cosine from the base lr down to min_lr
    (src/training/warmup.py:29-59: the same formula, step-based, state_dict = step_num).

    ``bind_device(counter)``: the step count lives in a device tensor that the Trainer advances
    inside its (captured) step only when the step was applied (non-finite steps are skipped like
    the reference's ``continue`` before ``scheduler.step()``, one_epoch_train.py:98-108), and the
    groups' lr tensors are recomputed on the device from it -- no host sync per step."""

    def __init__(self, optimizer, total_steps: int, warmup_steps: int, min_lr: float = 0.0):
        self.optimizer = optimizer
        self.total_steps, self.warmup_steps, self.min_lr = int(total_steps), int(warmup_steps), float(min_lr)
        self.base_lrs = [float(g["lr"]) for g in optimizer.param_groups]
        self._step_num = 0
        self._dev = None

    # host formula (warmup.py:38-52)
    def lr_at(self, t: int, base: float) -> float:
        if self.warmup_steps > 0 and t <= self.warmup_steps:
            return base * t / self.warmup_steps
        prog = (min(t, self.total_steps) - self.warmup_steps) / max(1, self.total_steps - self.warmup_steps)
        return self.min_lr + (base - self.min_lr) * 0.5 * (1.0 + math.cos(math.pi * prog))

    def bind_device(self, counter: torch.Tensor):
        counter.fill_(float(self._step_num))
        self._dev = counter

    def device_step(self, found: torch.Tensor, nonfinite: torch.Tensor):
        """counter += 1 - found, nonfinite += found, every group's lr tensor = lr(counter): one
        native single-thread launch (ogv_schedule_step), capturable, no host sync."""
        from . import _lib
        lib = _lib.load()
        groups = self.optimizer.param_groups
        ptrs = (ctypes.c_void_p * len(groups))(*[g["lr"].data_ptr() for g in groups])
        base = (ctypes.c_float * len(groups))(*self.base_lrs)
        _lib.check(lib.ogv_schedule_step(found.data_ptr(), self._dev.data_ptr(), nonfinite.data_ptr(), ptrs, base,
                                         len(groups), self.warmup_steps, self.total_steps, self.min_lr,
                                         torch.cuda.current_stream().cuda_stream), "ogv_schedule_step")

    def apply_device(self):
        """Write lr(step_num) into every group's device lr tensor (reads the counter: a sync;
        used on resume / a manual scheduler.step(), never inside the training step)."""
        t = self.step_num
        for g, base in zip(self.optimizer.param_groups, self.base_lrs):
            g["lr"].fill_(self.lr_at(t, base))

    @property
    def step_num(self) -> int:
        return int(self._dev.item()) if self._dev is not None else self._step_num

    @step_num.setter
    def step_num(self, v: int):
        self._step_num = int(v)
        if self._dev is not None:
            self._dev.fill_(float(v))

    def step(self):
        if self._dev is not None:
            self.step_num = self.step_num + 1
            self.apply_device()
            return
        self._step_num += 1
        for g, base in zip(self.optimizer.param_groups, self.base_lrs):
            v = self.lr_at(self._step_num, base)
            if isinstance(g["lr"], torch.Tensor):
                g["lr"].fill_(v)
            else:
                g["lr"] = v

    def state_dict(self):
        return {"step_num": self.step_num}

    def load_state_dict(self, d):
        self.step_num = int(d.get("step_num", 0))
        if self._dev is not None:
            self.apply_device()


def load_optimizer_state(optimizer: torch.optim.Optimizer, state_dict: dict):
    """optimizer.load_state_dict that keeps a capturable/fused optimizer usable and any hipGraph
    recorded over it valid: the runtime flags (fused, capturable, foreach) and the device lr
    tensors of the groups are kept (a saved float / CPU lr is copied INTO the existing device
    tensor), and state tensors that already exist are overwritten in place instead of replaced."""
    old_groups = [dict(g) for g in optimizer.param_groups]
    old_state = {p: dict(st) for p, st in optimizer.state.items()}
    optimizer.load_state_dict(state_dict)
    for g, og in zip(optimizer.param_groups, old_groups):
        for k in ("fused", "capturable", "foreach", "differentiable"):
            if k in og:
                g[k] = og[k]
        if isinstance(og["lr"], torch.Tensor):
            og["lr"].fill_(float(g["lr"]))
            g["lr"] = og["lr"]
    for g in optimizer.param_groups:
        if not (g.get("fused") or g.get("capturable")):
            continue
        # torch placed each state['step'] from the SAVED groups' flags: a plain (non-fused,
        # non-capturable) AdamW checkpoint -- the reference's (src/training/train_full_model.py:56-57)
        # -- leaves them as CPU scalars, which a fused / capturable step cannot use (and a captured
        # graph would not record the CPU increment).  Move them next to their parameters.
        for p in g["params"]:
            st = optimizer.state.get(p)
            if st and isinstance(st.get("step"), torch.Tensor) and st["step"].device != p.device:
                st["step"] = st["step"].to(p.device, torch.float32)
    for p, st in optimizer.state.items():
        old = old_state.get(p, {})
        for k, v in list(st.items()):
            o = old.get(k)
            if isinstance(v, torch.Tensor) and isinstance(o, torch.Tensor) and o.shape == v.shape:
                o.copy_(v)
                st[k] = o
            elif isinstance(v, torch.Tensor) and v.shape == p.shape and v.dim() == 4 and v.stride() != p.stride():
                # a reference checkpoint holds contiguous moments; the model is channels_last: re-lay
                # them like their parameter (ogv_clip_adamw walks parameter, gradient and moments with
                # one index, and otherwise falls back to torch every step)
                st[k] = torch.empty_like(p, dtype=v.dtype).copy_(v)


# ------------------------------------------------------------------------------- distributed
def setup_distributed(cpu: bool = False, force_group: bool = False):
    """One process per GPU (torchrun env).  Returns (rank, world, local_rank, device).  The process
    group uses "nccl" (= RCCL over xGMI on ROCm) on HIP devices, "gloo" on the CPU (``cpu=True``
    forces the CPU: bench.py's launcher rehearsal and the world-2 tests).  ``force_group``: create the
    group at world size 1 too (the DP path on one GPU, bench.py --force-dp)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not cpu and torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if (world > 1 or force_group) and not torch.distributed.is_initialized():
        backend = "nccl" if device.type == "cuda" else "gloo"
        torch.distributed.init_process_group(backend=backend, device_id=device if device.type == "cuda" else None)
    return rank, world, local, device


def wrap_ddp(model: nn.Module, device, bucket_cap_mb: float = 8.0):
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return model
    if torch.distributed.get_world_size() == 1:
        return model
    return nn.parallel.DistributedDataParallel(
        model, device_ids=[device.index] if device.type == "cuda" else None, bucket_cap_mb=bucket_cap_mb,
        gradient_as_bucket_view=True, broadcast_buffers=True)


# ------------------------------------------------------------------------------- step
def _dist_world():
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_world_size()
    return 1


class _Bucket:
    """A run of parameters (reverse registration order ~ the order backward produces their
    gradients) whose gradients are all-reduced together as soon as the last one is accumulated."""

    def __init__(self, params, device):
        self.params = params
        self.sizes = [p.numel() for p in params]
        self.flat = torch.zeros(sum(self.sizes), device=device, dtype=torch.float32)
        self.ready = 0
        self.work = None


def _capture_unsupported(e: BaseException) -> bool:
    """True for the error a runtime raises when an operation (here: a collective) cannot be recorded into a
    graph; False for everything else (out of memory, a kernel error, a layout error): those are re-raised."""
    msg = str(e).lower()
    if "out of memory" in msg:
        return False
    return any(k in msg for k in ("capture", "not permitted when stream is capturing", "not supported"))


def agree_status(status: int, device) -> int:
    """max(status) over the ranks of the default process group (status itself without one)."""
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return int(status)
    t = torch.tensor([float(status)], device=device)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return int(t.item())


class Trainer:
    """Holds model/optimizer/schedule; ``step(x, y)`` is one full training iteration
    (src/training/one_epoch_train.py:85-153 without its host syncs).

    ``graphs=True`` (HIP device only): the first ``capture_warmup`` calls run eagerly, the next one
    runs eagerly on a side stream and records the step into hipGraphs, every later call copies its
    batch into trainer-owned input buffers and replays them.  A batch of another shape / dtype (a
    ragged last batch) runs as an eager step instead.

    Non-finite loss (one_epoch_train.py:98-108): on a HIP device the guard is a device flag, no host
    sync -- the fused AdamW skips the update when it is set (``found_inf``: parameters, moments and
    step counts unchanged), and the device step counter that drives the warmup-cosine schedule is
    not advanced, exactly as the reference ``continue``s before ``optimizer.step()`` /
    ``scheduler.step()``.  ``nonfinite_steps`` counts them (reading it syncs).  On the CPU the check
    is the reference's host ``if``.

    With world_size > 1 (pass the bare model, not DDP): parameters and buffers are broadcast from
    rank 0 at start; every step all-reduces the gradients (pre-divided by world size), the float
    buffers (BatchNorm running statistics: rank 0 contributes them, the others zeros, so the sum IS
    rank 0's values -- DDP's ``broadcast_buffers`` riding in the same collective) and the
    non-finite flag (so every rank takes the same skip decision).  Graph mode on RCCL: ``bucket_mb``
    buckets all-reduced inside the step's one graph as backward completes them (``dp_overlap``, default);
    gloo / ``dp_overlap=False``: graph A (fwd + bwd + flatten into one bucket) -> one all_reduce -> graph B
    (unflatten + clip + AdamW); eager mode: ``bucket_mb`` buckets all-reduced asynchronously as backward
    produces them."""

    def __init__(self, model: nn.Module, lr=5e-4, weight_decay=0.05, clip=1.0, label_smoothing=0.1,
                 total_steps=10_000, warmup_ratio=0.05, min_lr=1e-6, amp_dtype: Optional[torch.dtype] = torch.bfloat16,
                 graphs: bool = False, capture_warmup: int = 3, capture_hook=None, bucket_mb: float = 8.0,
                 broadcast_buffers: bool = True, defer_reductions: bool = True, native_optimizer: bool = True,
                 force_dp: bool = False, dp_capture_collective: bool = False, label_check_every: int = 100,
                 dp_overlap: Optional[bool] = None):
        self.model = model
        core = model.module if hasattr(model, "module") else model
        self.core = core
        self.ddp = core is not model
        dev = next(core.parameters()).device
        self.device_side = dev.type == "cuda"      # fused AdamW, device guard + schedule
        self.graphs = bool(graphs) and self.device_side
        lr0 = torch.tensor(float(lr), device=dev) if self.device_side else lr
        self.opt = torch.optim.AdamW(param_groups_no_wd(core, weight_decay), lr=lr0, fused=self.device_side,
                                     capturable=self.device_side)
        if self.device_side:
            for g in self.opt.param_groups:     # one device lr tensor per group
                g["lr"] = g["lr"].clone()
        self.sched = WarmupCosineLR(self.opt, total_steps, int(warmup_ratio * total_steps), min_lr)
        self.params = [p for p in core.parameters() if p.requires_grad]
        self.clip, self.ls, self.amp_dtype = clip, label_smoothing, amp_dtype
        # parameter-gradient column reductions batched into one launch at the end of backward
        # (functional.deferred_param_reductions: every .grad is None when backward starts here).  Not
        # under DDP: its reducer copies each gradient into its bucket as AccumulateGrad fires, before
        # the flush has written it (ditto any user hook that reads .grad as soon as it is accumulated).
        hooked = any(getattr(p, "_post_accumulate_grad_hooks", None) for p in core.parameters())
        self.defer_reductions = bool(defer_reductions) and self.device_side and not self.ddp and not hooked
        # clip_grad_norm_ + AdamW.step() as the native ogv_clip_adamw (2 launches per 64 tensors) on
        # the torch optimizer's own state tensors; torch's foreach clip + fused AdamW otherwise
        self.native_optimizer = bool(native_optimizer) and self.device_side
        self.native_optimizer_fallbacks = 0
        self.capture_warmup = int(capture_warmup)
        self.capture_hook = capture_hook          # called right before recording starts
        self._eager_steps = 0
        self.eager_fallbacks = 0
        self._g = None
        self._nonfinite_host = 0
        self.label_check_every = int(label_check_every)
        self._steps_taken = 0
        if self.device_side:
            self._found = torch.zeros((), dtype=torch.float32, device=dev)
            self.opt.found_inf = self._found       # read by the fused AdamW kernel (1 = skip)
            self._nonfinite = torch.zeros((), dtype=torch.float32, device=dev)
            # rows whose class index is outside [0, K) (and not -100): the native loss counts them here;
            # read (one sync, summed over the ranks) after the first step, every label_check_every steps and by
            # check_labels(), raising ValueError as torch's cross_entropy would (a bad label is a data
            # error, not a silently skipped step)
            self._bad_labels = torch.zeros((), dtype=torch.float32, device=dev)
            self.sched.bind_device(torch.zeros((), dtype=torch.float32, device=dev))
        self.world = 1 if self.ddp else _dist_world()
        # the data-parallel path (broadcast at start, gradient / buffer exchange every step); force_dp
        # takes it at world size 1 as well (a world-1 process group: the collective path on one GPU)
        self.dp = self.world > 1 or (bool(force_dp) and not self.ddp)
        if self.dp and not (torch.distributed.is_available() and torch.distributed.is_initialized()):
            raise RuntimeError("Trainer(force_dp=True) needs an initialised torch.distributed process group")
        self.rank = torch.distributed.get_rank() if self.dp else 0
        self.backend = torch.distributed.get_backend() if self.dp else None
        # graph mode: the all_reduce captured INSIDE the step's one graph (RCCL collectives are
        # capturable; gloo's are host work and never are) instead of graph A -> all_reduce -> graph B
        self.dp_capture_collective = bool(dp_capture_collective) and self.dp and self.backend == "nccl"
        # graph mode on RCCL (default): the gradients are all-reduced in ~bucket_mb buckets INSIDE the step's
        # one graph, each launched (asynchronously, on RCCL's stream) as soon as backward has produced its
        # last gradient, overlapping the rest of the backward; the optimizer reads the reduced gradients
        # where the collectives left them (no unflatten).  Needs the Linear weight-gradient fork off (OGV_FORK=0, the default): the
        # bucket's deferred reductions are flushed on the main stream when it completes.
        from .functional import _FORK
        self.dp_overlap = (self.dp and self.graphs and self.backend == "nccl" and not self.dp_capture_collective
                           and not _FORK and (dp_overlap is None or bool(dp_overlap)))
        self._bucket_mb = float(bucket_mb) if bucket_mb and bucket_mb > 0 else 8.0
        self._warned_fallback = False
        if self.dp:
            with torch.no_grad():   # identical start on every rank (what DDP's constructor does)
                for t in list(core.parameters()) + list(core.buffers()):
                    torch.distributed.broadcast(t.data, 0)
            self._bufs = [b for b in core.buffers() if b.is_floating_point()] if broadcast_buffers else []
            self._sizes = [p.numel() for p in self.params]
            self._bsizes = [b.numel() for b in self._bufs]
            self._ng, self._nb = sum(self._sizes), sum(self._bsizes)
            self.flat = torch.zeros(self._ng + self._nb + 1, device=dev, dtype=torch.float32)
            self.meta = torch.zeros(self._nb + 1, device=dev, dtype=torch.float32)
            self._zbuf = torch.zeros(self._nb, device=dev, dtype=torch.float32)   # a non-zero rank's buffer share
            self._buckets = []
            self._overlap = False
            if bucket_mb and bucket_mb > 0 and not self.graphs:
                self._make_buckets(float(bucket_mb), dev)

    # -- data-parallel buckets (eager mode) ----------------------------------------------------
    def _make_buckets(self, bucket_mb, dev):
        cap = int(bucket_mb * 2 ** 20) // 4
        cur, n = [], 0
        for p in reversed(self.params):
            if cur and n + p.numel() > cap:
                self._buckets.append(_Bucket(cur, dev))
                cur, n = [], 0
            cur.append(p)
            n += p.numel()
        if cur:
            self._buckets.append(_Bucket(cur, dev))
        self._bucket_of = {}
        for b in self._buckets:
            for p in b.params:
                self._bucket_of[p] = b
                p.register_post_accumulate_grad_hook(self._grad_ready)

    def _launch_bucket(self, b):
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in b.params]
        torch.cat([g.reshape(-1).float() for g in grads], out=b.flat)
        b.flat.mul_(1.0 / self.world)
        b.work = torch.distributed.all_reduce(b.flat, async_op=True)

    def _grad_ready(self, p):
        if not self._overlap:
            return
        b = self._bucket_of[p]
        b.ready += 1
        if b.ready == len(b.params):
            self._launch_bucket(b)

    # -- pieces of one step -------------------------------------------------------------------
    def _loss(self, x, y):
        """(loss, found_written): the reference's F.cross_entropy(logits.float(), y, label_smoothing)
        (one_epoch_train.py:96) on the native kernel for class-index targets on the device, which also
        writes the step's found_inf guard in the same launch."""
        with torch.autocast("cuda", dtype=self.amp_dtype or torch.float32, enabled=self.amp_dtype is not None,
                            cache_enabled=not self.graphs):
            logits = self.model(x)
        if y.is_floating_point():   # soft targets from MixUp/CutMix (one_epoch_train.py:89-92)
            from .mix import soft_target_cross_entropy
            return soft_target_cross_entropy(logits.float(), y), False
        if logits.is_cuda and logits.dim() == 2 and y.dtype == torch.int64:
            from .functional import cross_entropy_ls
            found = self._found.view(1) if self.device_side else None
            bad = self._bad_labels.view(1) if self.device_side else None
            return cross_entropy_ls(logits, y, self.ls, found=found, bad_labels=bad), found is not None
        return F.cross_entropy(logits.float(), y, label_smoothing=self.ls), False

    def _fwd_bwd(self, x, y):
        loss, flagged = self._loss(x, y)
        if self.device_side and not flagged:
            self._flag(loss.detach(), 0)
        if self.dp and self._overlap:
            self._launch_meta(loss)
        from .functional import deferred_param_reductions
        # not under the eager DP overlap: its bucket hooks read gradients as soon as they are produced
        with deferred_param_reductions(self.defer_reductions and not (self.dp and self._overlap)):
            loss.backward()
        return loss.detach()

    def _meta_values(self, loss):
        """[BatchNorm running buffers | non-finite flag]: rank 0 contributes its buffers, every other
        rank contributes ZEROS (not b * 0: a non-finite running statistic on another rank -- a skipped
        NaN batch still updates them in train mode -- would turn the sum into NaN on every rank)."""
        flag = self._found.view(1) if self.device_side else \
            torch.tensor([0.0 if bool(torch.isfinite(loss)) else 1.0], device=self.flat.device)
        if self.rank == 0:
            return [b.detach().reshape(-1).float() for b in self._bufs] + [flag]
        return [self._zbuf, flag]

    def _launch_meta(self, loss):
        torch.cat(self._meta_values(loss), out=self.meta)
        self._meta_work = torch.distributed.all_reduce(self.meta, async_op=True)

    def _copy_segments(self, segs, scale=1.0):
        """dst <- src * scale (src None: zeros) for every (src, dst, numel) of fp32 device pointers, in
        ceil(n / 64) native launches (ogv_copy_batch_f32) instead of one hipMemcpyAsync per tensor."""
        from . import _lib
        if not segs:
            return
        arr = (_lib.CopySeg * len(segs))(*[_lib.CopySeg(s, d, n) for s, d, n in segs])
        _lib.check(_lib.load().ogv_copy_batch_f32(arr, len(segs), float(scale),
                                                  torch.cuda.current_stream().cuda_stream), "ogv_copy_batch_f32")

    def _flat_offsets(self):
        if getattr(self, "_offs", None) is None:
            offs, o = [], 0
            for n in self._sizes + self._bsizes:
                offs.append(o)
                o += n
            self._offs = offs
        return self._offs

    def _dense_fp32(self, t):
        return (t is not None and t.is_cuda and t.dtype == torch.float32
                and (t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))))

    def _flatten(self, loss):
        """[gradients / world | rank 0's buffers (others: zeros) | non-finite flag] -> self.flat.  On the
        device: batched native copies of every dense fp32 tensor straight from its storage (a dense
        tensor's bytes are its elements in memory order, channels_last included: the unflatten writes
        them back the same way), torch.cat otherwise."""
        # (native copies only when every gradient is laid out like its parameter: the unflatten -- or a rank
        # whose gradient is None, unflattened into empty_like(p) -- then reads the bytes back in the same order)
        if self.device_side and all(p.grad is None or _dense_like(p.grad, p) for p in self.params) \
                and all(self._dense_fp32(b) for b in self._bufs):
            base, esz = self.flat.data_ptr(), 4
            offs = self._flat_offsets()
            segs = [(p.grad.data_ptr() if p.grad is not None else None, base + esz * o, n)
                    for p, o, n in zip(self.params, offs, self._sizes)]
            self._copy_segments(segs, 1.0 / self.world)
            boffs = offs[len(self._sizes):]
            bsegs = [(b.data_ptr() if self.rank == 0 else None, base + esz * o, n)
                     for b, o, n in zip(self._bufs, boffs, self._bsizes)]
            bsegs.append((self._found.data_ptr(), base + esz * (self._ng + self._nb), 1))
            self._copy_segments(bsegs)
            return
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.params]
        torch.cat([g.reshape(-1) for g in grads] + self._meta_values(loss), out=self.flat)
        self.flat[:self._ng].mul_(1.0 / self.world)

    def _apply_meta(self, meta):
        """Copy the all-reduced buffers (= rank 0's) back; returns the all-reduced non-finite count."""
        if self._bufs:
            views = meta[:self._nb].split(self._bsizes)
            with torch.no_grad():
                torch._foreach_copy_(self._bufs, [v.view_as(b) for v, b in zip(views, self._bufs)])
        return meta[self._nb:]

    def _unflatten(self):
        for p in self.params:
            if p.grad is None:
                p.grad = torch.empty_like(p)
        if self.device_side and all(_dense_like(p.grad, p) for p in self.params) \
                and all(self._dense_fp32(b) for b in self._bufs):
            base, esz = self.flat.data_ptr(), 4
            offs = self._flat_offsets()
            segs = [(base + esz * o, p.grad.data_ptr(), n) for p, o, n in zip(self.params, offs, self._sizes)]
            segs += [(base + esz * o, b.data_ptr(), n) for b, o, n in zip(self._bufs, offs[len(self._sizes):], self._bsizes)]
            self._copy_segments(segs)
            return self.flat[self._ng + self._nb:]
        views = [v.view_as(p) for v, p in zip(self.flat[:self._ng].split(self._sizes), self.params)]
        torch._foreach_copy_([p.grad for p in self.params], views)
        return self._apply_meta(self.flat[self._ng:])

    def _finish_buckets(self):
        for b in self._buckets:
            if b.work is None:          # parameters that got no gradient this step
                self._launch_bucket(b)
        for b in self._buckets:
            b.work.wait()
            views = b.flat.split(b.sizes)
            for p, v in zip(b.params, views):
                if p.grad is None:
                    p.grad = torch.empty_like(p)
            torch._foreach_copy_([p.grad for p in b.params], [v.view_as(p) for v, p in zip(views, b.params)])
            b.ready, b.work = 0, None
        self._meta_work.wait()
        return self._apply_meta(self.meta)

    def _flag(self, x, mode):
        """_found = !isfinite(x) (mode 0, x = the fp32 loss) or x > 0 (mode 1, x = the all-reduced
        count of non-finite ranks): one native launch, no host sync."""
        from . import _lib
        x = x.reshape(1).float().contiguous()
        _lib.check(_lib.load().ogv_step_flag(x.data_ptr(), mode, self._found.data_ptr(),
                                             torch.cuda.current_stream().cuda_stream), "ogv_step_flag")

    def _update(self, flag=None):
        """clip + AdamW + schedule.  Device side: gated by the found_inf flag with no host sync."""
        if self.device_side:
            if flag is not None:
                self._flag(flag, 1)
            if not (self.native_optimizer and self._native_clip_adamw()):
                if self.native_optimizer and not self._warned_fallback:
                    import warnings
                    self._warned_fallback = True
                    warnings.warn("ogv_clip_adamw declined this optimizer state (a moment tensor not laid out like "
                                  "its parameter, > 4 groups, amsgrad / maximize, or a non-device lr): running "
                                  "torch's clip_grad_norm_ + fused AdamW instead", RuntimeWarning, stacklevel=3)
                if self.clip is not None:
                    torch.nn.utils.clip_grad_norm_(self.params, self.clip, foreach=True)
                self.opt.step()                               # skipped entirely when _found == 1
            # nonfinite += found; the schedule's step counter advances on applied steps only
            self.sched.device_step(self._found, self._nonfinite)
            return
        if flag is not None and float(flag.view(())) > 0:   # host check: CPU only (no device to sync)
            self._nonfinite_host += 1
            self.opt.zero_grad(set_to_none=True)
            return
        if self.clip is not None:
            torch.nn.utils.clip_grad_norm_(self.params, self.clip, foreach=True)
        self.opt.step()
        self.sched.step()

    def _native_clip_adamw(self) -> bool:
        """clip_grad_norm_(params, clip) + AdamW.step() through ogv_clip_adamw (include/ogv.h), on the
        state tensors torch's AdamW(fused, capturable) keeps (created here on the first step exactly as
        its _init_group does, so state_dict / load_state_dict are unchanged).  Returns False (and the
        caller runs the torch path) when some tensor is not dense with the parameter's strides."""
        from . import _lib
        opt = self.opt
        ents, groups = [], []
        for gi, g in enumerate(opt.param_groups):
            if g.get("amsgrad") or g.get("maximize") or len(opt.param_groups) > 4:
                self.native_optimizer_fallbacks += 1
                return False
            b1, b2 = g["betas"]
            lr = g["lr"]
            if not (torch.is_tensor(lr) and lr.is_cuda and lr.dtype == torch.float32):
                self.native_optimizer_fallbacks += 1
                return False
            groups.append(_lib.AdamWGroup(lr.data_ptr(), float(g["weight_decay"]), float(b1), float(b2), float(g["eps"]),
                                          1.0 - float(b1), 1.0 - float(b2)))
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = opt.state[p]
                if len(st) == 0:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                ts = (p, p.grad, st["exp_avg"], st["exp_avg_sq"])
                if not all(_dense_like(t, p) for t in ts) \
                        or st["step"].dtype != torch.float32 or not st["step"].is_cuda:
                    self.native_optimizer_fallbacks += 1
                    return False
                ents.append(_lib.AdamWTensor(p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                             st["exp_avg_sq"].data_ptr(), st["step"].data_ptr(), p.numel(), gi))
        if not ents:
            return True
        lib = _lib.load()
        tarr = (_lib.AdamWTensor * len(ents))(*ents)
        garr = (_lib.AdamWGroup * len(groups))(*groups)
        nbytes = lib.ogv_clip_adamw_ws_bytes(tarr, len(ents))
        ws = torch.empty(nbytes // 4, dtype=torch.float32, device=self._found.device)
        _lib.check(lib.ogv_clip_adamw(tarr, len(ents), garr, len(groups), self._found.data_ptr(),
                                      float(self.clip) if self.clip is not None else -1.0, ws.data_ptr(),
                                      torch.cuda.current_stream().cuda_stream), "ogv_clip_adamw")
        return True

    def _allreduce(self):
        torch.distributed.all_reduce(self.flat)

    def _agree(self, status: int) -> int:
        """The largest status over the ranks (0 ok, 1 capture unsupported, 2 any other failure): one small
        all_reduce outside any capture, so every rank takes the same capture decision."""
        return agree_status(status, self._found.device if self.backend == "nccl" else torch.device("cpu"))

    # -- graph mode on RCCL: bucketed collectives captured on a side stream, overlapping backward ------
    def _overlap_setup(self, dev):
        """Buckets of ~bucket_mb in reverse registration order (~ the order backward finishes them) laid
        out back to back in self.gflat, then [rank 0's buffers | non-finite flag]; per parameter a view of
        its slot with the parameter's strides (what the optimizer reads after the collectives)."""
        cap = int(self._bucket_mb * 2 ** 20) // 4
        order = list(range(len(self.params)))[::-1]
        self._gbuckets, cur, n = [], [], 0
        for i in order:
            if cur and n + self._sizes[i] > cap:
                self._gbuckets.append(cur)
                cur, n = [], 0
            cur.append(i)
            n += self._sizes[i]
        if cur:
            self._gbuckets.append(cur)
        # every slot starts on a 256-B boundary, as the allocator's own gradient tensors do (the native
        # optimizer takes its float4 path on 16-B aligned tensors: the same arithmetic as without DP)
        al = lambda v: (v + 63) // 64 * 64  # noqa: E731
        self._goff, self._gbrange, o = [0] * len(self.params), [], 0
        self._gbucket_of = {}
        for bi, b in enumerate(self._gbuckets):
            o0 = o
            for i in b:
                self._goff[i] = o
                self._gbucket_of[i] = bi
                o = al(o + self._sizes[i])
            self._gbrange.append((o0, o))
        self._gng = o                        # gradient part incl. alignment padding (zeros)
        self.gflat = torch.zeros(self._gng + self._nb + 1, device=dev, dtype=torch.float32)
        self._gviews = [torch.as_strided(self.gflat, p.shape, p.stride(), self._goff[i])
                        for i, p in enumerate(self.params)]

    def _overlap_launch(self, segs, lo, hi, scale):
        """Pack segs into gflat[lo:hi] (x scale) on the current stream, then all_reduce that slice
        asynchronously -- ProcessGroupNCCL runs it on RCCL's own stream behind an event on this one, so the
        collective overlaps the rest of the backward -- waited for at the end of backward.  (Packing AND
        reducing on a side stream of our own measured 0.8 ms slower per 7M step at world 1, the pack then
        competing with the backward's kernels; this form: world-1 overhead 0.09 ms over the non-DP step,
        profiles/r05g_dp_overlap.log.)"""
        self._copy_segments(segs, scale)
        self._gworks.append(torch.distributed.all_reduce(self.gflat[lo:hi], async_op=True))

    def _overlap_bucket(self, bi):
        base = self.gflat.data_ptr()
        segs = [(self.params[i].grad.data_ptr() if self.params[i].grad is not None else None, base + 4 * self._goff[i],
                 self._sizes[i]) for i in self._gbuckets[bi]]
        for i in self._gbuckets[bi]:
            g = self.params[i].grad
            if g is not None:
                if not _dense_like(g, self.params[i]):
                    raise RuntimeError(f"Trainer(dp_overlap): gradient of parameter {i} is not laid out like the "
                                       f"parameter (strides {tuple(g.stride())} vs {tuple(self.params[i].stride())})")
                self._glocal.append(g)          # the graph keeps reading it: hold it past the capture
        self._gdone[bi] = True
        lo, hi = self._gbrange[bi]
        self._overlap_launch(segs, lo, hi, 1.0 / self.world)

    def _overlap_ready(self, p):
        i = self._pidx[p]
        bi = self._gbucket_of[i]
        self._gseen[bi].add(i)                  # (a set: a parameter used twice fires twice)
        if len(self._gseen[bi]) == len(self._gbuckets[bi]) and not self._gdone[bi]:
            from .functional import flush_deferred_reductions
            flush_deferred_reductions()         # this bucket's parameter gradients are final from here on
            self._overlap_bucket(bi)

    def _fwd_bwd_overlap(self, x, y):
        """_fwd_bwd with the gradient buckets all-reduced as backward completes them (graph capture only)."""
        dev = self._found.device
        if getattr(self, "gflat", None) is None:
            self._overlap_setup(dev)
        self._pidx = {p: i for i, p in enumerate(self.params)}
        self._gseen = [set() for _ in self._gbuckets]
        self._gdone = [False] * len(self._gbuckets)
        self._glocal = []
        self._gworks = []
        loss, flagged = self._loss(x, y)
        if not flagged:
            self._flag(loss.detach(), 0)
        # [rank 0's BatchNorm buffers (final after the forward) | non-finite flag]: launched right away
        base = self.gflat.data_ptr() + 4 * self._gng
        boffs = [0]
        for n in self._bsizes:
            boffs.append(boffs[-1] + n)
        msegs = [(b.data_ptr() if self.rank == 0 else None, base + 4 * o, n)
                 for b, o, n in zip(self._bufs, boffs, self._bsizes)]
        msegs.append((self._found.data_ptr(), base + 4 * self._nb, 1))
        self._overlap_launch(msegs, self._gng, self._gng + self._nb + 1, 1.0)
        hooks = [p.register_post_accumulate_grad_hook(self._overlap_ready) for p in self.params]
        from .functional import deferred_param_reductions
        try:
            with deferred_param_reductions(self.defer_reductions):
                loss.backward()
        finally:
            for h in hooks:
                h.remove()
        for bi in range(len(self._gbuckets)):      # parameters that got no gradient: their slots are zeroed
            if not self._gdone[bi]:
                self._overlap_bucket(bi)
        for w in self._gworks:
            w.wait()
        self._gworks = []
        return loss.detach()

    def _overlap_finish(self):
        """After the collectives: every parameter's .grad is its view of the reduced buffer (the optimizer,
        clip and the caller read the all-reduced gradients there), rank 0's buffers copied back; returns the
        all-reduced non-finite count."""
        for p, v in zip(self.params, self._gviews):
            p.grad = v
        base = self.gflat.data_ptr() + 4 * self._gng
        segs, o = [], 0
        for b, n in zip(self._bufs, self._bsizes):
            segs.append((base + 4 * o, b.data_ptr(), n))
            o += n
        self._copy_segments(segs)
        return self.gflat[self._gng + self._nb:]

    def _eager(self, x, y):
        self.opt.zero_grad(set_to_none=True)
        if self.dp and self._buckets:
            self._overlap = True
            try:
                loss = self._fwd_bwd(x, y)
            finally:
                self._overlap = False
            self._update(self._finish_buckets())
            return loss
        loss = self._fwd_bwd(x, y)
        flag = None
        if self.dp:
            self._flatten(loss)
            self._allreduce()
            flag = self._unflatten()
        elif not self.device_side:
            flag = torch.tensor([0.0 if bool(torch.isfinite(loss)) else 1.0])
        self._update(flag)
        return loss

    def _capture(self, x, y):
        """This call's update runs eagerly on a side stream (allocator / library warm-up, as graph
        capture requires); then the step is recorded on trainer-owned copies of the batch --
        recording executes nothing."""
        # the warm-up step below allocates on a side stream, which cannot reuse blocks cached for the current one:
        # hand those back first (and the side stream's before recording, below), so at most one step's activations
        # are reserved at any time
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            loss = self._eager(x, y)
        torch.cuda.current_stream().wait_stream(side)
        loss = loss.clone()
        # (the layout of each gradient the backward produced, checked below before recording the DP overlap)
        bad_layout = [i for i, p in enumerate(self.params) if p.grad is not None and not _dense_like(p.grad, p)]
        strides = {i: (tuple(self.params[i].grad.stride()), tuple(self.params[i].stride())) for i in bad_layout[:1]}
        self.opt.zero_grad(set_to_none=True)
        # the graph records into a private memory pool: hand the eager steps' cached blocks back first, so the
        # step's activations are not reserved twice (Model-A-22M at 224^2, bs 128: 286 of 288 GB reserved with the
        # eager pool kept, round 5)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        self._x = x.detach().clone(memory_format=torch.preserve_format)
        self._y = y.detach().clone()
        if self.capture_hook is not None:
            self.capture_hook()
        pool = torch.cuda.graph_pool_handle()
        self._g = torch.cuda.CUDAGraph()
        # RCCL: ProcessGroupNCCL's watchdog thread polls the events of earlier collectives while this
        # thread captures; under the default "global" capture mode that poll is a capture-unsupported
        # call from another thread (hipErrorStreamCaptureUnsupported -> abort), so capture thread-locally
        mode = "thread_local" if self.backend == "nccl" else "global"
        if self.dp_overlap:
            # every gradient must be laid out like its parameter for the in-place reduced views: checked on the
            # warm-up step's gradients before recording (a layout error raised mid-capture would leave earlier
            # buckets' collectives recorded on this rank only)
            if bad_layout:
                i = bad_layout[0]
                raise RuntimeError(f"Trainer(dp_overlap): gradient of parameter {i} is not laid out like the "
                                   f"parameter (strides {strides[i][0]} vs {strides[i][1]})")
            status, err = 0, None
            try:
                with torch.cuda.graph(self._g, pool=pool, capture_error_mode=mode):
                    self._loss_static = self._fwd_bwd_overlap(self._x, self._y)
                    self._update(self._overlap_finish())
            except RuntimeError as e:
                status, err = (1 if _capture_unsupported(e) else 2), e
            # one decision for every rank: a rank that recorded the bucketed graph must not replay it
            # while another records the flat form -- their collective sequences would no longer match
            agreed = self._agree(status)
            if agreed == 0:
                self.graph_grads = [p.grad for p in self.params]   # views of the reduced-gradient buffer
                return loss
            if agreed == 2:
                if err is not None and status == 2:
                    raise err
                raise RuntimeError("Trainer: graph capture of the step failed on another rank")
            # a runtime that cannot record collectives into a graph: record the flat form instead -- one
            # all_reduce between two graphs, outside any capture -- rather than end the job
            import warnings
            warnings.warn(f"Trainer: capturing the bucketed all-reduces failed ({err if err is not None else 'on another rank'}); "
                          f"using the flat all-reduce between two graphs instead", RuntimeWarning, stacklevel=3)
            torch.cuda.synchronize()
            self.dp_overlap = False
            self._gworks, self._glocal = [], []
            self.opt.zero_grad(set_to_none=True)
            self._g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g, pool=pool, capture_error_mode=mode):
            self._loss_static = self._fwd_bwd(self._x, self._y)
            if self.dp:
                self._flatten(self._loss_static)
                if self.dp_capture_collective:
                    self._allreduce()
                    self._update(self._unflatten())
            else:
                self._update()
        self.graph_grads = [p.grad for p in self.params]   # the tensors the replays write
        if self.dp and not self.dp_capture_collective:
            self._g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g2, pool=pool, capture_error_mode=mode):
                self._update(self._unflatten())
        return loss

    def release_graphs(self):
        """Drop the recorded step graph(s) and the tensors only they hold (their private memory pool can
        then be returned with torch.cuda.empty_cache()); the trainer state -- parameters, moments, schedule
        -- is untouched and the next step() records the graph again."""
        for name in ("_g", "_g2"):
            g = getattr(self, name, None)
            if g is not None:
                g.reset()
            setattr(self, name, None)
        self._loss_static = None
        self.graph_grads = None
        self._gworks, self._glocal = [], []
        if getattr(self, "gflat", None) is not None:    # allocated inside the capture: re-made by the next one
            self.gflat, self._gviews = None, None
        self.opt.zero_grad(set_to_none=True)
        self._eager_steps = max(self._eager_steps, self.capture_warmup)

    def _replayable(self, x, y) -> bool:
        return (x.shape == self._x.shape and x.dtype == self._x.dtype and x.device == self._x.device
                and y.shape == self._y.shape and y.dtype == self._y.dtype and y.device == self._y.device)

    def step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        loss = self._step(x, y)
        self._steps_taken += 1
        if self.device_side and (self._steps_taken == 1 or (self.label_check_every > 0
                                                            and self._steps_taken % self.label_check_every == 0)):
            self.check_labels()
        return loss

    def check_labels(self):
        """Raise ValueError if any step so far had a class index outside [0, num_classes) other than -100
        (the native loss counts them on the device; torch's cross_entropy raises on the first such batch).
        One host sync; Trainer.step calls it after the first step and every ``label_check_every`` steps."""
        if self.device_side:
            bad = self._bad_labels
            if self.dp:   # every rank raises at the same check (a lone rank raising would leave the others
                bad = bad.detach().clone().reshape(1)          # blocked in the next step's collectives)
                if self.backend != "nccl":
                    bad = bad.cpu()
                torch.distributed.all_reduce(bad)
            n = int(bad.sum().item())
            if n:
                self._bad_labels.zero_()
                raise ValueError(f"Trainer: {n} target label(s) outside [0, num_classes) (and not -100) since the "
                                 f"last check; those steps were skipped (loss NaN) -- torch's cross_entropy raises "
                                 f"on such targets")

    def _step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        if not self.graphs or (self._g is None and self._eager_steps < self.capture_warmup):
            self._eager_steps += 1
            return self._eager(x, y)
        if self._g is None:
            return self._capture(x, y)
        if not self._replayable(x, y):      # e.g. a ragged last batch: same state, plain launches
            self.eager_fallbacks += 1
            return self._eager(x, y)
        self._x.copy_(x)
        self._y.copy_(y)
        self._g.replay()
        if self.dp and not self.dp_capture_collective and not self.dp_overlap:
            self._allreduce()
            self._g2.replay()
        return self._loss_static.clone()

    @property
    def nonfinite_steps(self) -> int:
        """Steps skipped by the non-finite guard so far (one host sync; no side effects)."""
        return int(self._nonfinite.item()) if self.device_side else self._nonfinite_host

    @property
    def bad_label_count(self) -> int:
        """This rank's rows with a class index outside [0, K) (and not -100) since the last check_labels()
        (one host sync; no side effects -- check_labels() raises and resets)."""
        return int(self._bad_labels.item()) if self.device_side else 0

    # -- checkpoint / resume (src/training/chekpoints.py dict keys) -----------------------------
    def state_dict(self):
        """Checkpoint dict (src/training/chekpoints.py keys).  Model tensors are cloned: the Outlooker's
        v / attn parameters are views into one padded [ld, C] buffer (_AliasedConcat), and a state dict
        of shared-storage views would make torch.save write the whole padded buffer and safetensors-style
        writers refuse it."""
        model = {k: v.detach().clone() for k, v in self.core.state_dict().items()}
        return {"model": model, "optimizer": self.opt.state_dict(), "scheduler": self.sched.state_dict()}

    def load_state_dict(self, sd):
        """In place: a recorded graph keeps reading the same parameter / moment / lr tensors."""
        self.core.load_state_dict(sd["model"])
        if sd.get("optimizer") is not None:
            load_optimizer_state(self.opt, sd["optimizer"])
        if sd.get("scheduler") is not None:
            self.sched.load_state_dict(sd["scheduler"])
