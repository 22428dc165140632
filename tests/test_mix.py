"""Batch mixing (src/training/cutmix_mixup_aug.py:17-64): host draw order + oracle pinned to the
reference's recorded outputs on CPU; the native kernels (ogv_mix_images / ogv_mix_targets) against
the same fixtures on the GPU.  Integer/selection work and fp32 blends: bit-exact."""
import random

import numpy as np
import pytest
import torch

import _fixtures as fx
import gen_params as gp
import ogv_oracle as orc
from ogv.mix import draw_mix_plan

MIX = fx.fixture_names("mix_")


def _case(name):
    meta, arr = fx.load(name)
    x = torch.from_numpy(gp.input_from_spec(meta["x"]))
    if meta["channels_last"]:
        x = x.contiguous(memory_format=torch.channels_last)
    return meta, arr, x, torch.from_numpy(arr["targets"])


def _plan(meta, device="cpu"):
    random.seed(meta["seed"])
    torch.manual_seed(meta["seed"])
    return draw_mix_plan(meta["B"], meta["H"], meta["W"], meta["mixup_alpha"], meta["cutmix_alpha"], meta["prob"],
                         device=device)


@pytest.mark.parametrize("name", MIX)
def test_host_draws_and_oracle_match_reference(name):
    meta, arr, x, t = _case(name)
    p = _plan(meta)
    out, soft = orc.mix_apply(x, t, meta["num_classes"], p.mix, p.cutmix, p.perm, p.lam, p.box)
    np.testing.assert_array_equal(out.contiguous().numpy(), arr["images_aug"])
    np.testing.assert_array_equal(soft.numpy(), arr["targets_soft"])


def test_fixture_set_covers_every_branch():
    kinds = set()
    for name in MIX:
        meta, _ = fx.load(name)
        p = _plan(meta)
        kinds.add("off" if not p.mix else ("cutmix" if p.cutmix else "mixup"))
    assert kinds == {"off", "cutmix", "mixup"}


@pytest.mark.gpu
@pytest.mark.parametrize("name", MIX)
@pytest.mark.parametrize("fmt", ["recorded", "nchw", "channels_last"])
def test_kernel_matches_reference(name, fmt):
    from ogv.mix import apply_plan
    meta, arr, x, t = _case(name)
    p = _plan(meta)                      # CPU generator, as the fixture was recorded
    xd = x.to("cuda")
    if fmt == "nchw":
        xd = xd.contiguous()
    elif fmt == "channels_last":
        xd = xd.contiguous(memory_format=torch.channels_last)
    out, soft = apply_plan(xd, t.to("cuda"), meta["num_classes"], p)
    np.testing.assert_array_equal(out.contiguous().cpu().numpy(), arr["images_aug"])
    np.testing.assert_array_equal(soft.cpu().numpy(), arr["targets_soft"])


@pytest.mark.gpu
def test_kernel_bf16_and_full_size_properties():
    """bs=512 CIFAR batch: CutMix output is a per-pixel selection of x / x[perm] (exact), MixUp is
    within one bf16 rounding of the fp32 blend, soft targets sum to 1."""
    from ogv.mix import MixPlan, apply_plan
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(512, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    t = torch.randint(0, 100, (512,), device="cuda", generator=g)
    perm = torch.randperm(512, device="cuda", generator=g)
    out, soft = apply_plan(x, t, 100, MixPlan(True, True, perm, 0.75, (4, 20, 9, 25)))
    ref = x.clone()
    ref[:, :, 4:20, 9:25] = x[perm, :, 4:20, 9:25]
    assert torch.equal(out, ref)
    torch.testing.assert_close(soft.sum(1), torch.ones(512, device="cuda"), rtol=0, atol=1e-6)
    xb = x.to(torch.bfloat16)
    out, _ = apply_plan(xb, t, 100, MixPlan(True, False, perm, 0.3))
    ref = (xb.float() * 0.3 + xb[perm].float() * 0.7).to(torch.bfloat16)
    assert (out.float() - ref.float()).abs().max().item() <= 2 ** -7 * ref.float().abs().max().item()


@pytest.mark.gpu
def test_out_of_range_label_gives_nan_row():
    """F.one_hot raises on a label outside [0, K); the kernel cannot raise without a sync, so the
    row turns NaN (the loss goes non-finite and the Trainer's device guard skips the step)."""
    from ogv.mix import MixPlan, apply_plan
    x = torch.randn(4, 3, 8, 8, device="cuda")
    t = torch.tensor([1, -100, 3, 10], device="cuda")
    perm = torch.tensor([1, 0, 3, 2], device="cuda")
    _, soft = apply_plan(x, t, 10, MixPlan(True, False, perm, 0.6))
    bad = ~torch.isfinite(soft).all(1)
    assert bad.tolist() == [True, True, True, True]     # every row touches label -100 or 10
    _, soft = apply_plan(x, torch.tensor([1, 2, 3, 10], device="cuda"), 10, MixPlan(False, False, None, 1.0))
    assert (~torch.isfinite(soft).all(1)).tolist() == [False, False, False, True]


def test_cpu_tensor_refused():
    from ogv.mix import MixPlan, apply_plan
    with pytest.raises(RuntimeError, match="HIP device"):
        apply_plan(torch.zeros(2, 3, 4, 4), torch.zeros(2, dtype=torch.long), 10,
                   MixPlan(True, False, torch.tensor([1, 0]), 0.5))
