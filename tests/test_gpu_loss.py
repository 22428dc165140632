"""The native training loss (ogv_ce_ls_fwd / _bwd) against the reference's own call,
F.cross_entropy(logits.float(), targets, label_smoothing=ls) (src/training/one_epoch_train.py:96),
in fp64 on the same inputs: loss and dlogits, label smoothing 0 / 0.1 / 1, the class counts of
the three Model-A configs, ignore_index rows, and a label outside [0, K) (NaN loss, found = 1)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [(512, 100, 0.1), (256, 200, 0.1), (128, 1000, 0.1), (3, 7, 0.0), (1, 100, 1.0), (64, 100, 0.0),
         (1000, 37, 0.3)]


@pytest.mark.parametrize("B,K,ls", CASES)
def test_cross_entropy_ls_matches_torch(B, K, ls):
    from ogv.functional import cross_entropy_ls
    g = torch.Generator().manual_seed(B * 7 + K)
    z = (torch.randn(B, K, generator=g) * 3).float()
    y = torch.randint(0, K, (B,), generator=g)
    zr = z.double().requires_grad_()
    ref = F.cross_entropy(zr, y, label_smoothing=ls)
    ref.backward(torch.tensor(2.5, dtype=torch.float64))
    zd = z.to(DEV).requires_grad_()
    found = torch.full((1,), 7.0, device=DEV)
    loss = cross_entropy_ls(zd, y.to(DEV), ls, found=found)
    (loss * 2.5).backward()
    assert abs(loss.item() - ref.item()) <= 2e-6 * max(1.0, abs(ref.item()))
    torch.testing.assert_close(zd.grad.double().cpu(), zr.grad, rtol=0, atol=2e-7 * 2.5)
    assert found.item() == 0.0


def test_cross_entropy_ls_ignore_index_and_bad_label():
    from ogv.functional import cross_entropy_ls
    B, K = 16, 100
    g = torch.Generator().manual_seed(3)
    z = torch.randn(B, K, generator=g)
    y = torch.randint(0, K, (B,), generator=g)
    y[[2, 5, 11]] = -100
    zr = z.double().requires_grad_()
    ref = F.cross_entropy(zr, y, label_smoothing=0.1)
    ref.backward()
    zd = z.to(DEV).requires_grad_()
    loss = cross_entropy_ls(zd, y.to(DEV), 0.1)
    loss.backward()
    assert abs(loss.item() - ref.item()) <= 2e-6 * max(1.0, abs(ref.item()))
    torch.testing.assert_close(zd.grad.double().cpu(), zr.grad, rtol=0, atol=2e-7)
    assert (zd.grad[[2, 5, 11]] == 0).all()
    # a label outside [0, K): torch raises; the native loss is NaN and the step guard is set
    y2 = y.clone()
    y2[0] = K
    y2[7] = -5
    found = torch.zeros(1, device=DEV)
    nbad = torch.full((1,), 2.0, device=DEV)       # the counter accumulates
    bad = cross_entropy_ls(z.to(DEV), y2.to(DEV), 0.1, found=found, bad_labels=nbad)
    assert torch.isnan(bad).item() and found.item() == 1.0 and nbad.item() == 4.0
    # ignored rows are not bad labels, and a NaN logit alone sets found but counts no bad label
    z3 = z.clone()
    z3[4, 9] = float("nan")
    found.zero_()
    nbad.zero_()
    l3 = cross_entropy_ls(z3.to(DEV), y.to(DEV), 0.1, found=found, bad_labels=nbad)
    assert torch.isnan(l3).item() and found.item() == 1.0 and nbad.item() == 0.0


@pytest.mark.parametrize("graphs", [False, True], ids=["eager", "graph"])
def test_trainer_raises_on_bad_labels(graphs):
    """a label outside [0, K) must not be skipped silently -- the Trainer raises ValueError (as
    torch's cross_entropy does) at its next label check: after the first step, every label_check_every
    steps, and whenever check_labels() is called; reading nonfinite_steps / bad_label_count has no side
    effects."""
    from ogv.train import Trainer
    from src.Model_A_OutGridNet import MaxOutNet
    from src.stage_config import StageCfg
    torch.manual_seed(0)
    m = MaxOutNet(10, [StageCfg(dim=48, depth=1, num_heads=2, grid_size=4, outlook_heads=2)], 3, 32, 0.0)
    m = m.to(DEV).to(memory_format=torch.channels_last).train()
    t = Trainer(m, graphs=graphs, capture_warmup=1, label_check_every=3)
    x = torch.randn(4, 3, 16, 16, device=DEV).contiguous(memory_format=torch.channels_last)
    y = torch.tensor([1, 2, 3, 4], device=DEV)
    t.step(x, y)                                    # the first-step check passes
    t.step(x, y)
    ybad = torch.tensor([1, 10, 3, 4], device=DEV)  # 10 classes: label 10 is out of range
    with pytest.raises(ValueError, match="outside"):
        t.step(x, ybad)                             # step 3: the periodic check
    assert t.nonfinite_steps == 1                   # the skipped step; the counter was reset by the raise
    assert t.bad_label_count == 0
    t.step(x, ybad)
    assert t.nonfinite_steps == 2 and t.bad_label_count == 1   # metrics: no raise, no reset
    assert t.bad_label_count == 1
    with pytest.raises(ValueError, match="outside"):
        t.check_labels()
    assert t.bad_label_count == 0


def test_cross_entropy_ls_rejects_host_tensors_and_soft_targets():
    from ogv.functional import cross_entropy_ls
    with pytest.raises(RuntimeError, match="HIP device tensors"):
        cross_entropy_ls(torch.randn(2, 3), torch.zeros(2, dtype=torch.int64), 0.1)
    with pytest.raises(ValueError, match="int64"):
        cross_entropy_ls(torch.randn(2, 3, device=DEV), torch.zeros(2, device=DEV), 0.1)
    with pytest.raises(ValueError, match="expected"):   # soft targets [B, K] stay on soft_target_cross_entropy
        cross_entropy_ls(torch.randn(2, 3, device=DEV), torch.zeros(2, 3, device=DEV), 0.1)
