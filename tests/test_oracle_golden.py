"""Pin the CPU oracle (oracle/ogv_oracle.py) to the golden vectors recorded from the reference
implementation itself (tests/golden/make_golden.py).  CPU only, fp32."""
import numpy as np
import pytest
import torch

import _fixtures as fx
import gen_params as gp
import ogv_oracle as orc

torch.set_num_threads(4)
RTOL, ATOL = 2e-5, 2e-5


def _run(meta, fwd):
    x, dy = fx.inputs(meta)
    p = fx.oracle_params(meta)
    xt = torch.from_numpy(x).requires_grad_(True)
    y = fwd(xt, p, meta)
    y.backward(torch.from_numpy(dy))
    grads = {k: t.grad for k, t in p.items() if isinstance(t, torch.Tensor) and t.requires_grad}
    return y, xt.grad, grads, p


def _check(name, fwd):
    meta, arr = fx.load(name)
    y, dx, grads, p = _run(meta, fwd)
    assert fx.maxabs(y.detach(), arr["y"]) <= ATOL + RTOL * np.abs(arr["y"]).max(), name
    assert fx.maxabs(dx, arr["dx"]) <= ATOL + RTOL * np.abs(arr["dx"]).max(), name
    n = fx.compare_grads(grads, arr, 1e-4, 1e-5, name)
    assert n > 0
    for k in arr:
        if k.startswith("buf_after."):
            key = k[len("buf_after."):]
            assert fx.maxabs(p[key], arr[k]) <= 1e-5 * max(1.0, np.abs(arr[k]).max()), (name, key)


@pytest.mark.parametrize("name", fx.fixture_names("outlook_attn_"))
def test_outlook_attention(name):
    _check(name, lambda x, p, m: orc.outlook_attention(x, p, "", m["heads"], m["k"], m.get("stride", 1)))


@pytest.mark.parametrize("name", [n for n in fx.fixture_names("grid_attn_") if "capture" not in n])
def test_grid_attention(name):
    _check(name, lambda x, p, m: orc.grid_attention(x, p, "", m["heads"], m["g"]))


def test_layernorm2d():
    _check("layernorm2d_s0", lambda x, p, m: orc.ln2d(x, p["ln.weight"], p["ln.bias"], m["eps"]))


def test_outlooker_block():
    _check("outlooker_block_s1", lambda x, p, m: orc.outlooker_block(x, p, "", m["heads"]))


@pytest.mark.parametrize("name", fx.fixture_names("mbconv_"))
def test_mbconv(name):
    _check(name, lambda x, p, m: orc.mbconv(x, p, "", m["train"]))


@pytest.mark.parametrize("name", fx.fixture_names("outgrid_block_"))
def test_outgrid_block(name):
    _check(name, lambda x, p, m: orc.outgrid_block(x, p, "", m["stage"], m["train"]))


def test_grid_partition_golden():
    meta, arr = fx.load("grid_partition_g2")
    x = torch.from_numpy(gp.input_from_spec(meta["x"]))
    g = orc.grid_partition(x, meta["g"])
    assert torch.equal(g, torch.from_numpy(arr["grids"]))
    assert torch.equal(orc.grid_unpartition(g, *x.shape[:3], meta["g"]), x)


def test_grid_capture_golden():
    meta, arr = fx.load("grid_attn_capture_s1")
    p = fx.oracle_params(meta, requires_grad=False)
    x = torch.from_numpy(gp.input_from_spec(meta["x"]))
    y, att = orc.grid_attention(x, p, "", meta["heads"], meta["g"], want_probs=True)
    assert fx.maxabs(y, arr["y"]) < 1e-5
    assert fx.maxabs(att, arr["last_attn"]) < 1e-6


MODEL_A_FIXTURES = fx.fixture_names("model_a_")
N_PARAMS = {"7m": 7518102, "14m": 14637698, "22m": 22850628}   # SURVEY.md §2 / §8d, measured on the reference


@pytest.mark.parametrize("name", MODEL_A_FIXTURES)
def test_model_a(name):
    """Model-A-7M (CIFAR 32x32), Model-A-14M (200 classes, 64x64: BASELINE configs[3]) and Model-A-22M
    (1000 classes, 224x224, depth 2/3/4/2: BASELINE configs[4]); B=2 plus the well-conditioned
    train-mode B=16 / B=8 cases: logits, loss, every parameter's gradient norm, and the (sketched)
    first- / last-block weight gradients."""
    meta, arr = fx.load(name)
    mode = meta["mode"]
    p = fx.oracle_params(meta)
    assert list(p.keys()) == list(fx.shapes_for(meta).keys())
    names = [k for k in p if p[k].requires_grad]
    assert names == meta["param_names"], "state_dict parameter order differs from the reference"
    x = torch.from_numpy(gp.input_from_spec(meta["x"]))
    logits = orc.model_a(x, p, meta["stages"], train=(mode == "train"))
    assert fx.maxabs(logits.detach(), arr["logits"]) < 2e-5 * max(1.0, np.abs(arr["logits"]).max())
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(arr["targets"]), label_smoothing=0.1)
    assert abs(loss.item() - arr["loss"][0]) < 2e-6 * max(1.0, arr["loss"][0])
    loss.backward()
    gn = np.array([p[k].grad.norm().item() if p[k].grad is not None else 0.0 for k in names])
    np.testing.assert_allclose(gn, arr["grad_norms"], rtol=2e-4, atol=1e-7)
    fx.compare_grads({k: p[k].grad for k in names}, arr, 1e-4, 1e-6, name)
    n_params = sum(p[k].numel() for k in names)
    assert n_params == meta["n_params"] == N_PARAMS[name.split("_")[2]]


# ---------------------------------------------------------------- Model B family (Grid_Only_Block.py,
# Model_B_OutGridNet.py), recorded by `make_golden.py model_b`
@pytest.mark.parametrize("name", fx.fixture_names("gridonly_block_"))
def test_gridonly_block(name):
    _check(name, lambda x, p, m: orc.gridonly_block(x, p, "", m["stage"], m["train"]))


@pytest.mark.parametrize("name", fx.fixture_names("stage_out_then_grid_"))
def test_stage_out_then_grid(name):
    _check(name, lambda x, p, m: orc.stage_out_then_grid(x, p, "", m["stage"], m["depth"], m["out_depth"],
                                                         m["train"]))


@pytest.mark.parametrize("name", fx.fixture_names("model_b_"))
def test_model_b(name):
    meta, arr = fx.load(name)
    mode = meta["mode"]
    p = fx.oracle_params(meta)
    names = [k for k in p if p[k].requires_grad]
    assert names == meta["param_names"], "state_dict parameter order differs from the reference"
    x = torch.from_numpy(gp.input_from_spec(meta["x"]))
    logits = orc.model_b(x, p, meta["stages"], meta["outlooker_front_depth"], train=(mode == "train"))
    assert fx.maxabs(logits.detach(), arr["logits"]) < 2e-5
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(arr["targets"]), label_smoothing=0.1)
    assert abs(loss.item() - arr["loss"][0]) < 2e-6
    loss.backward()
    gn = np.array([p[k].grad.norm().item() if p[k].grad is not None else 0.0 for k in names])
    np.testing.assert_allclose(gn, arr["grad_norms"], rtol=2e-4, atol=1e-7)
    fx.compare_grads({k: p[k].grad for k in names}, arr, 1e-4, 1e-6, name)
    assert sum(p[k].numel() for k in names) == meta["n_params"]


def test_train_steps_oracle():
    """The oracle's training loop (optimizer, warmup-cosine schedule, clip, non-finite skip) against
    the reference's own train_one_epoch run (fixture train_steps_7m_b16, make_golden.py r4)."""
    meta, arr = fx.load("train_steps_7m_b16")
    _, amp = fx.load("train_steps_7m_b16_amp")
    arr = dict(arr, **{k: v for k, v in amp.items() if k.startswith("pns")})
    shapes = orc.model_a_shapes(meta["stages"], meta["num_classes"], 3, meta["stem_dim"])
    p = orc.make_params(shapes, lambda k, s: gp.param_value(k, s, meta["seed"]))
    assert [k for k, t in p.items() if t.requires_grad] == meta["param_names"]
    p0 = {k: t.detach().clone() for k, t in p.items()}
    rec = []

    def on_step(t, loss, lr_used, skipped, step_num):
        e = fx.train_step_errors(meta, arr, t, {k: p[k] for k in meta["param_names"]}, p0)
        rec.append((t, float(loss), lr_used, skipped, step_num, e))

    orc.train_steps(fx.train_batches(meta), p, meta["stages"], lr=meta["lr"], weight_decay=meta["weight_decay"],
                    clip=meta["clip"], label_smoothing=meta["label_smoothing"], total_steps=meta["total_steps"],
                    warmup_steps=int(meta["total_steps"] * meta["warmup_ratio"]), min_lr=meta["min_lr"],
                    on_step=on_step)
    for t, loss, lr_used, skipped, step_num, e in rec:
        print(t, loss, e)
        assert skipped == bool(arr["skipped"][t])
        assert step_num == arr["sched_step"][t]
        assert lr_used == list(arr["lr_used"][t])
        if not skipped:
            assert abs(loss - arr["loss"][t]) <= 1e-5, (t, loss)
        assert e["upd"] <= 1e-3 and e["dn"] <= 1e-3 and e["norm"] <= 1e-5 and e.get("full", 0.0) <= 1e-6, (t, e)
        # the derived norm bars of tests/test_gpu_train_parity.py hold for two CPU fp32 implementations too
        dn = arr[f"dn{t}"]
        assert (e["pns_abs"] <= 1e-6 * amp[f"pns{t}"] + 2e-3 * dn).all(), t
        assert (e["pn_abs"] <= 1e-6 * arr[f"pn{t}"] + 2e-3 * dn + 2.0 * amp[f"noise{t}"]).all(), t


def test_train_steps_amp_fixture():
    """The bf16 step fixture (make_golden.py r5: the reference's train_one_epoch with use_amp=True) against the
    oracle's training loop under the same CPU bf16 autocast: the same skip / schedule, the first loss to 1e-5
    (same weights, same autocast ops; measured equal), later losses within the bf16 bar 1e-2 * max(1, |loss|)
    (two bf16 runs drift apart after the first Adam step: measured 1.1e-3 and 5.3e-3), and
    the oracle's own bf16-vs-fp32 update deviation of the same size as the reference's (it restates the same
    ops, so both are the one autocast run up to summation order) -- the fixture the GPU bf16 step test
    (tests/test_gpu_train_parity.py) takes its bars from is pinned by a second implementation."""
    meta, arr = fx.load("train_steps_7m_b16")
    mamp, amp = fx.load("train_steps_7m_b16_amp")
    assert mamp["base"] == "train_steps_7m_b16" and mamp["param_names"] == meta["param_names"]
    shapes = orc.model_a_shapes(meta["stages"], meta["num_classes"], 3, meta["stem_dim"])
    p = orc.make_params(shapes, lambda k, s: gp.param_value(k, s, meta["seed"]))
    params = {k: p[k] for k in meta["param_names"]}
    p0 = {k: t.detach().clone() for k, t in params.items()}
    masks = fx.train_stable_masks(meta, arr, params)
    rec = []

    def on_step(t, loss, lr_used, skipped, step_num):
        if skipped:
            rec.append((t, float(loss), skipped, step_num, None, None))
            return
        e = fx.train_step_errors(meta, arr, t, params, p0, masks)
        r = fx.amp_reference_errors(meta, arr, amp, t, params, masks)
        rec.append((t, float(loss), skipped, step_num, e, r))

    orc.train_steps(fx.train_batches(meta), p, meta["stages"], lr=meta["lr"], weight_decay=meta["weight_decay"],
                    clip=meta["clip"], label_smoothing=meta["label_smoothing"], total_steps=meta["total_steps"],
                    warmup_steps=int(meta["total_steps"] * meta["warmup_ratio"]), min_lr=meta["min_lr"],
                    on_step=on_step, autocast=True)
    for t, loss, skipped, step_num, e, r in rec:
        assert skipped == bool(amp["amp_skipped"][t]) and step_num == amp["amp_sched_step"][t]
        if skipped:
            continue
        live = arr[f"dn{t}"] > 0
        med, med_ref = np.median(e["upd_all"][live]), np.median(r["upd_all"][live])
        print(t, loss, float(amp["amp_loss"][t]), med, med_ref, e["dn"], r["dn"])
        assert abs(loss - float(amp["amp_loss"][t])) <= (1e-5 if t == 0 else 1e-2 * max(1.0, abs(loss))), (t, loss)
        assert 0.5 * med_ref <= med <= 1.5 * med_ref, (t, med, med_ref)
