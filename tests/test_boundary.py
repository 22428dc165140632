"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports every symbol
include/ogv.h declares; host-side argument validation returns error codes without touching a
GPU; the module tree has the reference's state_dict keys and error conventions; CPU tensors are
refused (no silent CPU fallback)."""
import ctypes
import pathlib
import re

import pytest
import torch

import _fixtures as fx

ROOT = pathlib.Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "ogv.h"


def _declared():
    txt = HEADER.read_text()
    return sorted(set(re.findall(r"\b(ogv_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    import ogv._lib as L
    lib = L.load()
    declared = _declared()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(L.SIGNATURES), "ctypes signature table out of sync with include/ogv.h"
    assert L.version().startswith("ogv-hip")


def test_host_validation_without_gpu():
    import ogv._lib as L
    lib = L.load()
    # null pointers / bad shapes are rejected before any launch
    rc = lib.ogv_outlook_agg_fwd(None, None, None, 1, 4, 4, 16, 3, 3, 27, 16, 0, None)
    assert rc == 1 and b"null" in lib.ogv_last_error()
    x = ctypes.c_void_p(16)
    rc = lib.ogv_outlook_agg_fwd(x, x, x, 1, 4, 4, 16, 3, 3, 27, 16, 0, None)     # 16 % 3 != 0
    assert rc == 1 and b"divisible" in lib.ogv_last_error()
    rc = lib.ogv_outlook_agg_fwd(x, x, x, 1, 4, 4, 18, 3, 4, 27, 18, 0, None)     # even kernel
    assert rc == 1
    rc = lib.ogv_outlook_agg_fwd(x, x, x, 1, 4, 4, 18, 3, 3, 27, 16, 0, None)     # ld_v < C
    assert rc == 1 and b"ld_v" in lib.ogv_last_error()
    rc = lib.ogv_outlook_agg_bwd(x, x, x, x, x, None, 1, 4, 4, 18, 3, 3, 27, 18, 18, 27, 20, 0, None)  # dl_cols < 27
    assert rc == 1 and b"dl_cols" in lib.ogv_last_error()
    rc = lib.ogv_grid_attn_fwd(x, x, x, None, 1, 6, 6, 16, 2, 4, 1.0, 0, None)  # 6 % 4
    assert rc == 1 and b"divisible" in lib.ogv_last_error()
    rc = lib.ogv_layernorm_fwd(x, None, None, x, None, None, 4, 6, 1e-5, 0, None)  # C % 4
    assert rc == 1
    rc = lib.ogv_gemm_fwd(x, 4, x, None, None, None, 0, x, 8, 16, 8, 8, 0, 0, None)  # lda < K
    assert rc == 1
    # dgrad reads W as [reduction][output] directly (no transposed copy): a fixed small workspace
    assert 0 < lib.ogv_gemm_dgrad_ws_bytes(18, 48) <= 4096
    assert lib.ogv_gemm_wgrad_ws_bytes(524288, 192, 48) > 0
    assert lib.ogv_layernorm_bwd_ws_bytes(1000, 48) > 0


def test_cpu_tensors_are_refused():
    from src.model.outlook_attention import OutlookAttention2d
    m = OutlookAttention2d(16, 4)
    with pytest.raises(RuntimeError, match="HIP device"):
        m(torch.randn(1, 16, 4, 4))


@pytest.mark.parametrize("name", ["outlook_attn_s0", "grid_attn_s1", "layernorm2d_s0", "outlooker_block_s1",
                                  "mbconv_s0_train", "outgrid_block_s2_eval", "outgrid_block_tiny_eval",
                                  "model_a_7m_eval_b2", "gridonly_block_b1_eval", "stage_out_then_grid_eval",
                                  "model_b_eval_b2"])
def test_state_dict_matches_reference_layout(name):
    import test_gpu_parity as tg
    meta, _ = fx.load(name)
    mod = tg._module(meta)
    ours = {k: tuple(v.shape) for k, v in mod.state_dict().items()}
    ref = {k: tuple(s) for k, s in fx.shapes_for(meta).items()}
    assert list(ours) == list(ref)
    assert ours == ref
    if meta["kind"] in ("model_a", "model_b"):
        assert [k for k, _ in mod.named_parameters()] == meta["param_names"]
        assert sum(p.numel() for p in mod.parameters()) == meta["n_params"]


def test_error_conventions():
    from src.model.outlook_attention import OutlookAttention2d, make_activation
    from src.model.grid_attention import GridAttention2D, GridAttention2DConfig, MultiHeadSelfAttention, AttentionConfig
    from src.model.grid_partition import grid_partition, grid_unpartition
    from src.model.Out_Grid_Block import MLP
    from src.model.mbc_conv import MBConv, SqueezeExcite
    with pytest.raises(AssertionError):
        OutlookAttention2d(10, 3)
    with pytest.raises(ValueError):
        OutlookAttention2d(12, 3, kernel_size=4)
    with pytest.raises(ValueError):
        OutlookAttention2d(12, 3, stride=0)
    with pytest.raises(ValueError):
        make_activation("tanh")
    with pytest.raises(ValueError):
        GridAttention2D(GridAttention2DConfig(mode="window", dim=8, num_heads=2, grid_size=2))
    with pytest.raises(ValueError):
        MultiHeadSelfAttention(AttentionConfig(dim=10, num_heads=3))
    with pytest.raises(ValueError):
        grid_partition(torch.zeros(1, 6, 6, 4), 4)
    with pytest.raises(ValueError):
        grid_partition(torch.zeros(6, 6, 4), 2)
    with pytest.raises(ValueError):
        grid_unpartition(torch.zeros(3, 2, 2, 4), (1, 4, 4, 4, 2))
    with pytest.raises(ValueError):
        MBConv(8, 8, stride=3)
    with pytest.raises(ValueError):
        SqueezeExcite(8, se_ratio=0.0)
    mlp = MLP(8)
    with pytest.raises(ValueError):
        mlp(torch.zeros(1, 2, 2, 6))
    g = GridAttention2D(GridAttention2DConfig(mode="grid", dim=8, num_heads=2, grid_size=3))
    with pytest.raises(ValueError):
        g(torch.zeros(1, 4, 4, 8))
    with pytest.raises(ValueError):
        g(torch.zeros(1, 6, 6, 4))


def test_grid_partition_roundtrip_cpu():
    """grid_partition/unpartition are pure index ops (no kernels) kept for analysis code."""
    import gen_params as gp
    from src.model.grid_partition import grid_partition, grid_unpartition
    meta, arr = fx.load("grid_partition_g2")
    x = torch.from_numpy(gp.input_from_spec(meta["x"]))
    grids, m = grid_partition(x, 2)
    assert torch.equal(grids, torch.from_numpy(arr["grids"]))
    assert torch.equal(grid_unpartition(grids, m), x)


def test_make_dpr_matches_reference_formula():
    from src.model.stem_head import make_dpr
    assert make_dpr(1, 0.3) == [0.3]
    assert make_dpr(7, 0.07) == [0.07 * i / 6 for i in range(7)]


def test_build_model_dispatch_matches_reference_aliases():
    """scripts/train.py:33-60: model.type aliases and the unknown-type error (constructed on the host)."""
    from ogv.train import MODEL_CONFIGS, build_model
    from src.Model_A_OutGridNet import MaxOutNet
    from src.Model_B_OutGridNet import OutlookerFrontGridNet
    stages = MODEL_CONFIGS["model_a_7m"]["stages"]
    for t in ("a", "model_a", "maxout", "outgrid"):
        assert isinstance(build_model(dict(type=t, stages=stages)), MaxOutNet)
    for t in ("b", "model_b", "outlooker_front", "front"):
        m = build_model(dict(type=t, stages=stages, outlooker_front_depth=1))
        assert isinstance(m, OutlookerFrontGridNet) and len(m.front) == 1
    with pytest.raises(ValueError, match="Unknown model.type"):
        build_model(dict(type="model_c", stages=stages))
    with pytest.raises(ValueError, match="at least one stage"):
        build_model(dict(type="model_b", stages=[]))


def test_classifier_head_native_path_only_for_plain_gpu_linear():
    """Model_A_OutGridNet.py:65-67 head: the native fp32 GEMM replaces nn.Linear.forward only when
    nothing can observe the difference -- on CPU features, a Linear subclass, or with module / global
    forward hooks the module itself is called (and the CPU result equals the reference's formula)."""
    from torch import nn
    from src.Model_A_OutGridNet import _native_classifier_ok, classifier_head
    lin = nn.Linear(8, 5)
    x = torch.randn(3, 8, 2, 2)
    pooled = x.mean(dim=(2, 3))
    assert not _native_classifier_ok(lin, pooled)                       # CPU tensor
    torch.testing.assert_close(classifier_head(x, lin), lin(pooled))   # runs the module on CPU

    class MyLinear(nn.Linear):
        pass

    fake_cuda = type("T", (), {"is_cuda": True})()
    assert _native_classifier_ok(lin, fake_cuda)
    assert not _native_classifier_ok(MyLinear(8, 5), fake_cuda)
    seen = []
    h = torch.nn.modules.module.register_module_forward_hook(lambda m, i, o: seen.append(type(m)))
    try:
        assert not _native_classifier_ok(lin, fake_cuda)
        classifier_head(x, lin)
        assert nn.Linear in seen                                        # the global hook saw the call
    finally:
        h.remove()
    h = lin.register_forward_pre_hook(lambda m, i: None)
    assert not _native_classifier_ok(lin, fake_cuda)
    h.remove()
    assert _native_classifier_ok(lin, fake_cuda)


def test_head_norm_folds_into_pool_only_when_unobservable():
    """The head BatchNorm2d + pool run as one native op (BN of the per-image means) only for the ogv
    BatchNorm2d itself on the GPU with no hooks; on CPU features the module runs and the result is the
    reference's head_norm -> mean -> classifier."""
    from torch import nn
    from ogv.layers import BatchNorm2d
    from src.Model_A_OutGridNet import _fused_head_norm_ok, classifier_head
    bn, lin = BatchNorm2d(8).eval(), nn.Linear(8, 5)
    x = torch.randn(3, 8, 2, 2)
    fake = type("T", (), {"is_cuda": True, "dim": lambda self: 4})()
    assert _fused_head_norm_ok(bn, fake)
    assert not _fused_head_norm_ok(bn, x)                                 # CPU tensor
    assert not _fused_head_norm_ok(nn.BatchNorm2d(8), fake)               # stock module: its own forward
    h = bn.register_forward_hook(lambda m, i, o: None)
    assert not _fused_head_norm_ok(bn, fake)
    h.remove()
    h = torch.nn.modules.module.register_module_forward_pre_hook(lambda m, i: None)
    try:
        assert not _fused_head_norm_ok(bn, fake)
    finally:
        h.remove()
    ref = nn.BatchNorm2d(8).eval()
    ref.load_state_dict(bn.state_dict())
    with torch.no_grad():
        torch.testing.assert_close(classifier_head(x, lin, ref), lin(ref(x).mean(dim=(2, 3))))


def test_gemm_routing_table():
    """Host-side planner (no GPU): which kernel a bf16 projection runs on (ogv_gemm_stream_route:
    1 streaming, 2 panel, 0 LDS-tiled), on the Model-A-7M shapes and the edges of each route."""
    import ogv._lib as L
    lib = L.load()
    route = lib.ogv_gemm_stream_route
    fwd, dgrad = 0, 1
    assert route(fwd, 524288, 48, 64, 0) == 1              # stage 0: streaming kernel
    assert route(fwd, 524288, 48, 192, 1) == 1             # fc2 with the GELU prologue, K <= 384
    assert route(fwd, 32768, 768, 192, 0) == 2             # stages 1-3: panel kernel
    assert route(fwd, 131072, 384, 96, 0) == 2             # stage 1 (M = 131072): panel since round 4
    assert route(fwd, 262144, 384, 96, 0) == 1             # sgemm_min_m = 262144
    assert route(fwd, 8192, 256, 1024, 1) == 2
    assert route(dgrad, 32768, 768, 192, 1) == 2
    assert route(dgrad, 524288, 256, 1024, 0) == 2         # long-reduction dgrad at large M
    assert route(fwd, 32768, 54, 192, 0) == 0              # N % 8 != 0: LDS-tiled kernel
    assert route(fwd, 32768, 768, 196, 0) == 0             # K % 8 != 0
    assert route(fwd, 32768, 768, 192, 3) == 0             # ReLU prologue: not compiled in the panel kernel
    try:
        assert lib.ogv_set_option(b"pgemm", 0) == 0
        assert route(fwd, 32768, 768, 192, 0) == 0
    finally:
        assert lib.ogv_set_option(b"pgemm", 1) == 0
    for name in (b"pg_rs", b"pg_tn", b"pg_per_cu", b"wg_blocks", b"wg_tile", b"sg_wgs"):
        assert lib.ogv_set_option(name, 0) == 0, name
    assert lib.ogv_set_option(b"pg_per_cu", 8) == 0 and lib.ogv_set_option(b"wg_blocks", 1024) == 0


def test_outlook_vproj_plan_and_knob():
    """Which shapes the fused Outlooker kernels take (host-side plan, no GPU): bf16, k = 3,
    16 | C <= 96, 8 | head_dim, ld = C + 9 heads rounded up to 8; knob outlook_vproj: 0 never,
    1 inference only, 2 also in training with the forward writing cat (default: returns 1 for
    training), 3 training with the recompute backward (returns 2 when ogv_outlook_vproj_bwd takes
    the shape); the tile knob vp_tile forces a candidate; unsupported calls fail before any launch."""
    import ogv._lib as L
    lib = L.load()
    ld = lambda C, h: (C + 9 * h + 7) // 8 * 8  # noqa: E731
    sup = lambda B, H, W, C, h, train, dt=L.OGV_BF16, k=3, l=None: lib.ogv_outlook_vproj_supported(  # noqa: E731
        B, H, W, C, h, k, ld(C, h) if l is None else l, int(train), dt)
    try:
        assert sup(512, 32, 32, 48, 2, False) == 1          # 7M stage 0
        assert sup(512, 16, 16, 96, 3, False) == 1          # 7M stage 1
        assert sup(128, 224, 224, 64, 2, False) == 1        # 22M stage 0
        # wide stages (C > 96) on images of <= 128 pixels: the per-head whole-image kernel (knob vp_head,
        # default on), forward with cat; larger wide-stage images keep the unfused GEMM + aggregation
        for shape in ((512, 8, 8, 192, 6), (512, 4, 4, 256, 8), (3, 5, 11, 128, 4), (256, 8, 8, 384, 12)):
            assert sup(*shape, False) == 1 and sup(*shape, True) == 1, shape
        # head_dim 64 (14M / 22M stage 3): a 125 KB weight slice, one workgroup per CU -- measured slower
        # than the unfused pair, so planned only with vp_head = 2
        assert sup(256, 8, 8, 384, 6, False) == 0 and sup(256, 4, 4, 256, 4, False) == 0
        assert lib.ogv_set_option(b"vp_head", 2) == 0
        assert sup(256, 8, 8, 384, 6, False) == 1 and sup(256, 4, 4, 256, 4, True) == 1
        assert lib.ogv_set_option(b"vp_head", 1) == 0
        assert sup(256, 32, 32, 128, 4, False) == 0         # 14M stage 1: 1024-pixel images
        assert sup(256, 16, 16, 256, 8, False) == 0         # 14M stage 2: 256-pixel images
        assert sup(512, 8, 8, 160, 5, False) == 0           # C = 160: no instantiation (C / 32 = 5)
        assert sup(512, 8, 8, 288, 6, False) == 0           # head_dim 48: the per-head kernel takes 32 / 64
        assert lib.ogv_set_option(b"vp_head", 0) == 0
        assert sup(512, 8, 8, 192, 6, False) == 0           # vp_head off: unfused GEMM + aggregation
        # the weight-streaming variant (opt-in, knob vp_big), forward with cat; no recompute backward
        assert lib.ogv_set_option(b"vp_big", 1) == 0
        for shape in ((512, 8, 8, 192, 6), (512, 4, 4, 256, 8), (256, 32, 32, 128, 4), (128, 14, 14, 384, 6)):
            assert sup(*shape, False) == 1 and sup(*shape, True) == 1, shape
            assert lib.ogv_outlook_vproj_bwd_supported(*shape[:3], shape[3], shape[4], 3, ld(shape[3], shape[4]),
                                                       L.OGV_BF16) == 0
        assert sup(512, 8, 8, 160, 5, False) == 0           # C = 160: no streaming instantiation (32 | C, C / 32 = 5)
        assert sup(512, 8, 8, 512, 4, False) == 0           # head_dim 128 > 64
        assert lib.ogv_set_option(b"vp_big", 0) == 0
        assert lib.ogv_outlook_vproj_bwd_supported(512, 32, 32, 48, 2, 3, ld(48, 2), L.OGV_BF16) == 1
        assert sup(2, 8, 8, 48, 2, False, dt=L.OGV_F32) == 0
        assert sup(2, 8, 8, 48, 2, False, k=5) == 0
        assert sup(2, 8, 8, 40, 5, False) == 0              # head_dim 8 but 16 does not divide C
        assert sup(2, 8, 8, 48, 2, False, l=72 + 8) == 0    # wrong row stride of cat
        assert sup(512, 32, 32, 48, 2, True) == 1           # default: fused forward writing cat in training
        assert lib.ogv_set_option(b"outlook_vproj", 3) == 0
        for shape in ((512, 32, 32, 48, 2), (512, 16, 16, 96, 3), (128, 224, 224, 64, 2), (2, 5, 7, 16, 2)):
            assert sup(*shape, True) == 2, shape            # the recompute backward takes every 7M/14M/22M shape
            assert sup(*shape, False) == 1
        assert lib.ogv_set_option(b"outlook_vproj", 1) == 0
        assert sup(512, 32, 32, 48, 2, True) == 0           # inference only
        assert sup(512, 32, 32, 48, 2, False) == 1
        assert lib.ogv_set_option(b"outlook_vproj", 0) == 0
        assert sup(512, 32, 32, 48, 2, False) == 0
        assert lib.ogv_set_option(b"outlook_vproj", 2) == 0
        assert lib.ogv_set_option(b"vp_tile", 1) == 0       # 8 x 16 at two workgroups per CU: the C = 96
        assert sup(512, 16, 16, 96, 3, False) == 0          # weight slab alone is 57 KB -- does not fit
        assert lib.ogv_set_option(b"vp_tile", 3) == 0       # 8 x 16 at one workgroup of 8 waves
        assert sup(512, 16, 16, 96, 3, False) == 1
    finally:
        assert lib.ogv_set_option(b"outlook_vproj", 2) == 0
        assert lib.ogv_set_option(b"vp_tile", 0) == 0
        assert lib.ogv_set_option(b"vp_big", 0) == 0
        assert lib.ogv_set_option(b"vp_head", 1) == 0
    x = ctypes.c_void_p(16)
    rc = lib.ogv_outlook_vproj_fwd(x, 192, x, None, None, 200, x, 2, 8, 8, 192, 6, 3, L.OGV_BF16, None)
    assert rc != 0 and b"unsupported" in lib.ogv_last_error()
    rc = lib.ogv_outlook_vproj_fwd(None, 48, x, None, None, 72, x, 2, 8, 8, 48, 2, 3, L.OGV_BF16, None)
    assert rc != 0 and b"null" in lib.ogv_last_error()


def test_workspace_sizes_follow_their_knobs():
    """Host-side workspace queries (no GPU): the cap on BatchNorm reduction slices (knob bn_slices,
    default 1024) and the AdamW work unit (knob opt_chunk, default 2048 elements) size the workspaces
    the launches then use -- the query and the launch read the same knob."""
    import ctypes
    import ogv._lib as L
    lib = L.load()
    M, C = 524288, 64
    try:
        assert lib.ogv_set_option(b"bn_slices", 256) == 0
        small = lib.ogv_bn_act_ws_bytes(M, C)
        assert lib.ogv_set_option(b"bn_slices", 1024) == 0
        big = lib.ogv_bn_act_ws_bytes(M, C)
        assert big > small > 0
    finally:
        assert lib.ogv_set_option(b"bn_slices", 1024) == 0
    t = (L.AdamWTensor * 2)()
    t[0].numel, t[1].numel = 10000, 1
    try:
        assert lib.ogv_set_option(b"opt_chunk", 8192) == 0
        assert lib.ogv_clip_adamw_ws_bytes(t, 2) == 4 * (2 + 1)
        assert lib.ogv_set_option(b"opt_chunk", 2048) == 0
        assert lib.ogv_clip_adamw_ws_bytes(t, 2) == 4 * (5 + 1)
        assert lib.ogv_set_option(b"opt_chunk", 3000) == 0          # rounded up to a power of two: 4096
        assert lib.ogv_clip_adamw_ws_bytes(t, 2) == 4 * (3 + 1)
    finally:
        assert lib.ogv_set_option(b"opt_chunk", 2048) == 0
    assert lib.ogv_set_option(b"bn_red_rg", 64) == 0 and lib.ogv_set_option(b"pg_conv_rs1", 1) == 0
