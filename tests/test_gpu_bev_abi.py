"""The one-call C ABI (``mvbev_bev_plan_init`` / ``mvbev_bev_fuse_prepare`` / ``mvbev_bev_fuse``,
SURVEY §8(b)) against the CPU oracle and against the Python engine that makes the same calls:
fp32 sources at the config-2 rig (the bench's path), backbone-resolution sources (the
detector's path, the 3x upsample of persp_trans_detector.py:65 fused), fp16 sources (the direct
conv1), a degenerate camera (non-finite samples -> the direct conv1 and the reference's NaN
pattern), and frames run back to back through one workspace."""
import pytest
import torch

from helpers import assert_parity_t
from oracle import cpu_path, fixtures

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _setup(ds, C, seed, B=1):
    from mvdet_amd.geometry import projection_matrices
    N = ds.num_cam
    params = fixtures.head_params(N, seed=seed, C=C)
    mc = torch.nn.Sequential(torch.nn.Conv2d(C * N + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False))
    mc.load_state_dict({k.replace("map_classifier.", ""): torch.from_numpy(v) for k, v in params.items()
                        if k.startswith("map_classifier.")})
    tp = {k: torch.from_numpy(v) for k, v in params.items()}
    return projection_matrices(ds), mc.to(DEV), tp


def _engine_mats(pm, up, grid):
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm
    return [kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), up, grid)[0] for M in pm]


def test_bev_fuse_cfg2_fp32_vs_oracle_and_engine():
    """Config 2 (7 views, C = 512, 270 x 480 -> 120 x 360), fp32 sources: the fused warp + B^T,
    the Winograd conv1, conv2 -> conv3 partials; bitwise the Python engine's map, within the
    gate of the oracle; two frames through one workspace."""
    from mvdet_amd import ProjectFuse, ops, synthetic
    spec = synthetic.CONFIGS[2]
    ds = spec["make"]()
    C, N = spec["C"], ds.num_cam
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm, mc, tp = _setup(ds, C, seed=2)
    bev = ops.BevFuse(_engine_mats(pm, up, grid), C, up, grid)
    bev.prepare(mc, DEV)
    assert bev.wino and bev.plan.frustum
    eng = ProjectFuse(pm, up, grid, C)
    for frame in range(2):
        feats = [synthetic.synthetic_features(1, C, [u // 3 for u in up], up, seed=2000 + 10 * frame + v, device=DEV)
                 for v in range(N)]
        with torch.no_grad():
            got = bev(feats).clone()
            ref_eng = eng.project_fuse(feats, mc)
            torch.cuda.synchronize()
            ref = cpu_path.project_fuse([f.cpu() for f in feats], [M.numpy() for M in pm], grid, tp)
        assert torch.equal(got, ref_eng), frame
        assert_parity_t(got, ref, f"bev_fuse cfg2 frame {frame}", normwise_tol=5e-5)


@pytest.mark.parametrize("cfg,C,up_src", [(1, 128, False), (3, 32, False), (1, 64, True)])
def test_bev_fuse_wino43_vs_engine_and_oracle(cfg, C, up_src):
    """ABI 12400: grids whose rows fill 16-row tiles run F(4,3) in the one-call path too (plan wino 2: the fused
    warp writes T43, conv1 F(4,3); wino2 2 where the launch is deep — config 3 — else F(3,3)); bitwise the
    Python engine's map (the same kernels, masks and order; from backbone maps to fp32 rounding: the engine's
    upsample warp reads a channels-last copy), within the gate of the oracle."""
    from mvdet_amd import ProjectFuse, _native, ops, synthetic
    ds = synthetic.CONFIGS[cfg]["make"]()
    N = ds.num_cam
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    lo = [u // 3 for u in up]
    pm, mc, tp = _setup(ds, C, seed=cfg)
    kw = dict(src_kind=_native.BEV_SRC_BACKBONE_F32, backbone_hw=lo) if up_src else {}
    bev = ops.BevFuse(_engine_mats(pm, up, grid), C, up, grid, **kw)
    bev.prepare(mc, DEV)
    eng = ProjectFuse(pm, up, grid, C)
    assert bev.plan.wino == 2 and bev.plan.wino2 == (2 if cfg == 3 else 1)
    if up_src:
        feats = [synthetic.backbone_features(1, C, lo, seed=300 + v, device=DEV) for v in range(N)]
    else:
        feats = [synthetic.synthetic_features(1, C, lo, up, seed=300 + v, device=DEV) for v in range(N)]
    with torch.no_grad():
        got = bev(feats).clone()
        ws = eng.workspace(1, DEV)
        (eng.warp_views_upsampled if up_src else eng.warp_views)(ws, list(range(N)), feats)
        ref_eng = eng.fuse(ws, mc)
        assert ws.t_form == 4
        torch.cuda.synchronize()
        src = [cpu_path.upsample(f.cpu(), up) for f in feats] if up_src else [f.cpu() for f in feats]
        ref = cpu_path.project_fuse(src, [M.numpy() for M in pm], grid, tp)
    if up_src:  # (the engine copies NCHW backbone maps to channels-last for its upsample warp: T to fp32 rounding)
        assert_parity_t(got, ref_eng, f"bev_fuse F(4,3) cfg{cfg} vs engine", normwise_tol=1e-5)
    else:
        assert torch.equal(got, ref_eng)
    assert_parity_t(got, ref, f"bev_fuse F(4,3) cfg{cfg}", normwise_tol=5e-5)


def test_bev_fuse_backbone_sources_vs_oracle():
    """Backbone-resolution sources (the detector's inference path: upsample + warp + B^T in one
    kernel), config 1's rig at C = 512, B = 2."""
    from mvdet_amd import _native, ops, synthetic
    ds = synthetic.CONFIGS[1]["make"]()
    C, N, B = 512, ds.num_cam, 2
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    lo = [u // 3 for u in up]
    pm, mc, tp = _setup(ds, C, seed=11, B=B)
    bev = ops.BevFuse(_engine_mats(pm, up, grid), C, up, grid, B=B, src_kind=_native.BEV_SRC_BACKBONE_F32,
                      backbone_hw=lo)
    bev.prepare(mc, DEV)
    low = [synthetic.backbone_features(B, C, lo, seed=70 + v, device=DEV) for v in range(N)]
    with torch.no_grad():
        got = bev(low)
        torch.cuda.synchronize()
        ref = cpu_path.project_fuse([cpu_path.upsample(f.cpu(), up) for f in low], [M.numpy() for M in pm], grid, tp)
    assert bev.wino
    assert_parity_t(got, ref, "bev_fuse backbone sources", normwise_tol=5e-5)


@pytest.mark.parametrize("backbone", [False, True])
def test_bev_fuse_channels_last_sources(backbone):
    """MVBEV_BEV_SRC_CHANNELS_LAST (ABI 11700): the same frames passed channels-last take the fused
    warps' line-per-pixel kernels; the map equals the NCHW plan's to fp32 rounding and the oracle's
    within the gate (config 1's rig, C = 64, B = 2; plain and backbone-resolution sources).  fp16 and
    C % 32 != 0 are refused."""
    from mvdet_amd import _native, ops, synthetic
    ds = synthetic.CONFIGS[1]["make"]()
    C, N, B = 64, ds.num_cam, 2
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    lo = [u // 3 for u in up]
    pm, mc, tp = _setup(ds, C, seed=13, B=B)
    kind = _native.BEV_SRC_BACKBONE_F32 if backbone else _native.BEV_SRC_F32
    kw = dict(B=B, backbone_hw=lo) if backbone else dict(B=B)
    nchw = ops.BevFuse(_engine_mats(pm, up, grid), C, up, grid, src_kind=kind, **kw)
    cl = ops.BevFuse(_engine_mats(pm, up, grid), C, up, grid, src_kind=kind | _native.BEV_SRC_CHANNELS_LAST, **kw)
    nchw.prepare(mc, DEV)
    cl.prepare(mc, DEV)
    if backbone:
        feats = [synthetic.backbone_features(B, C, lo, seed=130 + v, device=DEV) for v in range(N)]
    else:
        feats = [synthetic.synthetic_features(B, C, lo, up, seed=130 + v, device=DEV) for v in range(N)]
    with torch.no_grad():
        a = nchw(feats).clone()
        b = cl([f.contiguous(memory_format=torch.channels_last) for f in feats]).clone()
        c = cl(feats).clone()  # NCHW tensors handed to a channels-last plan are converted by the wrapper
        torch.cuda.synchronize()
        src = [cpu_path.upsample(f.cpu(), up) for f in feats] if backbone else [f.cpu() for f in feats]
        ref = cpu_path.project_fuse(src, [M.numpy() for M in pm], grid, tp)
    assert torch.equal(b, c)
    assert_parity_t(b, a, "bev_fuse channels-last vs NCHW", normwise_tol=1e-5)  # fp32 rounding of T, through the split convs
    assert_parity_t(b, ref, "bev_fuse channels-last vs oracle", normwise_tol=5e-5)
    for bad_kind, bad_c in ((_native.BEV_SRC_F16 | _native.BEV_SRC_CHANNELS_LAST, 64),
                            (kind | _native.BEV_SRC_CHANNELS_LAST, 40)):
        with pytest.raises(_native.NativeError):
            ops.BevFuse(_engine_mats(pm, up, grid), bad_c, up, grid, src_kind=bad_kind, **kw)


def test_bev_fuse_fp16_sources_direct_conv1():
    """fp16 sources (config 4's storage): the split slab from fp16 and the direct ring conv1."""
    from mvdet_amd import _native, ops, synthetic
    ds = synthetic.wildtrack_like(3, 4, seed=4, img_shape=(216, 384), worldgrid_shape=(96, 288))
    C, N, B = 64, 3, 2
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm, mc, tp = _setup(ds, C, seed=4, B=B)
    bev = ops.BevFuse(_engine_mats(pm, up, grid), C, up, grid, B=B, src_kind=_native.BEV_SRC_F16)
    bev.prepare(mc, DEV)
    assert not bev.wino
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=40 + v, device=DEV).half()
             for v in range(N)]
    with torch.no_grad():
        got = bev(feats)
        torch.cuda.synchronize()
        ref = cpu_path.project_fuse([f.float().cpu() for f in feats], [M.numpy() for M in pm], grid, tp)
    assert_parity_t(got, ref, "bev_fuse fp16 sources", normwise_tol=5e-5)


def test_bev_fuse_degenerate_camera_nan_pattern():
    """A camera whose homography overflows fp32 on part of the grid: prepare detects it, plans
    the direct conv1, and the map's NaN pattern is the oracle's."""
    from mvdet_amd import _native, ops, synthetic
    ds = synthetic.wildtrack_like(3, 4, seed=0, img_shape=(216, 384), worldgrid_shape=(96, 288))
    K = [k.copy() for k in ds.base.intrinsic_matrices]
    K[1][:2, :] *= 4e35
    ds.base.intrinsic_matrices = tuple(K)
    C, N = 512, 3
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    lo = [u // 3 for u in up]
    pm, mc, tp = _setup(ds, C, seed=7)
    bev = ops.BevFuse(_engine_mats(pm, up, grid), C, up, grid, src_kind=_native.BEV_SRC_BACKBONE_F32,
                      backbone_hw=lo)
    bev.prepare(mc, DEV)
    assert not bev.wino
    low = [synthetic.backbone_features(1, C, lo, seed=90 + v, device=DEV) for v in range(N)]
    with torch.no_grad():
        got = bev(low)
        torch.cuda.synchronize()
        ref = cpu_path.project_fuse([cpu_path.upsample(f.cpu(), up) for f in low], [M.numpy() for M in pm], grid, tp)
    assert 0 < int(torch.isnan(ref).sum()) < ref.numel()
    assert_parity_t(got, ref, "bev_fuse degenerate camera (NaN pattern included)")


def test_bev_fuse_refusals():
    import ctypes
    from mvdet_amd import _native, ops
    bev = ops.BevFuse([torch.eye(3)] * 2, 16, (20, 30), (10, 12))
    lib = _native.load()
    out = torch.empty((1, 1, 10, 12), device=DEV)
    arr = (ctypes.c_void_p * 2)(0, 0)
    # not prepared yet
    assert lib.mvbev_bev_fuse(ctypes.byref(bev.plan), arr, out.data_ptr(), out.data_ptr(), 4, None) == _native.ERR_SHAPE
    ws = torch.empty(int(bev.plan.workspace_bytes) + 512, dtype=torch.uint8, device=DEV)
    base = ws.data_ptr() + (-ws.data_ptr()) % 256
    # a workspace smaller than the plan's, or misaligned
    w = torch.zeros((512, 34, 3, 3), device=DEV)
    assert lib.mvbev_bev_fuse_prepare(ctypes.byref(bev.plan), w.data_ptr(), None, w.data_ptr(), None, w.data_ptr(),
                                      base, 16, None) == _native.ERR_SHAPE
    assert lib.mvbev_bev_fuse_prepare(ctypes.byref(bev.plan), w.data_ptr(), None, w.data_ptr(), None, w.data_ptr(),
                                      base + 4, int(bev.plan.workspace_bytes), None) == -4  # MVBEV_ERR_ALIGN


def test_bev_fuse_wrapper_refuses_mismatched_views_and_out():
    """The Python wrapper checks every view and ``out`` against the plan (the kernels behind the raw
    pointers cannot): wrong shape, dtype, device placement or out layout raise before a launch."""
    from mvdet_amd import ops, synthetic
    ds = synthetic.wildtrack_like(2, 4, seed=2, img_shape=(216, 384), worldgrid_shape=(96, 288))
    C = 16
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm, mc, tp = _setup(ds, C, seed=2)
    bev = ops.BevFuse(_engine_mats(pm, up, grid), C, up, grid)
    bev.prepare(mc, DEV)
    good = [torch.zeros((1, C) + up, device=DEV) for _ in range(2)]
    with pytest.raises(ValueError, match="view 1"):
        bev([good[0], torch.zeros((1, C, up[0], up[1] - 1), device=DEV)])
    with pytest.raises(ValueError, match="view 0"):
        bev([good[0].half(), good[1]])
    with pytest.raises(ValueError, match="out"):
        bev(good, out=torch.empty((1, 1, grid[0], grid[1] + 1), device=DEV))
    with pytest.raises(ValueError, match="out"):
        bev(good, out=torch.empty((1, 1) + grid, device=DEV, dtype=torch.float64))
    with pytest.raises(RuntimeError):
        bev([good[0].cpu(), good[1]])
    assert torch.isfinite(bev(good)).all()


def test_bev_fuse_nonfinite_features_guard():
    """The one-call ABI's non-finite guard (plan.guard): +inf and NaN injected into backbone-resolution
    features; the fused warp reports them and the gated exact path gives the oracle's NaN / inf pattern;
    a finite frame through the same workspace afterwards is the fast path's map."""
    from mvdet_amd import _native, ops, synthetic
    ds = synthetic.wildtrack_like(3, 4, seed=5, img_shape=(216, 384), worldgrid_shape=(96, 288))
    C, N = 64, 3
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    lo = [u // 3 for u in up]
    pm, mc, tp = _setup(ds, C, seed=9)
    bev = ops.BevFuse(_engine_mats(pm, up, grid), C, up, grid, src_kind=_native.BEV_SRC_BACKBONE_F32, backbone_hw=lo)
    bev.prepare(mc, DEV)
    assert bev.wino and bev.plan.guard
    low = [synthetic.backbone_features(1, C, lo, seed=20 + v, device=DEV) for v in range(N)]
    bad = [f.clone() for f in low]
    bad[0][0, 9, lo[0] // 2, lo[1] // 2] = float("inf")
    bad[2][0, 4, lo[0] // 2 - 3, lo[1] // 2 + 4] = float("nan")
    mats = [M.numpy() for M in pm]
    with torch.no_grad():
        got = bev(bad).clone()
        fine = bev(low).clone()
        torch.cuda.synchronize()
        ref = cpu_path.project_fuse([cpu_path.upsample(f.cpu(), up) for f in bad], mats, grid, tp)
        ref_fine = cpu_path.project_fuse([cpu_path.upsample(f.cpu(), up) for f in low], mats, grid, tp)
    assert 0 < int((~torch.isfinite(ref)).sum()) < ref.numel()
    assert_parity_t(got, ref, "bev_fuse non-finite features (NaN / inf pattern included)")
    assert torch.isfinite(fine).all()
    assert_parity_t(fine, ref_fine, "bev_fuse finite frame after a non-finite one", normwise_tol=5e-5)


def test_bev_fuse_guard_in_row_chunks_batch2(monkeypatch):
    """ABI 11900: the one-call guard's exact path in output-row chunks (``MVBEV_BEV_GUARD_BYTES`` small:
    several chunks, each reading its rows +- 7 through a same-size slab window) at B = 2, fp32 sources;
    the workspace holds one chunk's fp32 window, not a whole-grid slab; ``MVBEV_BEV_NO_GUARD`` drops the
    guard's regions."""
    from mvdet_amd import _native, ops, synthetic
    ds = synthetic.wildtrack_like(3, 4, seed=6, img_shape=(216, 384), worldgrid_shape=(128, 288))
    C, N, B = 64, 3, 2
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm, mc, tp = _setup(ds, C, seed=10)
    mats = _engine_mats(pm, up, grid)
    full = ops.BevFuse(mats, C, up, grid, B=B)
    per_row = N * B * C * grid[1] * 4
    monkeypatch.setenv("MVBEV_BEV_GUARD_BYTES", str(per_row * (12 + 14)))
    bev = ops.BevFuse(mats, C, up, grid, B=B)
    off = bev.plan.off
    assert off[16 + 1] - off[16] < per_row * grid[0] and bev.plan.workspace_bytes < full.plan.workspace_bytes
    noguard = ops.BevFuse(mats, C, up, grid, B=B, src_kind=_native.BEV_NO_GUARD)
    assert noguard.plan.workspace_bytes < bev.plan.workspace_bytes and not noguard.plan.guard
    bev.prepare(mc, DEV)
    assert bev.wino and bev.plan.guard
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=40 + v, device=DEV) for v in range(N)]
    feats[1][1, 7, up[0] // 2, up[1] // 2] = float("-inf")
    feats[0][0, 3, up[0] // 2 + 5, up[1] // 2 - 8] = float("nan")
    with torch.no_grad():
        got = bev(feats).clone()
        torch.cuda.synchronize()
        ref = cpu_path.project_fuse([f.cpu() for f in feats], [M.numpy() for M in pm], grid, tp)
    assert 0 < int((~torch.isfinite(ref)).sum()) < ref.numel()
    assert_parity_t(got, ref, "bev_fuse chunked guard B=2 (NaN / inf pattern included)")
