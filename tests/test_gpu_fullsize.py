"""Full-size parity of the measured path against the CPU oracle at every BASELINE.json config.

The path checked is the one ``bench.py`` times and ``PerspTransDetector`` runs by default:
the fused warp + row-Winograd transform (``warp_wino_kernel`` / ``warp_up_wino2_kernel``, and the
channels-last ``warp_wino_cl_kernel``), the
Winograd conv1 (``conv_wino_kernel``), conv2 with conv3's partials in its epilogue and the
partials' reduce — plus the direct ring conv1 as the second form at configs 1 and 2.

Oracle: ``oracle/cpu_path.py`` (kornia-0.6.11 restatement + ``torch.cat`` + ``F.conv2d``,
``persp_trans_detector.py:65-82``) on identical inputs.  At configs 3-5 the oracle's convs run
on row bands: output rows [r0, r1) need the fused input rows [r0 - 7, r1 + 7) (the receptive
field of the dilation-1/2/4 chain, ``:51-54``), so the band is exact wherever the cut is
not the image edge; the warp of every view is compared whole.

Gate (``helpers``): elementwise |d| <= 1e-3 |ref| + 1e-3 max|ref| and normwise <= 1e-3 (the
north star's "1e-3 relative fp32"); conv1 and map_result of the fp32-storage configs are
additionally held to 5e-5 normwise (the 3xbf16 split's fp32-class accuracy).  Config 4 has fp16
features as the config asks, so its oracle runs on the fp16-rounded inputs; since round 5 the fused
warp reads them in fp32 math into a split-bf16 T (no fp16 slab), so it is held to 5e-5 as well.
"""
import numpy as np
import pytest
import torch

from helpers import assert_parity_t
from oracle import cpu_path, fixtures

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HALO = 7  # 1 + 2 + 4: rows of input one output row of the three convs depends on, each side
TIGHT = 5e-5


def _setup(cfg, C=None, B=None):
    from mvdet_amd import synthetic
    from mvdet_amd.geometry import projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    B = spec["B"] if B is None else B
    C = spec["C"] if C is None else C
    N = ds.num_cam
    up = tuple(ds.upsample_shape)
    grid = tuple(ds.reducedgrid_shape)
    pm = projection_matrices(ds)
    params = fixtures.head_params(N, seed=cfg, C=C)
    mc = torch.nn.Sequential(torch.nn.Conv2d(C * N + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False))
    mc.load_state_dict({k.replace("map_classifier.", ""): torch.from_numpy(v) for k, v in params.items()
                        if k.startswith("map_classifier.")})
    tp = {k: torch.from_numpy(v) for k, v in params.items()}
    return ds, B, C, N, up, grid, pm, tp, mc.to(DEV)


def _oracle_band(warped, grid, params, r0, r1):
    """map rows [r0, r1) and conv1 rows [r0, r1) of the oracle from the warped views' rows
    [r0 - 7, r1 + 7) (clipped to the grid)."""
    H = grid[0]
    a, b = max(0, r0 - HALO), min(H, r1 + HALO)
    B = warped[0].shape[0]
    coord = cpu_path.coord_map(*grid)[:, :, a:b].repeat([B, 1, 1, 1])
    keep = {}
    with torch.no_grad():
        out = cpu_path.fuse(torch.cat([w[:, :, a:b] for w in warped] + [coord], 1), params, keep)
    return out[:, :, r0 - a:r1 - a], keep["conv1_relu"][:, :, r0 - a:r1 - a]


def _check_warp_whole(eng, ws, feats, warped, what):
    """Every view's warp vs the oracle, whole: a slab warp (the fused product warp writes
    conv1's row transform, not the slab) on the same engine and inputs."""
    fused = eng.wino_warp
    eng.wino_warp = False
    try:
        eng.warp_views(ws, list(range(len(feats))), feats)
        torch.cuda.synchronize()
        for v in range(len(feats)):
            assert_parity_t(eng.view_slice(ws, v).float(), warped[v].to(DEV), f"{what} warp view {v}")
    finally:
        eng.wino_warp = fused


@pytest.mark.parametrize("cfg,conv1,layout", [(1, "wino", "nchw"), (1, "direct", "nchw"), (2, "wino", "nchw"),
                                               (2, "direct", "nchw"), (2, "wino", "channels_last")])
def test_full_size_path_vs_oracle(cfg, conv1, layout):
    """Configs 1 and 2 whole: the bench's path (``conv1="wino"``: fused warp + B^T, row-Winograd
    conv1, conv2 -> conv3 partials; the default) and the direct ring conv1, vs the oracle:
    every view's warp, conv1, conv2 and map_result; at config 2 also from channels-last features
    (``warp_wino_cl_kernel``, the bench's ``channels_last`` line)."""
    from mvdet_amd import ProjectFuse, synthetic
    ds, B, C, N, up, grid, pm, tp, mc = _setup(cfg)
    hb = [u // 3 for u in up]
    feats = [synthetic.synthetic_features(B, C, hb, up, seed=1000 * cfg + v, device=DEV) for v in range(N)]
    if layout == "channels_last":
        feats = [f.contiguous(memory_format=torch.channels_last) for f in feats]
    eng = ProjectFuse(pm, up, grid, C, wino_conv1=conv1 == "wino")
    with torch.no_grad():
        got = eng.project_fuse(feats, mc)
        ws = eng.workspace(B, DEV)
        assert ws.t_from_warp == (conv1 == "wino") and eng.conv3_fused_applies(ws)
        y1 = eng.y1_fp32(ws).clone()
        eng.conv2(ws, mc[2])  # conv2 alone (the measured path never stores y2)
        y2 = ws.y2.clone()
        torch.cuda.synchronize()
        keep = {}
        feats_cpu = [f.cpu() for f in feats]
        ref = cpu_path.project_fuse(feats_cpu, [M.numpy() for M in pm], grid, tp, keep=keep)
    assert_parity_t(got, ref, f"cfg{cfg} {conv1} map_result", normwise_tol=TIGHT)
    assert_parity_t(y1, keep["conv1_relu"], f"cfg{cfg} {conv1} conv1", normwise_tol=TIGHT)
    assert_parity_t(y2, keep["conv2_relu"], f"cfg{cfg} {conv1} conv2", normwise_tol=TIGHT)
    with torch.no_grad():
        _check_warp_whole(eng, ws, feats, keep["warped"], f"cfg{cfg}")


@pytest.mark.parametrize("cfg,C,layout", [(2, 512, "nchw"), (1, 512, "nchw"), (2, 512, "channels_last")])
def test_detector_inference_path_vs_oracle(cfg, C, layout):
    """The drop-in module's own inference path at full size: backbone-resolution maps ->
    ``warp_views_upsampled`` (a4 + a5 + a6 + conv1's B^T in ``warp_up_wino_kernel``) -> Winograd
    conv1 -> conv2 / conv3 partials, vs the oracle's upsample (``:65``) + warp + cat + convs
    (``:65-82``); ``imgs_result`` vs the image head on the upsampled maps (``:65-66``).  The
    backbone halves are bypassed (they are not the path).  Config 1's rig at the module's
    C = 512 (resnet18's width)."""
    import torch.nn as nn
    from mvdet_amd import PerspTransDetector, synthetic
    ds, B, C, N, up, grid, pm, tp, mc = _setup(cfg, C=C)
    hb = [u // 3 for u in up]
    model = PerspTransDetector(ds)
    sd = model.state_dict()
    sd.update(tp)
    model.load_state_dict(sd)
    model.base_pt1, model.base_pt2 = nn.Identity(), nn.Identity()
    model.eval()
    low = [synthetic.backbone_features(B, C, hb, seed=2000 * cfg + v, device=DEV) for v in range(N)]
    imgs = torch.stack(low, 1)
    if layout == "channels_last":  # [B, N, C, h, w] stored as [B, N, h, w, C]: per-view channels_last maps
        imgs = torch.stack([f.permute(0, 2, 3, 1) for f in low], 1).permute(0, 1, 4, 2, 3)
        assert imgs[:, 0].is_contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        map_res, imgs_res = model(imgs)
        ws = model.engine.workspace(B, DEV)
        assert ws.t_from_warp and model.engine.wino_active(DEV)
        y1 = model.engine.y1_fp32(ws).clone()
        torch.cuda.synchronize()
        keep = {}
        ups = [cpu_path.upsample(f.cpu(), up) for f in low]
        ref = cpu_path.project_fuse(ups, [M.numpy() for M in pm], grid, tp, keep=keep)
        head = model.img_classifier.cpu()
        ref_imgs = [head(u) for u in ups]
    assert_parity_t(map_res, ref, f"detector cfg{cfg} map_result", normwise_tol=TIGHT)
    assert_parity_t(y1, keep["conv1_relu"], f"detector cfg{cfg} conv1", normwise_tol=TIGHT)
    for v in range(N):
        assert_parity_t(imgs_res[v], ref_imgs[v], f"detector cfg{cfg} imgs_result {v}")


def _bands(H):
    """The top edge band (row 0: conv padding and the first Winograd tile, which starts at row -1),
    an interior band crossing 12-row tile boundaries and the bottom edge band."""
    mid = (H // 2) - 13
    return [(0, 20), (mid, mid + 30), (H - 20, H)]


@pytest.mark.parametrize("cfg,layout", [(3, "nchw"), (5, "nchw"), (5, "channels_last")])
def test_large_config_path_vs_oracle_bands(cfg, layout):
    """Configs 3 (Wildtrack 480 x 1440 grid) and 5 (8 views at 4K, 1000 x 1000 grid) on one GPU:
    the default path over the whole grid; the oracle's warp of every view whole, its convs on
    three row bands (+ the 7-row halo); config 5 also from channels-last features."""
    from mvdet_amd import ProjectFuse, synthetic
    ds, B, C, N, up, grid, pm, tp, mc = _setup(cfg)
    hb = [u // 3 for u in up]
    feats = [synthetic.synthetic_features(B, C, hb, up, seed=1000 * cfg + v, device=DEV) for v in range(N)]
    if layout == "channels_last":
        feats = [f.contiguous(memory_format=torch.channels_last) for f in feats]
    eng = ProjectFuse(pm, up, grid, C)
    with torch.no_grad():
        got = eng.project_fuse(feats, mc)
        ws = eng.workspace(B, DEV)
        assert ws.t_from_warp and eng.wino_active(DEV)
        y1 = eng.y1_fp32(ws)
        torch.cuda.synchronize()
        warped = cpu_path.warp_views([f.cpu() for f in feats], [M.numpy() for M in pm], grid)
        for r0, r1 in _bands(grid[0]):
            ref, ref_y1 = _oracle_band(warped, grid, tp, r0, r1)
            assert_parity_t(got[:, :, r0:r1], ref, f"cfg{cfg} map rows {r0}:{r1}", normwise_tol=TIGHT)
            assert_parity_t(y1[:, :, r0:r1], ref_y1, f"cfg{cfg} conv1 rows {r0}:{r1}", normwise_tol=TIGHT)
        assert torch.isfinite(got).all()
        _check_warp_whole(eng, ws, feats, warped, f"cfg{cfg}")


@pytest.mark.parametrize("C", [512, 128])
def test_config4_fp16_batch8_vs_oracle_bands(C):
    """Config 4 (MultiviewX 6 views, B = 8, fp16 features, fp32 accumulation) at the reference's ResNet-18
    width C = 512 and at cfg1's C = 128 (SURVEY §8's shape table: BASELINE does not state C): the bench's
    path since round 5 — the fp16 features read by the fused warp + B^T (fp32 math, T split-bf16: no fp16
    slab rounding), the Winograd conv1, conv2 -> conv3 partials — vs the oracle on the fp16-rounded inputs
    (the config's own storage precision), held to 5e-5 normwise like the fp32 configs; warp whole, convs on
    three row bands of every batch item."""
    from mvdet_amd import ProjectFuse, synthetic
    ds, B, C, N, up, grid, pm, tp, mc = _setup(4, C=C)
    hb = [u // 3 for u in up]
    feats = [synthetic.synthetic_features(B, C, hb, up, seed=4000 + v, device=DEV).half() for v in range(N)]
    eng = ProjectFuse(pm, up, grid, C)
    with torch.no_grad():
        got = eng.project_fuse(feats, mc)
        ws = eng.workspace(B, DEV)
        assert ws.t_from_warp and eng.wino_active(DEV)  # the fused warp read the fp16 features
        y1 = eng.y1_fp32(ws)
        torch.cuda.synchronize()
        warped = cpu_path.warp_views([f.float().cpu() for f in feats], [M.numpy() for M in pm], grid)
        for r0, r1 in _bands(grid[0]):
            ref, ref_y1 = _oracle_band(warped, grid, tp, r0, r1)
            assert_parity_t(got[:, :, r0:r1], ref, f"cfg4 C={C} map rows {r0}:{r1}", normwise_tol=TIGHT)
            assert_parity_t(y1[:, :, r0:r1], ref_y1, f"cfg4 C={C} conv1 rows {r0}:{r1}", normwise_tol=TIGHT)
        _check_warp_whole(eng, ws, feats, warped, f"cfg4 C={C}")


def test_degenerate_homography_nan_pattern_through_the_detector():
    """A camera whose homography overflows fp32 on part of the grid (intrinsics scaled by 4e35:
    kornia's transform gives inf coordinates there, grid_sample NaN): the warped view is NaN on
    those pixels only.  The detector's default engine detects the geometry
    (``mvbev_warp_nonfinite_views``) and runs the direct conv1, so map_result's NaN pattern is
    the reference's (a NaN reaches the outputs whose taps read it).  The row-Winograd form,
    forced on the same input, spreads it further (B^T mixes a 3-row tile's rows) — the case the
    routing exists for."""
    import torch.nn as nn
    from mvdet_amd import PerspTransDetector, synthetic
    from mvdet_amd.geometry import projection_matrices
    ds = synthetic.wildtrack_like(3, 4, seed=0, img_shape=(216, 384), worldgrid_shape=(96, 288))
    K = [k.copy() for k in ds.base.intrinsic_matrices]
    K[1][:2, :] *= 4e35
    ds.base.intrinsic_matrices = tuple(K)
    N, C, B = 3, 512, 1
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    params = fixtures.head_params(N, seed=7, C=C)
    model = PerspTransDetector(ds)
    sd = model.state_dict()
    sd.update({k: torch.from_numpy(v) for k, v in params.items()})
    model.load_state_dict(sd)
    model.base_pt1, model.base_pt2 = nn.Identity(), nn.Identity()
    model.eval()
    eng = model.engine
    assert eng.wino_conv1 and eng.nonfinite_views(DEV) == 0b010 and not eng.wino_active(DEV)
    low = [synthetic.backbone_features(B, C, [u // 3 for u in up], seed=90 + v, device=DEV) for v in range(N)]
    with torch.no_grad():
        map_res, _ = model(torch.stack(low, 1))
        y1 = eng.y1_fp32(eng.workspace(B, DEV)).clone()
        torch.cuda.synchronize()
        ups = [cpu_path.upsample(f.cpu(), up) for f in low]
        keep = {}
        ref = cpu_path.project_fuse(ups, [M.numpy() for M in projection_matrices(ds)], grid,
                                    {k: torch.from_numpy(v) for k, v in params.items()}, keep=keep)
    nan_view = torch.isnan(keep["warped"][1][0, 0])
    assert 0 < int(nan_view.sum()) < nan_view.numel()  # partly NaN: the case that discriminates
    assert 0 < int(torch.isnan(ref).sum()) < ref.numel()
    assert_parity_t(y1, keep["conv1_relu"], "degenerate geometry conv1 (NaN pattern included)")
    assert_parity_t(map_res, ref, "degenerate geometry map_result (NaN pattern included)")
    # the Winograd form on the same input: its conv1 NaN pattern is not the reference's
    eng._nonfinite[str(torch.device(DEV))] = 0
    try:
        with torch.no_grad():
            model(torch.stack(low, 1))
            wy1 = eng.y1_fp32(eng.workspace(B, DEV)).clone()
            torch.cuda.synchronize()
        assert eng.workspace(B, DEV).t_from_warp
        assert not torch.equal(torch.isnan(wy1.cpu()), torch.isnan(keep["conv1_relu"]))
    finally:
        eng._nonfinite.clear()
