"""Row-Winograd conv1 (F(3,3) along the rows: mvbev_wino_rows_split_bf16 + mvbev_conv3x3_wino_bf16x3)
against torch's conv2d in float64 and against the direct 3xbf16 ring conv.

The reference op is conv1 of map_classifier (persp_trans_detector.py:51-52): a dense 3x3 conv,
padding 1, then ReLU; the Winograd form must give the same y within the 3xbf16 tolerance.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import assert_parity

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 5e-5  # CONV_TOL["bf16x3"] of test_gpu_parity.py: normwise vs the float64 conv

# the transform rows of B^T (points 0, 1, -1, 2, inf), as the kernel applies them
BT = np.array([[2, -1, -2, 1, 0], [0, -2, -1, 1, 0], [0, 2, -3, 1, 0], [0, -1, 0, 1, 0], [0, 2, -1, -2, 1]],
              dtype=np.float64)


def _split_encode(x: torch.Tensor) -> torch.Tensor:
    """fp32 [B, C, H, W] (C % 8 == 0) -> split-bf16 blocked [B, C/8, H, W, 2, 8]."""
    B, C, H, W = x.shape
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    t = torch.stack([hi, lo], 0).reshape(2, B, C // 8, 8, H, W)
    return t.permute(1, 2, 4, 5, 0, 3).contiguous()


def _setup(S, Cs, B, H, W, rows, cout, seed, zero_right=False):
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(seed)
    xs = torch.rand(S, B, Cs, H, W, generator=g)
    if zero_right:  # view 1 is zero from column W // 2 on: a mask has something exact to skip
        xs[1, :, :, :, W // 2:] = 0
    K = S * Cs
    w = (torch.rand(cout, K, 3, 3, generator=g) - 0.5) / np.sqrt(K * 9)
    bias = torch.rand(cout, generator=g) - 0.5
    init = torch.rand(cout, H, W, generator=g) - 0.5
    r0, r1 = rows
    x64 = xs.permute(1, 0, 2, 3, 4).reshape(B, K, H, W).double()
    ref = F.relu(F.conv2d(x64, w.double(), bias.double(), padding=1) + init.double())[:, :, r0:r1].float()
    slab = torch.stack([_split_encode(xs[v]) for v in range(S)]).to(DEV)
    desc = ops.conv_desc(B, K, H, W, group=Cs, group_stride=B * Cs * H * W, batch_stride=Cs * H * W,
                         out_row0=r0, out_rows=r1 - r0)
    return xs, w.to(DEV), bias.to(DEV), init.to(DEV), ref, slab, desc


@pytest.mark.parametrize("S,Cs,B,H,W,rows", [(3, 16, 1, 30, 360, (0, 30)),   # partial last tile column
                                              (2, 24, 2, 25, 76, (3, 25)),    # K % 16 == 8, row band, B = 2
                                              (1, 32, 1, 13, 32, (0, 13)),    # one tile column, 2 tile rows
                                              (4, 16, 1, 61, 45, (0, 61))])
def test_wino_conv_vs_float64_and_direct(S, Cs, B, H, W, rows):
    from mvdet_amd import ops
    cout = 256
    xs, w, bias, init, ref, slab, desc = _setup(S, Cs, B, H, W, rows, cout, seed=H * W + S)
    t = torch.zeros(ops.wino_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino_rows(slab, desc, t)
    pk = ops.PackedConv3x3(None, "bf16x3", wino=True).get(w)
    got = ops.conv3x3_wino(t, desc, pk, cout, bias=bias, init=init, relu=True)
    s = assert_parity(got.cpu(), ref, "wino vs float64", normwise_tol=TOL)
    direct = ops.conv3x3_desc(slab, desc, ops.PackedConv3x3(None, "bf16x3").get(w), cout, bias=bias, init=init,
                              relu=True, dilation=1)
    sd = assert_parity(direct.cpu(), ref, "direct vs float64", normwise_tol=TOL)
    # the transforms' roundings: the same order of error as the direct 3xbf16 conv
    assert s["normwise"] <= max(4 * sd["normwise"], 2e-6), (s, sd)
    # split-bf16 output (what conv2 reads) decodes to the fp32 output within the split's rounding
    ysplit = torch.empty(ops.split_shape(B, cout, rows[1] - rows[0], W), dtype=torch.bfloat16, device=DEV)
    ops.conv3x3_wino(t, desc, pk, cout, bias=bias, init=init, relu=True, out=ysplit)
    assert_parity(ops.split_decode(ysplit, cout).cpu(), got.cpu(), "split out", normwise_tol=2e-5)


def test_wino_rows_transform_matches_numpy():
    """T = split(B^T d) per 3-row output tile, input rows out_row0 + 3 r3 - 1 + m (zero outside)."""
    from mvdet_amd import ops
    S, Cs, B, H, W, rows = 2, 16, 1, 17, 40, (2, 17)
    xs, w, bias, init, ref, slab, desc = _setup(S, Cs, B, H, W, rows, 128, seed=5)
    t = torch.zeros(ops.wino_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino_rows(slab, desc, t)
    K, r0, nr = S * Cs, rows[0], rows[1] - rows[0]
    R5 = 5 * 4 * (-(-nr // 12))
    T = t.view(B, K // 8, R5, 2, W, 8).float().cpu()  # a row: hi plane [W][8], then lo plane
    T = (T[:, :, :, 0] + T[:, :, :, 1]).permute(0, 1, 4, 2, 3).reshape(B, K, R5, W).double().numpy()
    # the slab as the kernel sees it: hi + lo of the split encoding
    x = torch.stack([xs[v].to(torch.bfloat16).float() + (xs[v] - xs[v].to(torch.bfloat16).float())
                     .to(torch.bfloat16).float() for v in range(S)]).permute(1, 0, 2, 3, 4).reshape(B, K, H, W)
    x = x.double().numpy()
    for r3 in range(R5 // 5):
        d = np.zeros((5, B, K, W))
        for m in range(5):
            row = r0 + 3 * r3 - 1 + m
            if 0 <= row < H:
                d[m] = x[:, :, row]
        want = np.einsum("xm,mbkw->bkxw", BT, d)
        np.testing.assert_allclose(T[:, :, 5 * r3:5 * r3 + 5].transpose(0, 1, 2, 3), want, rtol=0,
                                   atol=2e-5 * max(1.0, np.abs(want).max()))


@pytest.mark.parametrize("B", [1, 2])
def test_wino_conv_masked_matches_unmasked(B):
    """With a frustum-style mask (cleared = the group is zero over the tile and its halo) and
    the heavy-first order, T is written only for the set (tile, group) pairs of a zero-filled
    buffer, and y equals the unmasked Winograd conv bit for bit (skipped products are zeros)."""
    from mvdet_amd import ops
    S, Cs, H, W, cout = 3, 16, 30, 100, 128
    xs, w, bias, init, ref, slab, desc = _setup(S, Cs, B, H, W, (0, H), cout, seed=77 + B, zero_right=True)
    tx, ty = -(-W // 32), -(-H // 12)
    m = [0b101 | (0b010 if (t % tx) * 32 - 1 < W // 2 else 0) for t in range(tx * ty)]
    gm = torch.tensor(m, dtype=torch.int32, device=DEV)
    order = ops.heavy_first_order(gm, B)
    pk = ops.PackedConv3x3(None, "bf16x3", wino=True).get(w)
    t_full = torch.zeros(ops.wino_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino_rows(slab, desc, t_full)
    t_mask = torch.zeros_like(t_full)
    ops.wino_rows(slab, desc, t_mask, gm)
    assert torch.equal(t_mask, t_full)  # the skipped pairs' true transform is exactly zero
    dense = ops.conv3x3_wino(t_full, desc, pk, cout, bias=bias, init=init, relu=True)
    masked = ops.conv3x3_wino(t_mask, desc, pk, cout, bias=bias, init=init, relu=True, group_mask=gm,
                              tile_order=order)
    assert torch.equal(masked, dense)
    assert_parity(masked.cpu(), ref, "masked wino", normwise_tol=TOL)


def test_wino_refusals():
    from mvdet_amd import _native, ops
    S, Cs, B, H, W = 2, 16, 1, 12, 32
    xs, w, bias, init, ref, slab, desc = _setup(S, Cs, B, H, W, (0, H), 128, seed=3)
    small = torch.zeros(16, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(_native.NativeError):
        ops.wino_rows(slab, desc, small)
    pk = ops.PackedConv3x3(None, "bf16x3", wino=True).get(w)
    t = torch.zeros(ops.wino_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    with pytest.raises((ValueError, _native.NativeError)):  # Cout not a multiple of 128
        ops.conv3x3_wino(t, desc, pk, 128 + 1)
    with pytest.raises(ValueError):
        ops.conv3x3_wino(small, desc, pk, 128)
    with pytest.raises(ValueError):
        ops.PackedConv3x3(None, "fp32", wino=True)


@pytest.mark.parametrize("cfg", [1, 2])
def test_engine_wino_conv1_matches_direct(cfg):
    """ProjectFuse(wino_conv1=True): the detector's map and y1 match the direct ring conv1 within
    the 3xbf16 tolerance at the config rigs (reduced channels), twice in a row bitwise (T reuse)."""
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    N, C, B = ds.num_cam, 32, 1
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm = projection_matrices(ds)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=19 + v, device=DEV)
             for v in range(N)]
    torch.manual_seed(cfg)
    mc = torch.nn.Sequential(torch.nn.Conv2d(N * C + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)
    direct = ProjectFuse(pm, up, grid, C, wino_conv1=False)
    wino = ProjectFuse(pm, up, grid, C)  # the default
    assert wino.wino_conv1 and wino.frustum
    with torch.no_grad():
        ref = direct.project_fuse(feats, mc)
        y1_ref = direct.y1_fp32(direct.workspace(B, DEV)).clone()
        got = wino.project_fuse(feats, mc)
        y1 = wino.y1_fp32(wino.workspace(B, DEV)).clone()
        got2 = wino.project_fuse(feats, mc)
    assert torch.equal(got, got2)
    assert_parity(y1.cpu(), y1_ref.cpu(), "wino y1", normwise_tol=TOL)
    assert_parity(got.cpu(), ref.cpu(), "wino map", normwise_tol=TOL)


@pytest.mark.parametrize("cfg", [1, 2])
def test_fused_warp_transform_matches_two_pass(cfg):
    """wino_warp (mvbev_warp_views_wino_rows: warp + B^T in one pass, no slab) gives the T of the
    two-pass path (split slab, then mvbev_wino_rows_split_bf16) within the split's rounding, and
    the same map; a later slab-writing warp (upsampled features) switches conv1 back to the
    slab's transform."""
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    N, C, B = ds.num_cam, 24, 1
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm = projection_matrices(ds)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=31 + v, device=DEV)
             for v in range(N)]
    torch.manual_seed(10 + cfg)
    mc = torch.nn.Sequential(torch.nn.Conv2d(N * C + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)
    # (F(3,3)'s T: the F(4,3) engines' T43 has its own test, test_gpu_wino43.py)
    fused = ProjectFuse(pm, up, grid, C, wino_conv1=True, wino43=False)
    two = ProjectFuse(pm, up, grid, C, wino_conv1=True, wino_warp=False, wino43=False)
    assert fused.wino_warp and not two.wino_warp
    with torch.no_grad():
        got = fused.project_fuse(feats, mc)
        wf = fused.workspace(B, DEV)
        assert wf.t_from_warp and wf.slab.abs().max().item() == 0  # the slab was never written
        ref = two.project_fuse(feats, mc)
        wt = two.workspace(B, DEV)
        tf = wf.wino_t.view(-1, 2, grid[1], 8).float()  # T rows: hi plane, then lo plane
        tt = wt.wino_t.view(-1, 2, grid[1], 8).float()
        a, b = tf.sum(1), tt.sum(1)
        # the two-pass T transforms the slab's hi + lo (each value rounded to ~2^-17): the 5-row
        # combinations (coefficient sums <= 6) differ by a few 1e-5 of the range
        assert (a - b).abs().max().item() <= 1e-4 * max(1.0, b.abs().max().item())
        assert_parity(got.cpu(), ref.cpu(), "fused-warp map", normwise_tol=TOL)
        # backbone-resolution input: the fused upsample + warp + B^T (mvbev_warp_views_upsampled_wino_rows)
        # vs upsample + warp into the slab, then the transform
        low = [torch.nn.functional.avg_pool2d(f, 3) for f in feats]
        fused.warp_views_upsampled(wf, list(range(N)), low)
        assert wf.t_from_warp
        m1 = fused.fuse(wf, mc)
        two.warp_views_upsampled(wt, list(range(N)), low)
        m2 = two.fuse(wt, mc)
        assert_parity(m1.cpu(), m2.cpu(), "fused upsample + warp + B^T map", normwise_tol=TOL)
        # after the fused warp the slab holds no frame: a slab warp of a subset of the views is
        # refused (its other slots would be stale); a slab warp of every view switches conv1 back
        # to the slab's transform, after which single-view warps are fine again
        with pytest.raises(RuntimeError):
            fused.warp_view(wf, 0, feats[0])
        fused.wino_warp = False
        with pytest.raises(RuntimeError):
            fused.warp_views(wf, [0], feats[:1])
        assert wf.t_from_warp
        fused.warp_views(wf, list(range(N)), feats)
        assert not wf.t_from_warp
        for v in range(N):
            fused.warp_view(wf, v, feats[v])
        m3 = fused.fuse(wf, mc)
        # the direct conv1 and conv1_partial read the slab: refused while T came from the fused warp
        fused.wino_warp = True
        fused.warp_views(wf, list(range(N)), feats)
        assert wf.t_from_warp
        fused.wino_conv1 = False
        with pytest.raises(RuntimeError):
            fused.conv1(wf, mc[0])
        with pytest.raises(RuntimeError):
            fused.conv1_partial(wf, mc, torch.empty((B, 512) + grid, device=DEV))
        fused.wino_conv1 = True
    assert_parity(m3.cpu(), ref.cpu(), "slab path after the fused warp", normwise_tol=TOL)


def _t_value(t: torch.Tensor, Wo: int) -> torch.Tensor:
    """T rows (hi plane then lo plane, bf16) -> hi + lo in fp32."""
    h = t.view(torch.bfloat16).view(-1, 2, Wo, 8).float()
    return h[:, 0] + h[:, 1]


def _assert_same_t(va: torch.Tensor, vb: torch.Tensor) -> None:
    """Same NaN / inf positions; finite values equal up to the fp32 rounding of the bilinear sums
    (an fp32 ulp of t can move lo = bf16(t - hi) by one of its own ulps: <= 2^-16 |t|)."""
    assert torch.equal(va.isnan(), vb.isnan()) and torch.equal(va.isinf(), vb.isinf())
    inf = va.isinf()
    assert torch.equal(va[inf], vb[inf])
    fin = va.isfinite()
    scale = va[fin].abs().max().item()
    assert ((va[fin] - vb[fin]).abs() <= 2.0 ** -15 * va[fin].abs() + 1e-6 * scale).all()


@pytest.mark.parametrize("cfg,C,B", [(1, 32, 1), (2, 64, 2), (2, 40, 1)])
def test_fused_warp_channels_last_matches_nchw(cfg, C, B):
    """Channels-last sources (sC == 1, C % 32 == 0: warp_wino_cl_kernel, one 128-B line per source
    pixel) give the T of the NCHW kernel for the same logical tensor (to fp32 rounding): zero and NaN
    geometry (one view's matrix made non-finite), an inf feature, the non-finite report and
    skip_zero included.  C = 40 (not whole 32-channel groups) takes the NCHW kernel with the
    channels-last strides — the same T again."""
    from mvdet_amd import ops, synthetic
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm, projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    N = ds.num_cam
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    ms = [kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), up, grid)[0] for M in projection_matrices(ds)]
    ms[-1] = ms[-1].clone()
    ms[-1][0, 2] = float("inf")  # every sample of the last view is non-finite -> NaN T
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=71 + v, device=DEV)
             for v in range(N)]
    feats[0][B - 1, C - 1, up[0] // 2, up[1] // 2] = float("inf")
    Ho, Wo = grid
    r3 = 4 * (-(-Ho // 12))
    numel = B * (N * C // 8) * 5 * r3 * Wo * 16
    outs = []
    for layout in (torch.contiguous_format, torch.channels_last):
        src = [f.contiguous(memory_format=layout) for f in feats]
        for zeroed in (False, True):
            t = torch.zeros(numel, dtype=torch.bfloat16, device=DEV)
            flag = torch.zeros(1, dtype=torch.int32, device=DEV)
            ops.warp_views_wino_rows_into(src, ms, t, list(range(N)), C, N * C, Ho, Wo, dst_zeroed=zeroed,
                                          nonfinite=(flag, 7))
            outs.append((t.view(torch.int16).cpu(), int(flag.item())))
    (a, fa), (az, fz), (b, fb), (bz, fbz) = outs
    assert fa == fz == fb == fbz == 7
    assert torch.equal(a, az) and torch.equal(b, bz)

    _assert_same_t(_t_value(a, Wo), _t_value(b, Wo))


@pytest.mark.parametrize("cfg,C,B,half,cl", [(1, 32, 1, False, False), (2, 64, 2, False, False), (2, 24, 1, False, False),
                                           (4, 16, 2, True, False), (2, 64, 2, False, True), (1, 32, 1, False, True)])
def test_fused_warp_box_table_is_bitwise_the_block_reduction(cfg, C, B, half, cl):
    """Round 6: the NCHW fused warp + B^T with the per-geometry staging boxes (``mvbev_warp_wino_boxes`` ->
    ``mvbev_warp_views_wino_rows_ex``) writes bitwise the T of the per-block box reduction (same box, same
    staged / direct choice, same arithmetic), with skip_zero on and off (blocks without an inside sample
    return at once), a view with non-finite geometry (its NaN T still written), an inf feature (the
    non-finite report), B = 2 and fp16 sources; the table marks the empty and non-finite blocks.  ``cl``:
    channels-last sources (warp_wino_cl_kernel, the same block tiles: the table's early return)."""
    from mvdet_amd import ops, synthetic
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm, projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    N = ds.num_cam
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    ms = [kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), up, grid)[0] for M in projection_matrices(ds)]
    ms[-1] = ms[-1].clone()
    ms[-1][0, 2] = float("inf")
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=81 + v, device=DEV)
             for v in range(N)]
    feats[0][B - 1, C - 1, up[0] // 2, up[1] // 2] = float("inf")
    if half:
        feats = [f.half() for f in feats]
    if cl:  # the line-per-pixel kernel (channels-last sources): the table's early return only
        feats = [f.contiguous(memory_format=torch.channels_last) for f in feats]
    Ho, Wo = grid
    r3 = 4 * (-(-Ho // 12))
    boxes = ops.warp_wino_boxes(ms, up, grid, DEV)
    bc = boxes.cpu()
    assert (bc[:-1, :, 1] < 0).any() and (bc[:-1, :, 1] >= 0).any()  # empty and non-empty blocks
    assert ((bc[-1, :, 3] >> 30) == 1).all()                          # the NaN view: every block non-finite
    numel = B * (N * C // 8) * 5 * r3 * Wo * 16
    for zeroed in (False, True):
        outs = []
        for bx in (None, boxes):
            t = torch.zeros(numel, dtype=torch.bfloat16, device=DEV)
            flag = torch.zeros(1, dtype=torch.int32, device=DEV)
            ops.warp_views_wino_rows_into(feats, ms, t, list(range(N)), C, N * C, Ho, Wo, dst_zeroed=zeroed,
                                          nonfinite=(flag, 5), boxes=bx)
            outs.append((t.view(torch.int16).cpu(), int(flag.item())))
        assert outs[0][1] == outs[1][1] == 5
        assert torch.equal(outs[0][0], outs[1][0]), f"skip_zero={zeroed}: T differs with the box table"


@pytest.mark.parametrize("cfg,C,B", [(1, 32, 1), (2, 64, 2), (5, 32, 1)])
def test_fused_upsample_warp_box_table_is_bitwise_the_block_reduction(cfg, C, B):
    """Round 6: the channels-last fused upsample warp + B^T (the detector's default path) with the per-geometry
    backbone-window boxes (``mvbev_warp_upsampled_wino_boxes`` -> ``..._upsampled_wino_rows_ex``) writes bitwise
    the T of the per-block reduction: skip_zero on and off, a view with non-finite geometry, an inf feature
    (the non-finite report), B = 2."""
    from mvdet_amd import ops, synthetic
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm, projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    N = ds.num_cam
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    hb = tuple(u // 3 for u in up)
    ms = [kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), up, grid)[0] for M in projection_matrices(ds)]
    ms[-1] = ms[-1].clone()
    ms[-1][0, 2] = float("inf")
    low = [synthetic.backbone_features(B, C, hb, seed=91 + v, device=DEV) for v in range(N)]
    low[0][B - 1, C - 1, hb[0] // 2, hb[1] // 2] = float("inf")
    low = [f.contiguous(memory_format=torch.channels_last) for f in low]
    Ho, Wo = grid
    r3 = 4 * (-(-Ho // 12))
    boxes = ops.warp_wino_boxes(ms, up, grid, DEV, backbone_hw=hb)
    bc = boxes.cpu()
    assert (bc[:-1, :, 1] < 0).any() and (bc[:-1, :, 1] >= 0).any() and ((bc[-1, :, 3] >> 30) == 1).all()
    numel = B * (N * C // 8) * 5 * r3 * Wo * 16
    for zeroed in (False, True):
        outs = []
        for bx in (None, boxes):
            t = torch.zeros(numel, dtype=torch.bfloat16, device=DEV)
            flag = torch.zeros(1, dtype=torch.int32, device=DEV)
            ops.warp_views_wino_rows_into(low, ms, t, list(range(N)), C, N * C, Ho, Wo, dst_zeroed=zeroed,
                                          up_hw=up, nonfinite=(flag, 3), boxes=bx)
            outs.append((t.view(torch.int16).cpu(), int(flag.item())))
        assert outs[0][1] == outs[1][1] == 3
        assert torch.equal(outs[0][0], outs[1][0]), f"skip_zero={zeroed}: T differs with the box table"


@pytest.mark.parametrize("cfg,C,B", [(1, 32, 1), (2, 64, 2), (2, 40, 1)])
def test_fused_upsample_warp_channels_last_matches_nchw(cfg, C, B):
    """The fused 3x upsample + warp + B^T from channels-last backbone maps (warp_up_wino_cl_kernel:
    line-per-pixel box staging, the transform in registers) — given channels-last, or copied from NCHW
    by mvbev_nchw_to_nhwc_f32 — gives the T of the NCHW kernel (to fp32 rounding): NaN geometry, an inf
    feature, the non-finite report and skip_zero included.  The copy equals torch's channels_last
    copy exactly.  C = 40 (no whole 32-channel groups) with channels-last strides is refused."""
    from mvdet_amd import _native, ops, synthetic
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm, projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    N = ds.num_cam
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    ms = [kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), up, grid)[0] for M in projection_matrices(ds)]
    ms[-1] = ms[-1].clone()
    ms[-1][0, 2] = float("inf")
    low = [u // 3 for u in up]
    feats = [synthetic.backbone_features(B, C, low, seed=81 + v, device=DEV) for v in range(N)]
    feats[0][B - 1, C - 1, low[0] // 2, low[1] // 2] = float("inf")
    Ho, Wo = grid
    r3 = 4 * (-(-Ho // 12))
    numel = B * (N * C // 8) * 5 * r3 * Wo * 16

    def run(src, zeroed):
        t = torch.zeros(numel, dtype=torch.bfloat16, device=DEV)
        flag = torch.zeros(1, dtype=torch.int32, device=DEV)
        ops.warp_views_wino_rows_into(src, ms, t, list(range(N)), C, N * C, Ho, Wo, dst_zeroed=zeroed, up_hw=up,
                                      nonfinite=(flag, 5))
        assert int(flag.item()) == 5
        return t.view(torch.int16).cpu()

    cl = [f.contiguous(memory_format=torch.channels_last) for f in feats]
    if C % 32:
        with pytest.raises(_native.NativeError):
            run(cl, True)
        return
    bufs = [torch.empty(B, low[0], low[1], C, device=DEV) for _ in range(N)]
    copied = ops.to_channels_last_into(feats, bufs)
    for a_, b_ in zip(copied, cl):
        assert torch.equal(a_, b_) and ops.is_channels_last_source(a_)
    base = run(feats, False)
    assert torch.equal(base, run(feats, True))
    va = _t_value(base, Wo)
    got = run(cl, False)
    for src, zeroed in ((cl, True), (copied, False), (copied, True)):
        assert torch.equal(got, run(src, zeroed))
    vb = _t_value(got, Wo)
    # the NCHW kernel's near-field blocks load 4-column window rows (a zero-weight 4th column: an inf
    # there gives NaN), so it may hold NaN where the channels-last kernel (3 columns) does not; every
    # non-finite value of the channels-last T is non-finite there too, and the rest agree
    assert not (~vb.isfinite() & va.isfinite()).any()
    both = va.isfinite() & vb.isfinite()
    scale = va[both].abs().max().item()
    err = (va[both] - vb[both]).abs()
    bad = err > 2.0 ** -15 * va[both].abs() + 1e-6 * scale
    assert not bad.any(), (int(bad.sum()), int(bad.numel()), err.max().item(), scale,
                           va[both][bad][:8].tolist(), vb[both][bad][:8].tolist())
    assert both.float().mean().item() > 0.5


@pytest.mark.parametrize("cl_upsample", [False, True])
def test_engine_channels_last_backbone_maps(cl_upsample):
    """ProjectFuse from channels-last backbone maps (the line-per-pixel fused upsample warp), and from
    NCHW maps copied to channels-last (cl_upsample), gives the NCHW engine's map."""
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    ds = synthetic.CONFIGS[1]["make"]()
    N, C, B = ds.num_cam, 32, 1
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm = projection_matrices(ds)
    low = [synthetic.backbone_features(B, C, [u // 3 for u in up], seed=91 + v, device=DEV) for v in range(N)]
    torch.manual_seed(3)
    mc = torch.nn.Sequential(torch.nn.Conv2d(N * C + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)
    ref_eng = ProjectFuse(pm, up, grid, C)
    eng = ProjectFuse(pm, up, grid, C, cl_upsample=cl_upsample)
    with torch.no_grad():
        wr = ref_eng.workspace(B, DEV)
        ref_eng.warp_views_upsampled(wr, list(range(N)), low)
        ref = ref_eng.fuse(wr, mc)
        src = low if cl_upsample else [f.contiguous(memory_format=torch.channels_last) for f in low]
        w = eng.workspace(B, DEV)
        eng.warp_views_upsampled(w, list(range(N)), src)
        assert w.t_from_warp
        got = eng.fuse(w, mc)
    assert_parity(got.cpu(), ref.cpu(), "channels-last backbone maps", normwise_tol=TOL)


# -- conv2 (dilation 2) -> conv3 partials as row-Winograd (ABI 11500) ------------------------------
def _conv2_setup(B, K, H, W, rows, cout, seed):
    """y1-like split-bf16 input, conv2 weights / bias, conv3 weight, and the float64 reference
    map = conv2d_d4(relu(conv2d_d2(x) + b2), w3) over the output band ``rows``."""
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(B, K, H, W, generator=g)
    w = (torch.rand(cout, K, 3, 3, generator=g) - 0.5) / np.sqrt(K * 9)
    bias = torch.rand(cout, generator=g) - 0.5
    w3 = (torch.rand(1, cout, 3, 3, generator=g) - 0.5) / np.sqrt(cout * 9)
    y2 = F.relu(F.conv2d(x.double(), w.double(), bias.double(), padding=2, dilation=2))
    ref = F.conv2d(y2, w3.double(), padding=4, dilation=4)[:, :, rows[0]:rows[1]].float()
    xs = _split_encode(x).to(DEV)
    r0, r1 = max(0, rows[0] - 4), min(H, rows[1] + 4)  # conv2's output rows the map band reads
    desc = ops.conv_desc(B, K, H, W, group=K, group_stride=0, batch_stride=K * H * W, out_row0=r0,
                         out_rows=r1 - r0)
    return x, xs, w.to(DEV), bias.to(DEV), w3.to(DEV), y2, ref, desc


def test_wino_rows_dilation2_matches_numpy():
    """conv2's transform: row tile (r, r + 2, r + 4), r = 12 (r3 / 4) + {0, 1, 6, 7}[r3 % 4];
    T = B^T over input rows r - 2 + 2 m (zero outside the image)."""
    from mvdet_amd import ops
    B, K, H, W = 1, 16, 29, 40
    x, xs, *_, desc = _conv2_setup(B, K, H, W, (0, H), 128, seed=11)
    t = torch.zeros(ops.wino_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino_rows(xs, desc, t, dilation=2)
    R5 = 5 * 4 * (-(-H // 12))
    T = t.view(B, K // 8, R5, 2, W, 8).float().cpu()  # a row: hi plane [W][8], then lo plane
    T = (T[:, :, :, 0] + T[:, :, :, 1]).permute(0, 1, 4, 2, 3).reshape(B, K, R5, W).double().numpy()
    xe = (x.to(torch.bfloat16).float() + (x - x.to(torch.bfloat16).float()).to(torch.bfloat16).float()).double().numpy()
    for r3 in range(R5 // 5):
        base = 12 * (r3 // 4) + (0, 1, 6, 7)[r3 % 4]
        d = np.zeros((5, B, K, W))
        for m in range(5):
            row = base - 2 + 2 * m
            if 0 <= row < H:
                d[m] = xe[:, :, row]
        want = np.einsum("xm,mbkw->bkxw", BT, d)
        np.testing.assert_allclose(T[:, :, 5 * r3:5 * r3 + 5], want, rtol=0, atol=2e-5 * max(1.0, np.abs(want).max()))


@pytest.mark.parametrize("B,K,H,W,rows", [(1, 64, 30, 70, (0, 30)),    # partial tile row and column
                                          (2, 32, 41, 100, (9, 33)),  # map band, B = 2
                                          (1, 128, 12, 32, (0, 12))])  # one tile
def test_wino_conv2_partials_vs_float64_and_direct(B, K, H, W, rows):
    """conv2 -> conv3 partials from the dilation-2 transform (the inference default) vs float64
    and vs the direct ring conv's partials (mvbev_conv3x3_bf16x3_cout1_partials)."""
    from mvdet_amd import ops
    cout = 256
    x, xs, w, bias, w3, y2, ref, desc = _conv2_setup(B, K, H, W, rows, cout, seed=B * H + W)
    t = torch.zeros(ops.wino_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino_rows(xs, desc, t, dilation=2)
    need = ops.conv3x3_cout1_partials_bytes(desc, cout)
    p_w = torch.empty(need // 4, dtype=torch.float32, device=DEV)
    ops.conv3x3_wino_then_cout1_partials(t, desc, ops.PackedConv3x3(None, "bf16x3", wino=True).get(w), cout, bias,
                                         2, True, w3, p_w)
    got = ops.cout1_from_partials(p_w, desc, cout, 4, rows[0], rows[1] - rows[0]).cpu()
    p_d = torch.empty_like(p_w)
    ops.conv3x3_then_cout1_partials(xs, desc, ops.PackedConv3x3(None, "bf16x3").get(w), cout, bias, 2, True, w3, p_d)
    direct = ops.cout1_from_partials(p_d, desc, cout, 4, rows[0], rows[1] - rows[0]).cpu()
    s = assert_parity(got, ref, "wino conv2->conv3 vs float64", normwise_tol=TOL)
    sd = assert_parity(direct, ref, "direct conv2->conv3 vs float64", normwise_tol=TOL)
    assert s["normwise"] <= max(4 * sd["normwise"], 2e-6), (s, sd)
    # the dense dilation-2 conv from the same T (y stored): vs float64 relu(conv2)
    y = ops.conv3x3_wino_dil(t, desc, ops.PackedConv3x3(None, "bf16x3", wino=True).get(w), cout, 2, bias=bias,
                             relu=True)
    r0 = desc.out_row0
    assert_parity(y.cpu(), y2[:, :, r0:r0 + desc.out_rows].float(), "wino conv2 y", normwise_tol=TOL)


def test_wino_conv2_refusals():
    from mvdet_amd import _native, ops
    B, K, H, W, cout = 1, 16, 12, 32, 128
    x, xs, w, bias, w3, y2, ref, desc = _conv2_setup(B, K, H, W, (0, H), cout, seed=3)
    t = torch.zeros(ops.wino_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(_native.NativeError):
        ops.wino_rows(xs, desc, t, dilation=3)
    pk = ops.PackedConv3x3(None, "bf16x3", wino=True).get(w)
    p = torch.empty(ops.conv3x3_cout1_partials_bytes(desc, cout) // 4, dtype=torch.float32, device=DEV)
    with pytest.raises(_native.NativeError):  # the partials epilogue is conv2's: dilation 2 only
        ops.conv3x3_wino_then_cout1_partials(t, desc, pk, cout, bias, 1, True, w3, p)
    with pytest.raises(ValueError):
        ops.conv3x3_wino_then_cout1_partials(t[:16], desc, pk, cout, bias, 2, True, w3, p)


@pytest.mark.parametrize("cfg", [1, 2])
def test_engine_wino_conv2_matches_direct(cfg):
    """ProjectFuse's inference map with the Winograd conv2 (default) vs wino_conv2=False, same inputs."""
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    N, C = ds.num_cam, 32
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm = projection_matrices(ds)
    feats = [synthetic.synthetic_features(1, C, [u // 3 for u in up], up, seed=v, device=DEV) for v in range(N)]
    torch.manual_seed(cfg)
    mc = torch.nn.Sequential(torch.nn.Conv2d(N * C + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)
    a = ProjectFuse(pm, up, grid, C)
    b = ProjectFuse(pm, up, grid, C, wino_conv2=False)
    assert a.wino_conv2 and not b.wino_conv2
    with torch.no_grad():
        ma = a.project_fuse(feats, mc)
        assert a.workspace(1, DEV).wino_t2 is not None  # the Winograd conv2 ran
        mb = b.project_fuse(feats, mc)
        assert b.workspace(1, DEV).wino_t2 is None
    assert_parity(ma.cpu(), mb.cpu(), "wino conv2 map vs direct conv2 map", normwise_tol=TOL)
