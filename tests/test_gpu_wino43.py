"""Row-Winograd F(4,3) (ABI 12400: mvbev_wino43_rows_split_bf16 + mvbev_conv3x3_wino43_bf16x3 and its conv3
partials form) against torch's conv2d in float64, against the F(3,3) kernels and against the direct 3xbf16 ring
conv.

The reference ops are conv1 (persp_trans_detector.py:51-52: 3x3, padding 1, ReLU) and conv2 -> conv3
(:53-54: dilation 2, ReLU, then the single-output dilation-4 conv); the F(4,3) form must give the same
outputs within the 3xbf16 tolerance (its transforms round about twice as much as F(3,3)'s:
tools/wino_error.py, 1.8-2.3e-5 normwise emulated at K = 3584).
"""
import numpy as np
import pytest
import torch

from helpers import assert_parity
from test_gpu_wino import _conv2_setup, _setup

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 5e-5  # CONV_TOL["bf16x3"] of test_gpu_parity.py: normwise vs the float64 conv

# B^T of F(4,3) (points 0, +-1, +-2, inf), as the kernel applies it
BT43 = np.array([[4, 0, -5, 0, 1, 0], [0, -4, -4, 1, 1, 0], [0, 4, -4, -1, 1, 0], [0, -2, -1, 2, 1, 0],
                 [0, 2, -1, -2, 1, 0], [0, 4, 0, -5, 0, 1]], dtype=np.float64)


def _t43_values(t, B, K, nr, W):
    """T43 as float64 [B, K, R6, W] (hi + lo of each entry)."""
    R6 = 6 * 4 * (-(-nr // 16))
    T = t.view(B, K // 8, R6, 2, W, 8).float().cpu()  # a row: hi plane [W][8], then lo plane
    return (T[:, :, :, 0] + T[:, :, :, 1]).permute(0, 1, 4, 2, 3).reshape(B, K, R6, W).double().numpy(), R6


@pytest.mark.parametrize("dil", [1, 2])
def test_wino43_rows_transform_matches_numpy(dil):
    """T43 = split(B^T d) per 4-row output tile: dilation 1, rows out_row0 + 4 r4 - 1 + m; dilation 2,
    row tile r4 of a 16-row tile at base 16 (r4 / 4) + 8 ((r4 % 4) / 2) + r4 % 2, rows base - 2 + 2 m
    (zero outside the image)."""
    from mvdet_amd import ops
    if dil == 1:
        S, Cs, B, H, W, rows = 2, 16, 1, 21, 40, (2, 21)
        xs, *_, slab, desc = _setup(S, Cs, B, H, W, rows, 128, seed=5)
        K = S * Cs
        x = torch.stack([xs[v].to(torch.bfloat16).float() + (xs[v] - xs[v].to(torch.bfloat16).float())
                         .to(torch.bfloat16).float() for v in range(S)]).permute(1, 0, 2, 3, 4).reshape(B, K, H, W)
    else:
        B, K, H, W = 1, 16, 29, 40
        rows = (0, H)
        x0, slab, *_, desc = _conv2_setup(B, K, H, W, rows, 128, seed=11)
        x = x0.to(torch.bfloat16).float() + (x0 - x0.to(torch.bfloat16).float()).to(torch.bfloat16).float()
    t = torch.zeros(ops.wino43_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino43_rows(slab, desc, t, dilation=dil)
    r0, nr = desc.out_row0, desc.out_rows
    T, R6 = _t43_values(t, B, K, nr, W)
    x = x.double().numpy()
    for r4 in range(R6 // 6):
        q = r4 % 4
        base = r0 + 16 * (r4 // 4) + (4 * q if dil == 1 else 8 * (q // 2) + q % 2)
        d = np.zeros((6, B, K, W))
        for m in range(6):
            row = base + dil * (m - 1)
            if 0 <= row < H:
                d[m] = x[:, :, row]
        want = np.einsum("xm,mbkw->bkxw", BT43, d)
        np.testing.assert_allclose(T[:, :, 6 * r4:6 * r4 + 6], want, rtol=0,
                                   atol=2e-5 * max(1.0, np.abs(want).max()))


@pytest.mark.parametrize("S,Cs,B,H,W,rows", [(3, 16, 1, 30, 360, (0, 30)),   # partial last tile row and column
                                              (2, 24, 2, 25, 76, (3, 25)),    # K % 16 == 8, row band, B = 2
                                              (1, 32, 1, 13, 32, (0, 13)),    # one tile
                                              (4, 16, 1, 61, 45, (0, 61))])
def test_wino43_conv_vs_float64_and_f33(S, Cs, B, H, W, rows):
    from mvdet_amd import ops
    cout = 256
    xs, w, bias, init, ref, slab, desc = _setup(S, Cs, B, H, W, rows, cout, seed=H * W + S)
    t = torch.zeros(ops.wino43_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino43_rows(slab, desc, t)
    pk = ops.pack_wino43(w)
    got = ops.conv3x3_wino43(t, desc, pk, cout, bias=bias, init=init, relu=True)
    s = assert_parity(got.cpu(), ref, "wino43 vs float64", normwise_tol=TOL)
    t3 = torch.zeros(ops.wino_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino_rows(slab, desc, t3)
    f33 = ops.conv3x3_wino(t3, desc, ops.PackedConv3x3(None, "bf16x3", wino=True).get(w), cout, bias=bias,
                           init=init, relu=True)
    s3 = assert_parity(f33.cpu(), ref, "wino33 vs float64", normwise_tol=TOL)
    assert s["normwise"] <= max(6 * s3["normwise"], 4e-6), (s, s3)
    ysplit = torch.empty(ops.split_shape(B, cout, rows[1] - rows[0], W), dtype=torch.bfloat16, device=DEV)
    ops.conv3x3_wino43(t, desc, pk, cout, bias=bias, init=init, relu=True, out=ysplit)
    assert_parity(ops.split_decode(ysplit, cout).cpu(), got.cpu(), "split out", normwise_tol=2e-5)


@pytest.mark.parametrize("B", [1, 2])
def test_wino43_conv_masked_matches_unmasked(B):
    """With a frustum-style mask over 16 x 32 tiles and the heavy-first order: T43 written only for the set
    (tile, group) pairs of a zero-filled buffer equals the dense T43, and y equals the unmasked conv bit for bit."""
    from mvdet_amd import ops
    S, Cs, H, W, cout = 3, 16, 40, 100, 128
    xs, w, bias, init, ref, slab, desc = _setup(S, Cs, B, H, W, (0, H), cout, seed=77 + B, zero_right=True)
    tx, ty = -(-W // 32), -(-H // 16)
    m = [0b101 | (0b010 if (t % tx) * 32 - 1 < W // 2 else 0) for t in range(tx * ty)]
    gm = torch.tensor(m, dtype=torch.int32, device=DEV)
    order = ops.heavy_first_order(gm, B)
    pk = ops.pack_wino43(w)
    t_full = torch.zeros(ops.wino43_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino43_rows(slab, desc, t_full)
    t_mask = torch.zeros_like(t_full)
    ops.wino43_rows(slab, desc, t_mask, gm)
    assert torch.equal(t_mask, t_full)
    dense = ops.conv3x3_wino43(t_full, desc, pk, cout, bias=bias, init=init, relu=True)
    masked = ops.conv3x3_wino43(t_mask, desc, pk, cout, bias=bias, init=init, relu=True, group_mask=gm,
                                tile_order=order)
    assert torch.equal(masked, dense)
    assert_parity(masked.cpu(), ref, "masked wino43", normwise_tol=TOL)


@pytest.mark.parametrize("B,K,H,W,rows", [(1, 64, 30, 70, (0, 30)),    # partial tile row and column
                                          (2, 32, 41, 100, (9, 33)),  # map band, B = 2
                                          (1, 128, 16, 32, (0, 16))])  # one tile
def test_wino43_conv2_partials_vs_float64_and_f33(B, K, H, W, rows):
    """conv2 -> conv3 partials from the dilation-2 F(4,3) transform vs float64 and vs the F(3,3) kernel's."""
    from mvdet_amd import ops
    cout = 256
    x, xs, w, bias, w3, y2, ref, desc = _conv2_setup(B, K, H, W, rows, cout, seed=B * H + W)
    t = torch.zeros(ops.wino43_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino43_rows(xs, desc, t, dilation=2)
    need = ops.conv3x3_cout1_partials_bytes(desc, cout)
    p43 = torch.empty(need // 4, dtype=torch.float32, device=DEV)
    pk = ops.pack_wino43(w)
    ops.conv3x3_wino43_then_cout1_partials(t, desc, pk, cout, bias, True, w3, p43)
    got = ops.cout1_from_partials(p43, desc, cout, 4, rows[0], rows[1] - rows[0]).cpu()
    t3 = torch.zeros(ops.wino_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino_rows(xs, desc, t3, dilation=2)
    p33 = torch.empty_like(p43)
    ops.conv3x3_wino_then_cout1_partials(t3, desc, ops.PackedConv3x3(None, "bf16x3", wino=True).get(w), cout, bias,
                                         2, True, w3, p33)
    f33 = ops.cout1_from_partials(p33, desc, cout, 4, rows[0], rows[1] - rows[0]).cpu()
    s = assert_parity(got, ref, "wino43 conv2->conv3 vs float64", normwise_tol=TOL)
    s3 = assert_parity(f33, ref, "wino33 conv2->conv3 vs float64", normwise_tol=TOL)
    assert s["normwise"] <= max(6 * s3["normwise"], 4e-6), (s, s3)
    y = ops.conv3x3_wino43(t, desc, pk, cout, bias=bias, relu=True, dilation=2)
    r0 = desc.out_row0
    assert_parity(y.cpu(), y2[:, :, r0:r0 + desc.out_rows].float(), "wino43 conv2 y", normwise_tol=TOL)


def test_wino43_refusals():
    from mvdet_amd import _native, ops
    S, Cs, B, H, W = 2, 16, 1, 16, 32
    xs, w, bias, init, ref, slab, desc = _setup(S, Cs, B, H, W, (0, H), 128, seed=3)
    small = torch.zeros(16, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(_native.NativeError):
        ops.wino43_rows(slab, desc, small)
    t = torch.zeros(ops.wino43_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(_native.NativeError):
        ops.wino43_rows(slab, desc, t, dilation=3)
    pk = ops.pack_wino43(w)
    with pytest.raises((ValueError, _native.NativeError)):  # Cout not a multiple of 128
        ops.conv3x3_wino43(t, desc, pk, 128 + 1)
    with pytest.raises(ValueError):
        ops.conv3x3_wino43(small, desc, pk, 128)
    with pytest.raises(_native.NativeError):
        ops.conv3x3_wino43(t, desc, pk, 128, dilation=3)


# -- the fused warps writing T43 (MVBEV_WARP_WINO43) and the engine's F(4,3) path -----------------------------
def _rig(cfg, nan_view=True):
    from mvdet_amd import synthetic
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm, projection_matrices
    ds = synthetic.CONFIGS[cfg]["make"]()
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    ms = [kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), up, grid)[0] for M in projection_matrices(ds)]
    if nan_view:
        ms[-1] = ms[-1].clone()
        ms[-1][0, 2] = float("inf")  # every sample of the last view is non-finite -> NaN T
    return ds, up, grid, ms


def _t43_numel(B, K, Ho, Wo):
    from mvdet_amd import ops
    return B * (K // 8) * 6 * ops.wino_tile_rows(Ho, 4) * Wo * 16


@pytest.mark.parametrize("cfg,C,B,kind", [(1, 32, 1, "nchw"), (2, 64, 2, "nchw"), (2, 24, 1, "nchw"), (4, 16, 2, "f16"),
                                          (2, 64, 2, "cl"), (1, 32, 1, "cl"), (2, 32, 1, "up"), (1, 32, 2, "upcl"),
                                          (5, 32, 1, "upcl")])
def test_fused_warp43_matches_slab_transform_and_box_table(cfg, C, B, kind):
    """The fused warps with MVBEV_WARP_WINO43 (NCHW fp32 / fp16, channels-last, the fused upsample on NCHW and
    channels-last backbone maps) write the T43 of the two-pass path — the split slab of the plain warp, then
    mvbev_wino43_rows_split_bf16 — to the split's rounding, with finite geometry; and, with a NaN-geometry view
    and an inf feature, bitwise the same T43 with and without the per-geometry box table, skip_zero on and off,
    reporting the non-finite feature."""
    from mvdet_amd import ops, synthetic
    ds, up, grid, ms = _rig(cfg, nan_view=False)
    N = ds.num_cam
    Ho, Wo = grid
    hb = tuple(u // 3 for u in up)
    upk = kind in ("up", "upcl")
    if upk:
        feats = [synthetic.backbone_features(B, C, hb, seed=41 + v, device=DEV) for v in range(N)]
    else:
        feats = [synthetic.synthetic_features(B, C, hb, up, seed=41 + v, device=DEV) for v in range(N)]
    if kind == "f16":
        feats = [f.half() for f in feats]
    if kind in ("cl", "upcl"):
        feats = [f.contiguous(memory_format=torch.channels_last) for f in feats]
    K = N * C
    kw = dict(up_hw=up) if upk else {}
    t = torch.zeros(_t43_numel(B, K, Ho, Wo), dtype=torch.bfloat16, device=DEV)
    ops.warp_views_wino_rows_into(feats, ms, t, list(range(N)), C, K, Ho, Wo, dst_zeroed=True, form=4,
                                  boxes=ops.warp_wino_boxes(ms, up, grid, DEV, backbone_hw=hb if kind == "upcl" else None,
                                                            form=4), **kw)
    # two-pass: the split slab (per view: [B, C/8, Ho, Wo, 2, 8]) and its T43
    slab = torch.zeros((N,) + ops.split_shape(B, C, Ho, Wo), dtype=torch.bfloat16, device=DEV)
    src32 = [f.float().contiguous() for f in feats]
    if upk:
        ops.warp_views_upsampled_into(src32, up, ms, [slab[v] for v in range(N)], split=True, dst_zeroed=True)
    else:
        ops.warp_views_into(src32, ms, [slab[v] for v in range(N)], split=True, dst_zeroed=True)
    desc = ops.conv_desc(B, K, Ho, Wo, group=C, group_stride=B * C * Ho * Wo, batch_stride=C * Ho * Wo)
    t2 = torch.zeros(ops.wino43_rows_bytes(desc) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino43_rows(slab, desc, t2)
    a, b = _t43_values(t, B, K, Ho, Wo)[0], _t43_values(t2, B, K, Ho, Wo)[0]
    assert np.abs(a - b).max() <= 2e-4 * max(1.0, np.abs(b).max())
    # non-finite geometry and features: the box table changes nothing (bitwise), the report fires
    ds, up, grid, ms = _rig(cfg)
    feats = [f.clone() for f in feats]
    feats[0][B - 1, C - 1, feats[0].shape[2] // 2, feats[0].shape[3] // 2] = float("inf")
    boxes = ops.warp_wino_boxes(ms, up, grid, DEV, backbone_hw=hb if kind == "upcl" else None, form=4)
    for zeroed in (False, True):
        outs = []
        for bx in ((None, boxes) if kind != "up" else (None,)):
            t = torch.zeros(_t43_numel(B, K, Ho, Wo), dtype=torch.bfloat16, device=DEV)
            flag = torch.zeros(1, dtype=torch.int32, device=DEV)
            ops.warp_views_wino_rows_into(feats, ms, t, list(range(N)), C, K, Ho, Wo, dst_zeroed=zeroed,
                                          nonfinite=(flag, 9), boxes=bx, form=4, **kw)
            outs.append((t.view(torch.int16).cpu(), int(flag.item())))
        assert all(f == 9 for _, f in outs)
        assert all(torch.equal(outs[0][0], o) for o, _ in outs[1:])
        v = _t43_values(outs[0][0].view(torch.bfloat16), B, K, Ho, Wo)[0]
        assert np.isnan(v[:, (N - 1) * C // 8 * 8:]).any()  # the NaN view's T43 is written


def _head(N, C, seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Conv2d(N * C + 2, 512, 3, padding=1), torch.nn.ReLU(),
                               torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                               torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)


@pytest.mark.parametrize("cfg,C,B,up", [(1, 32, 1, False), (2, 24, 2, False), (1, 32, 1, True), (4, 16, 2, False),
                                        (2, 32, 1, True)])
def test_engine_wino43_matches_f33(cfg, C, B, up):
    """ProjectFuse(wino43=True): the fused warp writes T43, conv1 and conv2 -> conv3 run F(4,3); y1 and the map
    match the F(3,3) engine (wino43=False) within the 3xbf16 tolerance, and the slab path (wino_warp off:
    wino43_rows of the slab) gives the fused path's map."""
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    ds = synthetic.CONFIGS[cfg]["make"]()
    N = ds.num_cam
    upsz, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm = projection_matrices(ds)
    hb = [u // 3 for u in upsz]
    if up:
        feats = [synthetic.backbone_features(B, C, hb, seed=5 + v, device=DEV) for v in range(N)]
    else:
        feats = [synthetic.synthetic_features(B, C, hb, upsz, seed=5 + v, device=DEV) for v in range(N)]
    if cfg == 4:
        feats = [f.half() for f in feats]
    mc = _head(N, C, cfg)
    e33 = ProjectFuse(pm, upsz, grid, C, wino43=False)
    e43 = ProjectFuse(pm, upsz, grid, C, wino43=True)
    e43s = ProjectFuse(pm, upsz, grid, C, wino43=True, wino_warp=False)
    maps, y1s = [], []
    with torch.no_grad():
        for e in ((e33, e43) if cfg == 4 else (e33, e43, e43s)):  # (the slab path takes fp32 features)
            ws = e.workspace(B, DEV)
            (e.warp_views_upsampled if up else e.warp_views)(ws, list(range(N)), feats)
            maps.append(e.fuse(ws, mc).clone())
            y1s.append(e.y1_fp32(ws).clone())
            if e is e43:
                assert ws.t_from_warp and ws.t_form == 4 and ws.wino_t is None
    assert_parity(y1s[1].cpu(), y1s[0].cpu(), "F(4,3) y1 vs F(3,3)", normwise_tol=TOL)
    assert_parity(maps[1].cpu(), maps[0].cpu(), "F(4,3) map vs F(3,3)", normwise_tol=TOL)
    if len(maps) > 2:
        assert_parity(maps[2].cpu(), maps[1].cpu(), "F(4,3) slab path vs fused", normwise_tol=TOL)


def test_engine_wino43_nonfinite_guard_matches_f33():
    """A NaN / inf feature under the F(4,3) path: the fused warp's report gates the exact path, whose map keeps
    the reference's NaN / inf pattern — the F(3,3) engine's (pinned to the oracle in test_gpu_nonfinite.py)."""
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    ds = synthetic.CONFIGS[1]["make"]()
    N, C, B = ds.num_cam, 32, 1
    upsz, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm = projection_matrices(ds)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in upsz], upsz, seed=61 + v, device=DEV)
             for v in range(N)]
    feats[1][0, 3, upsz[0] // 2, upsz[1] // 3] = float("nan")
    feats[2][0, 5, upsz[0] // 3, upsz[1] // 2] = float("inf")
    mc = _head(N, C, 7)
    outs = []
    with torch.no_grad():
        for w43 in (False, True):
            e = ProjectFuse(pm, upsz, grid, C, wino43=w43)
            ws = e.workspace(B, DEV)
            e.warp_views(ws, list(range(N)), feats)
            outs.append(e.fuse(ws, mc).cpu())
    a, b = outs
    assert torch.equal(a.isnan(), b.isnan()) and torch.equal(a.isinf(), b.isinf())
    assert a.isnan().any() or a.isinf().any()
    fin = a.isfinite()
    assert_parity(b[fin].view(1, -1), a[fin].view(1, -1), "finite part", normwise_tol=TOL)
