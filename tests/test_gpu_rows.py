"""Row-window and guard building blocks of ABI 11900 (the multi-GPU modes' non-finite guard, the banded
exact path), each against the whole-grid form it restricts or against torch:

* ``mvbev_warp_views_split_bf16_rows`` — a row window of the split-bf16 warp is bitwise the same rows of
  the whole-grid warp (fp32 and fp16 sources; entries sharing a source), and its non-finite report fires
  exactly when a sample reads a NaN / inf feature;
* ``mvbev_warp_views_exact_rows`` — the same for the exact-order warp (+ upsample), fp16 sources equal to
  their fp32 upcast;
* ``mvbev_conv3x3_f32_ex`` — the row-banded output is bitwise the plain output's rows;
* ``mvbev_bias_relu_nonfinite_f32`` — torch's ``relu(y + init)`` (NaN kept) and its report;
* ``mvbev_zero_gated`` — writes only when the gate holds its tag.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rig(C=16, B=2, seed=5):
    from mvdet_amd import synthetic
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm, projection_matrices
    ds = synthetic.wildtrack_like(3, 4, seed=seed, img_shape=(216, 384), worldgrid_shape=(128, 288))
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    ms = [kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), up, grid)[0] for M in projection_matrices(ds)]
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=70 + v, device=DEV) for v in range(3)]
    return ms, up, grid, feats


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_split_warp_row_windows_equal_whole_grid_rows(dtype):
    from mvdet_amd import ops
    ms, up, grid, feats = _rig()
    feats = [f.to(dtype) for f in feats]
    B, C = feats[0].shape[:2]
    H, W = grid
    whole = [torch.zeros(ops.split_shape(B, C, H, W), dtype=torch.bfloat16, device=DEV) for _ in feats]
    ops.warp_views_into(feats, ms, whole, split=True)
    # windows of every view at several row offsets in one launch (entries share sources), incl. both edges
    E = 13
    row0s = [0, 7, H - E]
    dsts, srcs, mm, r0s, want = [], [], [], [], []
    for r0 in row0s:
        for v in range(3):
            dsts.append(torch.zeros(ops.split_shape(B, C, E, W), dtype=torch.bfloat16, device=DEV))
            srcs.append(feats[v])
            mm.append(ms[v])
            r0s.append(r0)
            want.append(whole[v][:, :, r0:r0 + E])
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    ops.warp_views_split_rows_into(srcs, mm, dsts, r0s, H, nonfinite=(flag, 3))
    torch.cuda.synchronize()
    for d, w in zip(dsts, want):
        assert torch.equal(d, w)
    assert int(flag.item()) == 0, "finite features must not fire the report"
    # zeroed destinations: out-of-source pixels skipped, same bits
    dz = [torch.zeros_like(d) for d in dsts]
    ops.warp_views_split_rows_into(srcs, mm, dz, r0s, H, dst_zeroed=True)
    assert all(torch.equal(a, b) for a, b in zip(dz, dsts))
    # a NaN feature that the warp samples fires the report with the tag
    bad = feats[1].clone()
    bad[0, 3, up[0] // 2, up[1] // 2] = float("nan")
    ops.warp_views_split_rows_into([bad], [ms[1]], [torch.zeros(ops.split_shape(B, C, H, W), dtype=torch.bfloat16,
                                                               device=DEV)], [0], H, nonfinite=(flag, 9))
    assert int(flag.item()) == 9


@pytest.mark.parametrize("upsample", [False, True])
def test_exact_warp_row_windows_and_fp16_sources(upsample):
    from mvdet_amd import ops, synthetic
    ms, up, grid, feats = _rig()
    if upsample:
        feats = [synthetic.backbone_features(2, 16, [u // 3 for u in up], seed=90 + v, device=DEV) for v in range(3)]
    B, C = feats[0].shape[:2]
    H, W = grid
    up_hw = up if upsample else None
    whole = [torch.zeros(B, C, H, W, device=DEV) for _ in feats]
    ops.warp_views_exact_into(feats, ms, whole, up_hw=up_hw)
    E, row0s = 11, [0, 5, H - 11]
    outs = [torch.full((B, C, E, W), 7.0, device=DEV) for _ in row0s]
    ops.warp_views_exact_into([feats[1]] * 3, [ms[1]] * 3, outs, up_hw=up_hw, row0s=row0s, grid_rows=H)
    for o, r0 in zip(outs, row0s):
        assert torch.equal(o, whole[1][:, :, r0:r0 + E])
    # fp16 sources: the same as their fp32 upcast, bit for bit (fp32 arithmetic in both)
    h16 = [f.half() for f in feats]
    a = [torch.zeros(B, C, H, W, device=DEV) for _ in feats]
    b = [torch.zeros(B, C, H, W, device=DEV) for _ in feats]
    ops.warp_views_exact_into(h16, ms, a, up_hw=up_hw, row0s=[0, 0, 0], grid_rows=H)
    ops.warp_views_exact_into([f.float() for f in h16], ms, b, up_hw=up_hw)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    # gated: nothing written unless the flag holds the tag
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    g = torch.full((B, C, E, W), 7.0, device=DEV)
    ops.warp_views_exact_into([feats[0]], [ms[0]], [g], up_hw=up_hw, row0s=[3], grid_rows=H, gate=(flag, 4))
    assert bool((g == 7.0).all())
    flag.fill_(4)
    ops.warp_views_exact_into([feats[0]], [ms[0]], [g], up_hw=up_hw, row0s=[3], grid_rows=H, gate=(flag, 4))
    assert torch.equal(g, whole[0][:, :, 3:3 + E])


def test_fp32_conv_row_banded_output_equals_plain_rows():
    from mvdet_amd import ops
    torch.manual_seed(0)
    B, K, H, W, cout = 2, 24, 29, 70, 128
    x = torch.randn(B, K, H, W, device=DEV)
    w = torch.randn(cout, K, 3, 3, device=DEV) * 0.1
    packed = ops.PackedConv3x3(None, "fp32").get(w)
    d = ops.conv_desc(B, K, H, W, group=K, group_stride=0, batch_stride=K * H * W)
    plain = ops.conv3x3_desc(x, d, packed, cout, dilation=1)
    n = 8
    banded = torch.full((-(-H // n), B, cout, n, W), 5.0, device=DEV)
    # two launches over rows [0, 13) and [13, H): each writes its rows' bands
    for r0, r1 in ((0, 13), (13, H)):
        dd = ops.conv_desc(B, K, H, W, group=K, group_stride=0, batch_stride=K * H * W, out_row0=r0, out_rows=r1 - r0)
        ops.conv3x3_desc(x, dd, packed, cout, dilation=1, out=banded, band_rows=n)
    for p in range(banded.shape[0]):
        a, b = p * n, min(H, (p + 1) * n)
        assert torch.equal(banded[p, :, :, :b - a], plain[:, :, a:b]), p


def test_bias_relu_nonfinite_matches_torch_and_reports():
    from mvdet_amd import ops
    torch.manual_seed(1)
    for W in (48, 50):  # vector and scalar forms
        C, H, rows, row0 = 16, 20, 9, 6
        init = torch.randn(C, H, W, device=DEV)
        y = torch.randn(2, C, rows, W, device=DEV)
        ref = torch.relu(y + init[:, row0:row0 + rows])
        flag = torch.zeros(1, dtype=torch.int32, device=DEV)
        ops.bias_relu_nonfinite_(y, init, row0, flag=(flag, 5))
        assert torch.equal(y, ref) and int(flag.item()) == 0
        y2 = torch.randn(2, C, rows, W, device=DEV)
        y2[1, 3, 4, 7] = float("nan")
        y2[0, 0, 0, 0] = float("inf")
        ref2 = torch.relu(y2 + init[:, row0:row0 + rows])
        ops.bias_relu_nonfinite_(y2, init, row0, flag=(flag, 5))
        assert torch.equal(torch.isnan(y2), torch.isnan(ref2)) and int(flag.item()) == 5
        fin = torch.isfinite(ref2)
        assert torch.equal(y2[fin], ref2[fin])


def test_zero_gated():
    from mvdet_amd import ops
    t = torch.ones(1000, device=DEV)
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    ops.zero_gated_(t, (flag, 2))
    assert bool((t == 1).all())
    flag.fill_(2)
    ops.zero_gated_(t, (flag, 2))
    assert bool((t == 0).all())


@pytest.mark.parametrize("W_src", [384, 376])  # source width 96 (8-B quad staging loads) and 94 (element path)
def test_fused_warp_fp16_sources_match_fp32_upcast(W_src):
    """``warp_views_wino_rows_into`` on fp16 features (config 4's path) writes the T of the same features
    upcast to fp32: fp32 arithmetic after the load in both (its 8-B fp16 quad loads widen to the 16-B fp32
    staging layout).  Not bitwise: the two kernel instantiations contract the bilinear sums into FMAs
    differently, so ~0.5 % of the transformed values differ by an fp32 ulp before the hi / lo split."""
    from mvdet_amd import ops, synthetic
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm, projection_matrices
    ds = synthetic.wildtrack_like(3, 4, seed=9, img_shape=(216, W_src), worldgrid_shape=(128, 288))
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    ms = [kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), up, grid)[0] for M in projection_matrices(ds)]
    B, C = 2, 16
    f16 = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=40 + v, device=DEV).half()
           for v in range(3)]
    H, W = grid
    K = 3 * C
    d = ops.conv_desc(B, K, H, W, group=C, group_stride=B * C * H * W, batch_stride=C * H * W)
    ta = torch.zeros((ops.wino_rows_bytes(d) + 1) // 2, dtype=torch.bfloat16, device=DEV)
    tb = torch.zeros_like(ta)
    ops.warp_views_wino_rows_into(f16, ms, ta, [0, 1, 2], C, K, H, W)
    ops.warp_views_wino_rows_into([f.float() for f in f16], ms, tb, [0, 1, 2], C, K, H, W)
    R5 = 5 * 4 * (-(-H // 12))
    n = B * (K // 8) * R5 * 2 * W * 8
    va = ta[:n].float().view(B, K // 8, R5, 2, W, 8).sum(3)  # hi + lo
    vb = tb[:n].float().view(B, K // 8, R5, 2, W, 8).sum(3)
    scale = float(vb.abs().max())
    assert scale > 0
    # an fp32-ulp difference of a transformed value can flip its hi / lo split: hi + lo keeps ~16 bits
    assert float((va - vb).abs().max()) <= 1e-5 * scale
