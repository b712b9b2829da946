"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle.

Tolerance (north_star: "within 1e-3 relative fp32"):
  elementwise |got-ref| <= 1e-3*|ref| + 1e-3*max|ref|  and  normwise max|got-ref|/max|ref| <= 1e-3
(``helpers.assert_parity``).  Warp outputs are additionally held to 2e-4 normwise
against the float64 closed form.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import assert_parity, load_golden, parity_stats
from oracle import cpu_path, fixtures, kornia_warp

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rand_h(rng, H, W, ho, wo):
    A = np.eye(3)
    A[0, 0] = wo / W * rng.uniform(0.6, 1.4)
    A[1, 1] = ho / H * rng.uniform(0.6, 1.4)
    A[0, 1], A[1, 0] = rng.uniform(-0.2, 0.2, 2)
    A[0, 2], A[1, 2] = rng.uniform(-3, 3, 2)
    A[2, 0], A[2, 1] = rng.uniform(-2e-3, 2e-3, 2)
    return A


# ---------------------------------------------------------------------------------- warp

@pytest.mark.parametrize("B,C,H,W,ho,wo", [(1, 5, 27, 48, 12, 36), (2, 67, 30, 41, 17, 23), (1, 3, 5, 7, 1, 9),
                                           (2, 130, 64, 96, 40, 63)])
def test_warp_vs_oracle_and_closed_form(B, C, H, W, ho, wo):
    from mvdet_amd import warp_perspective
    rng = np.random.default_rng(B * 1000 + C)
    src = np.maximum(rng.standard_normal((B, C, H, W)), 0).astype(np.float32)
    M = np.stack([_rand_h(rng, H, W, ho, wo) for _ in range(B)])
    Mt = torch.from_numpy(M).float()
    got = warp_perspective(torch.from_numpy(src).to(DEV), Mt.to(DEV), (ho, wo)).cpu()
    ref = kornia_warp.warp_perspective(torch.from_numpy(src), Mt, (ho, wo))
    assert_parity(got, ref, "warp vs restatement")
    if ho > 1 and wo > 1:
        s = parity_stats(got, kornia_warp.closed_form_warp_f64(src, M, (ho, wo)))
        assert s["normwise"] < 2e-4, s


@pytest.mark.parametrize("B,C,h,w,H,W,ho,wo", [(2, 20, 9, 16, 27, 48, 12, 36), (1, 67, 10, 14, 27, 41, 17, 23),
                                                 (1, 8, 5, 7, 5, 7, 6, 9), (2, 130, 30, 40, 90, 120, 40, 63)])
@pytest.mark.parametrize("split", [False, True])
def test_upsample_warp_fused_vs_oracle(B, C, h, w, H, W, ho, wo, split):
    """§8(f) row 1: the fused upsample+warp vs F.interpolate (torch CPU) then the kornia
    restatement; integer (3x) and non-integer scales, no-op scale, C not a multiple of 8."""
    from mvdet_amd import ops
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm
    rng = np.random.default_rng(B * 977 + C + h)
    feat = torch.from_numpy(np.maximum(rng.standard_normal((B, C, h, w)), 0).astype(np.float32))
    M = torch.from_numpy(_rand_h(rng, H, W, ho, wo)).float()[None]
    m_norm = kornia_src_norm_from_dst_norm(M, (H, W), (ho, wo))[0]
    ref = kornia_warp.warp_perspective(cpu_path.upsample(feat, (H, W)), M.repeat(B, 1, 1), (ho, wo))
    if split:
        dst = torch.zeros(ops.split_shape(B, C, ho, wo), dtype=torch.bfloat16, device=DEV)
        ops.warp_views_upsampled_into([feat.to(DEV)], (H, W), [m_norm], [dst], split=True)
        got = ops.split_decode(dst, C).cpu()
    else:
        dst = torch.zeros((B, C, ho, wo), device=DEV)
        ops.warp_views_upsampled_into([feat.to(DEV)], (H, W), [m_norm], [dst])
        got = dst.cpu()
    assert_parity(got, ref, "upsample+warp")
    assert parity_stats(got, ref)["normwise"] < 1e-4  # the warp's own fp32 coordinate rounding (cf. 2e-4)


def test_upsample_warp_fused_rejects_downsampling():
    from mvdet_amd import ops
    feat = torch.zeros((1, 8, 20, 20), device=DEV)
    with pytest.raises(ValueError):
        ops.warp_views_upsampled_into([feat], (10, 40), [torch.eye(3)], [torch.zeros((1, 8, 4, 4), device=DEV)])


def test_warp_identity_translation_oob_behind_camera():
    from mvdet_amd import warp_perspective
    rng = np.random.default_rng(5)
    src = torch.from_numpy(rng.standard_normal((1, 4, 9, 11)).astype(np.float32))
    out = warp_perspective(src.to(DEV), torch.eye(3)[None].to(DEV), (9, 11)).cpu()
    np.testing.assert_allclose(out.numpy(), src.numpy(), atol=1e-5)
    M = torch.tensor([[[1.0, 0, -0.5], [0, 1, 0], [0, 0, 1]]])
    out = warp_perspective(src.to(DEV), M.to(DEV), (9, 11)).cpu()
    np.testing.assert_allclose(out.numpy(), kornia_warp.warp_perspective(src, M, (9, 11)).numpy(), atol=1e-5)
    far = torch.tensor([[[1.0, 0, 100.0], [0, 1, 100.0], [0, 0, 1]]])
    assert warp_perspective(src.to(DEV), far.to(DEV), (4, 4)).abs().max().item() == 0
    Minv = -np.eye(3)
    M = torch.from_numpy(np.linalg.inv(Minv)).float()[None]
    out = warp_perspective(torch.ones(1, 1, 8, 8, device=DEV), M.to(DEV), (8, 8))
    assert out.min().item() > 0.99  # no cheirality mask (reference quirk)


def test_warp_strided_src_and_channel_slice_dst():
    from mvdet_amd import ops
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm
    rng = np.random.default_rng(9)
    big = torch.from_numpy(rng.standard_normal((2, 40, 30, 50)).astype(np.float32)).to(DEV)
    src = big[:, 5:25, :, 3:45]                          # non-contiguous view
    M = torch.from_numpy(np.stack([_rand_h(rng, 30, 42, 20, 24) for _ in range(2)])).float()
    m_norm = kornia_src_norm_from_dst_norm(M, (30, 42), (20, 24)).to(DEV).contiguous()
    dst_full = torch.full((2, 50, 20, 24), 7.0, device=DEV)
    ops.warp_into(src, m_norm, dst_full[:, 10:30])
    ref = kornia_warp.warp_perspective(src.cpu().contiguous(), M, (20, 24))
    assert_parity(dst_full[:, 10:30].cpu(), ref, "slice")
    assert (dst_full[:, :10] == 7).all() and (dst_full[:, 30:] == 7).all()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_warp_views_batched_launch(dtype):
    """mvbev_warp_views_*: several views in one launch, each into a slice of a shared slab."""
    from mvdet_amd import ops
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm
    rng = np.random.default_rng(17)
    B, C, H, W, ho, wo, N = 2, 24, 33, 61, 19, 45, 5
    srcs = [torch.from_numpy(np.maximum(rng.standard_normal((B, C, H, W)), 0).astype(np.float32)) for _ in range(N)]
    Ms = [torch.from_numpy(_rand_h(rng, H, W, ho, wo)).float()[None] for _ in range(N)]
    slab = torch.full((N, B, C + 8, ho, wo), 5.0, device=DEV, dtype=dtype)
    mn = [kornia_src_norm_from_dst_norm(M, (H, W), (ho, wo))[0] for M in Ms]
    ops.warp_views_into([s.to(DEV, dtype) for s in srcs], mn, [slab[i, :, :C] for i in range(N)])
    for i in range(N):
        ref = kornia_warp.warp_perspective(srcs[i].to(dtype).float(), Ms[i].repeat(B, 1, 1), (ho, wo))
        s = parity_stats(slab[i, :, :C].float().cpu(), ref)
        assert s["normwise"] < (1e-5 if dtype == torch.float32 else 2e-3), (i, s)
    assert (slab[:, :, C:] == 5).all()


@pytest.mark.parametrize("src_dtype", [torch.float32, torch.float16])
def test_warp_views_split_bf16_layout(src_dtype):
    """The pre-split slab layout: hi + lo reproduces the fp32 warp to ~2^-17 relative."""
    from mvdet_amd import ops
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm
    rng = np.random.default_rng(23)
    B, C, H, W, ho, wo, N = 2, 21, 30, 50, 17, 37, 3       # C not a multiple of 8: zero-filled tail
    srcs = [torch.from_numpy(rng.standard_normal((B, C, H, W)).astype(np.float32)).to(src_dtype) for _ in range(N)]
    Ms = [torch.from_numpy(_rand_h(rng, H, W, ho, wo)).float()[None] for _ in range(N)]
    slab = torch.full((N,) + ops.split_shape(B, C, ho, wo), 3.0, dtype=torch.bfloat16, device=DEV)
    mn = [kornia_src_norm_from_dst_norm(M, (H, W), (ho, wo))[0] for M in Ms]
    ops.warp_views_into([s.to(DEV) for s in srcs], mn, [slab[i] for i in range(N)], split=True)
    for i in range(N):
        ref = kornia_warp.warp_perspective(srcs[i].float(), Ms[i].repeat(B, 1, 1), (ho, wo))
        got = ops.split_decode(slab[i]).cpu()
        s = parity_stats(got[:, :C], ref)
        assert s["normwise"] < 2e-5, (i, s)
        assert (got[:, C:] == 0).all()


@pytest.mark.parametrize("upsampled", [False, True])
def test_warp_dst_zeroed_skips_exactly_the_outside_pixels(upsampled):
    """MVBEV_WARP_DST_ZEROED (the engine's persistent zero-filled slab): into a zeroed dst the
    result is bitwise the plain warp's; into a NaN-filled one only pixels whose sample falls
    outside the source (exact zeros of the plain warp) keep their old value."""
    from mvdet_amd import ops
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm
    rng = np.random.default_rng(29)
    B, C, h, w, H, W, ho, wo = 2, 16, 10, 16, 30, 48, 20, 40
    M = torch.tensor([[[1.2, 0.1, 20.0], [0.05, 1.1, -4.0], [0.0, 0.001, 1.0]]])  # grid columns u < ~19 sample x < 0
    m = kornia_src_norm_from_dst_norm(M, (H, W), (ho, wo))[0]
    if upsampled:
        src = torch.from_numpy(np.maximum(rng.standard_normal((B, C, h, w)), 0).astype(np.float32)).to(DEV)

        def run(dst, z):
            ops.warp_views_upsampled_into([src], (H, W), [m], [dst], split=True, dst_zeroed=z)
    else:
        src = torch.from_numpy(np.maximum(rng.standard_normal((B, C, H, W)), 0).astype(np.float32)).to(DEV)

        def run(dst, z):
            ops.warp_views_into([src], [m], [dst], split=True, dst_zeroed=z)
    shape = ops.split_shape(B, C, ho, wo)
    ref = torch.full(shape, float("nan"), dtype=torch.bfloat16, device=DEV)
    run(ref, False)
    zero = torch.zeros(shape, dtype=torch.bfloat16, device=DEV)
    run(zero, True)
    assert torch.equal(zero, ref)
    stale = torch.full(shape, float("nan"), dtype=torch.bfloat16, device=DEV)
    run(stale, True)
    got, want = ops.split_decode(stale, C), ops.split_decode(ref, C)
    kept = torch.isnan(got).all(dim=1)             # [B, ho, wo]: pixels the flagged warp skipped
    outside = (want == 0).all(dim=1)
    assert kept.any() and (~kept).any()
    assert not (kept & ~outside).any()             # only exact-zero pixels are skipped
    assert kept.sum() >= 0.95 * outside.sum()      # (inside pixels with all-zero ReLU features are rare)
    keep = (~kept)[:, None].expand_as(got)
    assert torch.equal(got[keep], want[keep])


def test_warp_f16_storage():
    from mvdet_amd import warp_perspective
    rng = np.random.default_rng(11)
    src = np.maximum(rng.standard_normal((2, 33, 27, 48)), 0).astype(np.float16)
    M = torch.from_numpy(np.stack([_rand_h(rng, 27, 48, 12, 36) for _ in range(2)])).float()
    got = warp_perspective(torch.from_numpy(src).to(DEV), M.to(DEV), (12, 36)).float().cpu()
    ref = kornia_warp.warp_perspective(torch.from_numpy(src.astype(np.float32)), M, (12, 36))
    s = parity_stats(got, ref)
    assert s["normwise"] < 2e-3, s  # fp16 output rounding (2^-11 relative)


def test_warp_rejects_bad_input_like_kornia():
    from mvdet_amd import warp_perspective
    with pytest.raises(ValueError):
        warp_perspective(torch.zeros(3, 4, 5, device=DEV), torch.eye(3)[None].to(DEV), (2, 2))
    with pytest.raises(ValueError):
        warp_perspective(torch.zeros(1, 3, 4, 5, device=DEV), torch.eye(3).to(DEV), (2, 2))
    with pytest.raises(TypeError):
        warp_perspective(np.zeros((1, 3, 4, 5)), torch.eye(3)[None], (2, 2))


# ---------------------------------------------------------------------------------- convs

# normwise bounds of the conv kernels vs torch fp32 (the 1e-3 parity gate is the outer bound)
CONV_TOL = {"fp32": 2e-5, "bf16x3": 5e-5}


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
@pytest.mark.parametrize("B,cin,H,W,d,relu,bias", [(1, 8, 4, 32, 1, True, True), (1, 770, 13, 37, 1, True, True),
                                                   (2, 19, 9, 70, 2, False, True), (1, 512, 20, 33, 2, True, True),
                                                   (1, 3, 3, 5, 1, False, False)])
def test_conv3x3_vs_torch(B, cin, H, W, d, relu, bias, precision):
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(cin * 7 + H)
    cout = 256 if cin < 100 else 128
    x = torch.rand(B, cin, H, W, generator=g)
    w = (torch.rand(cout, cin, 3, 3, generator=g) - 0.5) / np.sqrt(cin * 9)
    b = torch.rand(cout, generator=g) - 0.5 if bias else None
    ref = F.conv2d(x, w, b, padding=d, dilation=d)
    if relu:
        ref = F.relu(ref)
    K = ops.padded_channels(cin)
    xp = torch.full((B, K, H, W), 1e30)  # padding channels must not leak (zero weights)
    xp[:, :cin] = x
    pk = ops.PackedConv3x3(list(range(cin)) + [-1] * (K - cin), precision).get(w.to(DEV))
    got = ops.conv3x3(xp.to(DEV), pk, cout, b.to(DEV) if bias else None, d, relu).cpu()
    assert_parity(got, ref, f"conv3x3 {precision}", normwise_tol=CONV_TOL[precision])


def test_conv3x3_bf16x3_fp16_input_is_exact_split():
    """fp16-storage input (config 4): an fp16 value is exactly bf16 hi + lo."""
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(77)
    x = torch.rand(2, 64, 11, 40, generator=g).half()
    w = (torch.rand(128, 64, 3, 3, generator=g) - 0.5) / 24
    ref = F.relu(F.conv2d(x.float(), w, None, padding=1))
    pk = ops.PackedConv3x3(None, "bf16x3").get(w.to(DEV))
    got = ops.conv3x3(x.to(DEV), pk, 128, None, 1, True).cpu()
    assert_parity(got, ref, "bf16x3 f16-in", normwise_tol=5e-5)


@pytest.mark.parametrize("K,split", [(48, True), (520, False), (528, True), (1024, False)])
def test_conv3x3_bf16x3_split_k_tail(K, split):
    """The split-K tail (288 tiles: one full round + a tail whose tiles are cut into
    K-ranges, fixed-order fixup), 3-64 K-chunks (3: too short to split, plain schedule);
    matches torch, is deterministic, and agrees with the whole-round schedule to fp32
    summation-order rounding."""
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(K)
    B, H, W, cout = 1, 64, 288, 512
    x = torch.rand(B, K, H, W, generator=g)
    w = (torch.rand(cout, K, 3, 3, generator=g) - 0.5) / np.sqrt(K * 9)
    b = torch.rand(cout, generator=g) - 0.5
    ref = F.relu(F.conv2d(x, w, b, padding=1))
    pk = ops.PackedConv3x3(None, "bf16x3").get(w.to(DEV))
    xd = (_split_encode(x) if split else x).to(DEV)
    desc = ops.conv_desc(B, K, H, W, group=K, group_stride=0, batch_stride=K * H * W)
    need = ops.conv3x3_workspace_bytes(desc, cout)
    assert (need > 0) == (K >= 520)
    ws = torch.full((max(need, 4) // 4,), float("nan"), device=DEV)  # every read slot is written first
    bd = b.to(DEV)
    got = ops.conv3x3_desc(xd, desc, pk, cout, bias=bd, relu=True, workspace=ws).cpu()
    again = ops.conv3x3_desc(xd, desc, pk, cout, bias=bd, relu=True, workspace=ws).cpu()
    plain = ops.conv3x3_desc(xd, desc, pk, cout, bias=bd, relu=True).cpu()
    assert_parity(got, ref, "stream-K", normwise_tol=CONV_TOL["bf16x3"])
    assert torch.equal(got, again)
    torch.testing.assert_close(got, plain, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("cfg", [1, 2])
def test_frustum_mask_is_exact_and_conv1_unchanged(cfg):
    """A cleared mask bit means the view's warped features are exactly 0 over the tile and
    its halo; conv1 with the mask equals dense conv1 bit for bit (skipped products are
    exact zeros).  Config rigs at reduced channel count."""
    from mvdet_amd import ProjectFuse, ops, synthetic
    from mvdet_amd.geometry import projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    N, C, B = ds.num_cam, 32, 1
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm = projection_matrices(ds)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=9 + v, device=DEV)
             for v in range(N)]
    mc = torch.nn.Sequential(torch.nn.Conv2d(N * C + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)
    # the direct conv1 (the Winograd form's masked = unmasked is test_gpu_wino's); split-K tails
    # re-associate the sums
    dense = ProjectFuse(pm, up, grid, C, frustum=False, split_k=False, wino_conv1=False)
    sparse = ProjectFuse(pm, up, grid, C, split_k=False, wino_conv1=False)
    assert sparse.frustum
    with torch.no_grad():
        ref = dense.project_fuse(feats, mc)
        y1_ref = dense.workspace(B, DEV).y1.clone()
        got = sparse.project_fuse(feats, mc)
        ws = sparse.workspace(B, DEV)
    assert torch.equal(ws.y1, y1_ref)
    assert torch.equal(got, ref)
    H, W = grid
    th = sparse.conv1_tile_rows()
    mask = sparse.conv1_mask(DEV, 0, H).cpu().numpy().astype(np.uint32)
    tx = -(-W // 32)
    warped = [sparse.view_slice(ws, v).abs().amax(dim=(0, 1)).cpu() for v in range(N)]  # [H, W]
    kept = 0
    for t, bits in enumerate(mask):
        r0, c0 = (t // tx) * th, (t % tx) * 32
        for v in range(N):
            region = warped[v][max(0, r0 - 1):r0 + th + 1, max(0, c0 - 1):c0 + 33]
            if not (bits >> v) & 1:
                assert region.max().item() == 0, (t, v)
            else:
                kept += 1
    assert 0 < kept < mask.size * N  # the rig's frustums leave work to skip


def _split_encode(x: torch.Tensor) -> torch.Tensor:
    """fp32 [B, C, H, W] (C % 8 == 0) -> split-bf16 blocked [B, C/8, H, W, 2, 8]."""
    B, C, H, W = x.shape
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    t = torch.stack([hi, lo], 0).reshape(2, B, C // 8, 8, H, W)
    return t.permute(1, 2, 4, 5, 0, 3).contiguous()


@pytest.mark.parametrize("layout", ["f32", "split"])
@pytest.mark.parametrize("S,Cs", [(3, 8), (2, 24), (5, 16)])
def test_conv3x3_bf16x3_grouped_slab(S, Cs, layout):
    """View-major slab input (channel groups of Cs with a gap between groups), incl. groups
    that are not a multiple of the kernel's 16-channel chunk and an odd 8-channel tail."""
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(S * 100 + Cs)
    B, H, W, cout = 2, 9, 45, 128
    xs = torch.rand(S, B, Cs, H, W, generator=g)
    K = S * Cs
    w = (torch.rand(cout, K, 3, 3, generator=g) - 0.5) / np.sqrt(K * 9)
    ref = F.relu(F.conv2d(xs.permute(1, 0, 2, 3, 4).reshape(B, K, H, W), w, None, padding=1))
    pk = ops.PackedConv3x3(None, "bf16x3").get(w.to(DEV))
    if layout == "f32":
        slab = xs.to(DEV)
        desc = ops.conv_desc(B, K, H, W, group=Cs, group_stride=B * Cs * H * W, batch_stride=Cs * H * W)
    else:
        slab = torch.stack([_split_encode(xs[v]) for v in range(S)]).to(DEV)  # [S,B,G,H,W,2,8]
        # strides in 4-byte units of the logical fp32 element (one element = hi + lo bf16)
        desc = ops.conv_desc(B, K, H, W, group=Cs, group_stride=B * Cs * H * W, batch_stride=Cs * H * W)
    got = ops.conv3x3_desc(slab, desc, pk, cout, relu=True).cpu()
    assert_parity(got, ref, f"grouped {layout}", normwise_tol=CONV_TOL["bf16x3"])


@pytest.mark.parametrize("B,H,W,rows", [(1, 30, 360, (0, 30)),    # EW 8, 48-row strips (one partial)
                                         (2, 25, 76, (3, 25)),     # EW 16 (W % 32 = 12), row band
                                         (1, 61, 48, (0, 61)),     # EW 16 at W % 32 = 16, 3 strips
                                         (2, 13, 37, (0, 13))])    # EW 8, W % 32 = 5
@pytest.mark.parametrize("masked", [False, True])
def test_conv3x3_edge_strip_tiles(B, H, W, rows, masked):
    """MVBEV_TILES_EDGE_STRIP (mvbev_conv3x3_bf16x3_ex3): the last W % 32 columns as
    (384/EW) x EW tiles give y bitwise equal to the 12 x 32 grid tiles (same per-pixel K order),
    with and without a frustum-style group mask + heavy-first order, and match F.conv2d."""
    from mvdet_amd import _native, ops
    g = torch.Generator().manual_seed(H * W + B)
    S, Cs, cout = 3, 16, 256
    K = S * Cs
    xs = torch.rand(S, B, Cs, H, W, generator=g)
    # zero view 1 on the right part of the grid so a mask has something exact to skip
    xs[1, :, :, :, W // 2:] = 0
    w = (torch.rand(cout, K, 3, 3, generator=g) - 0.5) / np.sqrt(K * 9)
    init = torch.rand(cout, H, W, generator=g)
    r0, r1 = rows
    ref = F.relu(F.conv2d(xs.permute(1, 0, 2, 3, 4).reshape(B, K, H, W), w, None, padding=1) + init)[:, :, r0:r1]
    pk = ops.PackedConv3x3(None, "bf16x3").get(w.to(DEV))
    slab = torch.stack([_split_encode(xs[v]) for v in range(S)]).to(DEV)
    desc = ops.conv_desc(B, K, H, W, group=Cs, group_stride=B * Cs * H * W, batch_stride=Cs * H * W,
                         out_row0=r0, out_rows=r1 - r0)
    gx = _native.ring_tile_space(desc, _native.TILES_GRID)
    es = _native.ring_tile_space(desc, _native.TILES_EDGE_STRIP)
    assert es is not None and es[0] == W // 32 and es[3] == (8 if W % 32 <= 8 else 16)
    assert es[2] == -(-(r1 - r0) // es[4])

    def masks(space_geom):
        tx, ty, ne, ew, er = space_geom
        m = []
        for t in range(tx * ty + ne):
            c0 = (t % tx) * 32 if t < tx * ty else tx * 32
            m.append(0b101 | (0b010 if c0 - 1 < W // 2 else 0))  # view 1 is zero from column W // 2 on
        mt = torch.tensor(m, dtype=torch.int32, device=DEV)
        return mt, ops.heavy_first_order(mt, B)

    kw = dict(init=init.to(DEV), relu=True, dilation=1)
    if masked:
        gm, go = masks(gx)
        em, eo = masks(es)
        grid = ops.conv3x3_desc(slab, desc, pk, cout, group_mask=gm, tile_order=go, **kw)
        strip = ops.conv3x3_desc(slab, desc, pk, cout, group_mask=em, tile_order=eo,
                                 tile_space=_native.TILES_EDGE_STRIP, **kw)
    else:
        grid = ops.conv3x3_desc(slab, desc, pk, cout, **kw)
        strip = ops.conv3x3_desc(slab, desc, pk, cout, tile_space=_native.TILES_EDGE_STRIP, **kw)
    assert torch.equal(strip, grid)
    assert_parity(strip.cpu(), ref, "edge strip", normwise_tol=CONV_TOL["bf16x3"])
    # split-bf16 output (conv1 -> conv2 in the detector) is bitwise the same too
    ysplit = torch.empty(ops.split_shape(B, cout, r1 - r0, W), dtype=torch.bfloat16, device=DEV)
    ops.conv3x3_desc(slab, desc, pk, cout, out=ysplit, tile_space=_native.TILES_EDGE_STRIP, **kw)
    assert torch.equal(ops.split_decode(ysplit, cout), ops.split_decode(
        ops.conv3x3_desc(slab, desc, pk, cout, out=torch.empty_like(ysplit), **kw), cout))


def test_edge_strip_refusals():
    """Spaces that do not apply, and combinations the edge strip does not support, raise."""
    from mvdet_amd import _native, ops
    for W in (64, 250, 96):  # W % 32 == 0 or > 16: no strip
        assert _native.ring_tile_space(ops.conv_desc(1, 16, 12, W, 16, 0, 0), _native.TILES_EDGE_STRIP) is None
    x = torch.zeros(ops.split_shape(1, 16, 12, 40), dtype=torch.bfloat16, device=DEV)
    pk = ops.PackedConv3x3(None, "bf16x3").get(torch.zeros(128, 16, 3, 3, device=DEV))
    desc = ops.conv_desc(1, 16, 12, 40, 16, 0, 16 * 12 * 40)
    with pytest.raises(_native.NativeError):  # dilation 2 / no ReLU: conv1 + ReLU only
        ops.conv3x3_desc(x, desc, pk, 128, dilation=2, relu=True, tile_space=_native.TILES_EDGE_STRIP)
    with pytest.raises(_native.NativeError):
        ops.conv3x3_desc(x, desc, pk, 128, relu=False, tile_space=_native.TILES_EDGE_STRIP)


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
@pytest.mark.parametrize("d", [1, 2])
def test_conv3x3_row_band_and_init(d, precision):
    """Row bands (the multi-GPU fusion) and the init (coord-term) epilogue."""
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(40 + d)
    B, cin, H, W, cout = 2, 16, 23, 41, 128
    x = torch.rand(B, cin, H, W, generator=g)
    w = (torch.rand(cout, cin, 3, 3, generator=g) - 0.5) / 12
    init = torch.rand(cout, H, W, generator=g)
    ref = F.relu(F.conv2d(x, w, None, padding=d, dilation=d) + init)
    pk = ops.PackedConv3x3(None, precision).get(w.to(DEV))
    xd, initd = x.to(DEV), init.to(DEV)
    for (a, b_) in ((0, 7), (5, 19), (16, 23)):
        in0, in1 = max(0, a - d), min(H, b_ + d)
        xin = xd[:, :, in0:in1].contiguous()
        desc = ops.conv_desc(B, cin, H, W, group=cin, group_stride=0, batch_stride=cin * (in1 - in0) * W,
                             in_row0=in0, in_rows=in1 - in0, out_row0=a, out_rows=b_ - a)
        got = ops.conv3x3_desc(xin, desc, pk, cout, init=initd, dilation=d, relu=True).cpu()
        assert_parity(got, ref[:, :, a:b_], f"band {a}:{b_}", normwise_tol=CONV_TOL[precision])


@pytest.mark.parametrize("C,H,W,d", [(512, 12, 36, 4), (7, 5, 70, 1), (33, 9, 130, 2),
                                     (512, 20, 360, 4),   # 16-B quad kernel (W % 4 == 0, dilation 4)
                                     (40, 10, 30, 4)])    # dilation 4, W % 4 != 0: scalar kernel
def test_conv3x3_cout1_vs_torch(C, H, W, d):
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(C + H)
    x = torch.rand(2, C, H, W, generator=g)
    w = (torch.rand(1, C, 3, 3, generator=g) - 0.5) / np.sqrt(C * 9)
    ref = F.conv2d(x, w, None, padding=d, dilation=d)
    got = ops.conv3x3_cout1(x.to(DEV), w.to(DEV), d).cpu()
    assert_parity(got, ref, "cout1", normwise_tol=2e-5)
    # band: rows [2, H-1) from an input buffer holding rows [1, H)
    got_b = ops.conv3x3_cout1(x[:, :, 1:].contiguous().to(DEV), w.to(DEV), d, H=H, in_row0=1, out_row0=2,
                              out_rows=H - 3).cpu()
    sub = ref[:, :, 2:H - 1].clone()
    if d >= 2:  # rows that need input row 0 differ (not in the buffer): compare the rest
        keep = [r for r in range(2, H - 1) if r - d >= 1 or r - d < 0]
        sub, got_b = sub[:, :, [r - 2 for r in keep]], got_b[:, :, [r - 2 for r in keep]]
    assert_parity(got_b, sub, "cout1 band", normwise_tol=2e-5)


def test_packed_weight_cache_tracks_in_place_updates():
    from mvdet_amd import ops
    w = torch.randn(128, 16, 3, 3, device=DEV)
    pc = ops.PackedConv3x3()
    p0 = pc.get(w).clone()
    assert torch.equal(pc.get(w), p0)
    with torch.no_grad():
        w.mul_(2)
    assert torch.allclose(pc.get(w), 2 * p0)


# ---------------------------------------------------------------------------------- golden

def _ds_from_golden(g):
    from mvdet_amd.synthetic import SyntheticBase, SyntheticFrameDataset
    m = g["meta"]
    base = SyntheticBase("fixture", m["img_shape"], m["worldgrid_shape"], m["num_cam"], g["G"],
                         tuple(g["K"]), tuple(g["E"]))
    return SyntheticFrameDataset(base, grid_reduce=m["grid_reduce"], img_reduce=m["img_reduce"])


@pytest.mark.parametrize("name", ["module_wt2", "module_mx3_b2"])
def test_detector_forward_matches_reference_golden(name):
    """The drop-in module's forward (backbone bypassed exactly as the fixture did)
    reproduces the reference's own forward outputs."""
    import torch.nn as nn
    from mvdet_amd import PerspTransDetector
    g = load_golden(name)
    m = g["meta"]
    model = PerspTransDetector(_ds_from_golden(g))
    params = fixtures.head_params(m["num_cam"], m["weight_seed"])
    assert fixtures.params_sha256(params) == m["weights_sha256"]
    sd = model.state_dict()
    sd.update({k: torch.from_numpy(v) for k, v in params.items()})
    model.load_state_dict(sd)
    model.base_pt1, model.base_pt2 = nn.Identity(), nn.Identity()
    model.eval()
    with torch.no_grad():
        map_res, imgs_res = model(torch.from_numpy(g["feat_in"]))
        torch.cuda.synchronize()
    assert map_res.shape == g["map_result"].shape
    assert_parity(map_res.cpu(), g["map_result"], f"{name} map_result")
    assert_parity(torch.stack(imgs_res, 0).cpu(), g["imgs_result"], f"{name} imgs_result")
    eng = model.engine
    ws = eng.workspace(m["B"], "cuda:0")
    # the inference default writes conv1's row transform straight from the warp (no slab):
    # the intermediate-tensor checks below run the slab path of the same module
    assert eng.wino_warp and ws.t_from_warp
    with pytest.raises(RuntimeError):
        eng.view_slice(ws, 0)
    eng.wino_warp = False
    with torch.no_grad():
        map2, _ = model(torch.from_numpy(g["feat_in"]))
    assert not ws.t_from_warp
    assert_parity(map2.cpu(), g["map_result"], f"{name} map_result (slab path)")
    N, C = m["num_cam"], 512
    warped = torch.stack([eng.view_slice(ws, v) for v in range(N)], 1)  # [B, N, C, ho, wo]
    np.testing.assert_allclose(warped.double().sum(dim=(3, 4)).cpu().numpy(), g["warp_out_chsum"],
                               rtol=2e-3, atol=2e-2)
    if "warp_out" in g:
        assert_parity(warped.cpu(), g["warp_out"], "warp_out")
        assert_parity(eng.y1_fp32(ws).cpu(), g["conv1_relu"], "conv1")
        with torch.no_grad():  # inference fuses conv2 into conv3 (no y2 in HBM): run conv2 alone
            eng.conv2(ws, model.map_classifier[2])
        assert_parity(ws.y2.cpu(), g["conv2_relu"], "conv2")


def test_fill_coord_map_matches_reference_coord_map():
    from mvdet_amd import ops
    g = load_golden("module_mx3_b2")
    ho, wo = g["meta"]["reducedgrid_shape"]
    dst = torch.full((2, 5, ho, wo), 3.0, device=DEV)
    ops.fill_coord_map(dst[:, 1:3])
    np.testing.assert_array_equal(dst[:, 1:3].cpu().numpy(), np.repeat(g["coord_map"], 2, 0))
    assert (dst[:, 0] == 3).all() and (dst[:, 3:] == 3).all()


@pytest.mark.parametrize("hw,with_bias", [((120, 360), True), ((37, 70), False), ((2, 5), True)])
def test_coord_term_matches_conv2d_of_the_coord_map(hw, with_bias):
    """mvbev_coord_term_f32 (ABI 12300): conv1's bias + conv2d over the two coord channels (zero padding)
    equals torch's float64 conv2d of the reference's coord map (golden-pinned by
    test_fill_coord_map_matches_reference_coord_map) with the same weights, to fp32 rounding (1e-6 of
    the term's scale), on the cfg2 grid, a grid with ragged tiles and a 2-row grid (every row a border)."""
    import torch.nn.functional as F
    from mvdet_amd import ops
    from oracle.cpu_path import coord_map
    H, W = hw
    cin, c0, cout = 11, 8, 64
    gen = torch.Generator().manual_seed(H * W)
    w = torch.randn((cout, cin, 3, 3), generator=gen)
    b = torch.randn((cout,), generator=gen) if with_bias else None
    got = ops.coord_term(w.to(DEV), None if b is None else b.to(DEV), c0, (H, W)).cpu()
    ref = F.conv2d(coord_map(H, W).double(), w[:, c0:c0 + 2].double(), None if b is None else b.double(), padding=1)[0]
    err = (got.double() - ref).abs().max().item()
    assert err <= 1e-6 * max(1.0, ref.abs().max().item()), err
    with pytest.raises(Exception):
        ops.coord_term(w.to(DEV), None, cin - 1, (H, W))  # the y channel past the weight's channels


@pytest.mark.parametrize("band", [None, (5, 23)])
def test_conv2_conv3_fused_matches_unfused(band):
    """conv2 -> conv3 without y2 in HBM (conv2's epilogue writes conv3's per-tap partials,
    a reduce kernel sums them): same map as conv2 + conv3 on y2 to fp32 summation order, on a
    grid with partial tiles (37 x 70) and on a row band; bitwise identical between the band
    and the whole grid (per-pixel partials do not depend on the tile decomposition)."""
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    ds = synthetic.wildtrack_like(2, 4, seed=3, img_shape=(108, 192), worldgrid_shape=(148, 280))
    C = 32
    up = ds.upsample_shape
    feats = [synthetic.synthetic_features(1, C, [u // 3 for u in up], up, seed=70 + v, device=DEV) for v in range(2)]
    pm = projection_matrices(ds)
    params = fixtures.head_params(2, seed=9, C=C)
    mc = torch.nn.Sequential(torch.nn.Conv2d(C * 2 + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False))
    mc.load_state_dict({k.replace("map_classifier.", ""): torch.from_numpy(v) for k, v in params.items()
                        if k.startswith("map_classifier.")})
    mc = mc.to(DEV)
    outs = {}
    for fused in (True, False):
        # the direct conv1 and conv2: bands are bitwise the whole grid (the Winograd convs' 3-row
        # tiles start at the band's first row, so their band sums group differently;
        # test_gpu_wino.py covers the Winograd conv2's partials)
        eng = ProjectFuse(pm, tuple(up), tuple(ds.reducedgrid_shape), C, fuse_conv3=fused, wino_conv1=False,
                          wino_conv2=False)
        with torch.no_grad():
            ws = eng.workspace(1, DEV, band=band)
            eng.warp_views(ws, [0, 1], feats)
            assert eng.conv3_fused_applies(ws) == fused
            outs[fused] = eng.fuse(ws, mc).cpu()
            if band is not None and fused:
                whole = eng.workspace(1, DEV)
                eng.warp_views(whole, [0, 1], feats)
                full = eng.fuse(whole, mc).cpu()
                assert torch.equal(outs[fused], full[:, :, band[0]:band[1]])
    assert outs[True].shape == outs[False].shape
    assert_parity(outs[True], outs[False], "fused vs unfused conv3")
