"""GPU parity of the native backward against torch's CPU autograd.

The oracle for every gradient is what the reference trains with (``trainer.py:38-49``):
torch-CPU autograd through the kornia-0.6.11 restatement (grid_sample's backward) and
``F.conv2d`` / ReLU (``oracle/cpu_path.py``), or the closed-form ``torch.nn.grad`` adjoints in
float64 for the individual kernels.  Gate: ``helpers.assert_parity`` (elementwise
|got-ref| <= 1e-3*|ref| + 1e-3*max|ref| and normwise <= 1e-3), the north_star's 1e-3
relative fp32 tolerance.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import assert_parity, assert_parity_t, parity_stats
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


def _split_encode(x: torch.Tensor) -> torch.Tensor:
    """fp32 [B,C,H,W] (C % 8 == 0) -> the split-bf16 blocked layout [B, C/8, H, W, 2, 8]."""
    B, C, H, W = x.shape
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    t = torch.stack([hi, lo], 0).reshape(2, B, C // 8, 8, H, W)
    return t.permute(1, 2, 4, 5, 0, 3).contiguous()


# ---------------------------------------------------------------------------------- warp

@pytest.mark.parametrize("B,C,H,W,ho,wo", [(1, 5, 27, 48, 12, 36), (2, 19, 30, 41, 17, 23),
                                           (1, 3, 9, 11, 20, 30)])
def test_warp_backward_vs_grid_sample_autograd(B, C, H, W, ho, wo):
    """Adjoint gather == grid_sample's backward under the kornia restatement (CPU fp32)."""
    from mvdet_amd import ops
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm
    rng = np.random.default_rng(100 * B + C)
    n = 3
    Ms = [torch.from_numpy(_rand_h(rng, H, W, ho, wo)).float()[None] for _ in range(n)]
    gouts = [torch.from_numpy(rng.standard_normal((B, C, ho, wo)).astype(np.float32)) for _ in range(n)]
    refs = []
    for M, g in zip(Ms, gouts):
        src = torch.zeros((B, C, H, W), requires_grad=True)
        kornia_warp.warp_perspective(src, M.repeat(B, 1, 1), (ho, wo)).backward(g)
        refs.append(src.grad)
    mn = [kornia_src_norm_from_dst_norm(M, (H, W), (ho, wo))[0] for M in Ms]
    # grad_src rows inside a wider buffer (strided view) and pre-filled: the op accumulates
    bufs = [torch.full((B, C + 2, H, W), 0.5, device=DEV) for _ in range(n)]
    ops.warp_views_backward([g.to(DEV) for g in gouts], mn, [b[:, 1:C + 1] for b in bufs])
    for i in range(n):
        assert_parity(bufs[i][:, 1:C + 1].cpu() - 0.5, refs[i], f"warp adjoint view {i}")
        assert (bufs[i][:, 0] == 0.5).all() and (bufs[i][:, C + 1] == 0.5).all()


def _pix_views(splits, extra_groups=3):
    """The views' split-bf16 [B, C/8, Ho, Wo, 2, 8] gradients as group slices of ONE pixel-major tensor
    [B, Ho, Wo, G, 2, 8] (MVBEV_LAYOUT_SPLIT_BF16_PIX, as conv1's dgrad writes dslab), with
    ``extra_groups`` foreign groups after them (the per-pixel stride exceeds a view's C/8)."""
    B, g8, Ho, Wo = splits[0].shape[:4]
    parts = [sp.permute(0, 2, 3, 1, 4, 5) for sp in splits]
    parts.append(torch.full((B, Ho, Wo, extra_groups, 2, 8), float("nan"), dtype=splits[0].dtype,
                            device=splits[0].device))
    full = torch.cat(parts, dim=3).contiguous()
    return [full[:, :, :, v * g8:(v + 1) * g8] for v in range(len(splits))]


@pytest.mark.parametrize("B,C,h,w,H,W,ho,wo", [(1, 8, 9, 16, 27, 48, 12, 36), (2, 16, 10, 14, 27, 48, 17, 23),
                                               (1, 24, 30, 53, 90, 160, 120, 360), (1, 72, 7, 20, 20, 57, 15, 40),
                                               (1, 16, 5, 9, 30, 54, 11, 13)])
def test_upsampled_warp_adjoint_vs_autograd(B, C, h, w, H, W, ho, wo):
    """The fused 3x-upsample + warp adjoint (plan of S * U, <= 9 entries per output pixel):
    the gradient w.r.t. the backbone-resolution map equals torch-CPU autograd through
    F.interpolate (bilinear, align_corners=False; persp_trans_detector.py:65) and the kornia
    warp restatement (:69), from fp32 and split-bf16 grad_out (accumulating too); and the
    forward it is the adjoint of (warp_views_upsampled_into) matches the same composition.
    Scales 3x (the reference's), 2.7-3.4x and 6x; channel counts below, at and above a
    64-channel workgroup."""
    from mvdet_amd import ops
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm
    rng = np.random.default_rng(3 * C + h)
    n = 2
    Ms = [torch.from_numpy(_rand_h(rng, H, W, ho, wo)).float()[None] for _ in range(n)]
    gouts = [torch.from_numpy(rng.standard_normal((B, C, ho, wo)).astype(np.float32)) for _ in range(n)]
    feats = [torch.from_numpy(rng.standard_normal((B, C, h, w)).astype(np.float32)) for _ in range(n)]
    refs, fwd = [], []
    for M, g, f in zip(Ms, gouts, feats):
        src = f.clone().requires_grad_()
        out = kornia_warp.warp_perspective(F.interpolate(src, (H, W), mode="bilinear"), M.repeat(B, 1, 1), (ho, wo))
        out.backward(g)
        refs.append(src.grad)
        fwd.append(out.detach())
    mn = [kornia_src_norm_from_dst_norm(M, (H, W), (ho, wo))[0] for M in Ms]
    plans = [ops.WarpAdjointPlan(m, (H, W), (ho, wo), DEV, backbone_hw=(h, w)) for m in mn]
    assert plans[0].src_hw == (h, w) and plans[0].nnz <= 9 * ho * wo
    rp, col = plans[0].row_ptr.cpu(), plans[0].col[:plans[0].nnz].cpu()
    assert rp[0] == 0 and (rp[1:] >= rp[:-1]).all()
    for p in range(0, h * w, max(1, h * w // 53)):
        seg = col[rp[p]:rp[p + 1]]
        assert (seg[1:] > seg[:-1]).all()
    gdev = [g.to(DEV) for g in gouts]
    outs = [torch.full((B, C, h, w), float("nan"), device=DEV) for _ in range(n)]
    ops.warp_views_adjoint(gdev, plans, outs)
    for i in range(n):
        assert_parity(outs[i].cpu(), refs[i], f"upsampled adjoint view {i}")
    outs_s = [torch.full((B, C, h, w), float("nan"), device=DEV) for _ in range(n)]
    ops.warp_views_adjoint([_split_encode(g) for g in gdev], plans, outs_s)
    for i in range(n):
        assert_parity(outs_s[i].cpu(), refs[i], f"upsampled adjoint (split grad_out) view {i}")
    acc = [torch.full((B, C, h, w), 0.25, device=DEV) for _ in range(n)]
    ops.warp_views_adjoint([_split_encode(g) for g in gdev], plans, acc, accumulate=True)
    for i in range(n):
        assert_parity(acc[i].cpu() - 0.25, refs[i], f"upsampled adjoint, accumulating, view {i}")
    # the pixel-major split grad_out (ABI 12100): the same sums in the same order -> bitwise the split result
    pv = _pix_views([_split_encode(g) for g in gdev])
    outs_p = [torch.full((B, C, h, w), float("nan"), device=DEV) for _ in range(n)]
    ops.warp_views_adjoint(pv, plans, outs_p, pixel_major=True)
    assert all(torch.equal(a, b) for a, b in zip(outs_p, outs_s))
    acc_p = [torch.full((B, C, h, w), 0.25, device=DEV) for _ in range(n)]
    ops.warp_views_adjoint(pv, plans, acc_p, accumulate=True, pixel_major=True)
    assert all(torch.equal(a, b) for a, b in zip(acc_p, acc))
    # channels-last backbone-map gradients (the detector's maps): the same values, written in that layout
    cl = torch.channels_last
    outs_c = [torch.full((B, C, h, w), float("nan"), device=DEV).contiguous(memory_format=cl) for _ in range(n)]
    ops.warp_views_adjoint(pv, plans, outs_c, pixel_major=True)
    assert all(o.is_contiguous(memory_format=cl) and torch.equal(o.contiguous(), b) for o, b in zip(outs_c, outs_s))
    acc_c = [torch.full((B, C, h, w), 0.25, device=DEV).contiguous(memory_format=cl) for _ in range(n)]
    ops.warp_views_adjoint(pv, plans, acc_c, accumulate=True, pixel_major=True)
    assert all(torch.equal(a.contiguous(), b) for a, b in zip(acc_c, acc))
    dst = [torch.empty((B, C, ho, wo), device=DEV) for _ in range(n)]
    ops.warp_views_upsampled_into([f.to(DEV) for f in feats], (H, W), mn, dst)
    for i in range(n):
        assert_parity(dst[i].cpu(), fwd[i], f"fused forward view {i}")


@pytest.mark.parametrize("B,C,H,W,ho,wo", [(1, 5, 27, 48, 12, 36), (2, 37, 30, 41, 17, 23),
                                           (1, 3, 9, 11, 20, 30), (1, 72, 90, 160, 120, 360),
                                           (2, 16, 30, 41, 17, 23),
                                           (2, 24, 36, 48, 20, 30)])  # split: the pixel-quad kernel
def test_warp_adjoint_gather_vs_grid_sample_autograd(B, C, H, W, ho, wo):
    """The CSR-gather adjoint (plan once per geometry): equals grid_sample's backward, is
    bitwise deterministic, overwrites or accumulates, and its plan holds one entry per
    in-bounds corner of every inside sample."""
    from mvdet_amd import ops
    from mvdet_amd.geometry import kornia_src_norm_from_dst_norm
    rng = np.random.default_rng(7 * B + C)
    n = 2
    Ms = [torch.from_numpy(_rand_h(rng, H, W, ho, wo)).float()[None] for _ in range(n)]
    gouts = [torch.from_numpy(rng.standard_normal((B, C, ho, wo)).astype(np.float32)) for _ in range(n)]
    refs = []
    for M, g in zip(Ms, gouts):
        src = torch.zeros((B, C, H, W), requires_grad=True)
        kornia_warp.warp_perspective(src, M.repeat(B, 1, 1), (ho, wo)).backward(g)
        refs.append(src.grad)
    mn = [kornia_src_norm_from_dst_norm(M, (H, W), (ho, wo))[0] for M in Ms]
    plans = [ops.WarpAdjointPlan(m, (H, W), (ho, wo), DEV) for m in mn]
    rp = plans[0].row_ptr.cpu()
    assert rp[0] == 0 and (rp[1:] >= rp[:-1]).all() and plans[0].nnz <= 4 * ho * wo
    col = plans[0].col[:plans[0].nnz].cpu()
    for p in range(0, H * W, max(1, H * W // 97)):  # entries of a pixel sorted by output pixel
        seg = col[rp[p]:rp[p + 1]]
        assert (seg[1:] > seg[:-1]).all()
    gdev = [g.to(DEV) for g in gouts]
    outs = [torch.full((B, C, H, W), float("nan"), device=DEV) for _ in range(n)]  # overwritten
    ops.warp_views_adjoint(gdev, plans, outs)
    for i in range(n):
        assert_parity(outs[i].cpu(), refs[i], f"adjoint gather view {i}")
    again = [torch.empty_like(o) for o in outs]
    ops.warp_views_adjoint(gdev, plans, again)
    assert all(torch.equal(a, o) for a, o in zip(again, outs))
    ops.warp_views_adjoint(gdev, plans, again, accumulate=True)
    for a, o in zip(again, outs):
        assert torch.allclose(a, 2 * o, rtol=1e-6, atol=0)
    if C % 8 == 0:  # grad_out in the split-bf16 layout the dgrad conv writes (hi + lo)
        split = [_split_encode(g) for g in gdev]
        outs_s = [torch.empty_like(o) for o in outs]
        ops.warp_views_adjoint(split, plans, outs_s)
        for i in range(n):
            assert_parity(outs_s[i].cpu(), refs[i], f"adjoint gather (split grad_out) view {i}")
        acc_s = [o.clone() for o in outs_s]
        ops.warp_views_adjoint(split, plans, acc_s, accumulate=True)
        for a, o in zip(acc_s, outs_s):
            assert torch.allclose(a, 2 * o, rtol=1e-6, atol=0)
        # pixel-major split grad_out (ABI 12100): bitwise the split-layout result, overwriting and accumulating
        pv = _pix_views(split)
        outs_p = [torch.full_like(o, float("nan")) for o in outs]
        ops.warp_views_adjoint(pv, plans, outs_p, pixel_major=True)
        assert all(torch.equal(a, b) for a, b in zip(outs_p, outs_s))
        acc_p = [o.clone() for o in outs_p]
        ops.warp_views_adjoint(pv, plans, acc_p, accumulate=True, pixel_major=True)
        assert all(torch.equal(a, b) for a, b in zip(acc_p, acc_s))
        outs_c = [torch.full_like(o, float("nan")).contiguous(memory_format=torch.channels_last) for o in outs]
        ops.warp_views_adjoint(pv, plans, outs_c, pixel_major=True)
        assert all(torch.equal(a.contiguous(), b) for a, b in zip(outs_c, outs_s))


def test_warp_backward_no_gradient_from_outside_samples():
    from mvdet_amd import ops
    far = torch.tensor([[1.0, 0, 100.0], [0, 1, 100.0], [0, 0, 1]])  # every sample far outside
    g = torch.ones((1, 4, 6, 6), device=DEV)
    dst = torch.zeros((1, 4, 8, 8), device=DEV)
    ops.warp_views_backward([g], [far], [dst])
    assert dst.abs().max().item() == 0


# ---------------------------------------------------------------------------------- conv grads

# W % 4 == 0 with split input takes wgrad_dma_kernel (LDS-DMA staging): (12, 36, d1) and
# (13, 44, d2: a partial 64-channel tile and a partial last row segment); the others wgrad_kernel
@pytest.mark.parametrize("B,K,H,W,dil", [(1, 64, 12, 36, 1), (2, 136, 17, 37, 2), (1, 512, 30, 90, 2),
                                         (1, 24, 5, 70, 1), (2, 72, 13, 44, 2)])
@pytest.mark.parametrize("split", [False, True])
def test_conv_wgrad_vs_torch(B, K, H, W, dil, split):
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(K + H + dil)
    cout = 128
    x = F.relu(torch.randn((B, K, H, W), generator=g))
    dy = torch.randn((B, cout, H, W), generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (cout, K, 3, 3), dy.double(), padding=dil, dilation=dil)
    xd = _split_encode(x.to(DEV)) if split else x.to(DEV)
    d = ops.conv_desc(B, K, H, W, group=K, group_stride=0, batch_stride=K * H * W)
    got = ops.conv3x3_wgrad(xd, d, dy.to(DEV), dil, K)
    assert_parity(got.cpu(), ref, f"wgrad split={split}")


def test_conv_wgrad_grouped_slab_with_channel_map():
    """conv1's form: a view-major grouped slab (each group padded to a multiple of 8
    channels) scattered into the module weight through the channel map; coord channels and
    padding entries untouched by the kernel."""
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(7)
    S, B, C, Cs, H, W = 3, 2, 13, 16, 11, 40
    cin = S * C + 2
    slab = torch.zeros((S, B, Cs, H, W))
    slab[:, :, :C] = F.relu(torch.randn((S, B, C, H, W), generator=g))
    x = torch.cat([slab[s] [:, :C] for s in range(S)] + [torch.zeros((B, 2, H, W))], 1)
    dy = torch.randn((B, 128, H, W), generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (128, cin, 3, 3), dy.double(), padding=1)
    chan_map = torch.tensor([s * C + c if c < C else -1 for s in range(S) for c in range(Cs)], dtype=torch.int32)
    d = ops.conv_desc(B, S * Cs, H, W, group=Cs, group_stride=B * Cs * H * W, batch_stride=Cs * H * W)
    dw = torch.full((128, cin, 3, 3), 9.0, device=DEV)
    for layout in ("f32", "split"):
        xs = slab.to(DEV) if layout == "f32" else torch.stack([_split_encode(slab[s].to(DEV)) for s in range(S)])
        ops.conv3x3_wgrad(xs, d, dy.to(DEV), 1, cin, chan_map=chan_map.to(DEV), dw=dw)
        assert_parity(dw[:, :S * C].cpu(), ref[:, :S * C], f"grouped wgrad {layout}")
        assert (dw[:, S * C:] == 9.0).all()


def test_split_rows_rounding():
    """mvbev_split_rows_bf16: hi = bf16(x) (round to nearest even), lo = bf16(x - hi), per
    (channel, row, 8-pixel run) hi[8] then lo[8]; W % 8 != 0 rejected."""
    from mvdet_amd import _native, ops
    g = torch.Generator().manual_seed(5)
    x = torch.randn((2, 3, 5, 24), generator=g) * torch.logspace(-8, 8, 24)
    r = ops.split_rows(x.to(DEV)).cpu()
    assert tuple(r.shape) == ops.split_rows_shape(2, 3, 5, 24)
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    assert torch.equal(r[..., 0, :].reshape(x.shape), hi)
    assert torch.equal(r[..., 1, :].reshape(x.shape), lo)
    with pytest.raises(ValueError):
        ops.split_rows(torch.zeros((1, 1, 2, 12), device=DEV))
    st = _native.load().mvbev_split_rows_bf16(x.to(DEV).data_ptr(), 2, 12, r.to(DEV).data_ptr(), None)
    assert st == _native.ERR_SHAPE


@pytest.mark.parametrize("B,K,H,W,dil,lists", [(1, 64, 12, 40, 1, False), (2, 72, 13, 48, 2, False),
                                               (2, 192, 37, 96, 1, True)])
def test_conv_wgrad_presplit_dy_rows(B, K, H, W, dil, lists):
    """The LDS-DMA wgrad reading dy pre-split into bf16 rows (ops.split_rows, the training
    step's form) gives bitwise the dw of the same kernel splitting an fp32 dy itself, and
    matches torch; where that kernel does not apply (fp32 x) the fp32 dy is used instead."""
    from mvdet_amd import _native, ops
    g = torch.Generator().manual_seed(K + W)
    cout = 128
    x = F.relu(torch.randn((B, K, H, W), generator=g))
    dy = torch.randn((B, cout, H, W), generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (cout, K, 3, 3), dy.double(), padding=dil, dilation=dil)
    d = ops.conv_desc(B, K, H, W, group=K if not lists else 64, group_stride=0 if not lists else B * 64 * H * W,
                      batch_stride=K * H * W if not lists else 64 * H * W)
    if lists:  # three 64-channel groups (camera slots) with chunk lists from a frustum-like mask
        xs = torch.stack([_split_encode(x[:, 64 * s_:64 * (s_ + 1)].contiguous().to(DEV)) for s_ in range(3)])
        th, tw = _native.TILE_H, _native.TILE_W
        mask = torch.full(((-(-H // th)) * (-(-W // tw)),), 7, dtype=torch.int32)
        cl = ops.wgrad_chunk_lists(mask.to(DEV), 3, B, H, W)
    else:
        xs, cl = _split_encode(x.to(DEV)), None
    dyd = dy.to(DEV)
    a = ops.conv3x3_wgrad(xs, d, dyd, dil, K, chunk_lists=cl)
    b = ops.conv3x3_wgrad(xs, d, dyd, dil, K, chunk_lists=cl, dy_rows=ops.split_rows(dyd))
    assert torch.equal(a, b)
    assert_parity(b.cpu(), ref, "wgrad from pre-split dy rows")
    if not lists:  # fp32 x: the register kernel, which reads the fp32 dy
        c = ops.conv3x3_wgrad(x.to(DEV), d, dyd, dil, K, dy_rows=ops.split_rows(dyd))
        assert_parity(c.cpu(), ref, "wgrad, fp32 x, dy_rows ignored")


@pytest.mark.parametrize("split", [False, True])
def test_conv_wgrad_frustum_chunk_lists(split):
    """conv1's wgrad with per-group chunk lists from a frustum mask: skipping the chunks whose
    window is exactly zero leaves the gradient unchanged."""
    from mvdet_amd import _native, ops
    g = torch.Generator().manual_seed(21)
    S, B, Cs, H, W = 3, 2, 64, 37, 100
    slab = F.relu(torch.randn((S, B, Cs, H, W), generator=g))
    rects = [(0, 12, 0, 40), (10, 37, 30, 100), (5, 9, 60, 75)]     # each camera's footprint
    for s_, (r0, r1, c0, c1) in enumerate(rects):
        keep = torch.zeros((H, W))
        keep[r0:r1, c0:c1] = 1
        slab[s_] *= keep
    th, tw = _native.TILE_H, _native.TILE_W
    ty, tx = -(-H // th), -(-W // tw)
    mask = torch.zeros(ty * tx, dtype=torch.int32)
    for t in range(ty * tx):
        y0, x0 = (t // tx) * th, (t % tx) * tw
        win = slab[:, :, :, max(0, y0 - 1):y0 + th + 1, max(0, x0 - 1):x0 + tw + 1]
        mask[t] = sum(1 << s_ for s_ in range(S) if (win[s_] != 0).any())
    assert (mask != 7).any()
    dy = torch.randn((B, 128, H, W), generator=g)
    cin = S * Cs
    x = torch.cat([slab[s_] for s_ in range(S)], 1)
    ref = torch.nn.grad.conv2d_weight(x.double(), (128, cin, 3, 3), dy.double(), padding=1)
    d = ops.conv_desc(B, S * Cs, H, W, group=Cs, group_stride=B * Cs * H * W, batch_stride=Cs * H * W)
    lists = ops.wgrad_chunk_lists(mask.to(DEV), S, B, H, W)
    assert lists[1][-1].item() < B * H * tx * S
    xs = torch.stack([_split_encode(slab[s_].to(DEV)) for s_ in range(S)]) if split else slab.to(DEV)
    got = ops.conv3x3_wgrad(xs, d, dy.to(DEV), 1, cin, chunk_lists=lists)
    assert_parity(got.cpu(), ref, "wgrad with chunk lists")


@pytest.mark.parametrize("pieces", [0, 1, 3])
def test_dgrad_ring_schedule(pieces):
    """conv3x3_dgrad on the ring kernel run through a host schedule (schedule.plan: XCD
    shares, the last round cut into K-pieces, fixup in K order) equals the plain launch:
    bitwise for whole blocks (pieces=1: no cut), to fp32 rounding with pieces (the planner's
    own cut, or every block in 3 pieces) — with the output-side mask, unwritten tiles stay
    untouched."""
    from mvdet_amd import ops, schedule
    g = torch.Generator().manual_seed(11 + pieces)
    B, Cw, K, H, W = 2, 256, 128, 29, 70
    dy = torch.randn((B, K, H, W), generator=g)
    w = torch.randn((K, Cw, 3, 3), generator=g) * 0.05
    pk = ops.PackedDgrad3x3(Cw)
    dys = _split_encode(dy.to(DEV))
    th = ops.dgrad_tile_rows(True, 1)
    ntiles = -(-H // th) * -(-W // 32)
    mask = torch.tensor([(t * 5 + 1) % 4 for t in range(ntiles)], dtype=torch.int32)  # groups of 128 channels
    ref = ops.conv3x3_dgrad(dys, pk, w.to(DEV), 1, out=torch.full(ops.split_shape(B, Cw, H, W), 7.0,
                                                                      dtype=torch.bfloat16, device=DEV),
                            out_mask=mask.to(DEV), cot_per_group=1)
    if pieces == 0:
        sch = ops.dgrad_schedule(B, Cw, H, W, K, mask.to(DEV), 1, DEV)
    else:
        blocks = schedule.ring_blocks(B, -(-H // th), -(-W // 32), Cw // 128, K // 16,
                                      out_mask=mask.tolist(), cot_per_group=1)
        sch = schedule.plan(blocks, 256, DEV, split=False, force_pieces=pieces)
        assert (sch.nfix > 0) == (pieces > 1)
    got = ops.conv3x3_dgrad(dys, pk, w.to(DEV), 1, out=torch.full(ops.split_shape(B, Cw, H, W), 7.0,
                                                                      dtype=torch.bfloat16, device=DEV),
                            out_mask=mask.to(DEV), cot_per_group=1, sched=sch)
    # the pixel-major split output of the same schedule: the same pieces
    gotp = ops.conv3x3_dgrad(dys, pk, w.to(DEV), 1, out=torch.full(ops.split_pix_shape(B, Cw, H, W), 7.0,
                                                                       dtype=torch.bfloat16, device=DEV),
                             out_mask=mask.to(DEV), cot_per_group=1, sched=sch)
    assert torch.equal(gotp.permute(0, 3, 1, 2, 4, 5), got)
    r, o = ops.split_decode(ref).cpu(), ops.split_decode(got).cpu()
    assert torch.equal(o == 14.0, r == 14.0) and (r == 14.0).any()  # prefill hi 7 + lo 7 kept where masked
    if sch.nfix:  # pieces: another fp32 summation order
        assert_parity(o, r, f"dgrad, {sch.nfix} blocks in K-pieces")
    else:
        assert torch.equal(o, r)


@pytest.mark.parametrize("B,Cw,K,H,W,dil", [(1, 128, 40, 12, 36, 1), (2, 512, 512, 17, 37, 2),
                                            (1, 256, 200, 9, 64, 1)])
def test_conv_dgrad_vs_torch(B, Cw, K, H, W, dil):
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(Cw + K + dil)
    w = torch.randn((Cw, K, 3, 3), generator=g) * 0.05
    dy = torch.randn((B, Cw, H, W), generator=g)
    ref = torch.nn.grad.conv2d_input((B, K, H, W), w.double(), dy.double(), padding=dil, dilation=dil)
    pk = ops.PackedDgrad3x3(K)
    got = ops.conv3x3_dgrad(dy.to(DEV), pk, w.to(DEV), dil)
    assert got.shape[1] == pk.cout_p
    assert_parity(got[:, :K].cpu(), ref, "dgrad")
    assert (got[:, K:] == 0).all()


@pytest.mark.parametrize("B,Cw,K,H,W,dil", [(1, 128, 40, 25, 36, 1), (2, 512, 512, 17, 37, 2),
                                            (1, 256, 200, 9, 64, 1)])
def test_conv_dgrad_split_dy_ring_kernel(B, Cw, K, H, W, dil):
    """dy in the split-bf16 layout runs the data gradient on the LDS-DMA ring kernel (12-row
    tiles, partial last tiles here): same result as from fp32 dy, vs float64 torch."""
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(Cw + K + dil + 1)
    w = torch.randn((Cw, K, 3, 3), generator=g) * 0.05
    dy = torch.randn((B, Cw, H, W), generator=g)
    ref = torch.nn.grad.conv2d_input((B, K, H, W), w.double(), dy.double(), padding=dil, dilation=dil)
    pk = ops.PackedDgrad3x3(K)
    dys = _split_encode(dy).to(DEV)
    torch.testing.assert_close(ops.split_decode(dys, Cw).cpu(), dy, rtol=2e-5, atol=0)  # hi + lo: 16 mantissa bits
    got = ops.conv3x3_dgrad(dys, pk, w.to(DEV), dil)
    assert_parity(got[:, :K].cpu(), ref, "dgrad (split dy)")
    assert (got[:, K:] == 0).all()
    f32 = ops.conv3x3_dgrad(dy.to(DEV), pk, w.to(DEV), dil)
    assert_parity(got.cpu(), f32.cpu(), "split vs fp32 dy", normwise_tol=2e-5)


@pytest.mark.parametrize("B,C,H,W", [(1, 128, 25, 36), (2, 512, 17, 70)])
def test_conv2_dgrad_as_winograd_conv(B, C, H, W):
    """The training backward's conv2 data gradient (``autograd._dgrad2_wino``: the forward's
    dilation-2 row-Winograd conv with the weight transposed and flipped) vs float64 torch, twice
    with the weight changed in place (re-packed per parameter version)."""
    from types import SimpleNamespace
    from mvdet_amd import autograd, ops
    g = torch.Generator().manual_seed(C + H)
    eng = SimpleNamespace(grid_hw=(H, W), mid=C)
    st = SimpleNamespace()
    w = torch.empty((C, C, 3, 3), device=DEV)  # one parameter updated in place: re-packed per version
    for it in range(2):
        w.copy_(torch.randn((C, C, 3, 3), generator=g) * 0.05)
        dy = torch.randn((B, C, H, W), generator=g)
        ref = torch.nn.grad.conv2d_input((B, C, H, W), w.cpu().double(), dy.double(), padding=2, dilation=2)
        got = autograd._dgrad2_wino(eng, st, _split_encode(dy).to(DEV), w)
        assert_parity(got.cpu(), ref, f"conv2 dgrad (Winograd), weight {it}")


@pytest.mark.parametrize("B,Cw,K,H,W", [(1, 128, 256, 25, 70), (2, 256, 384, 14, 40), (1, 512, 256, 13, 40)])
def test_conv1_dgrad_as_masked_winograd_conv(B, Cw, K, H, W):
    """``ops.conv3x3_wino_dgrad`` (the training backward's conv1 data gradient: row-Winograd conv
    of the split dy with the weight swapped and flipped) vs float64 torch on the tiles its output
    mask keeps (one 128-channel group per bit, random bits per 12 x 32 tile); cleared tiles keep
    what ``out`` held."""
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(Cw + K + H)
    w = torch.randn((Cw, K, 3, 3), generator=g) * 0.05
    dy = torch.randn((B, Cw, H, W), generator=g)
    ref = torch.nn.grad.conv2d_input((B, K, H, W), w.double(), dy.double(), padding=1, dilation=1)
    d = ops.conv_desc(B, Cw, H, W, group=Cw, group_stride=0, batch_stride=Cw * H * W)
    t = torch.zeros((ops.wino_rows_bytes(d) + 1) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino_rows(_split_encode(dy).to(DEV), d, t)
    wt = w.flip(2, 3).transpose(0, 1).contiguous().to(DEV)
    packed = ops.PackedConv3x3(None, "bf16x3", wino=True).get(wt)
    # the dgrad packer reads the forward weight itself (swapped, reversed taps): the same bytes
    assert torch.equal(ops.PackedWinoDgrad3x3(K).get(w.to(DEV)), packed)
    wpad = torch.cat([w, torch.randn((Cw, 2, 3, 3), generator=g)], 1).to(DEV)  # extra (coord) inputs past K
    assert torch.equal(ops.PackedWinoDgrad3x3(K).get(wpad), packed)
    ty, tx = -(-H // 12), -(-W // 32)
    ngroups = K // 128
    mask = torch.randint(0, 1 << ngroups, (ty * tx,), generator=g, dtype=torch.int32)
    mask[0] = (1 << ngroups) - 1
    out = torch.full(ops.split_shape(B, K, H, W), 7.0, dtype=torch.bfloat16, device=DEV)
    ops.conv3x3_wino_dgrad(t, d, packed, K, out, out_mask=mask.to(DEV), cot_per_group=1)
    got = ops.split_decode(out, K).cpu().double()
    keep = torch.zeros((K, H, W), dtype=torch.bool)
    for i in range(ty):
        for j in range(tx):
            for gi in range(ngroups):
                if (int(mask[i * tx + j]) >> gi) & 1:
                    keep[gi * 128:(gi + 1) * 128, 12 * i:12 * i + 12, 32 * j:32 * j + 32] = True
    keep = keep.expand(B, K, H, W)
    assert keep.any() and (~keep).any()
    assert_parity(got[keep].reshape(-1, 1), ref[keep].reshape(-1, 1), "masked Winograd dgrad (kept tiles)")
    assert (got[~keep] == 14.0).all()  # hi 7 + lo 7: untouched
    # the pixel-major split output (MVBEV_LAYOUT_SPLIT_BF16_PIX, the warp adjoint's input): the same pieces
    outp = torch.full(ops.split_pix_shape(B, K, H, W), 7.0, dtype=torch.bfloat16, device=DEV)
    ops.conv3x3_wino_dgrad(t, d, packed, K, outp, out_mask=mask.to(DEV), cot_per_group=1)
    assert torch.equal(outp.permute(0, 3, 1, 2, 4, 5), out)
    # dense (no mask) equals the masked result on the kept tiles bit for bit
    dense = torch.empty((B, K, H, W), dtype=torch.float32, device=DEV)
    ops.conv3x3_wino_dgrad(t, d, packed, K, dense)
    assert_parity(dense.cpu().double(), ref, "Winograd dgrad (dense, fp32 out)")


def test_relu_backward_split():
    """dy *= [y > 0] with y = hi + lo in the split layout, and the split copy of the result."""
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(11)
    B, C, H, W = 2, 24, 7, 13
    y = F.relu(torch.randn((B, C, H, W), generator=g))
    y[0, 3, 2, 4] = 1e-30  # a tiny positive activation still passes its gradient
    dy = torch.randn((B, C, H, W), generator=g)
    ys = _split_encode(y).to(DEV)
    out = torch.empty(ops.split_shape(B, C, H, W), dtype=torch.bfloat16, device=DEV)
    got = ops.relu_backward_split_(dy.clone().to(DEV), ys, out).cpu()
    want = torch.where(ops.split_decode(ys, C).cpu() > 0, dy, torch.zeros_like(dy))
    assert torch.equal(got, want)
    assert torch.equal(out.cpu(), _split_encode(want))  # the kernel splits with the same roundings


def test_conv_dgrad_channel_map():
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(3)
    w = torch.randn((128, 30, 3, 3), generator=g) * 0.1
    dy = torch.randn((1, 128, 10, 20), generator=g)
    ref = torch.nn.grad.conv2d_input((1, 30, 10, 20), w.double(), dy.double(), padding=1)
    cmap = [29, 3, -1, 7, 0]
    got = ops.conv3x3_dgrad(dy.to(DEV), ops.PackedDgrad3x3(5, cmap), w.to(DEV), 1).cpu()
    for o, c in enumerate(cmap):
        if c < 0:
            assert (got[:, o] == 0).all()
        else:
            assert_parity(got[:, o], ref[:, c], f"dgrad channel {o}")


@pytest.mark.parametrize("split,split_dy", [(False, False), (True, False), (True, True)])
def test_conv_dgrad_output_mask(split, split_dy):
    """Output-side mask: tiles of a clear (tile, channel group) bit are skipped (left as they
    were), every other tile equals the unmasked dgrad (split_dy: the ring kernel, 12-row tiles)."""
    from mvdet_amd import _native, ops
    g = torch.Generator().manual_seed(5)
    B, Cw, K, H, W = 2, 256, 512, 20, 70          # 4 output groups of 128 channels
    w = torch.randn((Cw, K, 3, 3), generator=g) * 0.05
    dy = torch.randn((B, Cw, H, W), generator=g)
    dy = (_split_encode(dy) if split_dy else dy).to(DEV)
    pk = ops.PackedDgrad3x3(K)
    ref = ops.conv3x3_dgrad(dy, pk, w.to(DEV), 1)
    TH = ops.dgrad_tile_rows(split_dy, 1)
    assert TH == (12 if split_dy else _native.TILE_H)
    ty, tx = -(-H // TH), -(-W // _native.TILE_W)
    mask = torch.randint(0, 16, (ty * tx,), generator=g, dtype=torch.int32)
    if split:
        out = torch.zeros(ops.split_shape(B, K, H, W), dtype=torch.bfloat16, device=DEV)
        ops.conv3x3_dgrad(dy, pk, w.to(DEV), 1, out=out, out_mask=mask.to(DEV), cot_per_group=1)
        got = ops.split_decode(out, K).cpu()
    else:
        got = torch.full((B, K, H, W), 7.0, device=DEV)
        ops.conv3x3_dgrad(dy, pk, w.to(DEV), 1, out=got, out_mask=mask.to(DEV), cot_per_group=1)
        got = got.cpu()
    ref = ref.cpu()
    for t in range(ty * tx):
        r0, c0 = (t // tx) * TH, (t % tx) * _native.TILE_W
        for gi in range(4):
            blk = got[:, gi * 128:(gi + 1) * 128, r0:r0 + TH, c0:c0 + _native.TILE_W]
            want = ref[:, gi * 128:(gi + 1) * 128, r0:r0 + TH, c0:c0 + _native.TILE_W]
            if (int(mask[t]) >> gi) & 1:
                assert_parity(blk, want, f"dgrad tile {t} group {gi}", normwise_tol=2e-5 if split else 1e-6)
            else:
                assert (blk == (0.0 if split else 7.0)).all()


def test_bias_coord_relu_and_cout1_backward():
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(11)
    B, Co, H, W = 2, 128, 13, 29
    dy = torch.randn((B, Co, H, W), generator=g)
    # bias + coord-channel weight gradient (coord map = create_coord_map, channels 5, 6 of 7)
    cmap = cpu_path.coord_map(H, W).repeat(B, 1, 1, 1)
    x = torch.cat([torch.zeros((B, 5, H, W)), cmap], 1)
    ref_w = torch.nn.grad.conv2d_weight(x.double(), (Co, 7, 3, 3), dy.double(), padding=2, dilation=2)
    db = torch.empty(Co, device=DEV)
    dw = torch.full((Co, 7, 3, 3), 4.0, device=DEV)
    ops.conv3x3_bias_coord_grad(dy.to(DEV), 2, db=db, dw=dw, coord_ch=5)
    assert_parity(db.cpu(), dy.double().sum((0, 2, 3)), "bias grad")
    assert_parity(dw[:, 5:].cpu(), ref_w[:, 5:], "coord weight grad")
    assert (dw[:, :5] == 4.0).all()
    # ReLU backward (threshold_backward semantics: grad where the output > 0)
    y = F.relu(torch.randn((B, Co, H, W), generator=g))
    got = ops.relu_backward_(dy.clone().to(DEV), y.to(DEV)).cpu()
    assert torch.equal(got, torch.where(y > 0, dy, torch.zeros_like(dy)))
    # conv3 (Cout 1, dilation 4) backward with the previous ReLU's mask fused
    x2 = F.relu(torch.randn((B, 64, H, W), generator=g))
    w3 = torch.randn((1, 64, 3, 3), generator=g) * 0.1
    dmap = torch.randn((B, 1, H, W), generator=g)
    x2r = x2.double().requires_grad_()
    w3r = w3.double().requires_grad_()
    F.conv2d(F.relu(x2r), w3r, padding=4, dilation=4).backward(dmap.double())
    dx, dw3 = ops.conv3x3_cout1_backward(x2.to(DEV), w3.to(DEV), dmap.to(DEV), 4, relu_mask=True)
    assert_parity(dx.cpu(), x2r.grad, "cout1 dgrad (relu-masked)")
    assert_parity(dw3.cpu(), w3r.grad, "cout1 wgrad")


# ---------------------------------------------------------------------------------- end to end

def _head(num_cam, C, seed):
    p = fixtures.head_params(num_cam, seed, C)
    return {k: torch.from_numpy(v) for k, v in p.items() if k.startswith("map_classifier.")}


def _cpu_reference(feats, Ms, grid, params, gmap, masks=None):
    """Torch-CPU fp32 autograd through the reference path (kornia restatement + cat +
    map_classifier, ``oracle/cpu_path.py``).  ``masks`` = (m1, m2): the ReLUs of
    ``map_classifier[1]``/``[3]`` as multiplications by these 0/1 patterns (same gradient as
    ReLU where the pattern is the pre-activation's sign).  Returns (map, pre1, pre2, grads)."""
    fr = [f.clone().requires_grad_() for f in feats]
    pr = {k: v.clone().requires_grad_() for k, v in params.items()}
    B = feats[0].shape[0]
    warped = cpu_path.warp_views(fr, Ms, grid)
    x = torch.cat(warped + [cpu_path.coord_map(*grid).repeat([B, 1, 1, 1])], 1)
    pre1 = F.conv2d(x, pr["map_classifier.0.weight"], pr["map_classifier.0.bias"], padding=1)
    y1 = F.relu(pre1) if masks is None else pre1 * masks[0]
    pre2 = F.conv2d(y1, pr["map_classifier.2.weight"], pr["map_classifier.2.bias"], padding=2, dilation=2)
    y2 = F.relu(pre2) if masks is None else pre2 * masks[1]
    out = F.conv2d(y2, pr["map_classifier.4.weight"], None, padding=4, dilation=4)
    out.backward(gmap)
    return out.detach(), pre1.detach(), pre2.detach(), [f.grad for f in fr], {k: v.grad for k, v in pr.items()}


@pytest.mark.parametrize("precision", ["bf16x3", "fp32"])
@pytest.mark.parametrize("N,B,C,src,grid", [(2, 1, 8, (27, 48), (12, 36)), (3, 2, 13, (30, 41), (17, 45)),
                                             (2, 1, 128, (20, 30), (24, 96))])
def test_project_fuse_backward_vs_cpu_autograd(precision, N, B, C, src, grid):
    """ProjectFuseFunction (HIP forward + HIP backward) vs torch-CPU autograd through the
    reference path (kornia restatement + cat + map_classifier) on identical inputs."""
    from mvdet_amd.autograd import project_fuse
    from mvdet_amd.pipeline import ProjectFuse
    rng = np.random.default_rng(N * 31 + C)
    H, W = src
    ho, wo = grid
    Ms = [_rand_h(rng, H, W, ho, wo) for _ in range(N)]
    if C % 128 == 0:  # each view covers part of the grid: the frustum masks skip tiles
        Ms = [np.diag([0.45, 0.45, 1.0]) @ M + np.array([[0, 0, 40.0 * v], [0, 0, 0], [0, 0, 0]])
              for v, M in enumerate(Ms)]
    feats = [torch.from_numpy(np.maximum(rng.standard_normal((B, C, H, W)), 0).astype(np.float32))
             for _ in range(N)]
    params = _head(N, C, seed=N + C)
    gmap = torch.from_numpy(rng.standard_normal((B, 1, ho, wo)).astype(np.float32))
    # native
    eng = ProjectFuse([torch.from_numpy(M) for M in Ms], src, grid, C, precision=precision)
    mc = torch.nn.Sequential(torch.nn.Conv2d(N * C + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)
    mc.load_state_dict({k.split(".", 1)[1]: v for k, v in params.items()})
    fg = [f.to(DEV).requires_grad_() for f in feats]
    if C % 128 == 0 and precision == "bf16x3":
        assert eng.conv1_active_fraction(DEV, 0, ho) < 0.9
    out = project_fuse(eng, fg, mc)
    ws = out.grad_fn.ws                      # the activations the backward will use
    m1, m2 = (eng.y1_fp32(ws) > 0).float().cpu(), (ws.y2 > 0).float().cpu()
    out.backward(gmap.to(DEV))
    # reference, plain ReLU: forward parity, and the activation pattern differs only where the
    # pre-activation is within fp32 rounding of zero (a ReLU's gradient is discontinuous there)
    out_ref, pre1, pre2, _, _ = _cpu_reference(feats, Ms, grid, params, gmap)
    assert_parity(out.detach().cpu(), out_ref, "forward")
    for m, pre in ((m1, pre1), (m2, pre2)):
        flip = m != (pre > 0).float()
        assert flip.sum().item() <= max(2, pre.numel() // 20000)
        assert (pre[flip].abs() <= 1e-4 * pre.abs().max()).all(), pre[flip]
    # reference gradients given the same activation pattern
    _, _, _, gfeat, gpar = _cpu_reference(feats, Ms, grid, params, gmap, masks=(m1, m2))
    for i in range(N):
        assert_parity(fg[i].grad.cpu(), gfeat[i], f"d feat view {i}")
    for k, p in mc.named_parameters():
        assert_parity(p.grad.cpu(), gpar["map_classifier." + k], f"d {k}")


def test_detector_training_step_matches_cpu_autograd():
    """The drop-in module in training mode (grad enabled: ``trainer.py:38-47``) on the
    reference-fixture rig: forward equals the reference's golden map, and every gradient a
    ``loss.backward()`` produces (map/image heads, the input features through the upsample)
    matches torch-CPU autograd through the reference path."""
    import torch.nn as nn
    from helpers import load_golden
    from mvdet_amd import PerspTransDetector
    from test_gpu_parity import _ds_from_golden
    g = load_golden("module_wt2")
    m = g["meta"]
    model = PerspTransDetector(_ds_from_golden(g))
    params = {k: torch.from_numpy(v) for k, v in fixtures.head_params(m["num_cam"], m["weight_seed"]).items()}
    sd = model.state_dict()
    sd.update(params)
    model.load_state_dict(sd)
    model.base_pt1, model.base_pt2 = nn.Identity(), nn.Identity()
    model.train()
    feat_in = torch.from_numpy(g["feat_in"])                 # [B, N, 512, h, w]
    x = feat_in.to(DEV).requires_grad_()
    map_res, imgs_res = model(x)
    assert map_res.grad_fn is not None and type(map_res.grad_fn).__name__.startswith("ProjectFuseFunction")
    assert_parity(map_res.detach().cpu(), g["map_result"], "training-mode forward vs golden")
    rng = np.random.default_rng(0)
    gmap = torch.from_numpy(rng.standard_normal(map_res.shape).astype(np.float32))
    gimg = [torch.from_numpy(rng.standard_normal(r.shape).astype(np.float32)) for r in imgs_res]
    ws = map_res.grad_fn.ws
    masks = ((model.engine.y1_fp32(ws) > 0).float().cpu(), (ws.y2 > 0).float().cpu())
    loss = (map_res * gmap.to(DEV)).sum() + sum((r * gg.to(DEV)).sum() for r, gg in zip(imgs_res, gimg))
    loss.backward()
    # CPU reference: persp_trans_detector.py:61-87 with the backbone bypassed
    xr = feat_in.clone().requires_grad_()
    pr = {k: v.clone().requires_grad_() for k, v in params.items()}
    B, N = xr.shape[:2]
    ups, imgs_ref = [], []
    for cam in range(N):
        up = cpu_path.upsample(xr[:, cam], model.upsample_shape)
        h = F.relu(F.conv2d(up, pr["img_classifier.0.weight"], pr["img_classifier.0.bias"]))
        imgs_ref.append(F.conv2d(h, pr["img_classifier.2.weight"]))
        ups.append(up)
    grid = tuple(model.reducedgrid_shape)
    warped = cpu_path.warp_views(ups, list(g["proj_mats"]), grid)
    xc = torch.cat(warped + [cpu_path.coord_map(*grid).repeat([B, 1, 1, 1])], 1)
    pre1 = F.conv2d(xc, pr["map_classifier.0.weight"], pr["map_classifier.0.bias"], padding=1)
    pre2 = F.conv2d(pre1 * masks[0], pr["map_classifier.2.weight"], pr["map_classifier.2.bias"], padding=2,
                    dilation=2)
    out = F.conv2d(pre2 * masks[1], pr["map_classifier.4.weight"], None, padding=4, dilation=4)
    for msk, pre in zip(masks, (pre1, pre2)):
        flip = msk != (pre > 0).float()
        assert flip.sum().item() <= 2 and (pre[flip].abs() <= 1e-4 * pre.abs().max()).all()
    ((out * gmap).sum() + sum((r * gg).sum() for r, gg in zip(imgs_ref, gimg))).backward()
    assert_parity(x.grad.cpu(), xr.grad, "d input features")
    for k, p in model.named_parameters():
        if k in pr:
            assert_parity(p.grad.cpu(), pr[k].grad, f"d {k}")


def test_project_fuse_second_backward_raises():
    """The native backward frees its saved activations: a second backward through the same
    graph (retain_graph=True) raises a clear RuntimeError, and double backward is refused
    (once_differentiable) instead of silently building no second-order graph."""
    from mvdet_amd.autograd import project_fuse
    from mvdet_amd.pipeline import ProjectFuse
    rng = np.random.default_rng(11)
    N, B, C, (H, W), (ho, wo) = 2, 1, 8, (27, 48), (12, 36)
    Ms = [_rand_h(rng, H, W, ho, wo) for _ in range(N)]
    eng = ProjectFuse([torch.from_numpy(M) for M in Ms], (H, W), (ho, wo), C)
    mc = torch.nn.Sequential(torch.nn.Conv2d(N * C + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)
    fg = [torch.rand((B, C, H, W), device=DEV).requires_grad_() for _ in range(N)]
    out = project_fuse(eng, fg, mc)
    out.sum().backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="a second time"):
        out.sum().backward()
    out2 = project_fuse(eng, fg, mc)
    (g,) = torch.autograd.grad(out2.sum(), fg[0], create_graph=True)
    with pytest.raises(RuntimeError):
        g.sum().backward()


def test_training_steps_reuse_the_zeroed_slab():
    """Training forwards draw the split slab from the engine's pool (zero-filled once; the warp
    skips the out-of-source pixels, which stay exactly zero): two identical steps give
    identical outputs and gradients, and the second step reuses the first step's slab."""
    from mvdet_amd import ProjectFuse, autograd, synthetic
    from mvdet_amd.geometry import projection_matrices
    ds = synthetic.wildtrack_like(2, 4, seed=5, img_shape=(108, 192), worldgrid_shape=(96, 288))
    C = 32
    up = ds.upsample_shape
    feats = [synthetic.synthetic_features(1, C, [u // 3 for u in up], up, seed=40 + v, device=DEV) for v in range(2)]
    eng = ProjectFuse(projection_matrices(ds), tuple(up), tuple(ds.reducedgrid_shape), C)
    torch.manual_seed(0)
    mc = torch.nn.Sequential(torch.nn.Conv2d(C * 2 + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)
    results, slabs = [], []
    for _ in range(2):
        fg = [f.clone().requires_grad_() for f in feats]
        mc.zero_grad()
        out = autograd.project_fuse(eng, fg, mc)
        ws = out.grad_fn.ws
        # (the Winograd conv1's transform buffer travels with the slab: zero-filled once)
        slabs.append((ws.slab.data_ptr(), None if ws.wino_t is None else ws.wino_t.data_ptr()))
        assert (ws.wino_t is not None) == eng.wino_active(DEV)
        assert out.grad_fn.ws.slab_zeroed
        out.backward(torch.ones_like(out))
        results.append([out.detach().clone()] + [f.grad.clone() for f in fg] +
                       [p.grad.clone() for p in mc.parameters()])
    assert slabs[0] == slabs[1]
    for a, b in zip(*results):
        assert torch.equal(a, b)


@pytest.mark.parametrize("cfg", [2, 1])
def test_full_size_training_step_vs_cpu_autograd(cfg):
    """The training step at full size (config 2: Wildtrack 7 x 512 x 270 x 480 -> 120 x 360; config 1:
    MultiviewX 6 x 128 -> 160 x 250), ``trainer.py:38-47`` on ``persp_trans_detector.py:65-87`` past the
    upsample: the default engine (row-Winograd conv1 / conv2 forward and data gradients, conv1's with
    the output-side frustum mask; at config 2 the fused warp writes T and both weight gradients run from
    the forward transforms, at config 1 — W = 250, not a multiple of 8 — the slab path and the direct
    conv1 weight gradient) vs torch-CPU fp32 autograd through the reference path on identical inputs —
    the map and every gradient (view features, 5 head parameters) within the 1e-3 gate, given the
    GPU's ReLU patterns (the few pre-activations within rounding of zero are checked as in the small
    cases)."""
    from mvdet_amd import ProjectFuse, autograd, synthetic
    from mvdet_amd.geometry import projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    B, C, N = spec["B"], spec["C"], ds.num_cam
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm = projection_matrices(ds)
    params = _head(N, C, seed=2)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=2000 + v, device=DEV) for v in range(N)]
    eng = ProjectFuse(pm, up, grid, C)
    assert eng.wino_active(DEV) and autograd._dgrad1_wino_applies(eng, N * C, DEV)
    mc = torch.nn.Sequential(torch.nn.Conv2d(N * C + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)
    mc.load_state_dict({k.split(".", 1)[1]: v for k, v in params.items()})
    fg = [f.clone().requires_grad_() for f in feats]
    out = autograd.project_fuse(eng, fg, mc)
    ws = out.grad_fn.ws
    assert ws.t_from_warp == ws.train_t_only == (cfg == 2) and ws.t1_valid
    m1, m2 = (eng.y1_fp32(ws) > 0).float().cpu(), (ws.y2 > 0).float().cpu()
    gmap = torch.from_numpy(np.random.default_rng(2).standard_normal(tuple(out.shape)).astype(np.float32))
    out.backward(gmap.to(DEV))
    torch.cuda.synchronize()
    out_ref, pre1, pre2, gfeat, gpar = _cpu_reference([f.cpu() for f in feats], [M.numpy() for M in pm], grid,
                                                      params, gmap, masks=(m1, m2))
    assert_parity(out.detach().cpu(), out_ref, f"cfg{cfg} training forward")
    for m, pre, what in ((m1, pre1, "conv1"), (m2, pre2, "conv2")):
        flip = m != (pre > 0).float()
        assert flip.sum().item() <= max(2, pre.numel() // 20000), what
        assert (pre[flip].abs() <= 1e-4 * pre.abs().max()).all(), what
    for v in range(N):
        assert_parity_t(fg[v].grad, gfeat[v], f"cfg{cfg} d feat view {v}")
    for k, p in mc.named_parameters():
        assert_parity_t(p.grad, gpar["map_classifier." + k], f"cfg{cfg} d {k}")


def test_detector_full_size_training_step_vs_cpu_autograd():
    """VERDICT r04 missing 4: the drop-in module's OWN training path at config 2's full size — train mode,
    backbone-resolution maps [1, 7, 512, 90, 160] (the backbone bypassed), ``project_fuse_backbone``: the
    fused 3x upsample + warp forward and its adjoint, the Winograd convs and data gradients — vs torch-CPU
    fp32 autograd through ``persp_trans_detector.py:61-87`` (F.interpolate, the image head, the kornia
    warp, cat, map_classifier): the map, imgs_result, the gradient of every view's input features and of
    every head parameter (map_classifier's 5, img_classifier's 3), within the 1e-3 gate given the GPU's
    ReLU patterns (pre-activations within rounding of zero checked as in the small cases).  Non-finite
    features are outside training parity."""
    import torch.nn as nn
    from mvdet_amd import PerspTransDetector, synthetic
    spec = synthetic.CONFIGS[2]
    ds = spec["make"]()
    B, C, N = spec["B"], spec["C"], ds.num_cam
    model = PerspTransDetector(ds)
    params = {k: torch.from_numpy(v) for k, v in fixtures.head_params(N, 2, C=C).items()}
    sd = model.state_dict()
    sd.update(params)
    model.load_state_dict(sd)
    model.base_pt1, model.base_pt2 = nn.Identity(), nn.Identity()
    model.train()
    hb = [u // 3 for u in model.upsample_shape]
    low = torch.stack([synthetic.backbone_features(B, C, hb, seed=2600 + v, device=DEV) for v in range(N)], 1)
    x = low.clone().requires_grad_()
    # the image head's first conv outputs as the model computed them (its ReLU pattern is replayed below)
    g_head = []
    hook = model.img_classifier[0].register_forward_hook(lambda m, i, o: g_head.append(o.detach()))
    map_res, imgs_res = model(x)
    hook.remove()
    assert type(map_res.grad_fn).__name__.startswith("ProjectFuseFunction")
    eng = model.engine
    assert eng.wino_active(DEV)
    rng = np.random.default_rng(26)
    gmap = torch.from_numpy(rng.standard_normal(map_res.shape).astype(np.float32))
    gimg = [torch.from_numpy(rng.standard_normal(r.shape).astype(np.float32)) for r in imgs_res]
    ws = map_res.grad_fn.ws
    masks = ((eng.y1_fp32(ws) > 0).float().cpu(), (ws.y2 > 0).float().cpu())
    # the image head's ReLU pattern on the GPU (its 1x1 conv runs before the upsample there: the same
    # pre-activation up to rounding, so a few near-zero ones may flip, as the map head's)
    # (from the model's own head-conv outputs: MIOpen's solver choice and the maps' layout change the rounding)
    assert len(g_head) == N
    with torch.no_grad():
        mimg = [(F.interpolate(g_head[v], model.upsample_shape, mode="bilinear") > 0).float().cpu() for v in range(N)]
    loss = (map_res * gmap.to(DEV)).sum() + sum((r * gg.to(DEV)).sum() for r, gg in zip(imgs_res, gimg))
    loss.backward()
    torch.cuda.synchronize()
    # CPU reference: persp_trans_detector.py:61-87 with the backbone bypassed (ReLUs as the GPU's patterns)
    xr = low.cpu().requires_grad_()
    pr = {k: v.clone().requires_grad_() for k, v in params.items()}
    ups, imgs_ref = [], []
    for cam in range(N):
        up = cpu_path.upsample(xr[:, cam], model.upsample_shape)
        pre = F.conv2d(up, pr["img_classifier.0.weight"], pr["img_classifier.0.bias"])
        flip = mimg[cam] != (pre > 0).float()
        assert flip.sum().item() <= max(2, pre.numel() // 20000), f"img head {cam}"
        assert (pre[flip].abs() <= 1e-4 * pre.detach().abs().max()).all(), f"img head {cam}"
        imgs_ref.append(F.conv2d(pre * mimg[cam], pr["img_classifier.2.weight"]))
        ups.append(up)
    grid = tuple(model.reducedgrid_shape)
    warped = cpu_path.warp_views(ups, [M.numpy() for M in model.proj_mats], grid)
    xc = torch.cat(warped + [cpu_path.coord_map(*grid).repeat([B, 1, 1, 1])], 1)
    del warped
    pre1 = F.conv2d(xc, pr["map_classifier.0.weight"], pr["map_classifier.0.bias"], padding=1)
    pre2 = F.conv2d(pre1 * masks[0], pr["map_classifier.2.weight"], pr["map_classifier.2.bias"], padding=2,
                    dilation=2)
    out = F.conv2d(pre2 * masks[1], pr["map_classifier.4.weight"], None, padding=4, dilation=4)
    for msk, pre, what in zip(masks, (pre1, pre2), ("conv1", "conv2")):
        flip = msk != (pre > 0).float()
        assert flip.sum().item() <= max(2, pre.numel() // 20000), what
        assert (pre[flip].abs() <= 1e-4 * pre.detach().abs().max()).all(), what
    assert_parity(map_res.detach().cpu(), out.detach(), "cfg2 detector training forward map_result")
    for v in range(N):
        assert_parity(imgs_res[v].detach().cpu(), imgs_ref[v].detach(), f"cfg2 detector imgs_result {v}")
    ((out * gmap).sum() + sum((r * gg).sum() for r, gg in zip(imgs_ref, gimg))).backward()
    for v in range(N):
        assert_parity_t(x.grad[:, v], xr.grad[:, v], f"cfg2 detector d input features view {v}")
    for k, p in model.named_parameters():
        if k in pr:
            assert_parity_t(p.grad, pr[k].grad, f"cfg2 detector d {k}")
