"""conv1's weight gradient from the forward's row-Winograd transform (ABI 12000):
``ops.wino_dy_rows`` (D_xi = sum_j AT[j][xi] dy[3 r3 + j], split rows) and
``ops.conv3x3_wgrad_wino`` (M_xi[kw] = D_xi x T_xi shifted by kw, folded with G) against the
float64 ``torch.nn.grad.conv2d_weight`` of the same input — the closed-form adjoint of
``F.conv2d`` that the reference's autograd runs (``trainer.py:38-49`` through
``persp_trans_detector.py:51``) — under ``helpers.assert_parity`` (the north_star's 1e-3), and
against the direct LDS-DMA wgrad of the same operands.
"""
import pytest
import torch
import torch.nn.functional as F

from helpers import assert_parity, parity_stats

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _split_encode(x: torch.Tensor) -> torch.Tensor:
    B, C, H, W = x.shape
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    t = torch.stack([hi, lo], 0).reshape(2, B, C // 8, 8, H, W)
    return t.permute(1, 2, 4, 5, 0, 3).contiguous()


@pytest.mark.parametrize("dil", [1, 2])
def test_wino_dy_rows_transform_and_rounding(dil):
    """D over the forward's 3-row tiles: rows 3 r3 + j (dilation 1) or conv2's interleaved tiles
    12 (r3 // 4) + (0, 1, 6, 7)[r3 % 4] + 2 j (dilation 2); rows past H are zero."""
    from mvdet_amd import _native, ops
    g = torch.Generator().manual_seed(3)
    B, C, H, W = 2, 5, 13, 24  # H % 3 == 1 and H % 12 == 1: partial last tiles
    dy = torch.randn((B, C, H, W), generator=g)
    got = ops.wino_dy_rows(dy.to(DEV), dilation=dil).cpu()
    R3 = ops.wino_r3(H, dil)
    assert tuple(got.shape) == (B, 5, C, R3, W // 8, 2, 8)
    pad = torch.zeros((B, C, 12 * R3, W))
    pad[:, :, :H] = dy
    base = [3 * r if dil == 1 else 12 * (r // 4) + (0, 1, 6, 7)[r % 4] for r in range(R3)]
    r = torch.stack([pad[:, :, [b + dil * j for b in base]] for j in range(3)], 3)  # [B, C, R3, 3, W]
    a0, a1, a2 = r[:, :, :, 0], r[:, :, :, 1], r[:, :, :, 2]
    d = torch.stack([a0, (a0 + a1) + a2, (a0 - a1) + a2, (a0 + 2 * a1) + 4 * a2, a2], 1)  # [B,5,C,R3,W]
    hi = d.to(torch.bfloat16)
    lo = (d - hi.float()).to(torch.bfloat16)
    assert torch.equal(got[..., 0, :].reshape(d.shape), hi)
    assert torch.equal(got[..., 1, :].reshape(d.shape), lo)
    with pytest.raises(ValueError):
        ops.wino_dy_rows(torch.zeros((1, 1, 3, 12), device=DEV))
    out = torch.empty(16, device=DEV)
    st = _native.load().mvbev_wino_dy_rows_f32(out.data_ptr(), 1, 1, 3, 12, dil, out.data_ptr(), 64, None)
    assert st == _native.ERR_SHAPE
    st = _native.load().mvbev_wino_dy_rows_f32(out.data_ptr(), 1, 1, 3, 16, 3, out.data_ptr(), 64, None)
    assert st == _native.ERR_DILATION


@pytest.mark.parametrize("B,K,H,W", [(1, 64, 12, 64), (2, 72, 17, 40), (1, 256, 31, 96), (2, 128, 25, 200)])
@pytest.mark.parametrize("dil", [1, 2])
def test_wgrad_wino_vs_torch_and_direct(B, K, H, W, dil):
    """Partial 128-channel tiles (K = 72), partial row tiles (H % 3, H % 12), a last segment of 8 px;
    dilation 2 from conv2's interleaved-row transform (``wino_rows(dilation=2)``)."""
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(K + H + W + dil)
    cout = 128
    x = F.relu(torch.randn((B, K, H, W), generator=g))
    dy = torch.randn((B, cout, H, W), generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (cout, K, 3, 3), dy.double(), padding=dil, dilation=dil)
    d = ops.conv_desc(B, K, H, W, group=K, group_stride=0, batch_stride=K * H * W)
    xs = _split_encode(x.to(DEV))
    t = torch.zeros((ops.wino_rows_bytes(d) + 1) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino_rows(xs, d, t, dilation=dil)
    dyd = dy.to(DEV)
    got = ops.conv3x3_wgrad_wino(t, d, ops.wino_dy_rows(dyd, dilation=dil), K, dilation=dil)
    assert_parity(got.cpu(), ref, "Winograd wgrad")
    direct = ops.conv3x3_wgrad(xs, d, dyd, dil, K)
    s_w, s_d = parity_stats(got.cpu(), ref), parity_stats(direct.cpu(), ref)
    # the transforms add about as much rounding again as the direct form's split products
    assert s_w["normwise"] < 8 * max(s_d["normwise"], 1e-7), (s_w, s_d)


def test_wgrad_wino_grouped_slab_channel_map_and_frustum_lists():
    """conv1's form: camera slots of 128 channels (view-major, module columns through the channel
    map), T written only at a frustum mask's (12 x 32 tile, slot) pairs, chunk lists from that mask;
    the coord columns are untouched."""
    from mvdet_amd import ops
    g = torch.Generator().manual_seed(11)
    S, B, C, Cs, H, W = 3, 2, 128, 128, 37, 104
    slab = F.relu(torch.randn((S, B, Cs, H, W), generator=g))
    rects = [(0, 12, 0, 40), (10, 37, 30, 100), (5, 9, 60, 75)]
    for s_, (r0, r1, c0, c1) in enumerate(rects):
        keep = torch.zeros((H, W))
        keep[r0:r1, c0:c1] = 1
        slab[s_] *= keep
    ty, tx = -(-H // 12), -(-W // 32)
    mask = torch.zeros(ty * tx, dtype=torch.int32)
    for t_ in range(ty * tx):
        y0, x0 = (t_ // tx) * 12, (t_ % tx) * 32
        win = slab[:, :, :, max(0, y0 - 1):y0 + 13, max(0, x0 - 1):x0 + 33]
        mask[t_] = sum(1 << s_ for s_ in range(S) if (win[s_] != 0).any())
    assert (mask != 7).any()
    cout, cin = 256, S * C + 2
    x = torch.cat([slab[s_] for s_ in range(S)] + [torch.zeros((B, 2, H, W))], 1)
    dy = torch.randn((B, cout, H, W), generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (cout, cin, 3, 3), dy.double(), padding=1)
    # slot order reversed against the module's view order: the channel map carries it
    chan_map = torch.tensor([(S - 1 - s_) * C + c for s_ in range(S) for c in range(Cs)], dtype=torch.int32)
    xs = torch.stack([_split_encode(slab[S - 1 - s_].to(DEV)) for s_ in range(S)])
    mask_slots = torch.zeros_like(mask)
    for s_ in range(S):
        mask_slots |= ((mask >> (S - 1 - s_)) & 1) << s_
    d = ops.conv_desc(B, S * Cs, H, W, group=Cs, group_stride=B * Cs * H * W, batch_stride=Cs * H * W)
    t = torch.zeros((ops.wino_rows_bytes(d) + 1) // 2, dtype=torch.bfloat16, device=DEV)
    ops.wino_rows(xs, d, t, mask_slots.to(DEV))
    lists = ops.wgrad_wino_chunk_lists(mask_slots.to(DEV), S, B, H, W)
    assert lists[1][-1].item() < B * (-(-H // 3)) * tx * S
    dw = torch.full((cout, cin, 3, 3), 9.0, device=DEV)
    ops.conv3x3_wgrad_wino(t, d, ops.wino_dy_rows(dy.to(DEV)), cin, chan_map=chan_map.to(DEV), dw=dw,
                           chunk_lists=lists)
    assert_parity(dw[:, :S * C].cpu(), ref[:, :S * C], "grouped Winograd wgrad with chunk lists")
    assert (dw[:, S * C:] == 9.0).all()
