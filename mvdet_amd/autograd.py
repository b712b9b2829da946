"""Native training path through project+fuse.

The reference trains through the hot path with stock autograd (``trainer.py:38-49``:
``map_res, imgs_res = model(data)`` then ``loss.backward()``): grid_sample's backward under
``kornia.warp_perspective`` (``persp_trans_detector.py:69``), the concat (``:77``) and
``nn.Conv2d``/``nn.ReLU`` backward of ``map_classifier`` (``:51-54``).  ``ProjectFuseFunction``
is one ``torch.autograd.Function`` whose forward is the engine's HIP forward (warp into the
slab, conv1-3) and whose backward is all HIP:

  conv3 (Cout 1, d4)   dy2 = dgrad(dmap) * [y2 > 0] (conv2's ReLU fused), dw3     (cout1 kernels)
  conv2 (d2) + ReLU    db2, dw2 = wgrad(y1, dy2) (3xbf16 MFMA), dy1 = dgrad-conv(dy2) * [y1 > 0]
  conv1 (d1) + ReLU    db1 + coord-channel dw1, view-channel dw1 = wgrad(slab, dy1) — from the
                       forward's row-Winograd transform T of the slab where conv1 ran Winograd
                       (ABI 12000) — and dslab = dgrad-conv(dy1) (transposed + flipped taps)
  warp                 grad_feat[v] = S_v^T dslab[v]: CSR gather over the transposed
                       sampling matrix (plan built once per geometry; deterministic)

Activations saved for the backward: conv1's input — T when its weight gradient runs from T (the
fused warp + B^T then writes T and no slab, as in inference), else the slab (split-bf16 with
3xbf16) — y1 (split-bf16) and y2 in fp32 (a fresh set per training forward, so a second forward
before ``backward()`` cannot overwrite them).  Parity: gradients within the north_star's 1e-3
relative fp32 gate of torch's CPU autograd on the same inputs (``tests/test_gpu_backward.py``).
"""
from __future__ import annotations

from types import SimpleNamespace
from typing import Sequence

import torch

from . import _native, ops
from .pipeline import ProjectFuse, Workspace, band_rows


# optional stage hook (bench / tools): called with a stage name right before it is enqueued
_stage_hook = None



# conv1's data gradient written pixel-major (MVBEV_LAYOUT_SPLIT_BF16_PIX) for the warp adjoint's gathers
# (ABI 12100); False: the channel-group-major split layout
DSLAB_PIXEL_MAJOR = True

def set_stage_hook(fn) -> None:
    global _stage_hook
    _stage_hook = fn


def _mark(stage: str) -> None:
    if _stage_hook is not None:
        _stage_hook(stage)


def _train_workspace(engine: ProjectFuse, B: int, device) -> Workspace:
    """A fresh (never reused) forward workspace.  y1 in the layout the inference path uses
    (split-bf16 with 3xbf16: conv2 runs on the ring kernel, conv2's weight gradient on the
    LDS-DMA wgrad kernel, and the ReLU mask is read from hi + lo), y2 kept in fp32 (conv3's
    backward reads it: no conv2 -> conv3 fusion)."""
    H, W = engine.grid_hw
    slab, zeroed = None, False
    if engine.split:
        # Split slabs come from a per-engine pool: zero-filled once, written only by this engine's
        # warps, whose skipped (out-of-source) pixels are the same every step (geometry-only), so
        # a reused slab still holds exact zeros there and the warp may skip them
        # (MVBEV_WARP_DST_ZEROED).  A slab returns to the pool when its backward has been enqueued,
        # with an event after its last reader: the next forward's stream waits on it, so a forward
        # on another stream than the backward cannot overwrite the slab under the wgrad kernels.
        pool = _slab_pool(engine, B, device)
        t1 = t2 = None
        if pool:
            # (with the slab, its Winograd transform buffers: conv1's T is zero-filled once and written
            # only at the frustum mask's (tile, view) pairs, the same every step)
            slab, done, t1, t2 = pool.pop()
            torch.cuda.current_stream(device).wait_event(done)
        else:
            slab = torch.zeros((engine.S,) + ops.split_shape(B, engine.Cs, H, W), dtype=torch.bfloat16,
                               device=device)
        zeroed = True
    else:
        slab = torch.empty((engine.S, B, engine.Cs, H, W), dtype=engine.slab_dtype, device=device)
        slab[:, :, engine.C:].zero_()  # padding channels the warp does not write
    y1r, y2r = band_rows(0, H, H)
    if engine.y1_split:
        y1 = torch.empty(ops.split_shape(B, engine.mid, H, W), dtype=torch.bfloat16, device=device)
    else:
        y1 = torch.empty((B, engine.mid, H, W), dtype=torch.float32, device=device)
    y2 = torch.empty((B, engine.mid, H, W), dtype=torch.float32, device=device)
    # the per-view device matrices (geometry only): cached, since a pageable host -> device copy per step
    # makes the host wait for the stream to drain (~0.1-0.25 ms of idle GPU per training step)
    mkey = (str(torch.device(device)), int(B))
    m = engine.__dict__.setdefault("_train_m", {}).get(mkey)
    if m is None:
        m = engine.m_norm_cpu.to(device)[:, None].expand(engine.num_cam, B, 3, 3).contiguous()
        engine._train_m[mkey] = m
    ws = Workspace(slab, y1, y2, m, (0, H), y1r, y2r, slab_zeroed=zeroed, store_y2=True, slab_rows=(0, H))
    if engine.split:
        ws.wino_t, ws.wino_t2 = t1, t2
        # conv1's weight gradient from T (_wgrad1_wino) is the backward's only reader of the forward's
        # conv1 input: the fused warp may write T and skip the slab (one pass, no B^T of the slab)
        ws.train_t_only = _wgrad1_wino_fits(engine, B)
    return ws


def _slab_pool(engine: ProjectFuse, B: int, device) -> list:
    pools = engine.__dict__.setdefault("_train_slabs", {})
    return pools.setdefault((str(torch.device(device)), int(B)), [])


def _bwd_state(engine: ProjectFuse):
    st = getattr(engine, "_bwd", None)
    if st is None:
        nc = engine.num_cam * engine.C
        st = SimpleNamespace(dgrad1=ops.PackedDgrad3x3(nc), dgrad2=ops.PackedDgrad3x3(engine.mid), wg_ws={})
        engine._bwd = st
    return st


def _adjoint_plans(engine: ProjectFuse, st, device, backbone_hw=None):
    """Per view: the CSR transpose of the warp (or, with ``backbone_hw``, of the fused
    3x-upsample + warp from that backbone size); geometry only, built once per device."""
    key = (str(device), None if backbone_hw is None else tuple(backbone_hw))
    if not hasattr(st, "plans"):
        st.plans = {}
    plans = st.plans.get(key)
    if plans is None:
        plans = [ops.WarpAdjointPlan(engine.m_norm_cpu[v], engine.src_hw, engine.grid_hw, device,
                                     backbone_hw=backbone_hw) for v in range(engine.num_cam)]
        st.plans[key] = plans
    return plans


def _wgrad_lists(engine: ProjectFuse, st, device, B: int):
    """Frustum chunk lists of conv1's wgrad (per camera slot), or None when not applicable."""
    H, W = engine.grid_hw
    if engine.Cs % 64 != 0:
        return None
    m = engine.conv1_mask(device, 0, H, tile_h=_native.TILE_H)  # the wgrad kernel's 8-row tiles
    if m is None:
        return None
    if not hasattr(st, "lists"):
        st.lists = {}
    key = (str(device), B)
    if key not in st.lists:
        st.lists[key] = ops.wgrad_chunk_lists(m, engine.S, B, H, W)
    return st.lists[key]


def _dy_rows(dy: torch.Tensor, split_x: bool):
    """dy pre-split into bf16 hi / lo rows (``ops.split_rows``) for the LDS-DMA wgrad kernel
    (split-bf16 x, W % 8 == 0: its per-segment split pass is then gone, bitwise the same dw),
    or None.  conv1 at cfg2: 2.33 -> 2.26 ms including the 35 us split."""
    return ops.split_rows(dy) if split_x and dy.shape[3] % 8 == 0 else None


def _dgrad1_schedule(st, B, cout_p, H, W, K, out_mask, cot_per_group, device):
    """conv1's data gradient as a balanced ring-kernel schedule (``ops.dgrad_schedule``: the
    last partial round of its equal blocks cut into K-pieces; cfg2 2.10 -> 2.03 ms), built
    once per (device, batch) — the mask is the geometry's."""
    if not hasattr(st, "sched1"):
        st.sched1 = {}
    key = (str(device), B)
    if key not in st.sched1:
        st.sched1[key] = ops.dgrad_schedule(B, cout_p, H, W, K, out_mask, cot_per_group, device)
    return st.sched1[key]


def _dgrad2_wino(engine: ProjectFuse, st, dy2s: torch.Tensor, w2: torch.Tensor) -> torch.Tensor:
    """conv2's data gradient as the forward's dilation-2 row-Winograd conv (``conv3x3_wino_dil``):
    with padding = dilation, dgrad(dy) = conv(dy, w^T flipped) — the weight's in / out channels
    swapped and its taps reversed (``ops.PackedWinoDgrad3x3``: packed from w2 itself, no transposed
    copy).  dy2s: split-bf16 [B, 512, H, W]."""
    H, W = engine.grid_hw
    mid = engine.mid
    B = dy2s.shape[0]
    d = ops.conv_desc(B, mid, H, W, group=mid, group_stride=0, batch_stride=mid * H * W)
    if getattr(st, "pack2t", None) is None:
        st.pack2t = ops.PackedWinoDgrad3x3(mid)
        st.t2d = None
    need = ops.wino_rows_bytes(d)
    if st.t2d is None or st.t2d.numel() * 2 < need or st.t2d.device != dy2s.device:  # zero-filled once
        st.t2d = torch.zeros((need + 1) // 2, dtype=torch.bfloat16, device=dy2s.device)
    ops.wino_rows(dy2s, d, st.t2d, dilation=2)
    return ops.conv3x3_wino_dil(st.t2d, d, st.pack2t.get(w2), mid, 2)


def _dgrad1_wino_applies(engine: ProjectFuse, cp: int, device) -> bool:
    """conv1's data gradient runs row-Winograd (``_dgrad1_wino``): the forward's conv1 did (split
    slab, finite geometry), whole 128-channel Cout tiles per view, slot s = view s."""
    n, C = engine.num_cam, engine.C
    return (engine.wino_active(device) and C % ops.BN == 0 and engine.Cs == C and cp == n * C
            and engine.slot_views == list(range(n)))


def _dgrad1_wino(engine: ProjectFuse, st, dy1s: torch.Tensor, w1: torch.Tensor, dslab: torch.Tensor) -> None:
    """conv1's data gradient (the N*C view channels) as the dilation-1 row-Winograd conv
    (``ops.conv3x3_wino_dgrad``) of the split dy1 with w1's view columns swapped and flipped, into
    the split ``dslab``; a view's 12 x 32 tiles its warp never samples are skipped (the forward's
    frustum mask, a superset of the sampled pixels: the adjoint reads nothing else).  The ring
    form (``conv3x3_dgrad``) executes the direct conv's 9 K-blocks per kernel column, this one 5."""
    H, W = engine.grid_hw
    mid, C = engine.mid, engine.C
    nc = engine.num_cam * C
    B = dy1s.shape[0]
    d = ops.conv_desc(B, mid, H, W, group=mid, group_stride=0, batch_stride=mid * H * W)
    if getattr(st, "pack1t", None) is None or st.pack1t.cout != nc:
        st.pack1t = ops.PackedWinoDgrad3x3(nc)  # w1's first nc input channels: the views (the coord ones last)
        st.t1d = None
    need = ops.wino_rows_bytes(d)
    if st.t1d is None or st.t1d.numel() * 2 < need or st.t1d.device != dy1s.device:
        st.t1d = torch.zeros((need + 1) // 2, dtype=torch.bfloat16, device=dy1s.device)
    ops.wino_rows(dy1s, d, st.t1d)
    cm = engine.conv1_mask(dy1s.device, 0, H, tile_h=12)
    ops.conv3x3_wino_dgrad(st.t1d, d, st.pack1t.get(w1), nc, dslab, out_mask=cm, cot_per_group=C // ops.BN)


def _wgrad_wino_fits(K: int, cout: int, H: int, W: int, B: int, dilation: int) -> bool:
    """``mvbev_conv3x3_wgrad_wino_bf16x3``'s shape limits (backward.hip): W % 8, whole 128-channel output
    tiles, B < 128, at most 4096 three-row tiles and 32-px segments, 32-bit chunk-invariant offsets."""
    r3 = -(-H // 3) if dilation == 1 else 4 * (-(-H // 12))
    r5 = 20 * (-(-H // 12))
    return (W % 8 == 0 and cout % 128 == 0 and K % 8 == 0 and B < 128 and r3 <= 4096 and -(-W // 32) <= 4096
            and (K // 8) * 2 * r5 * W < 2 ** 31 - 1 and cout * r3 * W < 2 ** 31 - 1
            and _native.load().mvbev_version() >= 12000)


def _wgrad1_wino_fits(engine: ProjectFuse, B: int) -> bool:
    """conv1's Winograd weight gradient takes this geometry (128-channel slots and the native limits,
    ``_wgrad_wino_fits``), so the forward may skip the slab."""
    H, W = engine.grid_hw
    return engine.Cs % 128 == 0 and _wgrad_wino_fits(engine.S * engine.Cs, engine.mid, H, W, B, 1)


def _wgrad1_wino_applies(engine: ProjectFuse, ws: Workspace, dy1: torch.Tensor) -> bool:
    """conv1's weight gradient runs row-Winograd (``_wgrad1_wino``) when the forward's conv1 did
    (its whole-grid transform T is in ``ws.wino_t``), with whole 128-channel slot tiles."""
    return ws.t1_valid and ws.wino_t is not None and _wgrad1_wino_fits(engine, dy1.shape[0])


def _wgrad1_wino(engine: ProjectFuse, st, ws: Workspace, d1, dy1: torch.Tensor, dw1: torch.Tensor) -> None:
    """conv1's view-channel weight gradient from the forward's transform T (``ops.conv3x3_wgrad_wino``):
    D = A-transform of dy1 (``ops.wino_dy_rows``), then per xi the T x D products over its 3 kernel
    columns, folded with G — 5/9 of the direct form's MFMAs.  Chunk lists from the 12-row frustum
    mask T was written under (a chunk whose T row is zero contributes exactly 0)."""
    H, W = engine.grid_hw
    B, dev, mid = dy1.shape[0], dy1.device, engine.mid
    lists = None
    m = engine.conv1_mask(dev, 0, H)
    if m is not None:
        if not hasattr(st, "lists_wino"):
            st.lists_wino = {}
        key = (str(dev), B)
        if key not in st.lists_wino:
            st.lists_wino[key] = ops.wgrad_wino_chunk_lists(m, engine.S, B, H, W)
        lists = st.lists_wino[key]
    ops.conv3x3_wgrad_wino(ws.wino_t, d1, ops.wino_dy_rows(dy1), dw1.shape[1], chan_map=engine.pack1.map_dev(dev),
                           dw=dw1, workspace=_wgrad_wino_ws(st, d1, mid, 1, dev), chunk_lists=lists)


def _wgrad_wino_ws(st, desc, cout, dilation, device) -> torch.Tensor:
    """The Winograd weight gradients' partition workspace (shared buffer, grown once: one runs at a time)."""
    import ctypes
    need = int(_native.load().mvbev_conv3x3_wgrad_wino_workspace_bytes(ctypes.byref(desc), cout, dilation))
    buf = st.wg_ws.get(str(device))
    if buf is None or buf.numel() * 4 < need:
        buf = torch.empty((need + 3) // 4, dtype=torch.float32, device=device)
        st.wg_ws[str(device)] = buf
    return buf


def _wgrad_ws(st, desc, cout, device) -> torch.Tensor:
    import ctypes
    from . import _native
    need = int(_native.load().mvbev_conv3x3_wgrad_workspace_bytes(ctypes.byref(desc), cout))
    buf = st.wg_ws.get(str(device))
    if buf is None or buf.numel() * 4 < need:
        buf = torch.empty((need + 3) // 4, dtype=torch.float32, device=device)
        st.wg_ws[str(device)] = buf
    return buf


class ProjectFuseFunction(torch.autograd.Function):
    """``map = fuse(concat(warp(feats[v]) for v) + coord)``; inputs after the engine and the
    ``backbone`` flag: the N view features, then conv1.w, conv1.b, conv2.w, conv2.b, conv3.w.
    ``backbone`` False: the features are the upsampled [B,C,H,W] maps kornia receives
    (``persp_trans_detector.py:65`` done by the caller); True: the backbone-resolution [B,C,h,w]
    maps, upsampled inside the warp (``warp_views_upsampled``) and differentiated through the
    fused upsample + warp adjoint, so neither the upsampled maps nor their gradient exist."""

    @staticmethod
    def forward(ctx, engine: ProjectFuse, backbone: bool, *args):
        n = engine.num_cam
        feats, (w1, b1, w2, b2, w3) = args[:n], args[n:]
        if engine.slab_dtype != torch.float32 or engine.S != n:
            raise ValueError("the native backward needs an fp32-storage single-GPU engine")
        B = feats[0].shape[0]
        dev = feats[0].device
        ws = _train_workspace(engine, B, dev)
        _mark("warp")
        if backbone:
            engine.warp_views_upsampled(ws, list(range(n)), [f.detach() for f in feats])
        else:
            engine.warp_views(ws, list(range(n)), [f.detach() for f in feats])
        ctx.backbone = bool(backbone)
        mc = [SimpleNamespace(weight=w1, bias=b1), None, SimpleNamespace(weight=w2, bias=b2), None,
              SimpleNamespace(weight=w3, bias=None)]
        out = engine.fuse(ws, mc, mark=_stage_hook)
        ctx.engine = engine
        ctx.ws = ws
        ctx.feat_shape = tuple(feats[0].shape)
        # channels-last maps (the detector's backbone): their gradients are written channels-last too, so
        # autograd's grad-layout contract needs no copy
        ctx.feat_cl = (feats[0].dim() == 4 and not feats[0].is_contiguous()
                       and feats[0].is_contiguous(memory_format=torch.channels_last))
        ctx.save_for_backward(w1, b1, w2, b2, w3)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dmap):
        engine: ProjectFuse = ctx.engine
        ws: Workspace = ctx.ws
        if ws is None:
            raise RuntimeError("ProjectFuseFunction: trying to backward through this graph a second time; its saved "
                               "activations (slab, y1, y2) are released after the first backward (the native "
                               "kernels keep no retain_graph copy). Run the forward again.")
        w1, b1, w2, b2, w3 = ctx.saved_tensors
        n = engine.num_cam
        need = ctx.needs_input_grad[2:]
        need_feat = any(need[:n])
        st = _bwd_state(engine)
        H, W = engine.grid_hw
        B = ws.y1.shape[0]
        dev = ws.y1.device
        y1_split = ws.y1.dtype == torch.bfloat16
        dmap = dmap.contiguous().float()
        mid = engine.mid
        # conv3: dy2 = dgrad * relu'(y2); dw3
        _mark("bwd_conv3")
        # with split y1 the data gradients run on the ring kernel: dy2 also in the split layout
        dy2s = torch.empty(ops.split_shape(B, mid, H, W), dtype=torch.bfloat16, device=dev) if y1_split else None
        dy2, dw3 = ops.conv3x3_cout1_backward(ws.y2, w3, dmap, 4, relu_mask=True, dx_split=dy2s)
        # conv2: db2, dw2, dy1 = dgrad * relu'(y1)
        _mark("bwd_conv2_wgrad")
        db2 = torch.empty(mid, dtype=torch.float32, device=dev) if b2 is not None else None
        if db2 is not None:
            ops.conv3x3_bias_coord_grad(dy2, 2, db=db2)
        d_y1 = ops.conv_desc(B, mid, H, W, group=mid, group_stride=0, batch_stride=mid * H * W)
        if ws.t2_valid and _wgrad_wino_fits(mid, mid, H, W, B, 2):  # from conv2's own T (the native limits)
            dw2 = ops.conv3x3_wgrad_wino(ws.wino_t2, d_y1, ops.wino_dy_rows(dy2, dilation=2), mid, dilation=2,
                                         workspace=_wgrad_wino_ws(st, d_y1, mid, 2, dev))
        else:  # (the direct form reads the fp32 dy2: at its size the row split costs what it saves)
            dw2 = ops.conv3x3_wgrad(ws.y1, d_y1, dy2, 2, mid, workspace=_wgrad_ws(st, d_y1, mid, dev))
        _mark("bwd_conv2_dgrad")
        if dy2s is not None and engine.wino_conv2_active(ws):
            dy1 = _dgrad2_wino(engine, st, dy2s, w2)
        else:
            dy1 = ops.conv3x3_dgrad(dy2 if dy2s is None else dy2s, st.dgrad2, w2, 2)
        if dy1.shape[1] != mid:
            dy1 = dy1[:, :mid].contiguous()
        del dy2, dy2s
        dy1s = None
        if y1_split:  # the masked dy1 also in the split layout: conv1's dgrad on the ring kernel
            dy1s = torch.empty(ops.split_shape(B, mid, H, W), dtype=torch.bfloat16, device=dev)
            ops.relu_backward_split_(dy1, ws.y1, dy1s)
        else:
            ops.relu_backward_(dy1, ws.y1)
        # conv1: db1 + coord channels, view channels (slab order through the pack's channel map)
        _mark("bwd_conv1_wgrad")
        nc = n * engine.C
        dw1 = torch.zeros_like(w1)
        db1 = torch.empty(mid, dtype=torch.float32, device=dev) if b1 is not None else None
        ops.conv3x3_bias_coord_grad(dy1, 1, db=db1, dw=dw1, coord_ch=nc)
        chan_map = engine.pack1.map_dev(dev)  # (round 6: no re-pack of the direct conv1 weights it does not use)
        d1 = ops.conv_desc(B, engine.S * engine.Cs, H, W, group=engine.Cs, group_stride=B * engine.Cs * H * W,
                           batch_stride=engine.Cs * H * W)
        if _wgrad1_wino_applies(engine, ws, dy1):
            _wgrad1_wino(engine, st, ws, d1, dy1, dw1)
        elif ws.t_from_warp:
            raise RuntimeError("conv1's weight gradient needs the slab, but the fused warp wrote only T")
        else:
            ops.conv3x3_wgrad(ws.slab, d1, dy1, 1, w1.shape[1], chan_map=chan_map, dw=dw1,
                              workspace=_wgrad_ws(st, d1, mid, dev), chunk_lists=_wgrad_lists(engine, st, dev, B),
                              dy_rows=_dy_rows(dy1, ws.slab.dtype == torch.bfloat16))
        grads = [None] * n
        if need_feat:
            _mark("bwd_conv1_dgrad")
            C = engine.C
            cp = st.dgrad1.cout_p
            pixm = DSLAB_PIXEL_MAJOR and dy1s is not None and C % ops.KC == 0
            if C % ops.KC == 0:  # split-bf16 dslab: the adjoint gathers 8 channels per 32-B entry (pixel-major:
                # an output pixel's 64 channels per 256-B gather)
                dslab = torch.empty(ops.split_pix_shape(B, cp, H, W) if pixm else ops.split_shape(B, cp, H, W),
                                    dtype=torch.bfloat16, device=dev)
                if dy1s is not None and _dgrad1_wino_applies(engine, cp, dev):
                    _dgrad1_wino(engine, st, dy1s, w1, dslab)
                else:
                    # frustum: a view's tiles of dslab that its warp never samples are not computed
                    cm = (engine.conv1_mask(dev, 0, H, tile_h=ops.dgrad_tile_rows(dy1s is not None, 1))
                          if C % ops.BN == 0 else None)
                    sched = (_dgrad1_schedule(st, B, cp, H, W, mid, cm, C // ops.BN, dev) if dy1s is not None
                             else None)
                    ops.conv3x3_dgrad(dy1 if dy1s is None else dy1s, st.dgrad1, w1, 1, out=dslab, out_mask=cm,
                                      cot_per_group=C // ops.BN, sched=sched)
                g8 = C // ops.KC
                douts = [dslab[:, :, :, v * g8:(v + 1) * g8] if pixm else dslab[:, v * g8:(v + 1) * g8]
                         for v in range(n)]
            else:
                dslab = ops.conv3x3_dgrad(dy1, st.dgrad1, w1, 1)   # [B, round_up(nc,128), H, W]
                douts = [dslab[:, v * C:(v + 1) * C] for v in range(n)]
            _mark("bwd_warp")
            mf = torch.channels_last if (pixm and ctx.feat_cl) else torch.contiguous_format
            gs = [torch.empty(ctx.feat_shape, dtype=torch.float32, device=dev, memory_format=mf) for _ in range(n)]
            plans = _adjoint_plans(engine, st, dev, backbone_hw=ctx.feat_shape[2:] if ctx.backbone else None)
            ops.warp_views_adjoint(douts, plans, gs, pixel_major=pixm)
            grads = [g if need[v] else None for v, g in enumerate(gs)]
        _mark("bwd_end")
        if ws.slab_zeroed:  # its readers are enqueued: reusable once this stream passes this point
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(dev))
            _slab_pool(engine, B, dev).append((ws.slab, done, ws.wino_t, ws.wino_t2))
        ctx.ws = None
        return (None, None, *grads, dw1, db1, dw2, db2, dw3)


def project_fuse(engine: ProjectFuse, feats: Sequence[torch.Tensor], map_classifier) -> torch.Tensor:
    """Differentiable project+fuse: ``feats[v]`` the upsampled [B,C,H,W] features of view v,
    ``map_classifier`` the reference's ``nn.Sequential`` (``persp_trans_detector.py:51-54``)."""
    c1, c2, c3 = map_classifier[0], map_classifier[2], map_classifier[4]
    return ProjectFuseFunction.apply(engine, False, *feats, c1.weight, c1.bias, c2.weight, c2.bias, c3.weight)


def project_fuse_backbone(engine: ProjectFuse, feats: Sequence[torch.Tensor], map_classifier) -> torch.Tensor:
    """Differentiable upsample + project + fuse (``persp_trans_detector.py:65-87`` after the
    backbone): ``feats[v]`` view v's backbone-resolution [B,C,h,w] map; the 3x bilinear
    upsample runs inside the warp and its adjoint inside the warp's."""
    c1, c2, c3 = map_classifier[0], map_classifier[2], map_classifier[4]
    return ProjectFuseFunction.apply(engine, True, *feats, c1.weight, c1.bias, c2.weight, c2.bias, c3.weight)
