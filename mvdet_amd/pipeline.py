"""The project+fuse hot path as one reusable engine.

Data layout in HBM (per device, per batch size B):

* ``slab``  — the warped ground-plane features, **view-major**
  ``[S, B, Cs, Ho, Wo]`` fp32 (fp16 for the config-4 fp16-storage path) (S view slots, Cs = C rounded up to 8).  View ``v``'s
  warp writes slot ``slot_of[v]`` directly; this *is* the concatenation of
  ``persp_trans_detector.py:77`` (zero-copy).  View-major keeps each GPU's share
  of the views contiguous, so the multi-GPU all-gather needs no repack
  (``mvdet_amd.parallel``).
* ``coord_term`` — ``[512, Ho, Wo]``: conv1's contribution of the two constant
  coord channels (``:21,77``) plus conv1's bias.  It does not depend on the
  input, so it is computed once per weight version (with the same conv kernel)
  and enters conv1's epilogue as the ``init`` term instead of being read as two
  more input channels every forward.
* ``y1``, ``y2`` — conv1 / conv2 activations ``[B, 512, rows, Wo]`` (rows = the
  output band plus the halo the next layer needs; the whole grid on one GPU).

``precision`` selects the conv1/conv2 kernel: "bf16x3" (default: hi/lo bf16 split,
three bf16 MFMA passes, fp32 accumulate — the same parity vs the oracle as exact fp32,
3x faster) or "fp32" (fp32-input MFMA, exact fp32 products).

``warp_view`` is a5 for one view; ``fuse`` is a7-a9 (a10, the same-size bilinear
interpolate of ``:82``, is an exact identity and is elided).  Nothing here
allocates in steady state, copies to the host or synchronises.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _native, ops
from .geometry import kornia_src_norm_from_dst_norm

# halo rows each layer needs below/above its output rows (dilations 1, 2, 4 of :51-54)
HALO_CONV1, HALO_CONV2, HALO_CONV3 = 1, 2, 4


def band_rows(r0: int, r1: int, H: int):
    """Row ranges (global, half-open) of y1, y2 needed for output rows [r0, r1)."""
    y2 = (max(0, r0 - HALO_CONV3), min(H, r1 + HALO_CONV3))
    y1 = (max(0, y2[0] - HALO_CONV2), min(H, y2[1] + HALO_CONV2))
    return y1, y2


@dataclass
class Workspace:
    slab: torch.Tensor      # [S, B, Cs, Ho, Wo]
    y1: torch.Tensor        # [B, 512, y1_rows, Wo]
    y2: torch.Tensor        # [B, 512, y2_rows, Wo]
    m_norm: torch.Tensor    # [N, B, 3, 3] device fp32
    band: Tuple[int, int]   # output rows [r0, r1)
    y1_rows: Tuple[int, int]
    y2_rows: Tuple[int, int]
    # the slab was zero-filled at allocation and is only written by this engine's warps (or the
    # multi-GPU gather of them): a view's out-of-source pixels are already 0 and are skipped
    slab_zeroed: bool = False
    # conv2 -> conv3 fused (inference): conv3's per-(64-channel set, tap, pixel) partials
    # [B, 2 * 512 / 128, 9, y2_rows, Wo] fp32 replace y2 in HBM (allocated on first use)
    p3: Optional[torch.Tensor] = None
    # keep y2 in HBM (the training forward: conv3's backward reads it), i.e. no conv2 -> conv3 fusion
    store_y2: bool = False
    # row-Winograd transform of y1 for conv2 (dilation 2; allocated on first use)
    wino_t2: Optional[torch.Tensor] = None
    # row-Winograd transform of the slab for conv1 (bf16, zero-filled on first use; only the
    # frustum mask's (tile, slot) pairs are ever written)
    wino_t: Optional[torch.Tensor] = None
    # wino_t holds the current frame's transform, written by the fused warp (the slab was not)
    t_from_warp: bool = False
    # the F(4,3) transforms (ABI 12400, inference over the whole grid where ProjectFuse.wino43_pays): T43 of the
    # slab for conv1 (zero-filled on first use, as wino_t) and of y1 for conv2; t_form = the form of the
    # current frame's conv1 transform (3: wino_t, 4: wino_t43)
    wino_t43: Optional[torch.Tensor] = None
    wino_t2_43: Optional[torch.Tensor] = None
    t_form: int = 3
    # wino_t holds this forward's transform of the whole grid (conv1 ran row-Winograd over all rows):
    # the training backward's conv1 weight gradient reads it (autograd._wgrad1_wino)
    t1_valid: bool = False
    # wino_t2 holds this forward's dilation-2 transform of the whole y1 (conv2 ran row-Winograd): the
    # training backward's conv2 weight gradient reads it (autograd._wgrad_wino)
    t2_valid: bool = False
    # training forward whose backward reads conv1's T and never the slab (autograd._train_workspace):
    # the fused warp + B^T may run, as in inference
    train_t_only: bool = False
    # grid rows the slab holds: (0, Ho) for a warped slab; a row window for a band-local slab
    # filled by the multi-GPU band exchange (parallel.ViewBands)
    slab_rows: Tuple[int, int] = (0, 0)
    # the non-finite guard (ProjectFuse.nonfinite_guard): the fused warp stores nf_tag into nf[0] when
    # it samples a NaN / inf feature; guard_src = {slot: (cam, feat, up_hw)} of the frame's fused warps
    # (accumulated over the warp calls of one frame under one tag; None = no frame in flight), for the
    # exact path
    nf: Optional[torch.Tensor] = None
    nf_tag: int = 0
    guard_src: Optional[dict] = None
    # the exact path's buffers, sized for one row band of at most ProjectFuse.guard_bytes of fp32 slab:
    # slab [S, B, Cs, rows + 14, Wo], y1 / y2 [B, 512, rows + 12 / + 8, Wo]
    g_slab: Optional[torch.Tensor] = None
    g_y1: Optional[torch.Tensor] = None
    g_y2: Optional[torch.Tensor] = None
    nf2: Optional[torch.Tensor] = None   # the partial-sum mode's flag of the summed conv1 (finish_from_y1)
    nf2_tag: int = 0
    cl_maps: Optional[list] = None          # channels-last copies of NCHW backbone maps (cl_upsample)


class ProjectFuse:
    """Warp + zero-copy concat + fusion head for ``num_cam`` views of ``channels``.

    ``slot_views``: which view each slab slot holds (``None`` = empty slot); default
    slot s = view s.  The multi-GPU path uses a rank-major slot order.

    ``parts`` (the partial-sum multi-GPU mode's channel split, round 5): ``[(view, c0), ...]`` — this
    engine's "cameras" are channel slices ``[c0, c0 + part_channels)`` of those views of ``channels``
    each (conv1 is linear in its input channels, so a view's channels can be convolved on several ranks).
    Its slots, masks, warps and T are those of ``len(parts)`` cameras of ``part_channels``; only conv1's
    channel map (and the module's ``cin``) refer to the views: slot s channel c is module channel
    ``view_s * channels + c0_s + c``.  Callers pass the features' channel slices as the cameras' features.

    ``wino43`` (round 6, ABI 12400): the inference convs as row-Winograd F(4,3) — ``None`` (default) where
    ``wino43_pays``, ``True`` wherever the whole-grid inference path applies, ``False`` never (F(3,3)).
    """

    def __init__(self, proj_mats: Sequence[torch.Tensor], src_hw: Tuple[int, int], grid_hw: Tuple[int, int],
                 channels: int, mid_channels: int = 512, slot_views: Optional[Sequence[Optional[int]]] = None,
                 precision: str = "bf16x3", slab_dtype: torch.dtype = torch.float32,
                 all_views: bool = True, split_k: bool = True, frustum: bool = True, fuse_conv3: bool = True,
                 edge_strip: bool = True, wino_conv1: bool = True, wino_warp: bool = True,
                 wino_conv2: bool = True, nonfinite_guard: bool = True, cl_upsample: bool = True,
                 parts: Optional[Sequence[Tuple[int, int]]] = None, part_channels: Optional[int] = None,
                 wino43: Optional[bool] = None):
        if slab_dtype not in (torch.float32, torch.float16):
            raise ValueError("slab_dtype must be float32 or float16")
        if slab_dtype == torch.float16 and precision != "bf16x3":
            raise ValueError("an fp16 slab needs precision='bf16x3' (the fp32-MFMA conv reads fp32)")
        self.precision = precision
        self.slab_dtype = slab_dtype
        # 3xbf16 with fp32 storage: the warp writes the pre-split bf16 hi/lo blocked slab
        self.split = precision == "bf16x3" and slab_dtype == torch.float32
        n_views, view_ch = len(proj_mats), int(channels)
        self.parts = None if parts is None else [(int(v), int(c0)) for v, c0 in parts]
        if self.parts is not None:  # cameras = channel slices of views
            if part_channels is None or not all(0 <= v < n_views and 0 <= c0 and c0 + part_channels <= view_ch
                                                for v, c0 in self.parts):
                raise ValueError("parts need part_channels and channel slices inside their views")
            proj_mats = [proj_mats[v] for v, _ in self.parts]
            channels = int(part_channels)
        self.num_cam = len(proj_mats)
        self.src_hw = (int(src_hw[0]), int(src_hw[1]))
        self.grid_hw = (int(grid_hw[0]), int(grid_hw[1]))
        self.C = int(channels)
        self.Cs = ops.padded_channels(self.C)
        self.mid = int(mid_channels)
        self.cin = n_views * view_ch + 2                # conv1 input channels of the module
        self.slot_views = list(range(self.num_cam)) if slot_views is None else list(slot_views)
        self.S = len(self.slot_views)
        self.slot_of = {v: s for s, v in enumerate(self.slot_views) if v is not None}
        if all_views:
            assert sorted(self.slot_of) == list(range(self.num_cam)), "every view needs exactly one slot"
        else:  # partial-sum multi-GPU: this engine's slab holds a subset of the views
            assert set(self.slot_of) <= set(range(self.num_cam)) and self.S > 0
        # kornia steps 1-2 (normalize_homography + _torch_inverse_cast) on the host, fp32,
        # from the fp32-cast projection matrix exactly as :68-69 feeds kornia.
        self.m_norm_cpu = torch.stack([
            kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), self.src_hw, self.grid_hw)[0]
            for M in proj_mats])  # [N, 3, 3]
        # conv1 weight channels, in slab order: slot s channel c -> module channel v*C + c (a part: its view's
        # channel c0 + c)
        chan_map = []
        for v in self.slot_views:
            base = None if v is None else (v * self.C if self.parts is None else
                                           self.parts[v][0] * view_ch + self.parts[v][1])
            for c in range(self.Cs):
                chan_map.append(base + c if (v is not None and c < self.C) else -1)
        nc = n_views * view_ch
        self.pack1 = ops.PackedConv3x3(chan_map, precision)
        self.coord_c0 = nc  # conv1's input channels of the coord map (x, y) after the views' (:77)
        self.pack2 = ops.PackedConv3x3(None, precision)
        self._ws: Dict[tuple, Workspace] = {}
        self._coord_key = None
        self._coord_term: Optional[torch.Tensor] = None
        self._sk: Dict[str, torch.Tensor] = {}  # split-K-tail scratch per device (bf16x3 convs)
        self.split_k = split_k
        # conv1 skips, per output tile, the slots whose warp is exactly zero there (camera
        # frustum; geometry-only, so the mask is built once per device and row range)
        self.frustum = frustum and precision == "bf16x3" and self.Cs % 16 == 0 and self.S <= 16
        self._masks: Dict[tuple, torch.Tensor] = {}
        # conv1 writes y1 pre-split (bf16 hi/lo blocks) so conv2 stages it with 16-B copies;
        # the partial-sum multi-GPU mode turns this off (it sums fp32 partials)
        self.y1_split = precision == "bf16x3"
        # conv2's epilogue computes conv3's per-tap partial sums instead of storing y2
        # (split-bf16 y1, i.e. the ring conv); training keeps y2 (its backward reads it)
        self.fuse_conv3 = fuse_conv3
        # the forward conv1 (frustum-masked ring kernel) on edge-strip tiles where the grid width
        # leaves a partial last tile column (W % 32 in 1..16: Wildtrack's 360 = 11 x 32 + 8), so
        # no MFMA column is spent past W (mvbev_conv3x3_bf16x3_ex3); bitwise the same y1
        self.edge_strip = edge_strip
        # wino_conv1 (default): the inference conv1 as F(3,3) row-Winograd (ops.wino_rows +
        # conv3x3_wino: 5 instead of 9 MFMA K-blocks per chunk and kernel column, over the 12 x 32
        # grid tiles); split-bf16 slab only, not in training (its backward reads the direct form's
        # operands).  B^T mixes a 3-row tile's input rows, so a non-finite warp sample (a degenerate
        # homography: kornia's NaN output) would spread over its tile where the reference's direct
        # conv keeps it to the taps that read it: geometry that can produce a non-finite sample
        # (``nonfinite_views``, the warp kernels' own coordinate code) runs the direct conv1
        # instead (``wino_active``), so the NaN pattern stays the reference's.
        self.wino_conv1 = wino_conv1 and self.split
        self._nonfinite: Dict[str, int] = {}
        self.pack1w = ops.PackedConv3x3(chan_map, "bf16x3", wino=True) if self.wino_conv1 else None
        # wino_warp: warp_views writes the row transform T directly (one pass, no slab, no
        # separate transform); inference over the whole grid from fp32 features only (cfg2:
        # 0.55 ms vs warp 0.36 + transform 0.26)
        self.wino_warp = self.wino_conv1 and wino_warp
        # wino_conv2 (default): conv2 (dilation 2) -> conv3 partials as row-Winograd too (ops.wino_rows
        # with dilation 2 over y1, then conv3x3_wino_then_cout1_partials); under the same geometry
        # condition as conv1 (a NaN in y1 would spread over a 3-row tile)
        self.wino_conv2 = wino_conv2 and precision == "bf16x3" and self.y1_split
        self.pack2w = ops.PackedConv3x3(None, "bf16x3", wino=True) if self.wino_conv2 else None
        # nonfinite_guard (default): NaN / inf in the FEATURES (a diverging backbone, fp16 overflow
        # upstream).  The fused warp folds B^T (and the upsample's taps) before any product, so such a
        # value would not keep the reference's NaN / inf pattern (and the 3xbf16 split turns inf into
        # NaN).  The fused warp reports it into a device flag; after the fast path the exact path is
        # enqueued — the reference-order warp (+ upsample) into an fp32 slab, the fp32-MFMA conv1 /
        # conv2 (exact products: inf * w stays inf, torch's NaN-preserving ReLU) and conv3 — every
        # launch gated on the flag, so with finite features they exit at once and nothing is synced.
        self.nonfinite_guard = nonfinite_guard
        # the exact path runs in row bands whose fp32 slab holds at most this many bytes (a
        # whole-grid fp32 slab would double the fusion's largest buffer — 10 GB at cfg3 — for a rare path)
        self.guard_bytes = 1 << 30
        # cl_upsample (default): copy NCHW backbone maps to channels-last (mvbev_nchw_to_nhwc_f32, 16-B
        # accesses, 1/9 of the upsampled size) for the line-per-pixel fused upsample warp
        # (warp_up_wino_cl_kernel) when C % 32 == 0: copy + warp 0.36 ms vs the NCHW kernel's 0.376 at cfg2
        # (profiles/r04n_kbench.jsonl); maps that are channels-last already skip the copy
        self.cl_upsample = cl_upsample
        self._pack1f: Optional[ops.PackedConv3x3] = None
        self._pack2f: Optional[ops.PackedConv3x3] = None
        self._chan_map = chan_map
        # wino43 (ABI 12400; default: where it pays, ``wino43_pays``): the inference conv1 and conv2 -> conv3 over
        # the whole grid as row-Winograd F(4,3) (6 transformed rows per 4 output rows, 10 % fewer MFMAs than
        # F(3,3); 16 x 32 tiles, the K sum walked xi-major) — the fused warp then writes T43.  Not in training
        # (its backward reads F(3,3)'s T) nor in the partial-sum multi-GPU engines (conv1_partial).
        # (True: wherever it applies, without the wino43_pays rule — tests and A/B runs)
        self.wino43 = (self.wino_conv1 and all_views and self.parts is None) if wino43 is None else \
            (bool(wino43) and self.wino_conv1)
        self._wino43_forced = wino43 is True
        self.pack1w43 = ops.PackedConv3x3(chan_map, "bf16x3", wino=True, form=4) if self.wino43 else None
        self.pack2w43 = ops.PackedConv3x3(None, "bf16x3", wino=True, form=4) if self.wino43 else None
        self._cus: Dict[str, int] = {}

    def wino43_pays(self, rows: int, B: int, device, deep: bool = False) -> bool:
        """F(4,3) over ``rows`` output rows (whole grid): enabled and its 16-row tiles waste at most 3 % of the rows;
        ``deep`` (conv2 -> conv3, whose workgroups all cost the same): the launch is also at least 8 rounds of
        workgroups deep (16 x 32 pixel tiles x 4 Cout tiles over the CUs) — a shallow one loses a round to
        F(4,3)'s 1.2x larger workgroups.  Measured (interleaved kbench, ``profiles/r06aj_wino43_ab.jsonl``,
        ``r06am_wino43_wide_tiles_ab.jsonl``), conv1 (frustum-masked, workgroups dealt heaviest first) F(3,3) ->
        F(4,3): cfg1 0.350 -> 0.320 ms, cfg3 19.9 -> 18.0, cfg4 8.02 -> 7.12, cfg5 14.5 -> 13.3, cfg2 (120 rows:
        6.7 % of the 16-row tiles idle) 1.437 -> 1.438; conv2 -> conv3: cfg3 4.78 -> 4.43, cfg4 2.47 -> 2.18, cfg5
        7.05 -> 6.60, but cfg1 (1.25 rounds) 0.311 -> 0.343 and cfg2 0.327 -> 0.357."""
        if not self.wino43:
            return False
        if self._wino43_forced:
            return True
        rows = int(rows)
        h16 = -(-rows // 16) * 16
        if h16 - rows > 0.03 * rows:
            return False
        if not deep:
            return True
        key = str(torch.device(device))
        if key not in self._cus:
            dev = torch.device(device)
            self._cus[key] = (torch.cuda.get_device_properties(dev).multi_processor_count
                              if dev.type == "cuda" else 256)
        tiles = (h16 // 16) * -(-self.grid_hw[1] // 32) * int(B) * max(1, self.mid // ops.BN)
        return tiles >= 8 * self._cus[key]

    # -- buffers ----------------------------------------------------------------------------
    def workspace(self, B: int, device, band: Optional[Tuple[int, int]] = None,
                  slab_rows: Optional[Tuple[int, int]] = None, tag: int = 0) -> Workspace:
        """Buffers for output rows ``band`` (default: the whole grid).  ``slab_rows``: a slab
        holding only grid rows [r0, r1) (must cover conv1's input rows for the band) — the
        band-local slab the multi-GPU band exchange fills; warps refuse it.  ``tag`` keeps
        several workspaces of one shape apart (double buffering)."""
        device = torch.device(device)
        H, W = self.grid_hw
        band = (0, H) if band is None else (int(band[0]), int(band[1]))
        slab_rows = (0, H) if slab_rows is None else (int(slab_rows[0]), int(slab_rows[1]))
        key = (str(device), int(B), band, slab_rows, int(tag))
        ws = self._ws.get(key)
        if ws is None:
            y1r, y2r = band_rows(band[0], band[1], H)
            if not (0 <= slab_rows[0] <= max(0, y1r[0] - HALO_CONV1) and min(H, y1r[1] + HALO_CONV1) <= slab_rows[1] <= H):
                raise ValueError(f"slab rows {slab_rows} do not cover conv1's input rows for output band {band}")
            R = slab_rows[1] - slab_rows[0]
            if self.split:
                slab = torch.zeros((self.S,) + ops.split_shape(B, self.Cs, R, W), dtype=torch.bfloat16,
                                   device=device)
            else:
                slab = torch.zeros((self.S, B, self.Cs, R, W), dtype=self.slab_dtype, device=device)
            if self.y1_split:
                y1 = torch.empty(ops.split_shape(B, self.mid, y1r[1] - y1r[0], W), dtype=torch.bfloat16,
                                 device=device)
            else:
                y1 = torch.empty((B, self.mid, y1r[1] - y1r[0], W), dtype=torch.float32, device=device)
            y2 = torch.empty((B, self.mid, y2r[1] - y2r[0], W), dtype=torch.float32, device=device)
            m = self.m_norm_cpu.to(device)[:, None].expand(self.num_cam, B, 3, 3).contiguous()
            ws = Workspace(slab, y1, y2, m, band, y1r, y2r, slab_zeroed=True, slab_rows=slab_rows)
            self._ws[key] = ws
        return ws

    def y1_fp32(self, ws: Workspace) -> torch.Tensor:
        """conv1's output rows ``ws.y1_rows`` as fp32 [B, 512, rows, Wo] (decodes the split layout)."""
        return ops.split_decode(ws.y1, self.mid) if ws.y1.dtype == torch.bfloat16 else ws.y1

    def view_slice(self, ws: Workspace, cam: int) -> torch.Tensor:
        """[B, C, Ho, Wo] of ``cam``'s warped features: a view of the slab, or (split
        layout) its fp32 decode (hi + lo).  Not available after the fused warp (``wino_warp``),
        which writes conv1's row transform instead of the slab."""
        if ws.t_from_warp:
            raise RuntimeError("the slab was not written: the warp wrote conv1's row transform instead "
                               "(wino_warp); use wino_warp=False to keep the warped views")
        if self.split:
            return ops.split_decode(ws.slab[self.slot_of[cam]], self.C)
        return ws.slab[self.slot_of[cam], :, :self.C]

    def _slot_dst(self, ws: Workspace, cam: int) -> torch.Tensor:
        return ws.slab[self.slot_of[cam]] if self.split else ws.slab[self.slot_of[cam], :, :self.C]

    # -- a5 -------------------------------------------------------------------------------
    def warp_view(self, ws: Workspace, cam: int, feat: torch.Tensor) -> None:
        """a5 (+ zero-copy a6): warp one view's [B,C,h,w] features into its slab slot.  Not
        after a fused warp (``wino_warp``) of the same workspace: that wrote conv1's row transform,
        not the slab, so the slab's other slots would hold an older frame."""
        if tuple(feat.shape[2:]) != self.src_hw or feat.shape[1] != self.C:
            raise ValueError(f"view {cam}: features {tuple(feat.shape)} do not match "
                             f"[B,{self.C},{self.src_hw[0]},{self.src_hw[1]}]")
        self._check_warp_ws(ws)
        if ws.t_from_warp:
            raise RuntimeError("warp_view after a fused warp_views (wino_warp): the slab does not hold the "
                               "other views of this frame; warp every view with warp_views, or use "
                               "wino_warp=False to warp views one at a time")
        if self.split:
            ops.warp_views_into([feat], [self.m_norm_cpu[cam]], [self._slot_dst(ws, cam)], split=True,
                                dst_zeroed=ws.slab_zeroed)
        else:
            ops.warp_into(feat, ws.m_norm[cam], self._slot_dst(ws, cam))

    def nonfinite_views(self, device) -> int:
        """Bit s set when slot s's warp has an output pixel with non-finite sample coordinates
        (a NaN in the warped features, e.g. a degenerate homography or a 1-pixel grid side:
        ``mvbev_warp_nonfinite_views``, the warp kernels' own fp32 coordinate code); cached per
        device (geometry only)."""
        key = str(torch.device(device))
        bits = self._nonfinite.get(key)
        if bits is None:
            ms = [None if v is None else self.m_norm_cpu[v] for v in self.slot_views]
            bits = ops.warp_nonfinite_views(ms, self.src_hw, self.grid_hw, device)
            self._nonfinite[key] = bits
        return bits

    def wino_active(self, device) -> bool:
        """The row-Winograd conv1 runs on ``device``: requested (``wino_conv1``) and no view's
        geometry can produce a non-finite warp sample (else the direct conv1 keeps the
        reference's NaN pattern)."""
        return self.wino_conv1 and self.nonfinite_views(device) == 0

    def _wino_warp_applies(self, ws: Workspace, feats, half_ok: bool = False) -> bool:
        """The fused warp + B^T applies: inference (or a training forward whose backward reads T, not the
        slab) over the whole grid, fp32 features (or, ``half_ok``: fp16 ones — config 4; ABI 11900),
        finite geometry."""
        H = self.grid_hw[0]
        dts = (torch.float32, torch.float16) if half_ok else (torch.float32,)
        return (self.wino_warp and (not ws.store_y2 or ws.train_t_only) and ws.y1_rows == (0, H) and ws.slab_zeroed
                and all(f.dtype in dts for f in feats) and len({f.dtype for f in feats}) == 1
                and self.src_hw[1] >= 2 and self.wino_active(ws.slab.device))

    def _check_warp_ws(self, ws: Workspace) -> None:
        if ws.slab_rows != (0, self.grid_hw[0]):
            raise ValueError("a band-local slab (slab_rows) is filled by the band exchange, not by a warp")

    def _train_flag(self, device):
        """The training forwards' non-finite flag and frame tag (one per device, shared by their fresh
        workspaces, so each step needs no flag of its own)."""
        flags = self.__dict__.setdefault("_train_flags", {})
        key = str(torch.device(device))
        if key not in flags:
            from types import SimpleNamespace
            flags[key] = SimpleNamespace(nf=None, nf_tag=0)
        return flags[key]

    def _slab_after_t(self, ws: Workspace, cams) -> None:
        """A slab warp is about to run: after a fused warp (which wrote T, not the slab) only a
        warp of every view leaves the slab holding one frame."""
        if ws.t_from_warp and set(cams) != set(self.slot_of):
            raise RuntimeError("a slab warp of a subset of the views after a fused warp_views (wino_warp): the "
                               "slab's other slots hold an older frame; warp every view")
        ws.t_from_warp = False

    def _warp_views_t(self, ws: Workspace, cams, feats, up_hw=None) -> None:
        """The warp writing conv1's row transform T (``ops.warp_views_wino_rows_into``)."""
        H, W = self.grid_hw
        B = ws.slab.shape[1]
        form = 4 if (not ws.store_y2 and self.wino43_pays(H, B, ws.slab.device)) else 3
        if form == 4:
            need = ops.wino43_rows_bytes(self._conv1_desc(B))
            if ws.wino_t43 is None or ws.wino_t43.numel() * 2 < need:
                ws.wino_t43 = torch.zeros((need + 1) // 2, dtype=torch.bfloat16, device=ws.slab.device)
        else:
            need = ops.wino_rows_bytes(self._conv1_desc(B))
            if ws.wino_t is None or ws.wino_t.numel() * 2 < need:
                ws.wino_t = torch.zeros((need + 1) // 2, dtype=torch.bfloat16, device=ws.slab.device)
        nonfinite = None
        if self.nonfinite_guard:
            # a training forward's workspace is fresh every step: its flag and tag live on the engine (no
            # per-step flag allocation and fill)
            holder = self._train_flag(ws.slab.device) if ws.store_y2 else ws
            if holder.nf is None:
                holder.nf = torch.zeros(1, dtype=torch.int32, device=ws.slab.device)
            if ws.guard_src is None:  # a new frame: a fresh tag (no reset of the flag needed)
                holder.nf_tag = holder.nf_tag % 0x7FFFFFFE + 1
                if holder.nf_tag == 1:
                    holder.nf.zero_()
                ws.guard_src = {}
            ws.nf, ws.nf_tag = holder.nf, holder.nf_tag
            nonfinite = (ws.nf, ws.nf_tag)
            for c, f in zip(cams, feats):  # the frame's views so far (one tag for all its warp calls)
                ws.guard_src[self.slot_of[c]] = (c, f, up_hw)
        ops.warp_views_wino_rows_into(list(feats), [self.m_norm_cpu[c] for c in cams],
                                      ws.wino_t43 if form == 4 else ws.wino_t,
                                      [self.slot_of[c] for c in cams], self.Cs, self.S * self.Cs, H, W,
                                      dst_zeroed=True, up_hw=up_hw, nonfinite=nonfinite,
                                      boxes=self._wino_boxes(ws.slab.device, cams, None if up_hw is None else
                                                             tuple(feats[0].shape[2:]), form=form), form=form)
        ws.t_from_warp = True
        ws.t_form = form

    def _wino_boxes(self, device, cams, backbone_hw=None, form: int = 3) -> torch.Tensor:
        """The fused warps' per-(view, block) staging boxes for these cameras (geometry only, cached):
        ``ops.warp_wino_boxes``; ``backbone_hw``: of the upsample warp's backbone windows; ``form`` 4: of the
        F(4,3) fused warp's blocks."""
        key = ("boxes", str(torch.device(device)), tuple(cams), backbone_hw, form)
        b = self._masks.get(key)
        if b is None:
            b = ops.warp_wino_boxes([self.m_norm_cpu[c] for c in cams], self.src_hw, self.grid_hw, device,
                                    backbone_hw=backbone_hw, form=form)
            self._masks[key] = b
        return b

    def warp_views(self, ws: Workspace, cams: Sequence[int], feats: Sequence[torch.Tensor]) -> None:
        """a5 for several views in one launch (``feats[i]`` is view ``cams[i]``).  With
        ``wino_warp`` (inference, whole grid) a5 + a6 + conv1's row transform in one pass: the
        views land in ``ws.wino_t`` (``mvbev_warp_views_wino_rows``) and the slab is not written."""
        for cam, f in zip(cams, feats):
            if tuple(f.shape[2:]) != self.src_hw or f.shape[1] != self.C:
                raise ValueError(f"view {cam}: features {tuple(f.shape)} do not match "
                                 f"[B,{self.C},{self.src_hw[0]},{self.src_hw[1]}]")
        self._check_warp_ws(ws)
        if self._wino_warp_applies(ws, feats, half_ok=True):
            self._warp_views_t(ws, cams, feats)
            return
        self._slab_after_t(ws, cams)
        ops.warp_views_into(list(feats), [self.m_norm_cpu[c] for c in cams],
                            [self._slot_dst(ws, c) for c in cams], split=self.split,
                            dst_zeroed=self.split and ws.slab_zeroed)

    def warp_views_upsampled(self, ws: Workspace, cams: Sequence[int], feats: Sequence[torch.Tensor]) -> None:
        """a4 + a5 fused: ``feats[i]`` is view ``cams[i]``'s
        backbone-resolution map [B,C,h,w]; the 3x bilinear upsample to ``src_hw``
        (``persp_trans_detector.py:65``) happens inside the warp, never in HBM."""
        for cam, f in zip(cams, feats):
            if f.shape[1] != self.C or f.shape[2] > self.src_hw[0] or f.shape[3] > self.src_hw[1]:
                raise ValueError(f"view {cam}: features {tuple(f.shape)} cannot upsample to {self.src_hw}")
        self._check_warp_ws(ws)
        if self._wino_warp_applies(ws, feats) and all(
                f.shape[3] >= 4 and (f.stride(3) == 1 or ops.is_channels_last_source(f)) for f in feats):
            src = list(feats)
            if self.cl_upsample and self.C % 32 == 0 and not all(ops.is_channels_last_source(f) for f in src):
                src = self._channels_last_maps(ws, src)
            self._warp_views_t(ws, cams, src, up_hw=self.src_hw)  # a4 + a5 + a6 + conv1's B^T in one pass
            return
        self._slab_after_t(ws, cams)
        ops.warp_views_upsampled_into(list(feats), self.src_hw, [self.m_norm_cpu[c] for c in cams],
                                      [self._slot_dst(ws, c) for c in cams], split=self.split,
                                      dst_zeroed=self.split and ws.slab_zeroed)

    def _channels_last_maps(self, ws: Workspace, feats) -> list:
        """The views' backbone maps copied to channels-last buffers of the workspace (one launch)."""
        B, C, h, w = feats[0].shape
        shape = (B, h, w, C)
        if ws.cl_maps is None or len(ws.cl_maps) < len(feats) or tuple(ws.cl_maps[0].shape) != shape:
            ws.cl_maps = [torch.empty(shape, dtype=torch.float32, device=ws.slab.device)
                          for _ in range(max(len(feats), self.num_cam))]
        return ops.to_channels_last_into(list(feats), ws.cl_maps[:len(feats)])

    # -- coord term (a2 folded into conv1) --------------------------------------------------
    def coord_term(self, conv1: torch.nn.Conv2d) -> torch.Tensor:
        """[512, Ho, Wo]: bias + conv(coord channels) for the current conv1 parameters."""
        w, b = conv1.weight, conv1.bias
        key = (w.data_ptr(), w._version, None if b is None else (b.data_ptr(), b._version))
        if key != self._coord_key:  # (ABI 12300: one VALU pass; was an fp32-MFMA conv over a padded coord input)
            self._coord_term = ops.coord_term(w, b, self.coord_c0, self.grid_hw)  # (fresh: in-flight readers)
            self._coord_key = key
        return self._coord_term

    def _sk_ws(self, desc, device) -> Optional[torch.Tensor]:
        """Split-K-tail scratch for a bf16x3 conv (grown once, then reused: the convs of a
        step run in stream order).  ``split_k=False`` keeps whole-tile rounds (bitwise
        reproducible band decompositions)."""
        if self.precision != "bf16x3" or not self.split_k:
            return None
        need = ops.conv3x3_workspace_bytes(desc, self.mid)
        if need == 0:
            return None
        buf = self._sk.get(str(device))
        if buf is None or buf.numel() * 4 < need:
            buf = torch.empty((need + 3) // 4, dtype=torch.float32, device=device)
            self._sk[str(device)] = buf
        return buf

    def conv1_tile_rows(self) -> int:
        """Output rows per tile of the forward conv1 kernel (its mask / order granule)."""
        return _native.conv_tile_rows(_native.LAYOUT_SPLIT_BF16 if self.split else _native.LAYOUT_F16, 1)

    def conv1_mask(self, device, row0: int, rows: int, tile_h: Optional[int] = None) -> Optional[torch.Tensor]:
        """Per conv1 output tile (``tile_h`` rows: default the forward conv1's tile) of rows
        [row0, row0+rows): bit s = slot s can be non-zero in the tile's 3x3 halo
        (``mvbev_warp_tile_mask``); None when not used."""
        if not self.frustum:
            return None
        tile_h = self.conv1_tile_rows() if tile_h is None else int(tile_h)
        key = (str(device), row0, rows, tile_h)
        m = self._masks.get(key)
        if m is None:
            ms = [None if v is None else self.m_norm_cpu[v] for v in self.slot_views]
            m = ops.warp_tile_mask(ms, self.src_hw, self.grid_hw, row0, rows, 1, device, tile_h=tile_h)
            self._masks[key] = m
        return m

    def conv1_fwd_mask(self, device, row0: int, rows: int) -> Tuple[Optional[torch.Tensor], int]:
        """(mask, tile space) of the forward conv1 over rows [row0, row0+rows): the edge-strip
        space (``ops.ring_tile_mask``) where it applies, else the 12 x 32 grid of ``conv1_mask``."""
        if not (self.frustum and self.split and self.edge_strip):
            return self.conv1_mask(device, row0, rows), _native.TILES_GRID
        key = ("fwd", str(device), row0, rows)
        r = self._masks.get(key)
        if r is None:
            ms = [None if v is None else self.m_norm_cpu[v] for v in self.slot_views]
            m = ops.ring_tile_mask(ms, self.src_hw, self.grid_hw, row0, rows, device, _native.TILES_EDGE_STRIP)
            r = (m, _native.TILES_EDGE_STRIP) if m is not None else (self.conv1_mask(device, row0, rows),
                                                                     _native.TILES_GRID)
            self._masks[key] = r
        return r

    def conv1_order(self, device, row0: int, rows: int, B: int, grid: bool = False,
                    tile_h: Optional[int] = None) -> Optional[torch.Tensor]:
        """Heavy-first run order of the forward conv1's pixel tiles (``grid``: of the 12 x 32
        grid even where the forward uses edge strips; ``tile_h``: of the ``tile_h`` x 32 grid)."""
        key = ("order", str(device), row0, rows, B, grid, tile_h)
        o = self._masks.get(key)
        if o is None:
            m = (self.conv1_mask(device, row0, rows, tile_h=tile_h) if grid or tile_h
                 else self.conv1_fwd_mask(device, row0, rows)[0])
            if m is None:
                return None
            o = ops.heavy_first_order(m, B)
            self._masks[key] = o
        return o

    def conv1_active_fraction(self, device, row0: int, rows: int, grid: bool = False,
                              tile_h: Optional[int] = None) -> float:
        """Fraction of conv1's dense (pixel, slot) work the forward's frustum mask keeps (1.0 =
        dense): per tile its enabled slots x its pixels inside the grid.  ``grid``: over the
        12 x 32 grid tiles (the row-Winograd conv1's tile space) instead of the forward's;
        ``tile_h``: over the ``tile_h`` x 32 grid (16: F(4,3)'s)."""
        if tile_h:
            m = self.conv1_mask(device, row0, rows, tile_h=tile_h)
            if m is None:
                return 1.0
            W, S, th = self.grid_hw[1], self.S, int(tile_h)
            tx = -(-W // 32)
            bits = [bin(int(v) & 0xFFFFFFFF).count("1") for v in m.cpu().tolist()]
            return sum(bb * min(th, rows - (t // tx) * th) * min(32, W - (t % tx) * 32)
                       for t, bb in enumerate(bits[:tx * -(-rows // th)])) / (rows * W * S)
        m, space = ((self.conv1_mask(device, row0, rows), _native.TILES_GRID) if grid
                    else self.conv1_fwd_mask(device, row0, rows))
        if m is None:
            return 1.0
        W = self.grid_hw[1]
        d = ops.conv_desc(1, 8, self.grid_hw[0], W, group=8, group_stride=0, batch_stride=0, in_row0=row0,
                          in_rows=rows, out_row0=row0, out_rows=rows)
        tiles_x, tiles_y, edge_tiles, ew, edge_rows = _native.ring_tile_space(d, space)
        th, tw = self.conv1_tile_rows(), _native.TILE_W
        pix = [min(th, rows - (t // tiles_x) * th) * min(tw, W - (t % tiles_x) * tw) for t in range(tiles_x * tiles_y)]
        pix += [min(edge_rows, rows - e * edge_rows) * (W - tiles_x * tw) for e in range(edge_tiles)]
        bits = [bin(int(v) & 0xFFFFFFFF).count("1") for v in m.cpu().tolist()]
        return sum(b * p for b, p in zip(bits, pix)) / (rows * W * self.S)

    # -- a7-a9 ----------------------------------------------------------------------------
    def conv1(self, ws: Workspace, conv1: torch.nn.Conv2d, mark=None) -> torch.Tensor:
        """a7: y1 = relu(conv3x3(slab) + coord_term) on y1's rows (row-Winograd where
        ``wino_active`` and inference, else the direct ring conv)."""
        if conv1.weight.shape[1] != self.cin:
            raise ValueError(f"conv1 has {conv1.weight.shape[1]} input channels, expected {self.cin}")
        H, W = self.grid_hw
        B = ws.slab.shape[1]
        init = self.coord_term(conv1)
        a1, b1 = ws.y1_rows
        s0, s1 = ws.slab_rows
        R = s1 - s0
        d1 = ops.conv_desc(B, self.S * self.Cs, H, W, group=self.Cs, group_stride=B * self.Cs * R * W,
                           batch_stride=self.Cs * R * W, in_row0=s0, in_rows=R, out_row0=a1, out_rows=b1 - a1)
        if self.wino_active(ws.slab.device):  # inference, and the training forward (round 4)
            return self.conv1_wino(ws, conv1, d1, init, mark=mark)
        if ws.t_from_warp:
            raise RuntimeError("the direct conv1 reads the slab, but the fused warp wrote conv1's row transform")
        p1 = self.pack1.get(conv1.weight)
        gm, space = self.conv1_fwd_mask(ws.slab.device, a1, b1 - a1)
        return ops.conv3x3_desc(ws.slab, d1, p1, self.mid, bias=None, init=init, dilation=1, relu=True,
                                out=ws.y1, workspace=None if gm is not None else self._sk_ws(d1, ws.slab.device),
                                group_mask=gm, tile_order=self.conv1_order(ws.slab.device, a1, b1 - a1, B,
                                                                           grid=space == _native.TILES_GRID),
                                tile_space=space)

    def _conv1_desc(self, B: int, rows: Optional[Tuple[int, int]] = None):
        H, W = self.grid_hw
        a1, b1 = (0, H) if rows is None else rows
        return ops.conv_desc(B, self.S * self.Cs, H, W, group=self.Cs, group_stride=B * self.Cs * H * W,
                             batch_stride=self.Cs * H * W, in_row0=0, in_rows=H, out_row0=a1, out_rows=b1 - a1)

    def conv1_wino(self, ws: Workspace, conv1: torch.nn.Conv2d, d1, init: torch.Tensor, mark=None) -> torch.Tensor:
        """a7 as F(3,3) row-Winograd: T = B^T(slab rows) (``ops.wino_rows``), then the conv from T
        with the G w weights (``ops.conv3x3_wino``); same y1 as ``conv1`` within the 3xbf16 error."""
        a1, b1 = ws.y1_rows
        B = ws.slab.shape[1]
        if self.conv1_form(ws) == 4:  # F(4,3): T43 (from the fused warp, else of the slab) over 16 x 32 tiles
            th = ops.WINO43_TILE_ROWS
            gm = self.conv1_mask(ws.slab.device, a1, b1 - a1, tile_h=th)
            need = ops.wino43_rows_bytes(d1)
            if ws.wino_t43 is None or ws.wino_t43.numel() * 2 < need:
                ws.wino_t43 = torch.zeros((need + 1) // 2, dtype=torch.bfloat16, device=ws.slab.device)
            if not ws.t_from_warp:
                ops.wino43_rows(ws.slab, d1, ws.wino_t43, gm)
            ws.t1_valid = False  # (T43 is not the training backward's T)
            if mark:
                mark("conv1_wino")
            return ops.conv3x3_wino43(ws.wino_t43, d1, self.pack1w43.get(conv1.weight), self.mid, init=init,
                                      relu=True, out=ws.y1, group_mask=gm,
                                      tile_order=self.conv1_order(ws.slab.device, a1, b1 - a1, B, grid=True,
                                                                  tile_h=th))
        gm = self.conv1_mask(ws.slab.device, a1, b1 - a1)
        need = ops.wino_rows_bytes(d1)
        if ws.wino_t is None or ws.wino_t.numel() * 2 < need:
            ws.wino_t = torch.zeros((need + 1) // 2, dtype=torch.bfloat16, device=ws.slab.device)
        if not ws.t_from_warp:  # the slab's transform (else the fused warp wrote T)
            ops.wino_rows(ws.slab, d1, ws.wino_t, gm)
        ws.t1_valid = (a1, b1) == (0, self.grid_hw[0])
        if mark:
            mark("conv1_wino")  # between the transform and the conv (bench.py's stage events)
        return ops.conv3x3_wino(ws.wino_t, d1, self.pack1w.get(conv1.weight), self.mid, init=init, relu=True,
                                out=ws.y1, group_mask=gm,
                                tile_order=self.conv1_order(ws.slab.device, a1, b1 - a1, B, grid=True))

    def conv1_form(self, ws: Workspace) -> int:
        """The row-Winograd form of ``conv1_wino`` on this workspace: the fused warp's (``ws.t_form``), else 4 for
        an inference forward over the whole grid where ``wino43_pays``, else 3."""
        if ws.t_from_warp:
            return ws.t_form
        a1, b1 = ws.y1_rows
        return 4 if (not ws.store_y2 and (a1, b1) == (0, self.grid_hw[0])
                     and self.wino43_pays(b1 - a1, ws.slab.shape[1], ws.slab.device)) else 3

    def conv2_form(self, ws: Workspace) -> int:
        """The row-Winograd form of ``conv2_partials`` (0: not row-Winograd)."""
        if not self.wino_conv2_active(ws):
            return 0
        (a2, b2) = ws.y2_rows
        return 4 if self.wino43_pays(b2 - a2, ws.y1.shape[0], ws.y1.device, deep=True) else 3

    def conv2(self, ws: Workspace, conv2: torch.nn.Conv2d) -> torch.Tensor:
        """a8: y2 = relu(conv3x3_d2(y1) + b2) on y2's rows (row-Winograd where ``wino_conv2_active``:
        the training forward, which keeps y2 for conv3's backward)."""
        H, W = self.grid_hw
        (a1, b1), (a2, b2) = ws.y1_rows, ws.y2_rows
        B = ws.y1.shape[0]
        d2 = ops.conv_desc(B, self.mid, H, W, group=self.mid, group_stride=0,
                           batch_stride=self.mid * (b1 - a1) * W, in_row0=a1, in_rows=b1 - a1,
                           out_row0=a2, out_rows=b2 - a2)
        if self.wino_conv2_active(ws):
            tneed = ops.wino_rows_bytes(d2)
            if ws.wino_t2 is None or ws.wino_t2.numel() * 2 < tneed:
                ws.wino_t2 = torch.zeros((tneed + 1) // 2, dtype=torch.bfloat16, device=ws.y1.device)
            ops.wino_rows(ws.y1, d2, ws.wino_t2, dilation=2)
            ws.t2_valid = (a1, b1) == (a2, b2) == (0, H)  # the backward's conv2 weight gradient reads it
            return ops.conv3x3_wino_dil(ws.wino_t2, d2, self.pack2w.get(conv2.weight), self.mid, 2, bias=conv2.bias,
                                        relu=True, out=ws.y2)
        p2 = self.pack2.get(conv2.weight)
        return ops.conv3x3_desc(ws.y1, d2, p2, self.mid, bias=conv2.bias, dilation=2, relu=True, out=ws.y2,
                                workspace=self._sk_ws(d2, ws.y1.device))

    def _conv2_desc(self, ws: Workspace):
        H, W = self.grid_hw
        (a1, b1), (a2, b2) = ws.y1_rows, ws.y2_rows
        B = ws.y1.shape[0]
        return ops.conv_desc(B, self.mid, H, W, group=self.mid, group_stride=0,
                             batch_stride=self.mid * (b1 - a1) * W, in_row0=a1, in_rows=b1 - a1,
                             out_row0=a2, out_rows=b2 - a2)

    def conv3_fused_applies(self, ws: Workspace) -> bool:
        """conv2 -> conv3 without y2 in HBM: split-bf16 y1 (the ring conv) and fuse_conv3."""
        return self.fuse_conv3 and ws.y1.dtype == torch.bfloat16 and not ws.store_y2

    def conv2_partials(self, ws: Workspace, conv2: torch.nn.Conv2d, conv3: torch.nn.Conv2d) -> None:
        """a8 + the first half of a9: relu(conv3x3_d2(y1) + b2) never leaves the conv's
        registers; its epilogue writes conv3's per-(channel set, tap, pixel) partials."""
        d2 = self._conv2_desc(ws)
        need = ops.conv3x3_cout1_partials_bytes(d2, self.mid)
        if ws.p3 is None or ws.p3.numel() * 4 < need:
            ws.p3 = torch.empty((need + 3) // 4, dtype=torch.float32, device=ws.y1.device)
        if self.conv2_form(ws) == 4:
            tneed = ops.wino43_rows_bytes(d2)  # F(4,3) (ABI 12400)
            if ws.wino_t2_43 is None or ws.wino_t2_43.numel() * 2 < tneed:
                ws.wino_t2_43 = torch.zeros((tneed + 1) // 2, dtype=torch.bfloat16, device=ws.y1.device)
            ops.wino43_rows(ws.y1, d2, ws.wino_t2_43, dilation=2)
            ops.conv3x3_wino43_then_cout1_partials(ws.wino_t2_43, d2, self.pack2w43.get(conv2.weight), self.mid,
                                                   conv2.bias, True, conv3.weight, ws.p3)
            return
        if self.wino_conv2_active(ws):
            tneed = ops.wino_rows_bytes(d2)
            if ws.wino_t2 is None or ws.wino_t2.numel() * 2 < tneed:
                ws.wino_t2 = torch.zeros((tneed + 1) // 2, dtype=torch.bfloat16, device=ws.y1.device)
            ops.wino_rows(ws.y1, d2, ws.wino_t2, dilation=2)
            ops.conv3x3_wino_then_cout1_partials(ws.wino_t2, d2, self.pack2w.get(conv2.weight), self.mid,
                                                 conv2.bias, 2, True, conv3.weight, ws.p3)
            return
        ops.conv3x3_then_cout1_partials(ws.y1, d2, self.pack2.get(conv2.weight), self.mid, conv2.bias, 2, True,
                                        conv3.weight, ws.p3)

    def wino_conv2_active(self, ws: Workspace) -> bool:
        """conv2 -> conv3 partials run row-Winograd: requested (``wino_conv2``), y1 split-bf16 and no
        view's geometry can make y1 non-finite (as ``wino_active`` for conv1)."""
        return (self.wino_conv2 and ws.y1.dtype == torch.bfloat16
                and self.nonfinite_views(ws.y1.device) == 0)

    def conv3_from_partials(self, ws: Workspace, conv3: torch.nn.Conv2d) -> torch.Tensor:
        """The rest of a9: map rows ``ws.band`` from the partials (fixed summation order)."""
        r0, r1 = ws.band
        return ops.cout1_from_partials(ws.p3, self._conv2_desc(ws), self.mid, 4, r0, r1 - r0)

    def conv3(self, ws: Workspace, conv3: torch.nn.Conv2d) -> torch.Tensor:
        """a9: map = conv3x3_d4(y2) (Cout 1, no bias) on the output band → [B,1,rows,Wo]."""
        H = self.grid_hw[0]
        r0, r1 = ws.band
        return ops.conv3x3_cout1(ws.y2, conv3.weight, 4, H=H, in_row0=ws.y2_rows[0], out_row0=r0,
                                 out_rows=r1 - r0)

    # -- partial-sum multi-GPU (SURVEY §8(e) alternative, §8(f) row 3) -----------------------
    def conv1_partial(self, ws: Workspace, map_classifier: torch.nn.Sequential, out: torch.Tensor,
                      mark=None, band_rows: int = 0) -> torch.Tensor:
        """conv1 restricted to this engine's views (its slice of conv1's input channels), all grid
        rows, no bias / coord term / ReLU: one rank's term of conv1's channel sum (row-Winograd
        where ``wino_active``; from the fused warp's T when ``warp_views`` wrote it, else from the
        slab).  ``out``: contiguous fp32 [B, 512, Ho, Wo], or with ``band_rows`` > 0 the
        reduce-scatter's band-major [bands, B, 512, band_rows, Wo] (written in place)."""
        if ws.slab_rows != (0, self.grid_hw[0]):
            raise ValueError("conv1_partial needs a whole-grid slab")
        H, W = self.grid_hw
        B = ws.slab.shape[1]
        d1 = ops.conv_desc(B, self.S * self.Cs, H, W, group=self.Cs, group_stride=B * self.Cs * H * W,
                           batch_stride=self.Cs * H * W, in_row0=0, in_rows=H, out_row0=0, out_rows=H)
        gm = self.conv1_mask(ws.slab.device, 0, H)  # no ReLU: the grid tiles (edge strips are conv1+ReLU only)
        order = self.conv1_order(ws.slab.device, 0, H, B, grid=True)
        w1 = map_classifier[0].weight
        if ws.t_from_warp and ws.t_form != 3:
            raise RuntimeError("conv1_partial reads F(3,3)'s T: this engine's fused warp wrote T43 (wino43)")
        if self.wino_active(ws.slab.device):
            need = ops.wino_rows_bytes(d1)
            if ws.wino_t is None or ws.wino_t.numel() * 2 < need:
                ws.wino_t = torch.zeros((need + 1) // 2, dtype=torch.bfloat16, device=ws.slab.device)
            if not ws.t_from_warp:  # else the fused warp wrote T (no slab, no transform)
                ops.wino_rows(ws.slab, d1, ws.wino_t, gm)
            if mark:
                mark("conv1_wino")
            ops.conv3x3_wino(ws.wino_t, d1, self.pack1w.get(w1), self.mid, init=None, relu=False, out=out,
                             group_mask=gm, tile_order=order, band_rows=band_rows)
            if ws.t_from_warp and ws.guard_src is not None:
                self._partial_exact(ws, w1, out, band_rows)
                ws.guard_src = None  # the frame's produce step ends here
            return out
        if ws.t_from_warp:
            raise RuntimeError("the direct conv1 reads the slab, but the fused warp wrote conv1's row transform")
        full = out if not band_rows else torch.empty((B, self.mid, H, W), dtype=torch.float32, device=out.device)
        ops.conv3x3_desc(ws.slab, d1, self.pack1.get(w1), self.mid, bias=None, init=None, dilation=1,
                         relu=False, out=full, workspace=None if gm is not None else self._sk_ws(d1, ws.slab.device),
                         group_mask=gm, tile_order=order)
        if band_rows:  # the direct conv has no banded epilogue: copy the bands
            for p in range(-(-H // band_rows)):
                a, b = p * band_rows, min(H, (p + 1) * band_rows)
                out[p, :, :, :b - a].copy_(full[:, :, a:b])
        return out

    def _partial_exact(self, ws: Workspace, w1: torch.Tensor, out: torch.Tensor, band_rows: int) -> None:
        """The non-finite guard of ``conv1_partial``, gated on the fused warp's report: the reference-order
        warp of this engine's views into the exact path's fp32 slab and the fp32-MFMA conv1 over their
        channels (exact products, no bias / ReLU) over the partial sums — in row bands of bounded memory,
        written in ``out``'s layout (band-major with ``band_rows``).  Summed over the ranks, the partials
        then carry the reference's NaN / inf pattern (``finish_from_y1`` checks the sum)."""
        H, W = self.grid_hw
        B, dev = ws.slab.shape[1], ws.slab.device
        gate = (ws.nf, ws.nf_tag)
        p1, _ = self._exact_packs()
        chunks = self._guard_chunks(B, 0, H)
        self._guard_buffers(ws, B, max(b - a for a, b in chunks), dev)
        banded = out.view(1, B, self.mid, H, W) if not band_rows else out
        for a, b in chunks:
            s0, s1 = max(0, a - HALO_CONV1), min(H, b + HALO_CONV1)
            x = self._exact_warp_rows(ws, B, s0, s1, gate)
            d1 = ops.conv_desc(B, self.S * self.Cs, H, W, group=self.Cs, group_stride=B * self.Cs * (s1 - s0) * W,
                               batch_stride=self.Cs * (s1 - s0) * W, in_row0=s0, in_rows=s1 - s0, out_row0=a,
                               out_rows=b - a)
            ops.conv3x3_desc(x, d1, p1.get(w1), self.mid, dilation=1, relu=False, out=banded, gate=gate,
                             band_rows=band_rows or H)

    def finish_from_y1(self, ws: Workspace, map_classifier: torch.nn.Sequential, mark=None) -> torch.Tensor:
        """``ws.y1`` holds conv1's summed channel terms (no bias) for rows ``ws.y1_rows``:
        add the coord term (+ bias), ReLU, then conv2 and conv3 on the band.  With the non-finite guard
        the add + ReLU kernel reports a non-finite y1 (the sum of the ranks' exact partials carries the
        reference's NaN / inf pattern), and a gated fp32-MFMA conv2 (exact products) then rewrites y2
        before conv3 reads it."""
        a1, b1 = ws.y1_rows
        init = self.coord_term(map_classifier[0])
        flag = None
        if self.nonfinite_guard and ws.y1.dtype == torch.float32:
            if ws.nf2 is None:
                ws.nf2 = torch.zeros(1, dtype=torch.int32, device=ws.y1.device)
            ws.nf2_tag = ws.nf2_tag % 0x7FFFFFFE + 1
            if ws.nf2_tag == 1:
                ws.nf2.zero_()
            flag = (ws.nf2, ws.nf2_tag)
        if ws.y1.dtype == torch.float32:
            ops.bias_relu_nonfinite_(ws.y1, init, a1, relu=True, flag=flag)
        else:
            ws.y1.add_(init[:, a1:b1]).relu_()
        if mark:
            mark("conv2")
        self.conv2(ws, map_classifier[2])
        if flag is not None:  # y1 non-finite: the exact conv2 (the fast one splits inf into NaN)
            (a2, b2), H, W = ws.y2_rows, self.grid_hw[0], self.grid_hw[1]
            B = ws.y1.shape[0]
            d2 = ops.conv_desc(B, self.mid, H, W, group=self.mid, group_stride=0, batch_stride=self.mid * (b1 - a1) * W,
                               in_row0=a1, in_rows=b1 - a1, out_row0=a2, out_rows=b2 - a2)
            ops.conv3x3_desc(ws.y1, d2, self._exact_packs()[1].get(map_classifier[2].weight), self.mid,
                             bias=map_classifier[2].bias, dilation=2, relu=True, out=ws.y2, gate=flag)
        if mark:
            mark("conv3")
        return self.conv3(ws, map_classifier[4])

    # -- the band exchange / slab all-gather (parallel.ViewBands, ViewParallel) ---------------
    def window_buffer(self, n: int, B: int, rows: int, device) -> torch.Tensor:
        """``n`` zero-filled view windows of ``rows`` grid rows in the slab's layout (the exchange's send
        chunks): [n, *split_shape(B, Cs, rows, Wo)] bf16 (4 bytes per element, as fp32)."""
        W = self.grid_hw[1]
        if self.split:
            return torch.zeros((n,) + ops.split_shape(B, self.Cs, rows, W), dtype=torch.bfloat16, device=device)
        return torch.zeros((n, B, self.Cs, rows, W), dtype=self.slab_dtype, device=device)

    def warp_windows(self, dsts: Sequence[torch.Tensor], cams: Sequence[int], feats: Sequence[torch.Tensor],
                     row0s: Sequence[int], nonfinite=None) -> None:
        """a5 of ``cams[i]`` (features ``feats[i]``) for the row window of ``dsts[i]`` (``window_buffer``
        entries, zero-filled and only written by this warp) from grid row ``row0s[i]`` — the exchange's
        send chunks written straight by the warp (no whole-grid slab, no window copies), 16 per launch.
        ``nonfinite``: (flag, tag) — the non-finite report.  A non-split engine (``precision="fp32"``: fp32
        windows) warps its windows in the reference's own evaluation order (``mvbev_warp_views_exact_rows``,
        ungated; ADVICE r05: the band exchange under fp32 precision) and has no non-finite report (its convs
        take exact fp32 products already)."""
        H = self.grid_hw[0]
        if not self.split:
            if self.slab_dtype != torch.float32:
                raise ValueError("window warps write split-bf16 or fp32 windows (an fp16 slab is not supported)")
            for i in range(0, len(dsts), 16):
                sl = slice(i, i + 16)
                ops.warp_views_exact_into(list(feats[sl]), [self.m_norm_cpu[c] for c in cams[sl]],
                                          [d[:, :self.C] for d in dsts[sl]], row0s=list(row0s[sl]), grid_rows=H)
            return
        for i in range(0, len(dsts), 16):
            sl = slice(i, i + 16)
            ops.warp_views_split_rows_into(list(feats[sl]), [self.m_norm_cpu[c] for c in cams[sl]], list(dsts[sl]),
                                           list(row0s[sl]), H, dst_zeroed=True, nonfinite=nonfinite)

    def guard_windows(self) -> bool:
        """The exchange modes can run the exact path on exchanged fp32 windows: the non-finite guard is on
        and a window's channel planes are exactly the slab slot (Cs == C: no padding planes)."""
        return self.nonfinite_guard and self.split and self.Cs == self.C

    def warp_windows_exact(self, dsts: Sequence[torch.Tensor], cams: Sequence[int], feats: Sequence[torch.Tensor],
                           row0s: Sequence[int], gate) -> None:
        """The reference-order warp of the same windows as ``warp_windows``, gated on ``gate``, written as
        fp32 [B, C, rows, Wo] over the same bytes of each ``dsts[i]`` (the exact path's exchange payload)."""
        H = self.grid_hw[0]
        B = feats[0].shape[0]
        for i in range(0, len(dsts), 16):
            sl = slice(i, i + 16)
            xs = [d.view(-1).view(torch.float32).view(B, self.C, d.shape[2], self.grid_hw[1]) for d in dsts[sl]]
            ops.warp_views_exact_into(list(feats[sl]), [self.m_norm_cpu[c] for c in cams[sl]], xs, gate=gate,
                                      row0s=list(row0s[sl]), grid_rows=H)

    def clear_windows(self, buf: torch.Tensor, gate) -> None:
        """Re-zero ``buf`` (window chunks or a slab) when ``gate`` fired: the exact path wrote fp32 over
        bytes the window warps skip (out-of-source pixels of a zero-filled buffer)."""
        ops.zero_gated_(buf, gate)

    def fuse_exact_from_windows(self, ws: Workspace, map_classifier, out: torch.Tensor, gate) -> None:
        """The exact path on a slab whose bytes hold fp32 windows (``warp_windows_exact`` exchanged into
        ``ws.slab``, rows ``ws.slab_rows``): the fp32-MFMA convs for ``ws.band`` into ``out``, gated."""
        B = ws.slab.shape[1]
        s0, s1 = ws.slab_rows
        x = ws.slab.view(-1).view(torch.float32).view(self.S, B, self.Cs, s1 - s0, self.grid_hw[1])
        r0, r1 = ws.band
        self._guard_buffers(ws, B, r1 - r0, ws.slab.device, slab=False)
        self._exact_convs(ws, map_classifier, out, gate, x, (s0, s1), r0, r1, r0)

    def fuse(self, ws: Workspace, map_classifier: torch.nn.Sequential, mark=None) -> torch.Tensor:
        """a7-a9 on ``ws.slab`` for the output rows ``ws.band`` → [B, 1, rows, Wo].

        ``mark(stage)`` (optional) is called right before each conv is enqueued
        (``bench.py`` records HIP events there)."""
        if self.conv3_fused_applies(ws):
            if mark:
                mark("conv1")
            self.conv1(ws, map_classifier[0], mark=mark)
            if mark:
                mark("conv2")
            self.conv2_partials(ws, map_classifier[2], map_classifier[4])
            if mark:
                mark("conv3")
            out = self.conv3_from_partials(ws, map_classifier[4])
            if ws.t_from_warp and ws.guard_src is not None:
                if mark:
                    mark("guard")
                self._nonfinite_exact(ws, map_classifier, out, (ws.nf, ws.nf_tag))
                ws.guard_src = None  # the frame ends here
            return out
        for stage, idx, fn in (("conv1", 0, self.conv1), ("conv2", 2, self.conv2), ("conv3", 4, self.conv3)):
            if mark:
                mark(stage)
            out = fn(ws, map_classifier[idx])
        if ws.store_y2 and ws.t_from_warp and ws.guard_src is not None:
            # the training forward (round 6, VERDICT r05 missing 2): the same gated exact path, which also puts
            # its activations where the native backward reads them
            if mark:
                mark("guard")
            self._train_exact(ws, map_classifier, out, (ws.nf, ws.nf_tag))
            ws.guard_src = None  # the frame ends here (no workspace left in an in-flight guard state)
        return out

    def _exact_packs(self):
        if self._pack1f is None:
            self._pack1f = ops.PackedConv3x3(self._chan_map, "fp32")
            self._pack2f = ops.PackedConv3x3(None, "fp32")
        return self._pack1f, self._pack2f

    def _guard_chunks(self, B: int, r0: int, r1: int) -> List[Tuple[int, int]]:
        """Output row chunks of [r0, r1) whose exact-path slab window (rows + 14) fits ``guard_bytes``."""
        per_row = self.S * B * self.Cs * self.grid_hw[1] * 4
        n = max(12, self.guard_bytes // max(1, per_row) - 2 * 7)
        return [(a, min(r1, a + n)) for a in range(r0, r1, n)]

    def _guard_buffers(self, ws: Workspace, B: int, rows: int, dev, slab: bool = True) -> None:
        W = self.grid_hw[1]
        need = (self.S * B * self.Cs * (rows + 14) * W, B * self.mid * (rows + 12) * W, B * self.mid * (rows + 8) * W)
        if slab and (ws.g_slab is None or ws.g_slab.numel() < need[0]):
            # zero-filled once: the padding channels (Cs > C) stay 0, the warp writes the C real ones
            ws.g_slab = torch.zeros(need[0], dtype=torch.float32, device=dev)
        if ws.g_y1 is None or ws.g_y1.numel() < need[1]:
            ws.g_y1 = torch.empty(need[1], dtype=torch.float32, device=dev)
        if ws.g_y2 is None or ws.g_y2.numel() < need[2]:
            ws.g_y2 = torch.empty(need[2], dtype=torch.float32, device=dev)

    def _exact_convs(self, ws: Workspace, map_classifier, out: torch.Tensor, gate, x: torch.Tensor,
                     x_rows: Tuple[int, int], r0: int, r1: int, out_row0: int, packed=None) -> None:
        """conv1 + coord term + ReLU, conv2 + ReLU and conv3 on the fp32-MFMA kernels (exact products, torch's
        NaN-preserving ReLU) for map rows [r0, r1), every launch gated on ``gate``: ``x`` is the fp32 slab
        [S, B, Cs, rows, Wo] holding grid rows ``x_rows``; ``out`` [B, 1, rows, Wo] holds map rows from
        ``out_row0``.  ``packed``: (conv1, conv2) fp32 packs to use (default: the cached ones)."""
        H, W = self.grid_hw
        B = out.shape[0]
        c1, c2, c3 = map_classifier[0], map_classifier[2], map_classifier[4]
        if packed is None:
            e1, e2 = self._exact_packs()
            packed = (e1.get(c1.weight), e2.get(c2.weight))
        (a1, b1), (a2, b2) = band_rows(r0, r1, H)
        s0, s1 = x_rows
        R = s1 - s0
        y1 = ws.g_y1[:B * self.mid * (b1 - a1) * W].view(B, self.mid, b1 - a1, W)
        y2 = ws.g_y2[:B * self.mid * (b2 - a2) * W].view(B, self.mid, b2 - a2, W)
        d1 = ops.conv_desc(B, self.S * self.Cs, H, W, group=self.Cs, group_stride=B * self.Cs * R * W,
                           batch_stride=self.Cs * R * W, in_row0=s0, in_rows=R, out_row0=a1, out_rows=b1 - a1)
        ops.conv3x3_desc(x, d1, packed[0], self.mid, init=self.coord_term(c1), dilation=1, relu=True,
                         out=y1, gate=gate)
        d2 = ops.conv_desc(B, self.mid, H, W, group=self.mid, group_stride=0, batch_stride=self.mid * (b1 - a1) * W,
                           in_row0=a1, in_rows=b1 - a1, out_row0=a2, out_rows=b2 - a2)
        ops.conv3x3_desc(y1, d2, packed[1], self.mid, bias=c2.bias, dilation=2, relu=True, out=y2, gate=gate)
        if B == 1 or (r0 == out_row0 and r1 - r0 == out.shape[2]):
            ops.conv3x3_cout1(y2, c3.weight, 4, H=H, in_row0=a2, out_row0=r0, out_rows=r1 - r0,
                              out=out[:, :, r0 - out_row0:r1 - out_row0], gate=gate)
        else:  # a row chunk of B > 1 maps is not contiguous: one launch per item
            for b in range(B):
                ops.conv3x3_cout1(y2[b:b + 1], c3.weight, 4, H=H, in_row0=a2, out_row0=r0, out_rows=r1 - r0,
                                  out=out[b:b + 1, :, r0 - out_row0:r1 - out_row0], gate=gate)

    def _exact_warp_rows(self, ws: Workspace, B: int, s0: int, s1: int, gate) -> torch.Tensor:
        """The reference-order warp (+ upsample) of the frame's views (``ws.guard_src``) into the exact
        path's fp32 slab for grid rows [s0, s1), gated; returns the slab [S, B, Cs, s1 - s0, Wo]."""
        H, W = self.grid_hw
        x = ws.g_slab[:self.S * B * self.Cs * (s1 - s0) * W].view(self.S, B, self.Cs, s1 - s0, W)
        if self.Cs != self.C:  # padding channels meet zero weights: keep them 0 (the buffer is reused at other shapes)
            x[:, :, self.C:].zero_()
        groups = {}
        for slot, (cam, feat, up_hw) in ws.guard_src.items():
            groups.setdefault((up_hw, feat.dtype, tuple(feat.shape)), []).append((slot, cam, feat))
        for (up_hw, _, _), items in groups.items():
            for i in range(0, len(items), 16):
                part = items[i:i + 16]
                ops.warp_views_exact_into([f for _, _, f in part], [self.m_norm_cpu[c] for _, c, _ in part],
                                          [x[slot, :, :self.C] for slot, _, _ in part], up_hw=up_hw, gate=gate,
                                          row0s=[s0] * len(part), grid_rows=H)
        return x

    def _nonfinite_exact(self, ws: Workspace, map_classifier, out: torch.Tensor, gate) -> None:
        """The non-finite guard's exact path (``nonfinite_guard``), every launch gated on the fused warp's
        report ``gate`` = (flag, tag): the reference-order warp (+ upsample) of the same features into an
        fp32 slab (``:65-69``), the fp32-MFMA conv1 + coord term + ReLU (``:51``), conv2 + ReLU (``:53``) and
        conv3 (``:54``) into ``out`` — the map the fast path just wrote.  In row bands of at most
        ``guard_bytes`` of slab (each band's convs read its rows +- 7)."""
        H, W = self.grid_hw
        B, dev = ws.slab.shape[1], ws.slab.device
        r0, r1 = ws.band
        chunks = self._guard_chunks(B, r0, r1)
        self._guard_buffers(ws, B, max(b - a for a, b in chunks), dev)
        for a, b in chunks:
            (a1, b1), _ = band_rows(a, b, H)
            s0, s1 = max(0, a1 - HALO_CONV1), min(H, b1 + HALO_CONV1)
            x = self._exact_warp_rows(ws, B, s0, s1, gate)
            self._exact_convs(ws, map_classifier, out, gate, x, (s0, s1), a, b, r0)

    def _train_exact(self, ws: Workspace, map_classifier, out: torch.Tensor, gate) -> None:
        """The training forward's non-finite guard (round 6), every launch gated on the fused warp's report:
        ``_nonfinite_exact``'s reference-order warp and fp32-MFMA convs rewrite the map, and the exact
        activations are stored where the native backward (``autograd.ProjectFuseFunction``) reads them — y2
        (fp32), y1 (split-bf16, a non-finite value kept whole in hi: the ReLU masks are torch's), conv1's input
        (the pooled split slab) and, from those, conv1's and conv2's row-Winograd transforms T / T2 (the weight
        gradients' operands) — so the backward differentiates the reference's forward values, NaN / inf
        included (``persp_trans_detector.py:65-81`` under ``trainer.py:38-47``).  The exact fp32 weights are
        re-packed every step, gated (the optimizer changes them; a skipped pack is never cached)."""
        H, W = self.grid_hw
        B, dev = ws.slab.shape[1], ws.slab.device
        c1, c2 = map_classifier[0], map_classifier[2]
        if getattr(self, "_gpacks", None) is None:
            self._gpacks = (ops.PackedConv3x3(self._chan_map, "fp32"), ops.PackedConv3x3(None, "fp32"))
        packed = (self._gpacks[0].get_gated(c1.weight, gate), self._gpacks[1].get_gated(c2.weight, gate))
        chunks = self._guard_chunks(B, 0, H)
        # the exact path's fp32 buffers live on the engine (a training workspace is fresh every step: per-step
        # buffers would zero-fill ~0.7 GB of slab each step at cfg2); stream order keeps steps apart
        bufs = self.__dict__.setdefault("_train_guard_bufs", {})
        key = (str(dev), B)
        if key in bufs:
            ws.g_slab, ws.g_y1, ws.g_y2 = bufs[key]
        self._guard_buffers(ws, B, max(b - a for a, b in chunks), dev)
        bufs[key] = (ws.g_slab, ws.g_y1, ws.g_y2)
        S, Cs, mid = self.S, self.Cs, self.mid
        for a, b in chunks:
            (a1, b1), (a2, b2) = band_rows(a, b, H)
            s0, s1 = max(0, a1 - HALO_CONV1), min(H, b1 + HALO_CONV1)
            x = self._exact_warp_rows(ws, B, s0, s1, gate)
            self._exact_convs(ws, map_classifier, out, gate, x, (s0, s1), a, b, 0, packed=packed)
            # this chunk's own rows of conv1's input, y1 and y2 (a neighbour's halo rows are its own)
            xs = x.view(S * B, Cs, s1 - s0, W)[:, :, a - s0:b - s0]
            ops.store_gated_(xs, ws.slab.view((S * B,) + tuple(ws.slab.shape[2:]))[:, :, a:b], gate)
            y1 = ws.g_y1[:B * mid * (b1 - a1) * W].view(B, mid, b1 - a1, W)[:, :, a - a1:b - a1]
            ops.store_gated_(y1, ws.y1[:, :, a:b] if ws.y1.dtype == torch.bfloat16 else ws.y1[:, :, a:b], gate)
            y2 = ws.g_y2[:B * mid * (b2 - a2) * W].view(B, mid, b2 - a2, W)[:, :, a - a2:b - a2]
            ops.store_gated_(y2, ws.y2[:, :, a:b], gate)
        if ws.t1_valid and ws.wino_t is not None:  # conv1's weight gradient reads T: B^T of the exact input
            ops.wino_rows(ws.slab, self._conv1_desc(B), ws.wino_t, self.conv1_mask(dev, 0, H), gate=gate)
        if ws.t2_valid and ws.wino_t2 is not None and ws.y1.dtype == torch.bfloat16:  # conv2's reads T2
            ops.wino_rows(ws.y1, self._conv2_desc(ws), ws.wino_t2, dilation=2, gate=gate)

    def project_fuse(self, feats: Sequence[torch.Tensor], map_classifier) -> torch.Tensor:
        """Whole hot path on one device: warp every view, concat (zero-copy), fuse."""
        B = feats[0].shape[0]
        ws = self.workspace(B, feats[0].device)
        self.warp_views(ws, list(range(len(feats))), feats)
        return self.fuse(ws, map_classifier)
