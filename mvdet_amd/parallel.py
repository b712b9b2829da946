"""View-parallel project+fuse across GPUs (one process per GPU, torch.distributed).

SURVEY §8(e), §8(f) row 3.  The reference has no distributed code (everything on ``cuda:0``,
``persp_trans_detector.py:37-54``); this is the MI355X-native multi-GPU design of the north
star: views shard one per GPU (rank ``r`` owns views ``{v : v % P == r}``: their backbone,
upsample and warp run there), one exchange over xGMI, then the fusion split by row band.
Three forms of the exchange, all behind the same produce / exchange / consume steps:

* ``ViewBands`` (the ``bench.py --gpus N`` headline).  Every rank fuses output rows
  ``[r0, r1)`` (``ceil(Ho/P)`` rows), which need the ground-plane tensor's rows
  ``[r0 - 7, r1 + 7)`` only (the dilation-1/2/4 chain of ``:51-54``).  So instead of every rank
  receiving every view's whole slab, each rank cuts its views' warped slab into the P row
  windows and one **RCCL all-to-all** delivers to rank p exactly its window of every view: per
  rank ``(P-1)/P`` of its own views' slab (+ the 14 halo rows per window) goes out and the same
  comes in, against ``(P-1)`` whole slabs for the all-gather — 7x less xGMI traffic at config 3
  (P = 7), and all 7 links of the fully connected node carry a share at once.  The received
  windows are the band-local slab (``ProjectFuse.workspace(slab_rows=...)``) conv1 reads
  directly (row-Winograd transform + conv on the band).
* ``ViewParallel`` (``--mp-mode gather``; the north star's literal form): an in-place
  ``all_gather_into_tensor`` of the rank-major slab (each rank's chunk contiguous, no repack),
  then the same row-band fusion from the whole gathered slab.
* ``ViewPartialSum`` (``--mp-mode partial``; §8(e) "Alternative"): conv1 is linear in its
  input channels, so each rank convolves only its own views' channels over the whole grid
  (row-Winograd, no ReLU), **reduce-scatters** the [B, 512, Ho, Wo] partial sums by row band,
  all-gathers the 6 edge rows of every band as halo, then adds coord term + bias, ReLU, conv2,
  conv3 on its band.

``FramePipeline`` overlaps frame i's exchange (on a side stream, events guarding the double
buffers) with frame i-1's fusion and frame i+1's warp on the compute stream.

The compute engine is pluggable (``engine`` = ``pipeline.ProjectFuse`` on GPU; the CPU gloo
tests plug in an oracle engine), so the collective logic is tested without a GPU.  With the
``gloo`` backend and CUDA tensors the collectives are staged through host memory (single-GPU
rehearsals of the multi-rank path).
"""
from __future__ import annotations

import math
from types import SimpleNamespace
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .mp_model import balanced_parts, balanced_views, view_owners  # noqa: F401  (re-exported: the partial-sum mode's dealing)

# rows of the ground-plane tensor an output row of conv1 -> conv2 -> conv3 depends on, each side
HALO_IN = 1 + 2 + 4


def views_of(rank: int, world: int, num_cam: int) -> List[int]:
    return [v for v in range(num_cam) if v % world == rank]


def slot_views(world: int, num_cam: int) -> List[Optional[int]]:
    """Rank-major slot order: slot r*Vmax + j holds view r + P*j (or None)."""
    vmax = math.ceil(num_cam / world)
    out: List[Optional[int]] = []
    for r in range(world):
        vs = views_of(r, world, num_cam)
        out += vs + [None] * (vmax - len(vs))
    return out


def packed_slot_views(world: int, num_cam: int) -> List[int]:
    """Rank-major order without empty slots (the all-to-all's receive order)."""
    return [v for r in range(world) for v in views_of(r, world, num_cam)]


def row_band(H: int, rank: int, world: int) -> Tuple[int, int]:
    per = math.ceil(H / world)
    r0 = min(H, rank * per)
    return r0, min(H, r0 + per)


def _staged(t: torch.Tensor, group) -> bool:
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _all_gather_inplace(full: torch.Tensor, rank: int, world: int, group=None) -> None:
    """``full`` is [world * n, ...]; this rank's chunk is ``full[rank*n:(rank+1)*n]``."""
    n = full.shape[0] // world
    mine = full[rank * n:(rank + 1) * n]
    if _staged(full, group):
        host = full.cpu()
        dist.all_gather_into_tensor(host, host[rank * n:(rank + 1) * n].clone(), group=group)
        full.copy_(host)
        return
    dist.all_gather_into_tensor(full, mine, group=group)


def _reduce_scatter(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """``inp`` [world, *out.shape] summed over ranks; this rank's slice -> ``out``."""
    out = out.unsqueeze(0)
    if _staged(inp, group):
        host = inp.cpu()
        res = torch.empty_like(out, device="cpu")
        dist.reduce_scatter_tensor(res, host, op=dist.ReduceOp.SUM, group=group)
        out.copy_(res)
        return
    dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)


def _all_reduce_max(t: torch.Tensor, group=None) -> None:
    """In-place MAX over ranks (the non-finite guard's frame flag: 4 bytes)."""
    if _staged(t, group):
        host = t.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.MAX, group=group)
        t.copy_(host)
        return
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)


class _FrameGuard:
    """The non-finite guard of the exchange modes (``ViewBands``, ``ViewParallel``).  Each rank's
    window warp reports a NaN / inf sample into its frame's int32 flag under the frame's tag (the same
    frame counter on every rank); the exchange step first takes the MAX of the flags over the ranks
    (4 bytes), so every rank decides alike, on the device and in stream order: when any rank's features
    are non-finite, every rank overwrites its exchanged windows with the reference-order warp in fp32
    (same bytes as the split-bf16 windows) and every rank's fusion runs the gated fp32-MFMA exact path
    on them — the reference's NaN / inf pattern (``persp_trans_detector.py:65-81``); otherwise those
    launches exit at once.  The flag never needs a reset: tags only grow (reset at wrap-around)."""

    def __init__(self):
        self.tag = 0

    def next(self, fr) -> None:
        self.tag = self.tag % 0x7FFFFFFE + 1
        fr.tag = self.tag
        if self.tag == 1:
            fr.nf.zero_()

    @staticmethod
    def buffers(device):
        return torch.zeros(1, dtype=torch.int32, device=device), torch.zeros(1, dtype=torch.int32, device=device)

    @staticmethod
    def agree(fr, group) -> tuple:
        # the MAX of "this rank fired for THIS frame" (tag or 0), not of the raw flags: after a tag wrap-around
        # another frame buffer's stale pre-wrap tag must not outrank a current report
        torch.mul(fr.nf.eq(fr.tag), fr.tag, out=fr.gflag)
        _all_reduce_max(fr.gflag, group)
        return fr.gflag, fr.tag


def _all_to_all(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group=None) -> None:
    """1-D ``out`` / ``inp`` (element counts per peer in the split lists)."""
    if _staged(out, group):
        host = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(host, inp.cpu(), output_split_sizes=out_splits, input_split_sizes=in_splits,
                               group=group)
        out.copy_(host)
        return
    dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits, group=group)


class _ViewSharded:
    """Common driver: ``produce`` (this rank's warps, compute stream) -> ``exchange`` (the
    collectives; a side stream under ``FramePipeline``) -> ``consume`` (band fusion and the
    map all-gather, compute stream).  ``workspace(B, device, tag)`` returns one frame's buffers
    (``tag`` 0 / 1: the pipeline's double buffers)."""

    def __init__(self, proj_mats, grid_hw, rank: int, world: int, group=None):
        self.rank, self.world, self.group = rank, world, group
        self.num_cam = len(proj_mats)
        self.grid_hw = (int(grid_hw[0]), int(grid_hw[1]))
        self.my_views = views_of(rank, world, self.num_cam)
        self.vmax = math.ceil(self.num_cam / world)
        self.band = row_band(self.grid_hw[0], rank, world)
        self.band_rows = math.ceil(self.grid_hw[0] / world)
        self._frames = {}
        self._out = {}

    def _band_eff(self) -> Tuple[int, int]:
        r0, r1 = self.band
        return (r0, r1) if r1 > r0 else (0, 1)  # empty band (H < P): compute a dummy row

    def workspace(self, B: int, device, tag: int = 0):
        key = (str(torch.device(device)), int(B), int(tag))
        fr = self._frames.get(key)
        if fr is None:
            fr = self._make_frame(int(B), torch.device(device), int(tag))
            self._frames[key] = fr
        return fr

    def gather_map(self, band_out: torch.Tensor) -> torch.Tensor:
        """[B,1,rows,W] band of every rank -> [B,1,Ho,Wo] on every rank."""
        B, _, _, W = band_out.shape
        H = self.grid_hw[0]
        key = (band_out.device, B)
        buf = self._out.get(key)
        if buf is None:
            buf = torch.zeros((self.world, B, 1, self.band_rows, W), dtype=band_out.dtype, device=band_out.device)
            self._out[key] = buf
        r0, r1 = self.band
        if r1 > r0:
            buf[self.rank, :, :, :r1 - r0].copy_(band_out)
        _all_gather_inplace(buf, self.rank, self.world, self.group)
        full = buf.permute(1, 2, 0, 3, 4).reshape(B, 1, self.world * self.band_rows, W)
        return full[:, :, :H].clone()

    def step(self, fr, feats, map_classifier, mark=None) -> torch.Tensor:
        """One frame, unpipelined (``feats[j]`` is view ``my_views[j]``)."""
        if getattr(self, "fetches", False):
            if mark:
                mark("fetch")
            self.fetch(fr, feats)
        if mark:
            mark("warp")
        self.produce(fr, feats, map_classifier, mark=mark)
        if mark:
            mark("exchange")
        self.exchange(fr)
        return self.consume(fr, map_classifier, mark=mark)


class ViewParallel(_ViewSharded):
    """Slab all-gather + row-band fusion (``--mp-mode gather``).  With the engine's non-finite guard
    (``guard_windows``) the rank's views are warped with the non-finite report and ``_FrameGuard``'s
    exact path runs on the gathered slab."""

    def __init__(self, engine_factory, proj_mats: Sequence[torch.Tensor], grid_hw: Tuple[int, int],
                 rank: int, world: int, group=None):
        super().__init__(proj_mats, grid_hw, rank, world, group)
        self.engine = engine_factory(slot_views(world, self.num_cam))
        self.guard = bool(getattr(self.engine, "guard_windows", lambda: False)())
        self._fg = _FrameGuard()

    def _make_frame(self, B, device, tag):
        fr = SimpleNamespace(ws=self.engine.workspace(B, device, self._band_eff(), tag=tag), feats=None, tag=0)
        if self.guard:
            fr.nf, fr.gflag = _FrameGuard.buffers(device)
        return fr

    def _slots(self, fr):
        return [fr.ws.slab[self.engine.slot_of[v]] for v in self.my_views]

    def produce(self, fr, feats, map_classifier=None, mark=None) -> None:
        """Warp this rank's views into its rank-major slots."""
        if self.guard:
            self._fg.next(fr)
            fr.feats = list(feats)
            if self.my_views:
                self.engine.warp_windows(self._slots(fr), self.my_views, fr.feats, [0] * len(self.my_views),
                                         nonfinite=(fr.nf, fr.tag))
            return
        if hasattr(self.engine, "warp_views"):
            self.engine.warp_views(fr.ws, self.my_views, list(feats))
        else:
            for v, f in zip(self.my_views, feats):
                self.engine.warp_view(fr.ws, v, f)

    def exchange(self, fr) -> None:
        if self.guard:
            gate = _FrameGuard.agree(fr, self.group)
            if self.my_views:
                self.engine.warp_windows_exact(self._slots(fr), self.my_views, fr.feats, [0] * len(self.my_views), gate)
        _all_gather_inplace(fr.ws.slab, self.rank, self.world, self.group)

    def consume(self, fr, map_classifier, mark=None) -> torch.Tensor:
        band = self.engine.fuse(fr.ws, map_classifier, mark=mark)
        if self.guard:
            gate = (fr.gflag, fr.tag)
            self.engine.fuse_exact_from_windows(fr.ws, map_classifier, band, gate)
            self.engine.clear_windows(fr.ws.slab, gate)  # the warps skip out-of-source pixels of a zeroed slab
        if mark:
            mark("gather_map")
        return self.gather_map(band)


class ViewBands(_ViewSharded):
    """Row-window all-to-all + row-band fusion (``--mp-mode bands``).

    Rank p's conv1 input window is ``E = ceil(Ho/P) + 14`` rows starting at
    ``clamp(r0_p - 7, 0, Ho - E)`` (shifted inside the grid at the edges, so every window has E
    rows and the all-to-all's chunks are equal per view).  This rank's warp writes window p of each
    of its views straight into send chunk p (``warp_windows``: one launch, a row-window warp per
    (destination, view) — round 5: no whole-grid local slab and no window copies), and
    ``all_to_all_single`` delivers, from every rank q, q's views' rows of this rank's window: the
    receive buffer *is* the fusion engine's band-local slab, slots in rank-major packed order
    (``packed_slot_views``), so conv1 reads it in place.  Non-finite guard: ``_FrameGuard``."""

    def __init__(self, engine_factory, proj_mats, grid_hw, rank, world, group=None):
        super().__init__(proj_mats, grid_hw, rank, world, group)
        H = self.grid_hw[0]
        self.E = min(H, self.band_rows + 2 * HALO_IN)
        self.nv = [len(views_of(q, world, self.num_cam)) for q in range(world)]
        self.engine = engine_factory(packed_slot_views(world, self.num_cam))
        self.local = engine_factory(self.my_views, all_views=False) if self.my_views else None
        split = getattr(self.engine, "split", True)
        if not split and getattr(self.engine, "slab_dtype", torch.float32) != torch.float32:
            raise ValueError("the band exchange's windows are split-bf16 or fp32 (not an fp16 slab)")
        # every rank takes part in the flag's MAX, so the decision is the fusion engine's (the same on all)
        self.guard = bool(getattr(self.engine, "guard_windows", lambda: False)())
        self._fg = _FrameGuard()

    def window(self, p: int) -> Tuple[int, int]:
        H = self.grid_hw[0]
        r0, r1 = row_band(H, p, self.world)
        if r1 <= r0:
            r0 = 0
        lo = min(max(0, r0 - HALO_IN), H - self.E)
        return lo, lo + self.E

    def _make_frame(self, B, device, tag):
        ws = self.engine.workspace(B, device, self._band_eff(), slab_rows=self.window(self.rank), tag=tag)
        per_view = ws.slab[0].numel()  # elements of one view's window (the slab's slot)
        send = None
        if self.local is not None:
            nm = len(self.my_views)
            buf = self.local.window_buffer(self.world * nm, B, self.E, device)
            send = buf.view((self.world, nm) + tuple(buf.shape[1:]))
            assert send[0, 0].numel() == per_view
        fr = SimpleNamespace(ws=ws, send=send, per_view=per_view, B=B, device=device, feats=None, tag=0)
        if self.guard:
            fr.nf, fr.gflag = _FrameGuard.buffers(device)
        return fr

    def _entries(self, fr):
        """(send chunk, view, features index, window row0) of every (destination, own view)."""
        out = []
        for p in range(self.world):
            lo, _ = self.window(p)
            for j, v in enumerate(self.my_views):
                out.append((fr.send[p, j], v, j, lo))
        return out

    def produce(self, fr, feats, map_classifier=None, mark=None) -> None:
        if self.guard:
            self._fg.next(fr)
        fr.feats = list(feats)
        if self.local is None:
            return
        e = self._entries(fr)
        self.local.warp_windows([d for d, _, _, _ in e], [v for _, v, _, _ in e], [fr.feats[j] for _, _, j, _ in e],
                                [lo for _, _, _, lo in e], nonfinite=(fr.nf, fr.tag) if self.guard else None)

    def exchange(self, fr) -> None:
        gate = None
        if self.guard:
            gate = _FrameGuard.agree(fr, self.group)
            if self.local is not None:
                e = self._entries(fr)
                self.local.warp_windows_exact([d for d, _, _, _ in e], [v for _, v, _, _ in e],
                                              [fr.feats[j] for _, _, j, _ in e], [lo for _, _, _, lo in e], gate)
        n = fr.per_view
        inp = fr.send.reshape(-1) if fr.send is not None else fr.ws.slab.new_empty(0)
        _all_to_all(fr.ws.slab.reshape(-1), inp, [v * n for v in self.nv], [len(self.my_views) * n] * self.world,
                    self.group)
        if gate is not None and fr.send is not None:
            self.local.clear_windows(fr.send, gate)  # the window warps skip out-of-source pixels of zeroed chunks

    def consume(self, fr, map_classifier, mark=None) -> torch.Tensor:
        band = self.engine.fuse(fr.ws, map_classifier, mark=mark)
        if self.guard:
            self.engine.fuse_exact_from_windows(fr.ws, map_classifier, band, (fr.gflag, fr.tag))
        if mark:
            mark("gather_map")
        return self.gather_map(band)


class ViewPartialSum(_ViewSharded):
    """Partial-sum view-parallel fusion: conv1 split by views, reduce-scatter by rows.

    The engine of rank r holds only r's views (``all_views=False``); its warp writes conv1's row
    transform straight from the features (the fused warp + B^T: no slab, no transform pass) and
    conv1 over those views' channels writes its [B, 512, Ho, Wo] partial sums band-major, straight
    into the reduce-scatter's input (no staging copy).  A rank with no view contributes zeros.
    After the reduce-scatter rank r owns the summed conv1 pre-activation of rows
    ``[r*band, (r+1)*band)``; its halo rows (6 above and below: conv2's dilation 2 + conv3's 4)
    come from the neighbours' bands through one small all-gather of every band's top and bottom 6
    rows (bands of fewer than 6 rows fall back to gathering whole bands).  ``view_weights``
    (optional): per-view conv1 work; views are then dealt by ``balanced_views`` instead of v % P
    (fewer ranks than views: the frustum makes views' conv1 work uneven, 0.35-0.9 of a full view
    on the synthetic Wildtrack rig)."""

    HALO = 6

    def __init__(self, engine_factory, proj_mats, grid_hw, rank, world, group=None,
                 view_weights: Optional[Sequence[float]] = None, channels: Optional[int] = None,
                 min_part: int = 64, parts_k: int = 0, fetch_hw: Optional[Tuple[int, int]] = None,
                 fetch_dtype: torch.dtype = torch.float32, fetch_channels_last: bool = False):
        super().__init__(proj_mats, grid_hw, rank, world, group)
        self.my_parts, self.part_channels = None, None
        self.fetches = False
        if view_weights is not None and channels is not None:
            # round 5: views cut into channel parts dealt by their conv1 work (mp_model.balanced_parts): the
            # heaviest view no longer sets the rank time when P >= N.  The rank's engine takes the parts as
            # its cameras.  Round 6: each view's features (its backbone map) live on ONE rank, its owner
            # (mp_model.view_owners: where its backbone runs); ``fetch`` sends every other holder its parts'
            # channel slices (one all-to-all on the exchange stream), so the caller passes only the OWNED
            # views' features (``my_views``) and the timed region carries the transfer.
            assign, cp = balanced_parts(view_weights, world, int(channels), min_part=min_part, k=parts_k)
            self.assign, self.my_parts, self.part_channels = assign, assign[rank], cp
            self.owner = view_owners([w + 0.05 for w in view_weights], world)
            self.my_views = [v for v in range(self.num_cam) if self.owner[v] == rank]
            self.fetches = True
            self.fetch_hw = None if fetch_hw is None else (int(fetch_hw[0]), int(fetch_hw[1]))
            self.fetch_dtype, self.fetch_cl = fetch_dtype, bool(fetch_channels_last)
            # every part held away from its owner crosses xGMI once; both lists in rank order, parts sorted
            self.send_parts = [[(v, c0) for v, c0 in assign[q] if self.owner[v] == rank and q != rank]
                               for q in range(world)]
            self.recv_parts = [[(v, c0) for v, c0 in self.my_parts if self.owner[v] == p and p != rank]
                               for p in range(world)]
            self.moves = any(self.owner[v] != q for q in range(world) for v, _ in assign[q])
        elif view_weights is not None:
            self.my_views = balanced_views(view_weights, world)[rank]
        if self.my_parts is not None:
            self.engine = (engine_factory(list(range(len(self.my_parts))), parts=self.my_parts,
                                          part_channels=self.part_channels) if self.my_parts else None)
        else:
            self.engine = engine_factory(self.my_views, all_views=False) if self.my_views else None
        # a rank without views still runs the band fusion: give it an engine over view 0's
        # slot layout (its slab is never written or read) for the packed conv2 weights etc.
        self._fuse_engine = self.engine if self.engine is not None else engine_factory([0], all_views=False)
        for e in (self.engine, self._fuse_engine):  # the exchange sums fp32 partials into y1
            if e is not None and hasattr(e, "y1_split"):
                e.y1_split = False
        self._local_ws = {}

    def _make_frame(self, B, device, tag):
        ws = self._fuse_engine.workspace(B, device, self._band_eff(), tag=tag)
        if self.engine is not None:
            key = (str(device), B)
            if key not in self._local_ws:
                self._local_ws[key] = self.engine.workspace(B, device)
        mid = ws.y1.shape[1]
        H, W = self.grid_hw
        P, n = self.world, self.band_rows
        e = min(self.HALO, n)
        fr = SimpleNamespace(
            ws=ws, B=B, device=device, owned=None,
            stage=torch.zeros((P, B, mid, n, W), dtype=torch.float32, device=device),
            mine=torch.zeros((B, mid, n, W), dtype=torch.float32, device=device),
            edges=torch.zeros((P, 2, B, mid, e, W), dtype=torch.float32, device=device),
            full=None if n >= self.HALO else torch.zeros((P, B, mid, n, W), dtype=torch.float32, device=device))
        if self.fetches:  # the slice exchange's send / receive buffers, one [B, cp, h, w] piece per part
            h, w = self.fetch_hw if self.fetch_hw is not None else tuple(self._fuse_engine.src_hw)
            shape = (B, self.part_channels, h, w)
            fr.part_numel = B * self.part_channels * h * w
            ns, nr = sum(map(len, self.send_parts)), sum(map(len, self.recv_parts))
            fr.send = torch.empty(ns * fr.part_numel, dtype=self.fetch_dtype, device=device)
            fr.recv = torch.empty(nr * fr.part_numel, dtype=self.fetch_dtype, device=device)
            fr.send_views = self._part_views(fr.send, [p for ps in self.send_parts for p in ps], shape)
            fr.recv_views = self._part_views(fr.recv, [p for ps in self.recv_parts for p in ps], shape)
        return fr

    def _part_views(self, flat, parts, shape):
        """{(view, c0): [B, cp, h, w] view of ``flat``} for consecutive parts (channels-last memory when the
        wire format is)."""
        B, cp, h, w = shape
        n = B * cp * h * w
        out = {}
        for i, p in enumerate(parts):
            chunk = flat[i * n:(i + 1) * n]
            out[p] = chunk.view(B, h, w, cp).permute(0, 3, 1, 2) if self.fetch_cl else chunk.view(B, cp, h, w)
        return out

    def fetch(self, fr, feats) -> None:
        """The slice exchange (round 6): ``feats[j]`` is the owned view ``my_views[j]``'s map (at ``fetch_hw``,
        the backbone resolution, or at the warp's source size); each of its parts held by another rank is
        copied into the send buffer and one ``all_to_all_single`` delivers to every rank the slices of its
        parts whose views it does not own (a rank's own parts are read in place by its warp).  On the exchange
        stream under ``FramePipeline``, before the frame's produce."""
        if len(feats) != len(self.my_views):
            raise ValueError(f"rank {self.rank} owns views {self.my_views}: pass their {len(self.my_views)} maps")
        want = self.fetch_hw if self.fetch_hw is not None else tuple(self._fuse_engine.src_hw)
        for v, f in zip(self.my_views, feats):
            if tuple(f.shape[2:]) != tuple(want) or f.dtype != self.fetch_dtype:
                raise ValueError(f"view {v}: map {tuple(f.shape)} {f.dtype}, expected [B, C, {want[0]}, {want[1]}] "
                                 f"{self.fetch_dtype}")
        fr.owned = dict(zip(self.my_views, feats))
        if not self.moves:
            return
        cp = self.part_channels
        for q in range(self.world):
            for v, c0 in self.send_parts[q]:
                fr.send_views[(v, c0)].copy_(fr.owned[v][:, c0:c0 + cp])
        n = fr.part_numel
        _all_to_all(fr.recv, fr.send, [len(ps) * n for ps in self.recv_parts],
                    [len(ps) * n for ps in self.send_parts], self.group)

    def produce(self, fr, feats, map_classifier=None, mark=None) -> None:
        """Warp this rank's views or parts (into conv1's T where the engine fuses it; from backbone-resolution
        maps the fused upsample + warp), then conv1 over their channels for all rows, written band-major into
        the reduce-scatter's input.  With the slice exchange (``fetches``) the parts' features are the own
        views' slices and the fetched ones (``feats`` is not read: ``fetch`` took the owned maps)."""
        if self.engine is None:
            fr.stage.zero_()
            return
        lws = self._local_ws[(str(fr.device), fr.B)]
        cams, feats = self._cameras(fr, feats)
        if tuple(feats[0].shape[2:]) != tuple(self.engine.src_hw):
            self.engine.warp_views_upsampled(lws, cams, feats)  # a4 + a5 (+ conv1's B^T) from backbone maps
        elif hasattr(self.engine, "warp_views"):
            self.engine.warp_views(lws, cams, feats)
        else:
            for v, f in zip(cams, feats):
                self.engine.warp_view(lws, v, f)
        if mark:
            mark("conv1")
        self.engine.conv1_partial(lws, map_classifier, fr.stage, mark=mark, band_rows=self.band_rows)

    def _cameras(self, fr, feats):
        """(engine cameras, their features): the views, or with channel parts each part's channel slice
        (own views' slices in place, the others' from the slice exchange's receive buffer)."""
        if self.my_parts is None:
            return list(self.my_views), list(feats)
        cp = self.part_channels
        return (list(range(len(self.my_parts))),
                [fr.owned[v][:, c0:c0 + cp] if self.owner[v] == self.rank else fr.recv_views[(v, c0)]
                 for v, c0 in self.my_parts])

    @property
    def conv1_channels(self) -> int:
        """Input channels of this rank's conv1 partial (its views', or its parts')."""
        if self.my_parts is not None:
            return len(self.my_parts) * self.part_channels
        return None if self.engine is None else len(self.my_views) * self.engine.C

    def exchange(self, fr) -> None:
        """Reduce-scatter of the partial sums by band, then the halo rows into ``ws.y1``."""
        ws = fr.ws
        _reduce_scatter(fr.mine, fr.stage, self.group)
        H, P, n = self.grid_hw[0], self.world, self.band_rows
        a1, b1 = ws.y1_rows

        def rows_of(p):  # the summed rows of band p available locally after the exchange
            return min(H, p * n), min(H, (p + 1) * n)

        if fr.full is not None:  # bands thinner than the halo: gather whole bands
            fr.full[self.rank].copy_(fr.mine)
            _all_gather_inplace(fr.full, self.rank, P, self.group)
            for p in range(P):
                a, b = rows_of(p)
                lo, hi = max(a, a1), min(b, b1)
                if hi > lo:
                    ws.y1[:, :, lo - a1:hi - a1].copy_(fr.full[p][:, :, lo - a:hi - a])
            return
        e = self.HALO
        fr.edges[self.rank, 0].copy_(fr.mine[:, :, :e])
        r0, r1 = self.band
        if r1 > r0:
            last = r1 - r0
            fr.edges[self.rank, 1].copy_(fr.mine[:, :, max(0, last - e):max(0, last - e) + e])
        _all_gather_inplace(fr.edges, self.rank, P, self.group)
        if r1 > r0:  # own band
            ws.y1[:, :, r0 - a1:r1 - a1].copy_(fr.mine[:, :, :r1 - r0])
        # halo above: the last rows of band rank-1; below: the first rows of band rank+1
        if self.rank > 0 and a1 < r0:
            pa, pb = rows_of(self.rank - 1)
            top0 = max(pa, pb - e)  # global row of edges[rank-1, 1][:, :, 0]
            ws.y1[:, :, :r0 - a1].copy_(fr.edges[self.rank - 1, 1][:, :, a1 - top0:r0 - top0])
        if self.rank + 1 < P and b1 > r1:
            na, _ = rows_of(self.rank + 1)
            ws.y1[:, :, r1 - a1:].copy_(fr.edges[self.rank + 1, 0][:, :, :b1 - na])

    def consume(self, fr, map_classifier, mark=None) -> torch.Tensor:
        band = self._fuse_engine.finish_from_y1(fr.ws, map_classifier, mark=mark)
        if mark:
            mark("gather_map")
        return self.gather_map(band)


class FramePipeline:
    """Frames through a view-sharded driver with the exchange overlapped (§8(f) row 3).

    ``submit(feats)`` enqueues frame i's warp (+ pack / partial conv1) on the compute stream,
    its exchange on a side stream after an event, then frame i-1's fusion on the compute stream
    after frame i-1's exchange-done event; it returns frame i-1's map (None for the first).
    ``drain()`` finishes the last frame.  Two frame buffers alternate: frame i+2's produce runs
    after frame i's consume on the compute stream, and frame i+2's exchange waits for that
    produce, so no buffer is rewritten while a collective or the fusion still reads it.  With
    gloo (CPU tests, host-staged single-GPU rehearsals) the same order runs on one stream.

    A driver with an input exchange (``fetches``: the partial-sum mode's channel-slice exchange, round 6)
    adds a stage in front: ``submit(frame i)`` enqueues frame i's fetch on the side stream, then frame
    i-1's produce (after its fetch-done event) and exchange, then frame i-2's consume — the fetch of frame
    i+1 runs under frame i's produce, the reduce-scatter of frame i under frame i-1's fusion.  Three frame
    buffers rotate (frame i+3's fetch waits for an event recorded after frame i's produce was enqueued);
    ``submit`` then returns frame i-2's map and ``drain`` is called until it returns None."""

    def __init__(self, driver: _ViewSharded, B: int, device):
        self.d = driver
        device = torch.device(device)
        self.fetching = bool(getattr(driver, "fetches", False))
        self.frames = [driver.workspace(B, device, tag=t) for t in range(3 if self.fetching else 2)]
        self.comm = (torch.cuda.Stream(device) if device.type == "cuda" and dist.get_backend(driver.group) == "nccl"
                     else None)
        self.i = 0
        self.fetched = None   # (frame, fetch-done event): inputs exchanged, not yet produced
        self.pending = None   # (frame, exchange-done event): produced and exchanged, not yet consumed

    def _on_comm(self, fn):
        """Run ``fn`` on the side stream after everything enqueued so far on the compute stream."""
        if self.comm is None:
            fn()
            return None
        ready = torch.cuda.Event()
        ready.record()
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(ready)
            fn()
            done = torch.cuda.Event()
            done.record(self.comm)
        return done

    def _advance(self, fr, feats, fetched, map_classifier):
        """Produce + exchange ``fr`` (after its fetch-done event), then consume the pending frame."""
        if fetched is not None:
            torch.cuda.current_stream().wait_event(fetched)
        self.d.produce(fr, feats, map_classifier)
        done = self._on_comm(lambda: self.d.exchange(fr))
        out = self._consume(self.pending, map_classifier) if self.pending is not None else None
        self.pending = (fr, done)
        return out

    def submit(self, feats, map_classifier) -> Optional[torch.Tensor]:
        fr = self.frames[self.i % len(self.frames)]
        self.i += 1
        if not self.fetching:
            return self._advance(fr, feats, None, map_classifier)
        ev = self._on_comm(lambda: self.d.fetch(fr, feats))
        prev, self.fetched = self.fetched, (fr, ev)
        return self._advance(prev[0], None, prev[1], map_classifier) if prev is not None else None

    def _consume(self, pending, map_classifier):
        fr, done = pending
        if done is not None:
            torch.cuda.current_stream().wait_event(done)
        return self.d.consume(fr, map_classifier)

    def drain(self, map_classifier) -> Optional[torch.Tensor]:
        """The next map still in flight (None when every submitted frame has come back)."""
        if self.fetched is not None:
            fr, ev = self.fetched
            self.fetched = None
            return self._advance(fr, None, ev, map_classifier)
        if self.pending is None:
            return None
        out = self._consume(self.pending, map_classifier)
        self.pending = None
        return out

    def drain_all(self, map_classifier) -> List[torch.Tensor]:
        out = []
        while True:
            o = self.drain(map_classifier)
            if o is None:
                return out
            out.append(o)


def bench_main(args) -> None:
    """``bench.py`` under torchrun with WORLD_SIZE > 1.  ``value``: the view-parallel band
    exchange (``ViewBands``, pipelined; strong scaling: one frame's views across the ranks) at
    ``--config``; alongside: frame-parallel (weak), the slab all-gather and the partial-sum
    modes, and the band exchange at config 3 (the north star's 7-view 480 x 1440 workload)."""
    import json
    import os
    import time

    import numpy as np

    from bench import BF16_MFMA_PEAK_TFS, DTYPE_LABEL, FP32_MFMA_PEAK_TFS, build_mc, head_params
    from . import mp_model, synthetic
    from .geometry import projection_matrices
    from .pipeline import ProjectFuse

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("MVBEV_DIST_BACKEND", "nccl")
    # one GPU per rank; on a 1-GPU rehearsal box (gloo) ranks share device 0
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
    bf16 = args.precision == "bf16x3"

    def timed(run_steps, K):
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        run_steps(K)
        torch.cuda.synchronize()
        dist.barrier()
        dt = time.perf_counter() - t0
        t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def stage_times(step_fn, K):
        """Per-stage HIP-event times (rank 0) of K unpipelined steps."""
        marks = []
        for _ in range(K):
            m = []
            step_fn(lambda s, m=m: m.append((s, torch.cuda.Event(enable_timing=True))) or m[-1][1].record())
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            m.append(("end", e))
            marks.append(m)
        torch.cuda.synchronize()
        out = {}
        for m in marks:
            for (s, a), (_, b) in zip(m, m[1:]):
                out.setdefault(s, []).append(a.elapsed_time(b))
        return {s: round(float(np.mean(v)), 4) for s, v in out.items()}

    def setup(cfg):
        spec = synthetic.CONFIGS[cfg]
        ds = spec["make"]()
        B, C, N = spec["B"], spec["C"], ds.num_cam
        up = tuple(ds.upsample_shape)
        grid = tuple(ds.reducedgrid_shape)
        pm = projection_matrices(ds)
        mc = build_mc(C, N, head_params(N, seed=cfg, C=C), dev)
        half = cfg == 4  # fp16 features: the fused warp / window warps read them (split-bf16 slab / T)
        # cfg4's fp16 features feed the fused warp (split-bf16 T, bf16x3) or an fp32 slab (precision fp32)
        fact = (lambda sv, **kw: ProjectFuse(pm, up, grid, C, slot_views=sv, precision=args.precision, **kw))
        return SimpleNamespace(spec=spec, B=B, C=C, N=N, up=up, grid=grid, pm=pm, mc=mc, half=half, fact=fact)

    def feats_for(s, views, cfg, base_seed=0):
        return [synthetic.synthetic_features(s.B, s.C, [u // 3 for u in s.up], s.up, seed=1000 * cfg + base_seed + v,
                                             device=dev).to(torch.float16 if s.half else torch.float32)
                for v in views]

    def backbone_maps(s, views, cfg, channels_last):
        """The owned views' backbone-resolution maps (``:64``; the warp's source is their 3x upsample)."""
        out = []
        for v in views:
            x = synthetic.backbone_features(s.B, s.C, [u // 3 for u in s.up], seed=1000 * cfg + v, device=dev)
            x = x.to(torch.float16) if s.half else x
            out.append(x.contiguous(memory_format=torch.channels_last) if channels_last else x)
        return out

    def run(mode, cfg, K, W):
        s = setup(cfg)
        ho, wo = s.grid
        with torch.no_grad():
            if mode == "frames":  # each rank fuses its own frame batch (all views), no collective
                eng = s.fact(None)
                feats = feats_for(s, range(s.N), cfg, base_seed=100 * rank)
                ws = eng.workspace(s.B, dev)

                def fstep(mark=None):
                    if mark:
                        mark("warp")
                    eng.warp_views(ws, list(range(s.N)), feats)
                    return eng.fuse(ws, s.mc, mark=mark)
                for _ in range(W):
                    fstep()
                dt = timed(lambda k: [fstep() for _ in range(k)], K)
                st = stage_times(fstep, max(3, K // 4))
                y1r = ws.y1_rows
                value = world * s.B * K / dt
                band = (0, ho)
                act_eng, act_rows = eng, y1r
            else:
                cls = {"bands": ViewBands, "gather": ViewParallel, "partial": ViewPartialSum}[mode]
                kw = {}
                if mode == "partial":
                    # views cut into channel parts dealt by their conv1 work (frustum-active tiles), the split the
                    # cost model predicts fastest; each rank holds only the backbone-resolution maps of the views
                    # it owns (channels-last, as the drop-in detector's backbone writes them; fp16 NCHW at cfg4)
                    # and the slice exchange sends the other holders their parts inside the timed region
                    kw["view_weights"] = [float(a.mean()) for a in mp_model.config_inputs(cfg)[4]]
                    kw["channels"] = s.C
                    kw["parts_k"] = int(mp_model.predict_config(cfg, world)["partial"]["parts_k"]) \
                        if cfg in mp_model.SINGLE_GPU_MS else 0
                    kw["fetch_hw"] = tuple(u // 3 for u in s.up)
                    kw["fetch_dtype"] = torch.float16 if s.half else torch.float32
                    kw["fetch_channels_last"] = not s.half
                vp = cls(s.fact, s.pm, s.grid, rank, world, **kw)
                feats = (backbone_maps(s, vp.my_views, cfg, channels_last=not s.half) if mode == "partial"
                         else feats_for(s, vp.my_views, cfg))
                pipe = FramePipeline(vp, s.B, dev)
                for _ in range(W):
                    pipe.submit(feats, s.mc)
                pipe.drain_all(s.mc)

                def steps(k):
                    for _ in range(k):
                        pipe.submit(feats, s.mc)
                    pipe.drain_all(s.mc)
                dt = timed(steps, K)
                fr = vp.workspace(s.B, dev)
                st = stage_times(lambda mark: vp.step(fr, feats, s.mc, mark=mark), max(3, K // 4))
                st_total = round(sum(st.values()), 4)  # the marks partition the step
                value = s.B * K / dt
                band = vp.band
                y1r = fr.ws.y1_rows
                act_eng = vp.engine if mode != "partial" else vp._fuse_engine
                act_rows = y1r
        # conv1's input channels on rank 0: every view's, or (partial) its own parts' / views'
        nch = s.N * s.C if mode != "partial" else max(1, vp.conv1_channels or 0)
        rows = ho if mode == "partial" else act_rows[1] - act_rows[0]
        conv1_flop = 2.0 * s.B * rows * wo * 9 * nch * 512
        # conv1's marks: "conv1" before its row transform (none when the fused warp wrote T), then
        # "conv1_wino" right before the Winograd conv kernel; the roofline is the conv kernel's, as at N = 1
        wino = bool(bf16 and "conv1_wino" in st)
        conv_ms = st["conv1_wino"] if wino else st.get("conv1", 0.0)
        if "conv1_wino" in st:
            st["conv1_total"] = round(st.get("conv1", 0.0) + st["conv1_wino"], 4)
        ach = (conv1_flop / (conv_ms * 1e-3) / 1e12 * (3 * (5.0 / 9.0 if wino else 1.0) if bf16 else 1.0)
               if conv_ms > 0 else None)
        res = dict(value=round(value, 3), ms_per_step=round(dt * 1e3 / K, 4), stages_ms_rank0=st,
                   band_rank0=list(band), conv1_rows_rank0=list(act_rows), steps=K, warmup=W,
                   workload=f"cfg{cfg}: {s.spec['name']}")
        if mode == "partial":
            res["inputs"] = ("each rank: the backbone-resolution maps of the views it owns (mp_model.view_owners; "
                             + ("fp16 NCHW" if s.half else "fp32 channels-last") + "); the channel slices of the "
                             "parts held elsewhere cross in one all-to-all per frame inside the timed region, and "
                             "the a4 upsample runs fused into the warp (more work than the N = 1 value's step, but less time: "
                             "the like-for-like N = 1 figure is that line's plus_a4.fused_channels_last.value)")
            res["parts"] = dict(k=s.C // vp.part_channels, part_channels=vp.part_channels,
                                parts_rank0=[list(p) for p in vp.my_parts], owners=vp.owner,
                                fetched_bytes_rank0=int(sum(map(len, vp.recv_parts))) * fr.part_numel *
                                (2 if s.half else 4))
        elif mode != "frames":
            res["inputs"] = "each rank: the upsampled features of the views it owns (views_of: v % P)"
        if mode != "frames":
            res["unpipelined_ms_rank0"] = st_total
        if ach is not None:
            peak = BF16_MFMA_PEAK_TFS if bf16 else FP32_MFMA_PEAK_TFS
            res["conv1_roofline_rank0"] = {"achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                                           "frac": round(ach / peak, 4),
                                           "basis": ("3 bf16 passes x 5/9 (row Winograd) x " if wino else
                                                     "3 bf16 passes x " if bf16 else "") +
                                           "2*B*rows*Wo*9*(rank 0's conv1 input channels)*512 over conv1's event "
                                           "time (dense, no mask)"}
        return res

    mode = getattr(args, "mp_mode", "auto")
    predicted = None
    if mode == "auto":  # the mode the cost model predicts fastest at this config and world size
        if args.config in mp_model.SINGLE_GPU_MS:
            predicted = {k: round(v["frame"], 4) for k, v in mp_model.predict_config(args.config, world).items()}
        mode = mp_model.choose_mode(args.config, world)
    hows = {"frames": f"frame-parallel x{world}: each rank its own frame batch (all views), no collective",
            "bands": f"view-parallel x{world} ({backend}): rank r warps views v%{world}==r, RCCL all-to-all of "
                     "each output band's input row window (+7-row halo), row-band fusion, map-band all-gather; "
                     "exchange of frame i overlapped with fusion of frame i-1",
            "gather": f"view-parallel x{world} ({backend}): all-gather of the warped slab + row-band fusion, "
                      "pipelined",
            "partial": f"view-parallel x{world} ({backend}): views' conv1 partial sums, reduce-scatter by row band "
                       "+ edge-row all-gather, pipelined"}
    res = run(mode, args.config, args.steps, args.warmup)
    alts = {}
    if not getattr(args, "no_alt", False):
        def run_alt(m, cfg):
            # a failure in a reported-alongside mode (raised on every rank alike, e.g. a collective
            # the fabric rejects) must not cost the `value` line of the mode measured above
            try:
                return run(m, cfg, max(5, args.steps // 2), 2)
            except Exception as e:  # noqa: BLE001
                return {"error": f"{type(e).__name__}: {e}"[:300]}
        for m in ("frames", "bands", "gather", "partial"):
            if m != mode:
                alts[m] = run_alt(m, args.config)
        ns = getattr(args, "north_star_cfg", 3)
        if ns and ns != args.config:
            ns_mode = mp_model.choose_mode(ns, world)
            alts[f"north_star_cfg{ns}"] = dict(run_alt(ns_mode, ns), mode=ns_mode)
    if rank == 0:
        cpu = None
        if not getattr(args, "no_cpu_baseline", False):
            # rank 0 only, after every timed region (the other ranks wait at the final barrier): the
            # oracle on a bounded sample of the same workload, as the N = 1 line reports it
            from bench import cpu_baseline
            s0 = setup(args.config)
            # the N = 1 line's sample (BASELINE.md:26: 2 warm-ups + the median of 5, and the one-thread figure)
            cpu = cpu_baseline(s0.spec["make"](), 1 if s0.half else s0.B, s0.C, s0.pm,
                               head_params(s0.N, seed=args.config, C=s0.C), frames=5, config=args.config,
                               warmups=2, single_frames=3)
        rl = res.get("conv1_roofline_rank0", {})
        line = {
            "metric": "multi-view frames/sec (project+fuse)",
            "value": res["value"],
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak" if mode == "frames" else "strong",
            "vs_baseline": None,
            "dtype": DTYPE_LABEL[args.precision],
            "data": "synthetic (see single-GPU line)",
            "config": {"workload": res["workload"], "batch": synthetic.CONFIGS[args.config]["B"] *
                       (world if mode == "frames" else 1), "precision": args.precision, "parallelism": hows[mode]},
            "roofline": {"kernel": "conv1's conv kernel on rank 0 (its row band + halo)", "bound": "mfma",
                         "achieved": rl.get("achieved"), "peak": rl.get("peak"), "unit": "TFLOP/s",
                         "frac": rl.get("frac"), "traffic": None, "basis": rl.get("basis")},
            "cpu_baseline": cpu,
            "stages_ms_rank0": res["stages_ms_rank0"],
            "band_rank0": res["band_rank0"],
            # gloo with ranks sharing the devices (fewer GPUs than ranks): a rehearsal of the path, not a
            # multi-GPU measurement
            "rehearsal": backend != "nccl",
            "mode": mode,
            # mp_model's predicted per-frame ms of each view-parallel mode and what it chose
            "predicted_frame_ms": predicted,
        }
        if cpu:
            line["speedup_vs_cpu"] = round(res["value"] / cpu["value"], 1)
        if "unpipelined_ms_rank0" in res:
            line["unpipelined_ms_rank0"] = res["unpipelined_ms_rank0"]
        for k in ("inputs", "parts"):
            if k in res:
                line[k] = res[k]
        for m, r in alts.items():
            ns_key = m.startswith("north_star")
            key = m if ns_key else ("frame_parallel" if m == "frames" else f"view_parallel_{m}")
            if "error" not in r:
                r = dict(r, parallelism=hows[r.get("mode", "bands") if ns_key else m],
                         scaling="weak" if m == "frames" else "strong")
            line[key] = r
        print(json.dumps(line), flush=True)
    dist.barrier()
    dist.destroy_process_group()
