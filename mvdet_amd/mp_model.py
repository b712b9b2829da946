"""Per-mode cost model of the view-parallel multi-GPU path.

One frame's views shard over P ranks (rank r owns views v % P == r, ``parallel.views_of``);
the three exchange forms of ``parallel`` differ in what crosses xGMI and in how much of the
fusion each rank repeats:

* ``bands``   — every rank warps the P row windows of its views (the input rows of each output band +
  the 7-row halo of the dilation-1/2/4 chain, ``:51-54``) straight into its all-to-all send chunks
  (round 5: no whole-grid slab, no window copies); the all-to-all delivers to rank p its window of
  every view; each rank transforms and convolves a band of ``ceil(Ho/P) + 12`` conv1 rows (12-row tiles).
* ``partial`` — every rank warps its views straight into conv1's row transform and runs conv1 over
  its OWN views' channels for the whole grid (conv1 is linear in its input channels); the
  [B, 512, Ho, Wo] fp32 partial sums are reduce-scattered by row band; conv2 / conv3 on the band.
* ``gather``  — the slab is all-gathered (``N * C * Ho * Wo`` fp32 to every rank), then the band
  fusion of ``bands``.

Per rank and frame the compute stream runs produce + consume, the exchange runs on a side stream
(``parallel.FramePipeline``), so a pipelined frame costs ``max(produce + consume, exchange)``; the
slowest rank sets the rate.  Compute times scale the measured single-GPU stage times of the same
config (``SINGLE_GPU_MS``, from ``bench.py`` lines) by the work a rank does: conv1 by its share of
the frustum-active (12 x 32 tile, view) pairs, computed here from the geometry exactly as the conv's
mask is; conv2 / the transform by rows.  Link model (an assumption until the 8-GPU node measures
it): each of a GPU's 7 xGMI links carries ``LINK_GBS`` per direction; an all-to-all puts each
peer's chunk on its own link; RCCL's ring collectives (reduce-scatter, all-gather) reach
``COLL_EFF`` of the links' sum.  The model picks ``bench.py --gpus N``'s ``value`` mode per config.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

import numpy as np

LINK_GBS = 64.0     # effective GB/s per xGMI link and direction (153.6 GB/s per link both ways, ~83 %)
COLL_EFF = 0.7      # RCCL ring collectives: fraction of the P - 1 links' sum they sustain
A2A_EFF = 0.7       # all-to-all: fraction of one link per peer chunk
# the fused upsample + warp + B^T from channels-last backbone maps vs the NCHW fused warp from upsampled
# features (cfg2: 0.3004 vs 0.4852 ms, profiles/r05final_bench.json plus_a4.fused_channels_last), for the
# configs without their own ``warp_up`` figure
WARP_UP_RATIO = 0.62

# Single-GPU stage times (ms, one frame) of the bench's path on 1 x MI355X: warp = fused warp + row
# transform of every view, conv1 = the Winograd conv kernel (whole grid, frustum-masked), conv2 =
# Winograd conv2 + conv3 partials (incl. its transform), conv3 = the partials' reduce; transform =
# mvbev_wino_rows_split_bf16 over the whole slab (measured at cfg2 in round 2, scaled by size).
# profiles/r05d_bench.json (the cfg2 line and its cfg3 / cfg5 / cfg4 sub-objects; NCHW features; cfg4: B = 8,
# fp16 features on the fused warp).
SINGLE_GPU_MS: Dict[int, Dict[str, float]] = {
    2: dict(warp=0.4938, conv1=1.4174, conv2=0.3354, conv3=0.0253, transform=0.25, warp_up=0.3004),
    3: dict(warp=5.2145, conv1=20.3366, conv2=4.746, conv3=0.1937, transform=4.0),
    4: dict(warp=3.3355, conv1=8.2243, conv2=2.4732, conv3=0.151, transform=1.6),
    5: dict(warp=4.4294, conv1=15.0497, conv2=7.0832, conv3=0.1938, transform=2.3),
}


def view_tile_activity(m_norm, src_hw, grid_hw, tile_h: int = 12, tile_w: int = 32) -> np.ndarray:
    """Per 12 x 32 conv1 tile: 1 where the view's warp can be non-zero in the tile + 1-pixel halo
    (``mvbev_warp_tile_mask``'s rule: some sample inside the source), from the kornia matrix in
    float64 (a model input, not the product's mask).  Returns [tiles_y, tiles_x] bool."""
    H, W = int(src_hw[0]), int(src_hw[1])
    Ho, Wo = int(grid_hw[0]), int(grid_hw[1])
    m = np.asarray(m_norm, dtype=np.float64).reshape(3, 3)
    gy, gx = np.meshgrid((np.arange(Ho) / max(Ho - 1, 1) - 0.5) * 2, (np.arange(Wo) / max(Wo - 1, 1) - 0.5) * 2,
                         indexing="ij")
    p = np.stack([gx, gy, np.ones_like(gx)], -1) @ m.T
    z = p[..., 2]
    s = np.where(np.abs(z) > 1e-8, 1.0 / (z + 1e-8), 1.0)
    ix = ((p[..., 0] * s + 1) / 2) * (W - 1)
    iy = ((p[..., 1] * s + 1) / 2) * (H - 1)
    inside = (ix > -1) & (ix < W) & (iy > -1) & (iy < H)
    ty, tx = -(-Ho // tile_h), -(-Wo // tile_w)
    act = np.zeros((ty, tx), dtype=bool)
    for a in range(ty):
        r0, r1 = max(0, a * tile_h - 1), min(Ho, (a + 1) * tile_h + 1)
        rows = inside[r0:r1]
        for b in range(tx):
            act[a, b] = rows[:, max(0, b * tile_w - 1):min(Wo, (b + 1) * tile_w + 1)].any()
    return act


def balanced_views(weights: Sequence[float], world: int) -> List[List[int]]:
    """Views to ranks by longest-processing-time first: each view (heaviest first, by its conv1
    work ``weights[v]``, e.g. its frustum-active tile fraction) to the rank with the least work so far
    (ties: the lower rank); a deterministic function of the geometry, so every rank computes the same
    assignment.  Each rank's list is in view order."""
    load = [0.0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    for v in sorted(range(len(weights)), key=lambda v: (-weights[v], v)):
        r = min(range(world), key=lambda q: (load[q], q))
        out[r].append(v)
        load[r] += weights[v]
    return [sorted(vs) for vs in out]


def view_owners(weights: Sequence[float], world: int) -> List[int]:
    """The rank whose backbone produces each view (round 6): the longest-processing-time
    dealing of whole views (``balanced_views``), so whole-view parts never cross xGMI and, with P >= N, every
    view has a rank of its own.  Deterministic: every rank computes the same owners."""
    owner = [-1] * len(weights)
    for r, vs in enumerate(balanced_views(weights, world)):
        for v in vs:
            owner[v] = r
    return owner


def balanced_parts(weights: Sequence[float], world: int, C: int, warp_frac: float = 0.05,
                   min_part: int = 64, gain: float = 0.02, k: int = 0, affinity: float = 0.5):
    """The partial-sum mode's channel split (round 5): conv1 is linear in its input channels, so a view's
    channels can be convolved on several ranks.  Views are cut into k equal channel parts (k = 1, 2, 4, ...
    while the part keeps >= ``min_part`` channels) and the parts dealt by longest-processing-time, a part of
    view v weighing (weights[v] + warp_frac) / k (its conv1 share of the frustum-active work plus its share
    of the view's warp, ``warp_frac`` of a full view's conv1); the k with the smallest maximum rank load
    wins, a larger k only when it lowers that load by more than ``gain`` (each part is a slot of the rank's
    warp and conv1); ``k`` > 0 forces the split.  Round 6: a part goes to its view's owner (``view_owners``,
    where its backbone map is) instead of the least-loaded rank when that costs at most ``affinity`` of the
    part's weight in load, so fewer slices cross xGMI.  Returns (per rank the sorted (view, first channel)
    parts, part width); deterministic, so every rank computes the same assignment."""
    N = len(weights)
    owner = view_owners([w + warp_frac for w in weights], world)
    best = None
    kk = 1
    while C % kk == 0 and (kk == 1 or C // kk >= min_part):
        if k and kk != k:
            kk *= 2
            continue
        items = sorted(((weights[v] + warp_frac) / kk, v, j) for v in range(N) for j in range(kk))
        items.sort(key=lambda t: (-t[0], t[1], t[2]))
        load = [0.0] * world
        out: List[List[tuple]] = [[] for _ in range(world)]
        for w, v, j in items:
            r = min(range(world), key=lambda q: (load[q], q))
            if load[owner[v]] <= load[r] + affinity * w:
                r = owner[v]
            out[r].append((v, j * (C // kk)))
            load[r] += w
        m = max(load)
        if best is None or m < best[0] * (1.0 - gain):
            best = (m, [sorted(ps) for ps in out], C // kk)
        kk *= 2
    if best is None:
        raise ValueError(f"cannot split {C} channels into {k} parts of >= {min_part}")
    return best[1], best[2]


def fetch_link_bytes(assign, owner: Sequence[int], P: int, part_bytes: float) -> np.ndarray:
    """[P, P] bytes of backbone-map channel slices rank p sends to rank q per frame (the partial-sum
    mode's slice exchange: every part held by a rank that does not own its view)."""
    out = np.zeros((P, P))
    for q, ps in enumerate(assign):
        for v, _ in ps:
            if owner[v] != q:
                out[owner[v], q] += part_bytes
    return out


def _tiles(rows: int) -> int:
    return 12 * math.ceil(rows / 12)


def predict(N: int, C: int, grid_hw, B: int, P: int, single: Dict[str, float],
            activity: Sequence[np.ndarray], backbone_px: float = 0.0) -> Dict[str, dict]:
    """Predicted per-frame ms of each mode at P ranks (the slowest rank), with its parts.  ``backbone_px``:
    pixels of one backbone map (the partial-sum mode's slice exchange moves channel slices of those)."""
    Ho, Wo = int(grid_hw[0]), int(grid_hw[1])
    band = math.ceil(Ho / P)
    vmax = math.ceil(N / P)
    act = np.stack([a.astype(np.float64) for a in activity])         # [N, ty, tx]
    tot = act.sum()
    rows_all = _tiles(Ho)
    w_view = single["warp"] / N                                      # fused warp + T, per view
    slab_view = 4.0 * B * C * Ho * Wo                                # bytes of one view's split slab
    bw = LINK_GBS * 1e6                                              # bytes per ms per link
    # conv1 over band rows [r0, r0 + rows): the active (tile, view) pairs of those tile rows
    def conv1_band(r0: int, rows: int, views=None) -> float:
        t0, t1 = r0 // 12, min(act.shape[1], math.ceil((r0 + rows) / 12))
        sub = act[:, t0:t1] if views is None else act[list(views), t0:t1]
        return single["conv1"] * sub.sum() / tot
    out = {}
    # -- bands
    E = min(Ho, band + 14)
    a2a = vmax * B * C * E * Wo * 4.0 / (A2A_EFF * bw)
    worst = 0.0
    for p in range(P):
        r0 = min(Ho, p * band)
        y1 = (max(0, r0 - 6), min(Ho, r0 + band + 6))
        c1 = conv1_band(y1[0], y1[1] - y1[0])
        c2 = single["conv2"] * _tiles(min(Ho, band + 8)) / rows_all
        tr = single["transform"] * E / Ho
        worst = max(worst, c1 + c2 + tr)
    produce = vmax * w_view * 0.8 * P * E / Ho   # the split warp (~0.8 of the fused warp + B^T) of P windows
    out["bands"] = dict(produce=produce, exchange=a2a, consume=worst + single["conv3"] / P,
                        frame=max(produce + worst, a2a))
    # -- partial
    rs_bytes = 4.0 * B * 512 * Ho * Wo
    rs = rs_bytes * (P - 1) / P / (COLL_EFF * (P - 1) * bw) if P > 1 else 0.0
    # as parallel.ViewPartialSum deals them: channel parts of the views (balanced_parts); each rank owns the
    # backbone maps of its views (part_owners) and sends the other holders their parts' channel slices at
    # backbone resolution (src / 3), one all-to-all on the exchange stream (round 6): the rank's warp is
    # the fused upsample + warp + B^T of its parts
    weights = [float(a.mean()) for a in activity]
    owner = view_owners([w + 0.05 for w in weights], P)
    w_up = single.get("warp_up", single["warp"] * WARP_UP_RATIO) / N
    cons = single["conv2"] * _tiles(min(Ho, band + 8)) / rows_all + single["conv3"] / P
    best = None
    k = 1
    while C % k == 0 and (k == 1 or C // k >= 64):  # the split the bench takes: the fastest predicted k
        assign, cp = balanced_parts(weights, P, C, k=k)
        frac = cp / C
        prod = max((sum(w_up * frac + conv1_band(0, Ho, [v]) * frac for v, _ in ps)) if ps else 0.0
                   for ps in assign)
        links = fetch_link_bytes(assign, owner, P, 4.0 * B * cp * backbone_px)
        fetch = float(links.max()) / (A2A_EFF * bw) if P > 1 else 0.0
        cand = dict(produce=prod, exchange=rs + fetch, consume=cons, frame=max(prod + cons, rs + fetch), fetch=fetch,
                    fetch_bytes_max_rank=float(max(links.sum(0).max(), links.sum(1).max())), parts_k=k)
        if best is None or cand["frame"] < best["frame"] * 0.98:
            best = cand
        k *= 2
    out["partial"] = best
    # -- gather
    ag = N * slab_view * (P - 1) / P / (COLL_EFF * (P - 1) * bw) if P > 1 else 0.0
    out["gather"] = dict(produce=vmax * w_view * 0.8, exchange=ag, consume=worst + single["conv3"] / P,
                         frame=max(vmax * w_view * 0.8 + worst, ag))
    single_frame = single["warp"] + single["conv1"] + single["conv2"] + single["conv3"]
    for k, v in out.items():
        v["speedup_vs_1gpu"] = single_frame / v["frame"]
    return out


def config_inputs(cfg: int):
    """(N, C, grid, B, per-view activity) of a BASELINE config's synthetic rig."""
    from . import synthetic
    from .geometry import kornia_src_norm_from_dst_norm, projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    acts = [view_tile_activity(kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), up, grid)[0].numpy(),
                               up, grid) for M in projection_matrices(ds)]
    return ds.num_cam, spec["C"], grid, spec["B"], acts


def backbone_pixels(cfg: int) -> float:
    """Pixels of one backbone map at a BASELINE config (the upsampled warp source / 3 per side, ``:64-65``)."""
    from . import synthetic
    up = synthetic.CONFIGS[cfg]["make"]().upsample_shape
    return float((up[0] // 3) * (up[1] // 3))


def predict_config(cfg: int, P: int) -> Dict[str, dict]:
    """``predict`` at a BASELINE config's synthetic rig and measured single-GPU stage times."""
    N, C, grid, B, acts = config_inputs(cfg)
    return predict(N, C, grid, B, P, SINGLE_GPU_MS[cfg], acts, backbone_pixels(cfg))


def choose_mode(cfg: int, P: int) -> str:
    """The strong-scaling mode with the smallest predicted frame time at P ranks."""
    if P <= 1 or cfg not in SINGLE_GPU_MS:
        return "bands"
    pred = predict_config(cfg, P)
    return min(pred, key=lambda k: pred[k]["frame"])
