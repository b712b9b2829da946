"""Per-kernel micro-benchmark of the hot-path kernels at a BASELINE config (GPU box).

    python tools/kbench.py [--config 2] [--reps 20] [--only warp,warpup,conv1,conv2,conv3]

Times each stage alone with HIP events on torch's current stream (the stream the
kernels are launched on) and prints one JSON line per stage.  Used for A/B work on
the kernels and as the target of rocprofv3 --pmc passes.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import build_mc, head_params  # noqa: E402
from mvdet_amd import ProjectFuse, synthetic  # noqa: E402
from mvdet_amd.geometry import projection_matrices  # noqa: E402


def timeit(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for i in range(reps):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    t = [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]
    return float(np.median(t)), float(np.min(t))


def backward_stages(eng, ws, mc, B, ho, wo, N, C, dev):
    """conv1's weight and data gradient as the native training step runs them
    (mvdet_amd/autograd.py), on a random dy1 and the warped slab."""
    from mvdet_amd import _native, autograd, ops
    st = autograd._bwd_state(eng)
    w1 = mc[0].weight
    dy1 = torch.randn(B, w1.shape[0], ho, wo, device=dev).relu_()
    d1 = ops.conv_desc(B, eng.S * eng.Cs, ho, wo, group=eng.Cs, group_stride=B * eng.Cs * ho * wo,
                       batch_stride=eng.Cs * ho * wo)
    eng.pack1.get(w1)
    dw1 = torch.zeros_like(w1)
    wws = autograd._wgrad_ws(st, d1, w1.shape[0], dev)
    lists = autograd._wgrad_lists(eng, st, dev, B)
    cp = st.dgrad1.cout_p
    dslab = torch.empty(ops.split_shape(B, cp, ho, wo), dtype=torch.bfloat16, device=dev)
    # the training step's dgrad input: dy1 also split-bf16 (relu_backward_split_ with y1 > 0
    # everywhere), so the ring kernel runs, with its 12-row output mask
    y1_pos = torch.zeros(ops.split_shape(B, w1.shape[0], ho, wo), dtype=torch.bfloat16, device=dev)
    y1_pos[..., 0, :] = 1.0
    dy1s = torch.empty_like(y1_pos)
    ops.relu_backward_split_(dy1, y1_pos, dy1s)
    cm = eng.conv1_mask(dev, 0, ho, tile_h=ops.dgrad_tile_rows(True, 1))
    sch1 = ops.dgrad_schedule(B, cp, ho, wo, w1.shape[0], cm, C // ops.BN, dev)
    print(json.dumps({"dgrad1_schedule": {"items": sch1.nitems, "split_tiles": sch1.nfix, "pieces": sch1.nslots,
                                          "predicted": round(sch1.predicted, 1),
                                          "predicted_plain": round(sch1.predicted_plain, 1)}}), flush=True)
    flop = 2.0 * B * ho * wo * 9 * N * C * w1.shape[0]
    # conv2 (d2) on a split y1 and a random dy2, as the training step's conv2 backward
    w2 = mc[2].weight
    mid = w2.shape[0]
    y1s = torch.randn(ops.split_shape(B, mid, ho, wo), device=dev).to(torch.bfloat16)
    dy2 = torch.randn(B, mid, ho, wo, device=dev)
    dy2s = torch.randn(ops.split_shape(B, mid, ho, wo), device=dev).to(torch.bfloat16)
    d_y1 = ops.conv_desc(B, mid, ho, wo, group=mid, group_stride=0, batch_stride=mid * ho * wo)
    wws2 = autograd._wgrad_ws(st, d_y1, mid, dev)
    flop2 = 2.0 * B * ho * wo * 9 * mid * mid
    # the training step's form: dy pre-split into bf16 rows (timed with the split) where W % 8 == 0
    rows1 = torch.empty(ops.split_rows_shape(B, w1.shape[0], ho, wo), dtype=torch.bfloat16, device=dev)
    rows2 = torch.empty(ops.split_rows_shape(B, mid, ho, wo), dtype=torch.bfloat16, device=dev)
    pre = wo % 8 == 0
    # the Winograd form (autograd._wgrad1_wino): T of the slab under the forward's mask, D of dy1
    gm1 = eng.conv1_mask(dev, 0, ho)
    t1 = torch.zeros((ops.wino_rows_bytes(d1) + 1) // 2, dtype=torch.bfloat16, device=dev)
    ops.wino_rows(ws.slab, d1, t1, gm1)
    lists_w = ops.wgrad_wino_chunk_lists(gm1, eng.S, B, ho, wo) if gm1 is not None else None
    drows = torch.empty((B, 5, w1.shape[0], -(-ho // 3), wo // 8, 2, 8), dtype=torch.bfloat16, device=dev)
    wwsw = torch.empty((int(_native.load().mvbev_conv3x3_wgrad_wino_workspace_bytes(
        __import__("ctypes").byref(d1), w1.shape[0], 1)) + 3) // 4, device=dev)
    dw1w = torch.zeros_like(w1)
    if pre:
        ops.conv3x3_wgrad(ws.slab, d1, dy1, 1, w1.shape[1], chan_map=eng.pack1._map_dev, dw=dw1, workspace=wws,
                          chunk_lists=lists)
        ops.conv3x3_wgrad_wino(t1, d1, ops.wino_dy_rows(dy1, out=drows), w1.shape[1], chan_map=eng.pack1._map_dev,
                               dw=dw1w, workspace=wwsw, chunk_lists=lists_w)
        nc = N * C
        diff = (dw1w[:, :nc] - dw1[:, :nc]).abs().max().item() / max(dw1[:, :nc].abs().max().item(), 1e-30)
        print(json.dumps({"wgrad1w_vs_wgrad1_normwise": diff}), flush=True)
    t2w = torch.zeros((ops.wino_rows_bytes(d_y1) + 1) // 2, dtype=torch.bfloat16, device=dev)
    ops.wino_rows(y1s, d_y1, t2w, dilation=2)
    drows2 = torch.empty((B, 5, mid, ops.wino_r3(ho, 2), wo // 8, 2, 8), dtype=torch.bfloat16, device=dev)
    wwsw2 = torch.empty((int(_native.load().mvbev_conv3x3_wgrad_wino_workspace_bytes(
        __import__("ctypes").byref(d_y1), mid, 2)) + 3) // 4, device=dev)
    return {
        "wgrad1w": (lambda: ops.conv3x3_wgrad_wino(t1, d1, ops.wino_dy_rows(dy1, out=drows), w1.shape[1],
                                                   chan_map=eng.pack1._map_dev, dw=dw1w, workspace=wwsw,
                                                   chunk_lists=lists_w), flop),
        # conv2's from its forward transform (dilation-2 row tiles; autograd's training default)
        "wgrad2w": (lambda: ops.conv3x3_wgrad_wino(t2w, d_y1, ops.wino_dy_rows(dy2, out=drows2, dilation=2), mid,
                                                   dilation=2, workspace=wwsw2), flop2),
        "wgrad2": (lambda: ops.conv3x3_wgrad(y1s, d_y1, dy2, 2, mid, workspace=wws2,
                                             dy_rows=ops.split_rows(dy2, out=rows2) if pre else None), flop2),
        "wgrad2f": (lambda: ops.conv3x3_wgrad(y1s, d_y1, dy2, 2, mid, workspace=wws2), flop2),
        "dgrad2": (lambda: ops.conv3x3_dgrad(dy2s, st.dgrad2, w2, 2), flop2),
        "wgrad1": (lambda: ops.conv3x3_wgrad(ws.slab, d1, dy1, 1, w1.shape[1], chan_map=eng.pack1._map_dev,
                                             dw=dw1, workspace=wws, chunk_lists=lists,
                                             dy_rows=ops.split_rows(dy1, out=rows1) if pre else None), flop),
        "wgrad1f": (lambda: ops.conv3x3_wgrad(ws.slab, d1, dy1, 1, w1.shape[1], chan_map=eng.pack1._map_dev,
                                              dw=dw1, workspace=wws, chunk_lists=lists), flop),  # fp32 dy
        "dgrad1": (lambda: ops.conv3x3_dgrad(dy1s, st.dgrad1, w1, 1, out=dslab, out_mask=cm,
                                             cot_per_group=C // ops.BN), flop),
        "dgrad1s": (lambda: ops.conv3x3_dgrad(dy1s, st.dgrad1, w1, 1, out=dslab, out_mask=cm,
                                              cot_per_group=C // ops.BN, sched=sch1), flop),  # balanced schedule
    }


def _with(eng, flag, value, fn):
    """Run fn with the engine's boolean option ``flag`` (edge_strip, wino_warp) set to ``value``."""
    keep = getattr(eng, flag)
    setattr(eng, flag, value)
    try:
        return fn()
    finally:
        setattr(eng, flag, keep)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16x3", choices=["fp32", "bf16x3"],
                    help="conv1/conv2 arithmetic: fp32 MFMA or 3xbf16 split (fp32-class accuracy)")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--batch", type=int, default=0, help="override the config's batch size (0 = the config's)")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="warp,conv1,conv2,conv3")
    ap.add_argument("--libs", default="", help="comma-separated libmvbev variants to A/B (interleaved rounds)")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--no-frustum", action="store_true", help="dense conv1 (no frustum mask)")
    ap.add_argument("--check43", action="store_true", help="print the F(4,3) vs F(3,3) difference at full size")
    args = ap.parse_args()
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    B, C, N = (args.batch or spec["B"]), spec["C"], ds.num_cam
    up = tuple(ds.upsample_shape)
    ho, wo = ds.reducedgrid_shape
    dev = torch.device("cuda:0")
    pm = projection_matrices(ds)
    mc = build_mc(C, N, head_params(N, args.config, C), dev)
    eng = ProjectFuse(pm, up, (ho, wo), C, precision=args.precision, frustum=not args.no_frustum,
                      wino_conv1=False, wino_conv2=False)  # the direct conv stages (the Winograd ones use weng)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=v, device=dev) for v in range(N)]
    cfeats = [f.contiguous(memory_format=torch.channels_last) for f in feats]
    bfeats = [synthetic.backbone_features(B, C, [u // 3 for u in up], seed=v, device=dev) for v in range(N)]
    cbfeats = [f.contiguous(memory_format=torch.channels_last) for f in bfeats]
    ws = eng.workspace(B, dev)
    with torch.no_grad():
        for v in range(N):
            eng.warp_view(ws, v, feats[v])
        eng.fuse(ws, mc)
        from mvdet_amd import ops
        # the slab path (wino_warp off) so the transform stages run on real data; warpw / warpupw
        # switch the fused warp on (and leave T from the warp: run them last)
        weng = ProjectFuse(pm, up, (ho, wo), C, precision=args.precision, frustum=not args.no_frustum,
                           wino_conv1=True, wino_warp=False, wino43=False)  # (F(3,3): the F(4,3) stages below)
        wws = weng.workspace(B, dev)
        weng.warp_views(wws, list(range(N)), feats)
        weng.conv1(wws, mc[0])
        wd1 = ops.conv_desc(B, weng.S * weng.Cs, ho, wo, group=weng.Cs, group_stride=B * weng.Cs * ho * wo,
                            batch_stride=weng.Cs * ho * wo)
        wgm = weng.conv1_mask(dev, 0, ho)
        # row-Winograd F(4,3) (ABI 12400, xi-major): conv1 from the slab's T43 (16 x 32 mask / order) and
        # conv2 -> conv3 partials from y1's dilation-2 T43, beside the F(3,3) stages winoconv / conv23w
        wgm43 = weng.conv1_mask(dev, 0, ho, tile_h=ops.WINO43_TILE_ROWS)
        word43 = ops.heavy_first_order(wgm43, B) if wgm43 is not None else None
        t43 = torch.zeros((ops.wino43_rows_bytes(wd1) + 1) // 2, dtype=torch.bfloat16, device=dev)
        ops.wino43_rows(wws.slab, wd1, t43, wgm43)
        pk43 = ops.pack_wino43(mc[0].weight, weng.pack1w.map_dev(dev))
        d2 = weng._conv2_desc(wws)
        t243 = torch.zeros((ops.wino43_rows_bytes(d2) + 1) // 2, dtype=torch.bfloat16, device=dev)
        pk243 = ops.pack_wino43(mc[2].weight)
        p3_43 = torch.empty(ops.conv3x3_cout1_partials_bytes(d2, 512) // 4, dtype=torch.float32, device=dev)
        y1_43 = torch.empty_like(wws.y1)
        t43w = torch.zeros_like(t43)  # (warpw43's T43: its own zero-filled buffer, written only by that geometry)

        def conv23w43():
            ops.wino43_rows(wws.y1, d2, t243, dilation=2)
            ops.conv3x3_wino43_then_cout1_partials(t243, d2, pk243, 512, mc[2].bias, True, mc[4].weight, p3_43)
            return ops.cout1_from_partials(p3_43, d2, 512, 4, wws.band[0], wws.band[1] - wws.band[0])

        stages = {
            "winorows43": (lambda: ops.wino43_rows(wws.slab, wd1, t43, wgm43), None),
            "winoconv43": (lambda: ops.conv3x3_wino43(t43, wd1, pk43, 512, init=weng.coord_term(mc[0]), relu=True,
                                                      out=y1_43, group_mask=wgm43, tile_order=word43),
                           2.0 * B * ho * wo * 9 * N * C * 512),
            # the same without the coord-term init in the epilogue (what reading init costs; not a valid conv1)
            "winoconv_noinit": (lambda: ops.conv3x3_wino(wws.wino_t, wd1, weng.pack1w.get(mc[0].weight), 512,
                                                         init=None, relu=True, out=wws.y1, group_mask=wgm,
                                                         tile_order=weng.conv1_order(dev, 0, ho, B, grid=True)), None),
            "winoconv43_noinit": (lambda: ops.conv3x3_wino43(t43, wd1, pk43, 512, init=None, relu=True, out=y1_43,
                                                             group_mask=wgm43, tile_order=word43), None),
            "conv2w43": (lambda: ops.conv3x3_wino43_then_cout1_partials(t243, d2, pk243, 512, mc[2].bias, True,
                                                                        mc[4].weight, p3_43),
                         2.0 * B * ho * wo * 9 * 512 * 512),
            "winorows2_43": (lambda: ops.wino43_rows(wws.y1, d2, t243, dilation=2), None),
            "conv23w43": (conv23w43, 2.0 * B * ho * wo * 9 * 512 * 512),
            "warp": (lambda: eng.warp_views(ws, list(range(N)), feats), None),
            "warpup": (lambda: eng.warp_views_upsampled(ws, list(range(N)), bfeats), None),
            "warp1": (lambda: [eng.warp_view(ws, v, feats[v]) for v in range(N)], None),
            "conv1": (lambda: eng.conv1(ws, mc[0]), 2.0 * B * ho * wo * 9 * N * C * 512),
            "conv1g": (lambda: _with(eng, "edge_strip", False, lambda: eng.conv1(ws, mc[0])),
                       2.0 * B * ho * wo * 9 * N * C * 512),  # 12 x 32 grid tiles
            # row-Winograd conv1 (ProjectFuse(wino_conv1=True)): transform + conv, and each alone
            "conv1w": (lambda: weng.conv1(wws, mc[0]), 2.0 * B * ho * wo * 9 * N * C * 512),
            "winorows": (lambda: ops.wino_rows(wws.slab, wd1, wws.wino_t, wgm), None),
            "warpw": (lambda: _with(weng, "wino_warp", True, lambda: weng.warp_views(wws, list(range(N)), feats)),
                      None),  # warp + B^T in one pass (wino_warp; leaves T from the warp, run it last)
            # the same writing T43 (MVBEV_WARP_WINO43: the F(4,3) engine's fused warp) into its own buffer
            "warpw43": (lambda: ops.warp_views_wino_rows_into(
                feats, [weng.m_norm_cpu[c] for c in range(N)], t43w, list(range(N)), weng.Cs, weng.S * weng.Cs, ho, wo,
                dst_zeroed=True, boxes=weng._wino_boxes(dev, list(range(N)), form=4), form=4), None),
            # round 6: the same without the per-geometry box table (each block reduces its own box)
            "warpw0": (lambda: _with(weng, "_wino_boxes", lambda dev, cams, bb=None: None, lambda: _with(
                weng, "wino_warp", True, lambda: weng.warp_views(wws, list(range(N)), feats))), None),
            "warpwcl0": (lambda: _with(weng, "_wino_boxes", lambda dev, cams, bb=None: None, lambda: _with(
                weng, "wino_warp", True, lambda: weng.warp_views(wws, list(range(N)), cfeats))), None),
            # the same on channels-last features (warp_wino_cl_kernel)
            "warpwcl": (lambda: _with(weng, "wino_warp", True, lambda: weng.warp_views(wws, list(range(N)), cfeats)),
                        None),
            # the fused upsample warp on NCHW maps without the channels-last copy (the round-3/4 NCHW kernel),
            # and on maps that are channels-last already
            "warpupwn": (lambda: _with(weng, "cl_upsample", False, lambda: _with(weng, "wino_warp", True,
                         lambda: weng.warp_views_upsampled(wws, list(range(N)), bfeats))), None),
            # NCHW maps copied to channels-last first (cl_upsample), then the line-per-pixel kernel
            "warpupwt": (lambda: _with(weng, "cl_upsample", True, lambda: _with(weng, "wino_warp", True,
                         lambda: weng.warp_views_upsampled(wws, list(range(N)), bfeats))), None),
            "warpupwcl0": (lambda: _with(weng, "_wino_boxes", lambda dev, cams, bb=None: None, lambda: _with(
                weng, "wino_warp", True, lambda: weng.warp_views_upsampled(wws, list(range(N)), cbfeats))), None),
            "warpupwcl": (lambda: _with(weng, "wino_warp", True,
                                        lambda: weng.warp_views_upsampled(wws, list(range(N)), cbfeats)), None),
            "warpupw": (lambda: _with(weng, "wino_warp", True,
                                      lambda: weng.warp_views_upsampled(wws, list(range(N)), bfeats)), None),
            "winoconv": (lambda: ops.conv3x3_wino(wws.wino_t, wd1, weng.pack1w.get(mc[0].weight), 512,
                                                  init=weng.coord_term(mc[0]), relu=True, out=wws.y1,
                                                  group_mask=wgm, tile_order=weng.conv1_order(dev, 0, ho, B, grid=True)),
                         2.0 * B * ho * wo * 9 * N * C * 512),
            "conv2": (lambda: eng.conv2(ws, mc[2]), 2.0 * B * ho * wo * 9 * 512 * 512),
            "conv3": (lambda: eng.conv3(ws, mc[4]), None),
            # conv2 -> conv3 fused (the default inference path): partials epilogue + reduce
            "conv23": (lambda: (eng.conv2_partials(ws, mc[2], mc[4]), eng.conv3_from_partials(ws, mc[4])),
                       2.0 * B * ho * wo * 9 * 512 * 512),
            # the same with the row-Winograd conv2 (dilation-2 transform of y1 + conv; inference default)
            "conv23w": (lambda: (weng.conv2_partials(wws, mc[2], mc[4]), weng.conv3_from_partials(wws, mc[4])),
                        2.0 * B * ho * wo * 9 * 512 * 512),
        }
        if {"adjup", "adj", "adjpix", "adjuppix"} & set(args.only.split(",")):
            # the warp adjoints of the training step (autograd.py) on a random split grad_out
            from mvdet_amd import ops
            hb = tuple(bfeats[0].shape[2:])
            douts = [torch.randn(ops.split_shape(B, C, ho, wo), device=dev).to(torch.bfloat16) for _ in range(N)]
            gs = [torch.empty(B, C, *hb, device=dev) for _ in range(N)]
            gsu = [torch.empty(B, C, *up, device=dev) for _ in range(N)]
            plu = [ops.WarpAdjointPlan(eng.m_norm_cpu[v], up, (ho, wo), dev, backbone_hw=hb) for v in range(N)]
            stages["adjup"] = ((lambda: ops.warp_views_adjoint(douts, plu, gs)), None)
            pl = [ops.WarpAdjointPlan(eng.m_norm_cpu[v], up, (ho, wo), dev) for v in range(N)]
            stages["adj"] = ((lambda: ops.warp_views_adjoint(douts, pl, gsu)), None)
            # the same gradients in the pixel-major split layout (one [B, ho, wo, N * C / 8, 2, 8] tensor,
            # the views' group slices), as the training step's conv1 dgrad writes them (ABI 12100)
            g8 = C // ops.KC
            dpix = torch.stack([d.permute(0, 2, 3, 1, 4, 5) for d in douts], dim=3).reshape(
                B, ho, wo, N * g8, 2, ops.KC).contiguous()
            dpv = [dpix[:, :, :, v * g8:(v + 1) * g8] for v in range(N)]
            stages["adjpix"] = ((lambda: ops.warp_views_adjoint(dpv, pl, gsu, pixel_major=True)), None)
            stages["adjuppix"] = ((lambda: ops.warp_views_adjoint(dpv, plu, gs, pixel_major=True)), None)
        if {"wgrad1", "wgrad1w", "wgrad2w", "wgrad1f", "dgrad1", "dgrad1s", "wgrad2", "wgrad2f", "dgrad2"} & set(args.only.split(",")):
            stages.update(backward_stages(eng, ws, mc, B, ho, wo, N, C, dev))
        if args.check43:  # F(4,3) vs F(3,3) at this config's full size (normwise over y1 and the map)
            weng.conv1(wws, mc[0])
            y1_33 = weng.y1_fp32(wws).clone()
            ops.conv3x3_wino43(t43, wd1, pk43, 512, init=weng.coord_term(mc[0]), relu=True, out=y1_43,
                               group_mask=wgm43, tile_order=word43)
            y1_43f = ops.split_decode(y1_43, 512) if y1_43.dtype == torch.bfloat16 else y1_43
            m33 = (weng.conv2_partials(wws, mc[2], mc[4]), weng.conv3_from_partials(wws, mc[4]))[1].clone()
            m43 = conv23w43()
            def active(m, th):  # fraction of conv1's dense (pixel, slot) work a th x 32 tile mask keeps
                if m is None:
                    return 1.0
                tx = -(-wo // 32)
                bits = [bin(int(v) & 0xFFFFFFFF).count("1") for v in m.cpu().tolist()]
                return sum(bb * min(th, ho - (t // tx) * th) * min(32, wo - (t % tx) * 32)
                           for t, bb in enumerate(bits[:tx * -(-ho // th)])) / (ho * wo * weng.S)
            print(json.dumps({"check43": "mask_active", "config": args.config, "rows12": active(wgm, 12),
                              "rows16": active(wgm43, 16)}), flush=True)
            for name, a_, b_ in (("y1", y1_43f, y1_33), ("map_conv23", m43, m33)):
                print(json.dumps({"check43": name, "config": args.config, "normwise": float(
                    (a_.double() - b_.double()).abs().max() / b_.double().abs().max())}), flush=True)
        from mvdet_amd import _native
        libs = [("default", _native.load())]
        for path in filter(None, args.libs.split(",")):
            libs.append((Path(path).stem, _native.load(path)))
        for rnd in range(args.rounds):
            for lname, lib in libs:
                _native._lib = lib
                for name in args.only.split(","):
                    fn, flop = stages[name]
                    med, mn = timeit(fn, args.reps)
                    rec = {"stage": name, "lib": lname, "round": rnd, "config": args.config,
                           "median_ms": round(med, 4), "min_ms": round(mn, 4)}
                    if flop:
                        rec["TFLOPs"] = round(flop / (med * 1e-3) / 1e12, 2)
                    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
