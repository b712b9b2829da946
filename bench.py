"""Benchmark of the MVDet project+fuse hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2] [--no-cpu-baseline]

A *step* is one pass of the hot path over one frame batch of synthetic input
already resident in HBM: the warp of every view (a5), the zero-copy concat (a6),
conv1+ReLU, conv2+ReLU, conv3 (a7-a9); the identity interpolate (a10) is elided.
The backbone, the 3x upsample (a4) and the image head are NOT in the step
(SURVEY §8(d)).  Metric: frames/s (= B * K / wall).  N>1 (torchrun, one rank per
GPU) runs the view-parallel path of ``mvdet_amd.parallel``.

Rank 0 prints ONE JSON line; see DESIGN.md §Measurement for every field.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_MFMA_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: fp32 matrix peak (spec)


def progress(msg: str) -> None:
    """A progress line on stderr (a long default run — the CPU baselines take minutes — keeps writing,
    so a supervisor that watches the output does not take it for hung)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def build_mc(C, num_cam, params, device):
    mc = torch.nn.Sequential(torch.nn.Conv2d(C * num_cam + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False))
    if params is not None:
        mc.load_state_dict({k.replace("map_classifier.", ""): torch.from_numpy(v)
                            for k, v in params.items() if k.startswith("map_classifier.")})
    return mc.to(device)


def head_params(num_cam, seed, C):
    """Default-Conv2d-bound uniform init (same recipe as the test fixtures)."""
    rng = np.random.default_rng(seed)
    cin = C * num_cam + 2
    shapes = {"map_classifier.0.weight": (512, cin, 3, 3), "map_classifier.0.bias": (512,),
              "map_classifier.2.weight": (512, 512, 3, 3), "map_classifier.2.bias": (512,),
              "map_classifier.4.weight": (1, 512, 3, 3)}
    fan = {"map_classifier.0": cin * 9, "map_classifier.2": 512 * 9, "map_classifier.4": 512 * 9}
    out = {}
    for k, s in shapes.items():
        b = 1.0 / np.sqrt(fan[k.rsplit(".", 1)[0]])
        out[k] = rng.uniform(-b, b, size=s).astype(np.float32)
    return out


def cpu_baseline(ds, B, C, pm, params, frames: int, config: int = 2, warmups: int = 2, single_frames: int = 3,
                 single_warmups: int = 1, single_band: int = 1):
    """The oracle (reference CPU path restated over torch-CPU ops) on the host cores:
    ``warmups`` untimed frames, then the median of ``frames`` timed ones (2 warm-ups,
    >= 5 timed, median); the reference's own one-thread setting (main.py:3) as the median of
    ``single_frames`` after ``single_warmups`` warm-ups (0 = skipped).  ``single_band`` > 1 bounds the
    one-thread sample of the large configs (a whole cfg3 / cfg5 frame is ~100 s of one core): the same
    frame over the output rows [0, H / single_band) (the warp into that band, the three convs over it with
    their zero padding), its time x H / band rows; every output row costs the same
    grid_sample + conv work, so the scaled band is the frame's time less one call's fixed overheads (checked
    on cfg2 here: the x4 band gave 0.0559 frames/s against 0.0525 for whole frames, i.e. it errs ~6% in the
    CPU's favour)."""
    from mvdet_amd import synthetic
    from oracle import cpu_path
    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    torch.set_num_threads(threads)
    up = ds.upsample_shape
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=1000 * config + v)
             for v in range(ds.num_cam)]
    tp = {k: torch.from_numpy(v) for k, v in params.items()}
    mats = [M.numpy() for M in pm]
    grid = tuple(ds.reducedgrid_shape)

    def frame(stages=None, band=1):
        g, ms = grid, mats
        if band > 1:  # output rows [0, H / band): the band starts at row 0, so the matrices stay
            g = (max(1, grid[0] // band), grid[1])
        t = time.perf_counter()
        cpu_path.project_fuse(feats, ms, g, tp, timings=stages)
        dt = (time.perf_counter() - t) * (grid[0] / g[0])
        progress(f"cpu baseline cfg{config}: frame {dt:.2f} s ({torch.get_num_threads()} threads"
                 + (f", rows [0, {g[0]}) x {grid[0] / g[0]:.2f})" if band > 1 else ")"))
        return dt

    with torch.no_grad():
        for _ in range(warmups):
            frame()
        stages = {}
        times = [frame(stages) for _ in range(frames)]
        single = None
        if single_frames:
            # the reference's own setting (main.py:3, OMP_NUM_THREADS=1)
            torch.set_num_threads(1)
            for _ in range(single_warmups):
                frame(band=single_band)
            t1 = [frame(band=single_band) for _ in range(single_frames)]
            torch.set_num_threads(threads)
            rows = max(1, grid[0] // single_band)
            single = dict(value=round(B / float(np.median(t1)), 4), unit="frames/s", cores=1,
                          sample=f"median of {single_frames} frame(s) after {single_warmups} warm-up(s) with "
                                 "torch.set_num_threads(1) (main.py:3 OMP_NUM_THREADS=1)"
                                 + ("" if single_warmups else " (right after the multi-thread frames)")
                                 + (f"; bounded sample: output rows [0, {rows}) of {grid[0]} (warp + 3 convs over "
                                    f"the band), time x {grid[0] / rows:.2f}" if rows < grid[0] else ""))
    dt = float(np.median(times))
    return dict(value=round(B / dt, 4), unit="frames/s", cores=threads, kind="port", single_thread=single,
                sample=f"median of {frames} frame(s) (B={B}) of the bench workload after {warmups} warm-up(s) "
                       f"(BASELINE.md:26); oracle/cpu_path.py (kornia-0.6.11 restatement over torch-CPU grid_sample "
                       f"+ torch.cat + 3x F.conv2d) on identical synthetic inputs; last frame stages (s): "
                       + ", ".join(f"{k}={v:.3f}" for k, v in stages.items()))


DTYPE_LABEL = {"fp32": "f32 (fp32-input MFMA, exact fp32 products, fp32 accumulate)",
               "bf16x3": "f32 (3xbf16-split products hi*hi+hi*lo+lo*hi on the bf16 MFMA, fp32 accumulate)"}
BF16_MFMA_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16


def mfma_probe(settle_s: float = 1.5):
    """Sustained bf16 MFMA TFLOP/s of this device now (tools/mfma_shape_bench.hip built as
    mvdet_amd/lib/libmfmaprobe.so by __graft_entry__.build()); None when not built."""
    import ctypes
    lib_path = ROOT / "mvdet_amd" / "lib" / "libmfmaprobe.so"
    if not lib_path.exists():
        return None
    lib = ctypes.CDLL(str(lib_path))
    lib.mfma_probe_tflops.restype = ctypes.c_double
    lib.mfma_probe_tflops.argtypes = [ctypes.c_int, ctypes.c_double]
    torch.cuda.synchronize()
    v = lib.mfma_probe_tflops(0, settle_s)
    return v if v > 0 else None


def run_single(args, precision, steps, warmup, with_cpu, config=None, cpu_plan=None, layout=None):
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices, touched_footprint

    config = args.config if config is None else config
    progress(f"run_single cfg{config} {precision} {layout or args.layout}")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    spec = synthetic.CONFIGS[config]
    ds = spec["make"]()
    B, C = spec["B"], spec["C"]
    N = ds.num_cam
    up = tuple(ds.upsample_shape)
    ho, wo = ds.reducedgrid_shape
    pm = projection_matrices(ds)
    params = head_params(N, seed=config, C=C)
    mc = build_mc(C, N, params, dev)
    half = config == 4  # fp16 features (BASELINE configs[3]); round 5: read by the fused warp + B^T (fp32 math,
    # split-bf16 T) like fp32 ones — no fp16 slab (the fp32-MFMA alt precision keeps an fp16 slab)
    eng = ProjectFuse(pm, up, (ho, wo), C, precision=precision,
                      slab_dtype=torch.float16 if half and precision == "fp32" else torch.float32,
                      wino_conv1=args.conv1 == "wino" and precision == "bf16x3",
                      wino_conv2=args.conv1 == "wino" and precision == "bf16x3")
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=1000 * config + v,
                                          device=dev).to(torch.float16 if half else torch.float32)
             for v in range(N)]
    layout = layout or args.layout
    if layout == "channels_last":  # the same logical [B, C, H, W] tensors in torch's channels_last memory format
        feats = [f.contiguous(memory_format=torch.channels_last) for f in feats]
    ws = eng.workspace(B, dev)
    views = list(range(N))

    K, W = steps, warmup
    ev = {k: [torch.cuda.Event(enable_timing=True) for _ in range(K)]
          for k in ("warp", "conv1", "conv1_wino", "conv2", "conv3", "guard")}
    end_ev = [torch.cuda.Event(enable_timing=True) for _ in range(K)]

    def step(i=None):
        if i is not None:
            ev["warp"][i].record()
        eng.warp_views(ws, views, feats)
        mark = (lambda stage: ev[stage][i].record()) if i is not None else None
        return eng.fuse(ws, mc, mark=mark)

    with torch.no_grad():
        for _ in range(W):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            step(i)
            end_ev[i].record()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0

    def avg(a, b):
        return float(np.mean([a[i].elapsed_time(b[i]) for i in range(K)]))

    t_warp = avg(ev["warp"], ev["conv1"])
    t_c1 = avg(ev["conv1"], ev["conv2"])
    wino = eng.wino_active(dev)  # conv1 = conv_wino_kernel (its row transform came from the warp)
    t_rows = avg(ev["conv1"], ev["conv1_wino"]) if wino else 0.0
    t_c1k = t_c1 - t_rows  # conv1's conv kernel alone
    t_c2 = avg(ev["conv2"], ev["conv3"])
    # the non-finite guard's four gated launches after conv3 (they exit at once on finite features)
    guarded = ws.guard_src is not None
    t_c3 = avg(ev["conv3"], ev["guard"] if guarded else end_ev)
    t_guard = avg(ev["guard"], end_ev) if guarded else 0.0
    wino2 = eng.wino_conv2_active(ws)  # conv2 -> conv3 partials as row-Winograd
    # the row-Winograd forms that ran (F(4,3) where ProjectFuse.wino43_pays: 6 transformed rows per 4 output rows,
    # 1/2 of the direct MFMA work; F(3,3): 5 per 3, 5/9)
    f1 = eng.conv1_form(ws) if wino else 0
    f2 = eng.conv2_form(ws) if wino2 else 0
    wf = {0: 1.0, 3: 5.0 / 9.0, 4: 0.5}
    value = B * K / dt
    # algorithmic work; conv1 runs over the N*C view channels per step (the
    # 2 coord channels are folded into a per-weight-version init term)
    conv1_flop = 2.0 * B * ho * wo * 9 * (N * C) * 512
    conv2_flop = 2.0 * B * ho * wo * 9 * 512 * 512
    s = 2 if half else 4  # bytes per element (fp16 features at cfg4)
    tv = [touched_footprint(M.numpy(), up, (ho, wo)) for M in pm]
    # warp bytes = sum_v s * B * C * (T_v + Ho * Wo) — the touched source pixels and the warped
    # output at the source's element size, whatever the kernel physically writes (the
    # dense 5/3-size T is what the fused warp + B^T may write at most, not the algorithm's bytes)
    warp_bytes = sum(s * B * C * (t + ho * wo) for t in tv)
    # what the kernel's output buffer would take if dense: the slab, or with the fused B^T conv1's row transform
    # T (5 split-bf16 rows per 3-row tile, 4 B per element; it writes only the frustum mask's tiles)
    warp_out_dense = ((N * B * C * 4 * 6 * 4 * -(-ho // 16) * wo if f1 == 4 else N * B * C * 4 * 5 * 4 * -(-ho // 12) * wo)
                      if eng.wino_warp else N * B * C * eng.slab_dtype.itemsize * ho * wo)
    # conv3's stage: with conv2 -> conv3 fused (bf16x3) it reads the [B, 8 sets, 9 taps, rows, Wo] fp32
    # partials conv2's epilogue wrote (y2 never reaches HBM) and writes the map; on a stored y2 (fp32
    # path) it reads y2's 512 channels
    fused3 = eng.conv3_fused_applies(ws)
    y2rows = ws.y2_rows[1] - ws.y2_rows[0]
    conv3_read = 4.0 * B * (2 * 512 // 128) * 9 * y2rows * wo if fused3 else 4.0 * B * 512 * y2rows * wo
    conv3_bytes = conv3_read + 4.0 * B * ho * wo
    conv1_alg_tfs = conv1_flop / (t_c1k * 1e-3) / 1e12  # over the conv kernel's time
    active = eng.conv1_active_fraction(dev, *ws.y1_rows[:1], ws.y1_rows[1] - ws.y1_rows[0], grid=wino,
                                       tile_h=16 if f1 == 4 else None) if precision == "bf16x3" else 1.0
    # the end-to-end floor prices the algorithm that executes: conv1's frustum-active products, the
    # row-Winograd forms at 5/9 of the direct MFMA work, 3 bf16 passes (bf16x3) or the fp32 MFMA peak
    w1 = wf[f1]
    w2 = wf[f2]
    mfma_s = (3 * (active * w1 * conv1_flop + w2 * conv2_flop) / (BF16_MFMA_PEAK_TFS * 1e12) if precision == "bf16x3"
              else (active * conv1_flop + conv2_flop) / (FP32_MFMA_PEAK_TFS * 1e12))
    hbm_s = (warp_bytes + conv3_bytes) / (HBM_PEAK_GBS * 1e9)
    e2e_floor_ms = 1e3 * (hbm_s + mfma_s)
    if precision == "bf16x3":
        # bf16 MFMA work the split needs: 3 passes per fp32 product (no padding MFMAs; the
        # tile-edge columns a 32-wide tile computes past W=360 are waste, not counted).
        # Algorithmic = the reference's dense conv; the frustum mask executes `active` of it.
        # Winograd F(3,3) along the rows executes 5 of the direct conv's 9 MFMA K-blocks per
        # (chunk, kernel column): its MFMA work is 5/9 of the direct count
        achieved, peak = conv1_alg_tfs * 3 * w1, BF16_MFMA_PEAK_TFS
        kname = ("conv_wino43_kernel (conv1: row-Winograd F(4,3) walked xi-major, 3xbf16 MFMA, LDS-DMA unit ring, "
                 "frustum-masked 16 x 32 tiles)" if f1 == 4 else
                 "conv_wino_kernel (conv1: row-Winograd F(3,3), 3xbf16 MFMA, LDS-DMA unit ring, frustum-masked)"
                 if wino else "conv_ring_kernel (conv1: 3xbf16 MFMA, LDS-DMA ring, frustum-masked)")
    else:
        achieved, peak = conv1_alg_tfs, FP32_MFMA_PEAK_TFS
        kname = "conv3x3_mfma_f32 (conv1)"
    sustained = mfma_probe() if precision == "bf16x3" and not args.no_probe else None
    traffic, warp_traffic, traffic_src = None, None, None
    tfile = ROOT / "profiles" / f"traffic_cfg{config}_{precision}{'_wino' if wino else ''}.json"
    if tfile.exists():
        tj = json.loads(tfile.read_text())
        traffic, warp_traffic = tj.get("conv1_hbm_bytes_per_launch"), tj.get("warp_hbm_bytes_per_launch")
        warp_traffic = tj.get("warp_cl_hbm_bytes_per_launch") if layout == "channels_last" else warp_traffic
        traffic_src = (f"{tfile.relative_to(ROOT)}: rocprofv3 PMC passes of this kernel (committed profile, not "
                       f"measured in this run: PMC collection needs its own rocprofv3 runs)")
    res = {
        "value": round(value, 3),
        "ms_per_step": round(dt * 1e3 / K, 4),
        "dtype": DTYPE_LABEL[precision],
        "config": {"workload": f"cfg{config}: {spec['name']}", "views": N, "channels": C, "batch": B,
                   "src_hw": list(up), "grid_hw": [ho, wo], "precision": precision,
                   "storage": ("fp16 features" + (", fp16 slab" if eng.slab_dtype == torch.float16 else
                                                     ", fp32-math warp into a split-bf16 T") if half else "fp32"),
                   "feature_layout": layout, "parallelism": "single GPU"},
        # achieved/frac = the MFMA work conv1 actually has to do (the frustum-masked products;
        # the skipped ones are exact zeros) over its measured time: the MFMA utilisation.
        # The reference's dense FLOP count over the same time is kept as dense_* (it reads
        # above the MFMA rate the kernel really sustains, by 1/active).
        "roofline": {"kernel": kname, "bound": "mfma", "achieved": round(achieved * active, 2), "peak": peak,
                     "unit": "TFLOP/s", "frac": round(achieved * active / peak, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "basis": (("3 bf16 MFMA passes x " + ("1/2 (row Winograd F(4,3))" if f1 == 4 else
                                                               "5/9 (row Winograd F(3,3))") +
                                " x 2*B*Ho*Wo*9*(N*C)*512 x frustum_active_fraction over the conv kernel's time" if wino else
                                "3 bf16 MFMA passes x 2*B*Ho*Wo*9*(N*C)*512 x frustum_active_fraction")
                               if precision == "bf16x3" else "2*B*Ho*Wo*9*(N*C)*512 at the fp32 MFMA peak"),
                     "frustum_active_fraction": round(active, 4),
                     "dense_algorithmic_achieved": round(achieved, 2),
                     "dense_algorithmic_frac": round(achieved / peak, 4),
                     "dense_fp32_equiv_tflops": round(conv1_alg_tfs, 2),
                     # the rate this device holds right after the timed steps on a bare
                     # 32x32x16 bf16 MFMA loop over random operands (the chip lowers its clock
                     # under MFMA load: MI355X_MICROARCH.md "DVFS give-back"), and conv1's
                     # executed rate as a fraction of it
                     "sustained_peak": round(sustained, 1) if sustained else None,
                     "frac_of_sustained": round(achieved * active / sustained, 4) if sustained else None,
                     # the direct conv's executed bf16 work over conv1's whole time (transform included)
                     "direct_equiv_achieved": round(3 * conv1_flop * active / (t_c1 * 1e-3) / 1e12, 2)
                     if precision == "bf16x3" else None},
        "stages_ms": {"warp_all_views": round(t_warp, 4), "conv1": round(t_c1, 4), "conv2": round(t_c2, 4),
                      "conv3": round(t_c3, 4), "nonfinite_guard": round(t_guard, 4),
                      **({"conv1_wino_rows": round(t_rows, 4), "conv1_wino_conv": round(t_c1k, 4)} if wino else {})},
        # SURVEY §8(d) "achieved fraction": the stages' roofline floors over the measured step;
        # conv1+conv2 priced as the 3 bf16 MFMA passes the split executes (bf16x3) or at the
        # fp32 MFMA peak (fp32); conv1 counted for its frustum-active products only (the
        # skipped ones are exact zeros), the dense count kept as dense_*
        "e2e_roofline": {
            "floor_ms": round(e2e_floor_ms, 4),
            "frac": round(e2e_floor_ms / (dt * 1e3 / K), 4),
            "basis": "warp_bytes/8 TB/s + (conv1 flop x frustum_active" + {0: "", 3: " x 5/9", 4: " x 1/2"}[f1] +
                     " + conv2 flop" + {0: "", 3: " x 5/9", 4: " x 1/2"}[f2] + ") " +
                     ("x3 / 2.5 PF bf16" if precision == "bf16x3" else "/ 157.3 TF fp32") +
                     " + conv3_bytes/8 TB/s (the executed algorithm)",
        },
        "stage_roofline": {
            "warp": {"bound": "hbm", "algorithmic_bytes": warp_bytes,
                     "algorithmic_basis": "SURVEY §8(d): sum_v s*B*C*(T_v + Ho*Wo), T_v = touched source pixels",
                     # with the Winograd conv1 the warp writes the row transform T (warp_wino_kernel:
                     # 5/3 of the slab's rows, the separate transform gone), so its time includes B^T
                     "output": (("row-Winograd T43 (warp + F(4,3) B^T fused)" if f1 == 4 else
                                 "row-Winograd T (warp + B^T fused)") if eng.wino_warp else "split-bf16 slab"),
                     "output_dense_bytes": warp_out_dense,
                     "achieved_GBs": round(warp_bytes / (t_warp * 1e-3) / 1e9, 1), "peak_GBs": HBM_PEAK_GBS,
                     # PMC bytes (read at 128-B granules: NCHW rows are gathered, not streamed)
                     "traffic": warp_traffic,
                     "physical_GBs": round(warp_traffic / (t_warp * 1e-3) / 1e9, 1) if warp_traffic else None},
            "conv2": {"bound": "mfma", "algorithmic_fp32_TFs": round(conv2_flop / (t_c2 * 1e-3) / 1e12, 2),
                      # executed bf16 MFMA work over conv2's stage time (its dilation-2 row transform
                      # included when row-Winograd: 3 passes x 5/9 of the direct products)
                      "executed_bf16_frac": (round(3 * conv2_flop * w2 / (t_c2 * 1e-3)
                                                   / (BF16_MFMA_PEAK_TFS * 1e12), 4)
                                             if precision == "bf16x3" else None),
                      "form": {0: "direct", 3: "row-Winograd F(3,3), dilation 2",
                               4: "row-Winograd F(4,3) xi-major, dilation 2"}[f2]},
            "conv3": {"bound": "hbm", "algorithmic_bytes": conv3_bytes,
                      "reads": "conv2's conv3 partials [B, 8, 9, rows, Wo] fp32" if fused3 else "y2 [B, 512, rows, Wo] fp32",
                      "achieved_GBs": round(conv3_bytes / (t_c3 * 1e-3) / 1e9, 1), "peak_GBs": HBM_PEAK_GBS},
        },
    }
    if with_cpu:
        plan = cpu_plan or dict(frames=args.cpu_frames or 5, warmups=2, single_frames=3)
        res["cpu_baseline"] = cpu_baseline(ds, 1 if half else B, C, pm, params, config=config, **plan)
    return res


def run_plus_a4(args, precision, steps, warmup):
    """The "+a4" variant: the step starts from the
    backbone-resolution maps, so the 3x upsample of :65 is inside the timed region.
    fused = mvbev_warp_views_upsampled (the upsampled tensor never exists) + fusion;
    unfused = torch F.interpolate on the GPU + the warp + fusion (what the reference does)."""
    import torch.nn.functional as F
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices

    progress("plus_a4")
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    spec = synthetic.CONFIGS[args.config]
    ds = spec["make"]()
    B, C, N = spec["B"], spec["C"], ds.num_cam
    up = tuple(ds.upsample_shape)
    lo = [u // 3 for u in up]
    ho, wo = ds.reducedgrid_shape
    pm = projection_matrices(ds)
    mc = build_mc(C, N, head_params(N, seed=args.config, C=C), dev)
    eng = ProjectFuse(pm, up, (ho, wo), C, precision=precision,
                      wino_conv1=args.conv1 == "wino" and precision == "bf16x3",
                      wino_conv2=args.conv1 == "wino" and precision == "bf16x3")
    flo = [synthetic.backbone_features(B, C, lo, seed=1000 * args.config + v, device=dev) for v in range(N)]
    ws = eng.workspace(B, dev)
    views = list(range(N))
    out = {}
    flo_cl = [f.contiguous(memory_format=torch.channels_last) for f in flo]
    for mode in ("fused", "unfused", "fused_channels_last"):
        e0 = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
        e1 = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
        e2 = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]

        def step(i=None):
            if i is not None:
                e0[i].record()
            if mode == "fused":
                eng.warp_views_upsampled(ws, views, flo)
            elif mode == "fused_channels_last":  # the same maps in channels_last memory format
                eng.warp_views_upsampled(ws, views, flo_cl)
            else:
                eng.warp_views(ws, views, [F.interpolate(f, list(up), mode="bilinear") for f in flo])
            if i is not None:
                e1[i].record()
            eng.fuse(ws, mc)
            if i is not None:
                e2[i].record()

        with torch.no_grad():
            for _ in range(warmup):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                step(i)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        out[mode] = {"value": round(B * steps / dt, 3), "ms_per_step": round(dt * 1e3 / steps, 4),
                     "upsample_and_warp_ms": round(float(np.mean([e0[i].elapsed_time(e1[i]) for i in range(steps)])), 4)}
    out["note"] = ("step from backbone-resolution features: a4 upsample (:65) + warp + concat + fusion; "
                   "fused = upsample evaluated inside the warp kernel (NCHW maps: a transposing copy, then "
                   "warp_up_wino_cl_kernel); fused_channels_last = the same maps in channels_last memory format, "
                   "as mvdet_amd.PerspTransDetector's channels-last backbone produces them by default (no copy)")
    out["detector_default"] = "fused_channels_last"
    return out


def torch_warp(feat, m, ho, wo):
    """kornia steps 3-6 in stock torch GPU ops (autograd through grid_sample): the reference's
    own op sequence on the GPU, used as the training-step comparison."""
    import torch.nn.functional as F
    B = feat.shape[0]
    xs = (torch.linspace(0, wo - 1, wo, device=feat.device) / (wo - 1) - 0.5) * 2
    ys = (torch.linspace(0, ho - 1, ho, device=feat.device) / (ho - 1) - 0.5) * 2
    gy, gx = torch.meshgrid(ys, xs, indexing="ij")
    pts = torch.stack([gx, gy, torch.ones_like(gx)], -1) @ m.T
    z = pts[..., 2:]
    scale = torch.where(z.abs() > 1e-8, 1.0 / (z + 1e-8), torch.ones_like(z))
    grid = (scale * pts[..., :2]).unsqueeze(0).expand(B, ho, wo, 2)
    return F.grid_sample(feat, grid, mode="bilinear", padding_mode="zeros", align_corners=True)


def run_train_step(config: int, precision: str, steps: int, warmup: int, with_torch: bool):
    """Training step of the hot path: forward + backward of warp + concat +
    fusion head over one frame batch (inputs resident in HBM; gradients w.r.t. the upsampled view
    features and every head parameter), as ``trainer.py:38-47`` runs it.  "native" =
    ``autograd.ProjectFuseFunction`` (HIP forward and backward); "torch_gpu" = the reference's
    own op sequence on this GPU (grid_sample + cat + nn.Conv2d under autograd, MIOpen)."""
    from mvdet_amd import ProjectFuse, autograd, synthetic
    from mvdet_amd.geometry import projection_matrices
    progress("train_step")
    spec = synthetic.CONFIGS[config]
    ds = spec["make"]()
    B, C, N = spec["B"], spec["C"], ds.num_cam
    up = tuple(ds.upsample_shape)
    ho, wo = ds.reducedgrid_shape
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    pm = projection_matrices(ds)
    mc = build_mc(C, N, head_params(N, config, C), dev)
    eng = ProjectFuse(pm, up, (ho, wo), C, precision=precision)
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=v, device=dev).requires_grad_()
             for v in range(N)]
    gmap = torch.randn((B, 1, ho, wo), device=dev)
    res = {"workload": f"cfg{config}: {spec['name']}", "precision": precision}

    def run(step, K, W, hook_stages=False):
        for _ in range(W):
            step()
        torch.cuda.synchronize()
        evs = []
        t0 = time.perf_counter()
        for _ in range(K):
            marks = {}
            if hook_stages:
                autograd.set_stage_hook(
                    lambda s: marks.setdefault(s, torch.cuda.Event(enable_timing=True)).record())
            step()
            autograd.set_stage_hook(None)
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            marks["end"] = e
            evs.append(marks)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out = {"value": round(B * K / dt, 3), "unit": "frames/s", "ms_per_step": round(dt * 1e3 / K, 3)}
        if hook_stages:
            names = [s for s in evs[0] if s not in ("end", "bwd_end")]
            st = {}
            for a, b in zip(names, names[1:] + ["end"]):
                st[a] = round(float(np.mean([m[a].elapsed_time(m[b]) for m in evs])), 4)
            out["stages_ms"] = st
        return out

    # trainer.py:48: optimizer.step() after every backward — an in-place update of every head parameter, which
    # bumps the weights' _version, so the next forward re-packs conv1's / conv2's (Winograd) weights and the
    # backward its data-gradient packs, inside the timed step.  SGD with momentum as the
    # reference trains (main.py:69,146-147: momentum 0.5, weight decay 5e-4); a small lr keeps the synthetic weights in range.
    opt = torch.optim.SGD(mc.parameters(), lr=1e-4, momentum=0.5, weight_decay=5e-4)

    def optimizer_step():
        if autograd._stage_hook is not None:
            autograd._stage_hook("optimizer")
        opt.step()

    def native_step(update=True):
        for f in feats:
            f.grad = None
        mc.zero_grad(set_to_none=True)
        autograd.project_fuse(eng, feats, mc).backward(gmap)
        if update:
            optimizer_step()

    # the same step without the update (packs reused from the cache): the repacking's cost is the difference.
    # Three interleaved rounds (no-update / update, update / no-update, no-update / update), each variant's
    # median run reported: one pair timed back to back swung by ±0.3-0.9 ms between boxes and orders
    # (round 6: the first-timed variant ran its MFMA kernels up to ~15 % slower on some boxes, on others not)
    for _ in range(warmup):
        native_step()
    runs = {"u": [], "nu": []}
    fns = {"u": native_step, "nu": lambda: native_step(update=False)}
    for order in (("nu", "u"), ("u", "nu"), ("nu", "u")):
        for v in order:
            runs[v].append(run(fns[v], steps, warmup, hook_stages=True))

    def median_run(rs):
        return sorted(rs, key=lambda r: r["ms_per_step"])[len(rs) // 2]

    nu = median_run(runs["nu"])
    nu["runs_ms"] = [r["ms_per_step"] for r in runs["nu"]]
    res["native"] = median_run(runs["u"])
    res["native"]["runs_ms"] = [r["ms_per_step"] for r in runs["u"]]
    res["native"]["optimizer"] = "SGD(lr=1e-4, momentum=0.5, weight_decay=5e-4).step() per step (weights re-packed every step)"
    res["native"]["sample"] = (f"median of 3 runs of {steps} steps, interleaved with the no-update runs "
                               "(nu/u, u/nu, nu/u)")
    res["native_no_update"] = nu
    res["weight_update_cost_ms"] = round(res["native"]["ms_per_step"] - nu["ms_per_step"], 3)
    if with_torch:
        ms = [eng.m_norm_cpu[v].to(dev) for v in range(N)]
        cmap = torch.from_numpy(np.stack(np.meshgrid(np.arange(wo) / (wo - 1) * 2 - 1,
                                                     np.arange(ho) / (ho - 1) * 2 - 1), 0)).float()[None].to(dev)

        def torch_step():
            for f in feats:
                f.grad = None
            mc.zero_grad(set_to_none=True)
            world = [torch_warp(f, m, ho, wo) for f, m in zip(feats, ms)]
            mc(torch.cat(world + [cmap.repeat(B, 1, 1, 1)], 1)).backward(gmap)
            opt.step()

        res["torch_gpu"] = run(torch_step, max(2, steps // 4), 1)
        res["speedup_vs_torch_gpu"] = round(res["native"]["value"] / res["torch_gpu"]["value"], 2)
    # "+a4": the step the drop-in module trains through (trainer.py:38-47 calling
    # persp_trans_detector.py:65-87): from the backbone-resolution maps, the 3x upsample included
    # (native: fused into the warp and its adjoint into the warp adjoint)
    # (channels-last maps: PerspTransDetector's backbone runs channels_last by default)
    bfeats = [synthetic.backbone_features(B, C, [u // 3 for u in up], seed=v, device=dev)
              .contiguous(memory_format=torch.channels_last).requires_grad_() for v in range(N)]

    def native_a4():
        for f in bfeats:
            f.grad = None
        mc.zero_grad(set_to_none=True)
        autograd.project_fuse_backbone(eng, bfeats, mc).backward(gmap)
        optimizer_step()

    a4 = {"native": run(native_a4, steps, warmup, hook_stages=True)}
    if with_torch:
        def torch_a4():
            for f in bfeats:
                f.grad = None
            mc.zero_grad(set_to_none=True)
            world = [torch_warp(torch.nn.functional.interpolate(f, up, mode="bilinear"), m, ho, wo)
                     for f, m in zip(bfeats, ms)]
            mc(torch.cat(world + [cmap.repeat(B, 1, 1, 1)], 1)).backward(gmap)
            opt.step()

        a4["torch_gpu"] = run(torch_a4, max(2, steps // 4), 1)
        a4["speedup_vs_torch_gpu"] = round(a4["native"]["value"] / a4["torch_gpu"]["value"], 2)
    a4["note"] = ("from backbone-resolution maps (a4 upsample :65 included) as the drop-in module trains: "
                  "channels-last maps, as its backbone produces them")
    res["plus_a4"] = a4
    return res


def spawn_ranks(n: int) -> int:
    """``--gpus N`` (N > 1) without a launcher: start N rank processes through
    ``torch.distributed.run`` (one per GPU, rendezvous on 127.0.0.1) and return their exit code.
    This parent makes no GPU call: ``torch.cuda.device_count()`` does not initialise the device
    on this image, and the children are started with ``subprocess`` (never an exec).  With
    fewer GPUs than ranks (a 1-GPU rehearsal box) the ranks share the devices over ``gloo``."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    if torch.cuda.device_count() < n:
        env.setdefault("MVBEV_DIST_BACKEND", "gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py")] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--layout", default="nchw", choices=["nchw", "channels_last"],
                    help="memory format of the view features (the same logical tensors); the other one is "
                         "reported as a sub-object")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--conv1", default="wino", choices=["direct", "wino"],
                    help="form of conv1 and conv2 (bf16x3): the direct ring convs or row-Winograd F(3,3) "
                         "(ProjectFuse wino_conv1 / wino_conv2)")
    ap.add_argument("--precision", default="bf16x3", choices=["fp32", "bf16x3"],
                    help="conv1/conv2 arithmetic: 3xbf16 split (default) or fp32-input MFMA")
    ap.add_argument("--config", type=int, default=2, help="BASELINE.json config index (1-based)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the sustained-MFMA-rate probe (roofline.sustained_peak)")
    ap.add_argument("--no-alt", action="store_true", help="skip the other-precision comparison line")
    ap.add_argument("--cpu-frames", type=int, default=0, help="frames for the CPU baseline (0 = auto)")
    ap.add_argument("--no-train", action="store_true", help="skip the training-step (forward+backward) line")
    ap.add_argument("--train-torch", type=int, default=1,
                    help="1 = also time the reference op sequence (torch GPU autograd) for the training step")
    ap.add_argument("--mp-mode", default="auto", choices=["auto", "bands", "gather", "partial", "frames"],
                    help="N>1 `value`: auto (default: the view-parallel mode mvdet_amd.mp_model predicts fastest for "
                         "this config and N, DESIGN.md §6), the band exchange (all-to-all of each row band's input "
                         "window), slab all-gather, conv1 partial sums + reduce-scatter, or frame-parallel; the other "
                         "modes are reported alongside")
    ap.add_argument("--north-star-cfg", type=int, default=3,
                    help="also run this config (the north star's 480x1440 Wildtrack grid) as a sub-object "
                         "(N=1: single GPU with a reduced-sample CPU baseline; N>1: the band exchange); 0 = skip")
    ap.add_argument("--roofline-cfg", type=int, default=5,
                    help="also run this config (BASELINE's rocprof roofline run: 8 views at 4K -> 1000 x 1000) as a "
                         "sub-object with its roofline and a reduced-sample CPU baseline; 0 = skip")
    ap.add_argument("--batch-cfg", type=int, default=4,
                    help="also run this config (BASELINE's MultiviewX B = 8 fp16 one) as a sub-object with its "
                         "roofline and a CPU baseline; 0 = skip")
    args = ap.parse_args()

    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus {args.gpus} < 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        # a launcher and the flag disagree: a line for the wrong N must never be printed
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        from mvdet_amd import parallel
        return parallel.bench_main(args)

    res = run_single(args, args.precision, args.steps, args.warmup, with_cpu=not args.no_cpu_baseline and rank == 0)
    result = {
        "metric": "multi-view frames/sec (project+fuse)",
        "value": res["value"],
        "unit": "frames/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": res["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",  # N > 1: one frame's views across the GPUs (the band exchange)
        "vs_baseline": None,
        "dtype": res["dtype"],
        "data": "synthetic (ReLU N(0,1) features upsampled 3x, synthetic pinhole rig through the reference "
                "matrix chain, random-init fusion weights)",
        "config": res["config"],
        "roofline": res["roofline"],
        "cpu_baseline": res.get("cpu_baseline"),
        "stages_ms": res["stages_ms"],
        "e2e_roofline": res["e2e_roofline"],
        "stage_roofline": res["stage_roofline"],
    }
    if result["cpu_baseline"]:
        result["speedup_vs_cpu"] = round(res["value"] / result["cpu_baseline"]["value"], 1)
    if args.config != 4 and args.precision == "bf16x3":
        # the same step on the other feature memory format (channels-last: warp_wino_cl_kernel reads
        # one 128-B line per source pixel instead of NCHW's per-channel boxes)
        other_layout = "channels_last" if args.layout == "nchw" else "nchw"
        ol = run_single(args, args.precision, max(5, args.steps // 2), 2, with_cpu=False, layout=other_layout)
        result[other_layout] = {k: ol[k] for k in ("value", "ms_per_step", "stages_ms")}
        result[other_layout]["warp"] = ol["stage_roofline"]["warp"]
    if args.config != 4:  # the fused upsample+warp writes fp32 / split slabs (not the fp16 slab)
        result["plus_a4"] = run_plus_a4(args, args.precision, max(5, args.steps // 2), 2)
    subs = []
    if args.north_star_cfg and args.north_star_cfg != args.config:
        # the size the north star quotes its >= 5x at 1 GPU on (cfg3: 7 views, 480 x 1440 grid): the same
        # path, its roofline, and a CPU baseline on BASELINE.md:26's sample (2 warm-ups + the median of 5
        # frames, ~18 s of CPU work per frame at 16 threads)
        subs.append((args.north_star_cfg, dict(frames=5, warmups=2, single_frames=1, single_warmups=0, single_band=4)))
    if args.roofline_cfg and args.roofline_cfg not in (args.config, args.north_star_cfg):
        # BASELINE's "rocprof roofline run" config (8 views at 4K): 1 warm-up + the median of 3 frames
        # (~16 s of CPU work per frame)
        subs.append((args.roofline_cfg, dict(frames=3, warmups=1, single_frames=1, single_warmups=0, single_band=4)))
    if args.batch_cfg and args.batch_cfg not in (args.config, args.north_star_cfg, args.roofline_cfg):
        # BASELINE configs[3]: MultiviewX 6 views, B = 8, fp16 features (C = 512, the reference's ResNet-18
        # width); its CPU baseline on B = 1 frames (1 warm-up + the median of 3), frames/s = 1 / median
        subs.append((args.batch_cfg, dict(frames=3, warmups=1, single_frames=1, single_warmups=0)))
    for cfg, plan in subs:
        sub = run_single(args, args.precision, max(5, args.steps // 4), 2,
                         with_cpu=plan is not None and not args.no_cpu_baseline, config=cfg, cpu_plan=plan)
        sub = {k: sub[k] for k in ("value", "ms_per_step", "config", "roofline", "stages_ms", "e2e_roofline",
                                   "stage_roofline", "cpu_baseline") if k in sub}
        sub["unit"] = "frames/s"
        if sub.get("cpu_baseline"):
            sub["speedup_vs_cpu"] = round(sub["value"] / sub["cpu_baseline"]["value"], 1)
        else:
            sub["cpu_baseline"] = None  # --no-cpu-baseline
        result[f"cfg{cfg}"] = sub
    if not args.no_train and args.config != 4:
        result["train_step"] = run_train_step(args.config, args.precision, max(5, args.steps // 2), 2,
                                              with_torch=bool(args.train_torch))
    if not args.no_alt:
        other = "fp32" if args.precision == "bf16x3" else "bf16x3"
        alt = run_single(args, other, max(3, args.steps // 2), 2, with_cpu=False)
        result["alt_precision"] = {k: alt[k] for k in ("value", "ms_per_step", "dtype", "stages_ms")}
        result["alt_precision"]["roofline"] = alt["roofline"]
    print(json.dumps(result))


if __name__ == "__main__":
    main()
