"""Per-launch HBM-side traffic of each hot-path kernel from the rocprofv3 --pmc passes.

read bytes  = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B   (TCC_EA0 request sizes; the
              gfx950 FETCH_SIZE formula tallies 128-B requests at 64 B — MI355X_MICROARCH §HBM)
write bytes = WRITE_SIZE * 1024  (exact for 16-B-per-lane and 4-B-per-lane coalesced stores)
Dispatches are grouped by (kernel, grid size) — e.g. kbench's one-off per-view warps
during setup vs the all-views warp of the timed "warp" stage — and each group reports the
median over its dispatches.  Usage: python tools/traffic.py <pmc dir> <tag> <config> [precision]
(precision = the conv arithmetic kbench ran with: bf16x3 (default) or fp32; selects which
kernel is conv1: the ReLU dilation-1 conv over the view slab — the coord-term conv that runs
once per weight version is the non-ReLU instance and is not conv1).
"""
import collections
import csv
import glob
import json
import re
import statistics
import sys

out_dir, tag, cfg = sys.argv[1], sys.argv[2], int(sys.argv[3])
precision = sys.argv[4] if len(sys.argv) > 4 else "bf16x3"
wino = len(sys.argv) > 5 and sys.argv[5] in ("wino", "wino43")  # conv1 = the row-Winograd conv kernel (kbench winoconv)
w43 = len(sys.argv) > 5 and sys.argv[5] == "wino43"  # the F(4,3) kernels (kbench winoconv43, conv2w43, warpw43)
vals = collections.defaultdict(lambda: collections.defaultdict(dict))
for f in glob.glob(f"{out_dir}/{tag}_pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = f'{r["Kernel_Name"].split("(")[0]} [grid {r["Grid_Size"]}]'
        vals[name][r["Counter_Name"]][(f, r["Dispatch_Id"])] = float(r["Counter_Value"])

def med(name, counter):
    xs = list(vals[name].get(counter, {}).values())
    return statistics.median(xs) if xs else None

res = {"config": cfg, "precision": precision, "source": f"rocprofv3 --pmc passes over tools/kbench.py ({tag})", "kernels": {}}
for name in vals:
    if "mvbev::" not in name:
        continue
    n32, n64, n128 = (med(name, f"TCC_EA0_RDREQ_{s}_sum") for s in ("32B", "64B", "128B"))
    wr = med(name, "WRITE_SIZE")
    if None in (n32, n64, n128, wr):
        continue
    rd = 32 * n32 + 64 * n64 + 128 * n128
    res["kernels"][name] = {"read_bytes": rd, "write_bytes": wr * 1024, "hbm_bytes_per_launch": rd + wr * 1024,
                            "fetch_size_kb": med(name, "FETCH_SIZE")}
# conv1: the ReLU dilation-1 ring kernel without the fused cout1 epilogue (grid tiles "<1, true>",
# edge-strip tiles "<1, true, false, EW>"), or the fp32-MFMA kernel
pat = r"conv_ring_kernel<1, true(, false, \d+)?>" if precision == "bf16x3" else r"conv3x3_mfma_f32_kernel<1, true"
if wino:
    kn = "conv_wino43_kernel" if w43 else "conv_wino_kernel"
    pat = kn + r"<true, 1, false>"
    c2 = [k for k in res["kernels"] if kn + "<true, 2, true>" in k]
    if c2:  # conv2 -> conv3 partials, row-Winograd (ABI 11500)
        res["conv2_hbm_bytes_per_launch"] = res["kernels"][c2[0]]["hbm_bytes_per_launch"]
    rows = sorted((k for k in res["kernels"] if ("wino43_rows_kernel" if w43 else "wino_rows_kernel") in k),
                  key=lambda n: int(n.rsplit("grid ", 1)[1].rstrip("]")))  # (the smallest: conv2's y1 transform)
    if rows:
        res["wino_rows_hbm_bytes_per_launch"] = res["kernels"][rows[0]]["hbm_bytes_per_launch"]
conv1 = [k for k in res["kernels"] if re.search(pat, k)]
if conv1:
    res["conv1_hbm_bytes_per_launch"] = res["kernels"][conv1[0]]["hbm_bytes_per_launch"]
# the all-views warp of the timed "warp" stage: the largest-grid warp_tile_kernel dispatch
warps = [k for k in res["kernels"] if ("warp_wino_kernel" if wino else "warp_tile_kernel") in k
         and (not w43 or "float, 4>" in k)]
if warps:
    k = max(warps, key=lambda n: int(n.rsplit("grid ", 1)[1].rstrip("]")))
    res["warp_hbm_bytes_per_launch"] = res["kernels"][k]["hbm_bytes_per_launch"]
    res["warp_read_bytes_per_launch"] = res["kernels"][k]["read_bytes"]
# the same warp on channels-last features (warp_wino_cl_kernel, kbench warpwcl)
cls = [k for k in res["kernels"] if "warp_wino_cl_kernel" in k]
if cls:
    k = max(cls, key=lambda n: int(n.rsplit("grid ", 1)[1].rstrip("]")))
    res["warp_cl_hbm_bytes_per_launch"] = res["kernels"][k]["hbm_bytes_per_launch"]
    res["warp_cl_read_bytes_per_launch"] = res["kernels"][k]["read_bytes"]
# the detector's inference warp (fused 3x upsample + warp + B^T from backbone-resolution maps)
ups = [k for k in res["kernels"] if "warp_up_wino2_kernel" in k or "warp_up_wino_cl_kernel" in k]
if ups:
    k = max(ups, key=lambda n: int(n.rsplit("grid ", 1)[1].rstrip("]")))
    res["warp_up_hbm_bytes_per_launch"] = res["kernels"][k]["hbm_bytes_per_launch"]
print(json.dumps(res, indent=1))
