"""bench.py's one-line JSON contract on a small config (cfg1, 2 steps): the keys the driver and
the judge read, a roofline whose fraction is achieved / peak, and a CPU baseline that ran."""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.gpu
def test_bench_json_line_contract():
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--config", "1", "--steps", "2", "--warmup", "1",
                          "--no-train", "--no-alt", "--cpu-frames", "1", "--north-star-cfg", "2", "--roofline-cfg", "0",
                          "--batch-cfg", "0"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    r = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in r, k
    assert r["n_gpus"] == 1 and r["steps"] == 2 and r["warmup"] == 1 and r["higher_is_better"] is True
    assert r["value"] > 0 and abs(r["value"] * r["ms_per_step"] / 1e3 - 1.0) < 0.05  # B = 1 at cfg1
    rl = r["roofline"]
    assert rl["bound"] in ("hbm", "mfma") and rl["unit"] in ("GB/s", "TFLOP/s")
    assert rl["frac"] == pytest.approx(rl["achieved"] / rl["peak"], rel=1e-3)
    assert 0 < rl["frac"] <= 1.0  # executed MFMA work (frustum-skipped products not counted)
    assert rl["dense_algorithmic_frac"] >= rl["frac"]
    cb = r["cpu_baseline"]
    assert cb["value"] > 0 and cb["kind"] in ("port", "reference") and cb["cores"] >= 1
    assert cb["single_thread"]["cores"] == 1 and cb["single_thread"]["value"] > 0
    e2e = r["e2e_roofline"]
    assert 0 < e2e["frac"] <= 1.0 and e2e["floor_ms"] > 0
    for name, st in r["stage_roofline"].items():  # no stage may claim more than the peak it is priced at
        if "achieved_GBs" in st:
            assert 0 < st["achieved_GBs"] <= st["peak_GBs"], (name, st)
        if st.get("executed_bf16_frac") is not None:
            assert 0 < st["executed_bf16_frac"] <= 1.0, (name, st)
    assert r["config"]["workload"].startswith("cfg1") and r["config"]["feature_layout"] == "nchw"
    # the same step on channels-last features, and the +a4 legs (NCHW, torch upsample, channels-last maps)
    assert r["channels_last"]["value"] > 0 and 0 < r["channels_last"]["warp"]["achieved_GBs"] <= 8000
    for leg in ("fused", "unfused", "fused_channels_last"):
        assert r["plus_a4"][leg]["value"] > 0 and r["plus_a4"][leg]["upsample_and_warp_ms"] > 0, leg
    # the north-star sub-object (here cfg2 for speed; the default is cfg3): its own value, roofline, CPU baseline
    sub = r["cfg2"]
    assert sub["value"] > 0 and sub["config"]["workload"].startswith("cfg2") and 0 < sub["roofline"]["frac"] <= 1.0
    assert sub["cpu_baseline"]["value"] > 0 and sub["speedup_vs_cpu"] > 1


@pytest.mark.gpu
def test_bench_multi_rank_json_line():
    """The N > 1 path as the driver launches it (torch.distributed.run, one JSON line from rank 0),
    rehearsed with 2 gloo ranks sharing the box's one GPU: the view-parallel band exchange as
    `value` (strong scaling), frame-parallel and the other view-parallel modes alongside (RCCL
    itself only runs on the driver's 8-GPU node)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PYTHONUNBUFFERED="1", MVBEV_DIST_BACKEND="gloo")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"),
                          "--gpus", "2", "--config", "1", "--steps", "2", "--warmup", "1", "--north-star-cfg", "0"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["scaling"] == "strong" and r["value"] > 0
    assert r["config"]["batch"] == 1 and 0 < r["roofline"]["frac"] <= 1.0
    assert r["frame_parallel"]["scaling"] == "weak" and r["frame_parallel"]["value"] > 0
    for key in ("view_parallel_partial", "view_parallel_gather"):
        assert "error" not in r[key], r[key]
        assert r[key]["value"] > 0 and r[key]["scaling"] == "strong"
    _check_multi_rank_line(r, 2)


def _check_multi_rank_line(r, n):
    """The keys the N = 1 line carries, and conv1's roofline over the conv kernel's own time (its
    mark "conv1_wino"), never over the row transform before it."""
    assert r["n_gpus"] == n and r["rehearsal"] is True  # gloo ranks sharing the box's one GPU
    rl = r["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rl, k
    assert 0 < rl["frac"] <= 1.0 and rl["frac"] == pytest.approx(rl["achieved"] / rl["peak"], rel=1e-3)
    st = r["stages_ms_rank0"]
    if "conv1_wino" in st:
        assert st["conv1_total"] >= st["conv1_wino"] > 0
    cb = r["cpu_baseline"]
    assert cb["value"] > 0 and cb["kind"] == "port" and cb["cores"] >= 1


@pytest.mark.gpu
def test_bench_gpus_flag_spawns_ranks_without_a_launcher():
    """``python bench.py --gpus 2`` with no torchrun in front (WORLD_SIZE unset): bench.py starts the
    two ranks itself (gloo, sharing the one GPU of the test box) and the line says n_gpus 2."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONUNBUFFERED"] = "1"
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--config", "1", "--steps", "2",
                          "--warmup", "1", "--north-star-cfg", "0", "--no-alt"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["value"] > 0 and r["scaling"] == "strong"
    _check_multi_rank_line(r, 2)
