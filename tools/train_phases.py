"""bench.py's training step three times in a row (each: no-update run, then the SGD-update run), so the
no-update runs that follow an update run show whether weight_update_cost_ms is the update or the device's
clock drift.  GPU only: python tools/train_phases.py"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

for tag in ("first", "second", "third"):
    r = bench.run_train_step(2, "bf16x3", 20, 5, False)
    print(json.dumps({tag: {"update_ms": r["native"]["ms_per_step"], "no_update_ms": r["native_no_update"]["ms_per_step"],
                            "update_stages": r["native"]["stages_ms"],
                            "no_update_stages": r["native_no_update"]["stages_ms"]}}), flush=True)
