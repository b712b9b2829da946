"""Print DESIGN.md §6's table: mvdet_amd.mp_model's predicted per-frame time (ms) and speed-up over
one GPU of each view-parallel mode at configs 2-5 and P = 2, 4, 7, 8 (config 4 also at its P = 6) (CPU only).

    python tools/mp_cost_model.py
"""
from __future__ import annotations

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from mvdet_amd import mp_model  # noqa: E402


def main():
    print("| cfg | P | bands ms (x) | partial ms (x) | gather ms (x) | chosen |")
    print("|---|---|---|---|---|---|")
    for cfg in sorted(mp_model.SINGLE_GPU_MS):
        for P in ((2, 4, 6, 7, 8) if cfg == 4 else (2, 4, 7, 8)):
            pr = mp_model.predict_config(cfg, P)
            cells = [f"{pr[m]['frame']:.2f} ({pr[m]['speedup_vs_1gpu']:.1f}x)" for m in ("bands", "partial", "gather")]
            print(f"| {cfg} | {P} | " + " | ".join(cells) + f" | {mp_model.choose_mode(cfg, P)} |")


if __name__ == "__main__":
    main()
