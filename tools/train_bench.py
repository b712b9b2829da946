"""Training-step benchmark of the hot path on one GPU.

    python tools/train_bench.py [--config 2] [--steps 10] [--warmup 3] [--no-torch]

Thin CLI over ``bench.run_train_step`` (the same measurement ``bench.py`` reports as
``train_step``); prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import run_train_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--precision", default="bf16x3", choices=["fp32", "bf16x3"])
    ap.add_argument("--no-torch", action="store_true")
    args = ap.parse_args()
    print(json.dumps(run_train_step(args.config, args.precision, args.steps, args.warmup, not args.no_torch)))


if __name__ == "__main__":
    main()
