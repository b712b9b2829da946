"""Backbone forward time, NCHW vs channels_last (MIOpen), at the detector's Wildtrack input (7 views,
720 x 1280 -> 90 x 160 maps): whether a channels-last backbone (which feeds the fused warp's
line-per-pixel kernel without a copy) costs anything."""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from mvdet_amd.backbone import build_backbone  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    p1, p2, _ = build_backbone("resnet18")
    net = torch.nn.Sequential(p1, p2).to(dev).eval()
    x = torch.randn(7, 3, 720, 1280, device=dev)
    out = {}
    for fmt in ("nchw", "channels_last"):
        m, xi = net, x
        if fmt == "channels_last":
            m = net.to(memory_format=torch.channels_last)
            xi = x.contiguous(memory_format=torch.channels_last)
        with torch.no_grad():
            for _ in range(3):
                y = m(xi)
            torch.cuda.synchronize()
            t = []
            for _ in range(10):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                y = m(xi)
                e1.record()
                torch.cuda.synchronize()
                t.append(e0.elapsed_time(e1))
        out[fmt] = {"median_ms": sorted(t)[len(t) // 2], "shape": list(y.shape),
                    "channels_last_out": y.is_contiguous(memory_format=torch.channels_last)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
