"""The round-4 Winograd conv form (``conv_wino4_kernel``: one wave per SIMD, xi-major accumulation;
selected by ``MVBEV_WINO4`` for conv1 / conv2) against the round-3 kernel and the oracle.

The selection is read once per process, so the alternative runs in a child process that writes its
outputs; the parent computes the default kernel's and compares: the same products summed in the same
order per accumulator, and the A^T fold in the order of the round-3 epilogue, so the maps agree to
fp32 rounding of that fold."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

from helpers import assert_parity_t
from oracle import cpu_path, fixtures

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]

CHILD = r'''
import sys, torch
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
from test_gpu_wino4 import run_case
torch.save(run_case({cfg}, {C}), {out!r})
'''


def run_case(cfg, C):
    """map_result, y1 (fp32) of the default engine path at config ``cfg`` with C channels."""
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    spec = synthetic.CONFIGS[cfg]
    ds = spec["make"]()
    B, N = spec["B"], ds.num_cam
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm = projection_matrices(ds)
    params = fixtures.head_params(N, seed=cfg, C=C)
    mc = torch.nn.Sequential(torch.nn.Conv2d(C * N + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False))
    mc.load_state_dict({k.replace("map_classifier.", ""): torch.from_numpy(v) for k, v in params.items()
                        if k.startswith("map_classifier.")})
    mc = mc.cuda()
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=1000 * cfg + v, device="cuda")
             for v in range(N)]
    eng = ProjectFuse(pm, up, grid, C)
    with torch.no_grad():
        m = eng.project_fuse(feats, mc).cpu()
        y1 = eng.y1_fp32(eng.workspace(B, "cuda:0")).cpu()
    return {"map": m, "y1": y1, "feats": [f.cpu() for f in feats], "pm": [M.numpy() for M in pm], "grid": grid,
            "params": params}


@pytest.mark.parametrize("cfg,C", [(1, 128), (2, 512)])
def test_wino4_matches_round3_kernel_and_oracle(cfg, C, tmp_path):
    out = tmp_path / "w4.pt"
    env = dict(os.environ, MVBEV_WINO4="3")
    code = CHILD.format(root=str(ROOT), tests=str(ROOT / "tests"), cfg=cfg, C=C, out=str(out))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    w4 = torch.load(out, weights_only=False)
    ref = run_case(cfg, C)
    torch.testing.assert_close(w4["y1"], ref["y1"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(w4["map"], ref["map"], rtol=1e-5, atol=1e-6)
    with torch.no_grad():
        oracle = cpu_path.project_fuse(ref["feats"], ref["pm"], ref["grid"],
                                       {k: torch.from_numpy(v) for k, v in ref["params"].items()})
    assert_parity_t(w4["map"], oracle, f"cfg{cfg} wino4 map vs oracle", normwise_tol=5e-5)
