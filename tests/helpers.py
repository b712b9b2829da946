"""Shared test helpers: golden-fixture loading and the parity gate.

Parity gate (north_star "within 1e-3 relative fp32"):
per tensor  |got - ref| <= 1e-3 * |ref| + 1e-3 * max|ref|   elementwise, and
normwise    max|got - ref| / max|ref| <= 1e-3.
"""
import json
from pathlib import Path

import numpy as np
import torch

GOLDEN = Path(__file__).resolve().parent / "golden"
RTOL = 1e-3
ATOL_FRAC = 1e-3


def load_golden(name):
    d = dict(np.load(GOLDEN / f"{name}.npz", allow_pickle=False))
    if "meta" in d:
        d["meta"] = json.loads(str(d["meta"]))
    return d


def to_np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().to("cpu", torch.float64).numpy()
    return np.asarray(x, dtype=np.float64)


def parity_stats(got, ref):
    """Stats over the finite entries; the NaN/inf pattern itself must match exactly."""
    got, ref = to_np(got), to_np(ref)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    nf_g, nf_r = ~np.isfinite(got), ~np.isfinite(ref)
    assert np.array_equal(nf_g, nf_r), f"non-finite pattern differs ({int(nf_g.sum())} vs {int(nf_r.sum())})"
    assert np.array_equal(np.isnan(got), np.isnan(ref)), "NaN pattern differs"
    fin = ~nf_r
    got, ref = got[fin], ref[fin]
    scale = float(np.abs(ref).max()) if ref.size else 0.0
    diff = np.abs(got - ref)
    if diff.size == 0:
        return dict(normwise=0.0, n_bad=0, max_abs=0.0, scale=scale)
    normwise = float(diff.max() / scale) if scale > 0 else float(diff.max())
    bound = RTOL * np.abs(ref) + ATOL_FRAC * scale
    n_bad = int((diff > bound).sum())
    return dict(normwise=normwise, n_bad=n_bad, max_abs=float(diff.max()) if diff.size else 0.0, scale=scale)


def assert_parity(got, ref, what="", normwise_tol=1e-3):
    s = parity_stats(got, ref)
    assert s["n_bad"] == 0 and s["normwise"] <= normwise_tol, f"{what}: parity failed {s}"
    return s


def parity_stats_t(got: torch.Tensor, ref: torch.Tensor, chunk: int = 1 << 26):
    """``parity_stats`` on torch tensors where they live (e.g. the GPU: full-size configs hold
    GB-sized tensors), in float64 chunks; the same gate and NaN/inf rule."""
    assert tuple(got.shape) == tuple(ref.shape), (tuple(got.shape), tuple(ref.shape))
    g, r = got.reshape(-1), ref.reshape(-1).to(got.device)
    scale = 0.0
    for i in range(0, r.numel(), chunk):
        rc = r[i:i + chunk].double()
        gc = g[i:i + chunk].double()
        assert torch.equal(~torch.isfinite(gc), ~torch.isfinite(rc)), "non-finite pattern differs"
        assert torch.equal(torch.isnan(gc), torch.isnan(rc)), "NaN pattern differs"
        fin = torch.isfinite(rc)
        if fin.any():
            scale = max(scale, rc[fin].abs().max().item())
    n_bad, dmax = 0, 0.0
    for i in range(0, r.numel(), chunk):
        rc = r[i:i + chunk].double()
        gc = g[i:i + chunk].double()
        fin = torch.isfinite(rc)
        d = (gc[fin] - rc[fin]).abs()
        if d.numel():
            dmax = max(dmax, d.max().item())
            n_bad += int((d > RTOL * rc[fin].abs() + ATOL_FRAC * scale).sum().item())
    normwise = dmax / scale if scale > 0 else dmax
    return dict(normwise=normwise, n_bad=n_bad, max_abs=dmax, scale=scale)


def assert_parity_t(got, ref, what="", normwise_tol=1e-3):
    s = parity_stats_t(got, ref)
    assert s["n_bad"] == 0 and s["normwise"] <= normwise_tol, f"{what}: parity failed {s}"
    return s
