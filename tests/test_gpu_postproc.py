"""GPU post-processing vs the reference's nms golden vectors and the
oracle restatement of trainer.py's evaluation rows."""
import numpy as np
import pytest
import torch

from helpers import load_golden
from oracle import postproc

pytestmark = pytest.mark.gpu


def _topk(v):
    v = float(v)
    return int(v) if np.isfinite(v) else np.inf


def test_nms_tie_free_matches_oracle_exactly():
    from mvdet_amd import postprocess
    rng = np.random.default_rng(3)
    for K, dist, top_k in [(1, 20.0, np.inf), (7, 20.0, 3), (16, 20.0, np.inf), (17, 20.0, np.inf),
                           (500, 20.0, np.inf), (4096, 12.0, np.inf), (8192, 8.0, 100)]:
        pts = (rng.integers(0, 200, size=(K, 2)) * 4).astype(np.float32)
        sc = rng.permutation(K).astype(np.float32) / K + 0.4  # distinct scores
        ref_keep, ref_count = postproc.nms(torch.from_numpy(pts), torch.from_numpy(sc), dist, top_k)
        keep, count = postprocess.nms(torch.from_numpy(pts).cuda(), torch.from_numpy(sc).cuda(), dist, top_k)
        assert count == ref_count, (K, count, ref_count)
        np.testing.assert_array_equal(keep.cpu().numpy(), ref_keep.numpy())


@pytest.mark.parametrize("K,dist,top_k", [(8193, 20.0, np.inf), (20000, 20.0, 50), (43200, 20.0, np.inf),
                                          (43200, 4.0, 30000), (70000, 8.0, np.inf)])
def test_nms_large_k_matches_oracle_exactly(K, dist, top_k):
    """Large K (the sort's ranges span many chunks of the workgroup): the same points in the same
    order as the reference loop.  K = 43,200 is every cell of a cfg2 map over cls_thres
    (trainer.py:154)."""
    from mvdet_amd import postprocess
    rng = np.random.default_rng(K)
    if K == 43200:  # a 120 x 360 map's cells in grid coordinates x grid_reduce (trainer.py:103)
        ii, jj = np.meshgrid(np.arange(120), np.arange(360), indexing="ij")
        pts = (np.stack([ii.ravel(), jj.ravel()], 1) * 4).astype(np.float32)
    else:
        pts = (rng.integers(0, 400, size=(K, 2)) * 4).astype(np.float32)
    sc = rng.permutation(K).astype(np.float32) / K + 0.4  # distinct scores (tie-free)
    ref_keep, ref_count = postproc.nms(torch.from_numpy(pts), torch.from_numpy(sc), dist, top_k)
    keep, count = postprocess.nms(torch.from_numpy(pts).cuda(), torch.from_numpy(sc).cuda(), dist, top_k)
    assert count == ref_count, (K, count, ref_count)
    np.testing.assert_array_equal(keep.cpu().numpy(), ref_keep.numpy())


@pytest.mark.parametrize("K,levels,dist", [(12000, 50, 12.0), (43200, 20, 8.0), (3000, 3, 20.0), (700, 1, 4.0)])
def test_nms_ties_match_reference_order_exactly(K, levels, dist):
    """Exactly tied scores (few distinct levels; one level = every score equal): the kept indices
    and count equal the oracle's, whose order is torch's CPU sort itself (nms.py:22)."""
    from mvdet_amd import postprocess
    rng = np.random.default_rng(K + levels)
    pts = (rng.integers(0, 300, size=(K, 2)) * 2).astype(np.float32)
    sc = (rng.integers(0, levels, size=K) / max(levels, 1) + 0.4).astype(np.float32)
    ref_keep, ref_count = postproc.nms(torch.from_numpy(pts), torch.from_numpy(sc), dist, np.inf)
    keep, count = postprocess.nms(torch.from_numpy(pts).cuda(), torch.from_numpy(sc).cuda(), dist, np.inf)
    assert count == ref_count
    np.testing.assert_array_equal(keep.cpu().numpy(), ref_keep.numpy())


@pytest.mark.parametrize("n", [40, 300, 1200])
def test_nms_killer_sequence_heap_fallback(n):
    """McIlroy killer scores (``oracle.postproc.killer_sequence``) drive the introsort to its
    heap-sort fallback: the kernel's candidate order still equals torch's (top_k cut included)."""
    from mvdet_amd import postprocess
    sc = postproc.killer_sequence(n) / n
    pts = (np.random.default_rng(n).integers(0, 60, size=(n, 2)) * 4).astype(np.float32)
    for dist, top_k in ((0.5, np.inf), (20.0, n // 3)):
        ref_keep, ref_count = postproc.nms(torch.from_numpy(pts), torch.from_numpy(sc), dist, top_k)
        keep, count = postprocess.nms(torch.from_numpy(pts).cuda(), torch.from_numpy(sc).cuda(), dist, top_k)
        assert count == ref_count
        np.testing.assert_array_equal(keep.cpu().numpy(), ref_keep.numpy())


def test_nms_reference_golden_with_ties():
    """The reference's own cases (tests/golden/nms_cases.npz, made by its nms.py on this torch):
    keep and count exactly, although the scores contain exact ties."""
    from mvdet_amd import postprocess
    g = load_golden("nms_cases")
    for i in range(5):
        pts, sc = torch.from_numpy(g[f"c{i}_points"]), torch.from_numpy(g[f"c{i}_scores"])
        dist, top_k = float(g[f"c{i}_dist"]), _topk(g[f"c{i}_topk"])
        keep, count = postprocess.nms(pts.cuda(), sc.cuda(), dist, top_k)
        assert count == int(g[f"c{i}_count"]), i
        np.testing.assert_array_equal(keep.cpu().numpy(), g[f"c{i}_keep"])


def test_threshold_rows_and_frame_results_match_reference_golden():
    from mvdet_amd import postprocess
    g = load_golden("nms_cases")
    for j in range(2):
        m = torch.from_numpy(g[f"map{j}"])[None, None].cuda()
        rows = postprocess.threshold_rows(m, 7, 0.4, 4, str(g[f"map{j}_indexing"]))
        np.testing.assert_array_equal(rows.cpu().numpy(), g[f"map{j}_rows"])
        np.testing.assert_array_equal(postprocess.frame_results(rows).cpu().numpy(), g[f"map{j}_final"])


def test_nms_empty_and_threshold_empty():
    from mvdet_amd import postprocess
    keep = postprocess.nms(torch.zeros((0, 2)).cuda(), torch.zeros(0).cuda())
    assert isinstance(keep, torch.Tensor) and keep.numel() == 0  # the reference's quirk
    rows = postprocess.threshold_rows(torch.zeros((1, 1, 5, 7)).cuda(), 0, 0.4, 4)
    assert rows.shape == (0, 4)
