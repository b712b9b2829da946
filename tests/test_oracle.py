"""CPU tests: pin the oracle against the reference's golden vectors and the float64
closed form (no GPU needed).  See DESIGN.md §Oracle for what each pin covers."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import assert_parity, load_golden, parity_stats
from oracle import cpu_path, fixtures, kornia_warp


@pytest.fixture(scope="module", params=["module_wt2", "module_mx3_b2"])
def golden(request):
    return load_golden(request.param)


def _feats_up(g):
    """The reference's a4: bilinear upsample of the backbone features (``:65``)."""
    ups = g["meta"]["upsample_shape"]
    x = torch.from_numpy(g["feat_in"])
    return [F.interpolate(x[:, cam], ups, mode="bilinear") for cam in range(x.shape[1])]


def _params(g):
    p = fixtures.head_params(g["meta"]["num_cam"], g["meta"]["weight_seed"])
    assert fixtures.params_sha256(p) == g["meta"]["weights_sha256"], "weight recipe drifted"
    return {k: torch.from_numpy(v) for k, v in p.items()}


def test_weight_recipe_hash(golden):
    _params(golden)


def test_matrix_chain_matches_reference(golden):
    m = golden["meta"]
    got = cpu_path.proj_mats_from_rig(golden["K"], golden["E"], golden["G"], m["img_shape"], m["img_reduce"],
                                      m["grid_reduce"])
    np.testing.assert_allclose(np.stack(got), golden["proj_mats"], rtol=1e-12, atol=0)


def test_coord_map_matches_reference(golden):
    ho, wo = golden["meta"]["reducedgrid_shape"]
    assert torch.equal(cpu_path.coord_map(ho, wo), torch.from_numpy(golden["coord_map"]))


def test_warp_input_checksum(golden):
    feats = _feats_up(golden)
    got = np.stack([f.double().sum(dim=(2, 3)).numpy() for f in feats], 1)
    np.testing.assert_allclose(got, golden["warp_in_chsum"], rtol=1e-9, atol=1e-6)


def test_oracle_path_reproduces_reference_forward(golden):
    keep = {}
    ho, wo = golden["meta"]["reducedgrid_shape"]
    with torch.no_grad():
        out = cpu_path.project_fuse(_feats_up(golden), golden["proj_mats"], (ho, wo), _params(golden), keep=keep)
    # same torch-CPU ops in the same order as the reference: agreement to fp32 rounding
    s = assert_parity(out, golden["map_result"], "map_result", normwise_tol=1e-5)
    assert s["normwise"] < 1e-5
    chs = np.stack([w.double().sum(dim=(2, 3)).numpy() for w in keep["warped"]], 1)
    np.testing.assert_allclose(chs, golden["warp_out_chsum"], rtol=1e-6, atol=1e-4)
    if "warp_out" in golden:
        assert_parity(torch.stack(keep["warped"], 1), golden["warp_out"], "warp_out", normwise_tol=1e-6)
        assert_parity(keep["conv1_relu"], golden["conv1_relu"], "conv1", normwise_tol=1e-5)
        assert_parity(keep["conv2_relu"], golden["conv2_relu"], "conv2", normwise_tol=1e-5)


def test_geometry_configs_fixture():
    g = dict(np.load("tests/golden/geometry_configs.npz", allow_pickle=False))
    import json
    for k in range(1, 6):
        meta = json.loads(str(g[f"cfg{k}_meta"]))
        got = cpu_path.proj_mats_from_rig(g[f"cfg{k}_K"], g[f"cfg{k}_E"], g[f"cfg{k}_G"], meta["img_shape"],
                                          meta["img_reduce"], meta["grid_reduce"])
        np.testing.assert_allclose(np.stack(got), g[f"cfg{k}_proj_mats"], rtol=1e-12, atol=0)
    assert torch.equal(cpu_path.coord_map(120, 360), torch.from_numpy(g["cfg2_coord_map"]))


# --- kornia restatement vs the float64 closed form -----------------------------------------

def _random_homography(rng, H, W, ho, wo):
    """A homography mapping src pixels to dst pixels with mild perspective."""
    A = np.eye(3)
    A[0, 0] = wo / W * rng.uniform(0.6, 1.4)
    A[1, 1] = ho / H * rng.uniform(0.6, 1.4)
    A[0, 1], A[1, 0] = rng.uniform(-0.2, 0.2, 2)
    A[0, 2], A[1, 2] = rng.uniform(-3, 3, 2)
    A[2, 0], A[2, 1] = rng.uniform(-2e-3, 2e-3, 2)
    return A


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_restatement_vs_closed_form(seed):
    rng = np.random.default_rng(seed)
    B, C, H, W, ho, wo = 2, 5, 27, 48, 12, 36
    src = rng.standard_normal((B, C, H, W)).astype(np.float32)
    M = np.stack([_random_homography(rng, H, W, ho, wo) for _ in range(B)])
    got = kornia_warp.warp_perspective(torch.from_numpy(src), torch.from_numpy(M).float(), (ho, wo))
    ref = kornia_warp.closed_form_warp_f64(src, M, (ho, wo))
    s = parity_stats(got, ref)
    assert s["normwise"] < 2e-4, s


def test_identity_and_translation_known_answers():
    rng = np.random.default_rng(7)
    src = rng.standard_normal((1, 3, 9, 11)).astype(np.float32)
    t = torch.from_numpy(src)
    out = kornia_warp.warp_perspective(t, torch.eye(3)[None], (9, 11))
    np.testing.assert_allclose(out.numpy(), src, atol=1e-5)
    # shift by -0.5 px in x: out[u] = (src[u+0.5]) = mean of neighbours; last column half-zero
    M = torch.tensor([[[1.0, 0, -0.5], [0, 1, 0], [0, 0, 1]]])
    out = kornia_warp.warp_perspective(t, M, (9, 11)).numpy()
    exp = 0.5 * (src + np.concatenate([src[..., 1:], np.zeros_like(src[..., :1])], -1))
    np.testing.assert_allclose(out, exp, atol=1e-5)
    np.testing.assert_allclose(kornia_warp.closed_form_warp_f64(src, M.double().numpy(), (9, 11)), exp, atol=1e-6)


def test_out_of_bounds_is_zero_and_behind_camera_is_sampled():
    src = torch.ones(1, 1, 8, 8)
    far = torch.tensor([[[1.0, 0, 100.0], [0, 1, 100.0], [0, 0, 1]]])
    assert kornia_warp.warp_perspective(src, far, (4, 4)).abs().max() == 0
    # z < 0 everywhere (M^-1 has a negative last row): no cheirality mask, points still sampled
    Minv = np.array([[-1.0, 0, 0], [0, -1.0, 0], [0, 0, -1.0]])  # (u,v,1) -> (-u,-v,-1) == (u,v) after divide
    M = np.linalg.inv(Minv)
    out = kornia_warp.warp_perspective(src, torch.from_numpy(M).float()[None], (8, 8))
    assert float(out.min()) > 0.99
    ref = kornia_warp.closed_form_warp_f64(src.numpy(), M[None], (8, 8))
    np.testing.assert_allclose(out.numpy(), ref, atol=1e-5)


def test_touched_footprint_counts():
    M = np.eye(3)
    assert kornia_warp.touched_footprint(M, (6, 7), (6, 7)) == 42
    M2 = np.diag([0.5, 0.5, 1.0])  # dst is half-size: samples at even src pixels (+ corners)
    t = kornia_warp.touched_footprint(M2, (8, 8), (4, 4))
    assert 0 < t <= 64


# ------------------------------------------------------------------ post-processing (§8(f) row 4)

def test_postproc_oracle_matches_reference_nms_golden():
    """oracle/postproc.py vs the reference's own nms / evaluation rows (tests/golden/nms_cases.npz)."""
    import numpy as np
    import torch
    from helpers import load_golden
    from oracle import postproc
    g = load_golden("nms_cases")
    for i in range(5):
        top_k = float(g[f"c{i}_topk"])
        top_k = int(top_k) if np.isfinite(top_k) else np.inf
        keep, count = postproc.nms(torch.from_numpy(g[f"c{i}_points"]), torch.from_numpy(g[f"c{i}_scores"]),
                                   float(g[f"c{i}_dist"]), top_k)
        assert count == int(g[f"c{i}_count"])
        np.testing.assert_array_equal(keep.numpy(), g[f"c{i}_keep"])
    for j in range(2):
        rows = postproc.threshold_rows(torch.from_numpy(g[f"map{j}"])[None, None], 7, 0.4, 4, str(g[f"map{j}_indexing"]))
        np.testing.assert_array_equal(rows.numpy(), g[f"map{j}_rows"])
        np.testing.assert_array_equal(postproc.frame_results(rows).numpy(), g[f"map{j}_final"])


def test_sort_order_restatement_matches_torch_cpu_sort():
    """nms.py:22's ``scores.sort(0)`` on the pinned torch CPU: the restated libstdc++ introsort
    (sequential and the GPU kernel's level-synchronous form) gives torch's index order exactly,
    equal scores included: random ties, NaN, sorted / reversed runs, near-constant arrays, and
    McIlroy killer sequences that reach the heap-sort fallback."""
    from oracle import postproc
    rng = np.random.default_rng(11)
    cases = []
    for t in range(60):
        n = int(rng.integers(1, 1500))
        kind = t % 5
        if kind == 0:
            x = rng.integers(0, 5, n).astype(np.float32)
        elif kind == 1:
            x = rng.uniform(0.4, 1, n).astype(np.float32)
            x[rng.integers(0, n, n // 5)] = np.float32(0.75)
        elif kind == 2:
            x = np.sort(rng.integers(0, 50, n)).astype(np.float32)
        elif kind == 3:
            x = np.sort(rng.integers(0, 50, n))[::-1].astype(np.float32).copy()
        else:
            x = np.full(n, 1.0, np.float32)
            x[rng.integers(0, n, 3)] = 2
        if t % 7 == 0 and n > 4:
            x[rng.integers(0, n, 3)] = np.nan
        cases.append(x)
    cases += [postproc.killer_sequence(n) for n in (40, 300, 1200)]
    for x in cases:
        ref = torch.from_numpy(x).sort(0)[1].tolist()
        assert postproc.std_sort_order(x) == ref, len(x)
        assert postproc.level_sort_order(x) == ref, len(x)
