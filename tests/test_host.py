"""CPU tests of the product's host side: the C-ABI library loads and exports every
declared symbol, argument validation returns the documented codes (no GPU work is
launched for those), the host geometry matches the reference fixtures/oracle, and
the drop-in module keeps the reference's state_dict layout."""
import ctypes
import os
import re
from pathlib import Path

import numpy as np
import pytest
import torch

from helpers import load_golden
from mvdet_amd import _native, geometry
from oracle import kornia_warp

ROOT = Path(__file__).resolve().parents[1]


def _header_functions():
    text = (ROOT / "include" / "mvbev.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mvbev_\w+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    lib = _native.load()
    declared = _header_functions()
    assert declared == sorted(_native.EXPORTS)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.mvbev_version() == 12400
    assert lib.mvbev_status_string(0) == b"ok"
    assert lib.mvbev_status_string(-100) == b"HIP launch failed"


def test_pixel_major_split_layout_host_checks():
    """MVBEV_LAYOUT_SPLIT_BF16_PIX (ABI 12100) on the host side: the shape helper, the conv-output
    layout inference, and the adjoint's refusals before any launch (C % 8, group stride, mixed
    grad_src layouts) — no GPU compute."""
    from mvdet_amd import ops
    assert ops.split_pix_shape(2, 20, 3, 5) == (2, 3, 5, 3, 2, 8)
    f32 = torch.empty(2, 16, 3, 5)
    sp = torch.empty(ops.split_shape(2, 16, 3, 5), dtype=torch.bfloat16)
    px = torch.empty(ops.split_pix_shape(2, 16, 3, 5), dtype=torch.bfloat16)
    assert ops._out_layout(f32, 2, 16, 3, 5) == _native.LAYOUT_F32
    assert ops._out_layout(sp, 2, 16, 3, 5) == _native.LAYOUT_SPLIT_BF16
    assert ops._out_layout(px, 2, 16, 3, 5) == _native.LAYOUT_SPLIT_PIX
    with pytest.raises(ValueError):
        ops._out_layout(px, 2, 24, 3, 5)
    lib = _native.load()
    fake = ctypes.c_void_p(16)  # never dereferenced: validation fails first
    B, C, H, W, Ho, Wo, G = 1, 16, 6, 7, 4, 5, 4

    def view(gstr, sstr):
        return _native.WarpAdjointView(fake, _native._i64x4(*gstr), fake, _native._i64x4(*sstr), fake, fake, fake)
    good_g = (Ho * Wo * G, 1, Wo * G, G)
    planes = (C * H * W, H * W, W, 1)
    cl = (C * H * W, 1, W * C, C)
    arr = (_native.WarpAdjointView * 1)(view(good_g, planes))
    pix = _native.LAYOUT_SPLIT_PIX
    assert lib.mvbev_warp_views_adjoint(arr, 1, pix, B, 12, H, W, Ho, Wo, 0, None) == -2  # C % 8
    arr = (_native.WarpAdjointView * 1)(view((Ho * Wo * G, 2, Wo * G, G), planes))  # groups not adjacent
    assert lib.mvbev_warp_views_adjoint(arr, 1, pix, B, C, H, W, Ho, Wo, 0, None) == -3
    arr = (_native.WarpAdjointView * 1)(view((Ho * Wo, 1, Wo, 1), planes))  # pixel stride < C / 8 groups
    assert lib.mvbev_warp_views_adjoint(arr, 1, pix, B, C, H, W, Ho, Wo, 0, None) == -3
    arr = (_native.WarpAdjointView * 2)(view(good_g, cl), view(good_g, planes))  # one grad_src layout per launch
    assert lib.mvbev_warp_views_adjoint(arr, 2, pix, B, C, H, W, Ho, Wo, 0, None) == -3
    arr = (_native.WarpAdjointView * 1)(view((G * Ho * Wo, Ho * Wo, Wo, 1), cl))  # channels-last needs pixel-major
    assert lib.mvbev_warp_views_adjoint(arr, 1, _native.LAYOUT_SPLIT_BF16, B, C, H, W, Ho, Wo, 0, None) == -3


def test_argument_validation_codes():
    lib = _native.load()
    s4 = _native._i64x4(1, 1, 1, 1)
    assert lib.mvbev_warp_perspective_f32(None, 1, 1, 1, 1, s4, None, None, 1, 1, s4, None) == -5
    p = ctypes.c_void_p(16)  # never dereferenced: validation fails first
    assert lib.mvbev_warp_perspective_f32(p, 0, 1, 1, 1, s4, p, p, 1, 1, s4, None) == -1
    bad = _native._i64x4(1, 1, 1, 2)
    assert lib.mvbev_warp_perspective_f32(p, 1, 1, 1, 1, s4, p, p, 1, 1, bad, None) == -3
    d = _native.ConvDesc(1, 8, 4, 4, 8, 0, 128, 0, 4, 0, 4)
    assert lib.mvbev_conv3x3_f32(p, ctypes.byref(d), p, None, None, 100, 1, 1, p, None, 0, None) == -2  # Cout % 128
    assert lib.mvbev_conv3x3_f32(p, ctypes.byref(d), p, None, None, 128, 3, 1, p, None, 0, None) == -6  # dilation 3
    assert lib.mvbev_conv3x3_f32(p, ctypes.byref(d), ctypes.c_void_p(20), None, None, 128, 1, 1, p, None, 0, None) == -4
    bad = _native.ConvDesc(1, 12, 4, 4, 12, 0, 192, 0, 4, 0, 4)  # K not a multiple of 8
    assert lib.mvbev_conv3x3_f32(p, ctypes.byref(bad), p, None, None, 128, 1, 1, p, None, 0, None) == -2
    band = _native.ConvDesc(1, 8, 4, 4, 8, 0, 128, 0, 4, 2, 3)  # out rows 2..5 > H
    assert lib.mvbev_conv3x3_f32(p, ctypes.byref(band), p, None, None, 128, 1, 1, p, None, 0, None) == -2
    assert lib.mvbev_conv3x3_f32(p, None, p, None, None, 128, 1, 1, p, None, 0, None) == -5
    assert lib.mvbev_conv3x3_cout1_f32(p, 1, 8, 4, 4, 0, 4, 0, 4, p, 3, p, None, 0, None) == -6
    assert lib.mvbev_conv3x3_cout1_f32(p, 1, 8, 4, 4, 0, 4, 3, 4, p, 4, p, None, 0, None) == -2
    assert lib.mvbev_pack_conv3x3_weight_f32(p, 100, 8, None, 8, p, None) == -2
    assert lib.mvbev_pack_conv3x3_weight_f32(p, 128, 8, None, 16, p, None) == -2  # K != Cin without a map
    assert lib.mvbev_conv3x3_packed_floats(512, 3586) == 3592 * 9 * 512
    assert lib.mvbev_fill_coord_map_f32(None, 1, 2, 2, s4, None) == -5


def test_kornia_matrix_is_bitwise_the_oracle_recipe():
    rng = np.random.default_rng(3)
    for _ in range(5):
        M = torch.from_numpy(np.eye(3) + rng.uniform(-0.3, 0.3, (3, 3))).float()[None]
        got = geometry.kornia_src_norm_from_dst_norm(M, (270, 480), (120, 360))
        ref = kornia_warp.src_norm_from_dst_norm(M, (270, 480), (120, 360))
        assert torch.equal(got, ref)


@pytest.mark.parametrize("name", ["module_wt2", "module_mx3_b2"])
def test_geometry_matches_reference_fixture(name):
    g = load_golden(name)
    m = g["meta"]
    from mvdet_amd.synthetic import SyntheticBase, SyntheticFrameDataset
    base = SyntheticBase("fixture", m["img_shape"], m["worldgrid_shape"], m["num_cam"], g["G"],
                         tuple(g["K"]), tuple(g["E"]))
    ds = SyntheticFrameDataset(base, grid_reduce=m["grid_reduce"], img_reduce=m["img_reduce"])
    assert ds.reducedgrid_shape == m["reducedgrid_shape"] and ds.upsample_shape == m["upsample_shape"]
    got = torch.stack(geometry.projection_matrices(ds)).numpy()
    np.testing.assert_allclose(got, g["proj_mats"], rtol=1e-12, atol=0)
    assert torch.equal(geometry.coord_map(*m["reducedgrid_shape"]), torch.from_numpy(g["coord_map"]))


def test_touched_footprint_matches_oracle():
    g = dict(np.load(ROOT / "tests/golden/geometry_configs.npz", allow_pickle=False))
    for M in g["cfg1_proj_mats"][:2]:
        assert geometry.touched_footprint(M, (270, 480), (160, 250)) == \
            kornia_warp.touched_footprint(M, (270, 480), (160, 250))


def test_detector_state_dict_layout_matches_reference():
    g = load_golden("module_wt2")
    m = g["meta"]
    from mvdet_amd import PerspTransDetector
    from mvdet_amd.synthetic import SyntheticBase, SyntheticFrameDataset
    base = SyntheticBase("fixture", m["img_shape"], m["worldgrid_shape"], m["num_cam"], g["G"],
                         tuple(g["K"]), tuple(g["E"]))
    ds = SyntheticFrameDataset(base, grid_reduce=m["grid_reduce"], img_reduce=m["img_reduce"])
    model = PerspTransDetector(ds, device="cpu")
    shapes = {k: list(v.shape) for k, v in model.state_dict().items()}
    assert shapes == m["state_dict_shapes"]
    assert list(shapes) == list(m["state_dict_shapes"])
    assert model.upsample_shape == m["upsample_shape"]
    assert not any("proj_mats" in k or "coord_map" in k for k in shapes)  # quirk B.4: not buffers
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        model(torch.zeros(1, m["num_cam"], 3, 32, 32))


def test_schedule_plan_covers_every_chunk_once():
    """schedule.plan (host logic, no GPU): every block's chunk range is covered exactly once
    (whole, or by its pieces in K order with consecutive slots and one fixup); XCD i % 8
    order; on 2320 equal blocks over 256 CUs (conv1's dgrad at cfg2: 9.06 rounds) the last
    round is cut into pieces and the simulated makespan drops."""
    from mvdet_amd import schedule
    blocks = [(t, 32) for t in range(2320)]
    sc = schedule.plan(blocks, 256, "cpu")
    items = sc.items.tolist()[:sc.nitems]
    fix = {f[0]: f for f in sc.fixups.tolist()[:sc.nfix]}
    assert sc.nfix > 0 and sc.predicted < sc.predicted_plain
    seen = {}
    for t, c0, c1, slot in items:
        if t < 0:
            continue
        seen.setdefault(t, []).append((c0, c1, slot))
    assert sorted(seen) == list(range(2320))
    for t, parts in seen.items():
        parts.sort()
        assert parts[0][0] == 0 and parts[-1][1] == 32
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        if len(parts) == 1:
            assert parts[0][2] == -1 and t not in fix
        else:
            f = fix[t]
            assert f[2] == len(parts) and [p[2] for p in parts] == list(range(f[1], f[1] + f[2]))
    # masked, heavy-first forward blocks dealt by pixel tile: a tile's Cout blocks on one XCD
    fwd = schedule.ring_blocks(1, 2, 3, 4, 0, group_mask=[1, 3, 7, 0, 5, 1], cpg=2, order=[2, 1, 4, 0, 5, 3])
    assert [c for _, c in fwd[:4]] == [6] * 4 and all(c > 0 for _, c in fwd[:20]) and len(fwd) == 24
    assert all(c == 0 for _, c in fwd[20:])  # the empty pixel tile's blocks: kept (epilogue only)
    sc = schedule.plan(fwd, 16, "cpu", split=False, deal=4)
    its = sc.items.tolist()[:sc.nitems]
    for i, (t, c0, c1, slot) in enumerate(its):
        if t >= 0:
            assert (c0, slot) == (0, -1)
            assert all(j % 8 == i % 8 for j, it in enumerate(its) if it[0] >= 0 and it[0] // 4 == t // 4)


def test_bev_fuse_structs_and_plan_match_the_header(tmp_path):
    """The one-call ABI's structs: ctypes layout == the C header's (compiled here with g++), and
    mvbev_bev_plan_init (host only, no GPU) lays out a workspace whose regions are 256-B aligned,
    in order, and hold T or the slab for the config-2 geometry."""
    import ctypes
    import subprocess
    from mvdet_amd import _native
    src = tmp_path / "sz.cpp"
    src.write_text('#include <cstdio>\n#include <cstddef>\n#include "mvbev.h"\n'
                   'int main(){printf("%zu %zu %zu %zu\\n", sizeof(mvbev_bev_geometry), sizeof(mvbev_bev_plan),'
                   ' offsetof(mvbev_bev_plan, off), offsetof(mvbev_bev_plan, w3));}\n')
    exe = tmp_path / "sz"
    subprocess.run(["g++", "-I", str(Path(__file__).resolve().parents[1] / "include"), str(src), "-o", str(exe)],
                   check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [ctypes.sizeof(_native.BevGeometry), ctypes.sizeof(_native.BevPlan),
                   _native.BevPlan.off.offset, _native.BevPlan.w3.offset]
    g = _native.BevGeometry()
    g.num_views, g.src_kind, g.B, g.C, g.H, g.W, g.Ho, g.Wo = 7, _native.BEV_SRC_F32, 1, 512, 270, 480, 120, 360
    plan = _native.BevPlan()
    lib = _native.load()
    assert lib.mvbev_bev_plan_init(ctypes.byref(g), ctypes.byref(plan)) == 0
    offs = list(plan.off)[:13]
    assert offs == sorted(offs) and all(o % 256 == 0 for o in offs)
    assert plan.Cs == 512 and plan.frustum == 1 and plan.wino == 1 and plan.tiles == 10 * 12
    t_bytes = 1 * (7 * 512 // 8) * 5 * 4 * 10 * 360 * 32  # mvbev_wino_rows_bytes: 5/3 of the slab's rows
    # R_BIG = region 7 (R_MAP1, R_PACK1, R_PACK2, R_INIT, R_MASK, R_ORDER, R_NF, R_BIG, ...; ABI 12300 dropped
    # the coord term's padded input and fp32 pack)
    assert offs[8] - offs[7] >= max(t_bytes, 7 * 512 * 120 * 360 * 4)
    assert lib.mvbev_bev_fuse_workspace_bytes(ctypes.byref(g)) == plan.workspace_bytes
    g.src_kind = _native.BEV_SRC_F16  # fp16 sources: the direct conv1 on the split slab
    assert lib.mvbev_bev_plan_init(ctypes.byref(g), ctypes.byref(plan)) == 0 and plan.wino == 0
    # channels-last sources (ABI 11700): fp32 kinds with whole 32-channel groups only
    for kind, C, ok in ((_native.BEV_SRC_F32, 512, True), (_native.BEV_SRC_F16, 512, False),
                        (_native.BEV_SRC_F32, 40, False)):
        g.src_kind, g.C = kind | _native.BEV_SRC_CHANNELS_LAST, C
        st = lib.mvbev_bev_plan_init(ctypes.byref(g), ctypes.byref(plan))
        assert (st == 0 and plan.wino == 1) if ok else st == _native.ERR_SHAPE, (kind, C, st)
    g.src_kind, g.C = _native.BEV_SRC_F32, 512
    g.num_views = 17
    assert lib.mvbev_bev_plan_init(ctypes.byref(g), ctypes.byref(plan)) == _native.ERR_SHAPE


@pytest.mark.parametrize("gpus,world", [(2, "1"), (1, "2"), (8, "4"), (0, None)])
def test_bench_refuses_a_gpus_world_size_mismatch(gpus, world):
    """bench.py exits non-zero before touching a GPU when ``--gpus`` and the launcher's WORLD_SIZE
    disagree (a line for the wrong N must never be printed), and for ``--gpus < 1``."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    if world is not None:
        env["WORLD_SIZE"] = world
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(gpus), "--no-cpu-baseline"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert "--gpus" in out.stderr


def test_bev_fuse_wrapper_refuses_mismatched_tensors():
    """ops.BevFuse is the only guard in front of the one-call C ABI (raw pointers): wrong weight
    shapes / dtypes and calls before prepare raise before anything is launched."""
    from mvdet_amd import ops
    import torch.nn as nn
    bev = ops.BevFuse([torch.eye(3)] * 2, 16, (20, 30), (10, 12))
    with pytest.raises(RuntimeError, match="prepare"):
        bev([torch.zeros(1, 16, 20, 30)] * 2)
    bad = nn.Sequential(nn.Conv2d(33, 512, 3, padding=1), nn.ReLU(), nn.Conv2d(512, 512, 3, padding=2, dilation=2),
                        nn.ReLU(), nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False))
    with pytest.raises(ValueError, match=r"map_classifier\[0\].weight"):
        bev.prepare(bad, "cpu")
    bad[0] = nn.Conv2d(34, 512, 3, padding=1)
    bad[4] = nn.Conv2d(512, 2, 3, padding=4, dilation=4, bias=False)
    with pytest.raises(ValueError, match=r"map_classifier\[4\].weight"):
        bev.prepare(bad, "cpu")
    bad[4] = nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False).double()
    with pytest.raises(ValueError, match=r"map_classifier\[4\].weight"):
        bev.prepare(bad, "cpu")


def test_hot_kernels_use_no_scratch():
    """The inference and training hot kernels keep their accumulators in registers: no scratch
    (private segment) in the build's resource report (``build/obj/*.o.res``, written by the Makefile).
    A branch inside an unrolled epilogue once put the ring / Winograd convs' accumulators in 448 B of
    scratch per lane and made the training conv1 5x slower without any test failing."""
    res = sorted((ROOT / "build" / "obj").glob("*.o.res"))
    if not res:
        pytest.skip("no build resource reports (build with make -C mvdet_amd/csrc)")
    # every kernel but the register-tiled bf16x3 conv (b3::conv_kernel: the fallback form, no longer on
    # the product path, keeps a 12-36 B spill); round 5 found the bias / coord-gradient reduction
    # spilling 676 B per lane (block_sum's hoisted LDS loads), 2x slower, outside the old list
    legacy = re.compile(r"2b311conv_kernel")
    seen, bad = 0, []
    for f in res:
        name = None
        for line in f.read_text().splitlines():
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                name = m.group(1)
                continue
            m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
            if m and name and not legacy.search(name):
                seen += 1
                if int(m.group(1)):
                    bad.append((f.name, name, int(m.group(1))))
    assert seen >= 20, seen
    assert not bad, bad


def test_design_cost_model_table_is_current():
    """DESIGN.md §6's per-mode table is what mvdet_amd.mp_model predicts from its committed inputs
    (tools/mp_cost_model.py), so the documented N>1 mode choice is the one bench.py --mp-mode auto makes."""
    import subprocess
    import sys
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "mp_cost_model.py")], cwd=ROOT, capture_output=True,
                         text=True, timeout=300, check=True).stdout
    rows = [ln.replace(" ms (x)", "") for ln in out.splitlines() if ln.startswith("| ")]
    design = (ROOT / "DESIGN.md").read_text()
    assert len(rows) == 18  # header + 4 configs x 4 rank counts + config 4 at P = 6
    for row in rows:
        assert row in design, row


def test_wgrad_chunk_lists_match_brute_force():
    """Host planning of the conv1 weight gradients' frustum chunk lists: the direct form's (row y,
    32-px segment) chunks of 8-row tiles and the Winograd form's (3-row tile r3, segment) chunks of
    the 12-row mask T was written under, per channel group, against a brute-force enumeration."""
    from mvdet_amd import ops
    rng = np.random.default_rng(4)
    B, H, W, groups = 2, 37, 104, 3
    tx = -(-W // 32)
    for tile_h, lister, rows in ((_native.TILE_H, ops.wgrad_chunk_lists, H),
                                 (12, ops.wgrad_wino_chunk_lists, -(-H // 3))):
        ty = -(-H // tile_h)
        mask = torch.tensor(rng.integers(0, 1 << groups, ty * tx), dtype=torch.int32)
        lst, off = lister(mask, groups, B, H, W)
        lst, off = lst.tolist(), off.tolist()
        rows_per_tile = tile_h if lister is ops.wgrad_chunk_lists else 4  # 3-row tiles r3 per 12-row tile
        for g in range(groups):
            want = [b * rows * tx + r * tx + s for b in range(B) for r in range(rows) for s in range(tx)
                    if (int(mask[(r // rows_per_tile) * tx + s]) >> g) & 1]
            assert lst[off[g]:off[g + 1]] == want, (lister.__name__, g)
    with pytest.raises(ValueError):
        ops.wgrad_wino_chunk_lists(torch.zeros(5, dtype=torch.int32), groups, B, H, W)


def test_wino43_policy_per_config():
    """ProjectFuse.wino43_pays (ABI 12400): conv1 takes F(4,3) where its 16-row tiles waste <= 3 % of the grid's rows
    (configs 1, 3, 4, 5; config 2's 120 rows leave half a tile idle), conv2 -> conv3 only where the launch is also
    >= 8 rounds of workgroups deep (configs 3, 4, 5 on 256 CUs); wino43=False / True override; the partial-sum
    engines (view parts) never take it (conv1_partial reads F(3,3)'s T)."""
    from mvdet_amd import ProjectFuse, synthetic
    from mvdet_amd.geometry import projection_matrices
    want = {1: (True, False), 2: (False, False), 3: (True, True), 4: (True, True), 5: (True, True)}
    for cfg, (c1, c2) in want.items():
        spec = synthetic.CONFIGS[cfg]
        ds = spec["make"]()
        pm, up, grid = projection_matrices(ds), tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
        e = ProjectFuse(pm, up, grid, 32)
        e._cus["cpu"] = 256
        H = grid[0]
        assert (e.wino43_pays(H, spec["B"], "cpu"), e.wino43_pays(H, spec["B"], "cpu", deep=True)) == (c1, c2), cfg
        assert not ProjectFuse(pm, up, grid, 32, wino43=False).wino43_pays(H, spec["B"], "cpu")
        assert ProjectFuse(pm, up, grid, 32, wino43=True).wino43_pays(H, spec["B"], "cpu", deep=True)
    ds = synthetic.CONFIGS[3]["make"]()
    pm, up, grid = projection_matrices(ds), tuple(ds.upsample_shape), tuple(ds.reducedgrid_shape)
    part = ProjectFuse(pm, up, grid, 32, parts=[(0, 0), (1, 0)], part_channels=32, all_views=False)
    assert not part.wino43 and not part.wino43_pays(grid[0], 1, "cpu")

