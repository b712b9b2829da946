"""Generate the golden fixtures in ``tests/golden`` from the reference itself.

Runs ONLY in the build container (needs ``/root/reference``).  The reference's
``PerspTransDetector`` is imported through ``tools/ref_harness.py`` (kornia
stubbed with the oracle restatement, ``cuda:0`` redirected to CPU), its
``base_pt1``/``base_pt2`` backbone halves are replaced by ``nn.Identity`` so
that ``forward`` receives backbone-resolution features directly, and its
``img_classifier``/``map_classifier`` weights are set from the deterministic
recipe in ``oracle/fixtures.py``.  Everything downstream — the matrix chain
(``persp_trans_detector.py:18-30,89-101``), the coord map (``:103-112``), the
3x upsample (``:65``), the warp call (``:69``), concat (``:77``), the three
convs (``:51-54,81``) and the final interpolate (``:82``) — is the reference's
own code.

Usage:  python tools/gen_golden.py        (writes tests/golden/*.npz)
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))

from ref_harness import load_reference_detector  # noqa: E402
from oracle.fixtures import head_params, params_sha256, feature_input  # noqa: E402
from mvdet_amd import synthetic  # noqa: E402

OUT = ROOT / "tests" / "golden"


def _rig_arrays(ds):
    b = ds.base
    return dict(K=np.stack(b.intrinsic_matrices), E=np.stack(b.extrinsic_matrices),
                G=np.asarray(b.worldgrid2worldcoord_mat, np.float64))


def _meta(ds, **extra):
    d = dict(num_cam=ds.num_cam, img_shape=list(ds.img_shape), worldgrid_shape=list(ds.worldgrid_shape),
             grid_reduce=ds.grid_reduce, img_reduce=ds.img_reduce, reducedgrid_shape=ds.reducedgrid_shape,
             upsample_shape=ds.upsample_shape, rig=ds.base.name)
    d.update(extra)
    return json.dumps(d)


def run_module_case(name, ds, B, backbone_hw, wseed, fseed, store_full):
    P = load_reference_detector()
    torch.manual_seed(0)
    model = P(ds)
    full_sd_shapes = {k: list(v.shape) for k, v in model.state_dict().items()}
    model.base_pt1 = nn.Identity()
    model.base_pt2 = nn.Identity()
    params = head_params(ds.num_cam, wseed)
    sd = model.state_dict()
    for k, v in params.items():
        assert tuple(sd[k].shape) == v.shape, (k, sd[k].shape, v.shape)
        sd[k] = torch.from_numpy(v)
    model.load_state_dict(sd)
    model.eval()

    feats = feature_input((B, ds.num_cam, 512, *backbone_hw), fseed)
    # capture the warp inputs/outputs and the conv activations with hooks
    import oracle.kornia_warp as kw
    captured = {"warp_in": [], "warp_out": []}
    orig = kw.warp_perspective

    def spy(src, M, dsize, **kwargs):
        out = orig(src, M, dsize, **kwargs)
        captured["warp_in"].append(src.detach().clone())
        captured["warp_out"].append(out.detach().clone())
        return out

    sys.modules["kornia.geometry.transform"].warp_perspective = spy
    acts = {}
    hooks = [model.map_classifier[1].register_forward_hook(lambda m, i, o: acts.__setitem__("c1", o.detach().clone())),
             model.map_classifier[3].register_forward_hook(lambda m, i, o: acts.__setitem__("c2", o.detach().clone()))]
    with torch.no_grad():
        map_res, imgs_res = model(torch.from_numpy(feats))
    for h in hooks:
        h.remove()
    sys.modules["kornia.geometry.transform"].warp_perspective = orig

    warp_out = torch.stack(captured["warp_out"], 1).numpy()  # [B, N, C, ho, wo]
    warp_in = torch.stack(captured["warp_in"], 1).numpy()    # [B, N, C, h, w]
    arrays = dict(
        meta=np.array(_meta(ds, B=B, backbone_hw=list(backbone_hw), weight_seed=wseed, feature_seed=fseed,
                            weights_sha256=params_sha256(params), state_dict_shapes=full_sd_shapes)),
        proj_mats=np.stack([m.numpy() for m in model.proj_mats]),
        coord_map=model.coord_map.numpy(),
        feat_in=feats,
        imgs_result=torch.stack(imgs_res, 0).numpy(),
        map_result=map_res.numpy(),
        warp_in_chsum=warp_in.astype(np.float64).sum(axis=(3, 4)),
        warp_out_chsum=warp_out.astype(np.float64).sum(axis=(3, 4)),
        **_rig_arrays(ds),
    )
    if store_full:
        arrays.update(warp_out=warp_out, conv1_relu=acts["c1"].numpy(), conv2_relu=acts["c2"].numpy())
    np.savez_compressed(OUT / f"{name}.npz", **arrays)
    print(name, {k: v.shape for k, v in arrays.items()}, "map max", float(np.abs(arrays["map_result"]).max()))


def run_geometry_case():
    """Reference matrix chain at the BASELINE.json config sizes (synthetic rigs)."""
    P = load_reference_detector()
    arrays = {}
    for k, cfg in synthetic.CONFIGS.items():
        ds = cfg["make"]()
        torch.manual_seed(0)
        model = P(ds)
        arrays[f"cfg{k}_proj_mats"] = np.stack([m.numpy() for m in model.proj_mats])
        for key, v in _rig_arrays(ds).items():
            arrays[f"cfg{k}_{key}"] = v
        arrays[f"cfg{k}_meta"] = np.array(_meta(ds))
        if k == 2:
            arrays["cfg2_coord_map"] = model.coord_map.numpy()
        del model
    np.savez_compressed(OUT / "geometry_configs.npz", **arrays)
    print("geometry_configs", sorted(arrays))


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    run_module_case("module_wt2", synthetic.wildtrack_like(2, 4, seed=11, img_shape=(108, 192),
                                                           worldgrid_shape=(48, 144)),
                    B=1, backbone_hw=(9, 16), wseed=101, fseed=201, store_full=True)
    run_module_case("module_mx3_b2", synthetic.multiviewx_like(3, 2, seed=12, img_shape=(72, 128),
                                                               worldgrid_shape=(40, 60)),
                    B=2, backbone_hw=(6, 11), wseed=102, fseed=202, store_full=False)
    run_geometry_case()


if __name__ == "__main__":
    main()
