"""Oracle: the reference CPU path of the project+fuse hot path.  TEST INFRASTRUCTURE ONLY.

Restates ``PerspTransDetector`` steps a1-a10 with stock torch-CPU
ops — exactly the ops the reference calls, with kornia replaced by the
``kornia_warp`` restatement:

* a1  ``proj_mats_from_rig``   ``persp_trans_detector.py:18-30, 89-101``
* a2  ``coord_map``            ``:103-112``
* a4  ``upsample``             ``:65`` (the producer of the warp input; "+a4" variant)
* a5  warp per view            ``:68-69``  (``kornia_warp.warp_perspective``)
* a6  ``torch.cat``            ``:77``
* a7-a9 ``map_classifier``     ``:51-54, 81`` (``F.conv2d`` = what ``nn.Conv2d`` runs)
* a10 same-size interpolate    ``:82``

``project_fuse`` is also the ``cpu_baseline`` leg of ``bench.py`` (timed on the
GPU box's host cores, kind "port").
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .kornia_warp import warp_perspective


def proj_mats_from_rig(K, E, G, img_shape, img_reduce, grid_reduce) -> List[np.ndarray]:
    num_cam = len(K)
    perm = np.array([[0, 1, 0], [1, 0, 0], [0, 0, 1]])
    ups = [int(x / img_reduce) for x in img_shape]
    img_zoom = np.diag(np.append(np.array(img_shape) / np.array(ups), [1]))
    map_zoom = np.diag(np.append(np.ones([2]) / grid_reduce, [1]))
    out = []
    for cam in range(num_cam):
        w2i = K[cam] @ np.delete(E[cam], 2, 1) @ G
        out.append(map_zoom @ (perm @ np.linalg.inv(w2i)) @ img_zoom)
    return out


def coord_map(ho: int, wo: int) -> torch.Tensor:
    gx, gy = np.meshgrid(np.arange(wo), np.arange(ho))
    return torch.stack([torch.from_numpy(gx / (wo - 1) * 2 - 1).float(),
                        torch.from_numpy(gy / (ho - 1) * 2 - 1).float()], 0).unsqueeze(0)


def upsample(feat: torch.Tensor, size) -> torch.Tensor:
    """a4: ``F.interpolate(img_feature, self.upsample_shape, mode='bilinear')``
    (``persp_trans_detector.py:65``; align_corners defaults to False)."""
    return F.interpolate(feat, list(size), mode="bilinear")


def warp_views(feats: Sequence[torch.Tensor], proj_mats, grid_hw) -> List[torch.Tensor]:
    out = []
    for f, M in zip(feats, proj_mats):
        B = f.shape[0]
        m = torch.as_tensor(np.asarray(M)).reshape(1, 3, 3).repeat([B, 1, 1]).float()
        out.append(warp_perspective(f, m, list(grid_hw)))
    return out


def fuse(fused: torch.Tensor, params: Dict[str, torch.Tensor], keep: Optional[dict] = None) -> torch.Tensor:
    w1, b1 = params["map_classifier.0.weight"], params["map_classifier.0.bias"]
    w2, b2 = params["map_classifier.2.weight"], params["map_classifier.2.bias"]
    w3 = params["map_classifier.4.weight"]
    y1 = F.relu(F.conv2d(fused, w1, b1, padding=1))
    y2 = F.relu(F.conv2d(y1, w2, b2, padding=2, dilation=2))
    y3 = F.conv2d(y2, w3, None, padding=4, dilation=4)
    if keep is not None:
        keep.update(conv1_relu=y1, conv2_relu=y2)
    return F.interpolate(y3, list(y3.shape[2:]), mode="bilinear")


def project_fuse(feats: Sequence[torch.Tensor], proj_mats, grid_hw, params, keep: Optional[dict] = None,
                 timings: Optional[dict] = None) -> torch.Tensor:
    """feats: N x [B,C,h,w] CPU fp32 (the warp inputs); returns map_result [B,1,ho,wo]."""
    t0 = time.perf_counter()
    warped = warp_views(feats, proj_mats, grid_hw)
    t1 = time.perf_counter()
    B = feats[0].shape[0]
    fused = torch.cat(warped + [coord_map(*grid_hw).repeat([B, 1, 1, 1])], dim=1)
    t2 = time.perf_counter()
    out = fuse(fused, params, keep)
    t3 = time.perf_counter()
    if keep is not None:
        keep["warped"] = warped
        keep["fused"] = fused
    if timings is not None:
        timings.update(warp=t1 - t0, concat=t2 - t1, convs=t3 - t2, total=t3 - t0)
    return out
