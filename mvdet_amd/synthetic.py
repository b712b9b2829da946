"""Synthetic camera rigs and the dataset duck-type ``PerspTransDetector`` reads.

The real calibrations (Wildtrack / MultiviewX) are not in this image, so every
workload uses synthetic pinhole rigs (SURVEY §8(d) "Synthetic inputs"):
cameras on an ellipse around the ground-area centre, at a fixed height, aimed
at the centre with a seeded yaw jitter.  Their K / [R|t] go through the
reference's own matrix chain (``persp_trans_detector.py:89-101``), so the
homographies have the same structure (and quirks) as the real ones.

Conventions mirrored from the reference datasets:
* Wildtrack: img 1080x1920, worldgrid 480x1440 ('ij' indexing), units cm,
  ``worldgrid2worldcoord_mat = [[2.5,0,-300],[0,2.5,-900],[0,0,1]]``
  (``datasets/Wildtrack.py:20-25``).
* MultiviewX: img 1080x1920, worldgrid 640x1000 ('xy' indexing), units m,
  ``[[0,0.025,0],[0.025,0,0],[0,0,1]]`` (``datasets/MultiviewX.py:20-25``).
* frameDataset: ``reducedgrid_shape = worldgrid_shape / grid_reduce``,
  ``img_reduce = 4`` (``datasets/frameDataset.py:14,24``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Sequence

import numpy as np


def look_at_extrinsic(cam_pos: np.ndarray, target: np.ndarray) -> np.ndarray:
    """3x4 [R|t] of a camera at ``cam_pos`` looking at ``target`` (z up,
    image x right, image y down)."""
    fwd = target - cam_pos
    fwd = fwd / np.linalg.norm(fwd)
    right = np.cross(fwd, np.array([0.0, 0.0, 1.0]))
    right = right / np.linalg.norm(right)
    down = np.cross(fwd, right)
    R = np.stack([right, down, fwd], axis=0)
    t = -R @ cam_pos
    return np.hstack([R, t[:, None]])


def pinhole_intrinsic(img_shape: Sequence[int], focal_at_1080p: float = 1700.0) -> np.ndarray:
    H, W = img_shape
    f = focal_at_1080p * H / 1080.0
    return np.array([[f, 0.0, (W - 1) / 2.0], [0.0, f, (H - 1) / 2.0], [0.0, 0.0, 1.0]])


@dataclass
class SyntheticBase:
    """Duck-type of ``Wildtrack`` / ``MultiviewX`` (the fields the detector reads)."""
    name: str
    img_shape: List[int]
    worldgrid_shape: List[int]
    num_cam: int
    worldgrid2worldcoord_mat: np.ndarray
    intrinsic_matrices: tuple = field(default_factory=tuple)
    extrinsic_matrices: tuple = field(default_factory=tuple)
    root: str = "<synthetic>"


@dataclass
class SyntheticFrameDataset:
    """Duck-type of ``frameDataset`` (``datasets/frameDataset.py:13-24``)."""
    base: SyntheticBase
    grid_reduce: int = 4
    img_reduce: int = 4

    @property
    def num_cam(self) -> int:
        return self.base.num_cam

    @property
    def img_shape(self) -> List[int]:
        return list(self.base.img_shape)

    @property
    def worldgrid_shape(self) -> List[int]:
        return list(self.base.worldgrid_shape)

    @property
    def reducedgrid_shape(self) -> List[int]:
        return [int(x / self.grid_reduce) for x in self.base.worldgrid_shape]

    @property
    def upsample_shape(self) -> List[int]:
        return [int(x / self.img_reduce) for x in self.base.img_shape]


def make_rig(name: str, img_shape, worldgrid_shape, num_cam: int, G: np.ndarray,
             height: float, seed: int, radius_scale: float = 0.75) -> SyntheticBase:
    """Cameras on an ellipse around the ground-area centre (world units of G)."""
    rng = np.random.default_rng(seed)
    corners = np.array([[0, 0, 1], [worldgrid_shape[0], worldgrid_shape[1], 1]], dtype=np.float64)
    world = (G @ corners.T).T[:, :2]
    lo, hi = world.min(0), world.max(0)
    centre = (lo + hi) / 2
    half = (hi - lo) / 2
    K = pinhole_intrinsic(img_shape)
    intr, extr = [], []
    for cam in range(num_cam):
        ang = 2 * np.pi * cam / num_cam + rng.uniform(-0.15, 0.15)
        pos = np.array([centre[0] + radius_scale * 1.4 * half[0] * np.cos(ang),
                        centre[1] + radius_scale * 1.4 * half[1] * np.sin(ang), height])
        jitter = rng.uniform(-0.25, 0.25, size=2) * half
        target = np.array([centre[0] + jitter[0], centre[1] + jitter[1], 0.0])
        intr.append(K.copy())
        extr.append(look_at_extrinsic(pos, target))
    return SyntheticBase(name, list(img_shape), list(worldgrid_shape), num_cam,
                         np.asarray(G, dtype=np.float64), tuple(intr), tuple(extr))


WILDTRACK_G = np.array([[2.5, 0, -300], [0, 2.5, -900], [0, 0, 1]], dtype=np.float64)
MULTIVIEWX_G = np.array([[0, 0.025, 0], [0.025, 0, 0], [0, 0, 1]], dtype=np.float64)


def wildtrack_like(num_cam: int = 7, grid_reduce: int = 4, seed: int = 2,
                   img_shape=(1080, 1920), worldgrid_shape=(480, 1440)) -> SyntheticFrameDataset:
    base = make_rig("Wildtrack-synthetic", img_shape, worldgrid_shape, num_cam, WILDTRACK_G,
                    height=250.0, seed=seed)
    return SyntheticFrameDataset(base, grid_reduce=grid_reduce, img_reduce=4)


def multiviewx_like(num_cam: int = 6, grid_reduce: int = 4, seed: int = 1,
                    img_shape=(1080, 1920), worldgrid_shape=(640, 1000)) -> SyntheticFrameDataset:
    base = make_rig("MultiviewX-synthetic", img_shape, worldgrid_shape, num_cam, MULTIVIEWX_G,
                    height=2.5, seed=seed)
    return SyntheticFrameDataset(base, grid_reduce=grid_reduce, img_reduce=4)


def synthetic_4k(num_cam: int = 8, seed: int = 5) -> SyntheticFrameDataset:
    """Config 5: 8 views at 2160x3840, 1000x1000 grid (grid_reduce 1), 2.5 cm cells."""
    G = np.array([[0.025, 0, 0], [0, 0.025, 0], [0, 0, 1]], dtype=np.float64)
    base = make_rig("Synthetic-4K", (2160, 3840), (1000, 1000), num_cam, G, height=3.0, seed=seed)
    return SyntheticFrameDataset(base, grid_reduce=1, img_reduce=4)


# BASELINE.json configs -> (dataset factory, B, C, dtype)
CONFIGS = {
    1: dict(name="MultiviewX 6-view C=128 160x250", make=lambda: multiviewx_like(6, 4, seed=1), B=1, C=128),
    2: dict(name="Wildtrack 7-view C=512 120x360", make=lambda: wildtrack_like(7, 4, seed=2), B=1, C=512),
    3: dict(name="Wildtrack 7-view C=512 480x1440", make=lambda: wildtrack_like(7, 1, seed=3), B=1, C=512),
    4: dict(name="MultiviewX 6-view B=8 C=512 160x250 fp16", make=lambda: multiviewx_like(6, 4, seed=4), B=8, C=512),
    5: dict(name="Synthetic 8-view 4K C=256 1000x1000", make=lambda: synthetic_4k(8, seed=5), B=1, C=256),
}


def backbone_features(B: int, C: int, backbone_hw, seed: int, device="cpu"):
    """ReLU(N(0,1)) at backbone resolution [B, C, h, w] (the map ``:64`` produces)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return torch.randn(B, C, *backbone_hw, generator=g, device=device).clamp_min_(0)


def synthetic_features(B: int, C: int, backbone_hw, upsample_hw, seed: int, device="cpu"):
    """ReLU(N(0,1)) at backbone resolution, bilinearly upsampled (``:64-65``).

    Returns [B, C, h, w] float32 on ``device`` (generated on that device).
    """
    import torch.nn.functional as F
    x = backbone_features(B, C, backbone_hw, seed, device)
    return F.interpolate(x, list(upsample_hw), mode="bilinear")
