"""The project+fuse hot path as one reusable engine.

``ProjectFuse`` owns, per (device, batch size):

* ``fused``  — the ground-plane tensor ``[B, Cin_pad, Ho, Wo]`` fp32, NCHW, the
  concatenation of ``persp_trans_detector.py:77`` made zero-copy: view ``v``'s
  warp writes channels ``[v*C, (v+1)*C)``, the coord map occupies channels
  ``N*C`` and ``N*C+1`` (written once at allocation), channels up to
  ``Cin_pad = roundup(N*C+2, 8)`` are zero padding for the MFMA K granule.
* ``y1``, ``y2`` — conv1 / conv2 activations ``[B, 512, Ho, Wo]``.
* the per-view kornia ``src_norm <- dst_norm`` matrices, uploaded once.

``warp_view`` is a5 for one view, ``fuse`` is a7-a9 (a10, the same-size
bilinear interpolate of ``:82``, is an exact identity and is elided).  Nothing
here allocates in steady state, copies to the host or synchronises.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import torch

from . import ops
from .geometry import kornia_src_norm_from_dst_norm


@dataclass
class Workspace:
    fused: torch.Tensor
    y1: torch.Tensor
    y2: torch.Tensor
    m_norm: torch.Tensor  # [N, B, 3, 3] device fp32


class ProjectFuse:
    def __init__(self, proj_mats: Sequence[torch.Tensor], src_hw: Tuple[int, int], grid_hw: Tuple[int, int],
                 channels: int, mid_channels: int = 512):
        self.num_cam = len(proj_mats)
        self.src_hw = (int(src_hw[0]), int(src_hw[1]))
        self.grid_hw = (int(grid_hw[0]), int(grid_hw[1]))
        self.C = int(channels)
        self.mid = int(mid_channels)
        self.cin = self.num_cam * self.C + 2
        self.cin_pad = ops.padded_channels(self.cin)
        # kornia steps 1-2 (normalize_homography + _torch_inverse_cast) on the host, fp32,
        # from the fp32-cast projection matrix exactly as :68-69 feeds kornia.
        self.m_norm_cpu = torch.stack([
            kornia_src_norm_from_dst_norm(M.float().reshape(1, 3, 3), self.src_hw, self.grid_hw)[0]
            for M in proj_mats])  # [N, 3, 3]
        self._ws: Dict[Tuple[str, int], Workspace] = {}
        self.pack1 = ops.PackedConv3x3()
        self.pack2 = ops.PackedConv3x3()

    def workspace(self, B: int, device) -> Workspace:
        device = torch.device(device)
        key = (str(device), int(B))
        ws = self._ws.get(key)
        if ws is None:
            ho, wo = self.grid_hw
            fused = torch.zeros((B, self.cin_pad, ho, wo), dtype=torch.float32, device=device)
            nc = self.num_cam * self.C
            ops.fill_coord_map(fused[:, nc:nc + 2])
            y1 = torch.empty((B, self.mid, ho, wo), dtype=torch.float32, device=device)
            y2 = torch.empty_like(y1)
            m = self.m_norm_cpu.to(device)[:, None].expand(self.num_cam, B, 3, 3).contiguous()
            ws = Workspace(fused, y1, y2, m)
            self._ws[key] = ws
        return ws

    def view_slice(self, ws: Workspace, cam: int) -> torch.Tensor:
        return ws.fused[:, cam * self.C:(cam + 1) * self.C]

    def warp_view(self, ws: Workspace, cam: int, feat: torch.Tensor) -> None:
        """a5 (+ zero-copy a6): warp one view's [B,C,h,w] features into ``fused``."""
        if tuple(feat.shape[2:]) != self.src_hw or feat.shape[1] != self.C:
            raise ValueError(f"view {cam}: features {tuple(feat.shape)} do not match "
                             f"[B,{self.C},{self.src_hw[0]},{self.src_hw[1]}]")
        ops.warp_into(feat, ws.m_norm[cam], self.view_slice(ws, cam))

    def fuse(self, ws: Workspace, map_classifier: torch.nn.Sequential) -> torch.Tensor:
        """a7-a9 on ``ws.fused`` with the parameters of ``map_classifier`` → [B,1,Ho,Wo]."""
        c1, c2, c3 = map_classifier[0], map_classifier[2], map_classifier[4]
        p1 = self.pack1.get(c1.weight)
        p2 = self.pack2.get(c2.weight)
        ops.conv3x3(ws.fused, p1, self.cin, self.mid, c1.bias, dilation=1, relu=True, out=ws.y1)
        ops.conv3x3(ws.y1, p2, self.mid, self.mid, c2.bias, dilation=2, relu=True, out=ws.y2)
        return ops.conv3x3_cout1(ws.y2, c3.weight, dilation=4)

    def project_fuse(self, feats: Sequence[torch.Tensor], map_classifier) -> torch.Tensor:
        """Whole hot path: warp every view, concat (zero-copy), fuse."""
        B = feats[0].shape[0]
        ws = self.workspace(B, feats[0].device)
        for cam, f in enumerate(feats):
            self.warp_view(ws, cam, f)
        return self.fuse(ws, map_classifier)
