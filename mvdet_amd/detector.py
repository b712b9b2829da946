"""Drop-in ``PerspTransDetector`` (``multiview_detector/models/persp_trans_detector.py:13-112``).

Same constructor (``dataset`` duck-type, ``arch``), same attributes
(``num_cam``, ``img_shape``, ``reducedgrid_shape``, ``coord_map``,
``upsample_shape``, ``proj_mats``), same sub-modules and therefore the same
``state_dict`` keys (``base_pt1.*``, ``base_pt2.*``, ``img_classifier.*``,
``map_classifier.*``), same ``forward(imgs, visualize=False) ->
(map_result [B,1,Ho,Wo], imgs_result: list[N] of [B,2,h,w])``.

What changes is the hot path (upsample + warp + concat + fusion), which runs on the
HIP kernels of ``libmvbev.so`` through ``ProjectFuse``:
* the 3x upsample of ``:65`` is fused into the warp (the 265 MB/view upsampled map is
  never written) and all views warp in one launch, straight into the fused tensor;
* the image head's first 1x1 conv runs before the upsample (64 instead of 512 channels
  upsampled; it commutes with bilinear interpolation);
* the coord channels are written once, not copied every forward;
* conv1/conv2 are MFMA implicit GEMMs (default 3xbf16 split precision, fp32
  accumulation — same parity as exact fp32; ``precision="fp32"`` selects the
  fp32-input MFMA), conv3 a dot-product kernel;
* the same-size final interpolate (an exact identity) is elided.

Training (autograd through the hot path, ``trainer.py:38-49``):
when grad is required upsample + warp + concat + fusion run as
``autograd.ProjectFuseFunction`` from the backbone-resolution maps — HIP forward (the fused
upsample + warp), HIP backward (the fused upsample + warp adjoint, conv data/weight/bias
gradients).  There is no stock-torch fallback for the hot path.
The library is loaded at construction on a GPU, so a missing build fails there.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native
from . import autograd as native_autograd
from .backbone import build_backbone
from .geometry import coord_map as make_coord_map
from .geometry import projection_matrices, upsample_shape
from .pipeline import ProjectFuse


class PerspTransDetector(nn.Module):
    def __init__(self, dataset, arch: str = "resnet18", device=None, precision: str = "bf16x3",
                 wino_conv1: bool = True, wino_conv2: bool = True, channels_last: bool = True):
        super().__init__()
        self.num_cam = dataset.num_cam
        self.img_shape, self.reducedgrid_shape = list(dataset.img_shape), list(dataset.reducedgrid_shape)
        self.coord_map = make_coord_map(*self.reducedgrid_shape)          # :21 (not a buffer)
        self.upsample_shape = upsample_shape(self.img_shape, dataset.img_reduce)  # :23
        self.proj_mats = projection_matrices(dataset)                       # :18-30 (fp64 list)
        if device is None:
            device = "cuda:0" if torch.cuda.is_available() else "cpu"
        self._device = torch.device(device)
        if self._device.type == "cuda":
            _native.load()  # no fallback: fail at construction if the HIP library is missing
        self.base_pt1, self.base_pt2, out_channel = build_backbone(arch)
        self.img_classifier = nn.Sequential(nn.Conv2d(out_channel, 64, 1), nn.ReLU(),
                                            nn.Conv2d(64, 2, 1, bias=False))
        self.map_classifier = nn.Sequential(nn.Conv2d(out_channel * self.num_cam + 2, 512, 3, padding=1), nn.ReLU(),
                                            nn.Conv2d(512, 512, 3, padding=2, dilation=2), nn.ReLU(),
                                            nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False))
        self.to(self._device)
        # the backbone in torch's channels_last memory format (the same weights and state_dict): its maps then
        # reach the fused upsample warp's line-per-pixel kernel without a transposing copy (cfg2: 0.29-0.32 vs
        # 0.39 ms), and the MIOpen backbone itself ran no slower (7 x 720 x 1280: 21.4 vs 22.8 ms,
        # profiles/r05ah_backbone_layout.json)
        self.channels_last = bool(channels_last)
        if self.channels_last:
            self.base_pt1.to(memory_format=torch.channels_last)
            self.base_pt2.to(memory_format=torch.channels_last)
        # conv1 and conv2 as row-Winograd F(3,3) (ProjectFuse.conv1_wino, conv2_partials), inference and
        # training (forward, data and weight gradients: autograd.py)
        self.engine = ProjectFuse(self.proj_mats, tuple(self.upsample_shape), tuple(self.reducedgrid_shape),
                                  out_channel, precision=precision, wino_conv1=wino_conv1, wino_conv2=wino_conv2)

    # -- hot path --------------------------------------------------------------------------
    def _needs_autograd(self) -> bool:
        return torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())

    def forward(self, imgs: torch.Tensor, visualize: bool = False):
        B, N, C, H, W = imgs.shape
        assert N == self.num_cam
        dev = self._device
        if dev.type != "cuda":
            raise RuntimeError("PerspTransDetector.forward needs a ROCm GPU (the hot path has no CPU fallback)")
        training = self._needs_autograd()
        ws = None if training else self.engine.workspace(B, dev)
        imgs_result, low = [], []
        for cam in range(self.num_cam):
            x = imgs[:, cam].to(dev)
            feat = self.base_pt1(x.contiguous(memory_format=torch.channels_last) if self.channels_last else x)
            feat = self.base_pt2(feat)
            # the image head runs its first 1x1 conv before upsampling (it commutes with the
            # bilinear upsample: per-pixel affine, weights summing to 1) on 64 instead of 512
            # channels
            imgs_result.append(self._img_head_lowres(feat))
            # the 3x upsample (:65) happens inside the fused warp below (and, training, its
            # adjoint inside the warp adjoint)
            # (a channels-last backbone's maps stay channels-last: the fused warp's line-per-pixel kernel)
            cl = feat.dim() == 4 and feat.is_contiguous(memory_format=torch.channels_last)
            low.append(feat if cl else feat.contiguous())
            if visualize:
                up = F.interpolate(feat, self.upsample_shape, mode="bilinear")
                self._show(torch.norm(up[0].detach(), dim=0))
        if training:  # a4-a9 forward and backward on the HIP kernels (autograd.py)
            map_result = native_autograd.project_fuse_backbone(self.engine, low, self.map_classifier)
        else:
            self.engine.warp_views_upsampled(ws, list(range(self.num_cam)), low)  # a4 + a5 + a6
            map_result = self.engine.fuse(ws, self.map_classifier)
        if visualize:
            self._show(torch.norm(map_result[0].detach(), dim=0))
        return map_result, imgs_result

    def _img_head_lowres(self, feat: torch.Tensor) -> torch.Tensor:
        """``img_classifier(F.interpolate(feat, upsample_shape))`` (:65-66) evaluated as
        conv_b(relu(upsample(conv_a(feat)))): identical in exact arithmetic."""
        head = self.img_classifier
        if (len(head) == 3 and isinstance(head[0], nn.Conv2d) and head[0].kernel_size == (1, 1)
                and isinstance(head[1], nn.ReLU)):
            g = head[0](feat)
            return head[2](F.relu(F.interpolate(g, self.upsample_shape, mode="bilinear")))
        return head(F.interpolate(feat, self.upsample_shape, mode="bilinear"))

    @staticmethod
    def _show(img):
        import matplotlib.pyplot as plt
        plt.imshow(img.cpu().numpy())
        plt.show()

    # -- reference helpers (same names) ----------------------------------------------------
    def get_imgcoord2worldgrid_matrices(self, intrinsic_matrices, extrinsic_matrices, worldgrid2worldcoord_mat):
        from .geometry import imgcoord2worldgrid_matrices
        mats = imgcoord2worldgrid_matrices(intrinsic_matrices, extrinsic_matrices, worldgrid2worldcoord_mat,
                                           self.num_cam)
        return {cam: m for cam, m in enumerate(mats)}

    def create_coord_map(self, img_size, with_r=False):
        H, W, _ = img_size
        ret = make_coord_map(H, W)
        if with_r:
            rr = torch.sqrt(ret[:, 0] ** 2 + ret[:, 1] ** 2).view([1, 1, H, W])
            ret = torch.cat([ret, rr], dim=1)
        return ret
