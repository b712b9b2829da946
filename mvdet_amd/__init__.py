"""mvdet_amd — MI355X-native MVDet perspective-transform hot path.

Public surface (mirrors the reference's):
* ``PerspTransDetector`` — drop-in for
  ``multiview_detector.models.persp_trans_detector.PerspTransDetector``.
* ``warp_perspective`` — drop-in for kornia 0.6.11
  ``kornia.geometry.transform.warp_perspective`` (default-argument path).
* ``ProjectFuse`` — the hot path (warp + zero-copy concat + fusion) as an engine.
* ``postprocess.nms`` / ``threshold_rows`` / ``frame_results`` — drop-ins for
  ``multiview_detector.utils.nms.nms`` and the evaluation rows of ``trainer.py:97-157``.

The compute runs in ``mvdet_amd/lib/libmvbev.so`` (HIP, gfx950; C ABI in
``include/mvbev.h``); there is no CPU fallback.
"""
from .detector import PerspTransDetector  # noqa: F401
from .ops import warp_perspective  # noqa: F401
from .pipeline import ProjectFuse  # noqa: F401
from . import postprocess  # noqa: F401

__all__ = ["PerspTransDetector", "warp_perspective", "ProjectFuse", "postprocess"]
