"""Import the reference's own ``PerspTransDetector`` on CPU (build container only).

Used only by ``tools/gen_golden.py`` to produce the committed fixtures under
``tests/golden``.  Never imported by the product, tests, bench or smoke (the
reference does not exist on the GPU box).

Stubs installed before the import:
* ``kornia`` / ``kornia.geometry`` / ``kornia.geometry.transform``: the oracle's
  restatement of kornia 0.6.11 ``warp_perspective`` (kornia is not installed).
* ``torchvision.models.vgg``: a placeholder (only ``arch='vgg11'`` uses it).
* ``nn.Module.to`` / ``Tensor.to``: ``'cuda:0'`` is redirected to ``'cpu'``
  (the reference pins every module and tensor to ``cuda:0``).
"""
from __future__ import annotations

import sys
import types

import torch
import torch.nn as nn

REF_ROOT = "/root/reference"


_INSTALLED = False


def _install_stubs():
    global _INSTALLED
    if _INSTALLED:
        return
    _INSTALLED = True
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[1]))
    from oracle import kornia_warp

    kornia = types.ModuleType("kornia")
    geometry = types.ModuleType("kornia.geometry")
    transform = types.ModuleType("kornia.geometry.transform")
    transform.warp_perspective = kornia_warp.warp_perspective
    geometry.transform = transform
    kornia.geometry = geometry
    kornia.warp_perspective = kornia_warp.warp_perspective
    sys.modules.update({"kornia": kornia, "kornia.geometry": geometry,
                        "kornia.geometry.transform": transform})

    if "torchvision" not in sys.modules:
        tv = types.ModuleType("torchvision")
        models = types.ModuleType("torchvision.models")
        vgg = types.ModuleType("torchvision.models.vgg")

        def vgg11(*a, **k):
            raise RuntimeError("vgg11 is not available in the build container")

        vgg.vgg11 = vgg11
        models.vgg = vgg
        tv.models = models
        sys.modules.update({"torchvision": tv, "torchvision.models": models,
                            "torchvision.models.vgg": vgg})

    def _fix(args, kwargs):
        args = tuple("cpu" if (isinstance(a, str) and a.startswith("cuda")) else a for a in args)
        if isinstance(kwargs.get("device"), str) and kwargs["device"].startswith("cuda"):
            kwargs["device"] = "cpu"
        return args, kwargs

    orig_mod_to = nn.Module.to
    orig_t_to = torch.Tensor.to

    def mod_to(self, *args, **kwargs):
        args, kwargs = _fix(args, kwargs)
        return orig_mod_to(self, *args, **kwargs)

    def t_to(self, *args, **kwargs):
        args, kwargs = _fix(args, kwargs)
        return orig_t_to(self, *args, **kwargs)

    nn.Module.to = mod_to
    torch.Tensor.to = t_to


def load_reference_detector():
    _install_stubs()
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    import matplotlib
    matplotlib.use("Agg")
    from multiview_detector.models.persp_trans_detector import PerspTransDetector
    return PerspTransDetector
