"""CPU oracle for the MVDet project+fuse hot path.  TEST INFRASTRUCTURE ONLY.

This package is the parity checker for the HIP path in ``mvdet_amd``.  Only
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import it, and only as the checker / the timed CPU baseline;
the product (``mvdet_amd``) never imports, links or executes anything here.

Contents
--------
``kornia_warp``  restatement of kornia 0.6.11 ``warp_perspective`` (the
                 third-party op the reference calls at
                 ``multiview_detector/models/persp_trans_detector.py:69``),
                 run over stock torch-CPU ``F.grid_sample``; plus a float64
                 closed-form bilinear-homography sampler used to pin it.
``cpu_path``     the reference CPU path of the hot path
                 (``persp_trans_detector.py:62-82``): matrix chain, coord map,
                 warp of every view, channel concat, the three ``nn.Conv2d`` of
                 ``map_classifier`` and the same-size interpolate.

Pinning: kornia 0.6.11 is not installed and cannot be
fetched, so the warp restatement is pinned by (1) the float64 closed form and
(2) golden fixtures generated in the build container by running the
reference's own ``PerspTransDetector.forward`` (kornia stubbed with this
restatement) — ``tools/gen_golden.py``.  The fixtures pin the matrix chain,
coord map, concat order, layer hyper-parameters and the forward contract; the
closed form pins the warp arithmetic.
"""
