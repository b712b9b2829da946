"""One training-step variant alone (for a kernel trace of each): python tools/train_mode.py {update|no_update} [steps]
bench.py's cfg2 training step (native autograd, bf16x3), ``steps`` steps after 10 warm-ups.  GPU only."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from mvdet_amd import ProjectFuse, autograd, synthetic  # noqa: E402
from mvdet_amd.geometry import projection_matrices  # noqa: E402
import bench  # noqa: E402

mode, steps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 60
spec = synthetic.CONFIGS[2]
ds = spec["make"]()
B, C, N = spec["B"], spec["C"], ds.num_cam
up = tuple(ds.upsample_shape)
ho, wo = ds.reducedgrid_shape
dev = torch.device("cuda", 0)
mc = bench.build_mc(C, N, bench.head_params(N, 2, C), dev)
eng = ProjectFuse(projection_matrices(ds), up, (ho, wo), C, precision="bf16x3")
feats = [synthetic.synthetic_features(B, C, [u // 3 for u in up], up, seed=v, device=dev).requires_grad_()
         for v in range(N)]
gmap = torch.randn((B, 1, ho, wo), device=dev)
opt = torch.optim.SGD(mc.parameters(), lr=1e-4, momentum=0.5, weight_decay=5e-4)


def step():
    for f in feats:
        f.grad = None
    mc.zero_grad(set_to_none=True)
    autograd.project_fuse(eng, feats, mc).backward(gmap)
    if mode == "update":
        opt.step()


for _ in range(10):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize()
print(f"{mode}: {(time.perf_counter() - t0) * 1e3 / steps:.3f} ms/step", flush=True)
