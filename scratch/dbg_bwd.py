import sys, numpy as np, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from helpers import parity_stats
from oracle import cpu_path, fixtures
from mvdet_amd import ops
from mvdet_amd.autograd import project_fuse
from mvdet_amd.pipeline import ProjectFuse
import test_gpu_backward as T
DEV = "cuda:0"
for precision in ["bf16x3", "fp32"]:
  for frustum in [True, False]:
    N, B, C, src, grid = 2, 1, 8, (27, 48), (12, 36)
    rng = np.random.default_rng(N * 31 + C)
    H, W = src; ho, wo = grid
    Ms = [T._rand_h(rng, H, W, ho, wo) for _ in range(N)]
    feats = [torch.from_numpy(np.maximum(rng.standard_normal((B, C, H, W)), 0).astype(np.float32)) for _ in range(N)]
    params = T._head(N, C, seed=N + C)
    gmap = torch.from_numpy(rng.standard_normal((B, 1, ho, wo)).astype(np.float32))
    fr = [f.clone().requires_grad_() for f in feats]
    pr = {k: v.clone().requires_grad_() for k, v in params.items()}
    keep = {}
    out_ref = cpu_path.project_fuse(fr, Ms, grid, pr, keep=keep)
    for w in keep["warped"]: w.retain_grad()
    keep["conv1_relu"].retain_grad(); keep["conv2_relu"].retain_grad()
    out_ref.backward(gmap)
    cap = {}
    orig = ops.warp_views_backward
    def spy(g, m, d):
        cap["g"] = [x.clone() for x in g]; cap["m"] = m
        return orig(g, m, d)
    ops.warp_views_backward = spy
    import mvdet_amd.autograd as A
    eng = ProjectFuse([torch.from_numpy(M) for M in Ms], src, grid, C, precision=precision, frustum=frustum)
    mc = torch.nn.Sequential(torch.nn.Conv2d(N * C + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)
    mc.load_state_dict({k.split(".", 1)[1]: v for k, v in params.items()})
    fg = [f.to(DEV).requires_grad_() for f in feats]
    out = project_fuse(eng, fg, mc)
    out.backward(gmap.to(DEV))
    ops.warp_views_backward = orig
    print(precision, frustum, "fwd", parity_stats(out.detach(), out_ref.detach())["normwise"])
    for i in range(N):
        print(" dslab view", i, parity_stats(cap["g"][i].cpu(), keep["warped"][i].grad))
        print(" dfeat view", i, parity_stats(fg[i].grad.cpu(), fr[i].grad))
        # warp adjoint of the CPU dslab through the native kernel
        d = torch.zeros((B, C, H, W), device=DEV)
        orig([keep["warped"][i].grad.to(DEV)], [cap["m"][i]], [d])
        print(" adjoint(cpu dslab) view", i, parity_stats(d.cpu(), fr[i].grad))
        print(" m", cap["m"][i].flatten().tolist())
