import sys, numpy as np, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from helpers import parity_stats
from oracle import cpu_path
from mvdet_amd import ops
from mvdet_amd.autograd import project_fuse
from mvdet_amd.pipeline import ProjectFuse
import test_gpu_backward as T
DEV = "cuda:0"
def st(a, b):
    s = parity_stats(a, b); return {k: (round(v, 8) if isinstance(v, float) else v) for k, v in s.items()}
for precision, split_k in [("bf16x3", True), ("bf16x3", False), ("fp32", True)]:
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
    keep["conv1_relu"].retain_grad(); keep["conv2_relu"].retain_grad()
    out_ref.backward(gmap)
    cap = {}
    o_c1 = ops.conv3x3_cout1_backward; o_rb = ops.relu_backward_; o_dg = ops.conv3x3_dgrad
    def c1(x, w, d, dil, relu_mask=False, **k):
        cap["y2"] = x.clone(); r = o_c1(x, w, d, dil, relu_mask=relu_mask, **k); cap["dy2"] = r[0].clone(); return r
    def rb(dy, y):
        cap["y1"] = y.clone(); cap["dy1_pre"] = dy.clone(); r = o_rb(dy, y); cap["dy1"] = r.clone(); return r
    ops.conv3x3_cout1_backward = c1; ops.relu_backward_ = rb
    eng = ProjectFuse([torch.from_numpy(M) for M in Ms], src, grid, C, precision=precision, split_k=split_k)
    mc = torch.nn.Sequential(torch.nn.Conv2d(N * C + 2, 512, 3, padding=1), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 512, 3, padding=2, dilation=2), torch.nn.ReLU(),
                             torch.nn.Conv2d(512, 1, 3, padding=4, dilation=4, bias=False)).to(DEV)
    mc.load_state_dict({k.split(".", 1)[1]: v for k, v in params.items()})
    fg = [f.to(DEV).requires_grad_() for f in feats]
    out = project_fuse(eng, fg, mc)
    out.backward(gmap.to(DEV))
    ops.conv3x3_cout1_backward = o_c1; ops.relu_backward_ = o_rb
    y1r, y2r = keep["conv1_relu"], keep["conv2_relu"]
    print(precision, split_k)
    print(" y1", st(cap["y1"].cpu(), y1r.detach()), " y2", st(cap["y2"].cpu(), y2r.detach()))
    print(" dy2 (post mask)", st(cap["dy2"].cpu(), y2r.grad * (y2r > 0)))
    print(" dy1 pre", st(cap["dy1_pre"].cpu(), y1r.grad))
    print(" dy1 post", st(cap["dy1"].cpu(), y1r.grad * (y1r > 0)))
    flips1 = ((cap["y1"].cpu() > 0) != (y1r > 0)).sum().item(); flips2 = ((cap["y2"].cpu() > 0) != (y2r > 0)).sum().item()
    print(" relu flips y1", flips1, "y2", flips2)
    # dgrad of CPU dy2 with w2
    dd = o_dg((y2r.grad * (y2r > 0)).contiguous().to(DEV), eng._bwd.dgrad2, mc[2].weight, 2)
    print(" dgrad2(cpu dy2)", st(dd[:, :512].cpu(), y1r.grad))
