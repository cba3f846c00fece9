"""Diagnostic: stage-by-stage error of the explicit CNN forward (fused_cnn._Trunk) against an f64 CPU forward of the
same weights, at the G9P shape (Basic_CNN [32, 64, 64] / [8, 4, 3] / [4, 2, 1], batch 2048 of uniform uint8 frames).
The GPU runs the whole batch (library algorithm choice depends on it); rows [0, R) are compared."""
import sys
import os

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xuanpolicy_amd import fused_cnn  # noqa: E402
from xuanpolicy_amd.policies import BasicQnetwork, Basic_CNN  # noqa: E402

DEV = torch.device("cuda:0")
B, R = int(sys.argv[1]) if len(sys.argv) > 1 else 2048, 48
torch.manual_seed(0)


class Disc:
    n, shape = 18, ()


rep = Basic_CNN((84, 84, 4), [8, 4, 3], [4, 2, 1], [32, 64, 64], None, torch.nn.init.orthogonal_, torch.nn.ReLU, DEV)
pol = BasicQnetwork(Disc(), rep, [512], None, torch.nn.init.orthogonal_, torch.nn.ReLU, DEV)
fq = fused_cnn.FusedQNetwork(pol)
rng = np.random.default_rng(5)
x = rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)
xd = torch.as_tensor(x, device=DEV)
q, (tctx, s, outs) = fq.forward(xd)
hs = tctx[0]
torch.cuda.synchronize()
# f64 reference on rows [0, R)
xr = torch.as_tensor(x[:R].astype(np.float64) / 255.0).permute(0, 3, 1, 2)
convs = [m for m in rep.model if isinstance(m, torch.nn.Conv2d)]
h = xr
for i, c in enumerate(convs):
    h = F.relu(F.conv2d(h, c.weight.double().cpu(), c.bias.double().cpu(), c.stride, c.padding))
    got = hs[i + 1][:R].double().cpu().permute(0, 3, 1, 2)
    err = (got - h).abs()
    print("conv%d: max|err| %.3e  max|ref| %.3e  rel %.3e" % (i + 1, err.max(), h.abs().max(), err.max() / h.abs().max()))
    # f32 torch CPU on the same input (the reference's arithmetic class)
pooled = h.amax(dim=(2, 3))
print("pool: max|err| %.3e" % (s[:R].double().cpu() - pooled).abs().max())
lin = [m for m in pol.eval_Qhead.model if isinstance(m, torch.nn.Linear)]
z = F.relu(F.linear(pooled, lin[0].weight.double().cpu(), lin[0].bias.double().cpu()))
qq = F.linear(z, lin[1].weight.double().cpu(), lin[1].bias.double().cpu())
print("q: max|err| %.3e  max|q| %.3e" % ((q[:R].double().cpu() - qq).abs().max(), qq.abs().max()))
# the same convs through F.conv2d in f32 on the GPU, NCHW contiguous (library default layout)
h32 = torch.as_tensor(x, device=DEV).float().div(255.0).permute(0, 3, 1, 2).contiguous()
hr = xr
for i, c in enumerate(convs):
    h32 = F.relu(F.conv2d(h32, c.weight, c.bias, c.stride, c.padding))
    hr = F.relu(F.conv2d(hr, c.weight.double().cpu(), c.bias.double().cpu(), c.stride, c.padding))
    print("NCHW f32 conv%d: max|err| %.3e" % (i + 1, (h32[:R].double().cpu() - hr).abs().max()))
