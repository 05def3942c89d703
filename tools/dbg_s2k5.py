import sys, torch
sys.path.insert(0, '.')
import tests.test_gpu_kernels as T
from tests.isg_helpers import *
import torch.nn.functional as F
from instancesegmentation_amd import _lib as L
Ci, Co, H, W = 16, 16, 512, 512
N = 2
ge, OH, OW = T._geom(N, Ci, Co, H, W, 5, 2, 2, 1)
x = T.rnd(N, Ci, H, W, seed=11) * 0.7 + 0.2
w = T.rnd(Co, Ci, 5, 5, seed=12, scale=(2.0 / (Ci * 25)) ** 0.5)
b = T.rnd(Co, seed=13, scale=0.1)
ref = F.conv2d(x, w, b, stride=2, padding=2)
X = T.cuda32(x)
segs = [{"p": ptr(X), "n_stride": Ci * H * W, "C": Ci, "xform": L.XF_PLAIN}]
Y = torch.full((N, Co, OH, OW), float("nan"), device="cuda")
stats = rep_zeros(4 * Co)
B, Wt = T.cuda32(b), T.cuda32(w)
sk = sinks([{"p": ptr(Y), "n_stride": Co * OH * OW, "c0": 0, "C": Co, "mode": L.SINK_STORE, "bias": ptr(B), "stats": ptr(stats)}])
call("isg_conv_fwd", geom(**ge), vt(segs, N, H, W), ptr(Wt), sk, stream())
torch.cuda.synchronize()
e = (Y.double().cpu() - ref).abs()
print("max err", e.max().item(), "nan", torch.isnan(Y).sum().item())
bad = (e > 1e-3)
print("bad count", bad.sum().item(), "of", e.numel())
idx = bad.nonzero()
if len(idx):
    print("channels", torch.unique(idx[:, 1]).tolist())
    print("rows mod 4", torch.bincount(idx[:, 2] % 4).tolist(), "cols mod 32", torch.bincount(idx[:, 3] % 32, minlength=32).tolist())
    print("first", idx[:10].tolist())
