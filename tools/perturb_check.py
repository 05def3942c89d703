"""How chaotic is a full-size gradient check? (CPU diagnostic, no GPU.)

    python tools/perturb_check.py [--h 800] [--w 1344] [--n 2] [--keys k1,k2]

Runs the fp64 oracle train step, the plain fp32 one, and an fp32 one whose stem layer-2
convolution is evaluated in fp64 and rounded once to fp32 (the same conv, a different
rounding: what any other summation order of that one layer — e.g. a GPU kernel's — does).
Prints each gradient tensor's err/scale against fp64 for both fp32 runs: when the
perturbed run's error on a tensor is several times the plain run's, that tensor's
full-size bar (tests/grad_check.py, 4x the fp32 reference's own error) measures rounding
amplification, not kernel correctness.
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import segment_oracle as SO  # noqa: E402
from instancesegmentation_amd.data import device_batch  # noqa: E402
from instancesegmentation_amd.model.segment import Segment  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--h", type=int, default=800)
    ap.add_argument("--w", type=int, default=1344)
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--keys", default="bottle2_x.2.convs.2.conv.weight,bottle2_x.2.convs.2.bn.bias,"
                    "bottle2_x.3.convs.2.bn.bias,bottle2_x.3.convs.2.bn.weight")
    a = ap.parse_args()
    torch.manual_seed(1234)
    model = Segment(20)
    params = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    xs, mask = device_batch(a.n, a.h, a.w, "cpu", seed=100, cin=20)
    x = torch.cat(xs, 1).numpy()
    y = mask.numpy()
    _, _, g64, _ = SO.train_step(dict(params), x, y, torch.float64)
    _, _, g32, _ = SO.train_step(dict(params), x, y, torch.float32)
    orig = SO.conv

    def conv64(c, pre, xx, k=1, s=1, p=None, g=1, d=1, act=None):
        if pre != "init_conv.layer2":
            return orig(c, pre, xx, k, s, p, g, d, act)
        yy = F.conv2d(xx.double(), c.P[pre + ".conv.weight"].double(),
                      c.P[pre + ".conv.bias"].double(), stride=s, padding=p).float()
        yy = SO._bn(c, pre + ".bn", yy)
        return SO._act(c, pre + ".act", act, yy)

    SO.conv = conv64
    try:
        _, _, gp, _ = SO.train_step(dict(params), x, y, torch.float32)
    finally:
        SO.conv = orig
    rows = []
    for k, r in g64.items():
        if r is None:
            continue
        r = r.double()
        sc = max(r.abs().max().item(), 1e-30)
        e32 = (g32[k].double() - r).abs().max().item() / sc
        ep = (gp[k].double() - r).abs().max().item() / sc
        rows.append((ep / max(e32, 1e-30), k, e32, ep))
    rows.sort(reverse=True)
    print(f"{a.n}x{a.h}x{a.w}: err/scale vs fp64 — plain fp32, fp32 with layer2 rounded differently")
    for ratio, k, e32, ep in rows[:12]:
        print(f"  {k:45s} {e32:.2e} {ep:.2e}  x{ratio:.2f}")
    for k in a.keys.split(","):
        for ratio, kk, e32, ep in rows:
            if kk == k:
                print(f"  [{k}] {e32:.2e} -> {ep:.2e} (x{ratio:.2f})")


if __name__ == "__main__":
    main()
