"""Debug tool: run the same golden train step several times (fresh arenas each time) and
report, per arena buffer in production order, how far the runs disagree. fp32 atomics
make runs differ at ~1e-6 relative; a buffer far above that names the first op whose
result depends on timing (a race).

  python tools/race_hunt.py [fixture] [runs]
"""
import sys

import torch

sys.path.insert(0, ".")
from instancesegmentation_amd import runtime  # noqa: E402
from tests.golden_util import SegmentFixture  # noqa: E402
from tests.test_gpu_segment import load_model, run_step  # noqa: E402

arenas = []
_orig = runtime._arena


def _rec(n, dtype, dev):
    t = torch.zeros(n, dtype=dtype, device=dev)
    arenas.append(t)
    return t


runtime._arena = _rec


def one(fx):
    arenas.clear()
    m = load_model(fx)
    run_step(m, fx)
    torch.cuda.synchronize()
    plan = next(iter(m._plans.values())).plan
    grads = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    return plan, [a.detach().clone() for a in arenas], grads


def main():
    fx = SegmentFixture(sys.argv[1] if len(sys.argv) > 1 else "segment3_n2_64x96.npz")
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    plan, a0, g0 = one(fx)
    bufs = {0: ("act", plan.graph.act_bufs), 2: ("grad", plan.grad_bufs)}
    worst = {}
    for r in range(1, runs):
        _, a, g = one(fx)
        for ai, (nm, bl) in bufs.items():
            for b in bl:
                if b.numel == 0:
                    continue
                x = a0[ai][b.off:b.off + b.numel]
                y = a[ai][b.off:b.off + b.numel]
                rel = (x - y).abs().max().item() / max(x.abs().max().item(), 1e-12)
                key = (ai, b.off, nm + ":" + b.name)
                worst[key] = max(worst.get(key, 0.0), rel)
        for k in g0:
            rel = (g0[k] - g[k]).abs().max().item() / max(g0[k].abs().max().item(), 1e-12)
            worst[(9, 0, "pgrad:" + k)] = max(worst.get((9, 0, "pgrad:" + k), 0.0), rel)
    print("buffers (arena, offset order = production order) and run-to-run rel diff:")
    for key in sorted(worst):
        flag = " <<<" if worst[key] > 1e-4 else ""
        print(f"  {key[2]:50s} off {key[1]:10d} {worst[key]:.3e}{flag}")
    print("max over all:", max(worst.values()))


if __name__ == "__main__":
    main()
