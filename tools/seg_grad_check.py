"""Debug aid (GPU): per-tensor relative L2 / max-abs gradient error of one Segment train
step against a golden fixture, worst first. Env toggles (ISG_NO_TAP_CONV, ...) select
kernel paths.  python tools/seg_grad_check.py [fixture]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests.golden_util import SEGMENT_FIXTURES, SegmentFixture  # noqa: E402
from tests.test_gpu_segment import dead_bias, load_model, run_step  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else SEGMENT_FIXTURES[0]
    fx = SegmentFixture(name)
    m = load_model(fx)
    logits, loss = run_step(m, fx)
    ref = torch.from_numpy(fx.z["logits64"])
    print(f"{name} logits err {(logits.cpu() - ref).abs().max().item():.2e}")
    rows = []
    for k, p in m.named_parameters():
        if k in fx.grad_none or dead_bias(k):
            continue
        r = torch.from_numpy(fx.grad(k).copy()).double()
        g = p.grad.detach().double().cpu()
        l2 = ((g - r).norm() / max(r.norm().item(), 1e-12)).item()
        rows.append((l2, (g - r).abs().max().item() / max(r.abs().max().item(), 1e-12), k))
    rows.sort(reverse=True)
    for l2, mx, k in rows[:12]:
        print(f"  l2 {l2:.2e}  maxrel {mx:.2e}  {k}")
    # forward statistics: BN running buffers after the step vs the fp64 reference
    sd = m.state_dict()
    worst = []
    for k, v in fx.buffers64().items():
        if k.endswith("num_batches_tracked"):
            continue
        got = sd[k].double().cpu().numpy()
        worst.append((float(abs(got - v).max() / max(abs(v).max(), 1e-12)), k))
    worst.sort(reverse=True)
    print("  running-stat worst rel err:", [f"{e:.1e} {k}" for e, k in worst[:3]])


if __name__ == "__main__":
    main()
