"""Host enqueue time of the train step against its GPU time: if issuing a step takes
about as long on the host as the step takes on the GPU, the launch is host-paced.

    python tools/replay_host.py [--steps 20] [--eager]

Default: HIP-graph replay of the captured step. --eager: the step issued by the C++
executor (isg_exec_ms2: one host call per op list, one hipLaunchKernel per record) with no
graph — the other host floor.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from instancesegmentation_amd.data import device_batch  # noqa: E402
from instancesegmentation_amd.model.segment import Segment  # noqa: E402
from instancesegmentation_amd.train import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--eager", action="store_true", help="no graph: the C++ executor per step")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    model = Segment(20)
    xs, mask = device_batch(2, 1024, 1024, dev, seed=100, cin=20, keypoints=True)
    tr = Trainer(model, 2, [tuple(x.shape) for x in xs], device=dev)
    tr.step(xs, mask)
    if not a.eager:
        tr.capture()
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    # host time of the replay calls alone (the GPU runs behind them)
    host = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        h0 = time.perf_counter()
        tr.step()
        host.append(time.perf_counter() - h0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host per step {1e3 * sum(host) / len(host):.3f} ms (max {1e3 * max(host):.3f}); "
          f"wall per step {1e3 * (t2 - t0) / a.steps:.3f} ms; GPU drain after the last "
          f"replay {1e3 * (t2 - t1):.3f} ms; mode {'eager executor' if a.eager else 'graph replay'}; "
          f"graphs {len(tr.graphs) if tr.graphs else 0}; records per step "
          f"{len(tr.plan.fwd.recs) + len(tr.plan.bwd.recs)}")
    # the host cost itself: steps issued into an IDLE GPU queue (right after a sync) cannot
    # be held back by queue back-pressure, unlike the pipelined loop above, whose host time
    # per step converges to the GPU's step time once the host runs ~4 steps ahead
    cold = []
    for _ in range(10):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        tr.step()
        cold.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    cold.sort()
    print(f"host cost of one step issued into an idle queue: median {1e3 * cold[5]:.3f} ms "
          f"(min {1e3 * cold[0]:.3f}, max {1e3 * cold[-1]:.3f})")
    # GPU idle test: one step after the GPU has gone idle, with the host far ahead
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    tr.step()
    ev1.record()
    torch.cuda.synchronize()
    print(f"single step GPU time {ev0.elapsed_time(ev1):.3f} ms")


if __name__ == "__main__":
    main()
