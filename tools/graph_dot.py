"""Dump the captured train step's HIP graph as Graphviz dot (hipGraphDebugDotPrint via
torch's CUDAGraph debug mode) to inspect its dependency edges.

    python tools/graph_dot.py gpurun_out/step.dot
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from instancesegmentation_amd.data import device_batch  # noqa: E402
from instancesegmentation_amd.model.segment import Segment  # noqa: E402
from instancesegmentation_amd.train import Trainer  # noqa: E402

_G = torch.cuda.CUDAGraph


class _DebugGraph(_G):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.enable_debug_mode()


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/step.dot"
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    xs, mask = device_batch(2, 1024, 1024, dev, seed=100, cin=20, keypoints=True)
    tr = Trainer(Segment(20), 2, [tuple(x.shape) for x in xs], device=dev)
    tr.step(xs, mask)
    torch.cuda.CUDAGraph = _DebugGraph
    tr.capture()
    torch.cuda.CUDAGraph = _G
    graphs = [g for g in tr.graphs if isinstance(g, _G)]
    for i, g in enumerate(graphs):
        g.debug_dump(out if len(graphs) == 1 else f"{out}.{i}")
    print("graphs", len(graphs), "->", out)


if __name__ == "__main__":
    main()
