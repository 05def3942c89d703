"""Time the keypoint-stem ops alone at the bench configuration (ablation helper)."""
import sys
import torch
from instancesegmentation_amd import _lib as L
from instancesegmentation_amd.data import device_batch
from instancesegmentation_amd.model.segment import Segment
from instancesegmentation_amd.train import Trainer

dev = torch.device("cuda", 0)
torch.manual_seed(1234)
xs, mask = device_batch(2, 1024, 1024, dev, seed=100, keypoints=True)
tr = Trainer(Segment(20), 2, [tuple(x.shape) for x in xs], device=dev)
tr.step(xs, mask)
torch.cuda.synchronize()
for phase, ol in (("fwd", tr.plan.fwd), ("bwd", tr.plan.bwd)):
    for i, r in enumerate(ol.recs):
        if r.kind not in (L.OP_KP_STEM_FWD, L.OP_KP_STEM_WGRAD, L.OP_KP_POOL) and \
                r.label not in ("init_conv.layer1", "dw_init_conv.layer1"):
            continue
        sub = ol.slice(i, i + 1)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                sub.run(tr.table, L.stream_ptr(), None)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        print(f"{sys.argv[1] if len(sys.argv) > 1 else ''} {r.label:28s} {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us", flush=True)
