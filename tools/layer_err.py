"""Debug tool (GPU): where does the GPU forward's fp32 error come from, layer by layer?

Runs the train-mode forward of a golden fixture's Segment on the MI355X, reads every
activation buffer of the plan's arena, and compares each against the fp64 oracle's value of
the same tensor, next to the CPU-fp32 oracle's (the reference arithmetic's) distance to
fp64. Raw conv outputs (before their BatchNorm) are compared per channel in units of that
channel's fp64 standard deviation (what BatchNorm turns an error into); block outputs
(materialised residual tails) in units of the tensor's max |value|. The ratio column is
GPU error / CPU-fp32 error: a layer where it jumps is where the GPU loses accuracy the
reference keeps.

    python tools/layer_err.py [fixture.npz] [--adam1]

--adam1: the parameters after one CPU torch.optim.Adam step on the fixture's fp64
gradients (the deterministic step-2 parameters of tests/test_gpu_trainer.py).
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from instancesegmentation_amd.engine import Plan  # noqa: E402
from instancesegmentation_amd.model.segment import Segment  # noqa: E402
from instancesegmentation_amd.runtime import Runner, module_tensors  # noqa: E402
from oracle import segment_oracle as O  # noqa: E402
from tests.golden_util import SegmentFixture  # noqa: E402


def oracle_record(params, x, dtype):
    """fp32/fp64 oracle forward (train mode); returns (logits, {name: tensor}) with every
    BatchNorm input (raw conv output) and every block output, keyed like the plan's
    arena buffers."""
    rec = {}
    saved = {}

    def wrap_bn(f):
        def g(c, pre, y):
            k = pre[:-3] if pre.endswith(".bn") else pre
            rec[k] = y.detach().clone()
            return f(c, pre, y)
        return g

    def wrap_block(f):
        def g(c, pre, *a, **kw):
            out = f(c, pre, *a, **kw)
            rec[pre] = (out[0] if isinstance(out, tuple) else out).detach().clone()
            return out
        return g

    names = ["bottleneck3x3", "bottleneck5x5", "bottleneck_down2", "bottleneck_dim_res",
             "bottleneck_dim_relu", "bottleneck_up_res"]
    saved["_bn"] = O._bn
    O._bn = wrap_bn(O._bn)
    for n in names:
        saved[n] = getattr(O, n)
        setattr(O, n, wrap_block(getattr(O, n)))
    try:
        logits, _ = O.forward(params, x, train=True, dtype=dtype)
    finally:
        for n, f in saved.items():
            setattr(O, n, f)
    return logits, rec


def gpu_forward(params, fx):
    """(logits, act arena, plan) of the train-mode forward on the MI355X."""
    dev = torch.device("cuda", 0)
    m = Segment(fx.cin)
    sd = m.state_dict()
    m.load_state_dict({k: torch.as_tensor(v).to(sd[k].dtype) for k, v in params.items()})
    m = m.to(dev).train()
    xt = torch.from_numpy(fx.x).to(dev)
    xs = [xt[:, :3].contiguous(), xt[:, 3:].contiguous()] if fx.cin == 20 else [xt]
    plan = Plan(m, [tuple(t.shape) for t in xs], True, False, tuple(False for _ in xs))
    run = Runner(m, plan)
    with torch.no_grad():
        outs, (act, _, _, _, _) = run.forward(xs, module_tensors(m))
    torch.cuda.synchronize()
    return outs[0].double().cpu(), act.double().cpu(), plan


def seed_sweep(fx, n):
    from oracle.seeding import synth_params
    rows = []
    for seed in range(1000, 1000 + n):
        params = synth_params(fx.shapes, seed, fx.meta.get("head_scale", 1.0))
        got, _, _ = gpu_forward(params, fx)
        l64, _ = O.forward(params, fx.x, train=True, dtype=torch.float64)
        l32, _ = O.forward(params, fx.x, train=True, dtype=torch.float32)
        e_g = (got - l64).abs().max().item()
        e_c = (l32.double() - l64).abs().max().item()
        rows.append(e_g / e_c)
        print(f"seed {seed}: GPU {e_g:.3e} CPU-fp32 {e_c:.3e} ratio {e_g / e_c:.2f} "
              f"|logit|max {l64.abs().max().item():.2f}", flush=True)
    r = sorted(rows)
    print(f"ratio GPU/CPU-fp32 over {n} seeds: median {r[n // 2]:.2f} min {r[0]:.2f} "
          f"max {r[-1]:.2f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fixture", nargs="?", default="segment20_n2_128.npz")
    ap.add_argument("--adam1", action="store_true")
    ap.add_argument("--seeds", type=int, default=0,
                    help="logits only: GPU / CPU-fp32 error ratio over this many parameter seeds")
    a = ap.parse_args()
    fx = SegmentFixture(a.fixture)
    if a.seeds:
        return seed_sweep(fx, a.seeds)
    params = {k: np.array(v, copy=True) for k, v in fx.params.items()}
    if a.adam1:
        m = Segment(fx.cin)
        sd = m.state_dict()
        m.load_state_dict({k: torch.as_tensor(v).to(sd[k].dtype) for k, v in params.items()})
        opt = torch.optim.Adam(m.parameters())
        for k, p in m.named_parameters():
            p.grad = None if k in fx.grad_none else torch.from_numpy(fx.grad(k).copy()).float()
        opt.step()
        params = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
    got, act, plan = gpu_forward(params, fx)
    l64, r64 = oracle_record(params, fx.x, torch.float64)
    l32, r32 = oracle_record(params, fx.x, torch.float32)
    e_g = (got - l64).abs().max().item()
    e_c = (l32.double() - l64).abs().max().item()
    print(f"{a.fixture}{' adam1' if a.adam1 else ''}: logits err vs fp64 GPU {e_g:.3e} "
          f"CPU-fp32 {e_c:.3e} ratio {e_g / e_c:.2f}; |logit|max {l64.abs().max().item():.2f}")
    print(f"{'buffer':34s} {'kind':5s} {'GPU err':>10s} {'CPU32 err':>10s} {'ratio':>6s}")
    for b in plan.graph.act_bufs:
        k = b.name
        if k.endswith(".convT"):  # the ConvTranspose2d feeding BatchNorm convs.2 (:305-307)
            k = k[:-len(".convT")] + ".convs.2"
        if k not in r64:
            continue
        ref = r64[k]
        if tuple(ref.shape) != (b.N, b.C, b.H, b.W):
            print(f"{k:34s} shape {tuple(ref.shape)} vs {(b.N, b.C, b.H, b.W)}: skipped")
            continue
        g = act[b.off:b.off + b.numel].view(b.N, b.C, b.H, b.W)
        c = r32[k].double()
        raw = any(t in k for t in ("convs.", "resconv", "convm", "conv2.", "layer", "convT"))
        if raw:  # per-channel, in units of the channel's std
            sd_c = ref.std(dim=(0, 2, 3)).clamp_min(1e-30).view(1, -1, 1, 1)
            eg = ((g - ref).abs() / sd_c).max().item()
            ec = ((c - ref).abs() / sd_c).max().item()
            kind = "raw"
        else:
            sc = ref.abs().max().item()
            eg = (g - ref).abs().max().item() / sc
            ec = (c - ref).abs().max().item() / sc
            kind = "block"
        print(f"{k:34s} {kind:5s} {eg:10.3e} {ec:10.3e} {eg / max(ec, 1e-30):6.2f}")


if __name__ == "__main__":
    main()
