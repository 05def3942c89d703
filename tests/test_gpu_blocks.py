"""Block-level parity: every reference building block run standalone through the engine
(forward + backward, input gradient and every parameter gradient) against the oracle's
fp64 restatement of the same block. Odd plane sizes exercise partial tiles."""
import numpy as np
import pytest
import torch

from instancesegmentation_amd.model import segment as S
from oracle import segment_oracle as O
from oracle.seeding import synth_params

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (factory, oracle fn, input channels, extra oracle args, returns tuple)
BLOCKS = {
    "b3x3": (lambda: S.Bottleneck3x3(48, 16), lambda c, x: O.bottleneck3x3(c, "blk", x, 16), 48),
    "b3x3_d4": (lambda: S.Bottleneck3x3(48, 16, pad=4, dilation=4),
                lambda c, x: O.bottleneck3x3(c, "blk", x, 16, pad=4, dil=4), 48),
    "b5x5": (lambda: S.Bottleneck5x5(48, 16), lambda c, x: O.bottleneck5x5(c, "blk", x, 16), 48),
    "down2": (lambda: S.BottleneckDown2(36, 16, 48),
              lambda c, x: O.bottleneck_down2(c, "blk", x, 16), 36),
    "dimres_prelu": (lambda: S.BottleneckDim_Res(96, 16, 48, True),
                     lambda c, x: O.bottleneck_dim_res(c, "blk", x, 16, True), 96),
    "dimres_relu": (lambda: S.BottleneckDim_Res(96, 16, 48, False),
                    lambda c, x: O.bottleneck_dim_res(c, "blk", x, 16, False), 96),
    "dim_relu": (lambda: S.BottleneckDim(48, 16, 48, False),
                 lambda c, x: O.bottleneck_dim_relu(c, "blk", x), 48),
    "conv_prelu": (lambda: S.Conv(16, 16, k=5, s=2, p=2, act=torch.nn.PReLU(16)),
                   lambda c, x: O.conv(c, "blk", x, k=5, s=2, p=2, act="prelu"), 16),
    # A8 (segment.py:296-344): two inputs, x and the pooled skip features of the same
    # resolution; output at twice the resolution
    "up_res": (lambda: S.BottleneckUp_Res(128, 16, 48),
               lambda c, x, s: O.bottleneck_up_res(c, "blk", x, s), 128, 48),
    "up_res_other": (lambda: S.BottleneckUp_Res_Other(48, 4, 16, 36),
                     lambda c, x, s: O.bottleneck_up_res(c, "blk", x, s), 48, 36),
}
SIZES = [(16, 24), (32, 32), (12, 20)]


def run_block(name, hw, seed=0, stacked=False):
    make, ofn, cin = BLOCKS[name][:3]
    cskip = BLOCKS[name][3] if len(BLOCKS[name]) > 3 else 0
    torch.manual_seed(seed)
    blk = make()
    shapes = [(k, tuple(v.shape)) for k, v in blk.state_dict().items()]
    pv = synth_params([("blk." + k, s) for k, s in shapes], 11 + seed)
    sd = blk.state_dict()
    blk.load_state_dict({k: torch.as_tensor(pv["blk." + k]).to(sd[k].dtype) for k in sd})
    blk = blk.to(DEV).train()
    if stacked:  # the Trainer's flat layout: sibling 1x1 convs run as one stacked GEMM
        from instancesegmentation_amd.engine import param_layout
        from instancesegmentation_amd.train import flatten_module
        flatten_module(blk, DEV, order=param_layout(blk))
    H, W = hw
    rng = np.random.Generator(np.random.PCG64(seed))
    x = rng.normal(0, 1, (2, cin, H, W)).astype(np.float32)
    xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
    ins = [xt]
    if cskip:
        sk = rng.normal(0, 1, (2, cskip, H, W)).astype(np.float32)
        ins.append(torch.from_numpy(sk).to(DEV).requires_grad_(True))
    out = blk(*ins)
    outs = out if isinstance(out, tuple) else (out,)
    douts = [torch.from_numpy(rng.normal(0, 1, tuple(o.shape)).astype(np.float32)).to(DEV)
             for o in outs]
    torch.autograd.backward(outs, douts)
    # oracle
    P = {k: torch.as_tensor(v).double() if np.issubdtype(np.asarray(v).dtype, np.floating)
         else torch.as_tensor(v) for k, v in pv.items()}
    for k, v in P.items():
        if v.is_floating_point() and not k.endswith(("running_mean", "running_var")):
            v.requires_grad_(True)
    xr = torch.from_numpy(x).double().requires_grad_(True)
    rins = [xr]
    if cskip:
        rins.append(torch.from_numpy(sk).double().requires_grad_(True))
    ro = ofn(O.Ctx(P, True), *rins)
    ros = ro if isinstance(ro, tuple) else (ro,)
    torch.autograd.backward(ros, [d.double().cpu() for d in douts])
    return blk, outs, ins, ros, rins, P


def err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-6)


STACKED = ["dimres_prelu", "dimres_relu", "up_res", "up_res_other"]  # blocks with siblings()


@pytest.mark.parametrize("hw", SIZES)
@pytest.mark.parametrize("name", list(BLOCKS) + [n + ":stacked" for n in STACKED])
def test_block_parity(name, hw):
    stacked = name.endswith(":stacked")
    name = name.split(":")[0]
    blk, outs, ins, ros, rins, P = run_block(name, hw, stacked=stacked)
    if stacked:
        from instancesegmentation_amd.engine import ConvPairOp
        plan = next(iter(blk._plans.values())).plan
        assert sum(isinstance(op, ConvPairOp) for op in plan.graph.ops) == 1
    for o, r in zip(outs, ros):
        assert err(o, r) < 1e-5, f"output {err(o, r):.2e}"
    for i, (xt, xr) in enumerate(zip(ins, rins)):  # input (and skip) gradients
        assert err(xt.grad, xr.grad) < 1e-4, f"input {i} grad {err(xt.grad, xr.grad):.2e}"
    bad = []
    for k, p in blk.named_parameters():
        ref = P["blk." + k].grad
        if ref is None:
            assert p.grad is None, k
            continue
        if k.endswith(".conv.bias") or k.endswith("convs.1.bias") and "up" in name:
            continue  # conv bias ahead of train-mode BN: gradient is rounding noise
        e = err(p.grad, ref)
        if e > 1e-4:
            bad.append((round(e, 6), k))
    assert not bad, sorted(bad, reverse=True)[:6]
