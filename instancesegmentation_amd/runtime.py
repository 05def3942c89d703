"""Module runtime: `EngineModule.forward` builds (once per input shape / mode) a Plan
with `emit`, then runs it through libisg's executor; autograd is one Function per
module call whose backward replays the recorded backward op list.

This keeps the reference's nn.Module calling convention (forward, train/eval,
parameters(), state_dict) while all arithmetic runs in the HIP kernels.
"""
import ctypes
import os

import torch
import torch.nn as nn

from . import _lib as L
from .engine import (S_ACT, S_DIN, S_DOUT, S_GRAD, S_IN, S_OUT, S_PGRAD, S_STATS, S_TENSOR0,
                     S_WREP, Plan, param_layout)


# ISG_DEBUG_POISON=1: fill every arena with NaN before use so a read of memory that no
# op wrote (a missing STORE before an ACCUM, an uncovered halo) surfaces as NaN.
_POISON = os.environ.get("ISG_DEBUG_POISON", "0") == "1"


def _arena(n, dtype, dev):
    if _POISON:
        return torch.full((n,), float("nan"), dtype=dtype, device=dev)
    return torch.empty(n, dtype=dtype, device=dev)


class EngineModule(nn.Module):
    """Base class of every drop-in module. Subclasses implement `emit(g, *inputs)`."""

    def __init__(self):
        super().__init__()
        object.__setattr__(self, "_plans", {})

    def forward(self, *xs):
        return run_module(self, xs)

    def _apply(self, fn, *args, **kwargs):  # .to()/.cuda()/.double() invalidate recorded plans
        self._plans.clear()
        return super()._apply(fn, *args, **kwargs)

    def clear_plans(self):
        self._plans.clear()


def _check_inputs(xs):
    out = []
    for x in xs:
        if not isinstance(x, torch.Tensor):
            raise TypeError(f"expected a Tensor input, got {type(x).__name__}")
        if x.dim() == 3 and out:
            # keypoints [N, parts, 3] = (x, y, visible) standing for the heatmap channels
            # (engine.Keypoints): float64, as the reference's keypoint2heatmaps computes
            if x.shape[2] != 3 or x.dtype != torch.float64:
                raise RuntimeError("keypoints: expected a float64 [N, parts, 3] tensor, got "
                                   f"{x.dtype} {tuple(x.shape)}")
            if x.device.type != "cuda":
                raise RuntimeError("instancesegmentation_amd runs on the MI355X only: move the "
                                   "model and inputs to a GPU device (there is no CPU path)")
            out.append(x.contiguous())
            continue
        if x.dim() != 4:
            raise RuntimeError(f"expected a 4-D NCHW input, got shape {tuple(x.shape)}")
        if x.device.type != "cuda":
            raise RuntimeError("instancesegmentation_amd runs on the MI355X only: move the model "
                               "and inputs to a GPU device (there is no CPU path)")
        if x.dtype != torch.float32:
            raise RuntimeError(f"expected float32 input, got {x.dtype}")
        out.append(x.contiguous())
    if len({x.shape[0] for x in out}) != 1:
        raise RuntimeError("inputs disagree on batch size")
    return out


def module_tensors(mod):
    return [p for _, p in mod.named_parameters()] + [b for _, b in mod.named_buffers()]


class Runner:
    """Executes one Plan: allocates arenas, fills the pointer table, calls isg_exec."""

    def __init__(self, mod, plan):
        self.mod = mod
        self.plan = plan
        self.ntab = S_TENSOR0 + len(plan.graph.tensor_names)

    def table(self):
        return (ctypes.c_void_p * self.ntab)()

    def forward(self, xs, tensors):
        p = self.plan
        dev = xs[0].device
        for t in tensors:
            if t.device != dev or (t.is_floating_point() and t.dtype != torch.float32):
                raise RuntimeError("module parameters/buffers must be float32 on the input's "
                                   "device (call .to(device))")
        act = _arena(max(p.act_size, 1), torch.float32, dev)
        stats = _arena(p.stats_size, torch.float64, dev)
        # the weight-gradient replicas: zeroed by the forward's side-stream memset (Plan), so
        # they belong to this forward's saved state
        wrep = _arena(L.WREP * max(p.graph.pgrad_size, 1), torch.float64, dev) \
            if p.bwd is not None else None
        outs = [torch.empty(s, dtype=torch.float32, device=dev) for s in p.out_shapes]
        tab = self.table()
        tab[S_ACT] = act.data_ptr()
        tab[S_STATS] = stats.data_ptr()
        if wrep is not None:
            tab[S_WREP] = wrep.data_ptr()
        for i, x in enumerate(xs):
            tab[S_IN[i]] = x.data_ptr()
        for i, o in enumerate(outs):
            tab[S_OUT[i]] = o.data_ptr()
        for j, t in enumerate(tensors):
            tab[S_TENSOR0 + j] = t.data_ptr()
        with torch.cuda.device(dev):
            p.fwd.run(tab, L.stream_ptr(dev))
        return outs, (act, stats, xs, tensors, wrep)

    def backward(self, saved, douts, in_grad):
        p = self.plan
        act, stats, xs, tensors, wrep = saved
        dev = act.device
        grad = _arena(max(p.grad_size, 1), torch.float32, dev)
        pgrad = _arena(max(p.graph.pgrad_size, 1), torch.float32, dev)
        dins = []
        for i, x in enumerate(xs):
            if in_grad[i]:
                dins.append(torch.empty_like(x) if p.din_written[i] else torch.zeros_like(x))
            else:
                dins.append(None)
        tab = self.table()
        tab[S_ACT] = act.data_ptr()
        tab[S_STATS] = stats.data_ptr()
        tab[S_GRAD] = grad.data_ptr()
        tab[S_PGRAD] = pgrad.data_ptr()
        tab[S_WREP] = wrep.data_ptr()
        for i, x in enumerate(xs):
            tab[S_IN[i]] = x.data_ptr()
            if dins[i] is not None:
                tab[S_DIN[i]] = dins[i].data_ptr()
        for i, d in enumerate(douts):
            tab[S_DOUT[i]] = d.data_ptr()
        for j, t in enumerate(tensors):
            tab[S_TENSOR0 + j] = t.data_ptr()
        with torch.cuda.device(dev):
            p.bwd.run(tab, L.stream_ptr(dev), L.side_stream_ptr(dev))
        g = p.graph
        pgrads = []
        for k in g.params:  # autograd wants them in parameter order (not the layout's)
            if k in p.used_params:
                off = g.pgrad_off[k]
                n = 1
                for s in g.param_shapes[k]:
                    n *= s
                pgrads.append(pgrad[off:off + n].view(g.param_shapes[k]))
            else:
                pgrads.append(None)
        return dins, pgrads


class _PlanFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, runner, nin, in_grad, *args):
        xs = list(args[:nin])
        params = args[nin:]
        tensors = list(params) + [b for _, b in runner.mod.named_buffers()]
        outs, saved = runner.forward(xs, tensors)
        ctx.runner = runner
        ctx.saved = saved
        ctx.nin = nin
        ctx.in_grad = in_grad
        return tuple(outs) if len(outs) > 1 else outs[0]

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, *douts):
        douts = [d.contiguous() if d is not None else None for d in douts]
        for i, d in enumerate(douts):
            if d is None:
                douts[i] = torch.zeros(ctx.runner.plan.out_shapes[i], dtype=torch.float32,
                                       device=ctx.saved[0].device)
        dins, pgrads = ctx.runner.backward(ctx.saved, douts, ctx.in_grad)
        ctx.saved = None
        return (None, None, None, *dins, *pgrads)


def run_module(mod, xs):
    xs = _check_inputs(list(xs))
    train = mod.training
    params = [p for _, p in mod.named_parameters()]
    grad_on = torch.is_grad_enabled()
    need_grad = grad_on and any(p.requires_grad for p in params)
    in_grad = tuple(bool(grad_on and x.requires_grad) for x in xs)
    key = (tuple(tuple(x.shape) for x in xs), train, need_grad or any(in_grad), in_grad)
    runner = mod._plans.get(key)
    if runner is not None and not runner.plan.stacking_holds(module_tensors(mod)):
        runner = None  # a stacked pair's weights were rebound apart: plan again (two convs)
    if runner is None:
        # sibling 1x1 convs run stacked where their weights are adjacent in memory
        # (train.flatten_module with engine.param_layout); separate tensors: two convs
        plan = Plan(mod, [tuple(x.shape) for x in xs], train, need_grad or any(in_grad), in_grad,
                    layout=param_layout(mod))
        runner = Runner(mod, plan)
        mod._plans[key] = runner
    if need_grad or any(in_grad):
        return _PlanFunction.apply(runner, len(xs), in_grad, *xs, *params)
    outs, _ = runner.forward(xs, module_tensors(mod))
    return tuple(outs) if len(outs) > 1 else outs[0]


# ---- sigmoid (segment.py:534) ---------------------------------------------------------
class _Sigmoid(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        L.check(L.lib().isg_sigmoid_fwd(x.data_ptr(), y.data_ptr(), x.numel(),
                                        L.stream_ptr(x.device)), "sigmoid")
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(y)
        L.check(L.lib().isg_sigmoid_bwd(y.data_ptr(), dy.data_ptr(), dx.data_ptr(), y.numel(),
                                        L.stream_ptr(y.device)), "sigmoid_bwd")
        return dx


def sigmoid(x):
    if x.device.type != "cuda" or x.dtype != torch.float32:
        raise RuntimeError("sigmoid: float32 GPU tensor expected")
    return _Sigmoid.apply(x)
