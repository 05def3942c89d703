"""Fused training step for the reference train loop (train_instance.py:371-382):

    optimizer.zero_grad(); out = model.train_batch(x, hm); loss = BCELoss(out, mask)
    loss.backward(); optimizer.step(); loss.item()

One `Trainer.step` runs, on one HIP stream and without torch autograd:
  forward op list -> fused sigmoid+BCE (loss + dlogits) -> backward op list ->
  [RCCL all-reduce(avg) of the flat 1.06 MB gradient bucket when world_size > 1] ->
  multi-tensor Adam over the flat parameter buffer.
Parameters, gradients and BN running statistics live in flat buffers (module tensors
are re-bound as views), so the optimizer is one kernel and the gradient exchange is one
collective. The whole step is capturable into a HIP graph (`capture()`).

Data parallelism: one process per GPU, image-batch sharded, local BN
statistics per replica, running stats broadcast from rank 0 each step (DDP's
broadcast_buffers default), gradient mean over ranks.
"""
import ctypes

import torch
import torch.distributed as dist

from . import _lib as L
from .engine import (S_ACT, S_DOUT, S_GRAD, S_IN, S_OUT, S_PGRAD, S_STATS, S_TENSOR0, S_WREP,
                     Plan)


class GradSync:
    """The data-parallel exchange of one step, one process per GPU:
    rank 0's BatchNorm running statistics are broadcast before the step (DDP
    broadcast_buffers), and the flat gradient bucket is averaged over the ranks after
    the backward (one collective: RCCL AVG on "nccl"; SUM then scale on gloo, which has no
    AVG). BN batch statistics stay local to each replica, as in the reference run per
    replica."""

    def __init__(self, process_group=None):
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.avg = self.world > 1 and dist.get_backend(process_group) == "nccl"

    def buffers(self, flatb):
        if self.world > 1:
            dist.broadcast(flatb, 0, group=self.pg)

    def grads(self, grad_flat):
        if self.world == 1:
            return
        if self.avg:
            dist.all_reduce(grad_flat, op=dist.ReduceOp.AVG, group=self.pg)
        else:
            dist.all_reduce(grad_flat, op=dist.ReduceOp.SUM, group=self.pg)
            grad_flat.div_(self.world)


def flatten_module(model, device):
    """Re-bind every parameter and floating buffer of `model` as a view of one flat
    buffer (params) / (float buffers); returns (flat_params, flat_bufs, param_index)."""
    params = [p for _, p in model.named_parameters()]
    n = sum(p.numel() for p in params)
    flat = torch.empty(n, dtype=torch.float32, device=device)
    index = []
    off = 0
    with torch.no_grad():
        for p in params:
            k = p.numel()
            flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = flat[off:off + k].view_as(p)
            index.append((off, k))
            off += k
    fbufs = [(m, name, b) for m in model.modules() for name, b in m._buffers.items()
             if b is not None and b.is_floating_point()]
    nb = sum(b.numel() for _, _, b in fbufs)
    flatb = torch.empty(max(nb, 1), dtype=torch.float32, device=device)
    off = 0
    with torch.no_grad():
        for m, name, b in fbufs:
            k = b.numel()
            flatb[off:off + k].copy_(b.reshape(-1))
            m._buffers[name] = flatb[off:off + k].view_as(b)
            off += k
    for m in model.modules():
        for name, b in m._buffers.items():
            if b is not None and not b.is_floating_point():
                m._buffers[name] = b.to(device)
    return flat, flatb, index


class Trainer:
    """train_instance.py:294-382 step body on the MI355X (Segment + BCELoss + Adam)."""

    def __init__(self, model, batch, in_shapes, device=None, lr=1e-3, betas=(0.9, 0.999),
                 eps=1e-8, weight_decay=0.0, process_group=None):
        self.device = torch.device(device or "cuda")
        self.model = model.to(self.device).train()
        self.flat, self.flatb, self.index = flatten_module(self.model, self.device)
        self.in_shapes = [tuple(s) for s in in_shapes]
        self.plan = Plan(self.model, self.in_shapes, True, True,
                         tuple(False for _ in self.in_shapes))
        g = self.plan.graph
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.pg = process_group
        self.sync = GradSync(process_group)
        self.world = self.sync.world
        dev = self.device
        self.act = torch.empty(max(self.plan.act_size, 1), dtype=torch.float32, device=dev)
        self.stats = torch.empty(self.plan.stats_size, dtype=torch.float64, device=dev)
        self.gradarena = torch.empty(max(self.plan.grad_size, 1), dtype=torch.float32, device=dev)
        # the plan's packed param-grad layout is exactly the flat buffer's order
        self.grad_flat = torch.zeros_like(self.flat)
        self.pgrad = self.grad_flat
        self.wrep = torch.empty(L.WREP * g.pgrad_size, dtype=torch.float32, device=dev)
        assert g.pgrad_size == self.flat.numel()
        self.logits = torch.empty(self.plan.out_shapes[0], dtype=torch.float32, device=dev)
        self.dlogits = torch.empty_like(self.logits)
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=dev)
        self._pg_views = []
        for (k, p), (off, n) in zip(self.model.named_parameters(), self.index):
            self._pg_views.append((g.pgrad_off[k], off, n, k in self.plan.used_params))
        live = torch.zeros(self.flat.numel(), dtype=torch.uint8)
        for _, off, n, used in self._pg_views:
            if used:
                live[off:off + n] = 1
        self.live = live.to(dev)
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.step_count = 0
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)  # Adam's step, on device
        self.inputs = [torch.empty(s, dtype=torch.float32, device=dev) for s in self.in_shapes]
        self.target = torch.empty(self.plan.out_shapes[0], dtype=torch.float32, device=dev)
        self.table = self._make_table()
        self.graphs = None
        self.events = []
        self.split = None

    def _make_table(self):
        g = self.plan.graph
        tab = (ctypes.c_void_p * (S_TENSOR0 + len(g.tensor_names)))()
        tab[S_ACT] = self.act.data_ptr()
        tab[S_STATS] = self.stats.data_ptr()
        tab[S_GRAD] = self.gradarena.data_ptr()
        tab[S_PGRAD] = self.pgrad.data_ptr()
        tab[S_WREP] = self.wrep.data_ptr()
        for i, x in enumerate(self.inputs):
            tab[S_IN[i]] = x.data_ptr()
        tab[S_OUT[0]] = self.logits.data_ptr()
        tab[S_DOUT[0]] = self.dlogits.data_ptr()
        tensors = [p for _, p in self.model.named_parameters()] + \
                  [b for _, b in self.model.named_buffers()]
        for j, t in enumerate(tensors):
            tab[S_TENSOR0 + j] = t.data_ptr()
        return tab

    # ---- the step body -------------------------------------------------------------
    def _fwd_bwd(self):
        """forward -> sigmoid+BCE (loss, dlogits) -> backward; HIP work only."""
        lib = L.lib()
        st = L.stream_ptr(self.device)
        self.plan.fwd.run(self.table, st)
        n = self.logits.numel()
        L.check(lib.isg_fill_f64(self.loss_acc.data_ptr(), 1, 0.0, st), "fill")
        L.check(lib.isg_bce_sigmoid(self.logits.data_ptr(), self.target.data_ptr(), n,
                                    self.loss_acc.data_ptr(), self.dlogits.data_ptr(),
                                    1.0 / n, st), "bce")
        self.plan.bwd.run(self.table, st, L.side_stream_ptr(self.device))

    def _adam(self):
        L.check(L.lib().isg_adam_dev(self.flat.data_ptr(), self.grad_flat.data_ptr(),
                                     self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                                     self.live.data_ptr(), self.flat.numel(),
                                     self.step_dev.data_ptr(), self.lr, self.betas[0],
                                     self.betas[1], self.eps, self.wd,
                                     L.stream_ptr(self.device)), "adam")

    def _loss(self):
        lib = L.lib()
        st = L.stream_ptr(self.device)
        n = self.logits.numel()
        L.check(lib.isg_fill_f64(self.loss_acc.data_ptr(), 1, 0.0, st), "fill")
        L.check(lib.isg_bce_sigmoid(self.logits.data_ptr(), self.target.data_ptr(), n,
                                    self.loss_acc.data_ptr(), self.dlogits.data_ptr(),
                                    1.0 / n, st), "bce")

    def _schedule(self, split=None):
        """The step as a list of units: callables issuing HIP work, or the markers
        'coll' (eager RCCL all-reduce), 'tic'/'toc' (timing events around one op).
        split=(phase, idx) isolates op `idx` of the forward/backward list."""
        def run_list(ol):
            return lambda: ol.run(self.table, L.stream_ptr(self.device), L.side_stream_ptr(self.device))
        units = []
        for phase, ol in (("fwd", self.plan.fwd), ("bwd", self.plan.bwd)):
            if split and split[0] == phase:
                i = split[1]
                if i > 0:
                    units.append(run_list(ol.slice(0, i)))
                units += ["tic", run_list(ol.slice(i, i + 1)), "toc"]
                if i + 1 < len(ol.recs):
                    units.append(run_list(ol.slice(i + 1, len(ol.recs))))
            else:
                units.append(run_list(ol))
            if phase == "fwd":
                units.append(self._loss)
        if self.world > 1:
            units.append("coll")
        units.append(self._adam)
        return units

    def capture(self, split=None):
        """Record the step into HIP graphs: every run of consecutive HIP units becomes one
        graph; markers between them stay eager (RCCL collectives, timing events)."""
        torch.cuda.synchronize(self.device)
        plan = []
        cur = []
        for u in self._schedule(split) + ["end"]:
            if callable(u):
                cur.append(u)
                continue
            if cur:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for f in cur:
                        f()
                plan.append(g)
                cur = []
            if u != "end":
                plan.append(u)
        self.graphs = plan
        self.events = []
        return self

    def _run(self, units):
        ev = None
        for u in units:
            if isinstance(u, torch.cuda.CUDAGraph):
                u.replay()
            elif callable(u):
                u()
            elif u == "coll":
                self.sync.grads(self.grad_flat)
            elif u == "tic":
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
            elif u == "toc":
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                self.events.append((ev, e1))

    def step(self, x=None, target=None):
        """One optimisation step. x: list of input tensors (copied into the static input
        buffers), target: mask. Returns the loss as a device tensor (no host sync)."""
        if x is not None:
            for dst, src in zip(self.inputs, x):
                dst.copy_(src, non_blocking=True)
        if target is not None:
            self.target.copy_(target, non_blocking=True)
        self.step_count += 1
        self.sync.buffers(self.flatb)  # DDP broadcast_buffers: rank 0's BN running stats
        self._run(self.graphs if self.graphs else self._schedule(self.split))
        return self.loss_acc / self.logits.numel()

    def loss(self):
        return (self.loss_acc / self.logits.numel()).item()

    def grads(self):
        """Per-parameter gradient views of the last step (None for unused parameters)."""
        out = []
        for (k, p), (pgo, off, n, used) in zip(self.model.named_parameters(), self._pg_views):
            out.append(self.grad_flat[off:off + n].view_as(p) if used else None)
        return out
