"""Fused training step for the reference train loop (train_instance.py:371-382):

    optimizer.zero_grad(); out = model.train_batch(x, hm); loss = BCELoss(out, mask)
    loss.backward(); optimizer.step(); loss.item()

One `Trainer.step` runs, on one HIP stream and without torch autograd:
  forward op list -> fused sigmoid+BCE (loss + dlogits) -> backward part 1 ->
  [world > 1: RCCL SUM of gradient bucket 1 + running statistics, asynchronous] ->
  backward part 2 (the stem) -> [world > 1: bucket 2, wait] ->
  multi-tensor Adam over the flat parameter buffer.
Parameters, gradients and BN running statistics live in flat buffers (module tensors
are re-bound as views), so the optimizer is one kernel and the exchange is two
collectives over one buffer. The step is captured into HIP graphs (`capture()`): one
graph at world 1, three at world > 1 with the collectives issued between them.

Data parallelism: one process per GPU, image-batch sharded, local BN
statistics per replica, rank 0's running statistics on every replica after each step
(DDP's broadcast_buffers), gradient mean over ranks.
"""
import ctypes

import os

import torch
import torch.distributed as dist

from . import _lib as L
from .engine import (S_ACT, S_DOUT, S_EXPAVG, S_EXPAVGSQ, S_GRAD, S_HYPER, S_IN, S_OUT, S_OWNER,
                     S_PARAM, S_PGRAD, S_STAMP, S_STATS, S_STEP, S_TAILBNU, S_TAILGF, S_TENSOR0,
                     S_WREP, Plan, param_layout)

STAMP_HZ = 100e6  # s_memrealtime: the chip-global 100 MHz counter (MI355X_MICROARCH.md)


class GradSync:
    """The data-parallel exchange of one step, one process per GPU.

    Both gradient buckets and the BatchNorm running statistics travel in SUM all-reduces
    over one flat buffer `comm = [grad bucket 2 | grad bucket 1 | float buffers]`:
      * gradients arrive pre-divided by the world size (the BCE gradient scale is
        1/(pixels * world)), so the SUM is the replica mean DDP computes;
      * every rank but 0 zeroes its buffer slice first, so the SUM hands every replica
        rank 0's running statistics — DDP's `broadcast_buffers`, folded into the
        gradient collective instead of a second eager broadcast per step.
    Bucket 1 (every parameter but the stem's) is launched asynchronously as soon as the
    backward has finalised it, and overlaps the stem's backward; bucket 2 (the stem)
    follows the last weight gradient. On "nccl" (RCCL) the collectives run on the process
    group's own stream behind an event of the current stream and `wait()` makes the
    current stream wait for them; on gloo (CPU tests) they complete on the host. BN batch
    statistics stay local to each replica, as in the reference run per replica."""

    def __init__(self, process_group=None, force=False):
        """force: issue the collectives even at world size 1 when a process group exists
        (a one-rank RCCL communicator: the real exchange code path — communicator, RCCL's
        stream ordering, the asynchronous bucket-1 handle — on one GPU, where the SUM is the
        identity)."""
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.active = self.world > 1 or (bool(force) and dist.is_initialized())
        self._pending = []

    def begin(self, bucket):
        """Launch the SUM all-reduce of `bucket` (a view of comm) asynchronously."""
        if self.active and bucket.numel():
            self._pending.append(dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=self.pg,
                                                 async_op=True))

    def end(self):
        """Make the current stream (or host, on gloo) wait for every launched bucket."""
        for w in self._pending:
            w.wait()
        self._pending = []


def flatten_module(model, device, flatb=None, order=None):
    """Re-bind every parameter and floating buffer of `model` as a view of one flat
    buffer (params, laid out in `order` — parameter names, default the parameter order;
    the Trainer passes engine.param_layout, which puts sibling 1x1 conv weights next to
    each other) / (float buffers, into `flatb` when given: the Trainer passes the tail of its
    exchange buffer); returns (flat_params, flat_bufs, param_index) with param_index[i] =
    (offset, numel) of the i-th parameter in parameter order."""
    named = dict(model.named_parameters())
    order = list(order) if order is not None else list(named)
    if sorted(order) != sorted(named):
        raise ValueError("flatten_module: order is not a permutation of the parameters")
    n = sum(p.numel() for p in named.values())
    flat = torch.empty(n, dtype=torch.float32, device=device)
    where = {}
    off = 0
    with torch.no_grad():
        for k in order:
            p = named[k]
            c = p.numel()
            flat[off:off + c].copy_(p.detach().reshape(-1))
            p.data = flat[off:off + c].view_as(p)
            where[k] = (off, c)
            off += c
    index = [where[k] for k in named]
    fbufs = [(m, name, b) for m in model.modules() for name, b in m._buffers.items()
             if b is not None and b.is_floating_point()]
    nb = sum(b.numel() for _, _, b in fbufs)
    if flatb is None:
        flatb = torch.empty(max(nb, 1), dtype=torch.float32, device=device)
    elif flatb.numel() < nb:
        raise ValueError(f"flatten_module: buffer storage of {flatb.numel()} < {nb} floats")
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


def _float_buffer_count(model):
    return sum(b.numel() for m in model.modules() for b in m._buffers.values()
               if b is not None and b.is_floating_point())


class Trainer:
    """train_instance.py:294-382 step body on the MI355X (Segment + BCELoss + Adam).

    The flat parameter gradient and the flat BN running statistics share one buffer
    (`comm`), the data-parallel exchange unit (GradSync). A Trainer can be constructed
    on a CPU device (tests drive its exchange over gloo); `step()` needs the GPU."""

    def __init__(self, model, batch, in_shapes, device=None, lr=1e-3, betas=(0.9, 0.999),
                 eps=1e-8, weight_decay=0.0, process_group=None, dp_plan=None, fused_tail=None):
        """dp_plan: build the data-parallel step structure (two backward parts, two gradient
        buckets, three HIP graphs with the exchange markers between them) even at world
        size 1 — what that structure costs on one GPU (bench.py's dp_plan legs). Without a
        process group its exchanges are no-ops; with one (a world-size-1 "nccl" group) they
        are real one-rank RCCL all-reduces. Default: only at world size > 1.
        fused_tail: end the single-bucket step (no data-parallel exchange) in ONE launch —
        replica fold, gradient finalisation, Adam, BatchNorm running statistics
        (isg.h isg_step_tail, Plan fused_tail); default: whenever there is no exchange.
        False keeps the separate launches (the parity reference of the fused form)."""
        self.device = torch.device(device or "cuda")
        dev = self.device
        self.model = model.to(dev).train()
        world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.dp_plan = world > 1 if dp_plan is None else bool(dp_plan)
        self.sync = GradSync(process_group, force=self.dp_plan)
        self.world, self.rank = self.sync.world, self.sync.rank
        n = sum(p.numel() for p in self.model.parameters())
        nb = _float_buffer_count(self.model)
        self.comm = torch.zeros(n + max(nb, 1), dtype=torch.float32, device=dev)
        layout = param_layout(self.model)
        self.flat, self.flatb, self.index = flatten_module(self.model, dev, self.comm[n:], layout)
        self.in_shapes = [tuple(s) for s in in_shapes]
        # two gradient buckets only where an exchange overlaps the stem backward (Plan)
        buckets = int(os.environ.get("ISG_BUCKETS", "0")) or (2 if self.dp_plan else 1)
        self.fused_tail = (not self.dp_plan and buckets == 1) if fused_tail is None else bool(fused_tail)
        self.plan = Plan(self.model, self.in_shapes, True, True,
                         tuple(False for _ in self.in_shapes), buckets=buckets, layout=layout,
                         fused_tail=self.fused_tail)
        self.fused_tail = self.plan.fused_tail
        g = self.plan.graph
        assert g.pgrad_size == n
        for k, (off, _) in zip(g.params, self.index):  # the plan's gradient layout is the flat one
            assert g.pgrad_off[k] == off, k
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.act = torch.empty(max(self.plan.act_size, 1), dtype=torch.float32, device=dev)
        self.stats = torch.empty(self.plan.stats_size, dtype=torch.float64, device=dev)
        self.gradarena = torch.empty(max(self.plan.grad_size, 1), dtype=torch.float32, device=dev)
        # the plan's packed param-grad layout is exactly the flat buffer's order
        self.grad_flat = self.comm[:n]
        self.pgrad = self.grad_flat
        cut = self.plan.bucket_cut
        self.buckets = [self.comm[cut:], self.comm[:cut]]  # launch order: 1 (+buffers), 2
        self.wrep = torch.empty(L.WREP * g.pgrad_size, dtype=torch.float64, device=dev)
        self.logits = torch.empty(self.plan.out_shapes[0], dtype=torch.float32, device=dev)
        self.dlogits = torch.empty_like(self.logits)
        # BCELoss mean over this replica's pixels, pre-divided by the world size so the
        # exchange's SUM is the replica mean (GradSync)
        self.grad_scale = 1.0 / (self.logits.numel() * self.world)
        # zeroed by the forward's statistics memset (Plan.loss_off)
        self.loss_acc = self.stats[self.plan.loss_off:self.plan.loss_off + 1]
        self._pg_views = []
        for (k, p), (off, cnt) in zip(self.model.named_parameters(), self.index):
            self._pg_views.append((g.pgrad_off[k], off, cnt, k in self.plan.used_params))
        live = torch.zeros(self.flat.numel(), dtype=torch.uint8)
        for _, off, cnt, used in self._pg_views:
            if used:
                live[off:off + cnt] = 1
        self.live = live.to(dev)
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.step_count = 0
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)  # Adam's step, on device
        # 4-D: image / heatmaps (float32); 3-D: keypoints [N, parts, 3] (float64, engine.Keypoints)
        self.inputs = [torch.empty(s, dtype=torch.float32 if len(s) == 4 else torch.float64,
                                   device=dev) for s in self.in_shapes]
        self.target = torch.empty(self.plan.out_shapes[0], dtype=torch.float32, device=dev)
        # the fused tail's operands (Plan fused_tail): hyperparameters as device doubles (so
        # a captured graph follows load_optimizer_state_dict), the owner mask (bit 0: Adam
        # updates the element, bit 1: a grad_final item writes its gradient)
        self.hyper = torch.tensor(self._hyper_vec(), dtype=torch.float64, device=dev)
        owner = live.clone()
        for off, cnt in self.plan.tail_owned:
            owner[off:off + cnt] |= 2
        self.owner = owner.to(dev)
        self.table = self._make_table()
        self.tail_items = None
        if self.fused_tail:
            gf, bnu = self.plan.tail_tables(self.table)
            self.tail_items = [torch.frombuffer(bytearray(b or b"\0"), dtype=torch.uint8).to(dev)
                               for b in (gf, bnu)]
            self.table[S_TAILGF] = self.tail_items[0].data_ptr()
            self.table[S_TAILBNU] = self.tail_items[1].data_ptr() if bnu else None
        self.graphs = None
        self._captured = (None, None)
        self.events = []
        self.split = None
        self.stamp_at = None  # (phase, index): OP_STAMP records around that op (stamp_times)
        self.stamp_buf = torch.zeros(4, dtype=torch.int64, device=dev)  # isg_stamp's sums / max / min
        self.table[S_STAMP] = self.stamp_buf.data_ptr()

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
        tab[S_PARAM] = self.flat.data_ptr()
        tab[S_EXPAVG] = self.exp_avg.data_ptr()
        tab[S_EXPAVGSQ] = self.exp_avg_sq.data_ptr()
        tab[S_OWNER] = self.owner.data_ptr()
        tab[S_STEP] = self.step_dev.data_ptr()
        tab[S_HYPER] = self.hyper.data_ptr()
        tensors = [p for _, p in self.model.named_parameters()] + \
                  [b for _, b in self.model.named_buffers()]
        for j, t in enumerate(tensors):
            tab[S_TENSOR0 + j] = t.data_ptr()
        return tab

    # ---- the step body -------------------------------------------------------------
    def _hyper(self):
        return (float(self.lr), tuple(float(b) for b in self.betas), float(self.eps),
                float(self.wd))

    def _hyper_vec(self):
        return [float(self.lr), float(self.betas[0]), float(self.betas[1]), float(self.eps),
                float(self.wd)]

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
        L.check(lib.isg_bce_sigmoid(self.logits.data_ptr(), self.target.data_ptr(), n,
                                    self.loss_acc.data_ptr(), self.dlogits.data_ptr(),
                                    self.grad_scale, st), "bce")

    def _mask_buffers(self):
        """DDP broadcast_buffers through the SUM exchange: ranks > 0 contribute zeros."""
        if self.rank != 0:
            self.flatb.zero_()

    # exchange markers: run eagerly between captured graphs (RCCL is not captured)
    def exchange_begin(self):
        """Bucket 1 (all parameters but the stem's, plus the running statistics)."""
        self.sync.begin(self.buckets[0])

    def exchange_end(self):
        """Bucket 2 (the stem), then wait for both."""
        self.sync.begin(self.buckets[1])
        self.sync.end()

    def _schedule(self, split=None):
        """The step as a list of units: callables issuing HIP work, or the markers
        'coll1'/'coll2' (eager RCCL bucket exchange), 'tic'/'toc' (timing events around
        one op). split=(phase, idx) isolates op `idx` of the forward/backward list.
        self.stamp_at=(phase, idx): that op's list runs with OP_STAMP records around the op
        (OpList.stamped) — timed in place, the list (and the graph) not cut."""
        def run_list(ol):
            return lambda: ol.run(self.table, L.stream_ptr(self.device), L.side_stream_ptr(self.device),
                                  L.side_stream2_ptr(self.device))
        dp = self.dp_plan
        lists = [("fwd", self.plan.fwd)] + [("bwd", p) for p in self.plan.bwd_parts]
        units = []
        base = 0  # index of the current backward part's first op in the whole backward
        for j, (phase, ol) in enumerate(lists):
            if self.stamp_at and self.stamp_at[0] == phase:
                k = self.stamp_at[1] - (base if phase == "bwd" else 0)
                if 0 <= k < len(ol.recs):
                    ol = ol.stamped(k)
            i = None
            if split and split[0] == phase:
                i = split[1] - (base if phase == "bwd" else 0)
                if not 0 <= i < len(ol.recs):
                    i = None
            if i is not None:
                if i > 0:
                    units.append(run_list(ol.slice(0, i)))
                units += ["tic", run_list(ol.slice(i, i + 1)), "toc"]
                if i + 1 < len(ol.recs):
                    units.append(run_list(ol.slice(i + 1, len(ol.recs))))
            else:
                units.append(run_list(ol))
            if phase == "fwd":
                units.append(self._loss)
            else:
                base += len(ol.recs)
                if dp and j == 1:
                    units += [self._mask_buffers, "coll1"]
        if dp:
            units.append("coll2")
        if not self.fused_tail:  # (fused: Adam ran inside the backward's step tail)
            units.append(self._adam)
        return units

    def stamp_reset(self):
        self.stamp_buf.copy_(torch.tensor([0, 0, 0, 2 ** 63 - 1], dtype=torch.int64))

    def stamp_times(self, steps):
        """Since stamp_reset, over `steps` replays: (mean ms of the stamped op between its two
        stamps, mean ms of the back-to-back calibration pair, ms from the first to the last
        stamp), from the 100 MHz counter."""
        b = self.stamp_buf.cpu().tolist()
        ms = 1e3 / STAMP_HZ
        return b[0] * ms / steps, b[1] * ms / steps, (b[2] - b[3]) * ms

    def _state(self):
        return [self.comm, self.flat, self.exp_avg, self.exp_avg_sq, self.step_dev,
                self.loss_acc] + [b for _, b in self.model.named_buffers()
                                  if not b.is_floating_point()]

    def warm(self):
        """Run the step once eagerly (first-use initialisation in libisg, RCCL
        communicators) and restore the training state, so a capture can be the first
        training step."""
        saved = [t.clone() for t in self._state()]
        self._run(self._schedule())
        torch.cuda.synchronize(self.device)
        with torch.no_grad():
            for t, v in zip(self._state(), saved):
                t.copy_(v)

    def capture(self, split=None, warm=True):
        """Record the step into HIP graphs: every run of consecutive HIP units becomes one
        graph; markers between them stay eager (RCCL collectives, timing events)."""
        if warm:
            self.warm()
        torch.cuda.synchronize(self.device)
        self._captured = (split, self._hyper())
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
            elif u == "coll1":
                self.exchange_begin()
            elif u == "coll2":
                self.exchange_end()
            elif u == "tic":
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
            elif u == "toc":
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                self.events.append((ev, e1))

    def step(self, x=None, target=None, loss=True):
        """One optimisation step. x: list of input tensors (copied into the static input
        buffers), target: mask. Returns the loss as a device tensor (no host sync); with
        loss=False nothing (the mean is one more eager launch per step; the summed loss
        stays in loss_acc for loss())."""
        if self.device.type != "cuda":
            raise RuntimeError("Trainer.step runs on the MI355X only (no CPU path)")
        if x is not None:
            for dst, src in zip(self.inputs, x):
                dst.copy_(src, non_blocking=True)
        if target is not None:
            self.target.copy_(target, non_blocking=True)
        self.step_count += 1
        self._run(self.graphs if self.graphs else self._eager_units())
        return self.loss_acc / self.logits.numel() if loss else None

    def _eager_units(self):
        """The uncaptured step's units, built once per (split, stamp_at) — a stamped list is
        a compiled copy, not something to rebuild on every step."""
        key = (self.split, self.stamp_at)
        if getattr(self, "_eager_key", None) != key:
            self._eager = self._schedule(self.split)
            self._eager_key = key
        return self._eager

    def loss(self):
        return (self.loss_acc / self.logits.numel()).item()

    def grads(self):
        """Per-parameter gradient views of the last step (None for unused parameters).
        With world > 1 this is the exchanged replica mean."""
        out = []
        for (k, p), (pgo, off, n, used) in zip(self.model.named_parameters(), self._pg_views):
            out.append(self.grad_flat[off:off + n].view_as(p) if used else None)
        return out

    # ---- checkpoint interchange with the reference loop (train_instance.py:320-328, :497-503)
    def optimizer_state_dict(self):
        """The Adam state as `torch.optim.Adam(model.parameters()).state_dict()` would hold
        it (parameter indices in model.parameters() order; no entry for a parameter that
        never had a gradient, like torch's lazily created state)."""
        step = float(self.step_dev.item())
        state = {}
        if step > 0:
            for i, ((k, p), (_, off, n, used)) in enumerate(zip(self.model.named_parameters(),
                                                                self._pg_views)):
                if not used:
                    continue
                state[i] = {"step": torch.tensor(step, dtype=torch.float32),
                            "exp_avg": self.exp_avg[off:off + n].view_as(p).detach().cpu().clone(),
                            "exp_avg_sq": self.exp_avg_sq[off:off + n].view_as(p).detach().cpu().clone()}
        group = {"lr": self.lr, "betas": tuple(self.betas), "eps": self.eps,
                 "weight_decay": self.wd, "amsgrad": False, "maximize": False, "foreach": None,
                 "capturable": False, "differentiable": False, "fused": None,
                 "decoupled_weight_decay": False,
                 "params": list(range(len(self._pg_views)))}
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, sd):
        """Inverse of optimizer_state_dict; accepts the reference's saved optimizer."""
        groups = sd["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(self._pg_views):
            raise ValueError("optimizer state does not match Adam(model.parameters()) of this model")
        g = groups[0]
        self.lr, self.betas, self.eps, self.wd = (float(g["lr"]), tuple(g["betas"]),
                                                  float(g["eps"]), float(g["weight_decay"]))
        steps = []
        with torch.no_grad():
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            params = [p for _, p in self.model.named_parameters()]
            for i, st in sd["state"].items():
                i = int(i)
                _, off, n, _ = self._pg_views[i]
                self.exp_avg[off:off + n].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
                steps.append(int(float(st["step"])))
                assert st["exp_avg"].shape == params[i].shape
        self.step_dev.fill_(max(steps) if steps else 0)
        self.step_count = max(steps) if steps else 0
        self.hyper.copy_(torch.tensor(self._hyper_vec(), dtype=torch.float64))
        # isg_adam_dev takes lr/betas/eps/wd by value, so a captured graph holds the old
        # ones: re-record the step when the loaded hyperparameters differ
        if self.graphs and self._captured[1] != self._hyper():
            self.capture(split=self._captured[0])

    def load_state_dict(self, sd):
        """Model weights and buffers, copied into the flat buffers in place (the captured
        graphs keep pointing at them)."""
        self.model.load_state_dict(sd)

    # ---- evaluation helpers (train_instance.py:394-417) -------------------------------
    def probabilities(self):
        """sigmoid of the last step's logits (train-mode BN), the reference's outmask_ts."""
        out = torch.empty_like(self.logits)
        L.check(L.lib().isg_sigmoid_fwd(self.logits.data_ptr(), out.data_ptr(), out.numel(),
                                        L.stream_ptr(self.device)), "sigmoid")
        return out

    def predict(self, xs):
        """model.eval(); train_batch(x, heatmaps) under no_grad (train_instance.py:395-411)."""
        self.model.eval()
        try:
            with torch.no_grad():
                return self.model.train_batch(*xs)
        finally:
            self.model.train()
