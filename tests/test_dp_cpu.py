"""Data-parallel semantics on CPU (gloo, world_size 2), SURVEY.md §8e: each replica runs
the train step on its own sub-batch with LOCAL BatchNorm statistics; the exchanged
gradient equals the mean of the per-replica oracle gradients, and rank 0's BN running
statistics reach every replica (DDP broadcast_buffers). What runs is the Trainer's own
exchange (instancesegmentation_amd/train.py: comm buffer, two buckets, SUM) — the same
code path as RCCL on the GPUs, over gloo."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from instancesegmentation_amd.model.segment import Segment
from instancesegmentation_amd.train import Trainer
from oracle import segment_oracle
from oracle.seeding import synth_batch, synth_params


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _params():
    m = Segment(3)
    shapes = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    return synth_params(shapes, 5)


def _replica(params, x, mask):
    """Oracle fp64 train step of one replica on its sub-batch: (grads by key, params and
    updated BN buffers by key). train_step updates BN running statistics in place: give
    it private copies."""
    fresh = {k: np.array(v, copy=True) for k, v in params.items()}
    _, _, g, P = segment_oracle.train_step(fresh, x, mask, torch.float64)
    return g, P


def _load(m, params):
    sd = m.state_dict()
    m.load_state_dict({k: torch.as_tensor(v).to(sd[k].dtype) for k, v in params.items()})
    return m


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        params = _params()
        n, h, w = 2, 32, 48
        x, mask = synth_batch(n * world, 3, h, w, 9)  # global batch, 2 images per replica
        reps = [_replica(params, x[n * r:n * r + n], mask[n * r:n * r + n]) for r in range(world)]
        # the Trainer's own exchange state on this replica: its flat gradient (as the
        # step leaves it, pre-divided by the world size through the BCE scale) and its
        # locally updated BN running statistics, in the Trainer's flat layout
        tr = Trainer(_load(Segment(3), params), n, [(n, 3, h, w)], device="cpu")
        assert tr.world == world and tr.rank == rank
        assert tr.grad_scale == 1.0 / (n * h * w * world)
        g, P = reps[rank]
        names = [k for k, _ in tr.model.named_parameters()]
        with torch.no_grad():
            for k, (off, cnt) in zip(names, tr.index):
                gk = g.get(k)
                tr.grad_flat[off:off + cnt] = 0.0 if gk is None else \
                    (gk.reshape(-1) * tr.grad_scale * (n * h * w)).float()
            for k, b in tr.model.named_buffers():
                b.copy_(P[k].to(b.dtype))
        assert tr.plan.bucket_cut > 0 and len(tr.plan.bwd_parts) == 2
        tr._mask_buffers()
        tr.exchange_begin()
        tr.exchange_end()
        # reference: mean of every replica's gradient (each on its own sub-batch) and rank
        # 0's running statistics
        gerr = 0.0
        for k, (off, cnt) in zip(names, tr.index):
            ref = sum(rp[0][k] for rp in reps) / world if g.get(k) is not None else None
            got = tr.grad_flat[off:off + cnt].double()
            if ref is None:
                assert got.abs().max().item() == 0.0, k
                continue
            sc = max(ref.abs().max().item(), 1e-30)
            gerr = max(gerr, (got - ref.reshape(-1)).abs().max().item() / sc)
        berr, local_differs = 0.0, rank == 0
        for k, b in tr.model.named_buffers():
            if not b.is_floating_point():
                continue
            ref0 = reps[0][1][k].float()
            berr = max(berr, (b - ref0).abs().max().item())
            local_differs |= bool((P[k].float() - ref0).abs().max().item() > 0)
        out[rank] = (gerr, berr, local_differs)
    finally:
        dist.destroy_process_group()


def test_trainer_exchange_gloo():
    """The Trainer's own two-bucket exchange (comm buffer, buffer masking, SUM of
    world-scaled gradients) over gloo, world size 2."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        gerr, berr, local_differs = out[r]
        assert gerr < 1e-6, f"rank {r}: exchanged gradient != mean of replicas ({gerr:.2e})"
        assert berr == 0.0, f"rank {r}: running stats not rank 0's ({berr})"
        assert local_differs, "replicas must compute LOCAL batch statistics"


def test_single_process_exchange_is_identity():
    m = Segment(3)
    tr = Trainer(m, 2, [(2, 3, 32, 32)], device="cpu")
    g = torch.arange(tr.comm.numel(), dtype=torch.float32)
    tr.comm.copy_(g)
    tr._mask_buffers()
    tr.exchange_begin()
    tr.exchange_end()
    assert tr.world == 1 and torch.equal(tr.comm, g)
    assert tr.grad_scale == 1.0 / (2 * 32 * 32)


def test_bucket_split_covers_parameters():
    """Bucket 2 is the stem's parameters (a leading range of the flat gradient); the
    backward parts finalise exactly [cut, n) and [0, cut)."""
    from instancesegmentation_amd.engine import Plan
    m = Segment(20)
    shapes = [(2, 3, 64, 64), (2, 17, 64, 64)]
    plan = Plan(m, shapes, True, True, (False, False), buckets=2)
    names = [k for k, _ in m.named_parameters()]
    cut = plan.bucket_cut
    stem = sum(p.numel() for k, p in m.named_parameters() if k.startswith("init_conv."))
    assert cut == stem and names[0].startswith("init_conv.")
    p1, p2 = plan.bwd_parts
    assert [r.label for r in p2.recs if r.label.startswith("dw_")] == \
        ["dw_init_conv.layer2", "dw_init_conv.layer1"]
    assert not any(r.label.startswith(("dw_init", "dx_init")) for r in p1.recs)
    assert len(p1.recs) + len(p2.recs) == len(plan.bwd.recs)
    # world size 1: one backward part, one bucket (the whole flat gradient)
    tr = Trainer(m, 2, shapes, device="cpu")
    assert tr.world == 1 and len(tr.plan.bwd_parts) == 1 and tr.plan.bucket_cut == 0
    assert tr.buckets[0].numel() + tr.buckets[1].numel() == tr.comm.numel()
