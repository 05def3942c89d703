"""Data-parallel semantics on CPU (gloo, world_size 2), SURVEY.md §8e: each replica runs
the train step on its own sub-batch with LOCAL BatchNorm statistics; the exchanged
gradient equals the mean of the per-replica oracle gradients, and rank 0's BN running
statistics reach every replica (DDP broadcast_buffers). The exchange is the Trainer's own
GradSync (RCCL AVG on GPUs; SUM + scale on gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from instancesegmentation_amd.model.segment import Segment
from instancesegmentation_amd.train import GradSync
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


def _replica_grads(params, x, mask):
    # train_step updates BN running statistics in place: give it private copies
    fresh = {k: np.array(v, copy=True) for k, v in params.items()}
    _, _, g, P = segment_oracle.train_step(fresh, x, mask, torch.float64)
    keys = sorted(k for k, v in g.items() if v is not None)
    flat = torch.cat([g[k].reshape(-1) for k in keys])
    rm = torch.cat([P[k].reshape(-1) for k in sorted(P) if k.endswith("running_mean")])
    return flat, rm


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        params = _params()
        x, mask = synth_batch(2 * world, 3, 32, 48, 9)  # global batch, 2 images per replica
        sl = slice(2 * rank, 2 * rank + 2)
        g, rm = _replica_grads(params, x[sl], mask[sl])
        sync = GradSync()
        gx = g.clone()
        sync.grads(gx)
        # reference: mean of every replica's gradient, each from its own sub-batch
        ref = torch.stack([_replica_grads(params, x[2 * r:2 * r + 2], mask[2 * r:2 * r + 2])[0]
                           for r in range(world)]).mean(0)
        err = (gx - ref).abs().max().item() / ref.abs().max().item()
        # running statistics: each replica updated its own; the broadcast makes rank 0's win
        rmx = rm.clone()
        sync.buffers(rmx)
        rm0 = _replica_grads(params, x[0:2], mask[0:2])[1]
        berr = (rmx - rm0).abs().max().item()
        local_differs = rank == 0 or (rm - rm0).abs().max().item() > 0
        out[rank] = (err, berr, local_differs)
    finally:
        dist.destroy_process_group()


def test_dp_gradient_mean_and_buffer_broadcast_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        err, berr, local_differs = out[r]
        assert err < 1e-12, f"rank {r}: reduced gradient != mean of replicas ({err:.2e})"
        assert berr == 0.0, f"rank {r}: running stats not rank 0's ({berr})"
        assert local_differs, "replicas must compute LOCAL batch statistics"


def test_grad_sync_single_process_is_identity():
    g = torch.arange(5, dtype=torch.float32)
    s = GradSync()
    s.grads(g)
    s.buffers(g)
    assert s.world == 1 and torch.equal(g, torch.arange(5, dtype=torch.float32))
