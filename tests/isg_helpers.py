"""Direct C-ABI call helpers for kernel-level GPU tests (real pointers in the structs)."""
import ctypes

import torch

from instancesegmentation_amd import _lib as L
from instancesegmentation_amd.engine import _fill


def struct(cls, spec):
    obj = cls()
    fix = []
    _fill(obj, spec, 0, fix)
    assert not fix
    return obj


def ptr(t):
    return t.data_ptr() if t is not None else None


def rep_zeros(n, device="cuda"):
    """An accumulator of n doubles in its ISG_STAT_REP replicas (isg.h)."""
    return torch.zeros(L.STAT_REP * n, dtype=torch.float64, device=device)


def rep_from(vals, device="cuda"):
    """Replicated accumulator holding `vals` (replica 0) — precomputed stats input."""
    out = rep_zeros(vals.numel(), device)
    out[:vals.numel()] = vals.to(device=device, dtype=torch.float64)
    return out


def rep_fold(t, n):
    """Sum of the replicas of an accumulator of n values."""
    return t.view(L.STAT_REP, n).sum(0)


def bn_spec_eval(gamma, beta, rm, rv, eps=1e-5):
    return {"gamma": ptr(gamma), "beta": ptr(beta), "running_mean": ptr(rm),
            "running_var": ptr(rv), "C": gamma.numel(), "train": 0, "count": 1.0, "eps": eps}


def bn_spec_train(gamma, beta, stats, count, eps=1e-5):
    return {"gamma": ptr(gamma), "beta": ptr(beta), "stats": ptr(stats), "C": gamma.numel(),
            "train": 1, "count": float(count), "eps": eps}


def vt(segs, N, H, W):
    return struct(L.VTensor, {"s": segs, "nseg": len(segs), "N": N, "H": H, "W": W})


def sinks(lst):
    return struct(L.Sinks, {"s": lst, "nsink": len(lst)})


def geom(**kw):
    return struct(L.Geom, kw)


def stream():
    return L.stream_ptr()


def call(name, *args):
    fn = getattr(L.lib(), name)
    conv = []
    for a in args:
        if isinstance(a, ctypes.Structure):
            conv.append(ctypes.byref(a))
        else:
            conv.append(a)
    L.check(fn(*conv), name)
    torch.cuda.synchronize()
