"""ctypes binding of libisg.so (include/isg.h) — the only way Python reaches the kernels.

The library is built in-tree by `instancesegmentation_amd.build_lib` (hipcc,
gfx950). There is no fallback: if the .so is missing or fails to load, every op
raises. torch must be imported first so libisg.so binds to the HIP runtime torch
already loaded (both carry SONAME libamdhip64.so.7).
"""
import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_double, c_float, c_int32, c_int64, c_void_p

import torch  # noqa: F401  (load torch's HIP runtime before libisg)

# ISG_LIB: an alternative in-tree build (experiments: tools/build_variant.sh)
LIB_PATH = os.environ.get("ISG_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libisg.so")

ACT = {"none": 0, "relu": 1, "prelu": 2}
XF_PLAIN, XF_BN_FWD, XF_BN_BWD = 0, 1, 2
SINK_STORE, SINK_ACCUM, SINK_ACTBWD, SINK_NONE = 0, 1, 2, 3
MAX_SEGS = 3
LIST_CHUNK = 32
STAT_REP = int(os.environ.get("ISG_STAT_REP", "4"))  # accumulator replicas (isg.h ISG_STAT_REP)
ABI_VERSION = 11
WREP = int(os.environ.get("ISG_WREP", "16"))  # weight-gradient replicas (isg.h ISG_WREP)


class Bn(Structure):
    _fields_ = [("gamma", c_void_p), ("beta", c_void_p), ("running_mean", c_void_p),
                ("running_var", c_void_p), ("stats", c_void_p), ("C", c_int32),
                ("train", c_int32), ("count", c_float), ("eps", c_float), ("coef", c_void_p)]


class VSeg(Structure):
    _fields_ = [("p", c_void_p), ("y", c_void_p), ("n_stride", c_int64),
                ("y_n_stride", c_int64), ("C", c_int32), ("xform", c_int32), ("act", c_int32),
                ("pad_", c_int32), ("slope", c_void_p), ("bn", Bn)]


class VTensor(Structure):
    _fields_ = [("s", VSeg * MAX_SEGS), ("nseg", c_int32), ("N", c_int32), ("H", c_int32),
                ("W", c_int32), ("mat", c_void_p), ("mat_n_stride", c_int64), ("rbn", Bn)]


class Sink(Structure):
    _fields_ = [("p", c_void_p), ("n_stride", c_int64), ("c0", c_int32), ("C", c_int32),
                ("mode", c_int32), ("act", c_int32), ("bias", c_void_p), ("stats", c_void_p),
                ("y", c_void_p), ("y_n_stride", c_int64), ("slope", c_void_p),
                ("slope_grad", c_void_p), ("bn", Bn), ("r", c_void_p), ("r_n_stride", c_int64),
                ("old", c_void_p), ("old_n_stride", c_int64), ("p2", c_void_p),
                ("p2_n_stride", c_int64), ("p2_accum", c_int32), ("pad2_", c_int32), ("rbn", Bn)]


class Sinks(Structure):
    _fields_ = [("s", Sink * MAX_SEGS), ("nsink", c_int32), ("pad_", c_int32)]


class Geom(Structure):
    _fields_ = [(n, c_int32) for n in ("N", "Ci", "H", "W", "Co", "OH", "OW", "KH", "KW", "SH",
                                       "SW", "PH", "PW", "DH", "DW", "groups", "w_ci", "pad_")]


class Tail(Structure):
    _fields_ = [("term", VSeg * 3), ("up", c_int32 * 3), ("nterm", c_int32), ("act", c_int32),
                ("slope", c_void_p), ("out", c_void_p), ("out_n_stride", c_int64),
                ("N", c_int32), ("C", c_int32), ("H", c_int32), ("W", c_int32)]


class TailGrad(Structure):
    _fields_ = [("f", Tail), ("dout", c_void_p), ("dout_n_stride", c_int64), ("g", c_void_p),
                ("g_n_stride", c_int64), ("dterm", c_void_p * 3),
                ("dterm_n_stride", c_int64 * 3), ("dterm_accum", c_int32 * 3),
                ("slope_grad", c_void_p)]


class BnUpdate(Structure):
    _fields_ = [("stats", c_void_p), ("running_mean", c_void_p), ("running_var", c_void_p),
                ("num_batches_tracked", c_void_p), ("C", c_int32), ("count", c_float),
                ("momentum", c_float), ("pad_", c_int32)]


class GradFinal(Structure):
    _fields_ = [("stats", c_void_p), ("gamma", c_void_p), ("running_mean", c_void_p),
                ("running_var", c_void_p), ("dgamma", c_void_p), ("dbeta", c_void_p),
                ("dconv_bias", c_void_p), ("slope_acc", c_void_p), ("dslope", c_void_p),
                ("C", c_int32), ("train", c_int32), ("count", c_float), ("eps", c_float),
                ("slope_stride", c_int32), ("pad_", c_int32)]


class KpStem(Structure):
    _fields_ = [("kp", c_void_p), ("nparts", c_int32), ("c_kp0", c_int32), ("sigma", c_double),
                ("threshold", c_double), ("g", Geom), ("w", c_void_p), ("y", c_void_p),
                ("y_n_stride", c_int64), ("stats", c_void_p), ("dy", VTensor), ("dw", c_void_p),
                ("rep_stride", c_int64), ("nrep", c_int32), ("k", c_int32), ("out", c_void_p),
                ("out_n_stride", c_int64)]


class MaskHead(Structure):
    _fields_ = [("x", VTensor), ("w1", c_void_p), ("b1", c_void_p), ("w2", c_void_p),
                ("b2", c_void_p), ("out", c_void_p), ("out_n_stride", c_int64), ("dout", c_void_p),
                ("dout_n_stride", c_int64), ("dx", Sinks), ("dw1", c_void_p), ("db1", c_void_p),
                ("dw2", c_void_p), ("db2", c_void_p), ("rep_stride", c_int64), ("nrep", c_int32),
                ("N", c_int32), ("Hi", c_int32), ("Wi", c_int32), ("pad_", c_int32), ("ring", c_void_p),
                ("dw1_part", c_void_p)]


def head_part_floats(N, Hi, Wi):
    """isg_mask_head_part_floats: the backward's dW1 partial slab, [workgroups][4096] with one
    workgroup per two 32 x 64 logit tiles, at most 256 (mask_head.hip head_bwd_blocks)."""
    ntiles = N * -(-4 * Hi // 32) * -(-4 * Wi // 64)
    return min((ntiles + 1) // 2, 256) * 4096


def head_ring_floats(Hi, Wi):
    """Floats per image of the mask head's ring buffer (isg.h ISG_HEAD_RING x 4 channels)."""
    return 4 * (2 * (4 * Wi + 2) + 2 * 4 * Hi)


# executor records (api.cpp)
class ConvRec(Structure):
    _fields_ = [("g", Geom), ("a", VTensor), ("w", c_void_p), ("out", Sinks)]


class WgradRec(Structure):
    _fields_ = [("g", Geom), ("dy", VTensor), ("x", VTensor), ("dw", c_void_p), ("dbias", c_void_p),
                ("rep_stride", c_int64), ("nrep", c_int32), ("pad_", c_int32)]


class SumRepRec(Structure):
    _fields_ = [("dst", c_void_p), ("src", c_void_p), ("n", c_int64), ("stride", c_int64),
                ("nrep", c_int32), ("pad_", c_int32)]


class PoolRec(Structure):
    _fields_ = [("x", VTensor), ("k", c_int32), ("pad_", c_int32), ("out", c_void_p),
                ("out_ns", c_int64), ("dout", c_void_p), ("dout_ns", c_int64), ("dx", Sinks)]


class ListRec(Structure):
    _fields_ = [("n", c_int32), ("pad_", c_int32)]


class BceRec(Structure):
    _fields_ = [("logits", c_void_p), ("target", c_void_p), ("n", c_int64), ("loss", c_void_p),
                ("dlogits", c_void_p), ("grad_scale", c_float), ("pad_", c_int32)]


class MemsetRec(Structure):
    _fields_ = [("p", c_void_p), ("bytes", c_int64)]


class StampRec(Structure):
    _fields_ = [("buf", c_void_p), ("slot", c_int32), ("sign", c_int32)]


class DwBwdRec(Structure):
    _fields_ = [("g", Geom), ("dy", VTensor), ("w", c_void_p), ("dx", Sinks), ("x", VTensor),
                ("dw", c_void_p), ("dbias", c_void_p), ("rep_stride", c_int64), ("nrep", c_int32),
                ("pad_", c_int32)]


class StepTail(Structure):  # isg.h isg_step_tail_args (also the OP_STEP_TAIL record)
    _fields_ = [("grad", c_void_p), ("rep", c_void_p), ("n", c_int64), ("nrep", c_int32),
                ("ngf", c_int32), ("param", c_void_p), ("exp_avg", c_void_p),
                ("exp_avg_sq", c_void_p), ("owner", c_void_p), ("step", c_void_p),
                ("hyper", c_void_p), ("gf", c_void_p), ("bnu", c_void_p), ("nbnu", c_int32),
                ("pad_", c_int32)]


class StepIncRec(Structure):
    _fields_ = [("step", c_void_p)]


OP_CONV_FWD, OP_CONV_DGRAD, OP_CONV_WGRAD, OP_CONVT_FWD = 1, 2, 3, 4
OP_MAXPOOL_FWD, OP_MAXPOOL_BWD, OP_TAIL_FWD, OP_TAIL_BWD = 5, 6, 7, 8
OP_BN_UPDATE, OP_GRAD_FINAL, OP_BCE, OP_MEMSET = 9, 10, 11, 12
OP_SUM_REP, OP_BN_FINAL = 13, 14
OP_KP_STEM_FWD, OP_KP_STEM_WGRAD, OP_KP_POOL = 15, 16, 17
OP_HEAD_FWD, OP_HEAD_BWD = 18, 19
OP_STAMP = 20
OP_DW_BWD = 21
OP_HEAD_FOLD = 22
OP_STEP_TAIL, OP_STEP_INC = 24, 25

_RECORD_CHECK = [(0, VTensor), (1, Sinks), (2, ConvRec), (3, WgradRec), (4, PoolRec), (5, Tail),
                 (6, TailGrad), (7, BnUpdate), (8, GradFinal), (9, BceRec), (10, Geom), (11, Bn),
                 (12, VSeg), (13, Sink), (14, SumRepRec), (15, KpStem), (16, MaskHead),
                 (17, StampRec), (18, DwBwdRec), (19, StepTail)]

# exported symbol -> (restype, argtypes)
SIGNATURES = {
    "isg_conv_fwd": (c_int32, [POINTER(Geom), POINTER(VTensor), c_void_p, POINTER(Sinks), c_void_p]),
    "isg_conv_dgrad": (c_int32, [POINTER(Geom), POINTER(VTensor), c_void_p, POINTER(Sinks), c_void_p]),
    "isg_conv_wgrad": (c_int32, [POINTER(Geom), POINTER(VTensor), POINTER(VTensor), c_void_p,
                                 c_void_p, c_void_p]),
    "isg_conv_wgrad_rep": (c_int32, [POINTER(Geom), POINTER(VTensor), POINTER(VTensor), c_void_p,
                                     c_void_p, c_int64, c_int32, c_void_p]),
    "isg_sum_replicas": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_int64, c_void_p]),
    "isg_depthwise_bwd": (c_int32, [POINTER(Geom), POINTER(VTensor), c_void_p, POINTER(Sinks),
                                    POINTER(VTensor), c_void_p, c_void_p, c_int64, c_int32, c_void_p]),
    "isg_convT_fwd": (c_int32, [POINTER(Geom), POINTER(VTensor), c_void_p, POINTER(Sinks), c_void_p]),
    "isg_maxpool_fwd": (c_int32, [POINTER(VTensor), c_int32, c_void_p, c_int64, c_void_p]),
    "isg_maxpool_bwd": (c_int32, [POINTER(VTensor), c_int32, c_void_p, c_int64, POINTER(Sinks),
                                  c_void_p]),
    "isg_tail_fwd": (c_int32, [POINTER(Tail), c_void_p]),
    "isg_tail_bwd": (c_int32, [POINTER(TailGrad), c_void_p]),
    "isg_bn_update_running": (c_int32, [POINTER(BnUpdate), c_int32, c_void_p]),
    "isg_grad_finalize": (c_int32, [POINTER(GradFinal), c_int32, c_void_p]),
    "isg_bn_finalize": (c_int32, [POINTER(Bn), c_int32, c_int32, c_void_p]),
    "isg_bce_sigmoid": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_float, c_void_p]),
    "isg_sigmoid_fwd": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    "isg_sigmoid_bwd": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "isg_adam": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                           c_double, c_double, c_double, c_double, c_double, c_void_p]),
    "isg_adam_dev": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                               c_void_p, c_double, c_double, c_double, c_double, c_double,
                               c_void_p]),
    "isg_step_tail": (c_int32, [POINTER(StepTail), c_void_p]),
    "isg_step_inc": (c_int32, [c_void_p, c_void_p]),
    "isg_fill_f64": (c_int32, [c_void_p, c_int64, c_double, c_void_p]),
    "isg_stamp": (c_int32, [c_void_p, c_int32, c_int32, c_void_p]),
    "isg_mask_paste": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_int32, c_int32, c_void_p,
                                 c_void_p]),
    "isg_mask_nms_workspace": (c_int64, [c_int32, c_int32, c_int32]),
    "isg_mask_nms": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_float, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p]),
    "isg_mask_paste_nms": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_int32, c_int32, c_float,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "isg_instance_crop": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_int32,
                                    c_int32, c_void_p, c_void_p]),
    "isg_keypoint_heatmaps": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int32, c_double,
                                        c_double, c_void_p, c_void_p]),
    "isg_kp_stem_fwd": (c_int32, [POINTER(KpStem), c_void_p]),
    "isg_kp_stem_wgrad": (c_int32, [POINTER(KpStem), c_void_p]),
    "isg_kp_pool": (c_int32, [POINTER(KpStem), c_void_p]),
    "isg_mask_head_fwd": (c_int32, [POINTER(MaskHead), c_void_p]),
    "isg_mask_head_bwd": (c_int32, [POINTER(MaskHead), c_void_p]),
    "isg_mask_head_fold": (c_int32, [POINTER(MaskHead), c_void_p]),
    "isg_mask_head_part_floats": (c_int64, [c_int32, c_int32, c_int32]),
    "isg_exec": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p]),
    "isg_exec_ms": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    "isg_exec_ms2": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "isg_last_error": (c_char_p, []),
    "isg_abi_version": (c_int32, []),
    "isg_stat_replicas": (c_int32, []),
    "isg_record_size": (c_int32, [c_int32]),
}

_lib = None


def lib():
    """Load (once) and return the ctypes handle; raises if the HIP library is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libisg.so not found at {LIB_PATH}; build it with "
                "`python -m instancesegmentation_amd.build_lib` (there is no CPU fallback)")
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        if h.isg_abi_version() != ABI_VERSION or h.isg_stat_replicas() != STAT_REP:
            raise RuntimeError(f"ABI mismatch: libisg.so is version {h.isg_abi_version()} "
                               f"with {h.isg_stat_replicas()} stat replicas, expected "
                               f"{ABI_VERSION} / {STAT_REP}; rebuild it")
        for which, cls in _RECORD_CHECK:
            n = h.isg_record_size(which)
            if n != ctypes.sizeof(cls):
                raise RuntimeError(f"ABI mismatch: {cls.__name__} is {ctypes.sizeof(cls)} bytes "
                                   f"in Python, {n} in libisg.so")
        _lib = h
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = lib().isg_last_error().decode(errors="replace")
        raise RuntimeError(f"libisg {what} failed ({rc}): {msg}")
    return rc


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream


_SIDE = {}


def _new_side_stream(d):
    # (round 6, measured and dropped: side streams restricted to a CU mask
    # (hipExtStreamCreateWithCUMask, 4 or 6 of every 8 CUs) took the step 3.62 -> 7.0 ms)
    return torch.cuda.Stream(device=d)


def side_stream_ptr(device=None):
    """The executor's side stream of `device` (weight gradients fork onto it)."""
    d = torch.cuda.current_device() if device is None else torch.device(device).index
    if d is None:
        d = torch.cuda.current_device()
    if d not in _SIDE:
        _SIDE[d] = _new_side_stream(d)
    return _SIDE[d].cuda_stream


_SIDE2 = {}


def side_stream2_ptr(device=None):
    """The executor's second side stream (batches of weight gradients are dealt over both),
    or None — the default since round 6: with the eager executor and the fused step tail a
    second side stream made the step slower, 3.36 -> 3.46 ms (profiles/r08g_ab_side2.txt),
    its extra weight gradients in flight taking CUs from the input-gradient chain.
    ISG_SIDE2=1 enables it (under its own parity test)."""
    if os.environ.get("ISG_SIDE2", "0") != "1":
        return None
    d = torch.cuda.current_device() if device is None else torch.device(device).index
    if d is None:
        d = torch.cuda.current_device()
    if d not in _SIDE2:
        _SIDE2[d] = _new_side_stream(d)
    return _SIDE2[d].cuda_stream
