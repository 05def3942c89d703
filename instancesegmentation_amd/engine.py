"""Static-schedule engine: turns a module's `emit` description into two recorded op
lists (forward, backward) for the native executor `isg_exec` (include/isg.h).

Why: the reference runs ~300 forward and ~600 backward eager kernels per step, each
launched from Python (segment.py:44-45 is conv -> bn -> act as three kernels). Here
a module is traced once per input shape into a list of fused-op records whose
pointers are symbolic (slot, byte offset); a call replays the list with one ctypes
call and a fresh pointer table, and the same list can be captured into a HIP graph.

Values flowing between ops are *virtual tensors*: a raw conv output plus the
BatchNorm/activation its consumer applies on load (Conv.forward, segment.py:44-45),
possibly several channel segments (torch.cat, segment.py:31, 331, 485, 494).
Residual-block tails (`out = act(sum terms)`) are the only materialisation points.

Backward is derived op by op in reverse order:
  * a consumer of a virtual value writes g = dL/d(BN output) through an ACTBWD sink
    and accumulates the BN-backward statistics; the producer conv then rebuilds
    dL/dy on load (BN_BWD segment) for its dgrad and wgrad;
  * a consumer of a materialised value accumulates dL/dvalue (STORE first, then ACCUM);
  * BN gamma/beta, conv-bias-before-BN and PReLU gradients are finalised from the
    double-precision statistics in one pass at the end.
"""
import ctypes
import contextlib
import os
import struct

import torch
import torch.nn as nn

from . import _lib as L

# fixed pointer-table slots
S_ACT, S_GRAD, S_STATS, S_PGRAD, S_LOSS, S_TARGET = 0, 1, 2, 3, 4, 5
S_IN = (6, 7)
S_OUT = (8, 9)
S_DOUT = (10, 11)
S_DIN = (12, 13)
S_WREP = 14  # L.WREP fp64 replicas of the flat parameter gradient (wgrad atomics, isg.h)
S_STAMP = 15  # timestamp buffer of OP_STAMP records (isg_stamp: uint32 counter, then slots)
# the fused step tail (Plan fused_tail, isg.h isg_step_tail): the Trainer's flat parameters,
# Adam moments, per-element owner mask, device step counter, hyperparameters (5 doubles) and
# the device tables of its grad_final / BatchNorm-update items
S_PARAM, S_EXPAVG, S_EXPAVGSQ, S_OWNER, S_STEP, S_HYPER, S_TAILGF, S_TAILBNU = range(16, 24)
S_TENSOR0 = 24

ALIGN = 64  # elements (256 B) between arena buffers


class Ptr:
    __slots__ = ("slot", "off")

    def __init__(self, slot, off=0):
        self.slot = slot
        self.off = off

    def plus(self, nbytes):
        return Ptr(self.slot, self.off + nbytes)


# ---------------------------------------------------------------------------------
# record building
def _fill(obj, spec, base, fix):
    for k, v in spec.items():
        fld = getattr(type(obj), k)
        off = base + fld.offset
        if v is None:
            continue
        if isinstance(v, Ptr):
            fix.append((off, v.slot, v.off))
        elif isinstance(v, dict):
            _fill(getattr(obj, k), v, off, fix)
        elif isinstance(v, (list, tuple)):
            arr = getattr(obj, k)
            esz = ctypes.sizeof(arr._type_)
            for i, e in enumerate(v):
                if e is None:
                    continue
                if isinstance(e, dict):
                    _fill(arr[i], e, off + i * esz, fix)
                elif isinstance(e, Ptr):
                    fix.append((off + i * esz, e.slot, e.off))
                else:
                    arr[i] = e
        else:
            setattr(obj, k, v)


class Record:
    OPF_SIDE, OPF_JOIN, OPF_FORK_NOW = 1, 2, 4  # executor header flags (api.cpp)
    # a join's count of the most recent side records it does NOT wait for (_join_exclusions)
    EXCL_SHIFT, EXCL_MAX = 8, (1 << 20) - 1

    def __init__(self, kind, cls, spec, items_cls=None, items=None, label="", flops=0, nbytes=0):
        self.kind = kind
        self.flags = 0
        self.label = label
        self.flops = flops    # algorithmic FLOPs of this launch (2*MAC)
        self.nbytes = nbytes  # algorithmic HBM bytes (each operand read/written once)
        rec = cls()
        fix = []
        _fill(rec, spec, 0, fix)
        body = bytes(rec)
        if items_cls is not None:
            parts = [body]
            isz = ctypes.sizeof(items_cls)
            for i, it in enumerate(items):
                o = items_cls()
                _fill(o, it, len(body) + i * isz, fix)
                parts.append(bytes(o))
            body = b"".join(parts)
        self.body = body
        self.fix = fix

    def pack(self):
        n = len(self.body)
        pad = (-n) % 8
        out = [struct.pack("<iiii", self.kind, n, len(self.fix), self.flags), self.body,
               b"\0" * pad]
        out += [struct.pack("<iiq", loc, slot, off) for loc, slot, off in self.fix]
        return b"".join(out)


class OpList:
    def __init__(self):
        self.recs = []

    def add(self, rec):
        self.recs.append(rec)

    def compile(self):
        self.blob = b"".join(r.pack() for r in self.recs)
        self._buf = ctypes.create_string_buffer(self.blob, len(self.blob))
        return self

    def run(self, table, stream, side=None, side2=None):
        if side is None:
            L.check(L.lib().isg_exec(ctypes.addressof(self._buf), len(self.recs), table, stream),
                    "exec")
        else:
            L.check(L.lib().isg_exec_ms2(ctypes.addressof(self._buf), len(self.recs), table,
                                         stream, side, side2), "exec")

    def slice(self, i, j):
        """A compiled sub-list recs[i:j] (to bracket one op with events)."""
        o = OpList()
        o.recs = self.recs[i:j]
        return o.compile()

    def stamped(self, idx):
        """A compiled copy with OP_STAMP records (isg_stamp into slot S_STAMP) on the main
        stream: a calibration pair first (two stamps back to back, slot 1: what a bracket
        costs without an op), then one right before and one right after record `idx` (slot
        0) — the op timed where it runs in the step, side streams and all, without cutting
        the list."""
        import copy

        def stamp(slot, sign):
            return Record(L.OP_STAMP, L.StampRec, {"buf": Ptr(S_STAMP), "slot": slot,
                                                   "sign": sign}, label="stamp")
        op = copy.copy(self.recs[idx])
        before = stamp(0, -1)
        # a join the op carries happens before its first stamp; a side-stream op (a weight
        # gradient) is timed on the main stream
        # (with its exclusion count: the stamp adds no side record)
        before.flags = op.flags & (Record.OPF_JOIN | (Record.EXCL_MAX << Record.EXCL_SHIFT))
        was_side = op.flags & Record.OPF_SIDE
        op.flags = 0
        o = OpList()
        o.recs = [stamp(1, -1), stamp(1, 1)] + self.recs[:idx] + [before, op, stamp(0, 1)] + \
            self.recs[idx + 1:]
        if was_side:  # one side record fewer: recount (a join on the moved op waits for all)
            new = {id(r): copy.copy(r) for r in o.recs}
            for r in new.values():
                if getattr(r, "join_deps", None):
                    r.join_deps = {id(new[d]) for d in r.join_deps if d in new}
            o.recs = [new[id(r)] for r in o.recs]
            _join_exclusions(o.recs)
        return o.compile()


# ---------------------------------------------------------------------------------
# graph values
class Buf:
    """An NCHW fp32 region of an arena (act or grad) or an external slot."""

    def __init__(self, slot, N, C, H, W, name, off=0):
        self.slot, self.N, self.C, self.H, self.W, self.name = slot, N, C, H, W, name
        self.off = off  # elements

    @property
    def n_stride(self):
        return self.C * self.H * self.W

    @property
    def numel(self):
        return self.N * self.C * self.H * self.W

    def ptr(self, c0=0):
        return Ptr(self.slot, (self.off + c0 * self.H * self.W) * 4)


MAX_TENSOR_ELEMS = 2 ** 31 - 1


def check_elems(b):
    """The kernels address a tensor's elements (image stride x image + pixel) with 32-bit
    offsets; a tensor at or above 2^31 elements is refused here, at plan time."""
    if b.numel > MAX_TENSOR_ELEMS:
        raise RuntimeError(f"{b.name}: {b.N}x{b.C}x{b.H}x{b.W} = {b.numel} elements exceeds "
                           f"the kernels' 32-bit element offsets ({MAX_TENSOR_ELEMS}); "
                           "split the batch")


class BNRef:
    def __init__(self, mod, C, count, stats_off, names):
        self.mod, self.C, self.count, self.stats_off = mod, C, count, stats_off
        self.names = names  # dict: gamma, beta, rm, rv, nbt -> tensor slot


class SlopeRef:
    def __init__(self, mod, C, acc_off, slot):
        self.mod, self.C, self.acc_off, self.slot = mod, C, acc_off, slot
        self.used_in_bwd = False


class Val:
    """One channel segment: act(BN(buf[c0:c0+C])) (identity when bn is None, act none)."""

    def __init__(self, buf, c0, C, bn=None, act="none", slope=None, grad=True):
        self.buf, self.c0, self.C = buf, c0, C
        self.bn, self.act, self.slope = bn, act, slope
        self.grad = grad

    @property
    def virtual(self):
        return self.bn is not None or self.act != "none"


class Value:
    def __init__(self, segs):
        self.segs = list(segs)
        assert len({(s.buf.H, s.buf.W) for s in self.segs}) == 1
        self.H, self.W = self.segs[0].buf.H, self.segs[0].buf.W
        self.C = sum(s.C for s in self.segs)

    @property
    def grad(self):
        return any(s.grad for s in self.segs)


def cat(*vals):
    segs = []
    for v in vals:
        segs += v.segs
    return Value(segs)


class Keypoints:
    """Keypoint input [N, nparts, 3] float64 = (x, y, visible > 0) of slot `slot`, standing
    for `nparts` heatmap channels (train_instance.py:33-68) that are never materialised:
    the stem synthesises them on the fly (isg_kp_stem)."""

    def __init__(self, slot, N, nparts, sigma=10.0, threshold=0.01):
        self.slot, self.N, self.nparts = slot, N, nparts
        self.sigma, self.threshold = sigma, threshold
        self.C = nparts
        self.grad = False

    def spec(self):
        return {"kp": Ptr(self.slot), "nparts": self.nparts, "sigma": float(self.sigma),
                "threshold": float(self.threshold)}


# ---------------------------------------------------------------------------------
def param_layout(owner):
    """The flat parameter order of a Trainer (train.flatten_module): the module's
    parameter order, except that the weight of the second conv of each sibling pair — two
    1x1 Convs reading the same input, declared by a module's `siblings()` (BottleneckDim_Res
    convs.0 + resconv, segment.py:198-202; BottleneckUp_Res convs.0 + conv2, :326-331) —
    follows the first one's weight directly, so the pair's weights [W1; W2] (and their
    gradients) are ONE contiguous [C1 + C2][Ci] matrix and the pair runs as one GEMM
    (Graph.conv_pair)."""
    names = {id(m): pre for pre, m in owner.named_modules()}
    order = [k for k, _ in owner.named_parameters()]
    for m in owner.modules():
        sib = getattr(m, "siblings", None)
        if not callable(sib):
            continue
        a, b = sib()
        ka, kb = f"{names[id(a)]}.conv.weight", f"{names[id(b)]}.conv.weight"
        if ka in order and kb in order:
            order.remove(kb)
            order.insert(order.index(ka) + 1, kb)
    return order


class Graph:
    """Forward trace of an engine module at one input shape."""

    def __init__(self, owner, N, train, need_grad, layout=None):
        self.owner = owner
        self.N = N
        self.train = train
        self.need_grad = need_grad
        self.ops = []
        self.act_bufs = []
        self.act_size = 0
        self.stats_size = 0
        self.bns = []
        self.slopes = {}
        self.bn_by_mod = {}
        names = {}
        for pre, m in owner.named_modules():
            names[id(m)] = pre
        self.mod_names = names
        self.tensor_names = [k for k, _ in owner.named_parameters()] + \
                            [k for k, _ in owner.named_buffers()]
        self.tslot = {k: S_TENSOR0 + i for i, k in enumerate(self.tensor_names)}
        self.params = dict(owner.named_parameters())
        named = list(self.params)
        # the flat gradient's order: the parameter order, or a Trainer's layout (param_layout)
        self.param_names = list(layout) if layout is not None else named
        if sorted(self.param_names) != sorted(named):
            raise ValueError("parameter layout is not a permutation of the module's parameters")
        self.layout_pos = {k: i for i, k in enumerate(self.param_names)}
        self.param_shapes = {k: tuple(p.shape) for k, p in owner.named_parameters()}
        off = 0
        self.pgrad_off = {}
        for k in self.param_names:
            self.pgrad_off[k] = off
            off += self.params[k].numel()  # packed: the flat grad buffer in layout order
        self.pgrad_size = off
        self.used_params = set()
        # (tensor index of a's weight, of b's weight, a's weight bytes) of every sibling pair
        # emitted as ONE stacked GEMM: the plan reads b's rows through a's pointer, so it is
        # valid only while the two weights stay adjacent (Plan.stacking_holds)
        self.stacked = []

    # -- naming ------------------------------------------------------------------------
    def pname(self, mod, attr):
        pre = self.mod_names[id(mod)]
        return f"{pre}.{attr}" if pre else attr

    def tptr(self, mod, attr):
        return Ptr(self.tslot[self.pname(mod, attr)])

    def gptr(self, mod, attr):
        k = self.pname(mod, attr)
        self.used_params.add(k)
        return Ptr(S_PGRAD, self.pgrad_off[k] * 4)

    def wrep_ptr(self, mod, attr):
        """Replica 0 of a parameter's gradient in the S_WREP arena (L.WREP fp64 replicas of
        the flat gradient, stride pgrad_size doubles); folded into S_PGRAD by OP_SUM_REP."""
        k = self.pname(mod, attr)
        self.used_params.add(k)
        return Ptr(S_WREP, self.pgrad_off[k] * 8)

    # -- allocation ----------------------------------------------------------------------
    def act_buf(self, C, H, W, name):
        b = Buf(S_ACT, self.N, C, H, W, name, off=self.act_size)
        check_elems(b)
        self.act_size += (b.numel + ALIGN - 1) // ALIGN * ALIGN
        self.act_bufs.append(b)
        return b

    def stats_alloc(self, ndouble):
        """An accumulator of `ndouble` values, replicated L.STAT_REP times (isg.h)."""
        off = self.stats_size
        self.stats_size += (ndouble * L.STAT_REP + 7) // 8 * 8
        return off

    def bn_ref(self, bn, count):
        if id(bn) in self.bn_by_mod:
            raise ValueError("a BatchNorm module used twice in one trace is not supported")
        if not isinstance(bn, nn.BatchNorm2d) or bn.momentum is None or not bn.affine \
                or not bn.track_running_stats:
            raise NotImplementedError("BatchNorm2d(affine, momentum, tracked stats) only")
        ref = BNRef(bn, bn.num_features, count, self.stats_alloc(4 * bn.num_features), {
            "gamma": self.tptr(bn, "weight"), "beta": self.tptr(bn, "bias"),
            "rm": self.tptr(bn, "running_mean"), "rv": self.tptr(bn, "running_var"),
            "nbt": self.tptr(bn, "num_batches_tracked")})
        # finalised once per layer by an OP_BN_FINAL launch, or by every consumer
        ref.fin = _BN_FINAL or count >= _BN_FINAL_COUNT
        ref.gname = (bn, "weight")
        ref.bname = (bn, "bias")
        # finalised coefficients (isg_bn.coef): 8*C floats = 4*C doubles, 64-B aligned
        ref.coef_off = self.stats_size
        self.stats_size += (4 * bn.num_features + 7) // 8 * 8
        ref.coef_end = self.stats_size
        self.bns.append(ref)
        self.bn_by_mod[id(bn)] = ref
        return ref

    def slope_ref(self, prelu):
        if id(prelu) not in self.slopes:
            C = prelu.weight.numel()
            self.slopes[id(prelu)] = SlopeRef(prelu, C, self.stats_alloc(C),
                                              self.tslot[self.pname(prelu, "weight")])
        return self.slopes[id(prelu)]

    def act_of(self, act_mod):
        """(kind, SlopeRef|None) for an activation module of the reference."""
        if act_mod is None or isinstance(act_mod, nn.Identity):
            return "none", None
        if isinstance(act_mod, nn.ReLU):
            return "relu", None
        if isinstance(act_mod, nn.PReLU):
            return "prelu", self.slope_ref(act_mod)
        raise NotImplementedError(f"activation {type(act_mod).__name__} is not on the hot path")

    # -- ops -----------------------------------------------------------------------------
    def input(self, idx, C, H, W, grad):
        b = Buf(S_IN[idx], self.N, C, H, W, f"in{idx}")
        check_elems(b)
        return Value([Val(b, 0, C, grad=grad)])

    def keypoints(self, idx, N, nparts):
        return Keypoints(S_IN[idx], N, nparts)

    def kp_pool(self, kp, k, H, W, out, c0=0):
        """max_pool(k) of the keypoint heatmaps of an H x W image into out[:, c0:c0+parts]."""
        if H % k or W % k:
            raise RuntimeError(f"max_pool{k}: {H}x{W} not divisible")
        self.ops.append(KpPoolOp(self, kp, k, H, W, out, c0))
        return Value([Val(out, c0, kp.nparts, grad=False)])

    def conv(self, conv, x, bn=None, act="none", slope=None, name="", kp=None):
        """nn.Conv2d (dense or depthwise) on value x, optionally followed by BN/act
        applied lazily by the consumer. kp (Keypoints): the conv's input is cat(x, the
        keypoint heatmaps); x feeds the dense conv, the heatmap channels the keypoint
        stem kernels (isg_kp_stem)."""
        k, s, p, d = conv.kernel_size, conv.stride, conv.padding, conv.dilation
        if isinstance(p, str):
            raise NotImplementedError("string padding")
        H, W = x.H, x.W
        OH = (H + 2 * p[0] - d[0] * (k[0] - 1) - 1) // s[0] + 1
        OW = (W + 2 * p[1] - d[1] * (k[1] - 1) - 1) // s[1] + 1
        ckp = kp.nparts if kp is not None else 0
        if x.C + ckp != conv.in_channels:
            raise RuntimeError(f"{name}: expected {conv.in_channels} input channels, got {x.C + ckp}")
        if kp is not None and (conv.groups != 1 or x.grad):
            raise NotImplementedError("keypoint stem: dense conv of an input without gradient only")
        if conv.groups not in (1, conv.in_channels) or (conv.groups > 1 and
                                                         conv.in_channels != conv.out_channels):
            raise NotImplementedError("grouped conv other than depthwise")
        geom = dict(N=self.N, Ci=x.C, H=H, W=W, Co=conv.out_channels, OH=OH, OW=OW,
                    KH=k[0], KW=k[1], SH=s[0], SW=s[1], PH=p[0], PW=p[1], DH=d[0], DW=d[1],
                    groups=conv.groups)
        if kp is not None:
            geom["w_ci"] = conv.in_channels
        out = self.act_buf(conv.out_channels, OH, OW, name)
        bnr = self.bn_ref(bn, self.N * OH * OW) if bn is not None else None
        op = ConvOp(self, "conv", conv, geom, x, out, bnr)
        op.kp = kp
        self.ops.append(op)
        return Value([Val(out, 0, conv.out_channels, bnr, act, slope, grad=self.need_grad)])

    def conv_pair(self, ca, cb, x):
        """Two sibling Conv modules (1x1 conv + BatchNorm + act, segment.py:34-45) on the same
        input x as ONE stacked GEMM: weights [Wa; Wb] (contiguous in a Trainer's parameter
        layout, param_layout), output channels [0, Ca) to a's buffer and [Ca, Ca + Cb) to
        b's through two sinks (own bias and BatchNorm statistics); the backward is one
        K-stacked input gradient (Wa^T ga + Wb^T gb, no ACCUM pass) and one weight gradient
        over the stacked rows. Returns (value_a, value_b), or None when the pair does not
        qualify (then the caller emits two convs): not 1x1 / stride 1 / dense, no BN, or the
        weights not adjacent in the layout AND in memory (a module's own parameters are
        separate tensors)."""
        a, b = ca.conv, cb.conv
        for c in (a, b):
            if not (c.kernel_size == (1, 1) and c.stride == (1, 1) and c.padding == (0, 0)
                    and c.dilation == (1, 1) and c.groups == 1 and c.bias is not None):
                return None
        if a.in_channels != b.in_channels or a.in_channels != x.C:
            return None
        bna, bnb = getattr(ca, "bn", None), getattr(cb, "bn", None)
        if bna is None or bnb is None:
            return None
        ka, kb = self.pname(a, "weight"), self.pname(b, "weight")
        if self.layout_pos[kb] != self.layout_pos[ka] + 1:
            return None
        wa, wb = a.weight, b.weight
        if (wa.device != wb.device or not wa.is_contiguous() or not wb.is_contiguous()
                or wb.data_ptr() != wa.data_ptr() + wa.numel() * wa.element_size()):
            return None
        self.stacked.append((self.tensor_names.index(ka), self.tensor_names.index(kb),
                             wa.numel() * wa.element_size()))
        H, W = x.H, x.W
        geom = dict(N=self.N, Ci=x.C, H=H, W=W, Co=a.out_channels + b.out_channels, OH=H, OW=W,
                    KH=1, KW=1, SH=1, SW=1, PH=0, PW=0, DH=1, DW=1, groups=1)
        outs, vals = [], []
        for cm, c in ((ca, a), (cb, b)):
            out = self.act_buf(c.out_channels, H, W, self.mod_names.get(id(cm), "conv"))
            bnr = self.bn_ref(cm.bn, self.N * H * W)
            kind, slope = self.act_of(cm.act)
            outs.append((c, out, bnr))
            vals.append(Value([Val(out, 0, c.out_channels, bnr, kind, slope, grad=self.need_grad)]))
        self.ops.append(ConvPairOp(self, geom, x, outs))
        return vals[0], vals[1]

    def conv_transpose(self, ct, x, bn=None, act="none", slope=None, name=""):
        k, s, p = ct.kernel_size, ct.stride, ct.padding
        if ct.groups != 1 or ct.dilation != (1, 1) or any(ct.output_padding):
            raise NotImplementedError("convT: groups/dilation/output_padding")
        H, W = x.H, x.W
        OH = (H - 1) * s[0] - 2 * p[0] + k[0]
        OW = (W - 1) * s[1] - 2 * p[1] + k[1]
        geom = dict(N=self.N, Ci=ct.in_channels, H=H, W=W, Co=ct.out_channels, OH=OH, OW=OW,
                    KH=k[0], KW=k[1], SH=s[0], SW=s[1], PH=p[0], PW=p[1], DH=1, DW=1, groups=1)
        out = self.act_buf(ct.out_channels, OH, OW, name)
        if bn is None and ct.bias is not None:
            # the wgrad of a convT runs with swapped roles and cannot sum dY per output
            # channel: consumers' gradient sinks accumulate it here instead
            # (a BN-layout block: sinks add into its sum half, replica stride 4*C)
            out.need_sum = self.stats_alloc(4 * ct.out_channels)
        bnr = self.bn_ref(bn, self.N * OH * OW) if bn is not None else None
        op = ConvOp(self, "convT", ct, geom, x, out, bnr)
        self.ops.append(op)
        return Value([Val(out, 0, ct.out_channels, bnr, act, slope, grad=self.need_grad)])

    def head(self, ct, conv, x, name=""):
        """The mask head (segment.py:435-438, 504-505): ConvTranspose2d(16 -> 4, k8, s4, p2)
        then Conv2d(4 -> 1, 3x3, p1) as ONE fused op (isg_mask_head_*: the 4-channel
        intermediate never reaches HBM), or None when the modules / input do not have
        that exact shape (the caller then emits the two convolutions)."""
        if not (ct.in_channels == 16 and ct.out_channels == 4 and ct.kernel_size == (8, 8)
                and ct.stride == (4, 4) and ct.padding == (2, 2) and ct.groups == 1
                and ct.dilation == (1, 1) and not any(ct.output_padding)
                and conv.in_channels == 4 and conv.out_channels == 1
                and conv.kernel_size == (3, 3) and conv.stride == (1, 1)
                and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1
                and x.C == 16 and all(not s.virtual for s in x.segs)):
            return None
        out = self.act_buf(1, 4 * x.H, 4 * x.W, name)
        # the un-cropped intermediate on the ring outside the image, written by the forward
        # for the backward's 3x3 weight-gradient border term (isg.h isg_mask_head)
        ring = self.act_buf(1, 1, L.head_ring_floats(x.H, x.W), name + ".ring") \
            if self.need_grad else None
        op = HeadOp(self, ct, conv, x, out, ring)
        self.ops.append(op)
        return Value([Val(out, 0, 1, grad=self.need_grad)])

    def maxpool(self, x, k, out=None, c0=0, name=""):
        if x.H % k or x.W % k:
            raise RuntimeError(f"max_pool{k}: {x.H}x{x.W} not divisible (reference needs "
                               "H, W multiples of 16, SURVEY.md §0.5)")
        if out is None:
            out = self.act_buf(x.C, x.H // k, x.W // k, name)
        op = PoolOp(self, x, k, out, c0)
        self.ops.append(op)
        return Value([Val(out, c0, x.C, grad=x.grad)])

    @contextlib.contextmanager
    def side_branch(self):
        """Convolutions (and max-pools) emitted inside run on the executor's side stream in the forward
        pass (an independent residual branch: it reads only values produced before it
        and nothing reads its output until the block's tail), see _fork_branches."""
        n0 = len(self.ops)
        yield
        for op in self.ops[n0:]:
            if not isinstance(op, (ConvOp, PoolOp)):
                raise NotImplementedError("side branch: convolutions and max-pools only")
            op.side = True

    def tail(self, terms, act="none", slope=None, out=None, c0=0, name=""):
        """out = act(sum(terms)); terms = [(Value single-seg, up)]; BN'd terms must have
        act none (the activation of a Conv(act=None), segment.py:42)."""
        C = terms[0][0].C
        H, W = terms[0][0].H * (2 if terms[0][1] else 1), terms[0][0].W * (2 if terms[0][1] else 1)
        for v, up in terms:
            assert len(v.segs) == 1 and v.C == C
            assert v.H * (2 if up else 1) == H and v.W * (2 if up else 1) == W, (v.H, v.W, H, W)
            assert v.segs[0].act == "none"
        if out is None:
            out = self.act_buf(C, H, W, name)
        op = TailOp(self, [(v.segs[0], up) for v, up in terms], act, slope, out, c0)
        self.ops.append(op)
        return Value([Val(out, c0, C, grad=any(v.grad for v, _ in terms))])

    def materialize(self, v, out=None, c0=0, name=""):
        s = v.segs[0]
        assert len(v.segs) == 1
        term = Value([Val(s.buf, s.c0, s.C, s.bn, "none", None, s.grad)])
        return self.tail([(term, False)], s.act, s.slope, out, c0, name)


# ---------------------------------------------------------------------------------
# spec helpers
# BatchNorm coefficients. Default: every consumer evaluates them from the replicated fp64
# statistics itself (isg_bn.coef NULL; ISG_STAT_REP = 4 replicas, i.e. 8-16 loads per
# channel per workgroup), so no launch sits between a producer and its consumers.
# Measured on the bench step (profiles/r03h_bn_ab.txt, 2 x 200 steps each): 5.16 ms with
# one OP_BN_FINAL launch per BN point (140 per step, 16 replicas), 4.71 ms without them at
# 4 replicas (2 replicas 4.92: atomic contention in the producers; 8 replicas 4.82: more
# consumer reads; 16 replicas +0.8 ms, round 2). ISG_BN_FINAL=1 restores the launches.
_BN_FINAL = os.environ.get("ISG_BN_FINAL", "0") == "1"
# ISG_BN_FINAL_COUNT=n keeps one OP_BN_FINAL launch at BN points normalising >= n values
# (N*H*W). Default: none. (131072 — the stem and the 256^2 decoder — paid while thin_pw ran
# one-wave workgroups whose statistics atomics and reads piled on the same lines; after its
# four-wave form all-consumer-side measured 4.39 vs 4.41 ms/step, profiles/r03u_ab.txt.)
_BN_FINAL_COUNT = int(os.environ.get("ISG_BN_FINAL_COUNT", str(1 << 62)))


def _buf_range(buf):
    """(slot, lo, hi): the byte range of a whole arena buffer. A pool writes a channel slice
    of its output buffer, but a later record's pointer into that buffer names only where
    its own access STARTS (e.g. channel 0 of a concat it reads whole): any pointer into the
    buffer counts as touching the slice, so the join can never be placed after a reader
    whose start lies below the slice."""
    o = buf.ptr(0)
    return (o.slot, o.off, o.off + buf.numel * 4)


def _fork_pools(ol):
    """Max-pool forwards (and the keypoint heatmaps' pool) depend only on their input and
    nothing writes what they read or produce until their first consumer: fork each onto
    the executor's side stream and join right before the first later op that touches its
    output buffer (out_range = the whole buffer, _buf_range)."""
    recs = ol.recs
    pool = lambda r: r.kind in (L.OP_MAXPOOL_FWD, L.OP_KP_POOL) and getattr(r, "out_range", None) is not None
    for i, r in enumerate(recs):
        if not pool(r):
            continue
        slot, lo, hi = r.out_range
        for j in range(i + 1, len(recs)):
            # a pool right behind it into the same buffer (the stem's RGB max-pool and the
            # heatmaps' pool write disjoint channel slices of init_down) follows it on the
            # side stream: not a reader to join before
            if j == i + 1 and pool(recs[j]) and recs[j].out_range == r.out_range:
                continue
            if any(fs == slot and lo <= off < hi for _, fs, off in recs[j].fix):
                if j > i + 1:  # something to overlap with
                    r.flags |= Record.OPF_SIDE | Record.OPF_FORK_NOW
                    recs[j].flags |= Record.OPF_JOIN
                    _join_dep(recs[j], r)
                break


def _fork_branches(ol, side_recs):
    """Forward records of side-branch convolutions (Graph.side_branch) run on the
    executor's side stream, each forked at its place in the list (OPF_FORK_NOW: the side
    stream waits for everything issued on the main stream so far, i.e. the branch
    input). The first later main-stream record that reads any byte the branch writes —
    its output or its BN statistics/coefficients — joins the side stream. Forward only:
    backward sinks accumulate into shared gradient buffers."""
    if not side_recs:
        return
    recs = ol.recs
    pos = {id(r): i for i, r in enumerate(recs)}
    for r, ranges in side_recs:
        r.flags |= Record.OPF_SIDE | Record.OPF_FORK_NOW
    side_ids = {id(r) for r, _ in side_recs}
    for r, ranges in side_recs:
        for j in range(pos[id(r)] + 1, len(recs)):
            if id(recs[j]) in side_ids:
                continue
            if any(fs == slot and lo <= off < hi for _, fs, off in recs[j].fix
                   for slot, lo, hi in ranges):
                recs[j].flags |= Record.OPF_JOIN
                _join_dep(recs[j], r)
                break


def _join_dep(rec, side_rec):
    """Remember which forked record a join waits for (_join_exclusions)."""
    if not hasattr(rec, "join_deps"):
        rec.join_deps = set()
    rec.join_deps.add(id(side_rec))


def _join_exclusions(recs):
    """Narrow every join to the side work it depends on: a join made by _fork_pools /
    _fork_branches waits only for the side records up to the LAST one it reads (in list
    order), not for side records forked after that one — the executor's join would
    otherwise cover the side stream's whole tail, e.g. bottle1_1's 2x2 conv waiting for its
    own forked residual branch (pool + convm) when it only reads the stem's pools. The
    count of excluded (later) side records goes into the header flags' upper bits
    (api.cpp OPF_JOIN); joins without recorded dependencies wait for everything."""
    order = []
    for r in recs:
        if r.flags & Record.OPF_JOIN:
            r.flags &= (1 << Record.EXCL_SHIFT) - 1
            deps = getattr(r, "join_deps", None)
            pos = {i: k for k, i in enumerate(order)}
            if deps and all(d in pos for d in deps):
                excl = len(order) - 1 - max(pos[d] for d in deps)
                r.flags |= min(excl, Record.EXCL_MAX) << Record.EXCL_SHIFT
        if r.flags & Record.OPF_SIDE:
            order.append(id(r))


_FORK_DELAY = os.environ.get("ISG_FORK_DELAY", "1")  # 0 off, 1 the first fork group, 2 all


def _delay_forks(ol):
    """Capture a forward fork group behind the main-stream record that follows it (unless
    that record joins it). The graph runtime dispatches nodes in capture order and a node
    that waits on another queue waits for everything already dispatched there: with the
    side work captured first, the main stream's next node (at the step's start: the stem's
    first conv behind the replica memset and both stem pools) waited for the whole group
    (kernel trace: 40 us of the stem chain's start). Delaying a group only adds one main-
    stream dependency to it; nothing a main record between fork and join reads is written
    by the group (the join sits at its first reader, _fork_pools / _fork_branches)."""
    if _FORK_DELAY == "0":
        return
    recs, out, i, done = ol.recs, [], 0, False
    while i < len(recs):
        r = recs[i]
        if not r.flags & Record.OPF_SIDE or (done and _FORK_DELAY == "1"):
            out.append(r)
            i += 1
            continue
        j = i
        while j < len(recs) and recs[j].flags & Record.OPF_SIDE:
            j += 1
        done = True
        if j < len(recs) and not recs[j].flags & Record.OPF_JOIN:
            out.append(recs[j])
            out += recs[i:j]
            i = j + 1
        else:
            out += recs[i:j]
            i = j
    recs[:] = out


def _fork_late_wgrads(recs, late):
    """The executor defers side-stream weight gradients in batches until a join; at the end
    of the backward that parks the last batch (and the stem's own weight gradients, whose
    dy is ready before the stem's input-gradient chain runs) behind the whole stem chain.
    Fork the pending batch where the stem's backward begins, and each stem weight gradient
    at its place (OPF_FORK_NOW), so they overlap the stem's input-gradient kernels."""
    if not late:
        return
    tag = late.rstrip(".")
    first_late = next((i for i, r in enumerate(recs) if tag in r.label), None)
    if first_late is None:
        return
    prev = [r for r in recs[:first_late] if r.flags & Record.OPF_SIDE]
    if prev:
        prev[-1].flags |= Record.OPF_FORK_NOW
    for r in recs[first_late:]:
        if r.flags & Record.OPF_SIDE:
            r.flags |= Record.OPF_FORK_NOW
    # a stem weight gradient right behind its own input gradient moves in front of it: its
    # operands (dy, the forward input) are ready, so it forks before that kernel instead of
    # behind it (a weight gradient reads nothing the input gradient writes)
    for i in range(first_late, len(recs) - 1):
        a, b = recs[i], recs[i + 1]
        if (a.kind == L.OP_CONV_DGRAD and b.kind == L.OP_CONV_WGRAD and a.label.startswith("dx_")
                and b.label == "dw_" + a.label[3:]):
            recs[i], recs[i + 1] = b, a


def _trailing_on_main(recs):
    """Side records after the backward's last main-stream record (the stem's layer-1 weight
    gradients, behind the last input gradient) overlap nothing on the main stream, which then
    only waits at the final join, while on the side stream they queue behind every weight
    gradient forked before them: run them on the main stream instead (round 6 kernel trace:
    the main stream idled 161 us before the step tail)."""
    i = len(recs)
    while i > 0 and recs[i - 1].flags & Record.OPF_SIDE:
        i -= 1
    for r in recs[i:]:
        r.flags &= ~(Record.OPF_SIDE | Record.OPF_FORK_NOW)


def _fold_tails(g):
    """Residual tails folded into their first consumer: a tail
    out = act(BN(y) + x) (segment.py:75-77, 107-109, 259: BatchNorm'd raw conv output plus a
    materialised value, no upsampling) whose output is read FIRST by the very next op, a
    1x1 stride-1 conv on exactly that value, stops being a launch of its own:
      forward  — the conv reads act(BN(y) + x) on load (isg_vseg residual form) and its
                 first row block writes the materialised output on the way (vtensor.mat),
                 which every later reader (the next tail's residual term, skips, the
                 weight gradient) still finds in the tail's buffer;
      backward — the conv's input gradient, the last contribution to dL/d out, carries the
                 tail's backward in its sink (ACTBWD residual form: + the gradient already
                 accumulated for out, act' at BN(y) + x, BatchNorm-backward sums of y, the
                 PReLU slope gradient, and the residual term's gradient as a second
                 output), decided in ConvOp.bwd (falls back to the tail's own launch when
                 the gradient bookkeeping does not allow it).
    Train mode, and forward-only eval plans (infer: the BN-folded network's tails add a
    plain conv output, read as an identity-BN segment with the tail's activation);
    ISG_NO_TAIL_FOLD=1 off."""
    if os.environ.get("ISG_NO_TAIL_FOLD", "0") == "1" or (not g.train and g.need_grad):
        return
    ops = g.ops
    for i, t in enumerate(ops):
        if not isinstance(t, TailOp) or len(t.terms) != 2:
            continue
        (y, upy), (r, upr) = t.terms
        C = t.out.C
        # the residual: a materialised value, or a second BatchNorm'd conv output (the
        # BottleneckDown2 / BottleneckDim_Res tails, segment.py:147-148, 202-207)
        r_ok = not r.virtual or (g.train and r.bn is not None and r.act == "none" and r.c0 == 0
                                 and r.C == r.buf.C and r.buf is not y.buf)
        # y: a BatchNorm'd raw conv output, or (BN folded into the conv) a plain one under
        # the tail's activation (the residual form is a BN_FWD segment either way)
        y_ok = y.act == "none" and (y.bn is not None or (not y.virtual and t.act != "none"))
        if upy or upr or not y_ok or not r_ok or t.c0 != 0:
            continue
        if t.out.slot != S_ACT or y.C != C or r.C != C or y.c0 != 0 or y.buf.C != C:
            continue
        if (t.out.H * t.out.W) % 4 or C % 4 or C > 128:
            continue
        # the side-branch ops forked right after the tail (BottleneckUp_Res's conv2,
        # segment.py:230-236, reads the block input beside the main chain): each one either
        # does not read the tail's output or is a 1x1 conv folding the tail on its own load
        # (no materialised output); then the main-stream 1x1 that writes it
        side = []
        j = i + 1
        while j < len(ops) and getattr(ops[j], "side", False):
            if any(v.buf is t.out for v in ops[j].x.segs):
                side.append(ops[j])
            j += 1
        if j >= len(ops) or not all(_fold_reader_ok(o, t) for o in side + [ops[j]]):
            continue
        if r.virtual and isinstance(ops[j], ConvPairOp):
            continue  # the residual's own BatchNorm needs one sink (pw_gemm.hip host check)
        c = ops[j]
        t.fwd_folded = True
        for o in side:
            o.res_in, o.res_mat = t, False
        c.res_in, c.res_mat = t, True
        # the backward: the first reader's input gradient is the last contribution
        (side[0] if side else c).res_tail = t


def _fold_reader_ok(c, t):
    """A reader of a residual tail's output that can take the tail's forward on its input
    load (and, as the last gradient contributor, its backward in the input-gradient sink):
    a dense 1x1 stride-1 conv, or a stacked sibling pair of them (Graph.conv_pair), on exactly
    that value (pw_gemm.hip: 16-B rows, K, M <= 128)."""
    if not isinstance(c, (ConvOp, ConvPairOp)):
        return False
    ge = c.geom
    if isinstance(c, ConvOp) and not (c.kind == "conv" and c.kp is None):
        return False
    if not (ge["KH"] == 1 and ge["KW"] == 1 and ge["SH"] == 1 and ge["SW"] == 1
            and ge["PH"] == 0 and ge["PW"] == 0 and ge["DH"] == 1 and ge["DW"] == 1
            and ge["groups"] == 1 and "w_ci" not in ge):
        return False
    if len(c.x.segs) != 1:
        return False
    xv = c.x.segs[0]
    if xv.buf is not t.out or xv.c0 != 0 or xv.C != t.out.C or xv.virtual:
        return False
    return ge["Co"] <= 128 and ge["Co"] % 4 == 0


def sinks_spec(sinks):
    """isg_sinks spec from sink specs."""
    return {"s": sinks, "nsink": len(sinks)}


def bn_spec(bnr, train, coef=True):
    if bnr is None:
        return {"train": 1}
    n = bnr.names
    s = {"gamma": n["gamma"], "beta": n["beta"], "running_mean": n["rm"],
         "running_var": n["rv"], "stats": Ptr(S_STATS, bnr.stats_off * 8), "C": bnr.C,
         "train": 1 if train else 0, "count": float(bnr.count), "eps": float(bnr.mod.eps)}
    if train and coef and bnr.fin:
        # consumers read the coefficients OP_BN_FINAL wrote (forward half after the
        # producing conv, backward half after the op that completes gsum/gxsum)
        s["coef"] = Ptr(S_STATS, bnr.coef_off * 8)
    return s


def bn_final_record(bnrs, bwd):
    items = [bn_spec(b, True) for b in bnrs]
    return Record(L.OP_BN_FINAL, L.ListRec, {"n": len(items), "pad_": 1 if bwd else 0}, L.Bn,
                  items, label=("bn_final_bwd " if bwd else "bn_final ") +
                  ",".join(str(b.C) for b in bnrs))


def fwd_seg(val, train):
    s = {"p": val.buf.ptr(val.c0), "n_stride": val.buf.n_stride, "C": val.C,
         "xform": L.XF_BN_FWD if val.virtual else L.XF_PLAIN, "act": L.ACT[val.act]}
    if val.virtual:
        s["bn"] = bn_spec(val.bn, train) if val.bn is not None else {"train": 1}
        if val.slope is not None:
            s["slope"] = Ptr(val.slope.slot)
    return s


def vtensor(segs, N, H, W):
    return {"s": segs, "nseg": len(segs), "N": N, "H": H, "W": W}


class GradState:
    """Backward bookkeeping: gradient buffers in the grad arena."""

    def __init__(self, g):
        self.g = g
        self.size = 0
        self.D = {}       # id(buf) -> grad Buf (materialised values / plain raws)
        self.G = {}       # id(raw buf) -> g Buf (dL/d BN-output of a virtual value)
        self.inited = {}  # id(buf) -> set of (c0, C)
        self.external = {}  # id(buf) -> Buf (e.g. dlogits slot)
        self.pending_final = []  # BNs whose gsum/gxsum the last op completed

    def alloc(self, like, name):
        b = Buf(S_GRAD, like.N, like.C, like.H, like.W, name, off=self.size)
        check_elems(b)
        self.size += (b.numel + ALIGN - 1) // ALIGN * ALIGN
        return b

    def dbuf(self, buf):
        if id(buf) in self.external:
            return self.external[id(buf)]
        if id(buf) not in self.D:
            self.D[id(buf)] = self.alloc(buf, "d_" + buf.name)
        return self.D[id(buf)]

    def has_grad(self, buf, c0, C):
        return id(buf) in self.external or (c0, C) in self.inited.get(id(buf), set())

    def mark(self, buf, c0, C):
        first = (c0, C) not in self.inited.setdefault(id(buf), set())
        self.inited[id(buf)].add((c0, C))
        return first

    def sink_for(self, val, c0_glob, train):
        """Sink that receives dL/d(val) for channels [c0_glob, c0_glob+val.C) of a kernel's
        output rows."""
        if not val.grad:
            return {"c0": c0_glob, "C": val.C, "mode": L.SINK_NONE}
        if val.virtual:
            assert id(val.buf) not in self.G, f"virtual value {val.buf.name} consumed twice"
            gb = self.alloc(val.buf, "g_" + val.buf.name)
            self.G[id(val.buf)] = gb
            s = {"p": gb.ptr(val.c0), "n_stride": gb.n_stride, "c0": c0_glob, "C": val.C,
                 "mode": L.SINK_ACTBWD, "act": L.ACT[val.act],
                 "y": val.buf.ptr(val.c0), "y_n_stride": val.buf.n_stride,
                 "bn": bn_spec(val.bn, train) if val.bn is not None else {"train": 1}}
            if val.slope is not None:
                s["slope"] = Ptr(val.slope.slot)
                s["slope_grad"] = Ptr(S_STATS, val.slope.acc_off * 8)
                val.slope.used_in_bwd = True
            if val.bn is not None and val.bn.fin:
                self.pending_final.append(val.bn)
            return s
        d = self.dbuf(val.buf)
        first = self.mark(val.buf, val.c0, val.C)
        s = {"p": d.ptr(val.c0), "n_stride": d.n_stride, "c0": c0_glob, "C": val.C,
             "mode": L.SINK_STORE if first else L.SINK_ACCUM}
        ns = getattr(val.buf, "need_sum", None)
        if ns is not None:
            assert val.c0 == 0 and val.C == val.buf.C
            s["stats"] = Ptr(S_STATS, ns * 8)
        return s

    def dy_seg(self, buf, bnr, train):
        """The gradient w.r.t. a conv's raw output `buf`, as a virtual segment, or None
        when nothing downstream produced one (the output does not reach the loss)."""
        if bnr is not None:
            if id(buf) not in self.G:
                return None
            gb = self.G[id(buf)]
            return {"p": gb.ptr(), "y": buf.ptr(), "n_stride": gb.n_stride,
                    "y_n_stride": buf.n_stride, "C": buf.C, "xform": L.XF_BN_BWD,
                    "bn": bn_spec(bnr, train)}
        if not self.has_grad(buf, 0, buf.C):
            return None
        d = self.dbuf(buf)
        return {"p": d.ptr(), "n_stride": d.n_stride, "C": buf.C, "xform": L.XF_PLAIN}


# ---------------------------------------------------------------------------------
class _ResFold:
    """A residual tail folded into a 1x1 conv (ConvOp) or stacked sibling pair (ConvPairOp):
    read on the input load (res_in; res_mat: this op writes the tail's buffer), run in the
    input gradient's sink (res_tail). _fold_tails sets them."""
    res_in, res_mat, res_tail = None, False, None

    def _res_input(self):
        """The forward input of a folded tail act(BN(y) + x): one BN_FWD segment of y with
        the residual x and the tail's activation, and the tail's buffer as `mat`."""
        g, t = self.g, self.res_in
        (y, _), (r, _) = t.terms
        seg = fwd_seg(Val(y.buf, y.c0, y.C, y.bn, t.act, t.slope), g.train)
        seg["y"] = r.buf.ptr(r.c0)
        seg["y_n_stride"] = r.buf.n_stride
        vt = vtensor([seg], g.N, self.geom["H"], self.geom["W"])
        if self.res_mat:
            vt["mat"] = t.out.ptr()
            vt["mat_n_stride"] = t.out.n_stride
        if r.bn is not None:  # a BatchNorm'd residual: act(BN(y) + BN2(r))
            vt["rbn"] = bn_spec(r.bn, g.train)
        return vt

    def _res_sink(self, gs):
        """The input-gradient sink that also runs the folded tail's backward (isg.h ACTBWD
        residual form), or None when the gradient bookkeeping does not allow it (then the
        tail runs its own backward): dL/d out must be this conv's input gradient plus at
        most what later consumers accumulated over the whole buffer (`old`); the residual
        term's gradient goes out as the second output (p2: STORE when it is the first
        contribution, else ACCUM)."""
        g, t = self.g, self.res_tail
        (y, _), (r, _) = t.terms
        C = t.out.C
        ini = gs.inited.get(id(t.out), set())
        if id(t.out) in gs.external or ini - {(0, C)} or id(y.buf) in gs.G:
            return None
        if r.bn is not None and id(r.buf) in gs.G:
            return None
        gb = gs.alloc(y.buf, "g_" + y.buf.name)
        gs.G[id(y.buf)] = gb
        s = {"p": gb.ptr(), "n_stride": gb.n_stride, "c0": 0, "C": C, "mode": L.SINK_ACTBWD,
             "act": L.ACT[t.act], "y": y.buf.ptr(), "y_n_stride": y.buf.n_stride,
             "bn": bn_spec(y.bn, g.train), "r": r.buf.ptr(r.c0), "r_n_stride": r.buf.n_stride}
        if t.slope is not None:
            s["slope"] = Ptr(t.slope.slot)
            s["slope_grad"] = Ptr(S_STATS, t.slope.acc_off * 8)
            t.slope.used_in_bwd = True
        if (0, C) in ini:
            d = gs.dbuf(t.out)
            s["old"] = d.ptr()
            s["old_n_stride"] = d.n_stride
        if r.bn is not None:
            # a BatchNorm'd residual: its BN-output gradient is the same g (the tail's
            # backward gives both BN terms one buffer), its backward sums go to its own stats
            gs.G[id(r.buf)] = gb
            s["rbn"] = bn_spec(r.bn, g.train)
            if r.bn.fin:
                gs.pending_final.append(r.bn)
        elif r.grad:
            db = gs.dbuf(r.buf)
            first = gs.mark(r.buf, r.c0, r.C)
            s["p2"] = db.ptr(r.c0)
            s["p2_n_stride"] = db.n_stride
            s["p2_accum"] = 0 if first else 1
        if y.bn.fin:
            gs.pending_final.append(y.bn)
        t.bwd_folded = True
        return s


class ConvOp(_ResFold):
    def __init__(self, g, kind, mod, geom, x, out, bnr):
        self.g, self.kind, self.mod, self.geom, self.x, self.out, self.bnr = g, kind, mod, geom, x, out, bnr
        self.kp = None

    def _kp_spec(self):
        """isg_kp_stem fields shared by the forward and weight-gradient records."""
        ge = dict(self.geom)
        ge["Ci"] = ge.pop("w_ci")
        return dict(self.kp.spec(), c_kp0=self.x.C, g=ge)

    def _cost(self):
        """(flops, bytes of x, bytes of y, bytes of w) — algorithmic, fp32, each read once."""
        ge = self.geom
        N = ge["N"]
        if self.kind == "convT":
            macs = N * ge["H"] * ge["W"] * ge["Ci"] * ge["Co"] * ge["KH"] * ge["KW"]
        elif ge["groups"] > 1:
            macs = N * ge["OH"] * ge["OW"] * ge["Co"] * ge["KH"] * ge["KW"]
        else:
            macs = N * ge["OH"] * ge["OW"] * ge["Co"] * ge["Ci"] * ge["KH"] * ge["KW"]
        xb = 4 * N * ge["Ci"] * ge["H"] * ge["W"]
        yb = 4 * N * ge["Co"] * ge["OH"] * ge["OW"]
        wb = 4 * self.mod.weight.numel()
        return 2 * macs, xb, yb, wb

    def fwd(self, ops):
        g = self.g
        segs = [fwd_seg(v, g.train) for v in self.x.segs]
        sink = {"p": self.out.ptr(), "n_stride": self.out.n_stride, "c0": 0, "C": self.out.C,
                "mode": L.SINK_STORE}
        if self.mod.bias is not None:
            sink["bias"] = g.tptr(self.mod, "bias")
        if self.bnr is not None and g.train:
            sink["stats"] = Ptr(S_STATS, self.bnr.stats_off * 8)
        ge = self.geom
        a = self._res_input() if self.res_in is not None else vtensor(segs, g.N, ge["H"], ge["W"])
        rec = {"g": ge, "a": a, "w": g.tptr(self.mod, "weight"), "out": sinks_spec([sink])}
        kind = L.OP_CONVT_FWD if self.kind == "convT" else L.OP_CONV_FWD
        fl, xb, yb, wb = self._cost()
        if self.res_in is not None:
            xb *= 3 if self.res_mat else 2  # BN'd y and the residual read (+ the output written)
        ops.add(Record(kind, L.ConvRec, rec, label=self.out.name, flops=fl, nbytes=xb + yb + wb))
        if self.kp is not None:
            ks = dict(self._kp_spec(), w=g.tptr(self.mod, "weight"), y=self.out.ptr(),
                      y_n_stride=self.out.n_stride)
            if self.bnr is not None and g.train:
                ks["stats"] = Ptr(S_STATS, self.bnr.stats_off * 8)
            ops.add(Record(L.OP_KP_STEM_FWD, L.KpStem, ks, label="kp_" + self.out.name,
                           nbytes=2 * yb))

    def bwd(self, ops, gs):
        g = self.g
        ge = self.geom
        dy = gs.dy_seg(self.out, self.bnr, g.train)
        if dy is None:
            return
        fl, xb, yb, wb = self._cost()
        dyb = yb * (2 if dy["xform"] == L.XF_BN_BWD else 1)  # g and y for BN backward
        dyv = vtensor([dy], g.N, ge["OH"], ge["OW"])
        if (self.kind == "conv" and ge["groups"] > 1 and self.x.grad and self.kp is None
                and len(self.x.segs) == 1 and os.environ.get("ISG_NO_DW_FUSE", "0") != "1"):
            # a depthwise layer's input and weight gradients as ONE op on the main stream
            # (isg_depthwise_bwd: the dy tile staged once; the weight gradient is no
            # side-stream node of its own)
            sk = sinks_spec([gs.sink_for(self.x.segs[0], 0, g.train)])
            xv = vtensor([fwd_seg(self.x.segs[0], g.train)], g.N, ge["H"], ge["W"])
            rec = {"g": ge, "dy": dyv, "w": g.tptr(self.mod, "weight"), "dx": sk, "x": xv,
                   "dw": g.wrep_ptr(self.mod, "weight"), "rep_stride": g.pgrad_size,
                   "nrep": L.WREP}
            if self.mod.bias is not None and self.bnr is None:
                rec["dbias"] = g.wrep_ptr(self.mod, "bias")
            ops.add(Record(L.OP_DW_BWD, L.DwBwdRec, rec, label="dx_" + self.out.name,
                           flops=2 * fl, nbytes=2 * dyb + 2 * xb + wb))
            if self.mod.bias is not None and self.bnr is not None:
                gs.bias_from_bn.append((self.mod, self.bnr))
            return
        # ---- input gradient
        if self.x.grad:
            rs = self._res_sink(gs) if self.res_tail is not None else None
            sinks = [rs] if rs is not None else []
            c = 0
            for v in ([] if rs is not None else self.x.segs):
                sinks.append(gs.sink_for(v, c, g.train))
                c += v.C
            sk = sinks_spec(sinks)
            w = g.tptr(self.mod, "weight")
            if self.kind == "convT":
                # dx_T = conv(dy_T, W) with the forward conv's stride/pad/kernel
                tg = dict(N=g.N, Ci=ge["Co"], H=ge["OH"], W=ge["OW"], Co=ge["Ci"], OH=ge["H"],
                          OW=ge["W"], KH=ge["KH"], KW=ge["KW"], SH=ge["SH"], SW=ge["SW"],
                          PH=ge["PH"], PW=ge["PW"], DH=1, DW=1, groups=1)
                ops.add(Record(L.OP_CONV_FWD, L.ConvRec, {"g": tg, "a": dyv, "w": w, "out": sk},
                               label="dx_" + self.out.name, flops=fl, nbytes=dyb + xb + wb))
            else:
                ops.add(Record(L.OP_CONV_DGRAD, L.ConvRec, {"g": ge, "a": dyv, "w": w, "out": sk},
                               label="dx_" + self.out.name, flops=fl, nbytes=dyb + xb + wb))
        # ---- weight / bias gradient
        xsegs = [fwd_seg(v, g.train) for v in self.x.segs]
        dw = g.wrep_ptr(self.mod, "weight")
        rep = {"rep_stride": g.pgrad_size, "nrep": L.WREP}
        has_bias = self.mod.bias is not None
        if self.kind == "convT":
            tg = dict(N=g.N, Ci=ge["Co"], H=ge["OH"], W=ge["OW"], Co=ge["Ci"], OH=ge["H"],
                      OW=ge["W"], KH=ge["KH"], KW=ge["KW"], SH=ge["SH"], SW=ge["SW"],
                      PH=ge["PH"], PW=ge["PW"], DH=1, DW=1, groups=1)
            ops.add(Record(L.OP_CONV_WGRAD, L.WgradRec,
                           {"g": tg, "dy": vtensor(xsegs, g.N, ge["H"], ge["W"]), "x": dyv,
                            "dw": dw, **rep}, label="dw_" + self.out.name, flops=fl,
                           nbytes=dyb + xb + wb))
            if has_bias and self.bnr is None:
                gs.bias_sums.append((self.mod, self.out, dy))
        else:
            rec = {"g": ge, "dy": dyv, "x": vtensor(xsegs, g.N, ge["H"], ge["W"]), "dw": dw, **rep}
            if has_bias and self.bnr is None:
                rec["dbias"] = g.wrep_ptr(self.mod, "bias")
            ops.add(Record(L.OP_CONV_WGRAD, L.WgradRec, rec, label="dw_" + self.out.name,
                           flops=fl, nbytes=dyb + xb + wb))
            if self.kp is not None:
                ops.add(Record(L.OP_KP_STEM_WGRAD, L.KpStem,
                               dict(self._kp_spec(), dy=dyv, dw=dw, **rep),
                               label="dwkp_" + self.out.name))
        if has_bias and self.bnr is not None:
            gs.bias_from_bn.append((self.mod, self.bnr))


class ConvPairOp(_ResFold):
    """Two sibling 1x1 convs on one input as one stacked GEMM (Graph.conv_pair)."""

    def __init__(self, g, geom, x, outs):
        self.g, self.geom, self.x, self.outs = g, geom, x, outs  # outs: [(conv, buf, bnr)] x2
        self.bnr = None
        self.bnrs = [bnr for _, _, bnr in outs]
        self.label = "+".join(buf.name for _, buf, _ in outs)

    def _cost(self, co):
        ge = self.geom
        P = ge["N"] * ge["H"] * ge["W"]
        return 2 * P * co * ge["Ci"], 4 * P * ge["Ci"], 4 * P * co, 4 * co * ge["Ci"]

    def fwd(self, ops):
        g = self.g
        segs = [fwd_seg(v, g.train) for v in self.x.segs]
        sinks, c0 = [], 0
        for c, buf, bnr in self.outs:
            sk = {"p": buf.ptr(), "n_stride": buf.n_stride, "c0": c0, "C": buf.C,
                  "mode": L.SINK_STORE, "bias": g.tptr(c, "bias")}
            if g.train:
                sk["stats"] = Ptr(S_STATS, bnr.stats_off * 8)
            sinks.append(sk)
            c0 += buf.C
        ge = self.geom
        fl, xb, yb, wb = self._cost(ge["Co"])
        if self.res_in is not None:
            xb *= 3 if self.res_mat else 2  # BN'd y and the residual read (+ the output written)
        a = self._res_input() if self.res_in is not None else vtensor(segs, g.N, ge["H"], ge["W"])
        ops.add(Record(L.OP_CONV_FWD, L.ConvRec,
                       {"g": ge, "a": a,
                        "w": g.tptr(self.outs[0][0], "weight"), "out": sinks_spec(sinks)},
                       label=self.label, flops=fl, nbytes=xb + yb + wb))

    def bwd(self, ops, gs):
        g = self.g
        ge = self.geom
        parts = [(c, buf, bnr, gs.dy_seg(buf, bnr, g.train)) for c, buf, bnr in self.outs]
        live = [p for p in parts if p[3] is not None]
        if not live:
            return
        for c, buf, bnr, _ in live:
            gs.bias_from_bn.append((c, bnr))
        if len(live) == 1:  # one branch reaches the loss: its own conv's weight rows
            c, buf, bnr, dy = live[0]
            segs, w, dwp = [dy], g.tptr(c, "weight"), g.wrep_ptr(c, "weight")
            co = buf.C
        else:
            segs = [p[3] for p in parts]
            w = g.tptr(self.outs[0][0], "weight")
            dwp = g.wrep_ptr(self.outs[0][0], "weight")
            g.wrep_ptr(self.outs[1][0], "weight")  # its rows follow (param_layout)
            co = ge["Co"]
        sg = dict(ge, Co=co)
        fl, xb, yb, wb = self._cost(co)
        dyb = 2 * yb  # g and the saved y of the BatchNorm backward
        dyv = vtensor(segs, g.N, ge["H"], ge["W"])
        label = "+".join(p[1].name for p in live)
        if self.x.grad:
            rs = self._res_sink(gs) if self.res_tail is not None else None
            sinks, c = ([rs] if rs is not None else []), 0
            for v in ([] if rs is not None else self.x.segs):
                sinks.append(gs.sink_for(v, c, g.train))
                c += v.C
            ops.add(Record(L.OP_CONV_DGRAD, L.ConvRec,
                           {"g": sg, "a": dyv, "w": w, "out": sinks_spec(sinks)},
                           label="dx_" + label, flops=fl, nbytes=dyb + xb + wb))
        xsegs = [fwd_seg(v, g.train) for v in self.x.segs]
        ops.add(Record(L.OP_CONV_WGRAD, L.WgradRec,
                       {"g": sg, "dy": dyv, "x": vtensor(xsegs, g.N, ge["H"], ge["W"]),
                        "dw": dwp, "rep_stride": g.pgrad_size, "nrep": L.WREP},
                       label="dw_" + label, flops=fl, nbytes=dyb + xb + wb))


class HeadOp:
    """Fused mask head (Graph.head): one forward and one backward record."""

    def __init__(self, g, ct, conv, x, out, ring=None):
        self.g, self.ct, self.conv, self.x, self.out, self.ring = g, ct, conv, x, out, ring

    def _spec(self):
        g = self.g
        segs = [fwd_seg(v, g.train) for v in self.x.segs]
        s = {"x": vtensor(segs, g.N, self.x.H, self.x.W), "w1": g.tptr(self.ct, "weight"),
             "w2": g.tptr(self.conv, "weight"), "N": g.N, "Hi": self.x.H, "Wi": self.x.W}
        if self.ring is not None:
            s["ring"] = self.ring.ptr()
        if self.ct.bias is not None:
            s["b1"] = g.tptr(self.ct, "bias")
        if self.conv.bias is not None:
            s["b2"] = g.tptr(self.conv, "bias")
        return s

    def _cost(self):
        """(flops, bytes) of the forward: convT 2*16*4*64 MAC per input pixel, the 3x3
        2*36 per output pixel; input read once, logits written once."""
        g = self.g
        q = g.N * self.x.H * self.x.W
        p = 16 * q
        return 2 * (16 * 4 * 64 * q + 36 * p), 4 * (16 * q + p)

    def fwd(self, ops):
        s = dict(self._spec(), out=self.out.ptr(), out_n_stride=self.out.n_stride)
        fl, nb = self._cost()
        ops.add(Record(L.OP_HEAD_FWD, L.MaskHead, s, label=self.out.name, flops=fl, nbytes=nb))

    def bwd(self, ops, gs):
        g = self.g
        dy = gs.dy_seg(self.out, None, g.train)
        if dy is None:
            return
        s = dict(self._spec(), dout=dy["p"], dout_n_stride=dy["n_stride"],
                 rep_stride=g.pgrad_size, nrep=L.WREP)
        if self.x.grad:
            sinks, c = [], 0
            for v in self.x.segs:
                sinks.append(gs.sink_for(v, c, g.train))
                c += v.C
            s["dx"] = sinks_spec(sinks)
        else:
            s["dx"] = {"nsink": 0}
        s["dw1"] = g.wrep_ptr(self.ct, "weight")
        s["dw2"] = g.wrep_ptr(self.conv, "weight")
        if self.ct.bias is not None:
            s["db1"] = g.wrep_ptr(self.ct, "bias")
        if self.conv.bias is not None:
            s["db2"] = g.wrep_ptr(self.conv, "bias")
        # the convT weight gradient's per-workgroup partials go to a slab folded into the
        # replicas by a side-stream op (isg.h isg_mask_head.dw1_part): the kernel's tail was
        # its 4096 fp64 atomics per workgroup
        nslab = L.head_part_floats(g.N, self.x.H, self.x.W)
        if nslab > 0:
            part = gs.alloc(Buf(S_GRAD, 1, 1, 1, nslab, "head_dw1_part"), "head_dw1_part")
            s["dw1_part"] = part.ptr()
        fl, nb = self._cost()
        # algorithmic: input gradient + both weight gradients = 2x the forward (SURVEY
        # §8d). The kernel does not recompute the 4-channel intermediate: the 3x3's weight
        # gradient comes from W1·Z' plus the forward's border ring (isg.h ISG_HEAD_RING).
        ops.add(Record(L.OP_HEAD_BWD, L.MaskHead, s, label="d_" + self.out.name,
                       flops=2 * fl, nbytes=nb + 4 * 16 * g.N * self.x.H * self.x.W))
        if "dw1_part" in s:
            ops.add(Record(L.OP_HEAD_FOLD, L.MaskHead, s, label="fold_" + self.out.name))


class KpPoolOp:
    """max_pool(k) of the keypoint heatmaps (segment.py:31 on the heatmap channels)."""

    def __init__(self, g, kp, k, H, W, out, c0):
        self.g, self.kp, self.k, self.H, self.W, self.out, self.c0 = g, kp, k, H, W, out, c0

    def fwd(self, ops):
        g = self.g
        r = Record(L.OP_KP_POOL, L.KpStem,
                   dict(self.kp.spec(), g={"N": g.N, "H": self.H, "W": self.W}, k=self.k,
                        out=self.out.ptr(self.c0), out_n_stride=self.out.n_stride),
                   label="kp_pool_" + self.out.name,
                   nbytes=4 * g.N * self.kp.nparts * self.out.H * self.out.W)
        r.out_range = _buf_range(self.out)  # for _fork_pools
        ops.add(r)

    def bwd(self, ops, gs):
        return  # keypoints carry no gradient


class PoolOp:
    def __init__(self, g, x, k, out, c0):
        self.g, self.x, self.k, self.out, self.c0 = g, x, k, out, c0

    def fwd(self, ops):
        g = self.g
        segs = [fwd_seg(v, g.train) for v in self.x.segs]
        r = Record(L.OP_MAXPOOL_FWD, L.PoolRec,
                   {"x": vtensor(segs, g.N, self.x.H, self.x.W), "k": self.k,
                    "out": self.out.ptr(self.c0), "out_ns": self.out.n_stride},
                   label=self.out.name,
                   nbytes=4 * g.N * self.x.C * (self.x.H * self.x.W + self.out.H * self.out.W))
        r.out_range = _buf_range(self.out)  # for _fork_pools
        ops.add(r)

    def bwd(self, ops, gs):
        g = self.g
        if not self.x.grad or not gs.has_grad(self.out, self.c0, self.x.C):
            return
        d = gs.dbuf(self.out)
        sinks = []
        c = 0
        for v in self.x.segs:
            if v.virtual:
                raise NotImplementedError("max-pool of a virtual value needs materialisation")
            sinks.append(gs.sink_for(v, c, g.train))
            c += v.C
        segs = [fwd_seg(v, g.train) for v in self.x.segs]
        ops.add(Record(L.OP_MAXPOOL_BWD, L.PoolRec,
                       {"x": vtensor(segs, g.N, self.x.H, self.x.W), "k": self.k,
                        "dout": d.ptr(self.c0), "dout_ns": d.n_stride,
                        "dx": sinks_spec(sinks)}, label="dx_" + self.out.name,
                       nbytes=4 * g.N * self.x.C * (2 * self.x.H * self.x.W + self.out.H * self.out.W)))


class TailOp:
    def __init__(self, g, terms, act, slope, out, c0):
        self.g, self.terms, self.act, self.slope, self.out, self.c0 = g, terms, act, slope, out, c0

    def spec(self):
        g = self.g
        C = self.terms[0][0].C
        t = {"term": [fwd_seg(v, g.train) for v, _ in self.terms],
             "up": [1 if up else 0 for _, up in self.terms], "nterm": len(self.terms),
             "act": L.ACT[self.act], "out": self.out.ptr(self.c0),
             "out_n_stride": self.out.n_stride, "N": g.N, "C": C, "H": self.out.H,
             "W": self.out.W}
        if self.slope is not None:
            t["slope"] = Ptr(self.slope.slot)
        return t

    def fwd(self, ops):
        if getattr(self, "fwd_folded", False):
            return  # the next 1x1 conv computes and writes the output (_fold_tails)
        ops.add(Record(L.OP_TAIL_FWD, L.Tail, self.spec(), label=self.out.name))

    def bwd(self, ops, gs):
        g = self.g
        C = self.terms[0][0].C
        if getattr(self, "bwd_folded", False):
            return  # done in the consumer's input-gradient sink (ConvOp._res_sink)
        if not gs.has_grad(self.out, self.c0, C):
            return
        d = gs.dbuf(self.out)
        rec = {"f": self.spec(), "dout": d.ptr(self.c0), "dout_n_stride": d.n_stride}
        if self.slope is not None:
            rec["slope_grad"] = Ptr(S_STATS, self.slope.acc_off * 8)
            self.slope.used_in_bwd = True
        if any(v.bn is not None for v, _ in self.terms):
            gb = gs.alloc(Buf(S_GRAD, g.N, C, self.out.H, self.out.W, "gt"), "gt_" + self.out.name)
            rec["g"] = gb.ptr()
            rec["g_n_stride"] = gb.n_stride
            for v, _ in self.terms:
                if v.bn is not None:
                    assert v.c0 == 0 and v.C == v.buf.C
                    assert id(v.buf) not in gs.G
                    gs.G[id(v.buf)] = gb
                    if v.bn.fin:
                        gs.pending_final.append(v.bn)
        dterm, dns, dacc = [None] * 3, [0] * 3, [0] * 3
        for i, (v, up) in enumerate(self.terms):
            if v.bn is None and v.grad:
                if getattr(v.buf, "need_sum", None) is not None:
                    raise NotImplementedError("tail term that needs a bias-gradient sum")
                db = gs.dbuf(v.buf)
                first = gs.mark(v.buf, v.c0, v.C)
                dterm[i] = db.ptr(v.c0)
                dns[i] = db.n_stride
                dacc[i] = 0 if first else 1
        rec["dterm"] = dterm
        rec["dterm_n_stride"] = dns
        rec["dterm_accum"] = dacc
        ops.add(Record(L.OP_TAIL_BWD, L.TailGrad, rec, label="d_" + self.out.name))


# ---------------------------------------------------------------------------------
class Plan:
    """Compiled forward (+ optional backward) op lists of one module at one shape."""

    def __init__(self, owner, in_shapes, train, need_grad, in_grad, buckets=2, layout=None,
                 fused_tail=False):
        """buckets: gradient buckets of the backward (2: the stem's parameters finalised in a
        second part after the others, for a data-parallel exchange that overlaps the stem
        backward; 1: one part, every finalisation at the end — at world size 1 nothing
        needs bucket 1 early, and the part boundary's side-stream join made the stem's
        input-gradient chain wait ~0.6 ms for the queued weight gradients).
        fused_tail (a training plan with one bucket: the Trainer at world size 1): the
        backward ends in ONE OP_STEP_TAIL record — replica fold, gradient finalisation,
        Adam and the BatchNorm running-stat updates (isg.h isg_step_tail) — instead of the
        fold, the finalisation lists and the forward's BN-update lists; the Adam step
        counter advances in an OP_STEP_INC record forked at the backward's head. Its
        pointers come from slots S_PARAM..S_TAILBNU; the item tables to resolve and upload
        are tail_gf / tail_bnu (Records), the owned gradient ranges tail_owned."""
        self.n_buckets = buckets
        self.fused_tail = bool(fused_tail and train and need_grad and buckets == 1)
        self.tail_gf, self.tail_bnu, self.tail_owned = None, None, []
        N = in_shapes[0][0]
        g = Graph(owner, N, train, need_grad, layout)
        ins = [g.input(i, s[1], s[2], s[3], in_grad[i]) if len(s) == 4 else
               g.keypoints(i, s[0], s[1]) for i, s in enumerate(in_shapes)]
        outs = owner.emit(g, *ins)
        if isinstance(outs, Value):
            outs = (outs,)
        self.graph = g
        # outputs: materialise each into its output slot
        self.out_bufs = []
        for i, o in enumerate(outs):
            ob = Buf(S_OUT[i], N, o.C, o.H, o.W, f"out{i}")
            head = next((op for op in g.ops if isinstance(op, HeadOp) and len(o.segs) == 1
                         and op.out is o.segs[0].buf and not o.segs[0].virtual), None)
            if head is not None:
                head.out = ob  # the fused head writes the output slot itself (no copy)
            else:
                self._emit_output(g, o, ob)
            self.out_bufs.append(ob)
        self.out_shapes = [(N, b.C, b.H, b.W) for b in self.out_bufs]
        _fold_tails(g)
        # a training step's loss accumulator (one double): in the statistics arena, so the
        # forward's memset zeroes it (no separate fill launch before the loss kernel)
        self.loss_off = None
        if train and need_grad:
            self.loss_off = g.stats_size
            g.stats_size += 8
        # ---- forward list
        fw = OpList()
        if g.stats_size:
            fw.add(Record(L.OP_MEMSET, L.MemsetRec, {"p": Ptr(S_STATS), "bytes": g.stats_size * 8}))
        if need_grad:
            # the weight-gradient replicas (L.WREP fp64 copies of the flat gradient, 34 MB for
            # Segment(20)) are zeroed on the side stream under the forward instead of at the
            # head of the backward's critical path; the forward's final join covers it
            r = Record(L.OP_MEMSET, L.MemsetRec, {"p": Ptr(S_WREP),
                                                  "bytes": L.WREP * g.pgrad_size * 8},
                       label="zero_wgrad_replicas")
            r.flags |= Record.OPF_SIDE | Record.OPF_FORK_NOW
            fw.add(r)
        side_recs = []
        for op in g.ops:
            i0 = len(fw.recs)
            op.fwd(fw)
            bnr = getattr(op, "bnr", None)
            for b in getattr(op, "bnrs", [bnr]):
                if train and b is not None and b.fin:
                    fw.add(bn_final_record([b], False))
            if getattr(op, "side", False):
                rng = [_buf_range(op.out)]
                if bnr is not None:
                    rng.append((S_STATS, bnr.stats_off * 8, bnr.coef_end * 8))
                side_recs += [(r, rng) for r in fw.recs[i0:]]
        self.tail_bnu = None
        if train and g.bns:
            items = []
            for b in g.bns:
                items.append({"stats": Ptr(S_STATS, b.stats_off * 8),
                              "running_mean": b.names["rm"], "running_var": b.names["rv"],
                              "num_batches_tracked": b.names["nbt"], "C": b.C,
                              "count": float(b.count), "momentum": float(b.mod.momentum)})
            if self.fused_tail:  # updated by the step tail (the statistics stay intact)
                self.tail_bnu = Record(L.OP_BN_UPDATE, L.ListRec, {"n": len(items)}, L.BnUpdate,
                                       items)
                self.tail_bnu_n = len(items)
                items = []
            # (measured: forked as one side batch at the head of the backward instead, the
            # step was 0.1 ms slower, profiles/r07v_ab_bn_update.txt)
            for i in range(0, len(items), L.LIST_CHUNK):
                chunk = items[i:i + L.LIST_CHUNK]
                fw.add(Record(L.OP_BN_UPDATE, L.ListRec, {"n": len(chunk)}, L.BnUpdate, chunk))
        _fork_pools(fw)
        _fork_branches(fw, side_recs)
        _delay_forks(fw)
        _join_exclusions(fw.recs)
        self.fwd = fw.compile()
        self.act_size = g.act_size
        self.stats_size = max(g.stats_size, 8)
        self.bwd = None
        if need_grad:
            self._build_backward(g, ins)

    def stacking_holds(self, tensors):
        """True while every stacked sibling pair's weights (Graph.stacked) are still adjacent
        in memory in `tensors` (the module's parameters + buffers in named order). Parameters
        rebound after the plan was built (load_state_dict(assign=True), `p.data = ...`, a
        re-flatten) can break that; the caller then rebuilds the plan."""
        for ia, ib, nb in self.graph.stacked:
            wa, wb = tensors[ia], tensors[ib]
            if (wa.device != wb.device or not wa.is_contiguous() or not wb.is_contiguous()
                    or wb.data_ptr() != wa.data_ptr() + nb):
                return False
        return True

    def tail_tables(self, table):
        """The fused tail's item tables with every pointer resolved against `table` (the
        pointer-table array the Trainer runs the plan with): (grad_final items bytes,
        BatchNorm-update items bytes), to upload into the buffers of slots S_TAILGF /
        S_TAILBNU. The Trainer's arenas never move, so this is done once."""
        def resolve(rec):
            if rec is None:
                return b""
            body = bytearray(rec.body)
            for loc, slot, off in rec.fix:
                base = table[slot]
                struct.pack_into("<Q", body, loc, (base + off) if base else 0)
            return bytes(body[ctypes.sizeof(L.ListRec):])
        return resolve(self.tail_gf), resolve(self.tail_bnu)

    def _step_tail(self, g, ol, gf_items):
        """The fused end of the step (fused_tail): the Adam step counter advanced on the side
        stream from the backward's head (the tail's join waits for it), then one
        OP_STEP_TAIL record joining every forked weight gradient."""
        inc = Record(L.OP_STEP_INC, L.StepIncRec, {"step": Ptr(S_STEP)}, label="step_inc")
        inc.flags |= Record.OPF_SIDE | Record.OPF_FORK_NOW
        ol.recs.insert(0, inc)
        self.tail_gf = Record(L.OP_GRAD_FINAL, L.ListRec, {"n": len(gf_items)}, L.GradFinal,
                              gf_items)
        # gradient elements a grad_final item writes (the fold skips them): (offset, count)
        self.tail_owned = []
        for it in gf_items:
            for k in ("dgamma", "dbeta", "dconv_bias", "dslope"):
                v = it.get(k)
                if isinstance(v, Ptr):
                    assert v.slot == S_PGRAD and v.off % 4 == 0
                    self.tail_owned.append((v.off // 4, it["C"]))
        nbnu = self.tail_bnu_n if self.tail_bnu else 0
        r = Record(L.OP_STEP_TAIL, L.StepTail,
                   {"grad": Ptr(S_PGRAD), "rep": Ptr(S_WREP), "n": g.pgrad_size, "nrep": L.WREP,
                    "ngf": len(gf_items), "param": Ptr(S_PARAM), "exp_avg": Ptr(S_EXPAVG),
                    "exp_avg_sq": Ptr(S_EXPAVGSQ), "owner": Ptr(S_OWNER), "step": Ptr(S_STEP),
                    "hyper": Ptr(S_HYPER), "gf": Ptr(S_TAILGF),
                    "bnu": Ptr(S_TAILBNU) if nbnu else None, "nbnu": nbnu},
                   label="step_tail")
        r.flags |= Record.OPF_JOIN  # every forked weight gradient (and the counter) is done
        ol.add(r)

    @staticmethod
    def _late_prefix(g):
        """Module-name prefix of the late gradient bucket: the owner's first child module
        (Segment: `init_conv.`, whose parameters lead the parameter order and whose
        backward runs last), or None when the owner has no children with parameters."""
        for name, child in g.owner.named_children():
            if any(True for _ in child.parameters()):
                return name + "."
            return None
        return None

    def _bucket_split(self, g, gs, recs):
        """(cut, split): bucket 2 = the parameters under the late prefix, a leading range
        [0, cut) of the flat gradient; split = the first backward op after which no op
        touches (by any pointer) bucket 1's gradient replicas or the statistics its
        finalisation reads. Returns (0, len(recs)) when no such split exists."""
        late = self._late_prefix(g)
        if late is None or not g.train or self.n_buckets < 2:
            return 0, len(recs)
        cut = 0
        for k in g.param_names:
            if not k.startswith(late):
                break
            n = 1
            for s in g.param_shapes[k]:
                n *= s
            cut += n
        if any(k.startswith(late) for k in g.param_names[len([1 for k in g.param_names
                                                               if k.startswith(late)]):]):
            return 0, len(recs)  # late parameters are not a leading range
        # statistics ranges (bytes in S_STATS) of bucket-1 modules
        early_stats = []
        for b in g.bns:
            if not g.mod_names[id(b.mod)].startswith(late):
                n = (4 * b.C * L.STAT_REP + 7) // 8 * 8
                early_stats.append((b.stats_off * 8, (b.stats_off + n) * 8))
                early_stats.append((b.coef_off * 8, b.coef_end * 8))
        for sl in g.slopes.values():
            if not g.mod_names[id(sl.mod)].startswith(late):
                early_stats.append((sl.acc_off * 8, (sl.acc_off + sl.C * L.STAT_REP) * 8))
        for mod, out, _ in gs.bias_sums:
            if not g.mod_names[id(mod)].startswith(late):
                early_stats.append((out.need_sum * 8, (out.need_sum + 4 * out.C * L.STAT_REP) * 8))

        def touches_early(r):
            for _, slot, off in r.fix:
                if (slot == S_PGRAD and off >= cut * 4) or (slot == S_WREP and off >= cut * 8):
                    return True
                if slot == S_STATS and any(lo <= off < hi for lo, hi in early_stats):
                    return True
            return False

        split = 0
        for i, r in enumerate(recs):
            if touches_early(r):
                split = i + 1
        return cut, split

    def _emit_output(self, g, o, ob):
        # route the value into the output slot with a tail (copy / BN+act)
        c = 0
        for s in o.segs:
            term = Value([Val(s.buf, s.c0, s.C, s.bn, "none", None, s.grad)])
            g.tail([(term, False)], s.act, s.slope, out=ob, c0=c, name=ob.name)
            c += s.C

    def _build_backward(self, g, ins):
        gs = GradState(g)
        gs.bias_sums = []
        gs.bias_from_bn = []
        for i, ob in enumerate(self.out_bufs):
            gs.external[id(ob)] = Buf(S_DOUT[i], ob.N, ob.C, ob.H, ob.W, f"dout{i}")
        for i, v in enumerate(ins):
            if isinstance(v, Value) and v.grad:
                b = v.segs[0].buf
                gs.external[id(b)] = Buf(S_DIN[i], b.N, b.C, b.H, b.W, f"din{i}")
        # weight gradients accumulate (fp64 atomics of fp32 workgroup partials: exact, so
        # order-independent, isg.h ISG_WREP) into L.WREP replicas — zeroed by the forward
        # (its side-stream memset) — folded into S_PGRAD by OP_SUM_REP before the BN/PReLU
        # finalisation overwrites its own entries
        bw = OpList()
        body = OpList()
        gs.pending_final = []
        for op in reversed(g.ops):
            op.bwd(body, gs)
            if g.train and gs.pending_final:
                body.add(bn_final_record(gs.pending_final, True))
                gs.pending_final = []
        for r in body.recs:
            if r.kind in (L.OP_CONV_WGRAD, L.OP_KP_STEM_WGRAD, L.OP_HEAD_FOLD):
                r.flags |= Record.OPF_SIDE  # nothing later in the list reads a weight gradient
        _fork_late_wgrads(body.recs, self._late_prefix(g))
        _trailing_on_main(body.recs)
        self.din_written = [isinstance(v, Value) and v.grad and
                            bool(gs.inited.get(id(v.segs[0].buf))) for v in ins]
        # finalisation of BN / PReLU / conv-bias-before-BN gradients: (module, item)
        conv_before = {id(bnr): mod for mod, bnr in gs.bias_from_bn}
        items = []
        # bias of a convT with no BN after it (segment.py:435-436): the per-channel sum
        # of its output gradient, accumulated by the consumers' gradient sinks
        for mod, out, dy in gs.bias_sums:
            items.append((mod, {"slope_acc": Ptr(S_STATS, out.need_sum * 8),
                                "dslope": g.gptr(mod, "bias"), "C": out.C,
                                "slope_stride": 4 * out.C}))
        for b in g.bns:
            it = {"stats": Ptr(S_STATS, b.stats_off * 8), "gamma": b.names["gamma"],
                  "running_mean": b.names["rm"], "running_var": b.names["rv"],
                  "dgamma": g.gptr(b.mod, "weight"), "dbeta": g.gptr(b.mod, "bias"),
                  "C": b.C, "train": 1 if g.train else 0, "count": float(b.count),
                  "eps": float(b.mod.eps)}
            if id(b) in conv_before:
                it["dconv_bias"] = g.gptr(conv_before[id(b)], "bias")
            items.append((b.mod, it))
        for sl in g.slopes.values():
            if sl.used_in_bwd:
                items.append((sl.mod, {"slope_acc": Ptr(S_STATS, sl.acc_off * 8),
                                       "dslope": g.gptr(sl.mod, "weight"), "C": sl.C,
                                       "slope_stride": sl.C}))
        cut, split = self._bucket_split(g, gs, body.recs)
        late = self._late_prefix(g)

        def is_late(mod):
            return late is not None and g.mod_names[id(mod)].startswith(late)

        def close(ol, lo, hi, its, side=False):
            """Fold the weight-gradient replicas of parameter range [lo, hi) (floats) and
            finalise the statistics-derived gradients of that range. side: on the side
            stream behind the forked weight gradients (in order after them), forked from
            the main stream here (every statistic is complete), so the stem backward that
            follows overlaps it; the list's final join covers it."""
            recs = []
            if hi > lo:
                recs.append(Record(L.OP_SUM_REP, L.SumRepRec,
                                   {"dst": Ptr(S_PGRAD, lo * 4), "src": Ptr(S_WREP, lo * 8),
                                    "n": hi - lo, "stride": g.pgrad_size, "nrep": L.WREP},
                                   label="sum_wgrad_replicas"))
                if not side:  # every forked weight gradient is in the replicas
                    recs[-1].flags |= Record.OPF_JOIN
            for i in range(0, len(its), L.LIST_CHUNK):
                chunk = its[i:i + L.LIST_CHUNK]
                recs.append(Record(L.OP_GRAD_FINAL, L.ListRec, {"n": len(chunk)}, L.GradFinal,
                                   chunk))
            for r in recs:
                if side or r.kind == L.OP_GRAD_FINAL:
                    # the finalisation lists are independent of each other: forked behind
                    # the fold, dealt over both side streams (api.cpp), joined at the end
                    # of the list (5 launches of ~5 us each ran back to back on the main
                    # stream at the very end of the step)
                    r.flags |= Record.OPF_SIDE | Record.OPF_FORK_NOW
                ol.add(r)

        # Two gradient buckets for data parallelism: bucket 1 = parameters
        # [cut, n), final once body[:split] has run; bucket 2 = [0, cut) (the stem, whose
        # backward runs last). The Trainer all-reduces bucket 1 on RCCL's stream while the
        # stem backward (body[split:]) runs. split == len(body): one bucket at the end.
        part1, part2 = OpList(), OpList()
        for r in body.recs[:split]:
            part1.add(r)
        if split < len(body.recs):
            close(part1, cut, g.pgrad_size, [it for m, it in items if not is_late(m)],
                  side=os.environ.get("ISG_SIDE_CLOSE", "0") == "1")  # opt-in: measured
            # 377.9 -> 376.7 images/s on the side stream (r02h, 3 interleaved pairs)
            for r in body.recs[split:]:
                part2.add(r)
            close(part2, 0, cut, [it for m, it in items if is_late(m)])
        elif self.fused_tail:
            cut = 0
            self._step_tail(g, part1, [it for _, it in items])
        else:
            cut = 0
            close(part1, 0, g.pgrad_size, [it for _, it in items])
        for r in part1.recs + part2.recs:
            bw.add(r)
        self.bucket_cut = cut
        self.bwd_parts = [part1.compile()] + ([part2.compile()] if part2.recs else [])
        self.stats_size = max(g.stats_size, 8)
        self.bwd = bw.compile()
        self.grad_size = gs.size
        self.grad_bufs = list(gs.D.values()) + list(gs.G.values())  # for debugging tools
        self.used_params = set(g.used_params)
