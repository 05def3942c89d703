"""Kernel-level parity of libisg.so against fp64 CPU references (torch.nn.functional
semantics, the same ops the oracle uses). Calls go straight through the C-ABI."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from instancesegmentation_amd import _lib as L
from tests.isg_helpers import (bn_spec_eval, bn_spec_train, call, geom, ptr, rep_fold, rep_from,
                               rep_zeros, sinks, stream, struct, vt)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def close(got, ref, tol=2e-5, what=""):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    scale = max(ref.abs().max().item(), 1e-3)
    err = (got - ref).abs().max().item()
    assert err <= tol * scale + 1e-6, f"{what}: max err {err:.3e} (scale {scale:.3e})"


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g, dtype=torch.float64) * scale)


def bn_eval_params(C, seed):
    g = torch.Generator().manual_seed(seed)
    gamma = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    beta = torch.rand(C, generator=g, dtype=torch.float64) - 0.5
    rm = torch.rand(C, generator=g, dtype=torch.float64) - 0.5
    rv = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    slope = torch.rand(C, generator=g, dtype=torch.float64) * 0.4
    return gamma, beta, rm, rv, slope


def fwd_xform_ref(x, gamma, beta, rm, rv, slope, act):
    z = (x - rm[None, :, None, None]) / torch.sqrt(rv[None, :, None, None] + 1e-5) \
        * gamma[None, :, None, None] + beta[None, :, None, None]
    if act == "prelu":
        return torch.where(z > 0, z, z * slope[None, :, None, None])
    if act == "relu":
        return z.clamp_min(0)
    return z


def cuda32(t):
    return t.to(DEV, torch.float32).contiguous()


DENSE = [
    # (Ci, Co, H, W, k, s, p, d)
    (48, 16, 32, 32, 1, 1, 0, 1),
    (20, 16, 64, 48, 5, 2, 2, 1),
    (36, 16, 32, 32, 2, 2, 0, 1),
    (16, 16, 24, 40, 3, 1, 1, 1),
    (4, 1, 32, 32, 3, 1, 1, 1),
    (4, 16, 64, 64, 8, 4, 2, 1),
    (96, 48, 16, 16, 1, 1, 0, 1),
    (48, 128, 16, 16, 1, 1, 0, 1),
    (16, 16, 20, 20, 3, 1, 2, 2),
    # thin pointwise (pw_gemm.hip thin_pw_kernel: K, M <= 16, HW % 4 == 0; 5x7 falls back)
    (4, 16, 64, 64, 1, 1, 0, 1),
    (16, 4, 36, 20, 1, 1, 0, 1),
    (8, 8, 10, 6, 1, 1, 0, 1),
    (16, 16, 24, 24, 1, 1, 0, 1),
    (4, 4, 5, 7, 1, 1, 0, 1),
    (16, 48, 24, 20, 1, 1, 0, 1),
    (4, 32, 16, 12, 1, 1, 0, 1),
    # tap_conv coverage: Ci % 4 != 0, 3 row tiles, ragged edges, multi-tile grids
    (3, 16, 64, 48, 5, 2, 2, 1),
    (16, 36, 33, 45, 3, 1, 1, 1),
    (20, 16, 130, 100, 5, 2, 2, 1),
    (16, 4, 72, 88, 8, 4, 2, 1),
    (4, 4, 40, 36, 3, 1, 1, 1),
    # the Segment(20) 128^2 shapes (tile choices of tap_conv / tap_wgrad at network scale)
    (16, 16, 64, 64, 5, 2, 2, 1),
    (36, 16, 64, 64, 2, 2, 0, 1),
    (48, 16, 32, 32, 2, 2, 0, 1),
    (16, 16, 32, 32, 3, 1, 1, 1),
    (20, 16, 128, 128, 5, 2, 2, 1),
    (16, 16, 16, 16, 3, 1, 1, 1),
    (48, 16, 16, 16, 2, 2, 0, 1),
    # k 2S stride S pad S/2 with <= 4 input channels (down_conv: the sub-pixel convT's
    # input / weight gradients): ragged cell grids, 3 and 8 output channels
    (4, 16, 40, 56, 8, 4, 2, 1),
    (4, 3, 32, 32, 8, 4, 2, 1),
    (4, 16, 32, 48, 4, 2, 1, 1),
    (2, 8, 24, 40, 4, 2, 1, 1),
    # 5x5 s2 p2 input gradient as a sub-pixel transposed conv (sub2_dgrad): ragged, odd grid
    (16, 16, 62, 90, 5, 2, 2, 1),
    (8, 12, 40, 24, 5, 2, 2, 1),
    # ... on the LDS-staged form (cell columns % 4 == 0): two column blocks, ragged rows
    (16, 16, 74, 136, 5, 2, 2, 1),
    # 5x5 s2 with <= 16 channels (the stem's second conv; tap_conv by default, the
    # opt-in s2k5_fwd in test_s2k5_fwd): partial column block, odd output rows, fewer
    # channels than the 16-lane fragments
    (16, 16, 134, 200, 5, 2, 2, 1),
    (12, 8, 40, 36, 5, 2, 2, 1),
    # thin 3x3 (thin_conv / thin_wgrad, 4 pixels per lane): ragged row count, 1 -> 4
    (4, 1, 37, 96, 3, 1, 1, 1),
    (1, 4, 24, 20, 3, 1, 1, 1),
    # k4 s2 p1: the ConvTranspose2d input gradients (odd first tap column, stride-2 pairs)
    (16, 48, 32, 32, 4, 2, 1, 1),
    (16, 4, 64, 48, 4, 2, 1, 1),
]


def _geom(N, Ci, Co, H, W, k, s, p, d, groups=1):
    OH = (H + 2 * p - d * (k - 1) - 1) // s + 1
    OW = (W + 2 * p - d * (k - 1) - 1) // s + 1
    return dict(N=N, Ci=Ci, H=H, W=W, Co=Co, OH=OH, OW=OW, KH=k, KW=k, SH=s, SW=s, PH=p, PW=p,
                DH=d, DW=d, groups=groups), OH, OW


@pytest.mark.parametrize("cfg", DENSE)
def test_conv_fwd_dense(cfg):
    Ci, Co, H, W, k, s, p, d = cfg
    N = 2
    ge, OH, OW = _geom(N, Ci, Co, H, W, k, s, p, d)
    x = rnd(N, Ci, H, W, seed=1)
    w = rnd(Co, Ci, k, k, seed=2, scale=(2.0 / (Ci * k * k)) ** 0.5)
    b = rnd(Co, seed=3, scale=0.1)
    gamma, beta, rm, rv, slope = bn_eval_params(Ci, 4)
    # two segments: first half BN+PReLU on load, second half plain
    c1 = Ci // 2 if Ci > 1 else Ci
    xt = x.clone()
    xt[:, :c1] = fwd_xform_ref(x[:, :c1], gamma[:c1], beta[:c1], rm[:c1], rv[:c1], slope[:c1],
                               "prelu")
    ref = F.conv2d(xt, w, b, stride=s, padding=p, dilation=d)
    X = cuda32(x)
    G = [cuda32(t[:c1]) for t in (gamma, beta, rm, rv, slope)]
    segs = [{"p": ptr(X), "n_stride": Ci * H * W, "C": c1, "xform": L.XF_BN_FWD,
             "act": L.ACT["prelu"], "slope": ptr(G[4]), "bn": bn_spec_eval(*G[:4])}]
    if Ci - c1 > 0:
        segs.append({"p": X.data_ptr() + c1 * H * W * 4, "n_stride": Ci * H * W, "C": Ci - c1,
                     "xform": L.XF_PLAIN})
    Wt, B = cuda32(w), cuda32(b)
    Y = torch.full((N, Co, OH, OW), float("nan"), device=DEV)
    stats = rep_zeros(4 * Co)
    sk = sinks([{"p": ptr(Y), "n_stride": Co * OH * OW, "c0": 0, "C": Co,
                 "mode": L.SINK_STORE, "bias": ptr(B), "stats": ptr(stats)}])
    call("isg_conv_fwd", geom(**ge), vt(segs, N, H, W), ptr(Wt), sk, stream())
    close(Y, ref, what="conv fwd")
    stats = rep_fold(stats, 4 * Co)
    close(stats[:Co], ref.sum((0, 2, 3)), what="sum")
    close(stats[Co:2 * Co], (ref * ref).sum((0, 2, 3)), what="sumsq")


@pytest.mark.parametrize("cfg", [(16, 16, 512, 512), (16, 16, 134, 200), (12, 8, 40, 36),
                                 (16, 16, 400, 672), (3, 16, 64, 48), (3, 16, 1024, 1024, 20)],
                         ids=["stem_bench", "ragged", "narrow", "stem_1344x800", "three_channels",
                              "stem_rgb_layer1_wci20"])
def test_s2k5_fwd(cfg):
    """The persistent producer/consumer 5x5 s2 forward (down_conv.hip s2k5_fwd_kernel, the
    stem's layer 2) against fp64 at a bar of 4e-6 of scale — one fp32 rounding chain over
    400 taps — at the bench geometry (2x512^2 -> 256^2, 1024 tiles over persistent
    workgroups), BASELINE config 3's (2x400x672 -> 200x336: partial column and row tiles),
    ragged shapes and 3 input channels; training-mode BN + PReLU on load, bias and BN
    statistics through the STORE sink."""
    Ci, Co, H, W = cfg[:4]
    wci = cfg[4] if len(cfg) > 4 else Ci  # the keypoint stem's RGB part: weight over 20 channels
    N = 2
    ge, OH, OW = _geom(N, Ci, Co, H, W, 5, 2, 2, 1)
    if wci != Ci:
        ge["w_ci"] = wci
    x = rnd(N, Ci, H, W, seed=11) * 0.7 + 0.2
    wfull = rnd(Co, wci, 5, 5, seed=12, scale=(2.0 / (wci * 25)) ** 0.5)
    w = wfull[:, :Ci].contiguous()
    b = rnd(Co, seed=13, scale=0.1)
    gamma, beta, _, _, slope = bn_eval_params(Ci, 5)
    mean = x.mean((0, 2, 3))
    var = x.var((0, 2, 3), unbiased=False)
    xt = fwd_xform_ref(x, gamma, beta, mean, var, slope, "prelu")
    ref = F.conv2d(xt, w, b, stride=2, padding=2)
    X = cuda32(x)
    G = [cuda32(t) for t in (gamma, beta, mean, var, slope)]
    segs = [{"p": ptr(X), "n_stride": Ci * H * W, "C": Ci, "xform": L.XF_BN_FWD,
             "act": L.ACT["prelu"], "slope": ptr(G[4]), "bn": bn_spec_eval(*G[:4])}]
    Y = torch.full((N, Co, OH, OW), float("nan"), device=DEV)
    stats = rep_zeros(4 * Co)
    B, Wt = cuda32(b), cuda32(wfull)  # held: the kernel reads them after this frame's temporaries die
    sk = sinks([{"p": ptr(Y), "n_stride": Co * OH * OW, "c0": 0, "C": Co,
                 "mode": L.SINK_STORE, "bias": ptr(B), "stats": ptr(stats)}])
    call("isg_conv_fwd", geom(**ge), vt(segs, N, H, W), ptr(Wt), sk, stream())
    torch.cuda.synchronize()
    close(Y, ref, tol=4e-6, what="s2k5 fwd")
    stats = rep_fold(stats, 4 * Co)
    close(stats[:Co], ref.sum((0, 2, 3)), tol=4e-6, what="sum")
    close(stats[Co:2 * Co], (ref * ref).sum((0, 2, 3)), tol=4e-6, what="sumsq")


@pytest.mark.parametrize("cfg", [(16, 16, 512, 512), (16, 16, 134, 200), (12, 10, 72, 200),
                                 (3, 16, 64, 48), (3, 16, 1024, 1024, 20), (4, 12, 40, 72)],
                         ids=["stem_bench", "ragged", "narrow_partial_rows", "three_channels",
                              "stem_rgb_layer1_wci20", "four_channels_ragged"])
def test_s2k5_wgrad(cfg):
    """The LDS-staged 5x5 s2 weight gradient (down_conv.hip s2k5_wgrad_kernel, the stem's
    layer 2 on the bench step) through the replicated entry point, against fp64: dy with
    training-mode BatchNorm backward rebuilt on load, x with BatchNorm + PReLU on load, the
    dbias, at the bench geometry (2x512^2 -> 256^2, 1024 tiles over persistent workgroups),
    a partial last column tile, a partial last row tile with fewer than 16 channels on both
    sides, and 3-4 input channels (the narrow form: channels x taps in the MFMA's N), incl.
    the keypoint stem's RGB layer 1 whose weight spans w_ci = 20 channels."""
    Ci, Co, H, W = cfg[:4]
    wci = cfg[4] if len(cfg) > 4 else Ci
    N = 2
    ge, OH, OW = _geom(N, Ci, Co, H, W, 5, 2, 2, 1)
    if wci != Ci:
        ge["w_ci"] = wci
    x = rnd(N, Ci, H, W, seed=51)
    gamma, beta, rm, rv, slope = bn_eval_params(Ci, 52)
    xt = fwd_xform_ref(x, gamma, beta, rm, rv, slope, "prelu")
    yraw = rnd(N, Co, OH, OW, seed=53) + 0.3
    gbn = rnd(N, Co, OH, OW, seed=54)
    og, ob, st, _ = _bn_train_state(yraw, gbn, 55)
    dy = _bn_bwd_ref(yraw, gbn, og)
    ref = torch.nn.grad.conv2d_weight(xt, (Co, Ci, 5, 5), dy, stride=2, padding=2)
    X, G = cuda32(x), [cuda32(t) for t in (gamma, beta, rm, rv, slope)]
    xseg = {"p": ptr(X), "n_stride": Ci * H * W, "C": Ci, "xform": L.XF_BN_FWD,
            "act": L.ACT["prelu"], "slope": ptr(G[4]), "bn": bn_spec_eval(*G[:4])}
    Yr, Gb, GA, BE, ST = cuda32(yraw), cuda32(gbn), cuda32(og), cuda32(ob), rep_from(st)
    dyseg = {"p": ptr(Gb), "y": ptr(Yr), "n_stride": Co * OH * OW, "y_n_stride": Co * OH * OW,
             "C": Co, "xform": L.XF_BN_BWD, "bn": bn_spec_train(GA, BE, ST, N * OH * OW)}
    nw = Co * wci * 25
    stride_ = nw + Co + 5
    REP = torch.zeros(L.WREP * stride_, dtype=torch.float64, device=DEV)
    dbias_p = ptr(REP[nw:]) if wci == Ci else 0  # the partial-weight entry takes no bias
    call("isg_conv_wgrad_rep", geom(**ge), vt([dyseg], N, OH, OW), vt([xseg], N, H, W),
         ptr(REP), dbias_p, stride_, L.WREP, stream())
    OUT = torch.full((stride_,), float("nan"), device=DEV)
    call("isg_sum_replicas", ptr(OUT), ptr(REP), stride_, L.WREP, stride_, stream())
    torch.cuda.synchronize()
    full = OUT[:nw].view(Co, wci, 5, 5)
    close(full[:, :Ci], ref, what="s2k5 wgrad")
    if wci != Ci:
        assert torch.all(full[:, Ci:] == 0)  # the other weight channels are not touched
        return
    # the BatchNorm-backward dy sums to ~0 per channel: the dbias bar is relative to the
    # summed magnitudes (one fp32 rounding per partial over 2 x 256^2 terms)
    derr = (OUT[nw:nw + Co].double().cpu() - dy.sum((0, 2, 3))).abs().max().item()
    assert derr <= 1e-6 * dy.abs().sum((0, 2, 3)).max().item(), derr
    assert torch.all(OUT[nw + Co:] == 0)


def _bn_train_state(y, g, seed):
    """stats [sum, sumsq, gsum, gxsum] for raw y and BN-output grad g (gxsum centred)."""
    C = y.shape[1]
    gamma, beta, _, _, slope = bn_eval_params(C, seed)
    mean = y.mean((0, 2, 3), keepdim=True)
    stats = torch.cat([y.sum((0, 2, 3)), (y * y).sum((0, 2, 3)), g.sum((0, 2, 3)),
                       (g * (y - mean)).sum((0, 2, 3))])
    return gamma, beta, stats, slope


def _bn_bwd_ref(y, g, gamma):
    M = y.shape[0] * y.shape[2] * y.shape[3]
    mean = y.mean((0, 2, 3), keepdim=True)
    var = y.var((0, 2, 3), unbiased=False, keepdim=True)
    rstd = 1 / torch.sqrt(var + 1e-5)
    xhat = (y - mean) * rstd
    gm = g.mean((0, 2, 3), keepdim=True)
    gxm = (g * xhat).sum((0, 2, 3), keepdim=True) / M
    return gamma[None, :, None, None] * rstd * (g - gm - xhat * gxm)


@pytest.mark.parametrize("cfg", DENSE)
def test_conv_dgrad_dense(cfg):
    Ci, Co, H, W, k, s, p, d = cfg
    N = 2
    ge, OH, OW = _geom(N, Ci, Co, H, W, k, s, p, d)
    w = rnd(Co, Ci, k, k, seed=5, scale=0.3)
    yraw = rnd(N, Co, OH, OW, seed=6) + 0.3
    gbn = rnd(N, Co, OH, OW, seed=7)
    gamma, beta, st, _ = _bn_train_state(yraw, gbn, 8)
    dy = _bn_bwd_ref(yraw, gbn, gamma)
    ref = torch.nn.grad.conv2d_input((N, Ci, H, W), w, dy, stride=s, padding=p, dilation=d)
    # sink: ACTBWD with eval BN + PReLU on the input side
    xin = rnd(N, Ci, H, W, seed=9)
    ig, ib, irm, irv, islope = bn_eval_params(Ci, 10)
    z = fwd_xform_ref(xin, ig, ib, irm, irv, islope, "none")
    gref = torch.where(z > 0, ref, ref * islope[None, :, None, None])
    sref = torch.where(z > 0, torch.zeros_like(z), z * ref).sum((0, 2, 3))
    Yr, Gb, GA, BE, ST = cuda32(yraw), cuda32(gbn), cuda32(gamma), cuda32(beta), rep_from(st)
    dyseg = {"p": ptr(Gb), "y": ptr(Yr), "n_stride": Co * OH * OW, "y_n_stride": Co * OH * OW,
             "C": Co, "xform": L.XF_BN_BWD, "bn": bn_spec_train(GA, BE, ST, N * OH * OW)}
    DX = torch.full((N, Ci, H, W), float("nan"), device=DEV)
    XI = cuda32(xin)
    IG = [cuda32(t) for t in (ig, ib, irm, irv, islope)]
    istats = rep_zeros(4 * Ci)
    sgrad = rep_zeros(Ci)
    bn_in = bn_spec_eval(*IG[:4])
    bn_in["stats"] = ptr(istats)
    sk = sinks([{"p": ptr(DX), "n_stride": Ci * H * W, "c0": 0, "C": Ci, "mode": L.SINK_ACTBWD,
                 "act": L.ACT["prelu"], "y": ptr(XI), "y_n_stride": Ci * H * W,
                 "slope": ptr(IG[4]), "slope_grad": ptr(sgrad), "bn": bn_in}])
    call("isg_conv_dgrad", geom(**ge), vt([dyseg], N, OH, OW), ptr(cuda32(w)), sk, stream())
    close(DX, gref, what="dgrad g")
    istats, sgrad = rep_fold(istats, 4 * Ci), rep_fold(sgrad, Ci)
    close(istats[2 * Ci:3 * Ci], gref.sum((0, 2, 3)), what="gsum")
    close(istats[3 * Ci:], (gref * (xin - irm[None, :, None, None])).sum((0, 2, 3)),
          what="gxsum")
    close(sgrad, sref, what="slope grad")


@pytest.mark.parametrize("cfg", DENSE)
def test_conv_wgrad_dense(cfg):
    Ci, Co, H, W, k, s, p, d = cfg
    N = 2
    ge, OH, OW = _geom(N, Ci, Co, H, W, k, s, p, d)
    x = rnd(N, Ci, H, W, seed=11)
    gamma, beta, rm, rv, slope = bn_eval_params(Ci, 12)
    xt = fwd_xform_ref(x, gamma, beta, rm, rv, slope, "relu")
    dy = rnd(N, Co, OH, OW, seed=13)
    ref = torch.nn.grad.conv2d_weight(xt, (Co, Ci, k, k), dy, stride=s, padding=p, dilation=d)
    X, DY = cuda32(x), cuda32(dy)
    G = [cuda32(t) for t in (gamma, beta, rm, rv, slope)]
    xseg = {"p": ptr(X), "n_stride": Ci * H * W, "C": Ci, "xform": L.XF_BN_FWD,
            "act": L.ACT["relu"], "bn": bn_spec_eval(*G[:4])}
    dyseg = {"p": ptr(DY), "n_stride": Co * OH * OW, "C": Co, "xform": L.XF_PLAIN}
    DW = torch.zeros(Co, Ci, k, k, dtype=torch.float64, device=DEV)  # fp64 accumulators (isg.h)
    DB = torch.zeros(Co, dtype=torch.float64, device=DEV)
    call("isg_conv_wgrad", geom(**ge), vt([dyseg], N, OH, OW), vt([xseg], N, H, W), ptr(DW),
         ptr(DB), stream())
    DW, DB = DW.float(), DB.float()
    close(DW, ref, what="wgrad")
    close(DB, dy.sum((0, 2, 3)), what="dbias")


@pytest.mark.parametrize("xmode", ["eval", "train"])
@pytest.mark.parametrize("cfg", [(48, 128, 20, 24), (128, 48, 16, 16), (40, 20, 12, 36),
                                 (96, 48, 64, 64), (36, 48, 32, 32), (256, 128, 8, 8)])
@pytest.mark.parametrize("pwk", ["0", "1"])
def test_pw_wgrad_bn_bwd(cfg, xmode, pwk, monkeypatch):
    """1x1 weight gradient with the train plan's operands: dy = training-mode BatchNorm
    backward rebuilt on load from (grad, y) and consumer-side statistics, x = BatchNorm +
    PReLU on load (wgrad.hip pwg_kernel, and with ISG_PWK=1 pwk_kernel: ragged blocks and a
    partial last super-tile here), into replicas, against fp64."""
    monkeypatch.setenv("ISG_PWK", pwk)
    Ci, Co, H, W = cfg
    N = 2
    ge, OH, OW = _geom(N, Ci, Co, H, W, 1, 1, 0, 1)
    yraw = rnd(N, Co, H, W, seed=51) + 0.3
    gbn = rnd(N, Co, H, W, seed=52)
    gamma, beta, st, _ = _bn_train_state(yraw, gbn, 8)
    dy = _bn_bwd_ref(yraw, gbn, gamma)
    x = rnd(N, Ci, H, W, seed=53)
    xg, xb, xrm, xrv, xsl = bn_eval_params(Ci, 54)
    if xmode == "train":  # batch statistics, finalised by the consumer (the fast path)
        _, _, xst, _ = _bn_train_state(x, torch.zeros_like(x), 55)
        xrm, xrv = x.mean((0, 2, 3)), x.var((0, 2, 3), unbiased=False)
    xt = fwd_xform_ref(x, xg, xb, xrm, xrv, xsl, "prelu")
    ref = torch.nn.grad.conv2d_weight(xt, (Co, Ci, 1, 1), dy)
    Yr, Gb, GA, BE, ST = cuda32(yraw), cuda32(gbn), cuda32(gamma), cuda32(beta), rep_from(st)
    dyseg = {"p": ptr(Gb), "y": ptr(Yr), "n_stride": Co * H * W, "y_n_stride": Co * H * W,
             "C": Co, "xform": L.XF_BN_BWD, "bn": bn_spec_train(GA, BE, ST, N * H * W)}
    X = cuda32(x)
    XG = [cuda32(t) for t in (xg, xb, xrm, xrv, xsl)]
    xseg = {"p": ptr(X), "n_stride": Ci * H * W, "C": Ci, "xform": L.XF_BN_FWD,
            "act": L.ACT["prelu"], "slope": ptr(XG[4]), "bn": bn_spec_eval(*XG[:4])}
    if xmode == "train":
        XST = rep_from(xst)
        xseg["bn"] = bn_spec_train(XG[0], XG[1], XST, N * H * W)
    nw = Co * Ci
    stride_ = nw + Co + 19
    REP = torch.zeros(L.WREP * stride_, dtype=torch.float64, device=DEV)
    call("isg_conv_wgrad_rep", geom(**ge), vt([dyseg], N, H, W), vt([xseg], N, H, W),
         ptr(REP), ptr(REP[nw:]), stride_, L.WREP, stream())
    OUT = torch.full((stride_,), float("nan"), device=DEV)
    call("isg_sum_replicas", ptr(OUT), ptr(REP), stride_, L.WREP, stride_, stream())
    close(OUT[:nw].view(Co, Ci, 1, 1), ref, what="1x1 wgrad (BN-bwd dy)")
    # the BatchNorm-backward dy sums to ~0 per channel: bar relative to the summed magnitudes
    derr = (OUT[nw:nw + Co].double().cpu() - dy.sum((0, 2, 3))).abs().max().item()
    assert derr <= 1e-6 * dy.abs().sum((0, 2, 3)).max().item(), derr
    assert torch.all(OUT[nw + Co:] == 0)


@pytest.mark.parametrize("cfg", [(48, 128, 16, 16), (128, 48, 12, 20)])
def test_pw_bn_bwd_y_null(cfg):
    """a BatchNorm-backward segment with y = NULL (and y_n_stride = 0) means
    y = the segment's own input, at the input's image stride (isg.h isg_vseg). N = 2, so a
    y addressed with the zero stride would read image 0 for image 1. Through the 1x1 input
    gradient (pw_gemm.hip) and the 1x1 weight gradient (wgrad.hip), against fp64."""
    Ci, Co, H, W = cfg
    N = 2
    ge, OH, OW = _geom(N, Ci, Co, H, W, 1, 1, 0, 1)
    # g is also y: dy = gamma*rstd*(y - mean)*eps/(var + eps), so a spread near sqrt(eps)
    # keeps dy O(g) instead of a 1e-5 cancellation residue
    g = rnd(N, Co, H, W, seed=61, scale=0.003) + 0.2
    gamma, beta, st, _ = _bn_train_state(g, g, 62)
    dy = _bn_bwd_ref(g, g, gamma)
    w = rnd(Co, Ci, 1, 1, seed=63, scale=0.3)
    x = rnd(N, Ci, H, W, seed=64)
    Gb, GA, BE, ST = cuda32(g), cuda32(gamma), cuda32(beta), rep_from(st)
    dyseg = {"p": ptr(Gb), "y": 0, "n_stride": Co * H * W, "y_n_stride": 0,
             "C": Co, "xform": L.XF_BN_BWD, "bn": bn_spec_train(GA, BE, ST, N * H * W)}
    DX = torch.full((N, Ci, H, W), float("nan"), device=DEV)
    sk = sinks([{"p": ptr(DX), "n_stride": Ci * H * W, "c0": 0, "C": Ci, "mode": L.SINK_STORE}])
    call("isg_conv_dgrad", geom(**ge), vt([dyseg], N, H, W), ptr(cuda32(w)), sk, stream())
    close(DX, torch.nn.grad.conv2d_input((N, Ci, H, W), w, dy), what="1x1 dgrad (y NULL)")
    X = cuda32(x)
    xseg = {"p": ptr(X), "n_stride": Ci * H * W, "C": Ci, "xform": L.XF_PLAIN}
    DW = torch.zeros(Co, Ci, 1, 1, dtype=torch.float64, device=DEV)
    call("isg_conv_wgrad", geom(**ge), vt([dyseg], N, H, W), vt([xseg], N, H, W), ptr(DW), 0,
         stream())
    close(DW.float(), torch.nn.grad.conv2d_weight(x, (Co, Ci, 1, 1), dy), what="1x1 wgrad (y NULL)")


# folded residual tails (engine._fold_tails; isg.h residual forms): the fold's shapes
# (128^2 48 -> 16, 64^2 128 -> 48 and their input gradients) plus a ragged pixel count
RES = [(48, 16, 32, 32), (128, 48, 16, 16), (48, 16, 20, 12)]


def _bn_train_view(t, gamma, beta):
    """(train-mode BatchNorm of t, its statistics block [sum | sumsq | 0 | 0], mean)."""
    C = t.shape[1]
    st = torch.cat([t.sum((0, 2, 3)), (t * t).sum((0, 2, 3)), torch.zeros(2 * C, dtype=torch.float64)])
    mean = t.mean((0, 2, 3))
    rstd = 1 / torch.sqrt(t.var((0, 2, 3), unbiased=False) + 1e-5)
    return (t - mean[None, :, None, None]) * (gamma * rstd)[None, :, None, None] \
        + beta[None, :, None, None], st, mean


def _res_state(C, N, H, W, seed, rbn=False):
    """raw y, residual x, BN parameters and train statistics [sum | sumsq | 0 | 0] of y;
    rbn: the residual is itself a raw conv output with its own train-mode BatchNorm
    (returned as (gamma2, beta2, stats2, mean2))."""
    y = rnd(N, C, H, W, seed=seed) + 0.3
    xr = rnd(N, C, H, W, seed=seed + 1)
    gamma, beta, _, _, slope = bn_eval_params(C, seed + 2)
    by, st, mean = _bn_train_view(y, gamma, beta)
    r2 = None
    rv = xr
    if rbn:
        xr = xr * 0.7 - 0.2
        g2, b2, _, _, _ = bn_eval_params(C, seed + 3)
        rv, st2, mean2 = _bn_train_view(xr, g2, b2)
        r2 = (g2, b2, st2, mean2)
    return y, xr, gamma, beta, slope, st, mean, by + rv, r2


@pytest.mark.parametrize("act", ["prelu", "relu", "prelu-rbn", "prelu-pair"])
@pytest.mark.parametrize("cfg", RES)
def test_pw_residual_fwd(cfg, act):
    """Folded residual tail, forward: a 1x1 conv reading act(BN(y) + x) on load (BN_FWD
    segment with a residual y, statistics finalised by the consumer) that also writes the
    materialised act(BN(y) + x) to vtensor.mat — segment.py:75-77 then the next block's
    first conv — against fp64. "pair": a stacked sibling pair's two sinks (Graph.conv_pair,
    BottleneckUp_Res convs.0 + conv2 reading the tail, segment.py:326-331)."""
    C, Co, H, W = cfg
    N = 2
    ge, _, _ = _geom(N, C, Co, H, W, 1, 1, 0, 1)
    rbn = act.endswith("-rbn")
    pair = act.endswith("-pair")
    act = act.split("-")[0]
    y, xr, gamma, beta, slope, st, _, z, r2 = _res_state(C, N, H, W, 71, rbn)
    v = torch.where(z > 0, z, z * slope[None, :, None, None]) if act == "prelu" else z.clamp_min(0)
    w = rnd(Co, C, 1, 1, seed=74, scale=(2.0 / C) ** 0.5)
    b = rnd(Co, seed=75, scale=0.1)
    ref = F.conv2d(v, w, b)
    Y, XR, GA, BE, SL, ST = cuda32(y), cuda32(xr), cuda32(gamma), cuda32(beta), cuda32(slope), rep_from(st)
    seg = {"p": ptr(Y), "y": ptr(XR), "n_stride": C * H * W, "y_n_stride": C * H * W, "C": C,
           "xform": L.XF_BN_FWD, "act": L.ACT[act], "bn": bn_spec_train(GA, BE, ST, N * H * W)}
    if act == "prelu":
        seg["slope"] = ptr(SL)
    MAT = torch.full((N, C, H, W), float("nan"), device=DEV)
    B, Wt = cuda32(b), cuda32(w)  # kept alive: the call only sees their addresses
    vspec = {"s": [seg], "nseg": 1, "N": N, "H": H, "W": W, "mat": ptr(MAT),
             "mat_n_stride": C * H * W}
    if rbn:  # the residual's own BatchNorm (a two-BN tail)
        G2, B2, ST2 = cuda32(r2[0]), cuda32(r2[1]), rep_from(r2[2])
        vspec["rbn"] = bn_spec_train(G2, B2, ST2, N * H * W)
    a = struct(L.VTensor, vspec)
    if pair:  # channels [0, Ca) and [Ca, Co) to two buffers with their own statistics
        Ca = Co // 2 if Co % 8 == 0 else Co // 2 + 2
        parts = [(0, Ca), (Ca, Co - Ca)]
    else:
        parts = [(0, Co)]
    OUTS = [torch.full((N, c, H, W), float("nan"), device=DEV) for _, c in parts]
    OSTS = [rep_zeros(4 * c) for _, c in parts]
    sk = sinks([{"p": ptr(o), "n_stride": c * H * W, "c0": c0, "C": c, "mode": L.SINK_STORE,
                 "bias": ptr(B[c0:c0 + c]), "stats": ptr(st_)}
                for o, st_, (c0, c) in zip(OUTS, OSTS, parts)])
    call("isg_conv_fwd", geom(**ge), a, ptr(Wt), sk, stream())
    close(MAT, v, what="materialised block output")
    for o, st_, (c0, c) in zip(OUTS, OSTS, parts):
        r = ref[:, c0:c0 + c]
        close(o, r, what="1x1 on the folded tail")
        ost = rep_fold(st_, 4 * c)
        close(ost[:c], r.sum((0, 2, 3)), tol=4e-6, what="sum")
        close(ost[c:2 * c], (r * r).sum((0, 2, 3)), tol=4e-6, what="sumsq")


@pytest.mark.parametrize("parts", ["old+p2", "old", "p2", "none", "old+p2acc", "old+rbn", "old+p2-pair"])
@pytest.mark.parametrize("cfg", RES)
def test_pw_residual_dgrad(cfg, parts):
    """Folded residual tail, backward: the 1x1 input gradient's ACTBWD sink in residual
    form — v' = dx + old (what later consumers accumulated), g = v' * PReLU'(BN(y) + x)
    into p and p2, BatchNorm-backward sums of y and the PReLU slope gradient — the tail
    backward of segment.py:75-77 — against fp64. "pair": the gradient arrives as a stacked
    sibling pair's two segments (ConvPairOp.bwd: [Wa; Wb]^T [ga; gb])."""
    C, Co, H, W = cfg
    N = 2
    ge, _, _ = _geom(N, C, Co, H, W, 1, 1, 0, 1)
    rbn = "rbn" in parts
    y, xr, gamma, beta, slope, st, mean, z, r2 = _res_state(C, N, H, W, 81, rbn)
    dz = rnd(N, Co, H, W, seed=85)
    w = rnd(Co, C, 1, 1, seed=86, scale=(2.0 / C) ** 0.5)
    old = rnd(N, C, H, W, seed=87) if "old" in parts else torch.zeros(N, C, H, W, dtype=torch.float64)
    tot = torch.nn.grad.conv2d_input((N, C, H, W), w, dz) + old
    sl = slope[None, :, None, None]
    g = torch.where(z > 0, tot, tot * sl)
    Y, XR, GA, BE, SL, ST = cuda32(y), cuda32(xr), cuda32(gamma), cuda32(beta), cuda32(slope), rep_from(st)
    SG = rep_zeros(C)
    GB = torch.full((N, C, H, W), float("nan"), device=DEV)
    P2 = torch.full((N, C, H, W), float("nan"), device=DEV)
    OLD = cuda32(old)
    sk = {"p": ptr(GB), "n_stride": C * H * W, "c0": 0, "C": C, "mode": L.SINK_ACTBWD,
          "act": L.ACT["prelu"], "y": ptr(Y), "y_n_stride": C * H * W, "slope": ptr(SL),
          "slope_grad": ptr(SG), "bn": bn_spec_train(GA, BE, ST, N * H * W),
          "r": ptr(XR), "r_n_stride": C * H * W}
    if "old" in parts:
        sk["old"], sk["old_n_stride"] = ptr(OLD), C * H * W
    if rbn:  # the residual's own BatchNorm: its backward sums go to its statistics
        G2, B2, ST2 = cuda32(r2[0]), cuda32(r2[1]), rep_from(r2[2])
        sk["rbn"] = bn_spec_train(G2, B2, ST2, N * H * W)
    P2OLD = rnd(N, C, H, W, seed=88)
    if "p2acc" in parts:  # the residual term's gradient already holds a part: p2 += g
        P2.copy_(cuda32(P2OLD))
        sk["p2_accum"] = 1
    if "p2" in parts:
        sk["p2"], sk["p2_n_stride"] = ptr(P2), C * H * W
    DZ, Wt = cuda32(dz), cuda32(w)  # kept alive: the call only sees their addresses
    if "pair" in parts:  # two gradient segments, each its own buffer
        Ca = Co // 2 if Co % 8 == 0 else Co // 2 + 2
        DZS = [DZ[:, :Ca].contiguous(), DZ[:, Ca:].contiguous()]
        dysegs = [{"p": ptr(d), "n_stride": d.shape[1] * H * W, "C": d.shape[1], "xform": L.XF_PLAIN}
                  for d in DZS]
    else:
        dysegs = [{"p": ptr(DZ), "n_stride": Co * H * W, "C": Co, "xform": L.XF_PLAIN}]
    call("isg_conv_dgrad", geom(**ge), vt(dysegs, N, H, W), ptr(Wt), sinks([sk]), stream())
    close(GB, g, what="g (BN-output gradient of y)")
    if "p2acc" in parts:
        close(P2, g + P2OLD, what="p2 += g")
    elif "p2" in parts:
        assert torch.equal(P2, GB), "p2 must hold the same g"
    else:
        assert torch.isnan(P2).all()
    stf = rep_fold(ST, 4 * C).double().cpu()
    checks = [(stf[2 * C:3 * C], g, "gsum"), (stf[3 * C:], g * (y - mean[None, :, None, None]), "gxsum"),
              (rep_fold(SG, C).double().cpu(), torch.where(z > 0, 0 * z, z * tot), "slope grad")]
    if rbn:
        st2 = rep_fold(ST2, 4 * C).double().cpu()
        checks += [(st2[2 * C:3 * C], g, "residual gsum"),
                   (st2[3 * C:], g * (xr - r2[3][None, :, None, None]), "residual gxsum")]
    for got, terms, what in checks:
        err = (got - terms.sum((0, 2, 3))).abs().max().item()
        assert err <= 2e-6 * terms.abs().sum((0, 2, 3)).max().item() + 1e-9, (what, err)


def test_residual_forms_refused_elsewhere():
    """Every entry point but the 1x1 GEMM refuses the residual forms (isg.h) instead of
    silently dropping the residual: a 3x3 forward with a residual input, a 3x3 input
    gradient with a residual sink, a weight gradient with a residual input."""
    N, C, H, W = 2, 16, 8, 8
    ge, _, _ = _geom(N, C, C, H, W, 3, 1, 1, 1)
    X = torch.zeros(N, C, H, W, device=DEV)
    ST = rep_zeros(4 * C)
    G1 = torch.ones(C, device=DEV)
    seg = {"p": ptr(X), "y": ptr(X), "n_stride": C * H * W, "y_n_stride": C * H * W, "C": C,
           "xform": L.XF_BN_FWD, "bn": bn_spec_train(G1, G1, ST, N * H * W)}
    plain = {"p": ptr(X), "n_stride": C * H * W, "C": C, "xform": L.XF_PLAIN}
    out = sinks([{"p": ptr(X), "n_stride": C * H * W, "c0": 0, "C": C, "mode": L.SINK_STORE}])
    res_sink = sinks([{"p": ptr(X), "n_stride": C * H * W, "c0": 0, "C": C, "mode": L.SINK_ACTBWD,
                       "y": ptr(X), "y_n_stride": C * H * W, "r": ptr(X), "r_n_stride": C * H * W,
                       "bn": bn_spec_train(G1, G1, ST, N * H * W)}])
    W_ = torch.zeros(C, C, 3, 3, device=DEV)
    DW = torch.zeros(C * C * 9, dtype=torch.float64, device=DEV)
    lib = L.lib()
    import ctypes
    by = ctypes.byref
    assert lib.isg_conv_fwd(by(geom(**ge)), by(vt([seg], N, H, W)), ptr(W_), by(out), stream()) == -2  # ISG_ERR_UNSUPPORTED
    assert lib.isg_conv_dgrad(by(geom(**ge)), by(vt([plain], N, H, W)), ptr(W_), by(res_sink),
                              stream()) == -2  # ISG_ERR_UNSUPPORTED
    assert lib.isg_conv_wgrad(by(geom(**ge)), by(vt([plain], N, H, W)), by(vt([seg], N, H, W)),
                              ptr(DW), None, stream()) == -2  # ISG_ERR_UNSUPPORTED


@pytest.mark.parametrize("cfg", [DENSE[0], DENSE[1], DENSE[4], (16, 16, 24, 40, 3, 1, 1, 0)])
def test_conv_wgrad_replicated(cfg):
    """isg_conv_wgrad_rep adds into L.WREP replicas (the train plan's layout); folding them
    with isg_sum_replicas gives the plain weight gradient. Last case: depthwise (d=0 flag)."""
    Ci, Co, H, W, k, s, p, d = cfg
    depthwise = d == 0
    d = max(d, 1)
    N = 2
    if depthwise:
        Co = Ci
    ge, OH, OW = _geom(N, Ci, Co, H, W, k, s, p, d, groups=Ci if depthwise else 1)
    x = rnd(N, Ci, H, W, seed=41)
    dy = rnd(N, Co, OH, OW, seed=43)
    wshape = (Co, 1 if depthwise else Ci, k, k)
    ref = torch.nn.grad.conv2d_weight(x, wshape, dy, stride=s, padding=p, dilation=d,
                                      groups=Ci if depthwise else 1)
    X, DY = cuda32(x), cuda32(dy)
    nw = int(np.prod(wshape))
    stride_ = nw + Co + 37  # replica stride: weight, bias, padding (as in the flat layout)
    REP = torch.zeros(L.WREP * stride_, dtype=torch.float64, device=DEV)
    call("isg_conv_wgrad_rep", geom(**ge),
         vt([{"p": ptr(DY), "n_stride": Co * OH * OW, "C": Co, "xform": L.XF_PLAIN}], N, OH, OW),
         vt([{"p": ptr(X), "n_stride": Ci * H * W, "C": Ci, "xform": L.XF_PLAIN}], N, H, W),
         ptr(REP), ptr(REP[nw:]), stride_, L.WREP, stream())
    OUT = torch.full((stride_,), float("nan"), device=DEV)
    call("isg_sum_replicas", ptr(OUT), ptr(REP), stride_, L.WREP, stride_, stream())
    close(OUT[:nw].view(wshape), ref, what="replicated wgrad")
    close(OUT[nw:nw + Co], dy.sum((0, 2, 3)), what="replicated dbias")
    assert torch.all(OUT[nw + Co:] == 0)


DW_CFG = [  # (C, H, W, kh, kw, ph, pw, d)
    (16, 32, 32, 3, 3, 1, 1, 1),
    (48, 16, 24, 3, 3, 2, 2, 2),
    (48, 16, 16, 3, 3, 4, 4, 4),
    (48, 16, 16, 5, 1, 2, 0, 1),
    (48, 16, 16, 1, 5, 0, 2, 1),
    # the LDS-tiled kernel (16 x 64 tiles): partial tiles in both directions, dilation 4
    (16, 40, 84, 3, 3, 1, 1, 1),
    (24, 50, 84, 3, 3, 4, 4, 4),
    (8, 37, 132, 5, 1, 2, 0, 1),
]


@pytest.mark.parametrize("cfg", DW_CFG)
def test_depthwise(cfg):
    C, H, W, kh, kw, ph, pw, d = cfg
    N = 2
    ge = dict(N=N, Ci=C, H=H, W=W, Co=C, OH=H, OW=W, KH=kh, KW=kw, SH=1, SW=1, PH=ph, PW=pw,
              DH=d, DW=d, groups=C)
    x = rnd(N, C, H, W, seed=21)
    w = rnd(C, 1, kh, kw, seed=22, scale=0.4)
    b = rnd(C, seed=23, scale=0.1)
    gamma, beta, rm, rv, slope = bn_eval_params(C, 24)
    xt = fwd_xform_ref(x, gamma, beta, rm, rv, slope, "prelu")
    ref = F.conv2d(xt, w, b, padding=(ph, pw), dilation=d, groups=C)
    X, Wt, B = cuda32(x), cuda32(w), cuda32(b)
    G = [cuda32(t) for t in (gamma, beta, rm, rv, slope)]
    xseg = {"p": ptr(X), "n_stride": C * H * W, "C": C, "xform": L.XF_BN_FWD,
            "act": L.ACT["prelu"], "slope": ptr(G[4]), "bn": bn_spec_eval(*G[:4])}
    Y = torch.full((N, C, H, W), float("nan"), device=DEV)
    stats = rep_zeros(4 * C)
    sk = sinks([{"p": ptr(Y), "n_stride": C * H * W, "c0": 0, "C": C, "mode": L.SINK_STORE,
                 "bias": ptr(B), "stats": ptr(stats)}])
    call("isg_conv_fwd", geom(**ge), vt([xseg], N, H, W), ptr(Wt), sk, stream())
    close(Y, ref, what="dw fwd")
    stats = rep_fold(stats, 4 * C)
    close(stats[:C], ref.sum((0, 2, 3)), what="dw sum")
    # dgrad (plain dy -> plain store)
    dy = rnd(N, C, H, W, seed=25)
    dref = torch.nn.grad.conv2d_input((N, C, H, W), w, dy, padding=(ph, pw), dilation=d, groups=C)
    DY = cuda32(dy)
    DX = torch.full((N, C, H, W), float("nan"), device=DEV)
    sk = sinks([{"p": ptr(DX), "n_stride": C * H * W, "c0": 0, "C": C, "mode": L.SINK_STORE}])
    call("isg_conv_dgrad", geom(**ge),
         vt([{"p": ptr(DY), "n_stride": C * H * W, "C": C, "xform": L.XF_PLAIN}], N, H, W),
         ptr(Wt), sk, stream())
    close(DX, dref, what="dw dgrad")
    # wgrad
    wref = torch.nn.grad.conv2d_weight(xt, (C, 1, kh, kw), dy, padding=(ph, pw), dilation=d,
                                       groups=C)
    DWt = torch.zeros(C, 1, kh, kw, dtype=torch.float64, device=DEV)  # fp64 accumulators
    DB = torch.zeros(C, dtype=torch.float64, device=DEV)
    call("isg_conv_wgrad", geom(**ge),
         vt([{"p": ptr(DY), "n_stride": C * H * W, "C": C, "xform": L.XF_PLAIN}], N, H, W),
         vt([xseg], N, H, W), ptr(DWt), ptr(DB), stream())
    DWt, DB = DWt.float(), DB.float()
    close(DWt, wref, what="dw wgrad")
    close(DB, dy.sum((0, 2, 3)), what="dw dbias")


@pytest.mark.parametrize("ynull", [False, True], ids=["y", "ynull"])
@pytest.mark.parametrize("cfg", DW_CFG)
def test_depthwise_bwd_fused(cfg, ynull):
    """isg_depthwise_bwd (one launch, the dy tile staged once) against the two calls it
    replaces, bit for bit — dx through an ACTBWD sink with its BatchNorm-backward and PReLU
    slope sums, the weight/bias-gradient replicas — with dy the BatchNorm backward of the
    layer's output and x a BatchNorm + PReLU view; and the weight gradient against fp64.
    ynull: the fused call gets the BN_BWD segment with y = NULL (isg.h: y = p), the
    separate calls the same y spelled out — resolved at the entry point."""
    C, H, W, kh, kw, ph, pw, d = cfg
    N = 2
    ge = dict(N=N, Ci=C, H=H, W=W, Co=C, OH=H, OW=W, KH=kh, KW=kw, SH=1, SW=1, PH=ph, PW=pw,
              DH=d, DW=d, groups=C)
    yraw = rnd(N, C, H, W, seed=41) + 0.3
    gbn = rnd(N, C, H, W, seed=42)
    if ynull:  # y = p: the BatchNorm backward rebuilt from the gradient buffer itself
        yraw = gbn
    og, ob, st, _ = _bn_train_state(yraw, gbn, 43)
    dy = _bn_bwd_ref(yraw, gbn, og)
    x = rnd(N, C, H, W, seed=44)
    gamma, beta, rm, rv, slope = bn_eval_params(C, 45)
    xt = fwd_xform_ref(x, gamma, beta, rm, rv, slope, "prelu")
    w = rnd(C, 1, kh, kw, seed=46, scale=0.4)
    Yr, Gb, GA, BE, X, Wt = (cuda32(t) for t in (yraw, gbn, og, ob, x, w))
    G = [cuda32(t) for t in (gamma, beta, rm, rv, slope)]
    nw = C * kh * kw
    stride_ = nw + C + 3

    def run(fused):
        ST = rep_from(st)
        dyseg = {"p": ptr(Gb), "y": ptr(Yr), "n_stride": C * H * W, "y_n_stride": C * H * W,
                 "C": C, "xform": L.XF_BN_BWD, "bn": bn_spec_train(GA, BE, ST, N * H * W)}
        if ynull and fused:
            dyseg.update(y=0, y_n_stride=0)
        xseg = {"p": ptr(X), "n_stride": C * H * W, "C": C, "xform": L.XF_BN_FWD,
                "act": L.ACT["prelu"], "slope": ptr(G[4]), "bn": bn_spec_eval(*G[:4])}
        DX = torch.full((N, C, H, W), float("nan"), device=DEV)
        IST, SG = rep_zeros(4 * C), rep_zeros(C)
        bn_in = bn_spec_eval(*G[:4])
        bn_in["stats"] = ptr(IST)
        sk = sinks([{"p": ptr(DX), "n_stride": C * H * W, "c0": 0, "C": C, "mode": L.SINK_ACTBWD,
                     "act": L.ACT["prelu"], "y": ptr(X), "y_n_stride": C * H * W,
                     "slope": ptr(G[4]), "slope_grad": ptr(SG), "bn": bn_in}])
        REP = torch.zeros(L.WREP * stride_, dtype=torch.float64, device=DEV)
        if fused:
            call("isg_depthwise_bwd", geom(**ge), vt([dyseg], N, H, W), ptr(Wt), sk,
                 vt([xseg], N, H, W), ptr(REP), ptr(REP[nw:]), stride_, L.WREP, stream())
        else:
            call("isg_conv_dgrad", geom(**ge), vt([dyseg], N, H, W), ptr(Wt), sk, stream())
            call("isg_conv_wgrad_rep", geom(**ge), vt([dyseg], N, H, W), vt([xseg], N, H, W),
                 ptr(REP), ptr(REP[nw:]), stride_, L.WREP, stream())
        return DX, IST, SG, REP

    a, b = run(True), run(False)
    for u, v, what in zip(a, b, ("dx", "BN-backward sums", "slope gradient", "dW replicas")):
        assert not torch.isnan(u).any(), what
        assert torch.equal(u, v), f"fused {what} differs from the separate calls"
    if ynull:  # y = g: the BatchNorm backward of g w.r.t. itself is 0 up to rounding noise,
        return  # so only the bitwise agreement with the spelled-out y is meaningful
    OUT = torch.full((stride_,), float("nan"), device=DEV)
    call("isg_sum_replicas", ptr(OUT), ptr(a[3]), stride_, L.WREP, stride_, stream())
    wref = torch.nn.grad.conv2d_weight(xt, (C, 1, kh, kw), dy, padding=(ph, pw), dilation=d,
                                       groups=C)
    close(OUT[:nw].view(C, 1, kh, kw), wref, what="fused dw wgrad")


@pytest.mark.parametrize("cfg", [(16, 16, 2, 16, 16), (4, 4, 2, 32, 24), (16, 4, 4, 16, 16)])
def test_convT_fwd(cfg):
    Ci, Co, S, H, W = cfg
    N = 2
    K, P = 2 * S, S // 2
    x = rnd(N, Ci, H, W, seed=31)
    w = rnd(Ci, Co, K, K, seed=32, scale=0.2)
    b = rnd(Co, seed=33, scale=0.1)
    gamma, beta, rm, rv, slope = bn_eval_params(Ci, 34)
    xt = fwd_xform_ref(x, gamma, beta, rm, rv, slope, "relu")
    ref = F.conv_transpose2d(xt, w, b, stride=S, padding=P)
    OH, OW = ref.shape[2], ref.shape[3]
    X, Wt, B = cuda32(x), cuda32(w), cuda32(b)
    G = [cuda32(t) for t in (gamma, beta, rm, rv, slope)]
    xseg = {"p": ptr(X), "n_stride": Ci * H * W, "C": Ci, "xform": L.XF_BN_FWD,
            "act": L.ACT["relu"], "bn": bn_spec_eval(*G[:4])}
    Y = torch.full((N, Co, OH, OW), float("nan"), device=DEV)
    stats = rep_zeros(4 * Co)
    sk = sinks([{"p": ptr(Y), "n_stride": Co * OH * OW, "c0": 0, "C": Co, "mode": L.SINK_STORE,
                 "bias": ptr(B), "stats": ptr(stats)}])
    ge = dict(N=N, Ci=Ci, H=H, W=W, Co=Co, OH=OH, OW=OW, KH=K, KW=K, SH=S, SW=S, PH=P, PW=P,
              DH=1, DW=1, groups=1)
    call("isg_convT_fwd", geom(**ge), vt([xseg], N, H, W), ptr(Wt), sk, stream())
    close(Y, ref, what="convT")
    stats = rep_fold(stats, 4 * Co)
    close(stats[:Co], ref.sum((0, 2, 3)), what="convT sum")
    close(stats[Co:2 * Co], (ref * ref).sum((0, 2, 3)), what="convT sumsq")


@pytest.mark.parametrize("k", [2, 4])
def test_maxpool(k):
    N, C, H, W = 2, 6, 16, 24
    x = rnd(N, C, H, W, seed=41)
    x[0, 0, 0, :4] = 1.0  # ties: first max wins
    ref = F.max_pool2d(x, k, k)
    X = cuda32(x)
    Y = torch.full((N, C, H // k, W // k), float("nan"), device=DEV)
    xs = vt([{"p": ptr(X), "n_stride": C * H * W, "C": C, "xform": L.XF_PLAIN}], N, H, W)
    call("isg_maxpool_fwd", xs, k, ptr(Y), C * (H // k) * (W // k), stream())
    close(Y, ref, tol=0, what="maxpool")
    xr = x.clone().requires_grad_(True)
    dout = rnd(N, C, H // k, W // k, seed=42)
    F.max_pool2d(xr, k, k).backward(dout)
    DX = torch.full((N, C, H, W), float("nan"), device=DEV)
    sk = sinks([{"p": ptr(DX), "n_stride": C * H * W, "c0": 0, "C": C, "mode": L.SINK_STORE}])
    call("isg_maxpool_bwd", xs, k, ptr(cuda32(dout)), C * (H // k) * (W // k), sk, stream())
    close(DX, xr.grad, tol=0, what="maxpool bwd")


@pytest.mark.parametrize("act", ["prelu", "relu"])
@pytest.mark.parametrize("up", [False, True])
@pytest.mark.parametrize("H,W,accum", [(128, 132, True), (16, 14, False)],
                         ids=["128x132_2x4_accum", "16x14_quad"])
def test_tail(act, up, H, W, accum):
    """A >= 128^2 plane with W % 4 == 0 runs the 2x4-unit kernels (tail_fwd4 / tail_bwd4),
    16 x 14 the 2x2 form; accum: the term gradient adds onto an existing value (prefetched
    old value)."""
    N, C = 2, 8
    y = rnd(N, C, H, W, seed=51) + 0.2
    r = rnd(N, C, H // 2, W // 2, seed=52) if up else rnd(N, C, H, W, seed=52)
    gamma, beta, st0, slope = _bn_train_state(y, torch.zeros_like(y), 53)
    mean = y.mean((0, 2, 3), keepdim=True)
    var = y.var((0, 2, 3), unbiased=False, keepdim=True)
    bnout = (y - mean) / torch.sqrt(var + 1e-5) * gamma[None, :, None, None] + \
        beta[None, :, None, None]
    rr = F.interpolate(r, scale_factor=2, mode="nearest") if up else r
    pre = bnout + rr
    out = torch.where(pre > 0, pre, pre * slope[None, :, None, None]) if act == "prelu" \
        else pre.clamp_min(0)
    Y, R, GA, BE, SL = cuda32(y), cuda32(r), cuda32(gamma), cuda32(beta), cuda32(slope)
    ST = rep_from(st0)
    bnt = bn_spec_train(GA, BE, ST, N * H * W)
    t = {"term": [{"p": ptr(Y), "n_stride": C * H * W, "C": C, "xform": L.XF_BN_FWD,
                   "act": 0, "bn": bnt},
                  {"p": ptr(R), "n_stride": R[0].numel(), "C": C, "xform": L.XF_PLAIN}],
         "up": [0, 1 if up else 0, 0], "nterm": 2, "act": L.ACT[act], "slope": ptr(SL),
         "N": N, "C": C, "H": H, "W": W}
    O = torch.full((N, C, H, W), float("nan"), device=DEV)
    t["out"] = ptr(O)
    t["out_n_stride"] = C * H * W
    from instancesegmentation_amd import _lib as LL
    from tests.isg_helpers import struct
    call("isg_tail_fwd", struct(LL.Tail, t), stream())
    close(O, out, what="tail fwd")
    # backward
    dout = rnd(N, C, H, W, seed=54)
    g = torch.where(pre > 0, dout, dout * slope[None, :, None, None]) if act == "prelu" \
        else torch.where(pre > 0, dout, torch.zeros_like(dout))
    dr = F.avg_pool2d(g, 2) * 4 if up else g
    Gt = torch.full((N, C, H, W), float("nan"), device=DEV)
    DR0 = rnd(*tuple(r.shape), seed=55)
    DR = cuda32(DR0) if accum else torch.full(tuple(r.shape), float("nan"), device=DEV)
    if accum:
        dr = dr + DR0
    sg = rep_zeros(C)
    DO = cuda32(dout)  # held until the kernel has run
    tg = {"f": t, "dout": ptr(DO), "dout_n_stride": C * H * W, "g": ptr(Gt),
          "g_n_stride": C * H * W, "dterm": [None, ptr(DR), None],
          "dterm_n_stride": [0, R[0].numel(), 0], "dterm_accum": [0, 1 if accum else 0, 0],
          "slope_grad": ptr(sg)}
    call("isg_tail_bwd", struct(LL.TailGrad, tg), stream())
    torch.cuda.synchronize()
    close(Gt, g, what="tail g")
    close(DR, dr, what="tail dterm")
    ST, sg = rep_fold(ST, 4 * C), rep_fold(sg, C)
    close(ST[2 * C:3 * C], g.sum((0, 2, 3)), what="tail gsum")
    close(ST[3 * C:], (g * (y - mean)).sum((0, 2, 3)), what="tail gxsum")
    if act == "prelu":
        close(sg, torch.where(pre > 0, torch.zeros_like(pre), pre * dout).sum((0, 2, 3)),
              what="tail slope")


def test_bce_matches_golden(golden_dir):
    z = np.load(f"{golden_dir}/bce.npz")
    lg = torch.from_numpy(z["logits"]).to(DEV)
    tg = torch.from_numpy(z["target"]).to(DEV)
    n = lg.numel()
    acc = torch.zeros(1, dtype=torch.float64, device=DEV)
    dl = torch.empty_like(lg)
    call("isg_bce_sigmoid", ptr(lg), ptr(tg), n, ptr(acc), ptr(dl), 1.0 / n, stream())
    assert abs(acc.item() / n - float(z["loss"])) < 1e-6 * max(1, abs(float(z["loss"])))
    ref = torch.from_numpy(z["dlogits"]).double()
    got = dl.double().cpu()
    assert (got - ref).abs().max().item() < 1e-6 * ref.abs().max().item() + 1e-12
    # saturation semantics: logit 17 with y=0 -> zero gradient
    sat = (torch.from_numpy(z["logits"]) >= 17) & (torch.from_numpy(z["target"]) == 0)
    assert torch.all(got[sat] == ref[sat])


def test_adam_matches_golden(golden_dir):
    from tests.golden_util import SegmentFixture
    fx = SegmentFixture("segment20_n2_128.npz")
    z = np.load(f"{golden_dir}/adam_segment20.npz")
    p = torch.cat([torch.as_tensor(fx.params[k], dtype=torch.float32).reshape(-1)
                   for k in fx.param_names]).to(DEV)
    g = torch.from_numpy(fx.z["grad32"].copy()).to(DEV)
    live = torch.ones(p.numel(), dtype=torch.uint8)
    for i, k in enumerate(fx.param_names):
        if k in fx.grad_none:
            live[fx.offsets[i]:fx.offsets[i + 1]] = 0
    live = live.to(DEV)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for step, key in ((1, "step1"), (2, "step2")):
        call("isg_adam", ptr(p), ptr(g), ptr(m), ptr(v), ptr(live), p.numel(), step, 1e-3, 0.9,
             0.999, 1e-8, 0.0, stream())
        ref = torch.from_numpy(z[key])
        # within 2 ulp of torch's CPU Adam (its vectorised kernels may fuse multiply-adds)
        err = ((p.cpu() - ref).abs() / torch.clamp(ref.abs(), min=1.0)).max().item()
        assert err <= 2.5e-7, f"adam step {step}: {err}"


def test_adam_dev_counter_matches_host_steps():
    """isg_adam_dev: the device step counter advances on the stream before the update (the
    graph-replayable form). Three calls over a many-workgroup buffer match isg_adam with
    host steps 1, 2, 3 and the counter reads 3."""
    n = 3 * 1024 * 1024 + 17
    gen = torch.Generator().manual_seed(9)
    p0 = torch.randn(n, generator=gen)
    gs = [torch.randn(n, generator=gen) * 1e-2 for _ in range(3)]
    live = (torch.rand(n, generator=gen) > 0.1).to(torch.uint8).to(DEV)
    pa, pb = p0.clone().to(DEV), p0.clone().to(DEV)
    ma, va, mb, vb = (torch.zeros(n, device=DEV) for _ in range(4))
    step = torch.zeros(1, dtype=torch.int32, device=DEV)
    for k, g in enumerate(gs, 1):
        G = g.to(DEV)
        call("isg_adam", ptr(pa), ptr(G), ptr(ma), ptr(va), ptr(live), n, k, 1e-3, 0.9, 0.999,
             1e-8, 1e-4, stream())
        call("isg_adam_dev", ptr(pb), ptr(G), ptr(mb), ptr(vb), ptr(live), n, ptr(step), 1e-3,
             0.9, 0.999, 1e-8, 1e-4, stream())
    torch.cuda.synchronize()
    assert step.tolist() == [3]
    # the same formula; the bias corrections' pow runs on the host in one and on the device
    # in the other (a last-ulp difference of the double may survive the rounding to f32)
    for a_, b_ in ((pa, pb), (ma, mb), (va, vb)):
        assert ((a_ - b_).abs() / b_.abs().clamp_min(1e-3)).max().item() <= 3e-7


def test_paste_and_nms_bit_exact():
    from oracle import maskops_oracle as MO
    rng = np.random.Generator(np.random.PCG64(5))
    K, S, H, W = 12, 48, 97, 131
    prob = rng.uniform(0, 1, (K, S, S)).astype(np.float32)
    prob = np.where(prob > 0.35, prob, prob * 0.2).astype(np.float32)
    boxes = []
    for k in range(K):
        x0, y0 = rng.integers(-20, W - 10), rng.integers(-20, H - 10)
        boxes.append([x0, y0, x0 + rng.integers(8, 90), y0 + rng.integers(8, 90)])
    boxes = np.asarray(boxes, np.int32)
    ref = MO.paste_masks(prob, boxes, H, W)
    P = torch.from_numpy(prob).to(DEV)
    B = torch.from_numpy(boxes).to(DEV)
    O = torch.empty((K, H, W), dtype=torch.uint8, device=DEV)
    call("isg_mask_paste", ptr(P), K, S, ptr(B), H, W, ptr(O), stream())
    assert np.array_equal(O.cpu().numpy(), ref)
    keep_ref = MO.mask_nms(ref, 0.3)
    ws = L.lib().isg_mask_nms_workspace(K, H, W)
    work = torch.empty(ws, dtype=torch.uint8, device=DEV)
    sc = torch.empty(K, dtype=torch.float32, device=DEV)
    keep = torch.full((K,), -1, dtype=torch.int32, device=DEV)
    nk = torch.zeros(1, dtype=torch.int32, device=DEV)
    call("isg_mask_nms", ptr(O), K, H, W, 0.3, ptr(work), ptr(sc), ptr(keep), ptr(nk), stream())
    _, _, sref = MO.mask_stats(ref)
    assert np.array_equal(sc.cpu().numpy(), sref)
    assert np.array_equal(keep.cpu().numpy()[:nk.item()], keep_ref)


def _paste_nms_gpu(prob, boxes, H, W, thr):
    K, S = prob.shape[0], prob.shape[1]
    P = torch.from_numpy(prob).to(DEV)
    B = torch.from_numpy(boxes).to(DEV)
    O = torch.empty((K, H, W), dtype=torch.uint8, device=DEV)
    call("isg_mask_paste", ptr(P), K, S, ptr(B), H, W, ptr(O), stream())
    ws = L.lib().isg_mask_nms_workspace(K, H, W)
    work = torch.empty(max(ws, 1), dtype=torch.uint8, device=DEV)
    sc = torch.empty(K, dtype=torch.float32, device=DEV)
    keep = torch.full((K,), -1, dtype=torch.int32, device=DEV)
    nk = torch.zeros(1, dtype=torch.int32, device=DEV)
    call("isg_mask_nms", ptr(O), K, H, W, thr, ptr(work), ptr(sc), ptr(keep), ptr(nk), stream())
    # the product path's fused form (paste + NMS bit-packing in one pass) must agree bit
    # for bit with the two-call form
    O2 = torch.full((K, H, W), 77, dtype=torch.uint8, device=DEV)
    work2 = torch.full((max(ws, 1),), 0xAB, dtype=torch.uint8, device=DEV)
    sc2 = torch.empty(K, dtype=torch.float32, device=DEV)
    keep2 = torch.full((K,), -1, dtype=torch.int32, device=DEV)
    nk2 = torch.zeros(1, dtype=torch.int32, device=DEV)
    call("isg_mask_paste_nms", ptr(P), K, S, ptr(B), H, W, thr, ptr(O2), ptr(work2), ptr(sc2),
         ptr(keep2), ptr(nk2), stream())
    assert torch.equal(O2, O) and torch.equal(sc2, sc) and nk2.item() == nk.item()
    assert torch.equal(keep2[:nk.item()], keep[:nk.item()])
    return O.cpu().numpy(), sc.cpu().numpy(), keep.cpu().numpy()[:nk.item()]


def _person_probs(rng, K, S):
    """Ellipse-shaped high-probability blobs with noise (a crowded-scene stand-in)."""
    yy, xx = np.mgrid[0:S, 0:S].astype(np.float32) / S
    prob = np.empty((K, S, S), np.float32)
    for k in range(K):
        cy, cx = rng.uniform(0.35, 0.65, 2)
        ry, rx = rng.uniform(0.2, 0.45, 2)
        inside = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0
        noise = rng.uniform(0, 0.3, (S, S)).astype(np.float32)
        prob[k] = np.where(inside, 0.7 + noise, noise)
    return np.clip(prob, 0, 1).astype(np.float32)


@pytest.mark.parametrize("case", ["crowded16_480_to_1024", "max64", "max256", "single",
                                  "all_empty"])
def test_paste_and_nms_cases(case):
    """Config 4 (OCHuman-style crowded scene) at full size plus the edge cases: K at the
    kernel's maximum (64), one instance, and masks with no pixel above threshold. Paste
    and keep indices bit-exact to the build-defined oracle (parity with the reference
    unpinned: it has no NMS). max256: the kernel's instance capacity."""
    from oracle import maskops_oracle as MO
    rng = np.random.Generator(np.random.PCG64(21))
    if case == "crowded16_480_to_1024":
        K, S, H, W, thr = 16, 480, 1024, 1024, 0.5
        prob = _person_probs(rng, K, S)
        cx, cy = rng.integers(420, 600, K), rng.integers(420, 600, K)
        hw, hh = rng.integers(150, 260, K), rng.integers(200, 320, K)
        boxes = np.stack([cx - hw, cy - hh, cx + hw, cy + hh], 1).astype(np.int32)
    elif case == "max64":
        K, S, H, W, thr = 64, 32, 96, 128, 0.3
        prob = _person_probs(rng, K, S)
        x0, y0 = rng.integers(-10, W - 20, K), rng.integers(-10, H - 20, K)
        boxes = np.stack([x0, y0, x0 + rng.integers(10, 60, K), y0 + rng.integers(10, 60, K)],
                         1).astype(np.int32)
    elif case == "max256":
        K, S, H, W, thr = 256, 24, 120, 136, 0.4
        prob = _person_probs(rng, K, S)
        x0, y0 = rng.integers(-10, W - 20, K), rng.integers(-10, H - 20, K)
        boxes = np.stack([x0, y0, x0 + rng.integers(10, 60, K), y0 + rng.integers(10, 60, K)],
                         1).astype(np.int32)
    elif case == "single":
        K, S, H, W, thr = 1, 64, 80, 72, 0.5
        prob = _person_probs(rng, K, S)
        boxes = np.asarray([[5, 3, 60, 70]], np.int32)
    else:
        K, S, H, W, thr = 6, 40, 64, 64, 0.5
        prob = rng.uniform(0, 0.45, (K, S, S)).astype(np.float32)
        boxes = np.asarray([[0, 0, 40, 40]] * K, np.int32)
    ref = MO.paste_masks(prob, boxes, H, W)
    out, sc, keep = _paste_nms_gpu(prob, boxes, H, W, thr)
    assert np.array_equal(out, ref)
    _, _, sref = MO.mask_stats(ref)
    assert np.array_equal(sc, sref)
    keep_ref = MO.mask_nms(ref, thr)
    assert np.array_equal(keep, keep_ref), (keep, keep_ref)
    if case == "crowded16_480_to_1024":
        assert len(keep_ref) < K  # the overlap actually suppresses something
