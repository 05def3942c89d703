"""Fused mask head (isg_mask_head_fwd / _bwd, csrc/mask_head.hip) against an fp64 torch
restatement of the reference's two layers (segment.py:435-438, 504-505:
ConvTranspose2d(16 -> 4, k8, s4, p2) then Conv2d(4 -> 1, 3x3, p1)), forward and backward
(input gradient through a STORE and an ACCUM sink, all four parameter gradients summed
over the weight-gradient replicas), on whole and partial tiles."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from instancesegmentation_amd import _lib as L
from tests.isg_helpers import call, sinks, struct, vt

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(N, Hi, Wi, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, 16, Hi, Wi, generator=g)
    w1 = torch.randn(16, 4, 8, 8, generator=g) * 0.05
    b1 = torch.randn(4, generator=g) * 0.1
    w2 = torch.randn(1, 4, 3, 3, generator=g) * 0.3
    b2 = torch.randn(1, generator=g) * 0.1
    dl = torch.randn(N, 1, 4 * Hi, 4 * Wi, generator=g)
    return x, w1, b1, w2, b2, dl


def _ref(x, w1, b1, w2, b2, dl):
    P = [t.double().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    y = F.conv2d(F.conv_transpose2d(P[0], P[1], P[2], stride=4, padding=2), P[3], P[4], padding=1)
    y.backward(dl.double())
    return y.detach(), [p.grad for p in P]


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-12)


@pytest.mark.parametrize("N,Hi,Wi", [(2, 8, 16), (1, 5, 7), (2, 17, 33), (1, 64, 64)])
def test_mask_head_fwd_bwd(N, Hi, Wi):
    x, w1, b1, w2, b2, dl = _case(N, Hi, Wi, Hi * 100 + Wi)
    ref_y, ref_g = _ref(x, w1, b1, w2, b2, dl)
    d = {k: v.to(DEV).contiguous() for k, v in dict(x=x, w1=w1, b1=b1, w2=w2, b2=b2, dl=dl).items()}
    OH, OW = 4 * Hi, 4 * Wi
    out = torch.full((N, 1, OH, OW), 7.0, device=DEV)
    # two input segments (channels 0-9, 10-15) exercise the vtensor segment split
    xa, xb = d["x"][:, :10].contiguous(), d["x"][:, 10:].contiguous()
    seg = lambda t, C: {"p": t.data_ptr(), "n_stride": C * Hi * Wi, "C": C, "xform": L.XF_PLAIN}
    ring = torch.full((N, L.head_ring_floats(Hi, Wi)), float("nan"), device=DEV)
    base = {"x": {"s": [seg(xa, 10), seg(xb, 6)], "nseg": 2, "N": N, "H": Hi, "W": Wi},
            "w1": d["w1"].data_ptr(), "b1": d["b1"].data_ptr(), "w2": d["w2"].data_ptr(),
            "b2": d["b2"].data_ptr(), "N": N, "Hi": Hi, "Wi": Wi, "ring": ring.data_ptr()}
    a = struct(L.MaskHead, dict(base, out=out.data_ptr(), out_n_stride=OH * OW))
    call("isg_mask_head_fwd", a, L.stream_ptr())
    e = _rel(out, ref_y)
    print(f"{N}x16x{Hi}x{Wi}: logits rel err {e:.2e}")
    assert e < 2e-6
    # the ring: the un-cropped intermediate one pixel outside the image (isg.h)
    full = F.conv_transpose2d(x.double(), w1.double(), b1.double(), stride=4)  # no crop: p = -2
    OHf = full.shape[2]
    rg = ring.view(N, 4, -1).double().cpu()
    exp = torch.cat([full[:, :, 1, 1:OW + 3], full[:, :, OH + 2, 1:OW + 3],
                     full[:, :, 2:OH + 2, 1], full[:, :, 2:OH + 2, OW + 2]], 2)
    assert OHf == OH + 4 and rg.shape == exp.shape
    er = (rg - exp).abs().max().item() / max(exp.abs().max().item(), 1e-12)
    print(f"ring rel err {er:.2e}")
    assert er < 2e-6
    # backward: dx of channels 0-9 STOREd, 10-15 ACCUMulated onto a preset value
    dxa = torch.full((N, 10, Hi, Wi), 5.0, device=DEV)
    pre = torch.randn(N, 6, Hi, Wi, device=DEV)
    dxb = pre.clone()
    R, nrep = 4096 + 4 + 36 + 1, L.WREP
    rep = torch.zeros(nrep * R, dtype=torch.float64, device=DEV)  # fp64 replicas (isg.h)
    rp = rep.data_ptr()
    sk = [{"p": dxa.data_ptr(), "n_stride": 10 * Hi * Wi, "c0": 0, "C": 10, "mode": L.SINK_STORE},
          {"p": dxb.data_ptr(), "n_stride": 6 * Hi * Wi, "c0": 10, "C": 6, "mode": L.SINK_ACCUM}]
    b = struct(L.MaskHead, dict(base, dout=d["dl"].data_ptr(), dout_n_stride=OH * OW,
                                dx={"s": sk, "nsink": 2}, dw1=rp, db1=rp + 8 * 4096,
                                dw2=rp + 8 * 4100, db2=rp + 8 * 4136, rep_stride=R, nrep=nrep))
    call("isg_mask_head_bwd", b, L.stream_ptr())
    tot = rep.view(nrep, R).sum(0).float().cpu()
    dx = torch.cat([dxa.cpu(), (dxb - pre).cpu()], 1)
    errs = {"dx": _rel(dx, ref_g[0]), "dw1": _rel(tot[:4096].view(16, 4, 8, 8), ref_g[1]),
            "db1": _rel(tot[4096:4100], ref_g[2]), "dw2": _rel(tot[4100:4136].view(1, 4, 3, 3), ref_g[3]),
            "db2": _rel(tot[4136:4137], ref_g[4])}
    print({k: f"{v:.1e}" for k, v in errs.items()})
    assert all(v < 2e-5 for v in errs.values()), errs


@pytest.mark.parametrize("N,Hi,Wi", [(2, 8, 16), (1, 17, 33), (2, 64, 64)])
def test_mask_head_bwd_slab_fold_matches_atomics(N, Hi, Wi):
    """The convT weight gradient through the per-workgroup slab (isg_mask_head.dw1_part)
    and the later fold (isg_mask_head_fold, the train plan's side-stream op) equals the
    in-kernel fp64 atomics bit for bit (both are exact fp64 sums of the same fp32
    partials), and every other output is unchanged."""
    x, w1, b1, w2, b2, dl = _case(N, Hi, Wi, 7 * Hi + Wi)
    d = {k: v.to(DEV).contiguous() for k, v in dict(x=x, w1=w1, b1=b1, w2=w2, b2=b2, dl=dl).items()}
    OH, OW = 4 * Hi, 4 * Wi
    ring = torch.zeros(N, L.head_ring_floats(Hi, Wi), device=DEV)
    base = {"x": {"s": [{"p": d["x"].data_ptr(), "n_stride": 16 * Hi * Wi, "C": 16,
                         "xform": L.XF_PLAIN}], "nseg": 1, "N": N, "H": Hi, "W": Wi},
            "w1": d["w1"].data_ptr(), "b1": d["b1"].data_ptr(), "w2": d["w2"].data_ptr(),
            "b2": d["b2"].data_ptr(), "N": N, "Hi": Hi, "Wi": Wi, "ring": ring.data_ptr()}
    out = torch.zeros(N, 1, OH, OW, device=DEV)
    call("isg_mask_head_fwd", struct(L.MaskHead, dict(base, out=out.data_ptr(), out_n_stride=OH * OW)),
         L.stream_ptr())
    nslab = L.head_part_floats(N, Hi, Wi)
    assert nslab == L.lib().isg_mask_head_part_floats(N, Hi, Wi)
    R, nrep = 4096 + 4 + 36 + 1, L.WREP

    def run(slab):
        dx = torch.full((N, 16, Hi, Wi), float("nan"), device=DEV)
        rep = torch.zeros(nrep * R, dtype=torch.float64, device=DEV)
        part = torch.full((nslab,), float("nan"), device=DEV)
        rp = rep.data_ptr()
        sk = [{"p": dx.data_ptr(), "n_stride": 16 * Hi * Wi, "c0": 0, "C": 16, "mode": L.SINK_STORE}]
        b = struct(L.MaskHead, dict(base, dout=d["dl"].data_ptr(), dout_n_stride=OH * OW,
                                    dx={"s": sk, "nsink": 1}, dw1=rp, db1=rp + 8 * 4096,
                                    dw2=rp + 8 * 4100, db2=rp + 8 * 4136, rep_stride=R, nrep=nrep,
                                    dw1_part=part.data_ptr() if slab else None))
        call("isg_mask_head_bwd", b, L.stream_ptr())
        if slab:
            call("isg_mask_head_fold", b, L.stream_ptr())
        return dx, rep.view(nrep, R).sum(0)

    (dxa, ta), (dxb, tb) = run(True), run(False)
    assert torch.equal(dxa, dxb)
    assert torch.equal(ta, tb), (ta - tb).abs().max().item()
    ref_y, ref_g = _ref(x, w1, b1, w2, b2, dl)
    assert _rel(ta[:4096].float().view(16, 4, 8, 8), ref_g[1]) < 2e-5
