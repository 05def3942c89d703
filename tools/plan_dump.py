"""Dump every recorded op of the Segment train plan with its conv geometry (CPU only).

    python tools/plan_dump.py [--size 1024] [--batch 2] [--cin 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from instancesegmentation_amd import _lib as L  # noqa: E402
from instancesegmentation_amd.engine import Plan  # noqa: E402
from instancesegmentation_amd.model.segment import Segment  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--cin", type=int, default=20)
    a = ap.parse_args()
    m = Segment(a.cin)
    shapes = [(a.batch, 3, a.size, a.size)]
    if a.cin == 20:
        shapes.append((a.batch, 17, a.size, a.size))
    p = Plan(m, shapes, True, True, [False] * len(shapes))
    for ph, ol in (("fwd", p.fwd), ("bwd", p.bwd)):
        for i, r in enumerate(ol.recs):
            geo = ""
            if r.kind in (L.OP_CONV_FWD, L.OP_CONV_DGRAD, L.OP_CONVT_FWD, L.OP_CONV_WGRAD):
                cls = L.WgradRec if r.kind == L.OP_CONV_WGRAD else L.ConvRec
                rec = cls.from_buffer_copy(r.body[:L.ctypes.sizeof(cls)])
                g = rec.g
                geo = (f"N{g.N} Ci{g.Ci} {g.H}x{g.W} -> Co{g.Co} {g.OH}x{g.OW} k{g.KH}x{g.KW} "
                       f"s{g.SH} p{g.PH} d{g.DH} grp{g.groups}")
                v = rec.dy if r.kind == L.OP_CONV_WGRAD else rec.a
                geo += " src[" + ",".join(f"C{v.s[j].C}xf{v.s[j].xform}" for j in range(v.nseg)) + "]"
                if r.kind != L.OP_CONV_WGRAD:
                    geo += " sinks[" + ",".join(f"m{rec.out.s[j].mode}" for j in range(rec.out.nsink)) + "]"
            fl = "".join(c for c, b in (("S", 1), ("J", 2), ("F", 4)) if r.flags & b)
            print(f"{ph} {i:4d} kind={r.kind:2d} {fl:3s} {r.label:34s} {geo}")


if __name__ == "__main__":
    main()
