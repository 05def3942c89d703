"""Probe (GPU): can HIP events with timing be recorded INSIDE a captured graph and read
back per replay (bench.py's in-step roofline timing of one op without splitting the step
into several graphs)? Times the same matmul three ways: events around a split graph,
events recorded inside one graph (external / plain), and back-to-back replays.

    python tools/probe/graph_event_probe.py
"""
import torch


def main():
    dev = torch.device("cuda", 0)
    a = torch.randn(4096, 4096, device=dev)
    b = torch.randn(4096, 4096, device=dev)
    c = torch.empty_like(a)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            torch.mm(a, b, out=c)
    torch.cuda.synchronize()
    # reference: events outside graphs around eager launches
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(10):
        e0.record()
        torch.mm(a, b, out=c)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"eager events: median {sorted(ts)[5] * 1e3:.1f} us")
    for ext in (True, False):
        try:
            kw = {"external": True} if ext else {}
            ev = [torch.cuda.Event(enable_timing=True, **kw) for _ in range(2)]
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                torch.mm(a, b, out=c)
                ev[0].record()
                torch.mm(a, b, out=c)
                ev[1].record()
                torch.mm(a, b, out=c)
            ts = []
            for _ in range(10):
                g.replay()
                torch.cuda.synchronize()
                ts.append(ev[0].elapsed_time(ev[1]))
            print(f"in-graph events (external={ext}): median {sorted(ts)[5] * 1e3:.1f} us, "
                  f"all {[round(t * 1e3, 1) for t in ts]}")
        except Exception as e:  # noqa: BLE001 — a probe reports what the runtime refuses
            print(f"in-graph events (external={ext}): {type(e).__name__}: {e}")
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
