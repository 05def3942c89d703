"""Headline benchmark: train images/s of the reference model (Segment(20) = RGB + 17
keypoint heatmaps, BCE + Adam; train_instance.py:294-382) on synthetic COCO-person
1024x1024 batches, bs 2 per GPU (BASELINE.json configs[1]; configs[2] when launched on
8 GPUs is the same per-replica work). One process per GPU (torchrun), image-batch data
parallel with an RCCL gradient all-reduce.

    python bench.py [--gpus N] [--steps K] [--warmup W]

Prints ONE JSON line (rank 0) with the driver's contract fields plus:
  roofline     — the dominant kernel (largest share of step time, picked by a per-op
                 timing pass), timed live in every timed step by two timestamp launches
                 around it in its place in the step (minus a calibration pair's cost);
  cpu_baseline — the oracle's CPU restatement (fp32 torch eager) of the same train step,
                 timed on this host's cores (rank 0, N=1 only).
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist

PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix 157.3 TF (spec)
PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2, help="images per GPU")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--cin", type=int, default=20, choices=(3, 20))
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--profile-ops", default="", help="write per-op timing table to this path")
    ap.add_argument("--dominant", default="",
                    help="phase:label of the roofline op (skips the per-op timing pass, so a "
                         "profiler sees training steps only), e.g. bwd:d_out0")
    ap.add_argument("--eager", action="store_true", help="(the default) no HIP graph capture")
    ap.add_argument("--graph", action="store_true",
                    help="capture the step into HIP graphs (round 6 measured the executor's "
                         "eager issue faster: DESIGN §3.6)")
    ap.add_argument("--no-infer", action="store_true", help="skip the inference leg")
    ap.add_argument("--input", default="keypoints", choices=("keypoints", "heatmaps"),
                    help="what the data loader hands the step: keypoints (the 17 heatmaps "
                         "synthesised inside the stem, SURVEY.md §8f #1) or dense heatmaps")
    ap.add_argument("--no-dense-leg", action="store_true",
                    help="skip the second timing with dense heatmap inputs")
    ap.add_argument("--no-dp-leg", action="store_true",
                    help="skip the timing of the data-parallel step structure at world size 1")
    return ap.parse_args()


def launch_ranks(args):
    """`python bench.py --gpus N` outside a launcher: start N ranks (one process per GPU)
    with torch.distributed.run and exit with its status. This parent never touches the
    GPU (the children initialise HIP themselves)."""
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} "
                         "rank(s); run it without a launcher or with --nproc-per-node "
                         f"{args.gpus}")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def op_timing(trainer, reps=20):
    """Device time of every recorded op alone: the op repeated `reps` times inside one
    captured HIP graph, bracketed by HIP events (host launch latency excluded)."""
    from instancesegmentation_amd import _lib as L
    rows = []
    for phase, ol in (("fwd", trainer.plan.fwd), ("bwd", trainer.plan.bwd)):
        for i, r in enumerate(ol.recs):
            sub = ol.slice(i, i + 1)
            sub.run(trainer.table, L.stream_ptr(), L.side_stream_ptr())
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(reps):
                    sub.run(trainer.table, L.stream_ptr(), L.side_stream_ptr())
            graph.replay()
            stream = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            graph.replay()
            e1.record(stream)
            e1.synchronize()
            del graph
            rows.append(dict(phase=phase, idx=i, label=r.label, kind=r.kind,
                             ms=e0.elapsed_time(e1) / reps, flops=r.flops, nbytes=r.nbytes))
    # leave the trainer's arenas consistent: rerun a full fwd/bwd afterwards
    return rows


def roofline_of(rec, ms):
    ai = rec.flops / rec.nbytes if rec.nbytes else 0.0
    ridge = PEAK_F32_MFMA_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)
    if rec.flops and ai >= ridge:
        ach = rec.flops / (ms * 1e-3) / 1e12
        return {"bound": "mfma", "achieved": round(ach, 3), "peak": PEAK_F32_MFMA_TFLOPS,
                "unit": "TFLOP/s", "frac": round(ach / PEAK_F32_MFMA_TFLOPS, 4), "traffic": None}
    ach = rec.nbytes / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": None}


def pmc_traffic(label, args):
    """HBM bytes per launch of the dominant op from the committed PMC pass
    (profiles/traffic.json, written by tools/kbench/traffic.sh: 2*FETCH_SIZE + WRITE_SIZE,
    the gfx950 correction of MI355X_MICROARCH.md), or None when no pass covers this op at
    this configuration. PMC counters need rocprofv3 as the parent process, so they cannot
    be read live inside this run."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "traffic.json")
    try:
        with open(path) as f:
            runs = json.load(f)
    except (OSError, ValueError):
        return None
    for r in runs:
        if r.get("label") == label and r.get("config") == [args.batch, args.cin, args.size]:
            return r.get("hbm_bytes_per_launch")
    return None


# the stem's two 5x5 s2 convs (init_head_s4, segment.py:19-31): layer 2 (16 -> 16) in all
# three directions, layer 1's RGB part forward and weight gradient
BACKBONE_OPS = [("fwd", "init_conv.layer2"), ("bwd", "dx_init_conv.layer2"),
                ("bwd", "dw_init_conv.layer2"), ("fwd", "init_conv.layer1"),
                ("bwd", "dw_init_conv.layer1")]


def stamp_op(trainer, phase, label, args, rows=None):
    """The roofline of one recorded op timed in place: the step re-run with OP_STAMP records
    around it (Trainer.stamp_at), args.steps steps after 2 warm-up steps; a side-stream op (a
    weight gradient) is moved onto the main stream for its bracket. In place, the op shares
    the chip with whatever the side stream runs beside it (the stem's layer-2 input and
    weight gradients overlap each other); `rows` (the per-op pass: the op alone, 20 launches
    in a graph) adds the kernel's own time as `alone_ms` / `alone_frac`."""
    ol = trainer.plan.fwd if phase == "fwd" else trainer.plan.bwd
    idx = next((i for i, r in enumerate(ol.recs) if r.label == label), None)
    if idx is None:
        return None
    rec = ol.recs[idx]
    trainer.stamp_at = (phase, idx)
    if args.graph:
        trainer.capture()
    for _ in range(2):
        trainer.step(loss=False)
    torch.cuda.synchronize()
    trainer.stamp_reset()
    for _ in range(args.steps):
        trainer.step(loss=False)
    torch.cuda.synchronize()
    raw, brk, _ = trainer.stamp_times(args.steps)
    ms = max(raw - brk, 1e-6)
    r = roofline_of(rec, ms)
    r["kernel"] = f"{phase}:{label}"
    r["avg_ms"] = round(ms, 4)
    r["gflop"] = round(rec.flops / 1e9, 4)
    r["traffic"] = pmc_traffic(label, args)
    alone = next((x["ms"] for x in rows or [] if x["phase"] == phase and x["label"] == label), None)
    if alone:
        a = roofline_of(rec, alone)
        r["alone_ms"] = round(alone, 4)
        r["alone_frac"] = a["frac"]
    return r


def infer_scene(H, W, persons, dups, seed=11):
    """A crowded synthetic image (BASELINE config 4, OCHuman-style): `persons` overlapping
    person boxes with 17 keypoints each, plus `dups` repeated detections of the same people
    with a few-pixel jitter of box (+/-3 px) and keypoints (+/-2 px) — an over-complete
    detector's output, so mask-NMS ranks and compares genuinely different masks (exact
    repeats would make every duplicate's IoU exactly 1)."""
    import numpy as np
    rng = np.random.Generator(np.random.PCG64(seed))
    img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    boxes, kps = [], []
    for _ in range(persons):
        cx, cy = rng.uniform(0.3, 0.7) * W, rng.uniform(0.3, 0.7) * H
        bw, bh = rng.uniform(0.15, 0.3) * W, rng.uniform(0.35, 0.6) * H
        b = [int(cx - bw / 2), int(cy - bh / 2), int(cx + bw / 2), int(cy + bh / 2)]
        kp = np.zeros((17, 3))
        kp[:, 0] = rng.uniform(b[0], b[2], 17)
        kp[:, 1] = rng.uniform(b[1], b[3], 17)
        kp[:, 2] = rng.uniform(size=17) < 0.8
        boxes.append(b)
        kps.append(kp)
    for i in range(dups):  # repeated, jittered detections of the same people
        j = i % persons
        boxes.append([v + int(rng.integers(-3, 4)) for v in boxes[j]])
        kps.append(kps[j] + np.array([rng.uniform(-2, 2), rng.uniform(-2, 2), 0.0]))
    return img, np.asarray(boxes), np.asarray(kps)


def infer_bench(dev, reps=20):
    """BASELINE.json's inference half ("infer masks/sec + NMS p50") on config 4
    (OCHuman-style crowded scene): one 1024x1024 image with K=16 person instances (8 people
    + 8 repeated detections) through the infer.py product path as ONE HIP graph
    (instancesegmentation_amd/infer.py): per-instance crop to 480x480, Segment(20) eval with
    BatchNorm folded and the 17 keypoint heatmaps synthesised in its stem, sigmoid, paste-back onto
    the 1024x1024 canvas, greedy mask-NMS at IoU 0.5. masks/s = K / (graph time per
    image, inputs resident); NMS p50 = the NMS launches alone, on the same masks."""
    import numpy as np
    from instancesegmentation_amd import _lib as L
    from instancesegmentation_amd.infer import InstanceSegmenter
    from instancesegmentation_amd.model.segment import Segment
    K, H, W = 16, 1024, 1024
    torch.manual_seed(99)
    model = Segment(20)
    img, boxes, kps = infer_scene(H, W, 8, 8)
    # BatchNorm running statistics calibrated on the scene's own instances (one train-mode
    # pass with momentum 1: running = batch statistics), so the eval-mode network of the
    # random-init weights is well conditioned and its masks are not all-empty / all-full
    calib = InstanceSegmenter(model, (H, W), max_instances=K, device=dev, capture=False)
    calib.load(img, boxes, kps)
    calib.run()
    model = model.to(dev).train()
    bns = [m for m in model.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    for b in bns:
        b.momentum = 1.0
    with torch.no_grad():
        model(calib.x[:len(boxes)].contiguous(), calib.keypoints[:len(boxes)].contiguous())
    for b in bns:
        b.momentum = 0.1
    # the last conv's bias +3: every instance's mask then covers most of its crop window
    # (random-init logits are O(1)), a stand-in for a trained model's person masks, so the
    # jittered repeat detections overlap at IoU ~0.9 and the NMS really suppresses
    # (config 4's heavy-overlap case; with the raw random-init head no pair reached 0.5)
    with torch.no_grad():
        model.bottle6_2.bias.add_(3.0)
    model.eval()
    del calib
    eng = InstanceSegmenter(model, (H, W), max_instances=K, iou_thr=0.5, device=dev)
    eng.load(img, boxes, kps)
    for _ in range(3):
        eng.run()
    torch.cuda.synchronize(dev)
    t_pipe = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.run()
        e1.record()
        e1.synchronize()
        t_pipe.append(e0.elapsed_time(e1))
    masks, keep, scores = eng.result()
    nonempty = int((scores > 0).sum())
    # pairs above the IoU threshold among all instances (exact integer IoU, the NMS's own)
    b = (masks >= 128).reshape(len(boxes), -1).float()
    inter = b @ b.t()
    cnt = b.sum(1)
    union = cnt[:, None] + cnt[None, :] - inter
    iou = torch.where(union > 0, inter / union.clamp(min=1), torch.zeros_like(inter))
    pairs = int(torch.triu(iou > 0.5, diagonal=1).sum().item())
    st = L.stream_ptr(dev)
    t_nms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        L.check(L.lib().isg_mask_nms(eng.masks.data_ptr(), K, H, W, 0.5, eng.work.data_ptr(),
                                     eng.scores.data_ptr(), eng.keep.data_ptr(),
                                     eng.nkeep.data_ptr(), st), "mask_nms")
        e1.record()
        e1.synchronize()
        t_nms.append(e0.elapsed_time(e1))
    ms = float(np.median(t_pipe))
    return {"metric": "infer masks/sec (crop 480x480 + Segment(20) eval with the keypoint heatmaps "
                      "synthesised in its stem, BN folded + sigmoid + paste 1024x1024 + mask-NMS "
                      "IoU 0.5, one HIP graph)",
            "masks_per_s": round(K / (ms * 1e-3), 1), "ms_per_image": round(ms, 3),
            "nms_p50_ms": round(float(np.median(t_nms)), 4), "instances": K, "kept": len(keep),
            "suppressed": K - len(keep), "pairs_iou_gt_0.5": pairs, "nonempty_masks": nonempty,
            "config": "OCHuman-crowded synthetic: 8 people + 8 jittered repeat detections; "
                      "random-init Segment(20), BN statistics calibrated on the scene, head "
                      "bias +3 (masks cover the crop windows)",
            "dtype": "f32", "data": "synthetic"}


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), for the cpu_baseline record."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(args):
    """Oracle (torch eager fp32 CPU) train step on the same config: bounded sample."""
    import numpy as np
    from oracle import segment_oracle
    from oracle.seeding import synth_params
    from instancesegmentation_amd.model.segment import Segment
    threads = len(os.sched_getaffinity(0))
    env_t = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env_t:
        threads = min(threads, env_t)
    torch.set_num_threads(threads)
    m = Segment(args.cin)
    shapes = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    params = synth_params(shapes, 1)
    from instancesegmentation_amd.data import synthetic_batch
    img, hm, mask = synthetic_batch(args.batch, args.size, args.size, seed=3,
                                    with_heatmaps=args.cin == 20)
    x = np.concatenate([img, hm], 1) if hm is not None else img
    P = {k: torch.as_tensor(v).float() if np.issubdtype(np.asarray(v).dtype, np.floating)
         else torch.as_tensor(v) for k, v in params.items()}
    steps, t_total = 0, 0.0
    segment_oracle.train_step(P, x, mask, torch.float32)  # warm-up
    while t_total < args.cpu_seconds or steps < 2:
        t0 = time.perf_counter()
        segment_oracle.train_step(P, x, mask, torch.float32)
        t_total += time.perf_counter() - t0
        steps += 1
    return {"value": round(steps * args.batch / t_total, 3), "unit": "images/s",
            "cores": threads, "cpu_model": cpu_model(), "kind": "port",
            "sample": f"{steps} fp32 train steps (fwd+bwd) of Segment({args.cin}) at "
                      f"bs{args.batch} {args.size}x{args.size} on {threads} host threads"}


def train_leg(args, dev, world, rank, keypoints, roofline, dp_plan=None):
    """Time args.steps captured train steps (after args.warmup) on one input form; the
    dominant op (per-op timing pass) is bracketed by timestamp launches inside every timed
    step when `roofline`. dp_plan: the data-parallel step structure (Trainer dp_plan)."""
    from instancesegmentation_amd.data import device_batch
    from instancesegmentation_amd.model.segment import Segment
    from instancesegmentation_amd.train import Trainer

    torch.manual_seed(1234)
    model = Segment(args.cin)
    xs, mask = device_batch(args.batch, args.size, args.size, dev, seed=100 + rank, cin=args.cin,
                            keypoints=keypoints and args.cin == 20)
    in_shapes = [tuple(x.shape) for x in xs]
    trainer = Trainer(model, args.batch, in_shapes, device=dev, dp_plan=dp_plan)
    trainer.step(xs, mask)
    torch.cuda.synchronize()

    # ---- dominant op (per-op timing pass, untimed) ----------------------------------
    dom = None
    rows = None
    if roofline and args.dominant:
        ph, lab = args.dominant.split(":", 1)
        ol = trainer.plan.fwd if ph == "fwd" else trainer.plan.bwd
        dom = (ph, next(i for i, r in enumerate(ol.recs) if r.label == lab))
    elif roofline:
        rows = op_timing(trainer)
        if args.profile_ops and rank == 0:
            with open(args.profile_ops, "w") as f:
                tot = sum(r["ms"] for r in rows)
                for r in sorted(rows, key=lambda r: -r["ms"]):
                    f.write(f"{r['phase']} {r['idx']:4d} {r['ms']*1e3:9.1f}us "
                            f"{100*r['ms']/tot:5.1f}% {r['label']} kind={r['kind']} "
                            f"flops={r['flops']} bytes={r['nbytes']}\n")
        best = max(rows, key=lambda r: r["ms"])
        dom = (best["phase"], best["idx"])
    trainer.step()  # restore a consistent state after the per-op pass
    torch.cuda.synchronize()
    # capture the step into ONE HIP graph (world 1); the dominant op runs between two
    # timestamp launches (OP_STAMP: the 100 MHz chip counter) in its place in the step, plus
    # a back-to-back calibration pair — ROCm rejects timing events under graph capture, and
    # cutting the step into graphs around the op (the round-4 form) added a graph boundary
    # and a side-stream join to what was timed
    dom_rec = None
    if dom is not None:
        ol = trainer.plan.fwd if dom[0] == "fwd" else trainer.plan.bwd
        dom_rec = ol.recs[dom[1]]
        trainer.stamp_at = dom
    if args.graph:
        trainer.capture()
    # loss=False: the step's BCE still accumulates the summed loss in the graph (reported
    # through trainer.loss() below); only the per-step eager division for a returned mean
    # is not launched (nothing here reads it)
    for _ in range(args.warmup):
        trainer.step(loss=False)
    torch.cuda.synchronize()
    trainer.stamp_reset()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.step(loss=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    roof = None
    if dom_rec is not None:
        raw, brk, span = trainer.stamp_times(args.steps)  # stamp to stamp; a bracket alone
        ms = max(raw - brk, 1e-6)
        roof = roofline_of(dom_rec, ms)
        roof["kernel"] = f"{dom[0]}:{dom_rec.label}"
        roof["avg_ms"] = round(ms, 4)
        roof["bracket_ms"] = round(raw, 4)
        roof["bracket_overhead_ms"] = round(brk, 4)
        roof["timed_launches"] = args.steps
        # the counter against the host clock: first to last stamp of the timed steps over the
        # host-timed region (just under 1.0: the stamps sit inside the steps)
        roof["stamp_clock_check"] = round(span / (elapsed * 1e3), 3)
        roof["traffic"] = pmc_traffic(dom_rec.label, args)
    res = {"value": world * args.batch * args.steps / elapsed,
           "ms_per_step": 1e3 * elapsed / args.steps, "loss": trainer.loss(), "roofline": roof}
    if roofline:
        # north_star's target op: the backbone (stem) convs, each stamped in place the same
        # way in a re-captured step after the timed region (segment.py:19-31)
        res["roofline_backbone"] = [r for r in (stamp_op(trainer, ph, lab, args, rows)
                                                for ph, lab in BACKBONE_OPS) if r is not None]
    del trainer
    torch.cuda.synchronize()
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args))
    world, rank, local = setup_dist(args)
    dev = torch.device("cuda", local)
    kp = args.input == "keypoints" and args.cin == 20
    main_leg = train_leg(args, dev, world, rank, kp, not args.no_roofline)
    dense_leg = None
    if kp and not args.no_dense_leg:
        dense_leg = train_leg(args, dev, world, rank, False, False)
    dp_leg = dp_nccl_leg = None
    if world == 1 and not args.no_dp_leg:
        dp_leg = train_leg(args, dev, world, rank, kp, False, dp_plan=True)
        # the same structure with REAL one-rank RCCL all-reduces (a world-size-1 "nccl"
        # group): what the exchange code path itself costs on one GPU
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                                world_size=1, device_id=dev)
        try:
            dp_nccl_leg = train_leg(args, dev, world, rank, kp, False, dp_plan=True)
        finally:
            dist.destroy_process_group()

    value = main_leg["value"]
    out = {
        "metric": "train images/sec, COCO-person 1024x1024 synthetic (Segment(20) RGB+17 "
                  "heatmaps, BCE+Adam)",
        "value": round(value, 3), "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(main_leg["ms_per_step"], 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": ("synthetic, resident in HBM: seeded image + 17 keypoints per image (the "
                 "heatmaps synthesised on the GPU inside the stem, bit-identical to "
                 "keypoint2heatmaps) + ellipse mask" if kp else
                 "synthetic (seeded image/heatmaps/ellipse masks resident in HBM)"),
        "config": {"workload": f"train_instance.py step, Segment({args.cin}), bs{args.batch}/GPU, "
                               f"{args.size}x{args.size}", "global_batch": world * args.batch,
                   "image_size": args.size, "parallelism": f"dp{world}",
                   "input": "keypoints" if kp else ("heatmaps" if args.cin == 20 else "image"),
                   "execution": "hip-graph" if args.graph else
                                "eager C++ executor (isg_exec_ms2), one side stream"},
        "roofline": main_leg["roofline"], "loss": round(main_leg["loss"], 6),
    }
    if main_leg.get("roofline_backbone"):
        bb = main_leg["roofline_backbone"]
        # north_star's metric: fraction of the fp32 MFMA roofline on the backbone conv (the
        # stem's 5x5 s2 convs), each op stamped in place; aggregate = their flops / time
        tot_f = sum(r["gflop"] for r in bb)
        tot_ms = sum(r["avg_ms"] for r in bb)
        agg = lambda ms: round(tot_f * 1e9 / (ms * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 4)
        out["roofline_backbone"] = {
            "ops": bb, "aggregate_frac": agg(tot_ms),
            "aggregate_frac_alone": agg(sum(r["alone_ms"] for r in bb))
            if all("alone_ms" in r for r in bb) else None,
            "unit": "fraction of the fp32 MFMA peak (157.3 TFLOP/s); in place (stamped inside "
                    "the step) and alone (the per-op pass)"}
    if dense_leg is not None:
        out["dense_heatmaps"] = {"value": round(dense_leg["value"], 3),
                                 "ms_per_step": round(dense_leg["ms_per_step"], 3),
                                 "loss": round(dense_leg["loss"], 6),
                                 "input": "dense 17-channel heatmaps read from HBM "
                                          "(train_batch(x, heatmaps))"}
    if dp_leg is not None:
        out["dp_plan_at_world1"] = {
            "value": round(dp_leg["value"], 3), "ms_per_step": round(dp_leg["ms_per_step"], 3),
            "what": "the step as it runs at world > 1 (two backward parts, two gradient buckets, "
                    "the RCCL exchange points between the executor calls, no fused tail), at "
                    "world 1 where the exchanges are no-ops: the per-GPU ceiling of weak scaling"}
    if dp_nccl_leg is not None:
        out["dp_plan_at_world1_nccl"] = {
            "value": round(dp_nccl_leg["value"], 3),
            "ms_per_step": round(dp_nccl_leg["ms_per_step"], 3),
            "what": "the same data-parallel step with a world-size-1 RCCL process group: the "
                    "two bucket all-reduces are real one-rank RCCL collectives (bucket 1 "
                    "asynchronous under the stem backward, bucket 2, the wait)"}
    if rank == 0 and world == 1 and not args.no_infer:
        out["infer"] = infer_bench(dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
