"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run in the build container only (it reads /root/reference, which does not exist
on the GPU box):   PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
(`--well-conditioned` writes only segment20_n2_128_wc.npz, added in round 4;
`--strict-regime` writes only segment3_n2_64x96_wc.npz and kp20_n2_128_wc.npz, round 6)

What it does:
  * imports /root/reference/model/segment.py with a `cv2` stub (the import is unused,
    segment.py:6) and bytecode writing disabled, so nothing is written into the
    read-only reference tree;
  * loads seeded synthetic parameters (oracle/seeding.py, keyed by state_dict name)
    into the reference `Segment`, runs the reference train-step body
    (train_instance.py:375-379 with the self-consistent `Segment(20)` +
    `train_batch(x, heatmaps)` call) in float64 and float32;
  * records logits, loss, every parameter gradient, the updated BN running stats,
    eval-mode logits with the calibrated running stats, two Adam steps with the
    reference's `optim.Adam(model.parameters())` (train_instance.py:297), BCE edge
    cases (train_instance.py:299), and `keypoint2heatmaps` outputs
    (train_instance.py:33-68, extracted with `ast`; ymlib's key_combine is un-vendored
    so keypoints are passed with plain names).
Inputs are NOT stored: they are regenerated from the recorded seeds.
"""
import ast
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True

from oracle.seeding import synth_params, synth_batch  # noqa: E402


def load_reference_segment():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sys.path.insert(0, REF)
    from model.segment import Segment  # noqa: E402  (reference module)
    sys.path.remove(REF)
    return Segment


def set_params(model, pvals):
    sd = model.state_dict()
    with torch.no_grad():
        for k, v in sd.items():
            v.copy_(torch.as_tensor(pvals[k]).to(v.dtype))


def capture_train(Segment, cin, n, h, w, pseed, bseed, dtype, head_scale=1.0, batch=None):
    """batch: (x, mask) to use instead of the seeded synth_batch (the keypoint fixture)."""
    torch.manual_seed(0)
    m = Segment(cin)
    shapes = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    pv = synth_params(shapes, pseed, head_scale)
    m = m.to(dtype)
    set_params(m, pv)
    x, mask = synth_batch(n, cin, h, w, bseed) if batch is None else batch
    xt = torch.from_numpy(x).to(dtype)
    yt = torch.from_numpy(mask).to(dtype)
    cap = {}
    hdl = m.bottle6_2.register_forward_hook(lambda mod, i, o: cap.__setitem__("logits", o))
    m.train()
    if cin == 20:
        prob = m.train_batch(xt[:, :3], xt[:, 3:])           # segment.py:531-534
    else:
        prob = torch.sigmoid(m(xt))
    loss = torch.nn.BCELoss()(prob, yt)                       # train_instance.py:299,378
    loss.backward()                                           # :379
    hdl.remove()
    names = [k for k, _ in m.named_parameters()]
    gflat = []
    gnone = []
    for k, p in m.named_parameters():
        if p.grad is None:
            gnone.append(k)
            gflat.append(torch.zeros(p.numel(), dtype=torch.float64))
        else:
            gflat.append(p.grad.detach().reshape(-1).to(torch.float64))
    bufs = {k: v.detach().clone() for k, v in m.state_dict().items()
            if k.endswith(("running_mean", "running_var", "num_batches_tracked"))}
    # eval-mode logits with the running stats calibrated by this one train pass
    m.eval()
    with torch.no_grad():
        ev = m(xt)
    return dict(model=m, shapes=shapes, names=names, gflat=torch.cat(gflat), gnone=gnone,
                logits=cap["logits"].detach(), loss=loss.detach(), bufs=bufs,
                eval_logits=ev, params=pv)


def make_segment_fixture(Segment, cin, n, h, w, pseed, bseed, path, head_scale=1.0,
                         logits_dtype=np.float32, batch=None, extra=None):
    r64 = capture_train(Segment, cin, n, h, w, pseed, bseed, torch.float64, head_scale, batch)
    r32 = capture_train(Segment, cin, n, h, w, pseed, bseed, torch.float32, head_scale, batch)
    buf_keys = list(r64["bufs"].keys())
    out = dict(
        meta=np.array(json.dumps(dict(cin=cin, n=n, h=h, w=w, param_seed=pseed,
                                      batch_seed=bseed, shapes=r64["shapes"],
                                      param_names=r64["names"], grad_none=r64["gnone"],
                                      buffer_keys=buf_keys, head_scale=head_scale,
                                      torch=torch.__version__,
                                      threads=torch.get_num_threads()))),
        logits64=r64["logits"].numpy().astype(logits_dtype),
        logits32=r32["logits"].numpy().astype(np.float32),
        loss64=np.float64(r64["loss"].item()),
        loss32=np.float64(r32["loss"].item()),
        grad64=r64["gflat"].numpy().astype(np.float32),
        grad32=r32["gflat"].numpy().astype(np.float32),
        bufs64=np.concatenate([r64["bufs"][k].reshape(-1).to(torch.float64).numpy()
                               for k in buf_keys]).astype(np.float64),
        eval_logits64=r64["eval_logits"].numpy().astype(logits_dtype),
    )
    out.update(extra or {})
    np.savez_compressed(path, **out)
    return r32


def make_adam_fixture(r32, path, steps=2):
    """Two steps of the reference optimizer (train_instance.py:297,380) on the fp32
    model/grads from the segment fixture."""
    m = r32["model"]
    opt = torch.optim.Adam(m.parameters())                     # train_instance.py:297
    params = list(m.parameters())
    g = r32["gflat"].to(torch.float32)
    off = 0
    grads = []
    for (k, p) in m.named_parameters():
        n = p.numel()
        grads.append(None if k in r32["gnone"] else g[off:off + n].view_as(p).clone())
        off += n
    outs = []
    for _ in range(steps):
        for p, gg in zip(params, grads):
            p.grad = gg
        opt.step()                                              # :380
        outs.append(torch.cat([p.detach().reshape(-1).clone() for p in params]).numpy())
    np.savez_compressed(path, step1=outs[0], step2=outs[1])


def make_bce_fixture(path):
    """nn.BCELoss on sigmoid(logits) (segment.py:534, train_instance.py:299),
    fp32, including the saturating cases SURVEY.md §8a A11 lists."""
    vals = np.array([-120, -30, -17, -16.5, -5, -0.5, 0, 0.5, 5, 16.5, 17, 30, 120],
                    np.float32)
    lg = np.concatenate([vals, vals])
    tg = np.concatenate([np.zeros_like(vals), np.ones_like(vals)])
    rng = np.random.Generator(np.random.PCG64(7))
    lg = np.concatenate([lg, rng.normal(0, 3, 256).astype(np.float32)])
    tg = np.concatenate([tg, (rng.uniform(size=256) < 0.5).astype(np.float32)])
    lt = torch.from_numpy(lg).requires_grad_(True)
    p = torch.sigmoid(lt)
    loss = torch.nn.BCELoss()(p, torch.from_numpy(tg))
    loss.backward()
    np.savez_compressed(path, logits=lg, target=tg, loss=np.float32(loss.item()),
                        dlogits=lt.grad.numpy(), prob=p.detach().numpy())


def reference_keypoint2heatmaps():
    """The reference's keypoint2heatmaps (train_instance.py:33-68) and its part order,
    extracted with `ast` (the module's other imports — ymlib, imgaug, cv2 — are absent)."""
    src = open(os.path.join(REF, "train_instance.py")).read()
    tree = ast.parse(src)
    keep = [nd for nd in tree.body
            if (isinstance(nd, ast.FunctionDef) and nd.name == "keypoint2heatmaps")
            or (isinstance(nd, ast.Assign) and any(getattr(t, "id", "") == "ORDER_PART_NAMES"
                                                    for t in nd.targets))]
    ns = {"np": np, "math": __import__("math"), "key_combine": lambda a, b: a}
    exec(compile(ast.Module(body=keep, type_ignores=[]), "train_instance.py", "exec"), ns)
    return ns["keypoint2heatmaps"], ns["ORDER_PART_NAMES"]


def fixture_keypoints(seed, n, h, w, margin=30):
    """Seeded keypoints [n, 17, (x, y, visible)] placed so windows straddle the stem's
    16x16 output tiles and the image border (partly and almost wholly outside), with
    invisible parts — the same construction as tests/test_gpu_kp_stem._keypoints."""
    rng = np.random.Generator(np.random.PCG64(seed))
    kp = np.zeros((n, 17, 3), np.float64)
    kp[..., 0] = rng.uniform(-margin, w + margin, (n, 17))
    kp[..., 1] = rng.uniform(-margin, h + margin, (n, 17))
    kp[..., 2] = (rng.uniform(size=(n, 17)) < 0.8).astype(np.float64)
    kp[0, 0] = (w - 1.5, 7.25, 1.0)
    kp[0, 1] = (16.0 * 3, 16.0 * 2, 1.0)
    kp[-1, 2] = (-25.0, h / 2, 1.0)
    return kp


def make_kp_fixture(Segment, path, n=2, h=128, w=128, pseed=1234, bseed=99, kseed=17):
    """The keypoint path in the well-conditioned regime: the image and mask of
    synth_batch(cin=3), 17 heatmaps per image made by the REFERENCE's keypoint2heatmaps from
    seeded keypoints (stored in the fixture as `keypoints`), then the reference Segment(20)
    train step on cat(image, heatmaps) with the last conv's weight x0.35."""
    k2h, parts = reference_keypoint2heatmaps()
    img, mask = synth_batch(n, 3, h, w, bseed)
    kp = fixture_keypoints(kseed, n, h, w)
    maps = np.zeros((n, 17, h, w), np.float32)
    for b in range(n):
        pts = {parts[j]: {"status": "vis" if kp[b, j, 2] > 0 else "occ",
                          "point": (float(kp[b, j, 0]), float(kp[b, j, 1]))} for j in range(17)}
        maps[b] = np.stack(k2h(pts, (h, w))).astype(np.float32)
    x = np.concatenate([img, maps], 1)
    make_segment_fixture(Segment, 20, n, h, w, pseed, bseed, path, head_scale=0.35,
                         logits_dtype=np.float64, batch=(x, mask),
                         extra={"keypoints": kp, "heatmap_nonzero": np.int64((maps > 0).sum())})


def make_strict_regime(Segment):
    """Round 6: Segment(3) and the keypoint path in the regime where
    the CPU-fp32 reference is within 5e-5 of fp64, so the GPU-vs-CPU-fp32 1e-4 bar is
    asserted directly."""
    make_segment_fixture(Segment, 3, 2, 64, 96, 4321, 77,
                         os.path.join(HERE, "segment3_n2_64x96_wc.npz"), head_scale=0.35,
                         logits_dtype=np.float64)
    make_kp_fixture(Segment, os.path.join(HERE, "kp20_n2_128_wc.npz"))


def make_heatmap_fixture(path):
    src = open(os.path.join(REF, "train_instance.py")).read()
    tree = ast.parse(src)
    keep = [nd for nd in tree.body
            if (isinstance(nd, ast.FunctionDef) and nd.name == "keypoint2heatmaps")
            or (isinstance(nd, ast.Assign) and any(getattr(t, "id", "") == "ORDER_PART_NAMES"
                                                    for t in nd.targets))]
    ns = {"np": np, "math": __import__("math"), "key_combine": lambda a, b: a}
    exec(compile(ast.Module(body=keep, type_ignores=[]), "train_instance.py", "exec"), ns)
    parts = ns["ORDER_PART_NAMES"]
    rng = np.random.Generator(np.random.PCG64(11))
    cases = []
    arrays = {}
    for ci, (h, w) in enumerate([(480, 480), (96, 128), (64, 64)]):
        kp = {}
        vis = {}
        for j, name in enumerate(parts):
            x = float(rng.uniform(-10, w + 10))
            y = float(rng.uniform(-10, h + 10))
            st = "vis" if rng.uniform() < 0.75 else "occ"
            kp[name] = {"status": st, "point": (x, y)}
            if st == "vis":
                vis[j] = (x, y)
        # also hit the exact edge/boundary handling
        kp[parts[0]] = {"status": "vis", "point": (0.0, 0.0)}
        vis[0] = (0.0, 0.0)
        kp[parts[1]] = {"status": "vis", "point": (w - 1.0, h - 1.0)}
        vis[1] = (w - 1.0, h - 1.0)
        maps = np.stack(ns["keypoint2heatmaps"](kp, (h, w)))
        idx = np.flatnonzero(maps)
        arrays[f"idx{ci}"] = idx.astype(np.int64)
        arrays[f"val{ci}"] = maps.reshape(-1)[idx].astype(np.float32)
        cases.append(dict(h=h, w=w, points={str(k): v for k, v in vis.items()}))
    arrays["meta"] = np.array(json.dumps(cases))
    np.savez_compressed(path, **arrays)


def make_well_conditioned(Segment):
    """Segment(20) 2x128^2 with the last conv's weight x0.35 (|logit| <= 6): the CPU-fp32
    reference is within 5e-5 of fp64 here, so the GPU-vs-CPU-fp32 1e-4 bar is asserted
    directly (tests/grad_check.check_logits strict). fp64 logits are stored in fp64."""
    make_segment_fixture(Segment, 20, 2, 128, 128, 1234, 99,
                         os.path.join(HERE, "segment20_n2_128_wc.npz"), head_scale=0.35,
                         logits_dtype=np.float64)


def main():
    torch.set_num_threads(8)
    Segment = load_reference_segment()
    if "--well-conditioned" in sys.argv:  # added in round 4; leaves the others untouched
        make_well_conditioned(Segment)
        print("well-conditioned fixture written to", HERE)
        return
    if "--strict-regime" in sys.argv:  # added in round 6; leaves the others untouched
        make_strict_regime(Segment)
        print("strict-regime fixtures written to", HERE)
        return
    r32 = make_segment_fixture(Segment, 20, 2, 128, 128, 1234, 99,
                               os.path.join(HERE, "segment20_n2_128.npz"))
    make_adam_fixture(r32, os.path.join(HERE, "adam_segment20.npz"))
    make_segment_fixture(Segment, 3, 2, 64, 96, 4321, 77,
                         os.path.join(HERE, "segment3_n2_64x96.npz"))
    make_bce_fixture(os.path.join(HERE, "bce.npz"))
    make_heatmap_fixture(os.path.join(HERE, "heatmaps.npz"))
    make_well_conditioned(Segment)
    make_strict_regime(Segment)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
