"""Seeded synthetic parameters and inputs (TEST INFRASTRUCTURE — part of the oracle).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
package. The product path (instancesegmentation_amd) never does.

Everything is derived from numpy PCG64 with explicit seeds so the golden fixtures in
tests/golden/ can regenerate their inputs on the GPU box instead of storing them.

Parameter generation is keyed by the reference's state_dict key names
(`model/segment.py` module tree, e.g. `init_conv.layer1.conv.weight`), so the same
tensors load into the reference, the oracle and the HIP path.
"""
import math

import numpy as np


def _rng(seed, salt=0):
    return np.random.Generator(np.random.PCG64([seed, salt]))


def synth_params(shapes, seed, head_scale=1.0):
    """shapes: ordered list of (key, shape). Returns {key: float64 ndarray}.

    head_scale multiplies the last conv's weight (`bottle6_2.weight`, segment.py:438).
    The CPU-fp32 reference's own logits error scales linearly with it (it is the upstream
    fp32 noise carried through that conv): at 1.0 (|logit| 6-16) the CPU-fp32 path is
    1.1-2.7e-4 from fp64 at every size tried, at 0.35 (|logit| 2-6) 3.8-5.4e-5 — the
    well-conditioned regime where `north_star`'s "fp32 logits within 1e-4 of the CPU path"
    is a meaningful assertion rather than a measure of the CPU path's own rounding.

    Distributions are chosen to exercise every code path (non-zero biases,
    non-trivial BN affine, PReLU slopes != 0.25) while staying in the
    well-conditioned regime SURVEY.md §7 "parity conditioning" asks for.
    """
    out = {}
    for i, (key, shape) in enumerate(shapes):
        r = _rng(seed, i + 1)
        shape = tuple(shape)
        leaf = key.rsplit(".", 1)[-1]
        if leaf == "num_batches_tracked":
            out[key] = np.zeros(shape, dtype=np.int64)
        elif leaf == "running_mean":
            out[key] = r.uniform(-0.2, 0.2, shape)
        elif leaf == "running_var":
            out[key] = r.uniform(0.5, 2.0, shape)
        elif len(shape) == 4:  # conv / convT weight
            fan_in = shape[1] * shape[2] * shape[3]
            out[key] = r.normal(0.0, math.sqrt(2.0 / fan_in), shape)
        elif leaf == "weight":  # 1-D: BN gamma or PReLU slope
            out[key] = r.uniform(0.6, 1.4, shape) if _is_bn(key) else r.uniform(0.05, 0.45, shape)
        elif leaf == "bias":
            out[key] = r.uniform(-0.1, 0.1, shape)
        else:
            raise KeyError(key)
    if head_scale != 1.0 and "bottle6_2.weight" in out:
        out["bottle6_2.weight"] = out["bottle6_2.weight"] * head_scale
    return out


def _is_bn(key):
    """BN modules are attribute `bn` of `Conv` (segment.py:41) or index 2 of
    `BottleneckUp_Res.convs` (segment.py:307)."""
    parts = key.split(".")
    return "bn" in parts or (parts[0].endswith("up") and parts[1:3] == ["convs", "2"])


def synth_batch(n, c_in, h, w, seed):
    """Synthetic sample per SURVEY.md §8d: image = (U{0..255}/255 - 0.5)/0.5 for the
    first 3 channels; the remaining (c_in-3) channels are keypoint heatmaps
    (sigma 10, cut 0.01); the target is a filled ellipse around the keypoints."""
    r = _rng(seed, 1000)
    img = r.integers(0, 256, size=(n, 3, h, w)).astype(np.float32)
    img = (img / np.float32(255.0) - np.float32(0.5)) / np.float32(0.5)
    chans = [img]
    mask = np.zeros((n, 1, h, w), np.float32)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    for b in range(n):
        cx, cy = r.uniform(0.35, 0.65) * w, r.uniform(0.35, 0.65) * h
        ax, ay = r.uniform(0.15, 0.3) * w, r.uniform(0.2, 0.4) * h
        mask[b, 0] = (((xx - cx) / ax) ** 2 + ((yy - cy) / ay) ** 2 <= 1.0).astype(np.float32)
    if c_in > 3:
        hm = np.zeros((n, c_in - 3, h, w), np.float32)
        from .heatmaps_oracle import keypoint2heatmaps
        for b in range(n):
            pts = {}
            for j in range(c_in - 3):
                if r.uniform() < 0.8:
                    pts[j] = (r.uniform(0.2, 0.8) * w, r.uniform(0.2, 0.8) * h)
            hm[b] = np.stack(keypoint2heatmaps(pts, (h, w), n_parts=c_in - 3))
        chans.append(hm)
    x = np.concatenate(chans, axis=1)
    return np.ascontiguousarray(x), mask
