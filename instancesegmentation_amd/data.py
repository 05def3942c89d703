"""Synthetic COCO-person-style training batches, generated host-side once
and kept resident in HBM for benchmarking (no dataset/network access here).

    image    = (U{0..255}/255 - 0.5)/0.5                      (train_instance.py:80-85)
    heatmaps = 17 Gaussian keypoint maps, sigma 10, cut 0.01  (train_instance.py:33-68)
    mask     = filled ellipse around the person               ({0,1}, train_instance.py:87-89)
"""
import math

import numpy as np
import torch

N_PARTS = 17


def keypoint_heatmaps(points, h, w, sigma=10.0, threshold=0.01):
    """train_instance.py:33-68 semantics (see oracle/heatmaps_oracle.py for the pinned
    restatement): visible parts only; window [max(0,int(x-r)), min(w-1,int(x+r+1)))."""
    r = math.sqrt(math.log(threshold) * (-sigma ** 2))
    maps = np.zeros((N_PARTS, h, w), np.float32)
    for part, (x, y) in points.items():
        x0, x1 = max(0, int(x - r)), min(w - 1, int(x + r + 1))
        y0, y1 = max(0, int(y - r)), min(h - 1, int(y + r + 1))
        if x1 <= x0 or y1 <= y0:
            continue
        xs = np.arange(x0, x1)
        ys = np.arange(y0, y1)[:, None]
        e = np.exp(-((xs - x) ** 2 + (ys - y) ** 2) / sigma ** 2)
        win = maps[part, y0:y1, x0:x1]
        keep = e > threshold
        win[keep] = e[keep]
    return maps


def synthetic_batch(n, h, w, seed=0, with_heatmaps=True):
    """Returns (image [n,3,h,w], heatmaps [n,17,h,w] or None, mask [n,1,h,w]) float32."""
    rng = np.random.Generator(np.random.PCG64(seed))
    img = rng.integers(0, 256, size=(n, 3, h, w)).astype(np.float32)
    img = (img / np.float32(255.0) - np.float32(0.5)) / np.float32(0.5)
    hm = np.zeros((n, N_PARTS, h, w), np.float32) if with_heatmaps else None
    mask = np.zeros((n, 1, h, w), np.float32)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    for b in range(n):
        cx, cy = rng.uniform(0.35, 0.65) * w, rng.uniform(0.35, 0.65) * h
        ax, ay = rng.uniform(0.15, 0.3) * w, rng.uniform(0.2, 0.4) * h
        mask[b, 0] = (((xx - cx) / ax) ** 2 + ((yy - cy) / ay) ** 2 <= 1.0)
        if with_heatmaps:
            pts = {j: (cx + rng.uniform(-0.8, 0.8) * ax, cy + rng.uniform(-0.8, 0.8) * ay)
                   for j in range(N_PARTS) if rng.uniform() < 0.8}
            hm[b] = keypoint_heatmaps(pts, h, w)
    return img, hm, mask


def device_batch(n, h, w, device, seed=0, cin=20):
    img, hm, mask = synthetic_batch(n, h, w, seed, with_heatmaps=(cin == 20))
    xs = [torch.from_numpy(img).to(device)]
    if cin == 20:
        xs.append(torch.from_numpy(hm).to(device))
    return xs, torch.from_numpy(mask).to(device)
