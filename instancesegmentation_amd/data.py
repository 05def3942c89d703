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
    restatement): visible parts only; window [max(0,int(x-r)), min(w-1,int(x+r+1))).
    A non-finite coordinate (where the reference's int() raises) marks the part as not
    visible — the same rule as the GPU kernels (common.h kp_coord)."""
    r = math.sqrt(math.log(threshold) * (-sigma ** 2))
    maps = np.zeros((N_PARTS, h, w), np.float32)
    for part, (x, y) in points.items():
        if not (math.isfinite(x) and math.isfinite(y)):
            continue
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


def synthetic_batch(n, h, w, seed=0, with_heatmaps=True, keypoints_out=None):
    """Returns (image [n,3,h,w], heatmaps [n,17,h,w] or None, mask [n,1,h,w]) float32.
    keypoints_out: an [n,17,3] float64 array receiving the keypoints (x, y, visible) the
    heatmaps are drawn from (the same random stream either way)."""
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
        if with_heatmaps or keypoints_out is not None:
            pts = {j: (cx + rng.uniform(-0.8, 0.8) * ax, cy + rng.uniform(-0.8, 0.8) * ay)
                   for j in range(N_PARTS) if rng.uniform() < 0.8}
            if with_heatmaps:
                hm[b] = keypoint_heatmaps(pts, h, w)
            if keypoints_out is not None:
                keypoints_out[b] = 0.0
                for j, (x, y) in pts.items():
                    keypoints_out[b, j] = (x, y, 1.0)
    return img, hm, mask


def device_batch(n, h, w, device, seed=0, cin=20, keypoints=False):
    """[image, heatmaps] (or [image, keypoints [n,17,3] float64] with keypoints=True: the
    stem then synthesises the same heatmaps on the GPU) and the mask, on `device`."""
    kp = np.zeros((n, N_PARTS, 3), np.float64) if keypoints else None
    img, hm, mask = synthetic_batch(n, h, w, seed, with_heatmaps=(cin == 20 and not keypoints),
                                    keypoints_out=kp)
    xs = [torch.from_numpy(img).to(device)]
    if keypoints:
        xs.append(torch.from_numpy(kp).to(device))
    elif cin == 20:
        xs.append(torch.from_numpy(hm).to(device))
    return xs, torch.from_numpy(mask).to(device)


# ---- the reference's "common dataset" (train_instance.py:71-226) ------------------------
# Layout written by dataset/transfer_coco.py:118-227 (and the OCHuman / Supervisely
# converters): <root>/data/<name>.json per image, paths relative to <root>. Key names go
# through ymlib's `key_combine(key, type)`, which is un-vendored: a key
# is matched here by its plain name or by that name followed by a separator and a type
# suffix ("box", "box:box_xyxy", "box|box_xyxy", ...).
ORDER_PART_NAMES = ["right_shoulder", "right_elbow", "right_wrist",
                    "left_shoulder", "left_elbow", "left_wrist",
                    "right_hip", "right_knee", "right_ankle",
                    "left_hip", "left_knee", "left_ankle",
                    "right_ear", "left_ear",
                    "nose", "right_eye", "left_eye"]      # train_instance.py:25-30
_SEPS = (":", "|", ".", "@", "#", "/", "-", "_")


def ckey(d, key, default=None):
    """d[key] under the plain name or a key_combine'd name (`key` + separator + type)."""
    if not isinstance(d, dict):
        return default
    if key in d:
        return d[key]
    for k, v in d.items():
        if isinstance(k, str) and k.startswith(key) and len(k) > len(key) and k[len(key)] in _SEPS:
            return v
    return default


def _keypoint_table(body_keypoint):
    """{part: {status, point}} -> [17, 3] (x, y, visible) in ORDER_PART_NAMES order."""
    kp = np.zeros((N_PARTS, 3), np.float64)
    for j, name in enumerate(ORDER_PART_NAMES):
        k = ckey(body_keypoint, name)
        if k is None:
            continue
        x, y = ckey(k, "point", (0, 0))
        kp[j] = (float(x), float(y), 1.0 if ckey(k, "status") == "vis" else 0.0)
    return kp


def read_instances(json_path):
    """Person instances of one image from its common-dataset JSON: (boxes int [n,4],
    keypoints float64 [n,17,3]); a missing file means no instances."""
    import json
    import os
    if not os.path.exists(json_path):
        return np.zeros((0, 4), np.int64), np.zeros((0, N_PARTS, 3), np.float64)
    with open(json_path) as f:
        ann = json.load(f)
    boxes, kps = [], []
    for obj in ckey(ann, "object", []) or []:
        box = ckey(obj, "box")
        cls = ckey(obj, "class")
        if box is None or (cls is not None and cls != "person"):
            continue
        boxes.append([int(round(v)) for v in box[:4]])
        kps.append(_keypoint_table(ckey(obj, "body_keypoint", {}) or {}))
    return (np.asarray(boxes, np.int64).reshape(-1, 4),
            np.asarray(kps, np.float64).reshape(-1, N_PARTS, 3))


def keep_instance(obj):
    """The reference's per-object filter (train_instance.py:102-115): an instance mask,
    body keypoints with more than 9 non-missing parts, class person (if given), a box
    larger than 50 px on both sides."""
    if ckey(obj, "instance_mask") is None:
        return False
    bk = ckey(obj, "body_keypoint")
    if bk is None:
        return False
    if sum(ckey(k, "status") != "missing" for k in bk.values()) <= 9:
        return False
    cls = ckey(obj, "class")
    if cls is not None and cls not in ["person"]:
        return False
    box = ckey(obj, "box")
    if box is None:
        return False
    x0, y0, x1, y1 = box[:4]
    return (x1 - x0) > 50 and (y1 - y0) > 50


def mask_box(mask):
    """Bounding box (x0, y0, x1, y1), exclusive max, of a mask's non-zero pixels, or None
    (ymlib.mask2box, un-vendored: this is the build's definition)."""
    ys, xs = np.nonzero(np.asarray(mask))
    if len(xs) == 0:
        return None
    return int(xs.min()), int(ys.min()), int(xs.max()) + 1, int(ys.max()) + 1


def centring_valid(box, height, width):
    """Region of the image the reference's centring translation keeps in the frame
    (train_instance.py:141-149): x in [max(0,-tx), min(W, W-tx)), tx = int(W/2 - cx)."""
    x0, y0, x1, y1 = box
    tx = int(width / 2 - (x0 + x1) / 2)
    ty = int(height / 2 - (y0 + y1) / 2)
    return max(0, -tx), max(0, -ty), min(width, width - tx), min(height, height - ty)


def crop_resample(img, window, valid, size):
    """CPU form of the crop contract (csrc/infer_ops.hip, oracle/infer_oracle.py):
    window [x0,x1)x[y0,y1) of an HxWxC uint8 image, half-pixel-centre bilinear to
    size x size, coordinates clamped into the window, pixels outside `valid` = 0,
    rounded half up to uint8. Returns uint8 [size, size, C]."""
    f32 = np.float32
    img = np.asarray(img, np.uint8)
    if img.ndim == 2:
        img = img[:, :, None]
    H, W, C = img.shape
    x0, y0, x1, y1 = (int(v) for v in window)
    if x1 <= x0 or y1 <= y0:
        return np.zeros((size, size, C), np.uint8)
    vx0, vy0 = max(int(valid[0]), 0), max(int(valid[1]), 0)
    vx1, vy1 = min(int(valid[2]), W), min(int(valid[3]), H)
    u = np.arange(size).astype(f32)
    fx = ((u + f32(0.5)) * (f32(x1 - x0) / f32(size)) - f32(0.5)) + f32(x0)
    fy = ((u + f32(0.5)) * (f32(y1 - y0) / f32(size)) - f32(0.5)) + f32(y0)
    flx, fly = np.floor(fx), np.floor(fy)
    ax, ay = fx - flx, fy - fly
    ix, iy = flx.astype(np.int64), fly.astype(np.int64)
    cx = [np.clip(ix, x0, x1 - 1), np.clip(ix + 1, x0, x1 - 1)]
    cy = [np.clip(iy, y0, y1 - 1), np.clip(iy + 1, y0, y1 - 1)]

    def sample(yy, xx):
        ok = ((yy >= vy0) & (yy < vy1))[:, None] & ((xx >= vx0) & (xx < vx1))[None, :]
        v = img[np.clip(yy, 0, H - 1)[:, None], np.clip(xx, 0, W - 1)[None, :]].astype(f32)
        return np.where(ok[:, :, None], v, f32(0.0))

    bx, by = (f32(1.0) - ax)[None, :, None], (f32(1.0) - ay)[:, None, None]
    axx, ayy = ax[None, :, None], ay[:, None, None]
    top = (bx * sample(cy[0], cx[0])) + (axx * sample(cy[0], cx[1]))
    bot = (bx * sample(cy[1], cx[0])) + (axx * sample(cy[1], cx[1]))
    val = (by * top) + (ayy * bot)
    return np.clip((val + f32(0.5)).astype(np.int64), 0, 255).astype(np.uint8)


class InstanceCommonDataset(torch.utils.data.Dataset):
    """train_instance.py:71-216 on the common-dataset layout, without imgaug/ymlib.

    __getitem__ returns (image_tensor [3,480,480] in [-1,1], mask_tensor [1,480,480] in
    [0,1], out) like the reference; out also carries 'keypoints' [17,3] float64 in crop
    coordinates and, with_heatmaps, 'heatmaps' [17,480,480] (the reference computes them
    from the keypoints, :200-202, and drops them — Segment(20) needs them). The
    augmentation is the reference's active one (both branches, :148-196; the random ones
    are commented out there): translate the box centre to the image centre, crop/pad to
    the instance mask's box +/- 16 px, resize to 480x480 — one resampling, the same
    contract as the GPU crop kernel."""

    def __init__(self, dataset_dir, test: bool = False, with_heatmaps: bool = True) -> None:
        super().__init__()
        import glob
        import json
        import os
        self.test = test
        # False: out carries only the crop-space keypoints [17,3] (x, y, visible), from
        # which the GPU stem synthesises the same heatmaps (kp_stem.hip) — the dense
        # 17 x 480 x 480 maps are then neither computed on the host nor copied to HBM
        self.with_heatmaps = with_heatmaps
        self.out_size = (480, 480)
        self.root = dataset_dir
        self.results = []
        for path in sorted(glob.glob(os.path.join(dataset_dir, "data", "*.json"))):
            with open(path) as f:
                ann = json.load(f)
            image_path = ckey(ann, "image")
            for obj in ckey(ann, "object", []) or []:
                if not keep_instance(obj):
                    continue
                self.results.append(dict(obj, image=image_path))

    def __len__(self):
        return len(self.results)

    def __getitem__(self, index):
        import os

        from PIL import Image
        r = self.results[index]
        image = np.asarray(Image.open(os.path.join(self.root, r["image"])).convert("RGB"))
        mask = np.asarray(Image.open(os.path.join(self.root, ckey(r, "instance_mask"))).convert("L"))
        ih, iw = image.shape[:2]
        box = [float(v) for v in ckey(r, "box")[:4]]
        valid = centring_valid(box, ih, iw)
        ib = mask_box(mask)
        if ib is None:
            ib = (0, 0, iw, ih)                               # train_instance.py:163-164
        # a mask pixel pushed out of the frame by the translation is gone before mask2box
        m = np.zeros_like(mask)
        m[valid[1]:valid[3], valid[0]:valid[2]] = mask[valid[1]:valid[3], valid[0]:valid[2]]
        ib = mask_box(m) or ib
        pad = 16
        win = (ib[0] - pad, ib[1] - pad, ib[2] + pad, ib[3] + pad)
        S = self.out_size[0]
        img_c = crop_resample(image, win, valid, S)
        mask_c = crop_resample(mask, win, valid, S)[:, :, 0]
        kp = _keypoint_table(ckey(r, "body_keypoint", {}) or {})
        kp[:, 0] = (kp[:, 0] - win[0]) * S / (win[2] - win[0])
        kp[:, 1] = (kp[:, 1] - win[1]) * S / (win[3] - win[1])
        kp[:, 2] = (kp[:, 2] > 0).astype(np.float64)
        image_tensor = torch.from_numpy(
            ((img_c.astype(np.float32) / np.float32(255.0) - np.float32(0.5)) / np.float32(0.5))
            .transpose(2, 0, 1).copy())
        mask_tensor = torch.from_numpy((mask_c.astype(np.float32) / np.float32(255.0))[None])
        out = {"image": img_c, "mask": mask_c, "keypoints": torch.from_numpy(kp)}
        if self.with_heatmaps:
            pts = {j: (kp[j, 0], kp[j, 1]) for j in range(N_PARTS) if kp[j, 2] > 0}
            out["heatmaps"] = torch.from_numpy(keypoint_heatmaps(pts, S, S))
        return image_tensor, mask_tensor, out


def collate_fn(batch):
    """train_instance.py:219-226."""
    def deal(samples):
        if isinstance(samples[0], torch.Tensor):
            return torch.stack(samples, axis=0)
        return samples

    return [deal(list(samples)) for samples in zip(*batch)]
