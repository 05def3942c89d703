"""CPU restatement of the infer pre-process (TEST INFRASTRUCTURE — oracle).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.

The reference's per-instance input path is the test branch of
/root/reference/train_instance.py:139-196 (translate the image so the person box is
centred :141-149, crop/pad to the instance box +/- 16 px :166-178, resize to 480x480
:179-180, ToTensor + Normalize(0.5, 0.5) :80-85) followed by keypoint2heatmaps on the
transformed keypoints (:200-202). It runs through imgaug/cv2 and ymlib, none of which is
in this container and none of which any reference test pins: PARITY UNPINNED. What is
frozen here is the build's contract, which the HIP kernels (csrc/infer_ops.hip) match
bit for bit:

  window      = (x0 - 16, y0 - 16, x1 + 16, y1 + 16) of the instance box (exclusive max),
                in ORIGINAL image coordinates (translation and crop/pad are integer moves
                that cancel out; the window may reach outside the image)
  valid       = the image minus what the centring translation (tx, ty) =
                (int(W/2 - cx), int(H/2 - cy)) of the box centre pushes out of the frame
                (train_instance.py:141-149, zero fill): x in [max(0,-tx), min(W, W-tx))
  crop        = half-pixel-centre bilinear resampling of the window to SxS, sample
                coordinates clamped into the window, pixels outside `valid` = 0 (the
                Affine / CropAndPad fill), rounded half up to uint8, then
                (q/255 - 0.5)/0.5; every step one fp32 op in the order written in
                `crop_instances`
  keypoints   = x' = (x - wx0) * S / (wx1 - wx0) (imgaug's keypoint projection on
                resize, no half-pixel shift), in double
  heatmaps    = keypoint2heatmaps (oracle/heatmaps_oracle.py, pinned by the reference's
                own golden vectors) on the projected keypoints
"""
import numpy as np

from .heatmaps_oracle import keypoint2heatmaps

F32 = np.float32
PAD = 16   # train_instance.py:167
CROP = 480  # train_instance.py:77


def instance_windows(boxes, pad=PAD):
    """boxes [K,4] (x0,y0,x1,y1) -> crop windows [K,4] int32."""
    b = np.asarray(boxes, np.int64).reshape(-1, 4)
    return np.stack([b[:, 0] - pad, b[:, 1] - pad, b[:, 2] + pad, b[:, 3] + pad], 1).astype(np.int32)


def valid_rects(boxes, height, width):
    """Region of the original image still inside the frame after the reference's
    centring translation (train_instance.py:141-149; int() truncates toward zero)."""
    out = []
    for x0, y0, x1, y1 in np.asarray(boxes, np.float64).reshape(-1, 4):
        tx = int(width / 2 - (x0 + x1) / 2)
        ty = int(height / 2 - (y0 + y1) / 2)
        out.append([max(0, -tx), max(0, -ty), min(width, width - tx), min(height, height - ty)])
    return np.asarray(out, np.int32).reshape(-1, 4)


def crop_keypoints(keypoints, windows, size=CROP):
    """keypoints [K,P,3] (x, y, visible) in image coordinates -> crop coordinates (double)."""
    kp = np.array(keypoints, dtype=np.float64, copy=True).reshape(len(windows), -1, 3)
    for k, (x0, y0, x1, y1) in enumerate(np.asarray(windows, np.int64)):
        if x1 <= x0 or y1 <= y0:
            kp[k, :, 2] = 0.0
            continue
        kp[k, :, 0] = (kp[k, :, 0] - float(x0)) * float(size) / float(x1 - x0)
        kp[k, :, 1] = (kp[k, :, 1] - float(y0)) * float(size) / float(y1 - y0)
    return kp


def crop_instances(image, windows, valid=None, size=CROP):
    """image uint8 [H,W,3]; windows, valid int [K,4] -> float32 [K,3,size,size] in [-1,1]."""
    img = np.asarray(image, np.uint8)
    H, W = img.shape[:2]
    win = np.asarray(windows, np.int64).reshape(-1, 4)
    if valid is None:
        valid = np.tile(np.array([0, 0, W, H], np.int64), (len(win), 1))
    valid = np.asarray(valid, np.int64).reshape(-1, 4)
    K = len(win)
    out = np.empty((K, 3, size, size), F32)
    u = np.arange(size).astype(F32)
    for k in range(K):
        x0, y0, x1, y1 = (int(v) for v in win[k])
        if x1 <= x0 or y1 <= y0:
            out[k] = F32(-1.0)
            continue
        sx = F32(x1 - x0) / F32(size)
        sy = F32(y1 - y0) / F32(size)
        fx = ((u + F32(0.5)) * sx - F32(0.5)) + F32(x0)
        fy = ((u + F32(0.5)) * sy - F32(0.5)) + F32(y0)
        flx, fly = np.floor(fx), np.floor(fy)
        ax, ay = fx - flx, fy - fly
        ix, iy = flx.astype(np.int64), fly.astype(np.int64)
        cx0, cx1 = np.clip(ix, x0, x1 - 1), np.clip(ix + 1, x0, x1 - 1)
        cy0, cy1 = np.clip(iy, y0, y1 - 1), np.clip(iy + 1, y0, y1 - 1)
        bx, by = F32(1.0) - ax, F32(1.0) - ay

        vx0, vy0 = max(int(valid[k, 0]), 0), max(int(valid[k, 1]), 0)
        vx1, vy1 = min(int(valid[k, 2]), W), min(int(valid[k, 3]), H)

        def sample(cy, cx, c):
            ok = ((cy >= vy0) & (cy < vy1))[:, None] & ((cx >= vx0) & (cx < vx1))[None, :]
            v = img[np.clip(cy, 0, H - 1)[:, None], np.clip(cx, 0, W - 1)[None, :], c].astype(F32)
            return np.where(ok, v, F32(0.0))

        for c in range(3):
            s00, s01 = sample(cy0, cx0, c), sample(cy0, cx1, c)
            s10, s11 = sample(cy1, cx0, c), sample(cy1, cx1, c)
            top = (bx[None, :] * s00) + (ax[None, :] * s01)
            bot = (bx[None, :] * s10) + (ax[None, :] * s11)
            val = (by[:, None] * top) + (ay[:, None] * bot)
            q = np.clip((val + F32(0.5)).astype(np.int64), 0, 255).astype(F32)
            out[k, c] = ((q / F32(255.0)) - F32(0.5)) / F32(0.5)
    return out


def instance_heatmaps(keypoints_crop, size=CROP, n_parts=17):
    """keypoints [K,P,3] in crop coordinates -> float32 [K,P,size,size]."""
    kp = np.asarray(keypoints_crop, np.float64)
    out = np.zeros((len(kp), n_parts, size, size), F32)
    for k in range(len(kp)):
        pts = {j: (float(kp[k, j, 0]), float(kp[k, j, 1])) for j in range(n_parts)
               if kp[k, j, 2] > 0}
        out[k] = np.stack(keypoint2heatmaps(pts, (size, size), n_parts=n_parts))
    return out
