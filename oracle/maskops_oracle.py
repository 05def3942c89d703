"""CPU restatement of the build-defined infer post-process (TEST INFRASTRUCTURE — oracle).

The reference has NO implementation of this step: `infer.py:32-36` is a stub
(SURVEY.md §0.3, §8a A13/A14). The contract below is the build's own and is frozen
here; parity with the reference is therefore "parity unpinned" for these two
functions. The HIP kernels must be bit-exact to this file on
identical inputs. It follows the reference where the reference says anything:

  * crop window = instance box +/- 16 px, resized to 480x480
    (train_instance.py:166-193, test branch)
  * probability -> uint8 by `(p*255).astype(uint8)` truncation
    (train_instance.py:398-399 `tensor2mask`)

A13 paste (`paste_masks`): for canvas pixel (x, y) inside window [x0,x1)x[y0,y1):
    sx = S / (x1-x0)            (fp32, correctly rounded)
    fx = max(((x-x0) + 0.5) * sx - 0.5, 0);  ix = int(fx);  ax = fx - ix
    ix1 = min(ix+1, S-1)        (same for y)
    v  = (1-ay)*((1-ax)*p00 + ax*p01) + ay*((1-ax)*p10 + ax*p11)
    out = uint8(trunc(v*255))   ; 0 outside the window
  every operation is one fp32 IEEE op in exactly this order (no fused multiply-add).

A14 mask-NMS (`mask_nms`):
    bin = u8 >= 128; cnt = sum(bin); s = sum(u8 * bin)          (integers)
    score = float32(s) / (float32(cnt) * 255f)   (0 when cnt == 0)
    order = stable sort by (-score, index)
    iou(i,j) = float32(inter) / float32(cnt_i + cnt_j - inter)  (0 when union == 0)
    greedy: walk `order`; keep i unless suppressed; suppress later j with iou > thr
"""
import numpy as np

F32 = np.float32


def paste_masks(prob, boxes, height, width):
    """prob: [K,S,S] float32; boxes: [K,4] int (x0,y0,x1,y1), exclusive max.
    Returns uint8 [K,height,width]."""
    prob = np.ascontiguousarray(prob, dtype=np.float32)
    k, s, s2 = prob.shape
    assert s == s2
    out = np.zeros((k, height, width), np.uint8)
    for i in range(k):
        x0, y0, x1, y1 = (int(v) for v in boxes[i])
        if x1 <= x0 or y1 <= y0:
            continue
        cx0, cx1 = max(x0, 0), min(x1, width)
        cy0, cy1 = max(y0, 0), min(y1, height)
        if cx1 <= cx0 or cy1 <= cy0:
            continue
        sx = F32(s) / F32(x1 - x0)
        sy = F32(s) / F32(y1 - y0)
        xs = np.arange(cx0, cx1)
        ys = np.arange(cy0, cy1)
        fx = (((xs - x0).astype(F32) + F32(0.5)) * sx) - F32(0.5)
        fy = (((ys - y0).astype(F32) + F32(0.5)) * sy) - F32(0.5)
        fx = np.maximum(fx, F32(0.0))
        fy = np.maximum(fy, F32(0.0))
        ix = fx.astype(np.int64)
        iy = fy.astype(np.int64)
        ax = fx - ix.astype(F32)
        ay = fy - iy.astype(F32)
        ix1 = np.minimum(ix + 1, s - 1)
        iy1 = np.minimum(iy + 1, s - 1)
        p = prob[i]
        p00 = p[iy[:, None], ix[None, :]]
        p01 = p[iy[:, None], ix1[None, :]]
        p10 = p[iy1[:, None], ix[None, :]]
        p11 = p[iy1[:, None], ix1[None, :]]
        bx = (F32(1.0) - ax)[None, :]
        axx = ax[None, :]
        by = (F32(1.0) - ay)[:, None]
        ayy = ay[:, None]
        top = (bx * p00) + (axx * p01)
        bot = (bx * p10) + (axx * p11)
        v = (by * top) + (ayy * bot)
        out[i, cy0:cy1, cx0:cx1] = (v * F32(255.0)).astype(np.uint8)
    return out


def mask_stats(masks_u8):
    """masks_u8 [K,H,W] -> (cnt int64[K], sum int64[K], score float32[K])."""
    m = masks_u8.reshape(masks_u8.shape[0], -1)
    b = m >= 128
    cnt = b.sum(1).astype(np.int64)
    s = (m.astype(np.int64) * b).sum(1)
    score = np.zeros(len(cnt), np.float32)
    nz = cnt > 0
    score[nz] = s[nz].astype(np.float32) / (cnt[nz].astype(np.float32) * F32(255.0))
    return cnt, s, score


def pairwise_inter(masks_u8):
    b = (masks_u8.reshape(masks_u8.shape[0], -1) >= 128).astype(np.int64)
    return b @ b.T


def mask_nms(masks_u8, iou_thr=0.5, scores=None):
    """Greedy mask-NMS. Returns int32 keep indices in keep order.
    `scores` overrides the mask-derived scores (float32) when given."""
    cnt, _, sc = mask_stats(masks_u8)
    if scores is not None:
        sc = np.asarray(scores, np.float32)
    inter = pairwise_inter(masks_u8)
    k = len(cnt)
    order = sorted(range(k), key=lambda i: (-float(sc[i]), i))
    thr = F32(iou_thr)
    sup = np.zeros(k, bool)
    keep = []
    for a, i in enumerate(order):
        if sup[i]:
            continue
        keep.append(i)
        for j in order[a + 1:]:
            if sup[j]:
                continue
            u = cnt[i] + cnt[j] - inter[i, j]
            iou = F32(inter[i, j]) / F32(u) if u > 0 else F32(0.0)
            if iou > thr:
                sup[j] = True
    return np.asarray(keep, np.int32)
