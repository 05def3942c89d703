"""CPU restatement of `keypoint2heatmaps` (TEST INFRASTRUCTURE — oracle).

Follows /root/reference/train_instance.py:33-68:
  * r = sqrt(log(threshold) * -sigma^2)                        (:35)
  * one float32 map per part in ORDER_PART_NAMES order          (:39-41, :25-30)
  * only visible ('vis') keypoints are drawn                    (:45-47)
  * window [max(0,int(x-r)), min(w-1,int(x+r+1))) — the last row/column of the
    image is never written (:52-58)
  * value exp(-((xs-x)^2+(ys-y)^2)/sigma^2), kept where > threshold (:60-64)

The reference reads keypoints through ymlib's `key_combine` naming (un-vendored,
SURVEY.md §2 #10); here a keypoint set is `{part_index: (x, y)}` holding only the
visible parts. Pinned by tests/golden/heatmaps.npz, generated from the reference
function itself (tests/golden/make_golden.py).
"""
import math

import numpy as np

N_PARTS = 17


def keypoint2heatmaps(points, shape, sigma=10, threshold=0.01, n_parts=N_PARTS):
    r = math.sqrt(math.log(threshold) * (-sigma ** 2))
    h, w = shape
    maps = []
    for part in range(n_parts):
        hm = np.zeros(shape, dtype=np.float32)
        if part in points:
            x, y = points[part]
            x0 = max(0, int(x - r))
            x1 = min(w - 1, int(x + r + 1))
            y0 = max(0, int(y - r))
            y1 = min(h - 1, int(y + r + 1))
            xs = np.arange(x0, x1)
            ys = np.arange(y0, y1)[:, None]
            e = np.exp(-((xs - x) ** 2 + (ys - y) ** 2) / sigma ** 2)
            keep = e > threshold
            win = hm[y0:y1, x0:x1]
            win[keep] = e[keep]
        maps.append(hm)
    return maps
