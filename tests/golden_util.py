"""Helpers to load the golden fixtures and regenerate their seeded inputs."""
import json
import os

import numpy as np

from oracle.seeding import synth_batch, synth_params

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

SEGMENT_FIXTURES = ["segment20_n2_128.npz", "segment3_n2_64x96.npz", "segment20_n2_128_wc.npz",
                    "segment3_n2_64x96_wc.npz", "kp20_n2_128_wc.npz"]
# fixtures in the well-conditioned regime (oracle/seeding.synth_params head_scale): the GPU
# logits are asserted within 1e-4 of the reference's CPU-fp32 logits unconditionally
# (round 6: Segment(3) and the keypoint path too)
WELL_CONDITIONED_FIXTURES = ["segment20_n2_128_wc.npz", "segment3_n2_64x96_wc.npz",
                             "kp20_n2_128_wc.npz"]


class SegmentFixture:
    def __init__(self, name):
        z = np.load(os.path.join(GOLDEN, name))
        self.z = z
        self.meta = json.loads(str(z["meta"]))
        m = self.meta
        self.cin, self.n, self.h, self.w = m["cin"], m["n"], m["h"], m["w"]
        self.shapes = [(k, tuple(s)) for k, s in m["shapes"]]
        self.params = synth_params(self.shapes, m["param_seed"], m.get("head_scale", 1.0))
        # a keypoint fixture (make_golden.make_kp_fixture): the image and mask of the seeded
        # 3-channel batch, the 17 heatmaps made from the stored keypoints by the oracle's
        # keypoint2heatmaps (bit-exact to the reference's, tests/golden/heatmaps.npz)
        self.keypoints = z["keypoints"] if "keypoints" in z.files else None
        if self.keypoints is None:
            self.x, self.mask = synth_batch(self.n, self.cin, self.h, self.w, m["batch_seed"])
        else:
            from oracle.heatmaps_oracle import keypoint2heatmaps
            img, self.mask = synth_batch(self.n, 3, self.h, self.w, m["batch_seed"])
            maps = np.zeros((self.n, 17, self.h, self.w), np.float32)
            for b in range(self.n):
                pts = {j: (self.keypoints[b, j, 0], self.keypoints[b, j, 1])
                       for j in range(17) if self.keypoints[b, j, 2] > 0}
                maps[b] = np.stack(keypoint2heatmaps(pts, (self.h, self.w)))
            assert int((maps > 0).sum()) == int(z["heatmap_nonzero"])
            self.x = np.ascontiguousarray(np.concatenate([img, maps], 1))
        self.param_names = m["param_names"]
        self.grad_none = set(m["grad_none"])
        self.buffer_keys = m["buffer_keys"]
        sizes = [int(np.prod(dict(self.shapes)[k])) for k in self.param_names]
        self.offsets = np.concatenate([[0], np.cumsum(sizes)])

    def grad(self, key, which="grad64"):
        i = self.param_names.index(key)
        shape = dict(self.shapes)[key]
        return self.z[which][self.offsets[i]:self.offsets[i + 1]].reshape(shape)

    def buffers64(self):
        out = {}
        off = 0
        flat = self.z["bufs64"]
        for k in self.buffer_keys:
            n = int(np.prod(dict(self.shapes)[k])) if dict(self.shapes)[k] else 1
            out[k] = flat[off:off + n].reshape(dict(self.shapes)[k])
            off += n
        return out
