"""The infer.py product path: person instances of one image -> masks.

The reference's `infer.py` (:12-36) parses `-i/--test-image-dir -o/--output-dir
--continue-test`, globs the images and stops (a stub: no model, no output). This module
keeps that command line and supplies the missing path, built from the reference's own
per-instance input path (train_instance.py:139-202, test branch) and model:

  per instance k (box + 17 keypoints, the reference's training annotation):
    window   = box +/- 16 px                                  (train_instance.py:166-171)
    valid    = image minus what the centring translation drops (:141-149)
    crop     = window resampled to 480x480, normalised [-1,1] (:175-181, :80-85)
    heatmaps = keypoint2heatmaps of the projected keypoints   (:33-68, :200-202), made
               inside the stem kernels from the keypoints (never in HBM)
  logits   = Segment(20) in eval mode with every BatchNorm folded into its conv
             (Conv.fuseforward, segment.py:47-48)
  prob     = sigmoid                                           (segment.py:534)
  masks    = paste back through the window onto the image canvas (A13), uint8 by
             truncation of p*255 (tensor2mask, train_instance.py:398-399)
  keep     = greedy mask-NMS, IoU 0.5 (A14)

Everything after the host copy of the image runs on the GPU (csrc/infer_ops.hip,
maskops.hip, the Segment plan) and is captured into one HIP graph per (image size,
instance capacity). Instance counts below the capacity are padded with empty windows,
which produce empty masks, score 0, and never suppress anything; their indices are
dropped from `keep`.

    python -m instancesegmentation_amd.infer -i IMAGES -o OUT [--continue-test]
        [--checkpoint best.pth] [--max-instances 16]

Instances come from a sidecar annotation next to each image (`<name>.json`, the common
dataset format of dataset/transfer_coco.py:125-227: {"object": [{"box": [x0,y0,x1,y1],
"body_keypoint": {part: {"status": "vis", "point": [x, y]}}}]}; keys may carry ymlib
`key_combine` suffixes, see data.py). Output per image: `<out>/<name>/<i>.png` for each
kept instance and `<out>/<name>.json` with the kept indices and scores.
"""
import argparse
import ctypes
import glob
import json
import os

import numpy as np
import torch

from . import _lib as L
from .engine import S_ACT, S_IN, S_OUT, S_STATS, S_TENSOR0, Plan

CROP = 480   # train_instance.py:77
PAD = 16     # train_instance.py:167
N_PARTS = 17
NMS_MAX = 256  # masks one isg_mask_nms launch can rank (include/isg.h)


class InstanceSegmenter:
    """Segment(20) inference over the instances of one image, as one HIP graph.

    model: a Segment(20) whose weights are loaded (it is deep-copied and fused);
    image_hw: (H, W) of the images this instance serves; max_instances: capacity K."""

    def __init__(self, model, image_hw, max_instances=16, iou_thr=0.5, device=None,
                 capture=True):
        import copy
        self.device = torch.device(device or "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("InstanceSegmenter runs on the MI355X only (no CPU path)")
        dev = self.device
        self.model = copy.deepcopy(model).to(dev).fuse()
        self.H, self.W = int(image_hw[0]), int(image_hw[1])
        self.K = int(max_instances)
        self.iou_thr = float(iou_thr)
        K, S, H, W = self.K, CROP, self.H, self.W
        cin = self.model.init_conv.layer1.conv.in_channels
        if cin != 3 + N_PARTS:
            raise ValueError(f"InstanceSegmenter needs Segment(20) (RGB + 17 heatmaps), got {cin}")
        # the heatmaps are synthesised inside the stem from the projected keypoints
        # (engine.Keypoints): they are never written to HBM
        self.plan = Plan(self.model, [(K, 3, S, S), (K, N_PARTS, 3)], False, False,
                         (False, False))
        self.image = torch.zeros((H, W, 3), dtype=torch.uint8, device=dev)
        self.windows = torch.zeros((K, 4), dtype=torch.int32, device=dev)
        self.valid = torch.zeros((K, 4), dtype=torch.int32, device=dev)
        self.keypoints = torch.zeros((K, N_PARTS, 3), dtype=torch.float64, device=dev)
        self.x = torch.empty((K, 3, S, S), dtype=torch.float32, device=dev)
        self.logits = torch.empty(self.plan.out_shapes[0], dtype=torch.float32, device=dev)
        self.prob = torch.empty_like(self.logits)
        self.masks = torch.empty((K, H, W), dtype=torch.uint8, device=dev)
        self.work = torch.empty(L.lib().isg_mask_nms_workspace(K, H, W), dtype=torch.uint8,
                                device=dev)
        self.scores = torch.empty(K, dtype=torch.float32, device=dev)
        self.keep = torch.empty(K, dtype=torch.int32, device=dev)
        self.nkeep = torch.zeros(1, dtype=torch.int32, device=dev)
        self.act = torch.empty(max(self.plan.act_size, 1), dtype=torch.float32, device=dev)
        self.stats = torch.empty(self.plan.stats_size, dtype=torch.float64, device=dev)
        g = self.plan.graph
        tab = (ctypes.c_void_p * (S_TENSOR0 + len(g.tensor_names)))()
        tab[S_ACT] = self.act.data_ptr()
        tab[S_STATS] = self.stats.data_ptr()
        tab[S_IN[0]] = self.x.data_ptr()
        tab[S_IN[1]] = self.keypoints.data_ptr()
        tab[S_OUT[0]] = self.logits.data_ptr()
        tensors = [p for _, p in self.model.named_parameters()] + \
                  [b for _, b in self.model.named_buffers()]
        for j, t in enumerate(tensors):
            tab[S_TENSOR0 + j] = t.data_ptr()
        self.table = tab
        self.graph = None
        if capture:
            self._run()  # first-use initialisation outside the capture
            torch.cuda.synchronize(dev)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._run()

    def _run(self):
        lib = L.lib()
        st = L.stream_ptr(self.device)
        K, S = self.K, CROP
        L.check(lib.isg_instance_crop(self.image.data_ptr(), self.H, self.W,
                                      self.windows.data_ptr(), self.valid.data_ptr(), K, S,
                                      self.x.data_ptr(), st), "instance_crop")
        self.plan.fwd.run(self.table, st)
        L.check(lib.isg_sigmoid_fwd(self.logits.data_ptr(), self.prob.data_ptr(),
                                    self.prob.numel(), st), "sigmoid")
        # paste-back and the NMS bit-packing in one pass over the canvases (A13 + A14)
        L.check(lib.isg_mask_paste_nms(self.prob.data_ptr(), K, S, self.windows.data_ptr(),
                                       self.H, self.W, self.iou_thr, self.masks.data_ptr(),
                                       self.work.data_ptr(), self.scores.data_ptr(),
                                       self.keep.data_ptr(), self.nkeep.data_ptr(), st),
                "mask_paste_nms")

    def load(self, image, boxes, keypoints):
        """Copy one image's inputs into the static buffers (no launch).
        image: uint8 [H,W,3] (numpy or tensor); boxes: [n,4] (x0,y0,x1,y1);
        keypoints: [n,17,3] (x, y, visible) in image coordinates."""
        img = torch.as_tensor(np.ascontiguousarray(image) if isinstance(image, np.ndarray) else image)
        if tuple(img.shape) != (self.H, self.W, 3) or img.dtype != torch.uint8:
            raise ValueError(f"image must be uint8 [{self.H},{self.W},3], got "
                             f"{tuple(img.shape)} {img.dtype}")
        boxes = np.asarray(boxes, np.int64).reshape(-1, 4)
        n = len(boxes)
        if n > self.K:
            raise ValueError(f"{n} instances > capacity {self.K}")
        kp = np.zeros((self.K, N_PARTS, 3), np.float64)
        win = np.zeros((self.K, 4), np.int32)  # padding: empty windows
        val = np.zeros((self.K, 4), np.int32)
        if n:
            w = instance_windows(boxes)
            win[:n] = w
            val[:n] = valid_rects(boxes, self.H, self.W)
            kp[:n] = crop_keypoints(np.asarray(keypoints, np.float64).reshape(n, N_PARTS, 3), w)
        self.n = n
        self.image.copy_(img, non_blocking=False)
        self.windows.copy_(torch.from_numpy(win))
        self.valid.copy_(torch.from_numpy(val))
        self.keypoints.copy_(torch.from_numpy(kp))

    def run(self):
        """Launch the pipeline on the loaded inputs (asynchronous)."""
        if self.graph is not None:
            self.graph.replay()
        else:
            self._run()

    def result(self):
        """(masks uint8 [n,H,W] device view, keep list, scores [n]) of the last run."""
        torch.cuda.synchronize(self.device)
        nk = int(self.nkeep.item())
        keep = [int(i) for i in self.keep[:nk].cpu().tolist() if i < self.n]
        return self.masks[:self.n], keep, self.scores[:self.n].cpu().numpy()

    def __call__(self, image, boxes, keypoints):
        self.load(image, boxes, keypoints)
        self.run()
        return self.result()


def instance_windows(boxes, pad=PAD):
    """Crop window of each instance: its box +/- 16 px (train_instance.py:166-171)."""
    b = np.asarray(boxes, np.int64).reshape(-1, 4)
    return np.stack([b[:, 0] - pad, b[:, 1] - pad, b[:, 2] + pad, b[:, 3] + pad],
                    1).astype(np.int32)


def valid_rects(boxes, height, width):
    """The image minus what the reference's centring translation (tx, ty) =
    (int(W/2 - cx), int(H/2 - cy)) pushes out of the frame (train_instance.py:141-149)."""
    out = np.zeros((len(boxes), 4), np.int32)
    for i, (x0, y0, x1, y1) in enumerate(np.asarray(boxes, np.float64).reshape(-1, 4)):
        tx = int(width / 2 - (x0 + x1) / 2)
        ty = int(height / 2 - (y0 + y1) / 2)
        out[i] = (max(0, -tx), max(0, -ty), min(width, width - tx), min(height, height - ty))
    return out


def crop_keypoints(keypoints, windows, size=CROP):
    """Keypoints (x, y, visible) in image coordinates -> crop coordinates: the window
    offset, then imgaug's resize projection x * new/old (train_instance.py:176-181)."""
    kp = np.array(keypoints, dtype=np.float64, copy=True)
    for k, (x0, y0, x1, y1) in enumerate(np.asarray(windows, np.int64)):
        if x1 <= x0 or y1 <= y0:
            kp[k, :, 2] = 0.0
            continue
        kp[k, :, 0] = (kp[k, :, 0] - float(x0)) * float(size) / float(x1 - x0)
        kp[k, :, 1] = (kp[k, :, 1] - float(y0)) * float(size) / float(y1 - y0)
    return kp


# ---- command line (infer.py:12-36) ------------------------------------------------------
def parse_args(argv=None):
    parser = argparse.ArgumentParser(description="inference image")
    parser.add_argument("-i", "--test-image-dir", help="image test dir", required=True)
    parser.add_argument("-o", "--output-dir", help="image save dir", required=True)
    parser.add_argument("--continue-test", action="store_true", help="skip existing file.")
    parser.add_argument("--checkpoint", default=None,
                        help="checkpoint with 'state_dict' (train_instance.py:497-503) or a "
                             "bare state_dict; default: the model's own initialisation")
    parser.add_argument("--max-instances", type=int, default=16)
    parser.add_argument("--iou", type=float, default=0.5, help="mask-NMS IoU threshold")
    return parser.parse_args(argv)


def path_decompose(path):
    """infer.py:24-29."""
    basename = os.path.basename(path)
    dirname = os.path.dirname(path)
    ext = os.path.splitext(path)[-1][1:]
    basename = os.path.splitext(basename)[0]
    return dirname, basename, ext


def list_images(d):
    """The reference globs "*[jpg,png,jpgerr]" (a character class, infer.py:35); the
    intent — jpg / png files — is what is listed here."""
    return sorted(p for p in glob.glob(os.path.join(d, "*"))
                  if os.path.splitext(p)[1].lower() in (".jpg", ".jpeg", ".png"))


def load_model(checkpoint):
    from .model.segment import Segment
    m = Segment(3 + N_PARTS)
    if checkpoint:
        ck = torch.load(checkpoint, map_location="cpu", weights_only=True)
        m.load_state_dict(ck["state_dict"] if isinstance(ck, dict) and "state_dict" in ck else ck)
    return m


def main(argv=None):
    from PIL import Image

    from .data import read_instances
    args = parse_args(argv)
    os.makedirs(args.output_dir, exist_ok=True)
    model = load_model(args.checkpoint)
    engines = {}
    for filepath in list_images(args.test_image_dir):
        dirname, basename, ext = path_decompose(filepath)
        out_json = os.path.join(args.output_dir, basename + ".json")
        if args.continue_test and os.path.exists(out_json):
            continue
        img = np.asarray(Image.open(filepath).convert("RGB"))
        boxes, kps = read_instances(os.path.join(dirname, basename + ".json"))
        H, W = img.shape[:2]
        # one greedy NMS over ALL instances of the image: the capacity grows (doubling
        # from --max-instances, one captured engine per capacity) up to the NMS kernel's
        # limit of NMS_MAX masks; only beyond that is the image split into chunks, each
        # with its own NMS (duplicates in different chunks are then not suppressed; the
        # output JSON says so)
        cap = max(1, args.max_instances)
        while cap < min(len(boxes), NMS_MAX):
            cap *= 2
        cap = min(cap, NMS_MAX) if len(boxes) > args.max_instances else cap
        eng = engines.get((H, W, cap))
        if eng is None:
            eng = engines[(H, W, cap)] = InstanceSegmenter(model, (H, W), cap, args.iou)
        res = {"image": os.path.basename(filepath), "instances": len(boxes), "keep": [],
               "scores": []}
        if len(boxes) > eng.K:
            print(f"warning: {basename}: {len(boxes)} instances > {eng.K}: mask-NMS runs per "
                  f"chunk of {eng.K}")
            res["nms"] = f"per chunk of {eng.K}"
        if len(boxes):
            for b0 in range(0, len(boxes), eng.K):
                masks, keep, scores = eng(img, boxes[b0:b0 + eng.K], kps[b0:b0 + eng.K])
                odir = os.path.join(args.output_dir, basename)
                os.makedirs(odir, exist_ok=True)
                host = masks.cpu().numpy()
                for i in keep:
                    Image.fromarray(host[i]).save(os.path.join(odir, f"{b0 + i}.png"))
                res["keep"] += [b0 + i for i in keep]
                res["scores"] += [float(s) for s in scores]
        with open(out_json, "w") as f:
            json.dump(res, f)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
