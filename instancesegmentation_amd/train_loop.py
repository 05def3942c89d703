"""The train_instance.py driver around the fused step: epochs over the
common dataset, periodic validation IoU, best-checkpoint save / resume / collapse-reload
and the `syn_train` file-based model sharing — train_instance.py:272-517 with the
visualisation (cv.imshow, :429-469, :511-517) left out.

Differences from the reference, all deliberate:
  * the model is Segment(20) fed RGB + 17 heatmaps (the self-consistent configuration,
    SURVEY.md §0.4: the reference's `Segment(3)` + one-argument `train_batch` crashes);
    the loader hands over the keypoints and the stem synthesises the heatmaps on the GPU;
  * one optimisation step is `Trainer.step` (one HIP graph: forward, BCE, backward,
    Adam), one process per GPU with the two-bucket RCCL exchange when launched with
    torchrun; rank 0 alone validates and writes checkpoints;
  * checkpoints keep the reference's dict — {"branch_name", "best", "epoch",
    "state_dict", "optimizer"} (:497-503) — and the optimizer entry is a
    `torch.optim.Adam(model.parameters()).state_dict()`, so files move both ways
    between this trainer and the reference loop (`Trainer.optimizer_state_dict` /
    `load_optimizer_state_dict`).

    python -m instancesegmentation_amd.train_loop --train-dataset-dir D --val-dataset-dir V \\
        --checkpoint-dir C [--epoch 30 --batch-size 8 --val-iter 120 --show-iter 20 ...]
"""
import argparse
import os
import subprocess

import numpy as np
import torch

from .data import InstanceCommonDataset, collate_fn


def tensor2mask(tensor):
    """train_instance.py:398-399: (p[0]*255) truncated to uint8."""
    return (tensor[0] * 255).cpu().detach().numpy().astype(np.uint8)


def mask_iou(a, b):
    """IoU of two uint8 masks binarised at >= 128 (ymlib.eval_function.mask_iou is
    un-vendored: this threshold is the build's, the same as the NMS contract's).
    Two empty masks: 1.0."""
    a, b = np.asarray(a) >= 128, np.asarray(b) >= 128
    u = np.logical_or(a, b).sum()
    return 1.0 if u == 0 else float(np.logical_and(a, b).sum()) / float(u)


def mean(xs):
    xs = list(xs)
    return sum(xs) / len(xs)


def tensors_mean_iou(outmask_ts, mask_ts):
    """train_instance.py:402-403."""
    return mean(mask_iou(tensor2mask(o), tensor2mask(m)) for o, m in zip(outmask_ts, mask_ts))


def git_branch_name():
    """ymlib.common.get_git_branch_name (un-vendored): `git rev-parse --abbrev-ref HEAD`
    of the working directory, "nobranch" outside a repository."""
    try:
        out = subprocess.run(["git", "rev-parse", "--abbrev-ref", "HEAD"], capture_output=True,
                             text=True, timeout=10)
        return out.stdout.strip() or "nobranch"
    except (OSError, subprocess.SubprocessError):
        return "nobranch"


def save_checkpoint(path, trainer, branch_name, best, epoch):
    """train_instance.py:497-509 (the reference prints 'save_fail' on error)."""
    state = {"branch_name": branch_name, "best": best, "epoch": epoch,
             "state_dict": {k: v.detach().cpu() for k, v in trainer.model.state_dict().items()},
             "optimizer": trainer.optimizer_state_dict()}
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        torch.save(state, path)
        return True
    except OSError:
        print("save_fail")
        return False


def load_checkpoint(path, trainer):
    """train_instance.py:320-328: epoch, model and optimizer state; None on failure
    ('load fail')."""
    try:
        ck = torch.load(path, map_location="cpu", weights_only=True)
        trainer.load_state_dict(ck["state_dict"])
        trainer.load_optimizer_state_dict(ck["optimizer"])
        return int(ck["epoch"])
    except (OSError, KeyError, RuntimeError, ValueError) as e:
        print(f"load fail ({e})")
        return None


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="train Segment(20) (train_instance.py)")
    p.add_argument("--train-dataset-dir", required=True)
    p.add_argument("--val-dataset-dir", required=True)
    p.add_argument("--checkpoint-dir", required=True)
    p.add_argument("--checkpoint-save-path", default=None)
    p.add_argument("--pretrained-path", default=None)
    p.add_argument("--continue-train", action="store_true")
    p.add_argument("--syn-train", action="store_true")
    p.add_argument("--epoch", type=int, default=30)
    p.add_argument("--show-iter", type=int, default=20)
    p.add_argument("--val-iter", type=int, default=120)
    p.add_argument("--batch-size", type=int, default=8)
    p.add_argument("--cpu-num", type=int, default=2)
    p.add_argument("--max-steps", type=int, default=0, help="stop after this many steps (0: off)")
    return p.parse_args(argv)


def _batches(loader, device):
    """(inputs, mask, results) per batch. The second input is the keypoints [B,17,3]
    (float64, 408 B per image): the Trainer's stem synthesises the 17 heatmaps from them
    on the GPU (kp_stem.hip) instead of the loader building and uploading 17 x 480 x 480
    fp32 maps per image (train_instance.py:200-213)."""
    for image_ts, mask_ts, results in loader:
        kp = torch.stack([r["keypoints"] for r in results])
        yield ([image_ts.to(device, non_blocking=True), kp.to(device, non_blocking=True)],
               mask_ts.to(device, non_blocking=True), results)


def fit(args, device=None, process_group=None):
    """The reference loop (train_instance.py:272-515) on the fused Trainer."""
    import torch.distributed as dist

    from .model.segment import Segment
    from .train import Trainer
    device = torch.device(device or "cuda")
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    trainset = InstanceCommonDataset(args.train_dataset_dir, with_heatmaps=False)
    valset = InstanceCommonDataset(args.val_dataset_dir, test=True, with_heatmaps=False)
    sampler = (torch.utils.data.distributed.DistributedSampler(trainset) if world > 1 else None)
    trainloader = torch.utils.data.DataLoader(
        trainset, batch_size=args.batch_size, shuffle=sampler is None, sampler=sampler,
        num_workers=args.cpu_num, collate_fn=collate_fn, drop_last=True)
    valloader = torch.utils.data.DataLoader(valset, batch_size=args.batch_size, shuffle=True,
                                            num_workers=1, collate_fn=collate_fn)
    S = trainset.out_size[0]
    model = Segment(20)
    trainer = Trainer(model, args.batch_size, [(args.batch_size, 3, S, S),
                                               (args.batch_size, 17, 3)], device=device,
                      process_group=process_group)
    branch_name = git_branch_name()
    best_path = args.checkpoint_save_path or os.path.join(args.checkpoint_dir,
                                                          f"{branch_name}_best.pth")
    iou_max, start_epoch = 0.0, 0
    if os.path.exists(best_path):
        iou_max = float(torch.load(best_path, map_location="cpu", weights_only=True)["best"])
    if args.continue_train and os.path.exists(best_path):
        print(f"loading checkpoint from {best_path}")
        start_epoch = load_checkpoint(best_path, trainer) or 0
    elif args.pretrained_path and os.path.exists(args.pretrained_path):
        print(f"pretrained loading checkpoint from {args.pretrained_path}")
        load_checkpoint(args.pretrained_path, trainer)
        start_epoch = 0
    trainer.capture()
    steps = 0
    epoch = start_epoch
    history = []
    while epoch < args.epoch:
        if sampler is not None:
            sampler.set_epoch(epoch)
        loss_total = []
        restart = False
        for i0, (xs, mask, results) in enumerate(_batches(trainloader, device)):
            loss = trainer.step(xs, mask)
            loss_total.append(loss)
            steps += 1
            if i0 % args.show_iter == args.show_iter - 1 and rank == 0:
                print(f" [epoch {epoch}] [{i0 * args.batch_size}/{len(trainset)}]"
                      f" [loss: {round(float(torch.stack(loss_total).mean()), 6)}]")
                loss_total = []
            if i0 % args.val_iter == 0:
                train_iou = val_iou = 0.0
                if rank == 0:
                    train_iou = tensors_mean_iou(trainer.probabilities(), mask)
                    val_ious = []
                    for vxs, vmask, _ in _batches(valloader, device):
                        val_ious.append(tensors_mean_iou(trainer.predict(vxs), vmask))
                        break  # the reference validates on one batch (:414-415)
                    val_iou = mean(val_ious) if val_ious else 0.0
                    print(f"{branch_name} {device} [epoch {epoch}] [val_num:{len(valset)}]"
                          f" [train_batch_iou: {round(train_iou, 6)}] [val_iou: {round(val_iou, 6)}]")
                if world > 1:  # every replica takes the same checkpoint decisions
                    obj = [val_iou, train_iou]
                    dist.broadcast_object_list(obj, src=0)
                    val_iou, train_iou = obj
                history.append((epoch, i0, train_iou, val_iou))
                if iou_max - val_iou > 0.3 and os.path.exists(best_path):        # :472-477
                    print(f"val_iou too low, reload checkpoint from {best_path}")
                    start_epoch = load_checkpoint(best_path, trainer) or start_epoch
                    epoch = start_epoch - 1
                    restart = True
                elif os.path.exists(best_path):                                  # :480-489
                    ck_best = float(torch.load(best_path, map_location="cpu",
                                               weights_only=True)["best"])
                    if iou_max < ck_best or epoch - start_epoch > 10:
                        print(f"update model from {best_path}")
                        iou_max = ck_best
                        if args.syn_train:
                            print("syn_train...")
                            start_epoch = load_checkpoint(best_path, trainer) or start_epoch
                            epoch = start_epoch - 1
                            restart = True
                if not restart and val_iou > iou_max and val_iou > 0.7:          # :492-509
                    iou_max = val_iou
                    if rank == 0:
                        print("save branch best checkpoint " + best_path)
                        save_checkpoint(best_path, trainer, branch_name, iou_max, epoch + 1)
                    if world > 1:
                        dist.barrier()  # the file exists before anyone reads it
            if restart or (args.max_steps and steps >= args.max_steps):
                break
        if args.max_steps and steps >= args.max_steps:
            break
        epoch += 1
    return trainer, history


def main(argv=None):
    args = parse_args(argv)
    fit(args)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
