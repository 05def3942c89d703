"""The train_instance.py driver pieces that need no GPU: checkpoint
dict format and optimizer-state interchange with torch.optim.Adam (train_instance.py:
297, 320-328, 497-503), tensor2mask / IoU (:398-403)."""
import numpy as np
import torch

from instancesegmentation_amd import train_loop as TL
from instancesegmentation_amd.model.segment import Segment
from instancesegmentation_amd.train import Trainer


def _trainer():
    return Trainer(Segment(3), 2, [(2, 3, 32, 32)], device="cpu")


def test_optimizer_state_matches_torch_adam_layout():
    """A state written by the reference optimizer loads into the Trainer and comes back
    out identical (same indices, shapes, step), and vice versa."""
    torch.manual_seed(0)
    m = Segment(3)
    opt = torch.optim.Adam(m.parameters())
    tr = Trainer(Segment(3), 2, [(2, 3, 32, 32)], device="cpu")
    unused = {k for k in tr.model.state_dict() if k not in tr.plan.used_params}
    for _ in range(3):
        for k, p in m.named_parameters():
            p.grad = None if k in unused else torch.randn_like(p)
        opt.step()
    ref = opt.state_dict()
    tr.load_optimizer_state_dict(ref)
    assert int(tr.step_dev.item()) == 3
    out = tr.optimizer_state_dict()
    assert out["param_groups"][0].keys() == ref["param_groups"][0].keys()
    assert out["param_groups"][0]["params"] == ref["param_groups"][0]["params"]
    assert set(out["state"]) == set(ref["state"])
    for i, st in ref["state"].items():
        for key in ("step", "exp_avg", "exp_avg_sq"):
            assert torch.equal(out["state"][i][key], st[key]), (i, key)
    # and the Trainer's state drives a fresh torch Adam
    opt2 = torch.optim.Adam(Segment(3).parameters())
    opt2.load_state_dict(out)


def test_checkpoint_roundtrip(tmp_path):
    torch.manual_seed(1)
    a = _trainer()
    with torch.no_grad():
        a.flat.uniform_(-1, 1)
        a.exp_avg.uniform_(-1, 1)
        a.exp_avg_sq.uniform_(0, 1)
        a.step_dev.fill_(5)
        for _, b in a.model.named_buffers():
            if b.is_floating_point():
                b.uniform_(0.5, 1.5)
    path = tmp_path / "ck" / "main_best.pth"
    assert TL.save_checkpoint(str(path), a, "main", 0.8, 3)
    ck = torch.load(path, weights_only=True)
    assert set(ck) == {"branch_name", "best", "epoch", "state_dict", "optimizer"}
    assert len(ck["state_dict"]) == len(Segment(3).state_dict())
    b = _trainer()
    assert TL.load_checkpoint(str(path), b) == 3
    assert torch.equal(b.flat, a.flat) and torch.equal(b.flatb, a.flatb)
    assert int(b.step_dev.item()) == 5
    live = a.live.bool()
    assert torch.equal(b.exp_avg[live], a.exp_avg[live])
    assert TL.load_checkpoint(str(tmp_path / "nope.pth"), b) is None  # 'load fail'


def test_tensor2mask_and_iou():
    p = torch.tensor([[[0.0, 0.5, 0.999, 1.0]]])
    assert TL.tensor2mask(p).tolist() == [[0, 127, 254, 255]]  # truncation, :398-399
    a = np.array([[0, 200, 200, 0]], np.uint8)
    b = np.array([[0, 130, 0, 255]], np.uint8)
    assert TL.mask_iou(a, b) == 1 / 3
    assert TL.mask_iou(np.zeros(3, np.uint8), np.zeros(3, np.uint8)) == 1.0


def test_train_loop_args():
    a = TL.parse_args(["--train-dataset-dir", "t", "--val-dataset-dir", "v",
                       "--checkpoint-dir", "c", "--continue-train", "--syn-train"])
    assert a.continue_train and a.syn_train and a.epoch == 30 and a.batch_size == 8
    assert a.val_iter == 120 and a.show_iter == 20  # train_instance.py:243-246
