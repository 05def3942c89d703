"""Keypoint stem (include/isg.h isg_kp_stem): Segment(20) fed the
keypoints its 17 heatmap channels come from (train_instance.py:33-68), the maps
synthesised inside the stem kernels instead of read from HBM.

  * isg_kp_pool bit-exact to max_pool(4) of the oracle's heatmaps (oracle/heatmaps_oracle.py,
    pinned to the reference's own keypoint2heatmaps outputs, tests/golden/heatmaps.npz);
  * the whole network (autograd Runner path) on keypoints against the fp64 oracle run on
    the dense cat(image, heatmaps): logits, loss, every gradient, running statistics, eval
    logits — the same bars as the dense-heatmap tests (tests/grad_check.py);
  * the captured Trainer step at the bench configuration (bs2 1024^2) on keypoints against
    the fp64 oracle, and against the dense-heatmap Trainer on the same batch.
Keypoints are placed so windows straddle 16x16 output tiles, the image border (partly and
wholly outside) and include invisible parts.
"""
import numpy as np
import pytest
import torch

from instancesegmentation_amd import _lib as L
from instancesegmentation_amd.model.segment import Segment
from instancesegmentation_amd.train import Trainer
from oracle import segment_oracle
from oracle.heatmaps_oracle import keypoint2heatmaps
from oracle.seeding import synth_params
from tests.grad_check import check_grads, check_logits, reference_grads
from tests.isg_helpers import call, struct

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _keypoints(rng, n, h, w, margin=30):
    kp = np.zeros((n, 17, 3), np.float64)
    kp[..., 0] = rng.uniform(-margin, w + margin, (n, 17))
    kp[..., 1] = rng.uniform(-margin, h + margin, (n, 17))
    kp[..., 2] = (rng.uniform(size=(n, 17)) < 0.8).astype(np.float64)
    kp[0, 0] = (w - 1.5, 7.25, 1.0)      # on the right border, top rows
    kp[0, 1] = (16.0 * 3, 16.0 * 2, 1.0)  # exactly on a tile corner
    kp[-1, 2] = (-25.0, h / 2, 1.0)       # window almost wholly left of the image
    return kp


def _maps(kp, h, w):
    out = np.zeros((kp.shape[0], 17, h, w), np.float32)
    for b in range(kp.shape[0]):
        pts = {j: (kp[b, j, 0], kp[b, j, 1]) for j in range(17) if kp[b, j, 2] > 0}
        out[b] = np.stack(keypoint2heatmaps(pts, (h, w)))
    return out


def _image(rng, n, h, w):
    img = rng.integers(0, 256, size=(n, 3, h, w)).astype(np.float32)
    return (img / np.float32(255.0) - np.float32(0.5)) / np.float32(0.5)


def _mask(rng, n, h, w):
    yy, xx = np.mgrid[0:h, 0:w]
    m = np.zeros((n, 1, h, w), np.float32)
    for b in range(n):
        cx, cy = rng.uniform(0.3, 0.7) * w, rng.uniform(0.3, 0.7) * h
        m[b, 0] = ((xx - cx) / (0.25 * w)) ** 2 + ((yy - cy) / (0.3 * h)) ** 2 <= 1.0
    return m


@pytest.mark.parametrize("h,w", [(128, 128), (96, 160)])
def test_kp_pool_matches_pooled_oracle_heatmaps(h, w):
    rng = np.random.Generator(np.random.PCG64(5))
    n = 3
    kp = _keypoints(rng, n, h, w)
    ref = _maps(kp, h, w).reshape(n, 17, h // 4, 4, w // 4, 4).max(axis=(3, 5))
    C = 36  # init_down: pooled image 3 + pooled heatmaps 17 + conv 16
    out = torch.full((n, C, h // 4, w // 4), 7.0, device=DEV)  # poisoned
    K = torch.from_numpy(kp).to(DEV)
    a = struct(L.KpStem, {"kp": K.data_ptr(), "nparts": 17, "sigma": 10.0, "threshold": 0.01,
                          "g": {"N": n, "H": h, "W": w}, "k": 4,
                          "out": out.data_ptr() + 3 * (h // 4) * (w // 4) * 4,
                          "out_n_stride": C * (h // 4) * (w // 4)})
    call("isg_kp_pool", a, L.stream_ptr())
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got[:, 3:20], ref)
    assert np.all(got[:, :3] == 7.0) and np.all(got[:, 20:] == 7.0)  # nothing else written


def _copy(params):
    return {k: np.array(v, copy=True) for k, v in params.items()}


def _load(m, params):
    sd = m.state_dict()
    m.load_state_dict({k: torch.as_tensor(v).to(sd[k].dtype) for k, v in params.items()})
    return m.to(DEV)


@pytest.mark.parametrize("n,h,w", [(2, 128, 128), (1, 96, 160)])
def test_kp_segment_train_step_matches_oracle(n, h, w):
    rng = np.random.Generator(np.random.PCG64(11 + h))
    kp = _keypoints(rng, n, h, w)
    img = _image(rng, n, h, w)
    mask = _mask(rng, n, h, w)
    x = np.concatenate([img, _maps(kp, h, w)], 1)
    m0 = Segment(20)
    params = synth_params([(k, tuple(v.shape)) for k, v in m0.state_dict().items()], 23)
    m = _load(m0, params).train()
    logits = m(torch.from_numpy(img).to(DEV), torch.from_numpy(kp).to(DEV))
    prob = torch.sigmoid(logits)
    loss = torch.nn.BCELoss()(prob, torch.from_numpy(mask).to(DEV))
    loss.backward()
    # (the oracle updates running statistics in place: each pass gets its own copy)
    r64, l64, _, P64 = segment_oracle.train_step(_copy(params), x, mask, torch.float64)
    bufs64 = {k: v.detach().double().clone() for k, v in P64.items()
              if k.endswith(("running_mean", "running_var"))}
    r32, _, _, _ = segment_oracle.train_step(_copy(params), x, mask, torch.float32)
    check_logits(logits.detach().cpu(), r64.numpy(), r32.numpy(), f"kp {n}x{h}x{w}")
    assert abs(loss.item() - l64.item()) < 1e-5
    got = {k: p.grad for k, p in m.named_parameters()}
    ref, flo = reference_grads(_copy(params), x, mask, got, tag=f"kp {n}x{h}x{w}")
    none = {k for k, v in ref.items() if v is None}
    check_grads(got, ref, flo, none, f"kp {n}x{h}x{w}")
    # heatmap-channel weight gradients are where the keypoint kernels act: check them alone
    gw = got["init_conv.layer1.conv.weight"][:, 3:].detach().double().cpu()
    rw = torch.as_tensor(np.asarray(ref["init_conv.layer1.conv.weight"]))[:, 3:].double()
    assert (gw - rw).abs().max().item() <= 2e-3 * max(1e-6, rw.abs().max().item())
    sd = m.state_dict()
    for k, v in bufs64.items():
        np.testing.assert_allclose(sd[k].double().cpu().numpy(), v.numpy(), rtol=1e-4, atol=1e-5,
                                   err_msg=k)


def test_kp_segment_eval_matches_dense():
    """Eval mode (running statistics, no stats correction) and the fused (BN-folded) form."""
    rng = np.random.Generator(np.random.PCG64(31))
    n, h, w = 2, 128, 96
    kp = _keypoints(rng, n, h, w)
    img = _image(rng, n, h, w)
    x = np.concatenate([img, _maps(kp, h, w)], 1)
    m0 = Segment(20)
    params = synth_params([(k, tuple(v.shape)) for k, v in m0.state_dict().items()], 29)
    m = _load(m0, params).eval()
    with torch.no_grad():
        got = m(torch.from_numpy(img).to(DEV), torch.from_numpy(kp).to(DEV)).cpu()
        dense = m(torch.from_numpy(x).to(DEV)).cpu()
    ref64, _ = segment_oracle.forward(_copy(params), x, train=False, dtype=torch.float64)
    scale = max(1.0, ref64.abs().max().item())
    assert (got.double() - ref64).abs().max().item() <= 1e-4 * scale
    assert (got - dense).abs().max().item() <= 1e-4 * scale
    m.fuse()
    with torch.no_grad():
        fused = m(torch.from_numpy(img).to(DEV), torch.from_numpy(kp).to(DEV)).cpu()
    assert (fused.double() - ref64).abs().max().item() <= 2e-4 * scale


def test_kp_trainer_bench_config_matches_oracle_and_dense():
    """The benchmarked keypoint path: captured Trainer step, bs2 1024^2, the bench's batch
    (data.device_batch(keypoints=True)), against the fp64 oracle on the dense input and
    the dense-heatmap Trainer on the same batch."""
    from instancesegmentation_amd.data import device_batch
    n, h, w = 2, 1024, 1024
    torch.manual_seed(1234)
    model = Segment(20)
    params = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    xs, mask = device_batch(n, h, w, DEV, seed=100, keypoints=True)
    xd, mask_d = device_batch(n, h, w, DEV, seed=100)
    assert torch.equal(mask, mask_d)
    tr = Trainer(model, n, [tuple(t.shape) for t in xs], device=DEV).capture()
    tr.step(xs, mask)
    torch.cuda.synchronize()
    assert torch.isfinite(tr.logits).all() and torch.isfinite(tr.grad_flat).all()
    dense = Segment(20)
    dense.load_state_dict({k: torch.as_tensor(v) for k, v in params.items()})
    trd = Trainer(dense, n, [tuple(t.shape) for t in xd], device=DEV).capture()
    trd.step(xd, mask_d)
    torch.cuda.synchronize()
    scale = max(1.0, trd.logits.abs().max().item())
    dl = (tr.logits - trd.logits).abs().max().item()
    print(f"kp vs dense Trainer: logits {dl:.3e}, loss {tr.loss():.6f} vs {trd.loss():.6f}")
    assert dl <= 1e-4 * scale and abs(tr.loss() - trd.loss()) < 1e-6
    x = torch.cat([t.cpu() for t in xd], 1).numpy()
    y = mask.cpu().numpy()
    ref_l, ref_loss, ref_g, _ = segment_oracle.train_step(_copy(params), x, y, torch.float64)
    l32, _, g32, _ = segment_oracle.train_step(_copy(params), x, y, torch.float32)
    check_logits(tr.logits.cpu(), ref_l.numpy(), l32.numpy(), "kp bench")
    assert abs(tr.loss() - ref_loss.item()) < 1e-5
    none = {k for k, v in ref_g.items() if v is None}
    got = {k: (g.detach().cpu().clone() if g is not None else None)
           for (k, _), g in zip(tr.model.named_parameters(), tr.grads())}
    check_grads(got, ref_g, g32, none, "kp bench", full_size=True)
