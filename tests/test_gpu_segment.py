"""Whole-network parity on the MI355X (autograd path, runtime.py) against golden vectors
generated from the reference (tests/golden/make_golden.py): logits, loss, every parameter
gradient, BN running stats, eval-mode logits. Bars: tests/grad_check.py (logits within
max(1e-4, 2x the CPU-fp32 reference's own error) absolute; every gradient tensor within
max(2x the reference's own fp32 error, 2e-3 of its scale) — no allowance; a ReLU/PReLU
input inside the fp32 rounding band of 0 is resolved to the GPU's branch, grad_check.resolve_ties)."""
import os

import numpy as np
import pytest
import torch

from instancesegmentation_amd.model.segment import Segment
from tests.golden_util import SEGMENT_FIXTURES, WELL_CONDITIONED_FIXTURES, SegmentFixture
from tests.grad_check import check_grads, check_logits, reference_grads

pytestmark = pytest.mark.gpu
DEV = "cuda"


def load_model(fx):
    m = Segment(fx.cin)
    sd = m.state_dict()
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == fx.shapes
    m.load_state_dict({k: torch.as_tensor(v).to(sd[k].dtype) for k, v in fx.params.items()})
    return m.to(DEV)


def run_step(m, fx):
    x = torch.from_numpy(fx.x).to(DEV)
    y = torch.from_numpy(fx.mask).to(DEV)
    m.train()
    if fx.keypoints is not None:  # the keypoint path: heatmaps synthesised in the stem
        logits = m(x[:, :3].contiguous(), torch.from_numpy(fx.keypoints).to(DEV))
    elif fx.cin == 20:
        logits = m(x[:, :3].contiguous(), x[:, 3:].contiguous())
    else:
        logits = m(x)
    prob = torch.sigmoid(logits)
    loss = torch.nn.BCELoss()(prob, y)
    loss.backward()
    return logits.detach(), loss.detach()


@pytest.mark.parametrize("name", SEGMENT_FIXTURES)
def test_segment_train_step_matches_reference(name):
    fx = SegmentFixture(name)
    m = load_model(fx)
    logits, loss = run_step(m, fx)
    check_logits(logits.cpu(), fx.z["logits64"], fx.z["logits32"], name,
                 strict=name in WELL_CONDITIONED_FIXTURES)
    assert abs(loss.item() - float(fx.z["loss64"])) < 1e-5
    got = {k: p.grad for k, p in m.named_parameters()}
    ref, flo = reference_grads(fx.params, fx.x, fx.mask, got, fixture=fx, tag=name)
    dump = os.environ.get("ISG_DUMP_DIR")
    if dump:  # debugging aid: keep the GPU gradients of this run
        np.savez(os.path.join(dump, f"grads_{name}"), **{
            k: p.grad.detach().cpu().numpy() for k, p in m.named_parameters()
            if p.grad is not None}, logits=logits.cpu().numpy())
    check_grads(got, ref, flo, fx.grad_none, name)
    bufs = fx.buffers64()
    sd = m.state_dict()
    for k, v in bufs.items():
        got = sd[k].double().cpu().numpy()
        if k.endswith("num_batches_tracked"):
            assert int(got) == int(v), k
        else:
            np.testing.assert_allclose(got, v, rtol=1e-4, atol=1e-5, err_msg=k)


@pytest.mark.parametrize("name", SEGMENT_FIXTURES)
def test_segment_eval_matches_reference(name):
    fx = SegmentFixture(name)
    m = load_model(fx)
    sd = m.state_dict()
    with torch.no_grad():
        for k, v in fx.buffers64().items():
            sd[k].copy_(torch.as_tensor(v).to(sd[k].dtype))
    m.eval()
    x = torch.from_numpy(fx.x).to(DEV)
    with torch.no_grad():
        if fx.keypoints is not None:
            logits = m(x[:, :3].contiguous(), torch.from_numpy(fx.keypoints).to(DEV))
        else:
            logits = m(x)
    ref = torch.from_numpy(fx.z["eval_logits64"])
    err = (logits.cpu() - ref).abs().max().item()
    scale = max(1.0, ref.abs().max().item())
    print(f"{name}: eval logits err {err:.3e} scale {scale:.1f}")
    assert err <= 1e-4 * scale


def test_train_batch_matches_forward():
    fx = SegmentFixture("segment20_n2_128.npz")
    m = load_model(fx)
    x = torch.from_numpy(fx.x).to(DEV)
    m.eval()
    with torch.no_grad():
        p1 = m.train_batch(x[:, :3].contiguous(), x[:, 3:].contiguous())
        p2 = torch.sigmoid(m(x))
    assert (p1 - p2).abs().max().item() < 1e-6


def test_deterministic_forward():
    fx = SegmentFixture("segment3_n2_64x96.npz")
    m = load_model(fx).eval()
    x = torch.from_numpy(fx.x).to(DEV)
    with torch.no_grad():
        a = m(x)
        b = m(x)
    assert torch.equal(a, b)


def test_segment_eval_512_matches_oracle():
    """BASELINE config 1 (infer.py single 512x512 image) on the HIP path: Segment(20)
    eval, N=1, against the fp64 oracle with the same (non-trivial) running statistics."""
    from oracle import segment_oracle
    from oracle.seeding import synth_batch, synth_params
    m = Segment(20)
    shapes = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    params = synth_params(shapes, 31)
    sd = m.state_dict()
    m.load_state_dict({k: torch.as_tensor(v).to(sd[k].dtype) for k, v in params.items()})
    m = m.to(DEV).eval()
    x, _ = synth_batch(1, 20, 512, 512, 5)
    with torch.no_grad():
        logits = m(torch.from_numpy(x).to(DEV))
    ref64, _ = segment_oracle.forward(params, x, train=False, dtype=torch.float64)
    ref32, _ = segment_oracle.forward(params, x, train=False, dtype=torch.float32)
    err = (logits.double().cpu() - ref64).abs().max().item()
    floor = (ref32.double() - ref64).abs().max().item()
    scale = max(1.0, ref64.abs().max().item())
    print(f"512^2 eval: logits err {err:.3e}, CPU-fp32 err {floor:.3e}, |logit|max {scale:.1f}")
    assert torch.isfinite(logits).all()
    assert err <= max(1e-4, 2.0 * floor) and err <= 1e-4 * scale
