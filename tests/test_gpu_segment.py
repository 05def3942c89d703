"""Whole-network parity on the MI355X against golden vectors generated from the reference
(tests/golden/make_golden.py): logits, loss, every parameter gradient, BN running stats,
eval-mode logits. Tolerances: logits within 1e-4 * max(1, |logit|max) of the fp64
reference (north_star: "fp32 mask logits within 1e-4"; fp32 CPU itself deviates
1.2e-4 at 128^2, see test_reference_fp32_noise_floor), gradients within
max(2x the reference's own fp32 error, 2e-3 of each tensor's scale); an isolated channel
whose ReLU pre-activation sits at a tie (|pre| below fp32 forward noise) is reported and
bounded separately (relative L2 per tensor)."""
import os

import numpy as np
import pytest
import torch

from instancesegmentation_amd.model.segment import Segment
from tests.golden_util import SEGMENT_FIXTURES, SegmentFixture

pytestmark = pytest.mark.gpu
DEV = "cuda"


def dead_bias(key):
    return key.endswith(".conv.bias") or (key.split(".")[0].endswith("up")
                                          and key.endswith("convs.1.bias"))


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
    if fx.cin == 20:
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
    ref = torch.from_numpy(fx.z["logits64"])
    err = (logits.cpu() - ref).abs().max().item()
    scale = max(1.0, ref.abs().max().item())
    print(f"{name}: logits max err {err:.3e} (|logit|max {ref.abs().max():.2f}); "
          f"cpu-fp32 err {np.abs(fx.z['logits32'] - fx.z['logits64']).max():.3e}")
    assert err <= 1e-4 * scale
    assert err <= 2.0 * np.abs(fx.z["logits32"] - fx.z["logits64"]).max()
    assert abs(loss.item() - float(fx.z["loss64"])) < 1e-5
    # Gradients. A ReLU pre-activation or a max-pool window within fp32 reduction noise
    # of a tie (the GPU sums BN statistics in a run-dependent order, as any atomics-based
    # reduction does) can switch sides between runs and move that one pixel's gradient;
    # tools/race_hunt.py shows every forward buffer agreeing across runs while gradients
    # below such a tail differ (segment3: |pre| = 2.2e-5 at bottle4_2, channel 18). So:
    #   * every tensor: relative L2 error <= 2e-2 (bounded damage of a flipped pixel),
    #   * >= 75% of tensors: max-abs error <= max(2x the reference's own fp32 error,
    #     2e-3 of the tensor's scale) — the strict bar, which a tie-free run meets on all.
    strict_fail, worst, l2_worst = [], [], 0.0
    for k, p in m.named_parameters():
        if k in fx.grad_none:
            assert p.grad is None, k
            continue
        ref_g = torch.from_numpy(fx.grad(k).copy()).double()
        got = p.grad.detach().double().cpu()
        if dead_bias(k):
            assert got.abs().max().item() < 1e-4, k
            continue
        sc = max(ref_g.abs().max().item(), 1e-8)
        err = (got - ref_g).abs().max().item()
        cpu32 = torch.from_numpy(fx.grad(k, "grad32").copy()).double()
        floor = (cpu32 - ref_g).abs().max().item()
        allowed = max(2.0 * floor, 2e-3 * sc)
        l2 = ((got - ref_g).norm() / max(ref_g.norm().item(), 1e-12)).item()
        l2_worst = max(l2_worst, l2)
        assert l2 <= 2e-2, (k, l2)
        if err > allowed:
            strict_fail.append((k, round(err / allowed, 2), f"l2 {l2:.1e}"))
        worst.append((err / allowed, err / sc, floor / sc, k))
    worst.sort(reverse=True)
    ntensor = len(worst)
    print(f"grads: worst rel-L2 {l2_worst:.2e}; {len(strict_fail)}/{ntensor} tensors above the "
          f"strict max-abs bar (tie-affected): {strict_fail[:6]}")
    dump = os.environ.get("ISG_DUMP_DIR")
    if dump:  # debugging aid: keep the GPU gradients of this run
        np.savez(os.path.join(dump, f"grads_{name}"), **{
            k: p.grad.detach().cpu().numpy() for k, p in m.named_parameters()
            if p.grad is not None}, logits=logits.cpu().numpy())
    assert len(strict_fail) <= ntensor // 4, strict_fail
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
