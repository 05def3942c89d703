"""Pin the CPU oracle against golden vectors generated from the reference itself
(tests/golden/make_golden.py). CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import heatmaps_oracle, segment_oracle
from tests.golden_util import GOLDEN, SEGMENT_FIXTURES, SegmentFixture


def dead_bias(key):
    """Conv biases that feed a train-mode BN (segment.py:37-41; the convT at :305-307)."""
    return key.endswith(".conv.bias") or (key.split(".")[0].endswith("up")
                                          and key.endswith("convs.1.bias"))


@pytest.mark.parametrize("name", SEGMENT_FIXTURES)
def test_oracle_train_step_matches_reference(name):
    fx = SegmentFixture(name)
    params = {k: v.copy() for k, v in fx.params.items()}
    logits, loss, grads, P = segment_oracle.train_step(params, fx.x, fx.mask, torch.float64)
    np.testing.assert_allclose(logits.numpy(), fx.z["logits64"], rtol=0, atol=1e-5)
    assert abs(loss.item() - float(fx.z["loss64"])) < 1e-9
    for k in fx.param_names:
        if k in fx.grad_none:
            assert grads[k] is None, k
            continue
        ref = fx.grad(k)
        got = grads[k].numpy()
        scale = max(np.abs(ref).max(), 1e-6)
        # conv biases ahead of train-mode BN have pure-noise gradients
        if dead_bias(k):
            assert np.abs(got).max() < 1e-8 and np.abs(ref).max() < 1e-6, k
            continue
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6 * scale + 1e-9, err_msg=k)
    bufs = fx.buffers64()
    for k, v in bufs.items():
        np.testing.assert_allclose(P[k].numpy(), v, rtol=0, atol=1e-9, err_msg=k)


@pytest.mark.parametrize("name", SEGMENT_FIXTURES)
def test_oracle_eval_matches_reference(name):
    fx = SegmentFixture(name)
    params = {k: v.copy() for k, v in fx.params.items()}
    params.update(fx.buffers64())
    logits, _ = segment_oracle.forward(params, fx.x, train=False, dtype=torch.float64)
    np.testing.assert_allclose(logits.numpy(), fx.z["eval_logits64"], rtol=0, atol=1e-5)


def test_oracle_bce_matches_reference():
    z = np.load(os.path.join(GOLDEN, "bce.npz"))
    lt = torch.from_numpy(z["logits"]).requires_grad_(True)
    p = torch.sigmoid(lt)
    loss = segment_oracle.bce_loss(p, torch.from_numpy(z["target"]))
    loss.backward()
    assert loss.item() == float(z["loss"])
    np.testing.assert_array_equal(lt.grad.numpy(), z["dlogits"])


def test_oracle_adam_matches_reference():
    fx = SegmentFixture("segment20_n2_128.npz")
    z = np.load(os.path.join(GOLDEN, "adam_segment20.npz"))
    p = torch.cat([torch.as_tensor(fx.params[k], dtype=torch.float32).reshape(-1)
                   for k in fx.param_names])
    g = torch.from_numpy(fx.z["grad32"].copy())
    live = torch.ones_like(p, dtype=torch.bool)
    for i, k in enumerate(fx.param_names):
        if k in fx.grad_none:
            live[fx.offsets[i]:fx.offsets[i + 1]] = False
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for step, key in ((1, "step1"), (2, "step2")):
        pl, gl, ml, vl = p[live].clone(), g[live], m[live].clone(), v[live].clone()
        segment_oracle.adam_step(pl, gl, ml, vl, step)
        p[live], m[live], v[live] = pl, ml, vl
        np.testing.assert_allclose(p.numpy(), z[key], rtol=0, atol=2e-7)


def test_oracle_heatmaps_match_reference():
    z = np.load(os.path.join(GOLDEN, "heatmaps.npz"))
    cases = json.loads(str(z["meta"]))
    for ci, c in enumerate(cases):
        pts = {int(k): tuple(v) for k, v in c["points"].items()}
        maps = np.stack(heatmaps_oracle.keypoint2heatmaps(pts, (c["h"], c["w"])))
        idx = np.flatnonzero(maps)
        np.testing.assert_array_equal(idx, z[f"idx{ci}"])
        np.testing.assert_array_equal(maps.reshape(-1)[idx], z[f"val{ci}"])
