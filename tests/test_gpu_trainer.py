"""Parity of the BENCHMARKED path: `Trainer.step` (flat parameter/gradient buffers, fused
sigmoid+BCE kernel, the two-part backward with side-stream weight gradients, HIP-graph
capture, isg_adam_dev with its device step counter and live mask) against

  * the reference's own outputs (tests/golden/segment20_n2_128.npz, made by importing
    /root/reference/model/segment.py): logits, loss, every gradient, BN running stats;
  * the reference optimizer (`torch.optim.Adam(model.parameters())`,
    train_instance.py:297,380) applied on the CPU to the gradients the GPU produced, for
    two steps (bias corrections of step 1 and step 2, unused parameters untouched);
  * the fp64 CPU oracle (oracle/segment_oracle.py) for step 2 on the updated
    parameters, and at the bench configuration (bs2 1024x1024, Segment(20)).

Bars: logits |err| <= max(2x the CPU-fp32 reference's own error vs fp64,
1e-4 absolute) and <= 1e-4 * max(1, |logit|max); loss within 1e-5; gradients
tests/grad_check.py (strict per-tensor bar at fixture size, statistical at full size).
"""
import os

import numpy as np
import pytest
import torch

from instancesegmentation_amd.model.segment import Segment
from instancesegmentation_amd.train import Trainer
from oracle import segment_oracle
from tests.golden_util import SegmentFixture
from tests.grad_check import check_grads, check_logits, reference_grads, resolve_ties

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(fx):
    m = Segment(fx.cin)
    sd = m.state_dict()
    m.load_state_dict({k: torch.as_tensor(v).to(sd[k].dtype) for k, v in fx.params.items()})
    return m


def _inputs(x):
    xt = torch.from_numpy(x).to(DEV)
    return [xt[:, :3].contiguous(), xt[:, 3:].contiguous()]


def _cpu_state(model):
    return {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}


def _grads_by_key(tr):
    return {k: (g.detach().cpu().clone() if g is not None else None)
            for (k, _), g in zip(tr.model.named_parameters(), tr.grads())}


@pytest.mark.parametrize("captured", [False, True], ids=["eager", "graph"])
def test_trainer_two_steps_match_reference(captured):
    """Step 1 on the fixture's parameters; Adam step 1 on the GPU's own gradients against
    torch.optim.Adam; then step 2 from DETERMINISTIC parameters: p1 = torch.optim.Adam's
    step 1 on the reference's own fp64 gradients (CPU), loaded into the Trainer together
    with that optimizer's state. Before round 5 step 2 ran on the GPU Adam's p1, which
    carried the fp32-atomic summation order of the GPU's step-1 weight gradients into
    step 2 (Adam's first step is ~lr*sign(g)), so step 2's inputs, its CPU-fp32 floor and its
    error bar moved from run to run (Weak #1)."""
    fx = SegmentFixture("segment20_n2_128.npz")
    mode = "graph" if captured else "eager"
    model = _model(fx)
    cpu_model = _model(fx)  # the reference optimizer on the GPU's own gradients
    opt = torch.optim.Adam(cpu_model.parameters())  # train_instance.py:297
    det_model = _model(fx)  # the reference optimizer on the reference's own gradients
    det_opt = torch.optim.Adam(det_model.parameters())
    tr = Trainer(model, fx.n, [(fx.n, 3, fx.h, fx.w), (fx.n, 17, fx.h, fx.w)], device=DEV)
    if captured:
        tr.capture()
    xs = _inputs(fx.x)
    y = torch.from_numpy(fx.mask).to(DEV)

    # ---- step 1 against the reference's own outputs -------------------------------
    tr.step(xs, y)
    torch.cuda.synchronize()
    check_logits(tr.logits.cpu(), fx.z["logits64"], fx.z["logits32"], f"trainer {mode} step1")
    assert abs(tr.loss() - float(fx.z["loss64"])) < 1e-5
    g1 = _grads_by_key(tr)
    ref1, flo1 = reference_grads(fx.params, fx.x, fx.mask, g1, fixture=fx, tag="step1")
    check_grads(g1, ref1, flo1, fx.grad_none, "step1")
    sd = tr.model.state_dict()
    for k, v in fx.buffers64().items():
        got = sd[k].double().cpu().numpy()
        if k.endswith("num_batches_tracked"):
            assert int(got) == int(v), k
        else:
            np.testing.assert_allclose(got, v, rtol=1e-4, atol=1e-5, err_msg=k)

    # Adam step 1 (bias corrections at step 1) on the GPU's own gradients
    for (k, p) in cpu_model.named_parameters():
        p.grad = None if g1[k] is None else g1[k].clone()
    opt.step()
    for (k, p), (kk, q) in zip(cpu_model.named_parameters(), tr.model.named_parameters()):
        np.testing.assert_allclose(q.detach().cpu().numpy(), p.detach().numpy(), rtol=2e-6,
                                   atol=1e-9, err_msg=f"adam step 1: {k}")

    # ---- step 2 from deterministic parameters: Adam step 1 on the reference gradients
    for (k, p) in det_model.named_parameters():
        p.grad = None if k in fx.grad_none else torch.from_numpy(fx.grad(k).copy()).float()
    det_opt.step()
    with torch.no_grad():
        for p, q in zip(tr.model.parameters(), det_model.parameters()):
            p.copy_(q)
    tr.load_optimizer_state_dict(det_opt.state_dict())
    p1 = {k: v.detach().cpu().numpy().copy() for k, v in det_model.state_dict().items()}
    ref_l2, ref_loss2, _, _ = segment_oracle.train_step(dict(p1), fx.x, fx.mask, torch.float64)
    l32, _, _, _ = segment_oracle.train_step(dict(p1), fx.x, fx.mask, torch.float32)
    tr.step()  # same static inputs
    torch.cuda.synchronize()
    check_logits(tr.logits.cpu(), ref_l2.numpy(), l32.numpy(), f"trainer {mode} step2")
    assert abs(tr.loss() - ref_loss2.item()) < 1e-5
    g2 = _grads_by_key(tr)
    if os.environ.get("ISG_DUMP_DIR"):  # debugging aid: the step-2 state for CPU analysis
        np.savez(os.path.join(os.environ["ISG_DUMP_DIR"], f"step2_{int(captured)}.npz"),
                 **{"p1:" + k: v for k, v in p1.items()},
                 **{"g2:" + k: v.numpy() for k, v in g2.items() if v is not None})
    ref_g2, g32, _ = resolve_ties(p1, fx.x, fx.mask, g2, tag="step2")
    check_grads(g2, ref_g2, g32, fx.grad_none, "step2")
    assert int(tr.step_dev.item()) == 2

    # Adam step 2 (bias corrections at step 2; exp_avg/exp_avg_sq carried over)
    for (k, p) in det_model.named_parameters():
        p.grad = None if g2[k] is None else g2[k].clone()
    det_opt.step()
    for (k, p), (kk, q) in zip(det_model.named_parameters(), tr.model.named_parameters()):
        np.testing.assert_allclose(q.detach().cpu().numpy(), p.detach().numpy(), rtol=2e-6,
                                   atol=1e-9, err_msg=f"adam step 2: {k}")
    for k in fx.grad_none:  # torch.optim.Adam skips parameters whose grad is None
        np.testing.assert_array_equal(dict(tr.model.named_parameters())[k].detach().cpu().numpy(),
                                      fx.params[k].astype(np.float32), err_msg=k)


@pytest.mark.parametrize("cfg", ["fixture_128", "bench_1024_keypoints"])
def test_backward_is_bitwise_reproducible(cfg):
    """SURVEY.md §5 determinism ("run twice, compare bits"): the captured train step, replayed
    on the same inputs and parameters (lr 0), and a second Trainer built from scratch give
    bit-identical logits, loss and flat gradient. Every cross-workgroup reduction of the
    step adds fp32 workgroup partials into fp64 accumulators (BatchNorm statistics, PReLU
    slopes and, since round 5, the weight-gradient replicas), which is exact whatever the
    order the atomics land in (include/isg.h ISG_WREP); the round-4 fp32 replicas were not."""
    from instancesegmentation_amd.data import device_batch

    def trainer():
        if cfg == "fixture_128":
            fx = SegmentFixture("segment20_n2_128.npz")
            tr = Trainer(_model(fx), fx.n, [(fx.n, 3, fx.h, fx.w), (fx.n, 17, fx.h, fx.w)],
                         device=DEV)
            xs, y = _inputs(fx.x), torch.from_numpy(fx.mask).to(DEV)
        else:
            torch.manual_seed(1234)
            xs, y = device_batch(2, 1024, 1024, DEV, seed=100, cin=20, keypoints=True)
            tr = Trainer(Segment(20), 2, [tuple(x.shape) for x in xs], device=DEV)
        tr.capture()
        sd = tr.optimizer_state_dict()
        sd["param_groups"][0]["lr"] = 0.0  # parameters fixed: every replay has one answer
        tr.load_optimizer_state_dict(sd)
        return tr, xs, y

    def run(tr, xs, y):
        tr.step(xs, y)
        torch.cuda.synchronize()
        return (tr.logits.detach().clone(), tr.grad_flat.detach().clone(),
                tr.loss_acc.detach().clone())

    tr, xs, y = trainer()
    first = run(tr, xs, y)
    outs = [run(tr, xs, y) for _ in range(3)]
    del tr
    tr2, xs2, y2 = trainer()
    outs.append(run(tr2, xs2, y2))
    for i, o in enumerate(outs):
        diff = [int((a != b).sum().item()) for a, b in zip(o, first)]
        print(f"{cfg} run {i + 1}: elements differing from run 0 (logits, grads, loss): {diff}")
        assert diff[:2] == [0, 0], (cfg, i, diff)
        # the summed loss adds fp64 workgroup partials (isg.h ISG_WREP note): its last fp64
        # bits may follow the atomic order, so it is held to 4 fp64 ulps, not bits
        torch.testing.assert_close(o[2], first[2], rtol=1e-15, atol=0.0)


@pytest.mark.parametrize("cin,n,h,w", [(20, 2, 1024, 1024), (20, 2, 800, 1344),
                                       (20, 1, 1536, 2048)],
                         ids=["bench_bs2_1024", "coco_bs2_1344x800", "supervisely_bs1_2048x1536"])
def test_trainer_full_size_step_matches_oracle(cin, n, h, w):
    """BASELINE configs 2, 3 (per replica, 1333x800 padded to 1344x800) and 5 (per GPU) on
    the captured Trainer step: logits and loss against the fp64 oracle, every gradient
    with the statistical full-size bar (tests/grad_check.py). Weights are the model's own init (weights_init,
    segment.py:451-464) under the bench's seed; data is the bench's synthetic batch."""
    from instancesegmentation_amd.data import device_batch
    torch.manual_seed(1234)
    model = Segment(cin)
    params = _cpu_state(model)
    xs, mask = device_batch(n, h, w, DEV, seed=100, cin=cin)
    tr = Trainer(model, n, [tuple(x.shape) for x in xs], device=DEV).capture()
    tr.step(xs, mask)
    torch.cuda.synchronize()
    assert torch.isfinite(tr.logits).all() and torch.isfinite(tr.grad_flat).all()
    x = torch.cat([t.cpu() for t in xs], 1).numpy()
    y = mask.cpu().numpy()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    ref_l, ref_loss, ref_g, _ = segment_oracle.train_step(dict(params), x, y, torch.float64)
    l32, _, g32, _ = segment_oracle.train_step(dict(params), x, y, torch.float32)
    check_logits(tr.logits.cpu(), ref_l.numpy(), l32.numpy(), f"{n}x{h}x{w}")
    assert abs(tr.loss() - ref_loss.item()) < 1e-5
    none = {k for k, v in ref_g.items() if v is None}
    check_grads(_grads_by_key(tr), ref_g, g32, none, f"{n}x{h}x{w}", full_size=True)


def test_train_loop_runs_and_checkpoints(tmp_path):
    """The train_instance.py driver (instancesegmentation_amd/train_loop.py) on a tiny
    common-format dataset: captured steps, validation IoU, then a checkpoint written by
    this trainer reloads bit-exactly into a fresh one."""
    from instancesegmentation_amd import train_loop as TL
    from tests.test_infer_cpu import _write_dataset
    rng = np.random.default_rng(12)
    _write_dataset(tmp_path / "ds", rng)
    args = TL.parse_args(["--train-dataset-dir", str(tmp_path / "ds"), "--val-dataset-dir",
                          str(tmp_path / "ds"), "--checkpoint-dir", str(tmp_path / "ck"),
                          "--batch-size", "1", "--epoch", "2", "--val-iter", "1",
                          "--show-iter", "1", "--cpu-num", "0", "--max-steps", "2"])
    tr, history = TL.fit(args, device=DEV)
    assert len(history) >= 1 and all(0.0 <= v <= 1.0 for _, _, t, v in history)
    assert int(tr.step_dev.item()) == 2 and np.isfinite(tr.loss())
    path = str(tmp_path / "ck" / "x_best.pth")
    assert TL.save_checkpoint(path, tr, "x", 0.75, 1)
    tr2 = Trainer(Segment(20), 1, [(1, 3, 480, 480), (1, 17, 480, 480)], device=DEV)
    assert TL.load_checkpoint(path, tr2) == 1
    assert torch.equal(tr2.flat, tr.flat) and torch.equal(tr2.flatb, tr.flatb)
    assert torch.equal(tr2.exp_avg, tr.exp_avg) and int(tr2.step_dev.item()) == 2


def test_loaded_adam_hyperparameters_reach_the_captured_step():
    """Trainer.load_optimizer_state_dict after capture(): the Adam launch holds
    lr/betas/eps/wd by value, so the step is re-recorded when they change — here lr 0 from
    a loaded optimizer state must leave every parameter unchanged by the next step."""
    fx = SegmentFixture("segment20_n2_128.npz")
    tr = Trainer(_model(fx), fx.n, [(fx.n, 3, fx.h, fx.w), (fx.n, 17, fx.h, fx.w)], device=DEV)
    tr.capture()
    xs, y = _inputs(fx.x), torch.from_numpy(fx.mask).to(DEV)
    tr.step(xs, y)
    sd = tr.optimizer_state_dict()
    sd["param_groups"][0]["lr"] = 0.0
    tr.load_optimizer_state_dict(sd)
    before = tr.flat.clone()
    tr.step(xs, y)
    torch.cuda.synchronize()
    assert torch.equal(tr.flat, before)
    sd["param_groups"][0]["lr"] = 1e-3
    tr.load_optimizer_state_dict(sd)
    tr.step(xs, y)
    torch.cuda.synchronize()
    assert not torch.equal(tr.flat, before)


def test_side_close_orders_after_second_side_stream(monkeypatch):
    """ADVICE r03 (api.cpp flush): with two gradient buckets and bucket 1's replica fold +
    gradient finalisation on the side stream (ISG_SIDE_CLOSE=1), that fold must run after
    the weight gradients dealt onto the second side stream (ISG_SIDE2=1). The gradients must
    equal those of the same plan with one side stream (the default) and of the default plan,
    also with two side streams; a dropped weight-gradient contribution would show up as an
    O(1) relative error."""
    fx = SegmentFixture("segment20_n2_128.npz")
    xs, y = _inputs(fx.x), torch.from_numpy(fx.mask).to(DEV)

    def grads(env):
        for k in ("ISG_BUCKETS", "ISG_SIDE_CLOSE", "ISG_SIDE2"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        tr = Trainer(_model(fx), fx.n, [(fx.n, 3, fx.h, fx.w), (fx.n, 17, fx.h, fx.w)],
                     device=DEV).capture()
        sd = tr.optimizer_state_dict()
        sd["param_groups"][0]["lr"] = 0.0  # parameters fixed: every replay has one answer
        tr.load_optimizer_state_dict(sd)
        out = []
        for _ in range(3):  # replays: a race would not show on every one
            tr.step(xs, y)
            torch.cuda.synchronize()
            out.append(tr.grad_flat.detach().double().cpu().clone())
        return out

    base = grads({})[0]
    scale = base.abs().max().item()
    for env in ({"ISG_BUCKETS": "2", "ISG_SIDE_CLOSE": "1", "ISG_SIDE2": "1"},
                {"ISG_BUCKETS": "2", "ISG_SIDE_CLOSE": "1"}, {"ISG_SIDE2": "1"}, {}):
        for i, g in enumerate(grads(env)):
            err = (g - base).abs().max().item()
            print(env, i, f"max abs diff {err:.2e} (scale {scale:.2e})")
            assert err <= 1e-5 * scale, (env, i, err)


def test_bn_final_launches_match_default(monkeypatch):
    """the opt-in BatchNorm finalisation launches (ISG_BN_FINAL=1: one
    OP_BN_FINAL per layer turns the statistics into coefficients) must give the gradients of
    the default plan (coefficients evaluated by the consumers). Three replays each. (The
    fused form, finalised by the producer's last workgroup, failed this check in round 4 —
    1.4e-3 of scale, deterministic — and was removed in round 5.)"""
    from instancesegmentation_amd import engine
    fx = SegmentFixture("segment20_n2_128.npz")
    xs, y = _inputs(fx.x), torch.from_numpy(fx.mask).to(DEV)

    def grads(final):
        monkeypatch.setattr(engine, "_BN_FINAL", final)
        tr = Trainer(_model(fx), fx.n, [(fx.n, 3, fx.h, fx.w), (fx.n, 17, fx.h, fx.w)],
                     device=DEV).capture()
        sd = tr.optimizer_state_dict()
        sd["param_groups"][0]["lr"] = 0.0
        tr.load_optimizer_state_dict(sd)
        out = []
        for _ in range(3):
            tr.step(xs, y)
            torch.cuda.synchronize()
            out.append(tr.grad_flat.detach().double().cpu().clone())
        return out

    base = grads(False)[0]
    scale = base.abs().max().item()
    for i, g in enumerate(grads(True)):
        err = (g - base).abs().max().item()
        print("ISG_BN_FINAL=1", i, f"max abs diff {err:.2e} (scale {scale:.2e})")
        assert err <= 1e-5 * scale, (i, err)


@pytest.mark.parametrize("graph", [True, False], ids=["graph", "eager"])
def test_fused_step_tail_matches_separate_launches(graph):
    """The world-1 step's fused tail (isg.h isg_step_tail: replica fold + gradient
    finalisation + Adam + BatchNorm running statistics in one launch, the step counter
    advanced on the side stream) against the separate launches it replaces (OP_SUM_REP,
    the OP_GRAD_FINAL lists, isg_adam_dev, the forward's OP_BN_UPDATE lists): over three
    steps on the keypoint path, the flat gradient, parameters, both Adam moments, the
    running statistics and the step counter are bit-identical."""
    from instancesegmentation_amd.data import device_batch
    torch.manual_seed(321)
    init = Segment(20).state_dict()
    xs, mask = device_batch(2, 256, 256, DEV, seed=77, keypoints=True)

    def run(fused):
        m = Segment(20)
        m.load_state_dict(init)
        tr = Trainer(m, 2, [tuple(x.shape) for x in xs], device=DEV, fused_tail=fused)
        assert tr.fused_tail == fused
        if graph:
            tr.capture()
        out = []
        for _ in range(3):
            tr.step(xs, mask)
            torch.cuda.synchronize()
            out.append([t.detach().clone() for t in (tr.grad_flat, tr.flat, tr.exp_avg,
                                                     tr.exp_avg_sq, tr.flatb, tr.step_dev)])
        return out, tr.loss()

    (a, la), (b, lb) = run(True), run(False)
    names = ("grad", "params", "exp_avg", "exp_avg_sq", "running stats", "step")
    for k, (sa, sb) in enumerate(zip(a, b)):
        diff = [int((u != v).sum()) for u, v in zip(sa, sb)]
        print(f"step {k + 1}: elements differing fused vs separate {dict(zip(names, diff))}")
        assert diff == [0] * 6, (k, diff)
    assert int(a[-1][5].item()) == 3
    assert abs(la - lb) <= 1e-12 * max(1.0, abs(lb))
