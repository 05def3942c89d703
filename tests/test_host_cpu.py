"""CPU-only checks: the C-ABI library loads and exports every symbol include/isg.h
declares, the drop-in module matches the reference's state_dict/parameter layout,
plans trace, and errors surface as the reference's exception types."""
import os
import re
import subprocess

import numpy as np
import pytest
import torch

from instancesegmentation_amd import _lib as L
from instancesegmentation_amd.engine import Plan
from instancesegmentation_amd.model.segment import BottleneckDim_Res, BottleneckDown2, Segment
from instancesegmentation_amd.runtime import EngineModule
from oracle import maskops_oracle as MO
from tests.golden_util import SEGMENT_FIXTURES, SegmentFixture

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "isg.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|const char\*)\s+(isg_\w+)\s*\(",
                                 src, re.M)))


def test_library_exports_every_declared_symbol():
    lib = L.lib()  # also verifies every struct layout against isg_record_size
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (isg_\w+)", out))
    declared = header_symbols()
    assert declared, "no declarations parsed"
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    assert set(declared) <= set(L.SIGNATURES), set(declared) - set(L.SIGNATURES)
    assert lib.isg_abi_version() == L.ABI_VERSION
    assert lib.isg_stat_replicas() == L.STAT_REP


def test_head_slab_size_matches_library():
    """engine sizes the mask head's dW1 partial slab with _lib.head_part_floats, the Python
    mirror of isg_mask_head_part_floats (mask_head.hip head_bwd_blocks)."""
    lib = L.lib()
    for n, h, w in [(2, 256, 256), (1, 5, 7), (2, 17, 33), (1, 120, 120), (4, 200, 336)]:
        assert lib.isg_mask_head_part_floats(n, h, w) == L.head_part_floats(n, h, w), (n, h, w)


def test_library_error_path_without_gpu():
    # an invalid geometry is rejected before any device work
    g = L.Geom()
    rc = L.lib().isg_conv_fwd(g, None, None, None, None)
    assert rc == -1
    assert b"geometry" in L.lib().isg_last_error()


@pytest.mark.parametrize("name", SEGMENT_FIXTURES)
def test_state_dict_layout_matches_reference(name):
    fx = SegmentFixture(name)
    m = Segment(fx.cin)
    assert [(k, tuple(v.shape)) for k, v in m.state_dict().items()] == fx.shapes
    assert [k for k, _ in m.named_parameters()] == fx.param_names
    m.load_state_dict({k: torch.as_tensor(v).to(m.state_dict()[k].dtype)
                       for k, v in fx.params.items()})


@pytest.mark.parametrize("name", SEGMENT_FIXTURES)
def test_plan_traces_and_unused_params_match_reference(name):
    fx = SegmentFixture(name)
    m = Segment(fx.cin)
    shapes = [(fx.n, 3, fx.h, fx.w), (fx.n, 17, fx.h, fx.w)] if fx.cin == 20 \
        else [(fx.n, fx.cin, fx.h, fx.w)]
    p = Plan(m, shapes, True, True, tuple(False for _ in shapes))
    unused = [k for k in p.graph.param_names if k not in p.used_params]
    assert sorted(unused) == sorted(fx.grad_none)
    assert p.fwd.recs and p.bwd.recs


def test_weights_init_matches_reference_rules():
    torch.manual_seed(0)
    m = Segment(20)
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            assert torch.all(mod.weight == 1) and torch.all(mod.bias == 0)
        if type(mod) is torch.nn.Conv2d and mod.bias is not None:
            assert torch.all(mod.bias == 0), name
    # ConvTranspose2d keeps torch default init (not an nn.Conv2d subclass)
    assert m.bottle6_1.bias.abs().sum() > 0


def test_cpu_tensor_raises_runtime_error():
    m = Segment(3)
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 64, 64))


def test_bad_channel_count_raises():
    m = Segment(3)
    with pytest.raises(RuntimeError):
        Plan(m, [(1, 20, 64, 64)], True, True, (False,))


def test_non_multiple_of_16_raises():
    m = Segment(3)
    with pytest.raises(RuntimeError):
        Plan(m, [(1, 3, 72, 64)], True, True, (False,))


# ---- oracle properties for the build-defined post-process (parity unpinned) ----------
def test_paste_identity_window_reproduces_probability_truncation():
    rng = np.random.Generator(np.random.PCG64(1))
    S = 32
    prob = rng.uniform(0, 1, (1, S, S)).astype(np.float32)
    out = MO.paste_masks(prob, np.array([[0, 0, S, S]]), S, S)
    assert np.array_equal(out[0], (prob[0] * np.float32(255)).astype(np.uint8))


def test_paste_outside_window_is_zero():
    prob = np.ones((1, 8, 8), np.float32)
    out = MO.paste_masks(prob, np.array([[10, 10, 20, 20]]), 30, 30)
    assert out[0, :10].sum() == 0 and out[0, :, :10].sum() == 0
    assert np.all(out[0, 10:20, 10:20] == 255)


def test_nms_suppresses_duplicates_and_keeps_disjoint():
    m = np.zeros((4, 20, 20), np.uint8)
    m[0, 2:10, 2:10] = 200
    m[1, 2:10, 2:11] = 180   # near-duplicate of 0, lower score
    m[2, 12:18, 12:18] = 250  # disjoint
    m[3] = 0                 # empty mask
    keep = MO.mask_nms(m, 0.5)
    assert list(keep) == [2, 0, 3]


def test_nms_ties_break_by_index():
    m = np.zeros((3, 10, 10), np.uint8)
    m[:, 0:5, 0:5] = 200
    assert list(MO.mask_nms(m, 0.5)) == [0]


def test_bench_traffic_record_matches_dominant_op():
    """bench.py reports roofline.traffic from the committed PMC pass (profiles/traffic.json,
    tools/kbench/traffic.sh): the record must carry the op label bench.py keys on, the bench
    configuration and the gfx950-corrected byte count (fetch_scale*FETCH_SIZE + WRITE_SIZE,
    fetch_scale 2 only for 16-B/lane loads; round-2 records predate the per-kernel scale and
    doubled every kernel's FETCH_SIZE)."""
    import json
    import os
    import types

    import bench
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    runs = json.load(open(os.path.join(root, "profiles", "traffic.json")))
    by_label = {r["label"]: r for r in runs}
    assert "dw_init_conv.layer1" in by_label
    for r in runs:
        kern = [v for k, v in r["kernels"].items() if not k.startswith("__amd_rocclr")]
        if all("read_bytes_per_dispatch" in v for v in kern):
            # round-4 records (tools/pmc_traffic_all.sh): bytes, the FETCH_SIZE doubling applied
            expect = sum(v["read_bytes_per_dispatch"] + v["write_bytes_per_dispatch"] for v in kern)
        else:
            expect = sum(v.get("fetch_scale", 2.0) * v["FETCH_SIZE_kb_per_dispatch"]
                         + v["WRITE_SIZE_kb_per_dispatch"] for v in kern) * 1024.0
        assert abs(r["hbm_bytes_per_launch"] - expect) <= 1e-6 * expect
    args = types.SimpleNamespace(batch=2, cin=20, size=1024)
    got = bench.pmc_traffic("dw_init_conv.layer1", args)
    assert got == by_label["dw_init_conv.layer1"]["hbm_bytes_per_launch"]
    # another configuration is not covered by the committed pass
    assert bench.pmc_traffic("dw_init_conv.layer1", types.SimpleNamespace(batch=1, cin=20, size=1024)) is None
    # the keypoint-path dominant op (tools/pmc_bench.sh) is covered too
    assert bench.pmc_traffic("dx_init_conv.layer2", args) == by_label["dx_init_conv.layer2"]["hbm_bytes_per_launch"]


def test_plan_rejects_32bit_offset_overflow():
    """The kernels address tensor elements with 32-bit offsets: a tensor of >= 2^31
    elements (here the stem output of a 64 x 2048^2 batch) is refused at plan time."""
    import pytest as _pytest
    from instancesegmentation_amd.model.segment import Segment
    from instancesegmentation_amd.train import Trainer
    with _pytest.raises(RuntimeError, match="32-bit"):
        Trainer(Segment(20), 64, [(64, 3, 2048, 2048), (64, 17, 2048, 2048)], device="cpu")


def test_keypoint_stem_plan_and_synthetic_keypoints():
    """Segment(20) traced on (image, keypoints [N,17,3]): the stem's heatmap channels go to
    the keypoint records (pool, forward fix, weight gradient), the dense conv reads only the
    image with the weight's 20 input channels (w_ci), and the keypoints the synthetic batch
    reports redraw exactly its heatmaps."""
    import numpy as np
    from instancesegmentation_amd import _lib as L
    from instancesegmentation_amd.data import N_PARTS, keypoint_heatmaps, synthetic_batch
    from instancesegmentation_amd.engine import Plan
    m = Segment(20)
    p = Plan(m, [(2, 3, 64, 64), (2, 17, 3)], True, True, (False, False))
    kinds = [r.kind for r in p.fwd.recs]
    assert kinds.count(L.OP_KP_POOL) == 1 and kinds.count(L.OP_KP_STEM_FWD) == 1
    bk = [r for r in p.bwd.recs if r.kind == L.OP_KP_STEM_WGRAD]
    # the last records of the backward: on the main stream (engine._trailing_on_main), no
    # side record after the last main-stream record
    assert len(bk) == 1 and not bk[0].flags & 1
    last_main = max(i for i, r in enumerate(p.bwd.recs) if not r.flags & 1)
    assert p.bwd.recs.index(bk[0]) < last_main or all(r.flags & 1 == 0 for r in p.bwd.recs[last_main:])
    conv = next(r for r in p.fwd.recs if r.label == "init_conv.layer1")
    g = L.ConvRec.from_buffer_copy(conv.body).g
    assert (g.Ci, g.w_ci) == (3, 20)
    dense = Plan(m, [(2, 3, 64, 64), (2, 17, 64, 64)], True, True, (False, False))
    assert p.act_size == dense.act_size and p.graph.pgrad_size == dense.graph.pgrad_size
    kp = np.zeros((2, N_PARTS, 3))
    _, hm, mask = synthetic_batch(2, 96, 64, seed=7)
    _, none, mask2 = synthetic_batch(2, 96, 64, seed=7, with_heatmaps=False, keypoints_out=kp)
    assert none is None and np.array_equal(mask, mask2)
    for b in range(2):
        pts = {j: (kp[b, j, 0], kp[b, j, 1]) for j in range(N_PARTS) if kp[b, j, 2] > 0}
        assert np.array_equal(keypoint_heatmaps(pts, 96, 64), hm[b])


def _joined_before(recs, k):
    """The side-stream records (list indices) the main stream has waited for by the time
    record k runs, by the executor's rule (api.cpp isg_exec_ms2): a join with exclusion
    count e (header flags >> Record.EXCL_SHIFT, 0 < e <= side records so far) waits for all
    but the e most recent side records; any other join waits for every one."""
    from instancesegmentation_amd.engine import Record
    side, done = [], set()
    for j in range(k + 1):
        r = recs[j]
        if r.flags & Record.OPF_JOIN:
            e = r.flags >> Record.EXCL_SHIFT
            done |= set(side[:len(side) - e] if 0 < e <= len(side) else side)
        if r.flags & Record.OPF_SIDE:
            side.append(j)
    return done


def test_forward_side_branches_fork_and_join():
    """engine._fork_branches: the residual branches of BottleneckDown2 / BottleneckDim_Res /
    BottleneckUp_Res run on the side stream in the forward pass, and the first main-stream
    record that reads a branch's output joins the side stream first."""
    from instancesegmentation_amd.engine import Record
    m = Segment(20)
    p = Plan(m, [(2, 3, 128, 128), (2, 17, 3)], True, True, (False, False))
    recs = p.fwd.recs
    side_ops = [op for op in p.graph.ops if getattr(op, "side", False)]
    names = {op.out.name for op in side_ops}
    assert names == {"bottle1_1.pool", "bottle1_1.convm.0", "bottle2_1.pool",
                     "bottle2_1.convm.0", "bottle3_1.resconv.0", "bottle4_2.resconv.0",
                     "bottle4_1up.conv2.0", "bottle4_1up.uppool", "bottle5_1up.conv2.0",
                     "bottle5_1up.uppool"}
    side = [r for r in recs if r.flags & Record.OPF_SIDE]
    assert all(r.flags & Record.OPF_FORK_NOW for r in side)
    for op in side_ops:
        o = op.out.ptr()
        hi = o.off + op.out.numel * 4
        i = next(j for j, r in enumerate(recs) if r.label == op.out.name)
        assert recs[i].flags & Record.OPF_SIDE
        readers = [j for j, r in enumerate(recs[i + 1:], i + 1) if not r.flags & Record.OPF_SIDE
                   and any(fs == o.slot and o.off <= off < hi for _, fs, off in r.fix)]
        if readers:  # a join between the fork and the first main-stream reader, and one
            # that covers this record (a partial join excludes the side records after the
            # ones it reads)
            assert i in _joined_before(recs, readers[0]), op.out.name
    assert any(r.flags >> Record.EXCL_SHIFT for r in recs)  # partial joins are in use
    # backward: no branch work on the side stream (shared dx sinks); only bucket 1's
    # replica fold and gradient finalisation fork there (after every statistic is done),
    # and weight gradients (engine._fork_late_wgrads: the batch pending when the stem's
    # backward begins, and the stem's own weight gradients)
    assert not any(r.flags & Record.OPF_FORK_NOW for r in p.bwd.recs
                   if r.kind not in (L.OP_SUM_REP, L.OP_GRAD_FINAL, L.OP_CONV_WGRAD,
                                     L.OP_KP_STEM_WGRAD))
    assert all(r.flags & Record.OPF_SIDE for r in p.bwd.recs if r.flags & Record.OPF_FORK_NOW
               and r.kind in (L.OP_CONV_WGRAD, L.OP_KP_STEM_WGRAD))


def test_stamped_side_record_keeps_partial_joins_covering():
    """OpList.stamped(idx) on a forked forward record (bench.py times a side-stream op on
    the main stream): one side record fewer, so every partial join is recounted; every
    forked pool / branch output must still be joined before its first main-stream reader,
    by the executor's rule (_joined_before)."""
    from instancesegmentation_amd.engine import Record
    m = Segment(20)
    p = Plan(m, [(2, 3, 128, 128), (2, 17, 3)], True, True, (False, False))
    recs = p.fwd.recs
    outs = {op.out.name: op.out for op in p.graph.ops if getattr(op, "side", False)}

    def ranges(rs):
        for i, r in enumerate(rs):
            if not r.flags & Record.OPF_SIDE:
                continue
            if getattr(r, "out_range", None) is not None:
                yield i, r.out_range
            elif r.label in outs:
                o = outs[r.label].ptr()
                yield i, (o.slot, o.off, o.off + outs[r.label].numel * 4)

    side_idx = [i for i, r in enumerate(recs) if r.flags & Record.OPF_SIDE]
    assert len(side_idx) >= 6
    for idx in side_idx[:3] + side_idx[-3:]:
        st = p.fwd.stamped(idx).recs
        assert sum(1 for r in st if r.flags & Record.OPF_SIDE) == len(side_idx) - 1
        n = 0
        for i, (slot, lo, hi) in ranges(st):
            # (the moved record itself is no reader: the stem's two pools write disjoint
            # channel slices of init_down, the reason _fork_pools forks them together)
            readers = [j for j in range(i + 1, len(st)) if not st[j].flags & Record.OPF_SIDE
                       and st[j].label != recs[idx].label
                       and any(fs == slot and lo <= off < hi for _, fs, off in st[j].fix)]
            if readers:
                n += 1
                assert i in _joined_before(st, readers[0]), (recs[idx].label, st[i].label)
        assert n >= 4


def test_residual_tails_fold_into_the_next_1x1(monkeypatch):
    """engine._fold_tails: every Bottleneck3x3/5x5 tail act(BN(y) + x) whose output is read
    first by the next block's 1x1 conv is no launch of its own — forward: the conv record
    reads a BN_FWD segment with the residual and writes the tail's buffer (vtensor.mat);
    backward: the conv's input gradient carries the tail's backward (ACTBWD residual sink;
    where the residual term's gradient already holds a skip connection's part — the chain
    inputs of bottle1_x.0 / bottle2_x.0 — its second output accumulates).
    ISG_NO_TAIL_FOLD=1 off."""
    m = Segment(20)
    p = Plan(m, [(2, 3, 128, 128), (2, 17, 3)], True, True, (False, False))
    ops = p.graph.ops
    fwd = {t.out.name for t in ops if getattr(t, "fwd_folded", False)}
    bwd = {t.out.name for t in ops if getattr(t, "bwd_folded", False)}
    chain = [f"bottle1_x.{i}" for i in range(3)] + [f"bottle{s}_x.{i}" for s in (2, 3) for i in range(4)]
    # two-BatchNorm tails (BottleneckDown2, BottleneckDim_Res: act(BN(y) + BN2(r)))
    chain += ["bottle1_1", "bottle2_1", "bottle3_1", "bottle4_2"]
    # tails read by a side-branch 1x1 beside the next block's first 1x1 (BottleneckUp_Res's
    # conv2): both fold the tail on load, the main-stream one writes it, the side one (the
    # first reader) runs its backward
    chain += ["bottle3_x.4", "bottle4_3"]
    assert fwd == set(chain)
    assert bwd == set(chain)
    tails_f = [r for r in p.fwd.recs if r.kind == L.OP_TAIL_FWD]
    tails_b = [r for r in p.bwd.recs if r.kind == L.OP_TAIL_BWD]
    assert not any(r.label in fwd for r in tails_f)
    assert not any(r.label[2:] in bwd for r in tails_b)
    # the folded conv writes the tail's buffer: its record holds a pointer into it
    for t in ops:
        if getattr(t, "fwd_folded", False):
            readers = [op for op in ops if getattr(op, "res_in", None) is t]
            writers = [c for c in readers if c.res_mat]
            assert len(writers) == 1 and not getattr(writers[0], "side", False)
            o = t.out.ptr()
            for c in readers:
                r = next(r for r in p.fwd.recs if r.label == c.out.name)
                assert any(fs == o.slot and off == o.off for _, fs, off in r.fix) == c.res_mat
            bw = [op for op in ops if getattr(op, "res_tail", None) is t]
            assert len(bw) == 1 and bw[0] is min(readers, key=ops.index)
    monkeypatch.setenv("ISG_NO_TAIL_FOLD", "1")
    q = Plan(Segment(20), [(2, 3, 128, 128), (2, 17, 3)], True, True, (False, False))
    assert len([r for r in q.fwd.recs if r.kind == L.OP_TAIL_FWD]) == len(tails_f) + len(fwd)
    assert len([r for r in q.bwd.recs if r.kind == L.OP_TAIL_BWD]) == len(tails_b) + len(bwd)


def test_forward_fork_group_captured_behind_the_next_main_record(monkeypatch):
    """engine._delay_forks (ISG_FORK_DELAY=1, the default): the forward's first fork group
    (the replica memset and the stem's two pools) is captured after the stem's first conv,
    so that conv does not wait on the side queue's tail; every side record still precedes
    its join, and a group is never moved past a record that joins it. =0 keeps the capture
    order, =2 delays every group."""
    from instancesegmentation_amd import engine as E
    from instancesegmentation_amd.engine import Record

    def plan(mode):
        monkeypatch.setattr(E, "_FORK_DELAY", mode)
        return Plan(Segment(20), [(2, 3, 128, 128), (2, 17, 3)], True, True, (False, False))

    def check(recs):
        joins = [i for i, r in enumerate(recs) if r.flags & Record.OPF_JOIN]
        for i, r in enumerate(recs):
            if r.flags & Record.OPF_SIDE:  # a join follows every forked record
                assert any(j > i for j in joins), r.label

    p0, p1, p2 = plan("0"), plan("1"), plan("2")
    lab = lambda p: [r.label for r in p.fwd.recs]
    assert sorted(lab(p0)) == sorted(lab(p1)) == sorted(lab(p2))
    side0 = [r.label for r in p0.fwd.recs if r.flags & Record.OPF_SIDE]
    first = lab(p1).index("init_conv.layer1")
    assert lab(p0).index("init_conv.layer1") > lab(p0).index(side0[0])
    assert all(lab(p1).index(x) > first for x in ("zero_wgrad_replicas", "init_down",
                                                    "kp_pool_init_down"))
    for p in (p0, p1, p2):
        check(p.fwd.recs)
    # =1 moves only the first group: the later forward groups keep their places
    later = [x for x in side0 if x not in ("zero_wgrad_replicas", "init_down", "kp_pool_init_down")]
    assert [lab(p1).index(x) - lab(p1).index(later[0]) for x in later] == \
        [lab(p0).index(x) - lab(p0).index(later[0]) for x in later]


def test_residual_tails_fold_into_a_stacked_pair():
    """In the Trainer's flat parameter layout BottleneckUp_Res's convs.0 + conv2 run as one
    stacked GEMM (Graph.conv_pair) reading the previous tail: the pair takes that tail's
    forward on its input load (writing the tail's buffer) and its backward in the K-stacked
    input gradient's residual sink — bottle3_x.4 and bottle4_3 on top of the 15 folds."""
    from instancesegmentation_amd.engine import ConvPairOp, param_layout
    from instancesegmentation_amd.train import flatten_module
    m = Segment(20)
    lay = param_layout(m)
    flatten_module(m, "cpu", order=lay)
    p = Plan(m, [(2, 3, 128, 128), (2, 17, 3)], True, True, (False, False), layout=lay)
    ops = p.graph.ops
    pairs = {t.out.name: c for c in ops if isinstance(c, ConvPairOp) and c.res_in is not None
             for t in [c.res_in]}
    assert set(pairs) == {"bottle3_x.4", "bottle4_3"}
    for name, c in pairs.items():
        assert c.res_mat and c.res_tail is c.res_in and c.res_in.bwd_folded
        assert not any(r.kind == L.OP_TAIL_FWD and r.label == name for r in p.fwd.recs)
        assert not any(r.kind == L.OP_TAIL_BWD and r.label == "d_" + name for r in p.bwd.recs)
        dx = next(r for r in p.bwd.recs if r.label == "dx_" + c.label)
        assert dx.kind == L.OP_CONV_DGRAD and L.ConvRec.from_buffer_copy(dx.body).out.nsink == 1
    fwd = {t.out.name for t in ops if getattr(t, "fwd_folded", False)}
    assert len(fwd) == 17


class _Down2ThenDimRes(EngineModule):
    """A two-BatchNorm tail (BottleneckDown2: act(BN(y) + BN2(r))) read by a stacked sibling
    pair (BottleneckDim_Res's convs.0 + resconv) — no such edge exists in Segment(20)."""

    def __init__(self):
        super().__init__()
        self.down = BottleneckDown2(16, 8, 32)
        self.dimres = BottleneckDim_Res(32, 8, 48, True)

    def emit(self, g, x):
        y, _ = self.down.emit(g, x)
        return self.dimres.emit(g, y)


def _stacked_plan(m):
    from instancesegmentation_amd.engine import param_layout
    from instancesegmentation_amd.train import flatten_module
    lay = param_layout(m)
    flatten_module(m, "cpu", order=lay)
    return Plan(m, [(2, 16, 32, 32)], True, True, (False,), layout=lay)


def test_two_bn_tail_before_a_stacked_pair_stays_a_launch():
    """engine._fold_tails (cb9f310): a two-BatchNorm tail whose reader is a
    stacked pair is NOT folded (the residual's own BatchNorm rides on one sink in pw_gemm),
    so it keeps its own tail launch in both directions; the pair itself still stacks."""
    from instancesegmentation_amd.engine import ConvPairOp
    m = _Down2ThenDimRes()
    p = _stacked_plan(m)
    ops = p.graph.ops
    pair = [c for c in ops if isinstance(c, ConvPairOp)]
    assert len(pair) == 1 and pair[0].res_in is None
    assert not any(getattr(t, "fwd_folded", False) or getattr(t, "bwd_folded", False) for t in ops)
    # (out0: the output materialised into its slot)
    assert [r.label for r in p.fwd.recs if r.kind == L.OP_TAIL_FWD] == ["down", "dimres", "out0"]
    assert sorted(r.label for r in p.bwd.recs if r.kind == L.OP_TAIL_BWD) == ["d_dimres", "d_down", "d_out0"]


def test_stacked_pair_plan_rebuilt_when_weights_are_rebound_apart():
    """Plan.stacking_holds: a plan that runs a sibling pair as ONE stacked GEMM
    reads b's rows through a's pointer; once the weights stop being adjacent (here b's
    weight rebound to a copy of its own) the cached plan is no longer valid."""
    from instancesegmentation_amd.runtime import module_tensors
    m = _Down2ThenDimRes()
    p = _stacked_plan(m)
    assert len(p.graph.stacked) == 1
    assert p.stacking_holds(module_tensors(m))
    rc = m.dimres.resconv[0].conv
    rc.weight.data = rc.weight.detach().clone()
    assert not p.stacking_holds(module_tensors(m))
    q = Plan(m, [(2, 16, 32, 32)], True, True, (False,))  # layout order: no stacking at all
    assert q.graph.stacked == [] and q.stacking_holds(module_tensors(m))


def test_depthwise_backward_is_one_main_stream_op(monkeypatch):
    """Every depthwise layer's backward is one OP_DW_BWD record (isg_depthwise_bwd: input
    and weight gradient in one launch) on the main stream, with no depthwise weight gradient
    left on the side streams; ISG_NO_DW_FUSE=1 restores the dgrad + side-stream wgrad pair."""
    from instancesegmentation_amd.engine import ConvOp, Record
    m = Segment(20)
    p = Plan(m, [(2, 3, 128, 128), (2, 17, 3)], True, True, (False, False))
    dws = [op for op in p.graph.ops if isinstance(op, ConvOp) and op.geom["groups"] > 1]
    recs = [r for r in p.bwd.recs if r.kind == L.OP_DW_BWD]
    assert len(recs) == len(dws) > 0
    assert not any(r.flags & Record.OPF_SIDE for r in recs)
    names = {"dw_" + op.out.name for op in dws}
    assert not any(r.label in names for r in p.bwd.recs if r.kind == L.OP_CONV_WGRAD)
    monkeypatch.setenv("ISG_NO_DW_FUSE", "1")
    q = Plan(Segment(20), [(2, 3, 128, 128), (2, 17, 3)], True, True, (False, False))
    assert not any(r.kind == L.OP_DW_BWD for r in q.bwd.recs)
    assert sum(r.label in names for r in q.bwd.recs if r.kind == L.OP_CONV_WGRAD) == len(dws)


@pytest.mark.parametrize("n", [1, 2])
def test_forked_pools_join_before_any_reader_of_their_buffer(n):
    """engine._fork_pools at batch 1 and 2: the keypoint heatmaps' pool
    writes channels [3, 20) of init_down, but bottle1_1's convs read init_down from channel
    0. Every main-stream record whose pointer falls anywhere in a forked pool's output
    buffer must come after a join (at N == 1 the old start-pointer rule placed none)."""
    from instancesegmentation_amd.engine import Record
    m = Segment(20)
    p = Plan(m, [(n, 3, 64, 64), (n, 17, 3)], True, True, (False, False))
    recs = p.fwd.recs
    pools = [i for i, r in enumerate(recs) if r.kind in (L.OP_MAXPOOL_FWD, L.OP_KP_POOL)
             and r.flags & Record.OPF_SIDE]
    assert any(recs[i].kind == L.OP_KP_POOL for i in pools)
    for i in pools:
        slot, lo, hi = recs[i].out_range
        readers = [j for j in range(i + 1, len(recs)) if not recs[j].flags & Record.OPF_SIDE
                   and any(fs == slot and lo <= off < hi for _, fs, off in recs[j].fix)]
        if recs[i].kind == L.OP_KP_POOL:
            assert readers
        if readers:  # (bottle1_1.pool is read by side-stream branches only)
            assert i in _joined_before(recs, readers[0]), (n, recs[i].label, recs[readers[0]].label)


def test_library_has_no_undefined_isg_symbols():
    """Every isg_* function the library calls is defined in it: a C-ABI declaration in one
    translation unit against a C++-linkage definition in another links into a shared
    library with the symbol left undefined, and fails only when first called on a GPU."""
    import os
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(root, "instancesegmentation_amd", "libisg.so")
    nm = shutil.which("nm")
    if not nm or not os.path.exists(so):
        import pytest
        pytest.skip("nm or libisg.so missing")
    out = subprocess.run([nm, "-D", so], capture_output=True, text=True, check=True).stdout
    undef = [l.split()[-1] for l in out.splitlines() if " U " in l and l.split()[-1].startswith("isg_")]
    assert not undef, undef


def test_fused_step_tail_plan():
    """Plan(fused_tail=True) (the Trainer at world size 1): the forward has no BN-update
    list, the backward no replica fold / finalisation lists; it starts with the step
    counter forked on the side stream and ends in ONE OP_STEP_TAIL that joins every forked
    record; the item tables resolve to non-NULL pointers and the owned gradient ranges are
    exactly the grad_final outputs (BN gamma/beta, PReLU slopes, conv biases before BN)."""
    import ctypes
    from instancesegmentation_amd.engine import S_PGRAD, S_STATS, S_TENSOR0, Record, param_layout
    from instancesegmentation_amd.train import flatten_module
    m = Segment(20)
    lay = param_layout(m)
    flatten_module(m, "cpu", order=lay)
    shapes = [(2, 3, 128, 128), (2, 17, 3)]
    p = Plan(m, shapes, True, True, (False, False), buckets=1, layout=lay, fused_tail=True)
    q = Plan(m, shapes, True, True, (False, False), buckets=1, layout=lay)
    assert p.fused_tail and not q.fused_tail
    assert not any(r.kind == L.OP_BN_UPDATE for r in p.fwd.recs)
    assert not any(r.kind in (L.OP_SUM_REP, L.OP_GRAD_FINAL) for r in p.bwd.recs)
    first, last = p.bwd.recs[0], p.bwd.recs[-1]
    assert first.kind == L.OP_STEP_INC and first.flags & Record.OPF_SIDE and first.flags & Record.OPF_FORK_NOW
    assert last.kind == L.OP_STEP_TAIL and last.flags & Record.OPF_JOIN and not last.flags >> Record.EXCL_SHIFT
    assert [r.label for r in p.bwd.recs[1:-1]] == [r.label for r in q.bwd.recs
                                                   if r.kind not in (L.OP_SUM_REP, L.OP_GRAD_FINAL)]
    ngf = sum(len(r.body) - ctypes.sizeof(L.ListRec) for r in q.bwd.recs if r.kind == L.OP_GRAD_FINAL)
    nbnu = sum(len(r.body) - ctypes.sizeof(L.ListRec) for r in q.fwd.recs if r.kind == L.OP_BN_UPDATE)
    tab = (ctypes.c_void_p * (S_TENSOR0 + len(p.graph.tensor_names)))()
    for i in range(len(tab)):
        tab[i] = 0x100000 * (i + 1)
    gf, bnu = p.tail_tables(tab)
    assert len(gf) == ngf and len(bnu) == nbnu
    items = (L.GradFinal * (len(gf) // ctypes.sizeof(L.GradFinal))).from_buffer_copy(gf)
    base = tab[S_PGRAD]
    owned = set()
    for it in items:
        assert it.stats is None or it.stats >= tab[S_STATS]
        for f in ("dgamma", "dbeta", "dconv_bias", "dslope"):
            v = getattr(it, f)
            if v:
                owned |= set(range((v - base) // 4, (v - base) // 4 + it.C))
    want = set()
    for off, cnt in p.tail_owned:
        want |= set(range(off, off + cnt))
    assert owned == want and len(want) > 0
