"""Single-process unit tests: sharding, roles, datatypes, topologies, optimizer semantics
against pure-PyTorch oracles of the reference Lua, server rules end to end, checkpoints,
serialisation, metrics, tracing."""
import math
import os

import pytest
import torch

import mpit_amd as mp
from mpit_amd import datatypes as dt
from mpit_amd import launch, topology
from mpit_amd.ops import reference as R
from mpit_amd.parallel.ps import PClient, PServer, ServerOpt, reset_groups, shard_ranges


@pytest.fixture(scope="module")
def world():
    os.environ["MPIT_CPU_ONLY"] = "1"
    mp.Init()
    yield
    # Finalize at interpreter exit (other modules may reuse the runtime)


def test_shard_ranges_match_reference_split():
    # asyncsgd/pclient.lua:116-128: floor(P/S) each, remainder on the last shard
    assert shard_ranges(10, 3) == [(0, 3), (3, 3), (6, 4)]
    assert shard_ranges(7, 1) == [(0, 7)]
    assert sum(n for _, n in shard_ranges(25557032, 8)) == 25557032


def test_roles():
    assert launch.even_odd(6) == ([0, 2, 4], [1, 3, 5], [])
    assert launch.half_half(4) == ([0, 1], [2, 3], [])
    s, w, t = launch.master_freq(7, 3, "first")  # BiCNN/plaunch.lua:125-143
    assert t == [0] and s == [3, 6] and w == [1, 2, 4, 5]
    s, w, t = launch.master_freq(7, 3, "last")  # :145-163
    assert t == [6] and s == [2, 5] and w == [0, 1, 3, 4]
    assert launch.colocated(3) == ([0, 1, 2], [0, 1, 2], [])
    assert launch.dedicated(8, 1) == ([0], list(range(1, 8)), [])


def test_dims_create():
    assert topology.Dims_create(12, [0, 0]) == [4, 3]
    assert topology.Dims_create(8, [0, 0, 0]) == [2, 2, 2]
    assert topology.Dims_create(6, [0, 3]) == [2, 3]
    t = topology.CartTopo([2, 3], [True, False])
    assert t.coords(5) == [1, 2] and t.rank([1, 2]) == 5
    assert t.rank([2, 0]) == 0 and t.rank([0, 3]) == mp.PROC_NULL


def test_datatypes_pack_roundtrip():
    s = dt.Type_create_struct([1, 2], [0, 8], [dt.INT, dt.FLOAT]).Commit()
    assert s.Get_size() == 12 and s.Get_extent() == (0, 16)
    raw = torch.arange(32, dtype=torch.uint8)
    packed = s.pack(raw, 2)
    assert packed.tolist() == list(range(0, 4)) + list(range(8, 16)) + list(range(16, 20)) + list(range(24, 32))
    out = torch.zeros(32, dtype=torch.uint8)
    s.unpack(packed, out, 2)
    mask = torch.tensor([1] * 4 + [0] * 4 + [1] * 8 + [1] * 4 + [0] * 4 + [1] * 8, dtype=torch.bool)
    assert torch.equal(out[mask], raw[mask])
    sub = dt.Type_create_subarray([4, 4], [2, 2], [1, 1], dt.ORDER_C, dt.FLOAT)
    a = torch.arange(16, dtype=torch.float32)
    got = sub.pack(a, 1).view(torch.float32)
    assert got.tolist() == [5.0, 6.0, 9.0, 10.0]
    buf = torch.zeros(16, dtype=torch.uint8)
    pos = dt.Pack_external("external32", torch.tensor([1], dtype=torch.int32), 1, dt.INT, buf, 0)
    assert pos == 4 and buf[:4].tolist() == [0, 0, 0, 1]
    back = torch.zeros(1, dtype=torch.int32)
    dt.Unpack_external("external32", buf, 0, back, 1, dt.INT)
    assert back.item() == 1
    assert dt.Type_match_size(dt.TYPECLASS_REAL, 8) is dt.DOUBLE


def _feval_const(g):
    def f(w):
        return torch.tensor(0.0), g.clone()

    return f


def test_msgd_matches_reference(world):
    # asyncsgd/optim-msgd.lua, with momentum ramp off
    torch.manual_seed(0)
    w = torch.randn(1000)
    g = torch.randn(1000)
    wr, vr = w.clone(), torch.zeros(1000)
    cfg = dict(lr=0.1, mom=0.9, l2wd=1e-3, lrd=0.01, lrp=0.5)
    st = {}
    for t in range(3):
        mp.optim.msgd(_feval_const(g), w, cfg, st)
        vr, wr = R.nesterov_pre(vr, wr, 0.9)
        clr = 0.1 / (1 + t * 0.01) ** 0.5
        wr, vr = R.nesterov_post(wr, g, vr, None, clr, 1.0, 1e-3)
    torch.testing.assert_close(w, wr)
    assert st["pversion"] == 3


def _single_ps(plong, rule=None, init=None, dp=2):
    reset_groups()
    conf = dict(rank=0, sranks=[0], cranks=[0], plong=plong, opt=rule or ServerOpt("sum"), ps_id=7, datapath=dp)
    srv = PServer(conf)
    srv.start(block=False)
    pc = PClient(conf)
    p = init.clone() if init is not None else torch.zeros(plong)
    pc.start(p, torch.zeros(plong))
    return srv, pc


def test_downpour_semantics_single_worker(world):
    # su=1: the worker adopts the server weights each step (step 0 is a sync step)
    torch.manual_seed(1)
    w0 = torch.randn(512)
    g = torch.randn(512)
    srv, pc = _single_ps(512, init=w0)
    w = pc.rx
    cfg = dict(lr=0.5, su=1, pclient=pc)
    st = {}
    for _ in range(3):
        mp.optim.downpour(_feval_const(g), w, cfg, st)
    torch.testing.assert_close(w, w0 - 3 * 0.5 * g)
    torch.testing.assert_close(srv.p, w)
    pc.stop()
    srv.wait_done()


def test_downpour_su2_accumulates(world):
    torch.manual_seed(2)
    w0, g = torch.randn(256), torch.randn(256)
    srv, pc = _single_ps(256, init=w0)
    w = pc.rx
    cfg = dict(lr=0.25, su=2, pclient=pc)
    st = {}
    # step 0 (sync): acc = -lr g, push, pull -> w = w0 - lr g ; step 1 (local): w -= lr g
    mp.optim.downpour(_feval_const(g), w, cfg, st)
    torch.testing.assert_close(w, w0 - 0.25 * g)
    mp.optim.downpour(_feval_const(g), w, cfg, st)
    torch.testing.assert_close(w, w0 - 0.5 * g)
    torch.testing.assert_close(srv.p, w0 - 0.25 * g)  # server saw one push so far
    pc.stop()
    srv.wait_done()


def test_eamsgd_semantics(world):
    # asyncsgd/optim-eamsgd.lua with mom=0 (EASGD), su=1, one worker
    torch.manual_seed(3)
    w = torch.randn(300)
    g = torch.randn(300)
    center0 = w.clone() + 1.0  # server initialised from a different vector
    srv, pc = _single_ps(300, init=torch.zeros(300))
    pc.async_send_param(center0)
    pc.wait()
    cfg = dict(lr=0.1, mva=0.25, su=1, mom=0.0, pclient=pc)
    st = {}
    wr, cr = w.clone(), center0.clone()
    for _ in range(3):
        mp.optim.eamsgd(_feval_const(g), w, cfg, st)
        sug = 0.25 * (wr - cr)
        cr = cr + sug
        wr = wr - 0.1 * g - sug
    pc.wait()
    torch.testing.assert_close(w, wr)
    torch.testing.assert_close(srv.p, cr)
    pc.stop()
    srv.wait_done()


@pytest.mark.parametrize("rule", ["adam", "adamax", "adagrad", "adadelta", "rmsprop"])
def test_server_rules_end_to_end(world, rule):
    torch.manual_seed(4)
    n = 200
    p0 = torch.randn(n)
    g = torch.randn(n) * 0.1
    so = ServerOpt(rule, lr=0.01, decay=0.9, momentum=0.5, eps=1e-6, step_div=2, lr_decay=0.1)
    srv, pc = _single_ps(n, so, init=p0)
    cfg = dict(su=1, pclient=pc)
    st = {}
    w = pc.rx
    ref_p = p0.clone()
    s1, s2, s3 = torch.zeros(n), torch.zeros(n), torch.zeros(n)
    for t in range(1, 4):
        mp.optim.adam(_feval_const(g), w, cfg, st)  # global mode: raw gradient push + pull
        if rule == "adam":
            lr_t = mp.ops.adam_lr_t(0.01, 0.9, 0.999, t, 2)
            ref_p, s1, s2 = R.adam(ref_p, g, s1, s2, 0.9, 0.999, 1e-6, lr_t)
        elif rule == "adamax":
            ref_p, s1, s2 = R.adamax(ref_p, g, s1, s2, 0.9, 0.999, 1e-6, 0.01 / (1 - 0.9 ** t))
        elif rule == "adagrad":
            ref_p, s1 = R.adagrad(ref_p, g, s1, 1e-6, 0.01 / (1 + (t - 1) * 0.1))
        elif rule == "adadelta":
            ref_p, s1, s2 = R.adadelta(ref_p, g, s1, s2, 0.95, 1e-6, 0.01)
        else:
            ref_p, s1, s2, s3 = R.rmsprop(ref_p, g, s1, s2, s3, 0.9, 0.01, 0.5, 1e-6)
    torch.testing.assert_close(w, ref_p, rtol=1e-5, atol=1e-6)
    pc.stop()
    srv.wait_done()


def test_bounded_staleness_defers_fast_client(world):
    """SSP with staleness 0 and two clients: the second pull of a client that is ahead
    waits until the other client pushes (BASELINE config 4)."""
    from mp_util import run_ranks

    out = run_ranks("ssp_check.py", 3, {"MPIT_CPU_ONLY": "1"})
    assert "SSP_OK" in out and "SSP_PULL_OK" in out, out


def test_checkpoint_roundtrip(world, tmp_path):
    from mpit_amd.utils import checkpoint
    from mpit_amd.utils.flat import FlatParams

    m = torch.nn.Linear(10, 5)
    fp = FlatParams(m)
    st = {"vt": torch.randn(fp.numel), "pversion": 7}
    path = checkpoint.save(str(tmp_path), 3, 0, fp, st)
    saved = fp.flat.clone()
    with torch.no_grad():
        fp.flat.zero_()
    st2 = {"vt": torch.zeros(fp.numel)}
    checkpoint.load(checkpoint.latest(str(tmp_path), 0), fp, st2)
    assert torch.equal(fp.flat, saved) and torch.equal(st2["vt"], st["vt"]) and st2["pversion"] == 7
    assert path.endswith("_rank000.pt")


def test_serialize_and_metrics(tmp_path):
    from mpit_amd.utils.metrics import ConfusionMatrix, JsonLogger, RunningAverage
    from mpit_amd.utils.serialize import deserialize, serialize

    obj = {"a": torch.arange(4), "b": [1, 2.5, "x"]}
    back = deserialize(serialize(obj))
    assert torch.equal(back["a"], obj["a"]) and back["b"] == obj["b"]
    cm = ConfusionMatrix(3)
    cm.add(torch.tensor([0, 1, 2, 2]), torch.tensor([0, 1, 1, 2]))
    assert math.isclose(cm.total_valid, 0.75)
    lg = JsonLogger(str(tmp_path / "l.jsonl"))
    lg.log(loss=torch.tensor(1.5))
    lg.close()
    assert "1.5" in open(tmp_path / "l.jsonl").read()
    ra = RunningAverage(2)
    assert ra.add(1.0) is None and ra.add(3.0) == 2.0


def test_trace_and_pcontrol():
    from mpit_amd.utils import trace

    t = trace.Timers()
    with t("x"):
        pass
    assert t.count["x"] == 1
    mp.misc.Pcontrol(0)
    assert not trace.enabled()
    mp.misc.Pcontrol(1)
    with trace.range("r"):
        trace.mark("m")
    mp.misc.Pcontrol(0)


def test_info_errors_keyvals():
    from mpit_amd import misc

    i = misc.Info_create()
    i.Set("k", "v")
    assert i.Get_nkeys() == 1 and i.Get("k") == "v" and i.Get_nthkey(0) == "k" and i.Get_valuelen("k") == (1, True)
    c = misc.Add_error_class()
    code = misc.Add_error_code(c)
    misc.Add_error_string(code, "boom")
    assert misc.Error_class(code) == c and misc.Error_string(code) == "boom"
    assert "TRUNCATE" in misc.Error_string(misc.ERR_TRUNCATE)
    k = misc.Comm_create_keyval()
    assert misc.Comm_free_keyval(k) == misc.KEYVAL_INVALID


def test_bf16_wire_initialises_server_with_exact_fp32(world):
    """EASGD with a bf16 elastic-difference wire: the first client's fp32 weights reach the
    server shard bit for bit (the init push travels through the fp32 rx window,
    BiCNN/pserver.lua:272-278), not rounded through the bf16 push window."""
    reset_groups()
    torch.manual_seed(7)
    w = torch.randn(333) * 1.2345  # not representable in bf16
    conf = dict(rank=0, sranks=[0], cranks=[0], plong=333, opt=ServerOpt("sum"), ps_id=21,
                grad_dtype=torch.bfloat16)
    srv = PServer(conf)
    srv.start(block=False)
    pc = PClient(conf)
    pc.start(torch.zeros(333), torch.zeros(333, dtype=torch.bfloat16), init=w)
    pc.wait()
    srv.native.sync()
    assert torch.equal(srv.p.view(torch.int32), w.view(torch.int32))
    pc.stop()
    srv.wait_done()


def test_eamsgd_lr0_still_applies_elastic_step(world):
    """lr == 0: no local gradient step, but a sync step still pulls w toward the center by
    sug = mva*(w - center) (asyncsgd/optim-eamsgd.lua:69-70)."""
    torch.manual_seed(8)
    w = torch.randn(200)
    center = torch.randn(200)
    srv, pc = _single_ps(200, init=torch.zeros(200))
    pc.async_send_param(center)
    pc.wait()
    calls = []
    cfg = dict(lr=0.0, mva=0.3, su=1, mom=0.0, pclient=pc)
    w0 = w.clone()
    mp.optim.eamsgd(lambda x: calls.append(1) or (torch.tensor(0.0), torch.zeros_like(x)), w, cfg, {})
    pc.wait()
    sug = 0.3 * (w0 - center)
    torch.testing.assert_close(w, w0 - sug)
    torch.testing.assert_close(srv.p, center + sug)
    assert not calls  # no forward/backward at lr 0
    pc.stop()
    srv.wait_done()


def test_side_stream_cu_mask_spread():
    """MPIT_SIDE_CU_RESERVE keeps R CUs out of the side stream's mask, spread evenly over
    both candidate CU-id layouts (id % 8 and consecutive runs of 32)."""
    from mpit_amd.ops.conv import WgradStream

    for reserve in (32, 64):
        words = WgradStream.cu_mask(256, reserve)
        assert len(words) == 8
        off = [i for i in range(256) if not (words[i // 32] >> (i % 32)) & 1]
        assert len(off) == reserve
        assert all(sum(1 for i in off if i % 8 == x) == reserve // 8 for x in range(8))
        assert all(sum(1 for i in off if i // 32 == b) == reserve // 8 for b in range(8))


def test_inplace_grad_slots_skip_the_gather():
    """utils/flat.py grad_out: a backward writing its gradient straight into the flat
    gradient slot is not copied again by materialize(); the other gradients are gathered and
    the slots of parameters without a gradient are zeroed."""
    import torch.nn as nn

    from mpit_amd.utils.flat import FlatParams, grad_out

    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(8, 4), nn.Linear(4, 2))
    fp = FlatParams(m).steal_grads()
    w0 = m[0].weight
    g0 = grad_out(w0, w0.shape, w0.device)
    assert g0.data_ptr() == fp.grad.data_ptr() + fp.offsets[0] * fp.grad.element_size()
    assert grad_out(w0, (3, 3), w0.device).data_ptr() != g0.data_ptr()  # shape mismatch: a new tensor
    fp.grad.fill_(7.0)  # stale contents every slot must lose
    g0.fill_(3.0)
    w0.grad = g0  # as autograd steals it
    m[0].bias.grad = torch.full((4,), 1.0)
    m[1].weight.grad = torch.full((2, 4), 2.0)  # m[1].bias: no gradient this step
    out = fp.stolen().materialize()
    assert out.data_ptr() == fp.grad.data_ptr()
    seg = lambda i, p: out[fp.offsets[i]: fp.offsets[i] + p.numel()]  # noqa: E731
    assert torch.equal(seg(0, w0), torch.full((32,), 3.0))
    assert torch.equal(seg(1, m[0].bias), torch.full((4,), 1.0))
    assert torch.equal(seg(2, m[1].weight), torch.full((8,), 2.0))
    assert torch.equal(seg(3, m[1].bias), torch.zeros(2))
    assert all(p.grad is None for p in m.parameters())


def test_grad_slot_handed_out_once_per_step():
    """grad_out hands a parameter's flat-gradient slot to ONE backward per step: a second use
    of the same weight in one forward gets a fresh tensor (marked for the compute stream),
    which autograd then adds into the slot; gather() makes the slot available again."""
    import torch.nn as nn

    from mpit_amd.utils.flat import FlatParams, grad_out

    m = nn.Linear(4, 4)
    fp = FlatParams(m).steal_grads()
    w = m.weight
    slot = fp.grad.data_ptr() + fp.offsets[0] * fp.grad.element_size()
    g1 = grad_out(w, w.shape, w.device)
    g2 = grad_out(w, w.shape, w.device)
    assert g1.data_ptr() == slot and g2.data_ptr() != slot and getattr(g2, "_mpit_repeat", False)
    assert not getattr(g1, "_mpit_repeat", False)
    fp.stolen().materialize()
    assert grad_out(w, w.shape, w.device).data_ptr() == slot
