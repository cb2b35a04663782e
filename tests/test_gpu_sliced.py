"""Rumor-sliced engines (all nodes, a rumor slice per rank) vs CPU oracle, bit-exact.

`world` slice engines (gs_config.rumor_slice) hold the rumors [g*R//world,
(g+1)*R//world); each round's empty-RPC counts are reduced with MIN over the
slices and added back (gs_slice_apply), message counts are summed when
observed (safe_gossip_amd/sliced.py).  The observable
network must equal the unsliced one, which the oracle restates.  Transport
"local": the slices share one GPU and the MIN is a device reduction; "dist":
two processes over gloo (host-staged) and one RCCL rank (the all-reduce on the
process group's stream, applied on the engine stream one round later).
"""
import os
import socket
import sys
from dataclasses import astuple

import numpy as np
import pytest

from oracle_lib import SCHED_2P, OracleNet
from test_gpu_parity import SEED, run_parity

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _maker(world):
    from safe_gossip_amd.sliced import SlicedNetwork

    def make(n, R, seed, epoch, params, **faults):
        return SlicedNetwork(n, R, world, seed=seed, epoch=epoch, params=params, transport="local",
                             **faults)
    return make


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("n,R,kind,params", [
    (8, 4, "example", None),
    (5, 4, "trickle", None),
    (97, 16, "origins", None),
    (101, 32, "reinject", None),
    (300, 64, "trickle", None),
    (77, 100, "origins", None),        # ragged slices, R_g 25 / 33 / 50
    (130, 256, "reinject", None),      # wide slices (R_g >= 64)
    (300, 16, "origins", (3, 3, 14)),
    (1619, 4, "origins", None),
    (900, 7, "origins", (2, 3, 5)),
    (40, 8, "origins", (1, 1, 3)),
])
def test_sliced_parity(engine, world, n, R, kind, params):
    run_parity(engine, n, R, kind, params, make_net=_maker(world))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("n,R,kind,faults", [
    (8, 4, "example", (0.2, 0.1, 0.1)),
    (700, 6, "trickle", (0.1, 0.1, 0.1)),
    (600, 16, "origins", (0.05, 0.05, 0.05)),   # config 5 shape
    (520, 100, "reinject", (0.3, 0.2, 0.2)),
    (1000, 256, "origins", (0.1, 0.0, 0.3)),
])
def test_sliced_parity_faults(engine, world, n, R, kind, faults):
    run_parity(engine, n, R, kind, make_net=_maker(world), faults=faults)


@pytest.mark.parametrize("world,R", [(2, 128), (4, 256), (8, 256), (2, 32)])
def test_sliced_larger(engine, world, R):
    # the bench's slice shapes (R_g = 128 / 64 / 32 / 16) on 20k nodes
    run_parity(engine, 20000, R, "origins", check_every=4, make_net=_maker(world))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("n,R,kind,faults", [
    (8, 4, "example", None),
    (300, 16, "origins", None),
    (777, 20, "reinject", (0.05, 0.05, 0.05)),   # ragged slices, faults
    (130, 256, "origins", None),                 # wide slices (R_g >= 64)
    (1500, 32, "trickle", (0.1, 0.1, 0.1)),
])
def test_sliced_parity_seq(engine, world, n, R, kind, faults):
    # the SEQ schedule (the harness's literal order, src/gossiper.rs:217-234)
    # on rumor slices: each slice runs the SEQ kernels over its rumors, the
    # empty counts are the MIN over the slices (pinned on CPU by
    # tests/test_sliced_gloo.py::test_sliced_protocol_gloo_seq)
    run_parity(engine, n, R, kind, make_net=_maker(world), faults=faults, schedule="SEQ")


@pytest.mark.parametrize("pack", ["0", "u64", "u32x1", "default"])
def test_sliced_delivery_records(engine, monkeypatch, pack):
    # slices of R_g <= 16 run the delivery-record kernels (gs_dlv4.hip, and the
    # node-per-lane DLV kernel); config-5 faults
    if pack != "default":
        monkeypatch.setenv("SAFE_GOSSIP_AMD_DLV_PACK", pack)
    run_parity(engine, 700, 24, "origins", make_net=_maker(3), faults=(0.05, 0.05, 0.05))
    run_parity(engine, 2000, 16, "reinject", make_net=_maker(2))


def test_sliced_clear_and_counts(engine):
    from safe_gossip_amd.sliced import SlicedNetwork
    n, R = 500, 40
    net = SlicedNetwork(n, R, 3, transport="local")
    orc = OracleNet(n, R)
    for epoch in (0, 5):
        for r in range(R):
            x = engine.origin_of(SEED, epoch, r, n)
            net.send_new(x, r)
            orc.send_new(x, r)
        for _ in range(6):
            net.next_round()
            orc.next_round(SCHED_2P)
        np.testing.assert_array_equal(net.dump_state(), orc.dump_state())
        np.testing.assert_array_equal(net.statistics_all(), orc.statistics())
        kn = np.unpackbits(orc.known_all().view(np.uint8), axis=1, bitorder="little")[:, :R].sum(1)
        for mk in (1, 20, R):
            assert net.known_counts(mk) == (int(kn.sum()), int((kn >= mk).sum()))
        for op, f in (("sum", np.sum), ("min", np.min), ("max", np.max)):
            want = tuple(int(v) for v in f(orc.statistics(), axis=0))
            assert astuple(net.statistics_reduce(op)) == want, op
        net.clear(epoch=5)
        orc.clear(5)
        assert net.known_counts() == (0, 0)
    net.close()
    orc.close()


def test_slice_engine_refusals(engine):
    import safe_gossip_amd as sg
    from safe_gossip_amd.sliced import SlicedNetwork
    with pytest.raises(ValueError):
        SlicedNetwork(100, 2, 3, transport="local")  # fewer rumors than slices
    net = SlicedNetwork(100, 8, 2, transport="local")
    net.send_new(3, 5)
    net.next_round()
    net.next_round()
    frame = sg.rpc_encode(False, b"\x04\x00\x00\x00\x00\x00\x00\x00\x00\x00\x00\x05", 1)
    with pytest.raises(sg.GossipError):
        net.slices[0].net.handle_received(3, 1000, frame)  # no external RPCs on a slice
    s = net.slices[0]
    assert s.lib.gs_slice_defer(s.h, 3) != 0            # no such round buffer
    net.next_round()                                     # round 3: buffer 0 deferred
    assert s.lib.gs_slice_defer(s.h, 0) != 0            # deferring it twice would add it twice
    assert s.lib.gs_slice_apply(s.h, 0) == 0            # applying it now cancels the deferral
    orc = OracleNet(100, 8)
    orc.send_new(3, 5)
    for _ in range(3):
        orc.next_round(SCHED_2P)
    got = net.statistics_all()
    np.testing.assert_array_equal(got, orc.statistics())  # added exactly once
    orc.close()
    net.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cases, q, backend="gloo"):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        import safe_gossip_amd as sg
        from safe_gossip_amd.sliced import SlicedNetwork
        from test_gpu_parity import run_parity

        def make(n, R, seed, epoch, params, **faults):
            return SlicedNetwork(n, R, world, seed=seed, epoch=epoch, params=params, device=0,
                                 transport="dist", **faults)
        for n, R, kind, faults, *every in cases:
            if kind == "wire":  # external RPCs (tests/test_gpu_wire.py), answers all-gathered
                from test_gpu_wire import _batch_case, _handle_received_case, _push_batch_case

                def mk(n_, R_, **kw):
                    return SlicedNetwork(n_, R_, world, device=0, transport="dist", **kw)
                _handle_received_case(sg, n, R, faults, make=mk)
                _batch_case(sg, n, R, faults, "2P", make=mk)
                _push_batch_case(sg, n, R, faults, True, make=mk)
                continue
            if kind == "wire_limit":  # uneven slices: one network-wide first-Push bound
                from test_gpu_wire import _uneven_limit_case
                _uneven_limit_case(sg, lambda n_, R_: SlicedNetwork(n_, R_, world, device=0, transport="dist"))
                continue
            run_parity(sg, n, R, kind, make_net=make, faults=faults, check_every=every[0] if every else 1)
        q.put(("ok", rank))
    except BaseException as e:
        q.put(("fail", f"rank {rank}: {type(e).__name__}: {e}"))
        raise
    finally:
        dist.destroy_process_group()


def _spawn(world, cases, backend):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q, backend)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=200)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not q.empty():
        msgs.append(q.get())
    assert msgs and all(m[0] == "ok" for m in msgs), msgs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_sliced_dist_gloo_two_ranks(engine):
    _spawn(2, [(300, 64, "trickle", None), (600, 16, "origins", (0.05, 0.05, 0.05)),
               (130, 256, "reinject", None)], "gloo")


def test_sliced_dist_gloo_wire(engine):
    # the wire boundary on two slice processes: every rank makes the same
    # calls, the slices' answers are all-gathered and merged in key order
    _spawn(2, [(300, 16, "wire", None), (400, 64, "wire", (0.05, 0.05, 0.05)), (60, 9, "wire_limit", None)],
           "gloo")


def test_sliced_dist_rccl_single_rank(engine):
    # one RCCL rank: the all-reduce runs asynchronously on the process group's
    # stream and is applied on the engine stream a round later
    _spawn(1, [(300, 64, "trickle", None), (600, 16, "origins", (0.05, 0.05, 0.05)),
               (300, 16, "wire", (0.05, 0.05, 0.05))], "nccl")


def test_sliced_dist_rccl_deferred(engine):
    # the bench's path: rounds run unobserved, so each round's all-reduce is
    # folded into a later round kernel (gs_slice_defer, _apply_pending(keep=1))
    # instead of being applied by an observer; Statistics checked every 3rd /
    # 5th round against the oracle
    _spawn(1, [(300, 64, "trickle", None, 3), (600, 16, "origins", (0.05, 0.05, 0.05), 5),
               (130, 256, "origins", None, 4)], "nccl")
