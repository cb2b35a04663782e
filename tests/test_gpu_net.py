"""The multi-GPU network behind the C ABI alone (gs_net_*, DESIGN.md section
7d), driven by a C++ host (examples/net_rounds.cpp: no Python anywhere in
the process) and compared with the oracle every round: state codes of every
(node, rumor), all five Statistics of every node, and the network's any-live
flag (the harness's `processed`, src/gossiper.rs:209-212).  Semantics:
src/gossip.rs:79-166, src/message_state.rs:86-171; the loop the library runs
is the one safe_gossip_amd/sharded.py and sliced.py run from Python.

Transports: RCCL with one rank (the process-per-GPU path: its collectives are
RCCL's on the rank's communication stream; RCCL refuses two ranks on one GPU,
so one box tests one rank) and the in-process "local" transport with 2-4
ranks on the one GPU (the same loop, exchanged by device copies)."""
import os
import subprocess

import numpy as np
import pytest

from oracle_lib import SCHED_2P, SCHED_SEQ, OracleNet

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "examples", "net_rounds")
SEED = 0x5AFE6055


def _run(tmp_path, mode, transport, world, parts, n, R, faults=None, schedule="2P", epoch=0, rounds=80):
    dump = tmp_path / f"{mode}_{transport}_{world}_{n}_{R}.bin"
    cmd = [EXE, "--mode", mode, "--transport", transport, "--world", str(world), "--parts", str(parts),
           "--nodes", str(n), "--rumors", str(R), "--seed", hex(SEED), "--epoch", str(epoch),
           "--schedule", schedule, "--rounds", str(rounds), "--dump", str(dump)]
    if faults:
        cmd += ["--churn", str(faults[0]), "--drop-push", str(faults[1]), "--drop-pull", str(faults[2])]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    raw = np.fromfile(dump, dtype=np.uint8)
    rec = 8 + n * R * 2 + n * 5 * 8
    assert raw.size % rec == 0
    out = []
    for i in range(raw.size // rec):
        b = raw[i * rec:(i + 1) * rec]
        head = b[:8].view(np.uint32)
        codes = b[8:8 + n * R * 2].view(np.uint16).reshape(n, R)
        stats = b[8 + n * R * 2:].view(np.uint64).reshape(n, 5)
        out.append((int(head[0]), bool(head[1]), codes, stats))
    return out, r.stdout


def _check(rounds, n, R, faults=None, schedule="2P", epoch=0):
    import safe_gossip_amd as sg
    thr = [sg.fault_threshold(p) for p in faults] if faults else None
    orc = OracleNet(n, R, seed=SEED, epoch=epoch, faults=thr)
    try:
        for r in range(R):
            orc.send_new(sg.origin_of(SEED, epoch, r, n), r)
        sched = SCHED_SEQ if schedule == "SEQ" else SCHED_2P
        for rnd, live, codes, stats in rounds:
            _, olive = orc.next_round(sched)
            assert rnd == orc.round
            assert live == bool(olive), f"round {rnd}: any_live"
            np.testing.assert_array_equal(codes, orc.dump_state(), err_msg=f"round {rnd}: state")
            np.testing.assert_array_equal(stats, orc.statistics(), err_msg=f"round {rnd}: statistics")
        assert not rounds[-1][1], "ran to termination"
    finally:
        orc.close()


@pytest.mark.parametrize("mode,transport,world,parts,n,R,faults,schedule", [
    # RCCL, one rank per process (the path a multi-process host runs)
    ("shards", "rccl", 1, 2, 3000, 16, (0.05, 0.05, 0.05), "2P"),   # code rows, rows in place
    ("shards", "rccl", 1, 3, 2000, 70, None, "2P"),                 # class rows, RCCL self exchange
    ("slices", "rccl", 1, 1, 2000, 64, (0.05, 0.05, 0.05), "2P"),
    ("slices", "rccl", 1, 1, 900, 20, None, "SEQ"),
    # every rank in this process, device copies (the same loop at world > 1)
    ("shards", "local", 2, 1, 600, 16, (0.05, 0.05, 0.05), "2P"),
    ("shards", "local", 3, 2, 1100, 70, None, "2P"),
    ("shards", "local", 4, 2, 2000, 256, (0.03, 0.03, 0.03), "2P"),
    ("slices", "local", 2, 1, 700, 9, (0.05, 0.05, 0.05), "2P"),     # uneven slices
    ("slices", "local", 3, 1, 500, 40, None, "SEQ"),
    ("slices", "local", 4, 1, 1500, 256, None, "2P"),
])
def test_net_matches_oracle(engine, tmp_path, mode, transport, world, parts, n, R, faults, schedule):
    rounds, line = _run(tmp_path, mode, transport, world, parts, n, R, faults, schedule)
    _check(rounds, n, R, faults, schedule)
    assert f'"world": {world}' in line and (f'"engines_here": {1 if transport == "rccl" else world}' in line)


def test_net_later_epoch(engine, tmp_path):
    # a later epoch (the bench times epoch 1) through the same C++ host
    rounds, _ = _run(tmp_path, "shards", "local", 2, 2, 1500, 32, None, "2P", epoch=3)
    _check(rounds, 1500, 32, None, "2P", epoch=3)


def _net_vs_oracle(sg, net, n, R, faults=None, schedule="2P"):
    thr = [sg.fault_threshold(p) for p in faults] if faults else None
    orc = OracleNet(n, R, seed=SEED, faults=thr)
    try:
        for r in range(R):
            x = sg.origin_of(SEED, 0, r, n)
            net.send_new(x, r)
            orc.send_new(x, r)
        for _ in range(80):
            rep = net.next_round()
            _, live = orc.next_round(SCHED_SEQ if schedule == "SEQ" else SCHED_2P)
            assert rep.any_live == bool(live)
            np.testing.assert_array_equal(net.dump_state(), orc.dump_state())
            np.testing.assert_array_equal(net.statistics_all(), orc.statistics())
            if not live:
                break
        assert net.known_counts()[0] == orc.known_total()
    finally:
        orc.close()


@pytest.mark.parametrize("mode,world,n,R,faults,schedule", [
    ("shards", 3, 900, 16, (0.05, 0.05, 0.05), "2P"),
    ("shards", 2, 800, 100, None, "2P"),
    ("slices", 3, 700, 30, (0.05, 0.05, 0.05), "SEQ"),
])
def test_python_net_local(engine, mode, world, n, R, faults, schedule):
    # the same library loop bound from Python (safe_gossip_amd.net.Net)
    from safe_gossip_amd.net import Net
    fk = dict(churn=faults[0], drop_push=faults[1], drop_pull=faults[2]) if faults else {}
    net = Net(n, R, world, mode=mode, seed=SEED, transport="local", parts=2, schedule=schedule, **fk)
    try:
        _net_vs_oracle(engine, net, n, R, faults, schedule)
    finally:
        net.close()


def _rccl_worker(port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        import safe_gossip_amd as sg
        from safe_gossip_amd.net import Net
        for mode, n, R in (("shards", 1500, 70), ("slices", 1200, 16)):
            net = Net(n, R, 1, mode=mode, seed=SEED, transport="dist", parts=3)
            try:
                _net_vs_oracle(sg, net, n, R)
            finally:
                net.close()
        q.put("ok")
    except BaseException as e:
        q.put(f"fail: {type(e).__name__}: {e}")
        raise
    finally:
        dist.destroy_process_group()


def test_python_net_rccl_one_rank(engine):
    # one RCCL rank in a torch.distributed process: the library's RCCL (the
    # one torch loaded) joined through an id broadcast over the process group
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    p = ctx.Process(target=_rccl_worker, args=(port, q))
    p.start()
    p.join(timeout=200)
    if p.is_alive():
        p.kill()
    assert not q.empty() and q.get() == "ok"
    assert p.exitcode == 0


def _host_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import safe_gossip_amd as sg
        from safe_gossip_amd.net import Net
        for mode, n, R, parts, faults, schedule in (
                ("shards", 1500, 70, 2, None, "2P"),                 # class rows, ids a round ahead
                ("shards", 2000, 16, 2, (0.05, 0.05, 0.05), "2P"),   # code rows, faults
                ("slices", 900, 9, 1, (0.05, 0.05, 0.05), "2P"),     # uneven slices
                ("slices", 700, 20, 1, None, "SEQ")):
            fk = dict(churn=faults[0], drop_push=faults[1], drop_pull=faults[2]) if faults else {}
            net = Net(n, R, world, mode=mode, seed=SEED, transport="host", parts=parts, schedule=schedule, **fk)
            try:
                _net_vs_oracle(sg, net, n, R, faults, schedule)
            finally:
                net.close()
        q.put("ok")
    except BaseException as e:
        q.put(f"fail: rank {rank}: {type(e).__name__}: {e}")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_net_multi_process_host_collectives(engine, world):
    # the library's loop in `world` processes sharing the one GPU, joined by
    # the host's collectives (gs_net_create_with over gloo): the multi-rank
    # paths of gs_net -- exchange regions of every part, the slices' MIN
    # reduction, the any-live reduction, observers gathered over the ranks --
    # each rank checked against the oracle every round
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_host_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
    msgs = []
    while not q.empty():
        msgs.append(q.get())
    assert len(msgs) == world and all(m == "ok" for m in msgs), msgs
    assert all(p.exitcode == 0 for p in procs)
