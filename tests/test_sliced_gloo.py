"""Rumor-sliced protocol on CPU over torch.distributed (gloo, world 2 and 3).

Each process runs the reference-faithful oracle on its rumor slice only
(``[g*R//world, (g+1)*R//world)``, same seed and parameters: the same Philox
peer schedule and faults), reduces each round's empty-RPC counts with
``all_reduce(MIN)`` and sums the message counts -- the protocol of
``safe_gossip_amd/sliced.py`` and ``gs_slice_apply``.  Rank 0 checks the
gathered per-node state, records, |P|, Statistics and known sets against ONE
oracle over all R rumors, every round (bit-exact).  This pins the two facts
the sliced engine rests on: rumors evolve independently, and the network's
empty push / empty pull counts are the MIN over the slices.  Both hold under
the SEQ schedule too (the harness's literal order, src/gossiper.rs:217-234):
which pushes a node answers, and when, depends on the peer schedule only, and
"has a live entry" only ever turns on within a round, so a node's empty pulls
are a nondecreasing function of the first time it is live -- the MIN over the
slices again.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
SEED = 0x5AFE6055


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, R, params, kind, q, faults=None, sched="2P"):
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_lib
        from oracle_lib import SCHED_2P, SCHED_SEQ, OracleNet
        S = SCHED_SEQ if sched == "SEQ" else SCHED_2P
        L = oracle_lib.lib()
        thr = [oracle_lib.fault_threshold(p) for p in faults] if faults else None
        lo, hi = rank * R // world, (rank + 1) * R // world
        sl = OracleNet(n, hi - lo, seed=SEED, params=params, faults=thr)
        orc = OracleNet(n, R, seed=SEED, params=params, faults=thr) if rank == 0 else None
        rng = np.random.default_rng(n)
        prev = np.zeros((n, 5), dtype=np.int64)
        empties = np.zeros((n, 2), dtype=np.int64)  # network empty_pull / empty_push
        for rnd in range(1, 60):
            inj = []
            if kind == "origins" and rnd == 1:
                inj = [(L.or_origin(SEED, 0, r, n), r) for r in range(R)]
            if kind == "reinject" and rnd in (1, 2, 4):
                inj = [(int(rng.integers(n)), int(rng.integers(R))) for _ in range(R)]
            for x, r in inj:
                if 0 <= x < n and lo <= r < hi:
                    sl.send_new(x, r - lo)
                if orc:
                    orc.send_new(x, r)
            _, slive = sl.next_round(S)
            live = torch.tensor([int(slive)])
            dist.all_reduce(live, op=dist.ReduceOp.MAX)
            st = sl.statistics().astype(np.int64)
            d = torch.from_numpy(st[:, 1:3] - prev[:, 1:3])  # this round's, this slice
            prev = st
            dist.all_reduce(d, op=dist.ReduceOp.MIN)
            empties += d.numpy()
            full = torch.from_numpy(st[:, 3:5].copy())
            dist.all_reduce(full)
            rec, ps = sl.dump_records()
            part = (sl.dump_state(), rec, ps, sl.known_all())
            parts = [None] * world
            dist.all_gather_object(parts, part)
            if orc:
                _, olive = orc.next_round(S)
                assert bool(live.item()) == olive, f"round {rnd}: any_live"
                np.testing.assert_array_equal(np.concatenate([p[0] for p in parts], axis=1),
                                              orc.dump_state(), err_msg=f"state round {rnd}")
                orec, ops = orc.dump_records()
                np.testing.assert_array_equal(np.concatenate([p[1] for p in parts], axis=1), orec,
                                              err_msg=f"records round {rnd}")
                for p in parts:  # |peers_in_this_round| does not depend on the rumors
                    np.testing.assert_array_equal(p[2], ops, err_msg=f"psize round {rnd}")
                got = np.concatenate([st[:, :1], empties, full.numpy()], axis=1).astype(np.uint64)
                np.testing.assert_array_equal(got, orc.statistics(), err_msg=f"stats round {rnd}")
                bits = [np.unpackbits(p[3].view(np.uint8), axis=1, bitorder="little")[:, :b - a]
                        for p, a, b in zip(parts, [g * R // world for g in range(world)],
                                           [(g + 1) * R // world for g in range(world)])]
                ob = np.unpackbits(orc.known_all().view(np.uint8), axis=1, bitorder="little")[:, :R]
                np.testing.assert_array_equal(np.concatenate(bits, axis=1), ob)
            if not live.item():
                break
        sl.close()
        if orc:
            orc.close()
            q.put(("ok", rnd))
    except BaseException as e:  # report to the parent instead of hanging peers
        q.put(("fail", f"rank {rank}: {type(e).__name__}: {e}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,R,params,kind,faults", [
    (2, 600, 16, None, "origins", None),
    (2, 700, 8, (3, 2, 9), "reinject", None),
    (3, 600, 12, None, "origins", None),
    (3, 500, 7, None, "reinject", None),           # ragged slices 2/2/3
    (2, 600, 16, None, "origins", (0.1, 0.1, 0.1)),  # config 5 faults
    (3, 600, 8, None, "reinject", (0.3, 0.2, 0.2)),
    (2, 300, 2, (1, 1, 4), "reinject", None),      # one rumor per slice, cmax 1
])
def test_sliced_protocol_gloo(oracle, world, n, R, params, kind, faults):
    _run_world(world, n, R, params, kind, faults, "2P")


@pytest.mark.parametrize("world,n,R,params,kind,faults", [
    (2, 600, 16, None, "origins", None),
    (3, 500, 7, None, "reinject", None),             # ragged slices 2/2/3
    (3, 600, 8, None, "reinject", (0.2, 0.1, 0.1)),  # faults
    (2, 300, 2, (1, 1, 4), "reinject", None),        # one rumor per slice, cmax 1
])
def test_sliced_protocol_gloo_seq(oracle, world, n, R, params, kind, faults):
    # the SEQ schedule sliced: pull chains hop within a round, and the MIN of
    # the slices' empty counts is still the network's
    _run_world(world, n, R, params, kind, faults, "SEQ")


def _run_world(world, n, R, params, kind, faults, sched):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, R, params, kind, q, faults, sched))
             for r in range(world)]
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
    assert msgs and all(m[0] == "ok" for m in msgs), msgs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
