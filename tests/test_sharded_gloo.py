"""Sharded protocol on CPU over torch.distributed (gloo, world 2 and 3), with
code rows (R <= 16: one u32 push / pull code per row) and class rows.

Each process is one rank of tests/model_sharded.py: it owns a node range, moves
push rows to the owners of their targets and pull rows back with
equal-split all_to_all_single of fixed-size blocks (as the engine does: no
row counts are exchanged, each rank computes only its own sources' targets), ORs any-live with all_reduce, and rank 0 checks the
gathered per-node state, records, |P|, Statistics and known sets against the
reference-faithful oracle every round (bit-exact).
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


def _a2a(send, width):
    """Equal-split all-to-all of fixed-size blocks (the engine's exchanges)."""
    G = len(send)
    cap = len(send[0])
    assert all(len(p) == cap for p in send)
    flat = [v for part in send for row in part for v in row]
    inp = torch.tensor(flat, dtype=torch.int64) if flat else torch.zeros(0, dtype=torch.int64)
    out = torch.empty(G * cap * width, dtype=torch.int64)
    dist.all_to_all_single(out, inp)
    vals = out.tolist()
    return [[vals[(s * cap + i) * width:(s * cap + i + 1) * width] for i in range(cap)]
            for s in range(G)]


def _worker(rank, world, port, n, R, params, kind, q, faults=None, parts=1):
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_lib
        from model_sharded import ShardModel
        from oracle_lib import SCHED_2P, OracleNet
        L = oracle_lib.lib()
        thr = [oracle_lib.fault_threshold(p) for p in faults] if faults else None
        orc = OracleNet(n, R, seed=SEED, params=params, faults=thr) if rank == 0 else None
        prm = params or oracle_lib.derive_params(n)
        fault_fn = (lambda rnd, x: L.or_fault(SEED, 0, rnd, x, *thr)) if faults else None
        sm = ShardModel(n, R, SEED, 0, prm, L.or_peer, rank, world, _a2a, fault_fn, parts)
        rng = np.random.default_rng(n)
        for rnd in range(1, 50):
            inj = []
            if kind == "origins" and rnd == 1:
                inj = [(L.or_origin(SEED, 0, r, n), r) for r in range(R)]
            if kind == "reinject" and rnd in (1, 2, 4):
                inj = [(int(rng.integers(n)), int(rng.integers(R))) for _ in range(R)]
            for x, r in inj:
                if sm.lo <= x < sm.lo + sm.m:
                    sm.send_new(x, r)
                if orc:
                    orc.send_new(x, r)
            live = torch.tensor([int(sm.next_round())])
            dist.all_reduce(live, op=dist.ReduceOp.MAX)
            part = sm.observe_local()
            parts = [None] * world
            dist.all_gather_object(parts, part)
            if orc:
                _, olive = orc.next_round(SCHED_2P)
                assert bool(live.item()) == olive, f"round {rnd}: any_live"
                cat = [sum((p[i] for p in parts), []) for i in range(5)]
                codes, recs, psz, stats, known = cat
                np.testing.assert_array_equal(np.array(codes, np.uint16), orc.dump_state(),
                                              err_msg=f"state round {rnd}")
                orec, ops = orc.dump_records()
                psz, recs = np.array(psz, np.uint32), np.array(recs, np.uint16)
                if faults:  # offline nodes: stale records in the oracle, votes only here
                    off = orc.offline(rnd)
                    psz[off] = ops[off] = 0
                    recs[off] = orec[off] = 0
                np.testing.assert_array_equal(psz, ops)
                np.testing.assert_array_equal(recs, orec)
                np.testing.assert_array_equal(np.array(stats, np.uint64), orc.statistics())
                ok = orc.known_all()
                assert known == [int(ok[x][0]) for x in range(n)]
            if not live.item():
                break
        if orc:
            orc.close()
            q.put(("ok", rnd))
    except BaseException as e:  # report to the parent instead of hanging peers
        q.put(("fail", f"rank {rank}: {type(e).__name__}: {e}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,R,params,kind,faults,parts", [
    (2, 600, 16, None, "origins", None, 1),      # ranks own 512 / 88 nodes
    (2, 700, 8, (3, 2, 9), "reinject", None, 1),
    (3, 600, 12, None, "origins", None, 1),      # 256 / 256 / 88
    (2, 600, 16, None, "origins", (0.1, 0.1, 0.1), 1),    # config 5 faults
    (3, 600, 8, None, "reinject", (0.3, 0.2, 0.2), 1),
    (2, 5000, 16, None, "origins", None, 2),     # code rows: pipeline parts of 2048 / 512 nodes
    (3, 1600, 8, None, "reinject", (0.1, 0.1, 0.1), 3),  # 3 parts asked, 1 of 1024 nodes holds the range
    (2, 600, 40, None, "origins", None, 1),      # class rows (R_pad 64)
    (2, 1100, 33, None, "origins", None, 2),     # class rows: pipeline parts of 256 nodes
    (3, 1600, 20, None, "reinject", (0.1, 0.1, 0.1), 3),
])
def test_sharded_protocol_gloo(oracle, world, n, R, params, kind, faults, parts):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, R, params, kind, q, faults, parts))
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
