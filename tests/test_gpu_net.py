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
