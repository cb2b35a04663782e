"""No entry returns to A: the oracle's known sets only grow, round by round.

The round kernels' all-A store skips (gs_kernels.hip GS_RK_ZSKIP,
gs_dlv4.hip GS_DLV4_ZSKIP, gs_w32.hip GS_W32_ZSKIP) rest on it: a wave or
block all-A in round t+1 was all-A in round t-1, whose planes the other state
buffer holds.  MessageState has no transition back to absent
(src/message_state.rs:86-171: B -> C -> D, D stays D); this checks the
restatement keeps that under both schedules, harness faults and rumors
injected in later rounds (the send_messages pattern, src/gossiper.rs:173-259).
"""
import numpy as np
import pytest

from oracle_lib import SCHED_2P, SCHED_SEQ, OracleNet, fault_threshold


@pytest.mark.parametrize("n,R,schedule,faults", [
    (200, 16, SCHED_SEQ, None),
    (150, 8, SCHED_SEQ, None),
    (300, 70, SCHED_2P, None),
    (400, 16, SCHED_2P, (0.05, 0.05, 0.05)),
    (250, 33, SCHED_SEQ, (0.05, 0.0, 0.0)),
])
def test_known_sets_only_grow(n, R, schedule, faults):
    fl = tuple(fault_threshold(p) for p in faults) if faults else None
    orc = OracleNet(n, R, seed=0xC0FFEE, faults=fl)
    rng = np.random.default_rng(n * 1000 + R)
    try:
        prev = orc.known_all()
        injected = 0
        for rnd in range(40):
            # a few new rumors at random nodes while slots remain (later rounds too)
            while injected < R and rng.random() < 0.5:
                orc.send_new(int(rng.integers(n)), injected)
                injected += 1
            rc, live = orc.next_round(schedule)
            assert rc == 0
            cur = orc.known_all()
            lost = prev & ~cur
            assert not lost.any(), f"round {rnd + 1}: {int(np.count_nonzero(lost))} words lost known bits"
            prev = cur
            if not live and injected == R:
                break
    finally:
        orc.close()
