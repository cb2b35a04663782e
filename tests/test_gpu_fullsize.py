"""BASELINE configs 3 and 4 at their full sizes, and the packed delivery-record
kernel against the one-node-per-lane one at a config-5-shaped size.

Configs 3 and 4 (2^20 x 64, 2^24 x 256: the bench workload) are too large for
the oracle; here their first rounds are checked by the accounting laws of the
reference that a lost, duplicated or misrouted copy breaks
(src/gossip.rs:80,103,139,155): Statistics.rounds = rounds x n, every full copy
sent is received, known sets only grow, the processed flag
(src/gossiper.rs:209-212) agrees with the empty-push count, and no device limit
is hit.  Bit-exact checks of configs 3, 4 and 5 at full size, to termination,
are in test_gpu_dense_check.py (against oracle/gs_dense.c, which
test_dense_cpu.py holds equal to the oracle).

The packed DLV kernel (gs_dlv4.hip) is checked bit-exactly against the per-node
kernel of gs_kernels.hip -- itself bit-exact against the oracle at oracle sizes
(test_gpu_parity.py) -- on 2^24 + 12345 nodes x 16 rumors with config 5's
faults: every state code, Statistics row and known set, every round.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5AFE6055


@pytest.mark.parametrize("n,R,rounds", [(1 << 20, 64, 8), (1 << 24, 256, 5)])
def test_full_size_accounting(engine, n, R, rounds):
    net = engine.Network(n, R, seed=SEED)
    try:
        for r in range(R):
            net.send_new(engine.origin_of(SEED, 0, r, n), r)
        prev_known = net.known_all()
        prev = net.statistics_reduce("sum")
        for rnd in range(1, rounds + 1):
            rep = net.next_round()
            assert rep.round == rnd
            st = net.statistics_reduce("sum")
            assert st.rounds == rnd * n, f"round {rnd}: Statistics.rounds"
            assert st.full_message_received == st.full_message_sent, f"round {rnd}: copies lost"
            d_empty_push = st.empty_push_sent - prev.empty_push_sent
            assert rep.any_live == (d_empty_push < n), f"round {rnd}: processed flag"
            known = net.known_all()
            assert not np.any(prev_known & ~known), f"round {rnd}: a known rumor was lost"
            prev_known, prev = known, st
        t, _ = net.known_counts()
        assert t > R * 3 ** (rounds - 2)
        net.sync()  # no device limit hit
    finally:
        net.close()


def test_packed_dlv_matches_node_per_lane(engine, monkeypatch):
    n, R = (1 << 24) + 12345, 16
    faults = dict(churn=0.01, drop_push=0.01, drop_pull=0.01)
    monkeypatch.setenv("SAFE_GOSSIP_AMD_DLV_PACK", "1")
    a = engine.Network(n, R, seed=SEED, **faults)
    monkeypatch.setenv("SAFE_GOSSIP_AMD_DLV_PACK", "0")
    b = engine.Network(n, R, seed=SEED, **faults)
    try:
        for r in range(R):
            x = engine.origin_of(SEED, 0, r, n)
            a.send_new(x, r)
            b.send_new(x, r)
        for rnd in range(1, 7):
            ra, rb = a.next_round(), b.next_round()
            assert ra.any_live == rb.any_live
            np.testing.assert_array_equal(a.dump_state(), b.dump_state(), err_msg=f"state round {rnd}")
            np.testing.assert_array_equal(a.statistics_all(), b.statistics_all(),
                                          err_msg=f"statistics round {rnd}")
            np.testing.assert_array_equal(a.known_all(), b.known_all(), err_msg=f"known round {rnd}")
        a.sync()
        b.sync()
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("n", [(1 << 22) + 54321, (1 << 23) + 4321])
def test_dlv_partition_build_matches_gather_path(engine, monkeypatch, n):
    # The DLV build of networks with more than one coarse bucket (n > 2^21:
    # dl_coarse -> dl_fine -> inl_sort_dlv -> pb_fine -> pb_place) against the
    # class-plane gather path (SAFE_GOSSIP_AMD_NO_DLV=1: inl_bin / inl_sort and
    # the gathers of gs_kernels.hip), an independent build of the same round:
    # every state code, Statistics row and known set, every round, with faults.
    # 260 / 513 bins: quarter-bin sort parts over 3 / 5 coarse buckets, the
    # config-5 shape.
    R = 16
    faults = dict(churn=0.01, drop_push=0.01, drop_pull=0.01)
    a = engine.Network(n, R, seed=SEED, **faults)
    monkeypatch.setenv("SAFE_GOSSIP_AMD_NO_DLV", "1")
    b = engine.Network(n, R, seed=SEED, **faults)
    try:
        for r in range(R):
            x = engine.origin_of(SEED, 0, r, n)
            a.send_new(x, r)
            b.send_new(x, r)
        for rnd in range(1, 9):
            ra, rb = a.next_round(), b.next_round()
            assert ra.any_live == rb.any_live
            np.testing.assert_array_equal(a.dump_state(), b.dump_state(), err_msg=f"state round {rnd}")
            np.testing.assert_array_equal(a.statistics_all(), b.statistics_all(),
                                          err_msg=f"statistics round {rnd}")
            np.testing.assert_array_equal(a.known_all(), b.known_all(), err_msg=f"known round {rnd}")
        a.sync()
        b.sync()
    finally:
        a.close()
        b.close()


def test_w32_lane_kernel_matches_w64(engine, monkeypatch):
    # round_kernel_w32 (32-bit lanes, forced at R_pad 256; the default only at
    # R_pad 32, where a lane holds one node) against
    # the 64-bit lane round_kernel on a network larger than any oracle run:
    # 2^21 + 1234 nodes x 256 rumors with faults, a partial last block, every
    # state code, Statistics row and known set of 8 rounds
    n, R = (1 << 21) + 1234, 256
    faults = dict(churn=0.01, drop_push=0.02, drop_pull=0.02)
    monkeypatch.setenv("SAFE_GOSSIP_AMD_W32", "1")
    a = engine.Network(n, R, seed=SEED, **faults)
    monkeypatch.setenv("SAFE_GOSSIP_AMD_W32", "0")
    b = engine.Network(n, R, seed=SEED, **faults)
    try:
        for r in range(R):
            x = engine.origin_of(SEED, 0, r, n)
            a.send_new(x, r)
            b.send_new(x, r)
        for rnd in range(1, 9):
            ra, rb = a.next_round(), b.next_round()
            assert ra.any_live == rb.any_live
            if rnd % 2 == 0:
                np.testing.assert_array_equal(a.dump_state(), b.dump_state(), err_msg=f"state round {rnd}")
            np.testing.assert_array_equal(a.statistics_all(), b.statistics_all(),
                                          err_msg=f"statistics round {rnd}")
            np.testing.assert_array_equal(a.known_all(), b.known_all(), err_msg=f"known round {rnd}")
        a.sync()
        b.sync()
    finally:
        a.close()
        b.close()
