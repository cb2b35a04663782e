"""Engine API behaviour beyond per-round parity: observers between send_new
and next_round, Gossiper::add_peer's AlreadyStarted rule, Statistics
reductions (add / min / max) and the device popcounts, each against the
CPU oracle or numpy over the engine's own per-node dumps."""
import numpy as np
import pytest

from oracle_lib import SCHED_2P, OracleNet

pytestmark = pytest.mark.gpu

SEED = 0x5AFE6055


def test_messages_visible_right_after_send_new(engine):
    # Gossip::new_message inserts MessageState::new at once
    # (src/gossip.rs:71-75): the origin knows the rumor before next_round,
    # in state B{round 0, our_counter 1}, and observing changes nothing.
    n, R = 300, 70
    net = engine.Network(n, R, seed=SEED)
    orc = OracleNet(n, R, seed=SEED)
    try:
        for _ in range(3):
            net.next_round()
            orc.next_round(SCHED_2P)
        inj = [(5, 3), (5, 64), (17, 69), (299, 0), (5, 3)]
        before = net.known_all()
        for x, r in inj:
            net.send_new(x, r)
            orc.send_new(x, r)
            assert r in net.gossiper(x).messages()
        known = net.known_all()
        exp = before.copy()
        for x, r in inj:
            exp[x, r >> 6] |= np.uint64(1) << np.uint64(r & 63)
        np.testing.assert_array_equal(known, exp)
        st = net.dump_state()
        for x, r in inj:
            assert st[x, r] == (1 << 14) | (1 << 7)
        rec, _ = net.dump_records()
        for x, r in inj:
            assert rec[x, r] == 0
        t, c = net.known_counts(min_known=1)
        assert t == int(sum(bin(int(w)).count("1") for w in exp.ravel()))
        # the next round is unchanged by the observation
        for _ in range(4):
            net.next_round()
            orc.next_round(SCHED_2P)
            np.testing.assert_array_equal(net.dump_state(), orc.dump_state())
            np.testing.assert_array_equal(net.statistics_all(), orc.statistics())
    finally:
        net.close()
        orc.close()


def test_add_peer_already_started(engine):
    # Gossiper::add_peer fails with AlreadyStarted once a message exists
    # (src/gossiper.rs:45-48); parameters follow Gossip::add_peer (gossip.rs:59-64)
    net = engine.Network(100, 4, seed=SEED)
    try:
        assert net.params == engine.derive_params(100)
        net.set_params((3, 2, 9))
        assert net.params == (3, 2, 9)
        net.set_params((0, 0, 0))
        assert net.params == engine.derive_params(100)
        with pytest.raises(engine.DeviceError, match="status -2"):
            net.set_params((4, 3, 9))       # outside the packed layout
        net.send_new(3, 1)
        with pytest.raises(engine.AlreadyStarted):
            net.set_params((2, 2, 5))
        net.next_round()
        with pytest.raises(engine.AlreadyStarted):
            net.set_params((2, 2, 5))
        net.clear()
        net.set_params((2, 2, 5))
        assert net.params == (2, 2, 5)
        # a message received from an outside peer creates an entry too
        net.clear()
        net.next_round()  # (external RPCs join a round after its deliveries)
        net.handle_received(7, 100, engine.rpc_encode(False, b"", 0))  # empty push: no entry
        net.set_params((2, 2, 6))
        net.handle_received(7, 100, engine.rpc_encode(False, net.rumor_key(2), 1))
        with pytest.raises(engine.AlreadyStarted):
            net.set_params((2, 2, 5))
    finally:
        net.close()


def test_set_params_parity(engine):
    # parameters changed through the add_peer path drive the same protocol
    # as the oracle with the same parameters
    from test_gpu_parity import run_parity

    def make(n, R, seed, epoch, params, **kw):
        net = engine.Network(n, R, seed=seed, epoch=epoch, **kw)
        net.set_params(params)
        return net
    run_parity(engine, 400, 24, "origins", params=(2, 3, 7), make_net=make)


@pytest.mark.parametrize("n,R,faults", [(2000, 64, None), (3000, 16, (0.1, 0.05, 0.05)),
                                         (500, 300, None)])
def test_statistics_reduce_and_popcounts(engine, n, R, faults):
    # Statistics::add / min / max (src/gossip.rs:236-263) on the device vs
    # numpy over the per-node statistics; known popcounts vs the known sets
    fk = dict(churn=faults[0], drop_push=faults[1], drop_pull=faults[2]) if faults else {}
    net = engine.Network(n, R, seed=SEED, **fk)
    try:
        for r in range(R):
            net.send_new(engine.origin_of(SEED, 0, r, n), r)
        for rnd in range(9):
            net.next_round()
            if rnd % 3 != 2:
                continue
            st = net.statistics_all()
            assert net.statistics_reduce("sum").as_tuple() == tuple(int(v) for v in st.sum(axis=0))
            assert net.statistics_reduce("min").as_tuple() == tuple(int(v) for v in st.min(axis=0))
            assert net.statistics_reduce("max").as_tuple() == tuple(int(v) for v in st.max(axis=0))
            known = net.known_all()
            pc = np.array([sum(bin(int(w)).count("1") for w in row) for row in known])
            np.testing.assert_array_equal(net.known_popcounts(), pc)
            for mk in (1, R // 2, R):
                t, c = net.known_counts(min_known=mk)
                assert t == int(pc.sum()) and c == int((pc >= mk).sum())
        net.sync()
    finally:
        net.close()


def test_sync_and_clear_report_no_limit(engine):
    # no device limit in a normal run: gs_sync / gs_clear return OK
    net = engine.Network(50_000, 32, seed=SEED)
    try:
        for r in range(32):
            net.send_new(engine.origin_of(SEED, 0, r, 50_000), r)
        for _ in range(5):
            net.next_round(report=False)
        net.sync()
        net.clear()
    finally:
        net.close()
