"""Byte-level boundary on the GPU engine, against the CPU oracle:

* gs_push_batch = the bincode Push RPCs ``Gossiper::next_round`` returns
  (src/gossiper.rs:70-79, src/gossip.rs:79-113), in message-key order;
* gs_handle_received = ``Gossiper::handle_received_message`` (src/gossiper.rs:
  82-99 -> src/gossip.rs:118-166) from peers outside the simulated network,
  applied after the round's internal deliveries: the Pull responses must be
  the oracle's, and the state, records, |P|, Statistics and known sets after
  them -- and every later round -- must stay bit-exact.
"""
import numpy as np
import pytest

from oracle_lib import SCHED_2P, SCHED_SEQ, OracleNet
from test_gpu_parity import SEED

pytestmark = pytest.mark.gpu


def _decode_batch(engine, net, frames, pull):
    key_rumor = {net.rumor_key(r): r for r in range(net.R)}
    out = []
    for f in frames:
        p, msg, ctr = engine.rpc_decode(f)
        assert p == pull
        out.append((-1 if (msg == b"" and ctr == 0) else key_rumor[msg], ctr))
    return out


def _key_sorted(net, lst):
    # the oracle's maps are in rumor-index order; the reference's in key order
    return sorted(lst, key=lambda rc: net.rumor_key(rc[0]) if rc[0] >= 0 else b"")


def _compare(net, orc, off=None):
    """Records and |P| of nodes offline this round are the oracle's stale
    ones (see test_gpu_parity.run_parity); their state is compared."""
    np.testing.assert_array_equal(net.dump_state(), orc.dump_state())
    grec, gps = net.dump_records()
    orec, ops = orc.dump_records()
    if off is not None:
        grec[off] = orec[off] = 0
        gps[off] = ops[off] = 0
    np.testing.assert_array_equal(gps, ops)
    np.testing.assert_array_equal(grec, orec)
    np.testing.assert_array_equal(net.statistics_all(), orc.statistics())
    np.testing.assert_array_equal(net.known_all(), orc.known_all())


@pytest.mark.parametrize("n,R,faults,custom_keys", [
    (300, 16, None, False),          # delivery-record path
    (200, 64, None, True),           # gather path, keys whose byte order is not slot order
    (150, 130, (0.1, 0.05, 0.05), False),
    (400, 8, (0.05, 0.05, 0.1), True),
])
def test_push_batches_match_oracle(engine, n, R, faults, custom_keys):
    _push_batch_case(engine, n, R, faults, custom_keys)


def _push_batch_case(engine, n, R, faults, custom_keys, make=None):
    fk = dict(churn=faults[0], drop_push=faults[1], drop_pull=faults[2]) if faults else {}
    from oracle_lib import fault_threshold
    net = (make or engine.Network)(n, R, seed=SEED, **fk)
    orc = OracleNet(n, R, seed=SEED, faults=[fault_threshold(p) for p in faults] if faults else None)
    rng = np.random.default_rng(n + R)
    if custom_keys:
        for r in range(R):
            net.set_rumor_key(r, bytes(rng.integers(0, 256, size=int(rng.integers(1, 30)), dtype=np.uint8)))
    try:
        for r in range(R):
            x = engine.origin_of(SEED, 0, r, n)
            net.send_new(x, r)
            orc.send_new(x, r)
        for rnd in range(8):
            net.next_round()
            orc.next_round(SCHED_2P)
            for x in list(range(0, n, max(1, n // 40))) + [n - 1]:
                got = _decode_batch(engine, net, net.push_batch(x), pull=False)
                exp = _key_sorted(net, orc.push_list(x))
                assert got == exp, f"round {rnd + 1} node {x}: {got} vs {exp}"
    finally:
        net.close()
        orc.close()


@pytest.mark.parametrize("n,R,faults", [
    (300, 16, None),                  # delivery-record path
    (250, 64, None),                  # gather path, one word
    (120, 200, (0.05, 0.05, 0.05)),   # several words, faults
    (500, 4, (0.1, 0.1, 0.1)),
])
def test_handle_received_matches_oracle(engine, n, R, faults):
    _handle_received_case(engine, n, R, faults)


@pytest.mark.parametrize("n,R,faults", [
    (300, 16, None),                  # SEQ over R_pad 16 (gather path: DLV is 2P only)
    (250, 64, None),
    (120, 200, (0.05, 0.05, 0.05)),
])
def test_handle_received_seq(engine, n, R, faults):
    # the SEQ schedule (the reference harness's literal order): external RPCs
    # after the round's internal deliveries, as under 2P
    _handle_received_case(engine, n, R, faults, schedule="SEQ")


def _handle_received_case(engine, n, R, faults, schedule="2P", make=None):
    from oracle_lib import fault_threshold
    fk = dict(churn=faults[0], drop_push=faults[1], drop_pull=faults[2]) if faults else {}
    if schedule != "2P":
        fk["schedule"] = schedule
    osched = SCHED_SEQ if schedule == "SEQ" else SCHED_2P
    net = (make or engine.Network)(n, R, seed=SEED, **fk)
    orc = OracleNet(n, R, seed=SEED, faults=[fault_threshold(p) for p in faults] if faults else None)
    rng = np.random.default_rng(7 * n + R)
    params = net.params
    try:
        for r in range(0, R, 2):  # half the rumors start inside the network
            x = engine.origin_of(SEED, 0, r, n)
            net.send_new(x, r)
            orc.send_new(x, r)
        for rnd in range(1, 10):
            net.next_round()
            orc.next_round(osched)
            off = orc.offline(rnd) if faults else np.zeros(n, dtype=bool)
            if rnd in (2, 3, 5):
                # external peers n+1.. push / pull single rumors (some twice,
                # some empty) into a few nodes, after the round's deliveries
                for _ in range(25):
                    y = int(rng.integers(n))
                    peer = n + 1 + int(rng.integers(6))
                    push = bool(rng.random() < 0.6)
                    if rng.random() < 0.15:
                        rumor, ctr = -1, 0
                    else:
                        rumor = int(rng.integers(R))
                        ctr = int(rng.choice([0, 1, 2, 3, 7, 255, params[0] - 1 if params[0] > 1 else 1]))
                    msg = b"" if rumor < 0 else net.rumor_key(rumor)
                    got = _decode_batch(engine, net, net.handle_received(y, peer, engine.rpc_encode(not push, msg, ctr)),
                                        pull=True)
                    # a node offline this round (churn) drops it, like every RPC to it
                    exp = [] if off[y] else orc.receive(y, peer, push, rumor, ctr)
                    assert got == _key_sorted(net, exp), f"round {rnd} node {y} peer {peer}"
            if rnd in (2, 3, 5) or rnd % 2 == 0:
                _compare(net, orc, off)
    finally:
        net.close()
        orc.close()


def test_handle_received_errors(engine):
    net = engine.Network(50, 8, seed=SEED)
    try:
        msg = engine.rpc_encode(False, net.rumor_key(3), 1)
        with pytest.raises(engine.DeviceError, match="status -1"):
            net.handle_received(0, 55, msg)        # before the first round
        net.next_round()
        with pytest.raises(engine.DeviceError, match="status -1"):
            net.handle_received(0, 10, msg)        # peer inside the simulated network
        with pytest.raises(engine.DeviceError, match="status -1"):
            net.handle_received(0, 55, engine.rpc_encode(False, b"no such rumor", 1))
        with pytest.raises(engine.GossipError, match="status 5"):
            net.handle_received(0, 55, b"\x07\x00")  # undecodable
        # a first Push from a new peer is answered: node 0 knows nothing yet
        assert net.handle_received(0, 55, msg) == [engine.rpc_encode(True, b"", 0)]
        # its copy created rumor 3 at node 0, visible at once
        assert 3 in net.gossiper(0).messages()
        # a second Push from the same peer this round gets no responses
        assert net.handle_received(0, 55, engine.rpc_encode(False, net.rumor_key(5), 1)) == []
        # a Pull never gets responses
        assert net.handle_received(1, 56, engine.rpc_encode(True, net.rumor_key(5), 255)) == []
        with pytest.raises(engine.DeviceError, match="status -1"):
            net.set_rumor_key(2, net.rumor_key(3))  # keys are distinct
    finally:
        net.close()


@pytest.mark.parametrize("n,R,faults,schedule", [
    (2000, 16, None, "2P"),                  # delivery-record path
    (1500, 64, (0.05, 0.05, 0.05), "2P"),    # gather path, faults
    (800, 200, None, "2P"),                  # several words
    (1000, 64, None, "SEQ"),
])
def test_handle_received_batch_matches_oracle(engine, n, R, faults, schedule):
    # gs_handle_received_batch: 1000 external RPCs in one call (one
    # observation launch) = the same RPCs one by one through the oracle's
    # Gossip::receive (src/gossiper.rs:82-99 -> src/gossip.rs:118-166): every
    # response, then state, records, |P|, Statistics and known sets, and the
    # rounds after -- with repeated peers, repeated nodes (responses that show
    # the batch's earlier creations), empty RPCs and pulls
    _batch_case(engine, n, R, faults, schedule)


def _batch_case(engine, n, R, faults, schedule, make=None):
    from oracle_lib import fault_threshold
    fk = dict(churn=faults[0], drop_push=faults[1], drop_pull=faults[2]) if faults else {}
    if schedule != "2P":
        fk["schedule"] = schedule
    osched = SCHED_SEQ if schedule == "SEQ" else SCHED_2P
    net = (make or engine.Network)(n, R, seed=SEED, **fk)
    orc = OracleNet(n, R, seed=SEED, faults=[fault_threshold(p) for p in faults] if faults else None)
    rng = np.random.default_rng(11 * n + R)
    params = net.params
    try:
        for r in range(0, R, 2):
            x = engine.origin_of(SEED, 0, r, n)
            net.send_new(x, r)
            orc.send_new(x, r)
        for rnd in range(1, 8):
            net.next_round()
            orc.next_round(osched)
            off = orc.offline(rnd) if faults else np.zeros(n, dtype=bool)
            if rnd in (2, 4):
                hot = rng.integers(n, size=40)  # nodes hit many times
                rpcs, exp = [], []
                for _ in range(1000):
                    y = int(hot[rng.integers(40)] if rng.random() < 0.5 else rng.integers(n))
                    peer = n + 1 + int(rng.integers(30))
                    push = bool(rng.random() < 0.6)
                    if rng.random() < 0.1:
                        rumor, ctr = -1, 0
                    else:
                        rumor = int(rng.integers(R))
                        ctr = int(rng.choice([0, 1, 2, 3, 255, params[0] - 1 if params[0] > 1 else 1]))
                    msg = b"" if rumor < 0 else net.rumor_key(rumor)
                    rpcs.append((y, peer, engine.rpc_encode(not push, msg, ctr)))
                    exp.append([] if off[y] else orc.receive(y, peer, push, rumor, ctr))
                got = net.handle_received_batch(rpcs)
                assert len(got) == len(rpcs)
                for i, (g, e_) in enumerate(zip(got, exp)):
                    assert _decode_batch(engine, net, g, pull=True) == _key_sorted(net, e_), f"round {rnd} rpc {i}"
                _compare(net, orc, off)
            if rnd % 2 == 1:
                _compare(net, orc, off)
    finally:
        net.close()
        orc.close()


def test_handle_received_batch_all_or_nothing(engine):
    net = engine.Network(60, 8, seed=SEED)
    try:
        net.next_round()
        ok = engine.rpc_encode(False, net.rumor_key(3), 1)
        with pytest.raises(engine.GossipError, match="status 5"):  # one undecodable message: nothing applied
            net.handle_received_batch([(0, 70, ok), (1, 71, b"\x07\x00")])
        assert 3 not in net.gossiper(0).messages()
        # applied once it is well formed: node 0 answers its first Push (knows nothing yet)
        assert net.handle_received_batch([(0, 70, ok), (1, 71, ok)]) == [[engine.rpc_encode(True, b"", 0)]] * 2
        assert net.handle_received_batch([]) == []
    finally:
        net.close()


# ---------------------------------------------------------------- multi-engine networks
# The same boundary on a network split over several engines (local transport,
# one GPU): rumor slices (every slice takes every RPC, the owner's as sent and
# the others' emptied; answers merged in key order; safe_gossip_amd/sliced.py)
# and class-row node shards (the RPC goes to the shard owning the node, a
# global id; safe_gossip_amd/sharded.py).  Same oracle, same checks.

def _sliced(world):
    from safe_gossip_amd.sliced import SlicedNetwork
    return lambda n, R, **kw: SlicedNetwork(n, R, world, transport="local", **kw)


def _sharded(world, parts):
    from safe_gossip_amd.sharded import ShardedNetwork
    return lambda n, R, **kw: ShardedNetwork(n, R, world, transport="local", parts=parts, **kw)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("n,R,faults,schedule", [
    (300, 16, None, "2P"),                 # slices of R_pad 8 (delivery records)
    (250, 64, None, "2P"),
    (120, 200, (0.05, 0.05, 0.05), "2P"),  # ragged wide slices, faults
    (500, 4, (0.1, 0.1, 0.1), "2P"),
    (250, 64, None, "SEQ"),
])
def test_handle_received_sliced(engine, world, n, R, faults, schedule):
    _handle_received_case(engine, n, R, faults, schedule, make=_sliced(world))


@pytest.mark.parametrize("world,parts", [(2, 1), (3, 2)])
@pytest.mark.parametrize("n,R,faults", [
    (250, 64, None),
    (120, 200, (0.05, 0.05, 0.05)),
    (900, 100, (0.1, 0.1, 0.1)),           # every rank owns nodes
])
def test_handle_received_sharded(engine, world, parts, n, R, faults):
    _handle_received_case(engine, n, R, faults, make=_sharded(world, parts))


@pytest.mark.parametrize("world,parts,n,R,faults", [
    (2, 2, 5000, 16, (0.05, 0.05, 0.05)),   # R_pad 16: two nodes per lane
    (3, 1, 3000, 5, None),                  # R_pad 8: four nodes per lane
])
def test_handle_received_sharded_code_rows(engine, world, parts, n, R, faults):
    # code rows (R_pad <= 16, 2P): the packed DLV round kernel's external-RPC
    # variant applies the queue (gs_dlv4.hip EXT); observers unpack the pulls
    _handle_received_case(engine, n, R, faults, make=_sharded(world, parts))


def test_handle_received_sharded_class_rows_small_r(engine, monkeypatch):
    # R_pad <= 16 with SAFE_GOSSIP_AMD_NO_DLV=1: class rows, external RPCs apply
    monkeypatch.setenv("SAFE_GOSSIP_AMD_NO_DLV", "1")
    _handle_received_case(engine, 600, 16, (0.05, 0.05, 0.05), make=_sharded(3, 2))


@pytest.mark.parametrize("make", [_sliced(3), _sharded(3, 2)], ids=["sliced", "sharded"])
@pytest.mark.parametrize("n,R,faults,custom_keys", [
    (300, 16, None, True),
    (150, 130, (0.1, 0.05, 0.05), True),
    (600, 64, None, False),
])
def test_push_batches_multi_engine(engine, make, n, R, faults, custom_keys):
    _push_batch_case(engine, n, R, faults, custom_keys, make=make)


@pytest.mark.parametrize("make", [_sliced(2), _sharded(2, 2)], ids=["sliced", "sharded"])
@pytest.mark.parametrize("n,R,faults,schedule", [
    (1500, 64, (0.05, 0.05, 0.05), "2P"),
    (800, 200, None, "2P"),
    (3000, 16, (0.05, 0.05, 0.05), "2P"),   # slices of R_pad 8 / code-row shards: the packed DLV kernel
])
def test_handle_received_batch_multi_engine(engine, make, n, R, faults, schedule):
    _batch_case(engine, n, R, faults, schedule, make=make)


def test_handle_received_batch_sliced_seq(engine):
    _batch_case(engine, 1000, 64, None, "SEQ", make=_sliced(3))


def test_multi_engine_wire_errors(engine):
    from safe_gossip_amd.sharded import ShardedNetwork
    from safe_gossip_amd.sliced import SlicedNetwork
    for net in (SlicedNetwork(50, 8, 2, transport="local"), ShardedNetwork(600, 40, 2, transport="local")):
        n = net.n
        try:
            msg = engine.rpc_encode(False, net.rumor_key(3), 1)
            with pytest.raises(engine.DeviceError, match="status -1"):
                net.handle_received(0, n + 5, msg)        # before the first round
            net.next_round()
            with pytest.raises(engine.DeviceError, match="status -1"):
                net.handle_received(0, 10, msg)           # peer inside the network
            with pytest.raises(engine.DeviceError, match="status -1"):
                net.handle_received(0, n + 5, engine.rpc_encode(False, b"no such rumor", 1))
            with pytest.raises(engine.GossipError, match="status 5"):
                net.handle_received_batch([(0, n + 5, msg), (1, n + 6, b"\x07\x00")])  # nothing applied
            assert (int(net.known_all()[0, 0]) >> 3) & 1 == 0
            assert net.handle_received(0, n + 5, msg) == [engine.rpc_encode(True, b"", 0)]
            assert (int(net.known_all()[0, 0]) >> 3) & 1 == 1  # the copy created rumor 3 at once
            with pytest.raises(engine.DeviceError, match="status -1"):
                net.set_rumor_key(2, net.rumor_key(3))    # keys are distinct
            net.set_rumor_key(3, b"renamed")
            assert net.rumor_key(3) == b"renamed"
            net.set_rumor_key(2, engine.default_rumor_key(3))  # free again
        finally:
            net.close()


def test_sliced_first_push_limit(engine):
    # a slice counts empty answers to external first Pushes in its one-byte
    # per-round count: at most slice_ext_limit per node and round
    from safe_gossip_amd.sliced import SlicedNetwork
    net = SlicedNetwork(40, 4, 2, transport="local")  # R_pad 2 per slice: 64 first Pushes
    try:
        net.next_round()
        empty = engine.rpc_encode(False, b"", 0)
        assert net.handle_received_batch([(0, 100 + i, empty) for i in range(64)])[63] == [engine.rpc_encode(True, b"", 0)]
        with pytest.raises(engine.DeviceError, match="status -5"):
            net.handle_received(0, 1000, empty)
        net.handle_received(1, 1000, empty)  # another node, and pulls, still go through
        net.handle_received(0, 1001, engine.rpc_encode(True, b"", 0))
        net.next_round()
        net.handle_received(0, 1000, empty)  # a new round
    finally:
        net.close()


def _uneven_limit_case(sg, make):
    """R = 9 over 2 slices (4 + 5 rumors, R_pad 4 and 8: own bounds 128 and
    200): every slice takes the network's bound, 128, so the 129th first Push
    to a node is refused whole by both slices, which stay equal."""
    from safe_gossip_amd.sliced import slice_ext_limit
    assert slice_ext_limit(9, 2) == 128 and slice_ext_limit(3, 2) == 32
    net = make(60, 9)
    try:
        assert net.ext_limit == 128
        net.next_round()
        st0 = net.statistics_all().astype(np.int64)
        empty = sg.rpc_encode(False, b"", 0)
        pull_empty = sg.rpc_encode(True, b"", 0)
        out = net.handle_received_batch([(5, 100 + i, empty) for i in range(128)])
        assert out[127] == [pull_empty]
        with pytest.raises(sg.DeviceError, match="status -5"):
            net.handle_received_batch([(5, 1000, empty), (6, 1000, empty)])
        # nothing of the refused batch was applied: node 6 still answers
        assert net.handle_received(6, 1000, empty) == [pull_empty]
        st = net.statistics_all().astype(np.int64) - st0
        assert st[5][1] == 128 and st[6][1] == 1  # empty pulls sent (the MIN over the slices)
        net.next_round()
        net.handle_received(5, 1000, empty)  # a new round
    finally:
        net.close()


def test_sliced_uneven_first_push_limit(engine):
    from safe_gossip_amd.sliced import SlicedNetwork
    _uneven_limit_case(engine, lambda n, R: SlicedNetwork(n, R, 2, transport="local"))
    with pytest.raises(engine.DeviceError, match="status -1"):  # above a slice's own bound
        net = SlicedNetwork(40, 4, 2, transport="local")
        try:
            s = net.slices[0]
            from safe_gossip_amd import _check
            _check(s.lib.gs_slice_set_ext_limit(s.h, 65))
        finally:
            net.close()
