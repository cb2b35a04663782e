"""GPU engine vs CPU oracle, round by round, bit-exact (2P schedule).

Each round compares, for every (node, rumor): the MessageState after delivery
(tag, round, our_counter, rounds_in_state_b), the summary of B.peer_counters
that the next MessageState::next_round consumes (anyC, #counters in [1,cmax),
#counters == 2), |peers_in_this_round|, the five Statistics counters of every
node, the known-rumor sets (Gossiper::messages) and the harness's
`processed` flag.  Integer work: the bar is exact equality.
"""
import numpy as np
import pytest

from oracle_lib import SCHED_2P, SCHED_SEQ, OracleNet, fault_threshold

pytestmark = pytest.mark.gpu

SEED = 0x5AFE6055


def _injections(kind, n, R, seed, epoch, rnd, eng):
    """Injections (node, rumor) applied before round `rnd` (1-based)."""
    out = []
    if kind == "origins":          # every rumor injected in round 1 (cfg3/cfg4)
        if rnd == 1:
            out = [(eng.origin_of(seed, epoch, r, n), r) for r in range(R)]
    elif kind == "example":        # examples/network.rs:467-469: random, random, node 0
        if rnd == 1:
            out = [(eng.origin_of(seed, epoch, 0, n), 0), (eng.origin_of(seed, epoch, 1, n), 1),
                   (0, 2)][:R]
    elif kind == "trickle":        # first at a random node, then 50%/node/round
        st = _injections.state
        if rnd == 1:
            st["next"] = 0
            out.append((eng.origin_of(seed, epoch, 0, n), 0))
            st["next"] = 1
        for x in range(n):
            if st["next"] >= R:
                break
            if eng.coin_of(seed, epoch, rnd, x):
                out.append((x, st["next"]))
                st["next"] += 1
    elif kind == "reinject":       # re-sending known rumors exercises insert-replace
        if rnd in (1, 2, 4, 5):
            rng = np.random.default_rng(rnd * 7919 + n)
            out = [(int(rng.integers(n)), int(rng.integers(R))) for _ in range(max(1, R // 2))]
    elif kind == "steady":         # rumors re-sent every 6 rounds: a dissemination that never ends
        if rnd % 6 == 1:
            rng = np.random.default_rng(rnd * 7919 + n)
            out = [(int(rng.integers(n)), int(rng.integers(R))) for _ in range(max(1, R // 2))]
    return out


_injections.state = {}


def _first_diff(a, b):
    idx = np.argwhere(a != b)
    return tuple(idx[0]) if len(idx) else None


def run_parity(engine, n, R, kind, params=None, max_rounds=60, seed=SEED, epoch=0,
               check_every=1, make_net=None, faults=None, schedule="2P"):
    """faults = (churn, drop_push, drop_pull) probabilities (harness-injected).

    A node offline in the current round keeps the peer_counters and
    peers_in_this_round of its last online round in the oracle; the engine
    keeps only the two votes next_round derives from them, so records and |P|
    are compared for online nodes (their effect on offline nodes is checked
    through the state when they return)."""
    fk = {}
    if faults:
        fk = dict(churn=faults[0], drop_push=faults[1], drop_pull=faults[2])
    if schedule != "2P":
        fk["schedule"] = schedule
    osched = SCHED_SEQ if schedule == "SEQ" else SCHED_2P
    if make_net is None:
        net = engine.Network(n, R, seed=seed, epoch=epoch, params=params, **fk)
    else:
        net = make_net(n, R, seed=seed, epoch=epoch, params=params, **fk)
    orc = OracleNet(n, R, seed=seed, epoch=epoch, params=params,
                    faults=[fault_threshold(p) for p in faults] if faults else None)
    assert net.params == orc.params
    rounds = 0
    try:
        for rnd in range(1, max_rounds + 1):
            for (x, r) in _injections(kind, n, R, seed, epoch, rnd, engine):
                net.send_new(x, r)
                orc.send_new(x, r)
            rep = net.next_round()
            rc, olive = orc.next_round(osched)
            assert rc == 0
            assert rep.round == rnd == orc.round
            assert rep.any_live == olive, f"round {rnd}: any_live"
            rounds = rnd
            if rnd % check_every == 0 or not olive:
                gs = net.dump_state()
                os_ = orc.dump_state()
                d = _first_diff(gs, os_)
                assert d is None, (f"round {rnd}: state differs at (node,rumor)={d}: "
                                   f"gpu {gs[d]:#06x} oracle {os_[d]:#06x}")
                grec, gps = net.dump_records()
                orec, ops = orc.dump_records()
                if faults and faults[0] > 0:
                    off = orc.offline(rnd)
                    grec[off] = orec[off] = 0
                    gps[off] = ops[off] = 0
                d = _first_diff(gps, ops)
                assert d is None, f"round {rnd}: |P| differs at node {d}"
                d = _first_diff(grec, orec)
                assert d is None, (f"round {rnd}: records differ at {d}: gpu {grec[d]:#06x} "
                                   f"oracle {orec[d]:#06x}")
                gst = net.statistics_all()
                ost = orc.statistics()
                d = _first_diff(gst, ost)
                assert d is None, f"round {rnd}: statistics differ at {d}: {gst[d[0]]} vs {ost[d[0]]}"
                np.testing.assert_array_equal(net.known_all(), orc.known_all())
            if not olive:
                break
    finally:
        net.close()
        orc.close()
    return rounds


@pytest.mark.parametrize("n,R,kind,params", [
    (8, 3, "example", None),        # config 1: examples/network.rs default network
    (2, 1, "origins", None),        # smallest mesh: max_rounds 1
    (3, 2, "origins", None),
    (5, 3, "trickle", None),
    (20, 1, "trickle", None),       # README row 1 size
    (200, 1, "trickle", None),      # README row 2 size
    (2000, 1, "trickle", None),     # README row 3 size (cmax 3)
    (16, 5, "origins", None),       # cmax 2 boundary (n=16)
    (1619, 4, "origins", None),     # cmax 3 boundary (n > e^e^2)
    (97, 16, "origins", None),
    (101, 32, "reinject", None),
    (64, 64, "origins", None),
    (300, 64, "trickle", None),
    (77, 100, "origins", None),     # R not a power of two (padded to 128)
    (50, 256, "origins", None),
    (130, 256, "reinject", None),
    (33, 512, "origins", None),
    (40, 7, "origins", (1, 1, 3)),
    (40, 7, "origins", (2, 3, 5)),
    (300, 16, "origins", (3, 3, 14)),
    (500, 8, "reinject", (3, 2, 9)),
    (1000, 3, "trickle", (3, 3, 32)),
])
def test_round_parity(engine, n, R, kind, params):
    rounds = run_parity(engine, n, R, kind, params)
    assert rounds >= 1


@pytest.mark.parametrize("n,R,kind,faults", [
    (8, 3, "example", (0.2, 0.1, 0.1)),        # config 1 network under faults
    (200, 1, "trickle", (0.1, 0.0, 0.0)),      # churn only
    (300, 16, "origins", (0.0, 0.3, 0.0)),     # push drops only
    (300, 16, "origins", (0.0, 0.0, 0.3)),     # pull drops only
    (500, 16, "origins", (0.05, 0.05, 0.05)),  # config 5 shape (R=16, small segments)
    (400, 64, "reinject", (0.3, 0.1, 0.1)),    # injections into frozen nodes
    (130, 256, "origins", (0.1, 0.1, 0.2)),    # multi-word segments
    (2000, 1, "trickle", (0.5, 0.2, 0.2)),
    (64, 8, "origins", (1.0, 0.0, 0.0)),       # every node offline every round
])
def test_round_parity_faults(engine, n, R, kind, faults):
    run_parity(engine, n, R, kind, faults=faults)


@pytest.mark.parametrize("n,R,kind,params,faults", [
    (8, 3, "example", None, None),       # config 1 under the literal harness order
    (2, 1, "origins", None, None),
    (3, 2, "origins", None, None),
    (5, 3, "trickle", None, None),
    (20, 1, "trickle", None, None),      # README rows under SEQ: the published harness
    (200, 1, "trickle", None, None),
    (2000, 1, "trickle", None, None),
    (97, 16, "origins", None, None),
    (101, 32, "reinject", None, None),
    (300, 64, "trickle", None, None),
    (77, 100, "origins", None, None),
    (130, 256, "reinject", None, None),
    (40, 7, "origins", (1, 1, 3), None),
    (40, 7, "origins", (2, 3, 5), None),
    (500, 8, "reinject", (3, 2, 9), None),
    (300, 16, "origins", None, (0.05, 0.05, 0.1)),
    (400, 64, "reinject", None, (0.3, 0.1, 0.1)),
    (130, 256, "origins", None, (0.1, 0.2, 0.2)),
])
def test_round_parity_seq(engine, n, R, kind, params, faults):
    run_parity(engine, n, R, kind, params, faults=faults, schedule="SEQ")


def test_parity_seq_larger(engine):
    # 20k nodes: pull chains of depth ~7 (levels of the SEQ pull passes)
    run_parity(engine, 20000, 64, "origins", check_every=4, schedule="SEQ")


def test_parity_seq_larger_small_words(engine):
    # 20k nodes x 16 rumors (four nodes per 64-bit word): level-0 pulls built
    # inline by the round kernel next to listed ones, with t(x)'s deeper
    # pusher walks (rank > 3) and in-list tails, under faults
    run_parity(engine, 20000, 16, "reinject", check_every=3, schedule="SEQ",
               faults=(0.02, 0.05, 0.05))


@pytest.mark.parametrize("seed,epoch", [(1, 0), (0xDEADBEEF, 3), (2**63 + 5, 77)])
def test_round_parity_seeds(engine, seed, epoch):
    run_parity(engine, 600, 48, "origins", seed=seed, epoch=epoch)


def test_parity_larger(engine):
    # 20k nodes x 64 rumors: one u64 word per node (the ballot-path config at
    # a size the oracle finishes in seconds); full dumps every 4th round.
    run_parity(engine, 20000, 64, "origins", check_every=4)


def test_no_peers(engine):
    net = engine.Network(1, 4)
    with pytest.raises(engine.NoPeers):
        net.send_new(0, 0)
    with pytest.raises(engine.NoPeers):
        net.next_round()
    net.close()


def test_clear_and_observe_idempotent(engine):
    net = engine.Network(500, 32)
    orc = OracleNet(500, 32)
    for r in range(32):
        x = engine.origin_of(SEED, 0, r, 500)
        net.send_new(x, r)
        orc.send_new(x, r)
    for _ in range(3):
        net.next_round()
        orc.next_round(SCHED_2P)
    a = net.dump_state()
    b = net.dump_state()          # observing twice changes nothing
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(a, orc.dump_state())
    net.next_round()
    orc.next_round(SCHED_2P)
    np.testing.assert_array_equal(net.dump_state(), orc.dump_state())
    net.clear(epoch=9)
    orc.clear(9)
    assert net.known_counts() == (0, 0)
    assert int(net.statistics_all().sum()) == 0
    net.close()
    orc.close()


@pytest.mark.parametrize("n,R,kind,faults,schedule", [
    (3000, 64, "origins", None, "2P"),
    (2000, 16, "trickle", (0.05, 0.05, 0.05), "2P"),
    (1500, 32, "origins", None, "SEQ"),
])
def test_parity_generic_inlists(engine, monkeypatch, n, R, kind, faults, schedule):
    # the in-list build for n > 2^27 (exact global CSR), forced at a small size
    monkeypatch.setenv("SAFE_GOSSIP_AMD_GENERIC_INLISTS", "1")
    run_parity(engine, n, R, kind, faults=faults, schedule=schedule)


def test_parity_many_bins(engine):
    # 2^26 + 2^14 nodes: 4097 bins of the binned in-list build (16-bit per-bin
    # LDS state, beyond the former 4096-bin limit).  Too large for the oracle;
    # an edge lost or duplicated by the build breaks these conservation laws.
    n = (1 << 26) + (1 << 14)
    net = engine.Network(n, 1, seed=SEED)
    net.send_new(engine.origin_of(SEED, 0, 0, n), 0)
    for _ in range(6):
        rep = net.next_round()
    st = net.statistics_reduce("sum")
    # every full copy sent is received; every node ran every round
    assert st.full_message_sent == st.full_message_received
    assert st.rounds == 6 * n
    known, _ = net.known_counts()
    assert known > 1
    net.close()


@pytest.mark.parametrize("n,R,kind", [
    (40, 4096, "origins"),      # the largest R (64 words per node)
    (60, 1000, "reinject"),     # R padded to 1024
    (50, 65, "origins"),        # one bit past a word
    (90, 33, "trickle"),        # small-R segments of 64 bits holding one node
])
def test_round_parity_wide_and_ragged(engine, n, R, kind):
    run_parity(engine, n, R, kind)


def test_config2_full_size(engine):
    # BASELINE config 2 at its full size: 10^6 nodes x 1 rumor to termination,
    # every round bit-exact against the oracle (state, records, |P|,
    # Statistics, known sets); the dissemination takes O(ln n) rounds.
    rounds = run_parity(engine, 1_000_000, 1, "origins")
    assert 14 <= rounds <= 30


@pytest.mark.parametrize("n,R,kind,faults", [
    (300, 16, "origins", None),
    (2000, 1, "trickle", (0.1, 0.05, 0.05)),
    (500, 8, "reinject", (0.05, 0.1, 0.1)),
])
def test_parity_small_gather_path(engine, monkeypatch, n, R, kind, faults):
    # R_pad <= 16 runs on delivery records by default; the class-plane gather
    # path stays bit-exact too (SAFE_GOSSIP_AMD_NO_DLV=1)
    monkeypatch.setenv("SAFE_GOSSIP_AMD_NO_DLV", "1")
    run_parity(engine, n, R, kind, faults=faults)


@pytest.mark.parametrize("n,R,kind,faults", [
    (5, 16, "origins", None),                  # one lane, one partial field
    (1030, 1, "trickle", (0.05, 0.05, 0.05)),  # 16 lanes per word, ragged last word
    (1023, 2, "origins", None),                # 8 lanes per word
    (777, 4, "reinject", (0.1, 0.1, 0.1)),     # 4 lanes per word
    (999, 7, "origins", (0.02, 0.0, 0.1)),     # R_pad 8: 2 lanes per word
    (1026, 16, "reinject", (0.2, 0.1, 0.1)),   # one word per lane, ragged last lane
])
def test_parity_delivery_records_packed(engine, n, R, kind, faults):
    # the DLV transition kernel with several nodes per 32-bit lane word
    # (gs_dlv4.hip: two at R_pad 16, four below): every R_pad <= 16 field
    # width, partial lanes and words, churn (pend votes)
    run_parity(engine, n, R, kind, faults=faults)


@pytest.mark.parametrize("n,R,kind,faults", [
    (5, 16, "origins", None),
    (1026, 16, "reinject", (0.2, 0.1, 0.1)),
    (2050, 13, "origins", (0.02, 0.05, 0.05)),
])
def test_parity_delivery_records_packed_u64(engine, monkeypatch, n, R, kind, faults):
    # R_pad 16 with four nodes per 64-bit lane word (SAFE_GOSSIP_AMD_DLV_PACK=u64)
    monkeypatch.setenv("SAFE_GOSSIP_AMD_DLV_PACK", "u64")
    run_parity(engine, n, R, kind, faults=faults)


@pytest.mark.parametrize("n,R,kind,faults", [
    (300, 16, "origins", None),
    (2000, 1, "trickle", (0.1, 0.05, 0.05)),
    (500, 8, "reinject", (0.05, 0.1, 0.1)),
])
def test_parity_delivery_records_node_per_lane(engine, monkeypatch, n, R, kind, faults):
    # the one-node-per-lane DLV transition (SAFE_GOSSIP_AMD_DLV_PACK=0), the
    # kernel observation launches use, stays bit-exact as a transition too
    monkeypatch.setenv("SAFE_GOSSIP_AMD_DLV_PACK", "0")
    run_parity(engine, n, R, kind, faults=faults)


def test_parity_delivery_records_larger(engine):
    # delivery records at 20k nodes: many in-list tails (in-degree > 2) and
    # pull scans through t(x)'s tail, with faults, every 3rd round checked
    run_parity(engine, 20000, 16, "reinject", check_every=3, faults=(0.02, 0.05, 0.05))


def test_filtered_full_dissemination(engine, monkeypatch):
    # 2^20 nodes x 256 rumors, all injected in round 1 (the config-4 workload
    # at 1/16 size) through 24 rounds: the live-filtered gathers (the default)
    # end bit-identical to the unfiltered kernel, and the traffic counted by
    # the kernels stays below the dense model and above the streamed floor
    n, R = 1 << 20, 256
    out = {}
    for filt in ("0", "1"):
        monkeypatch.setenv("SAFE_GOSSIP_AMD_FILTER", filt)
        net = engine.Network(n, R, seed=SEED)
        for r in range(R):
            net.send_new(engine.origin_of(SEED, 0, r, n), r)
        net.set_timing(True)
        for _ in range(24):
            net.next_round(report=False)
        net.sync()
        b, launches = net.round_traffic()
        dense = net.round_kernel_bytes()
        name = net.round_kernel_name()
        if filt == "0":  # no maps: the static model
            assert launches == 0 and b == dense
            assert "filtered" not in name
        else:            # every deliver launch counted by the kernels
            assert launches == 23
            # (the filtered count includes t(x)'s earlier pushers' rows, which
            # the static model leaves out)
            assert n * 68 < b < dense, (b, dense)
            assert "live-filtered" in name
        out[filt] = (net.known_all(), net.statistics_all(), [net.push_batch(x) for x in range(0, n, 4099)])
        net.close()
    np.testing.assert_array_equal(out["1"][0], out["0"][0])
    np.testing.assert_array_equal(out["1"][1], out["0"][1])
    assert out["1"][2] == out["0"][2]


@pytest.mark.parametrize("n,R,kind,faults", [
    (101, 32, "reinject", None),                # small segments (R_pad 32)
    (300, 64, "trickle", None),
    (130, 256, "reinject", (0.1, 0.1, 0.2)),
    (33, 512, "origins", None),
    (500, 16, "origins", (0.05, 0.05, 0.05)),   # small gather path (no DLV)
])
def test_parity_unfiltered(engine, monkeypatch, n, R, kind, faults):
    # every other 2P gather-path test runs the live-filtered gathers (the
    # default); the unfiltered kernel (SAFE_GOSSIP_AMD_FILTER=0) stays exact
    monkeypatch.setenv("SAFE_GOSSIP_AMD_FILTER", "0")
    monkeypatch.setenv("SAFE_GOSSIP_AMD_NO_DLV", "1")
    run_parity(engine, n, R, kind, faults=faults)


def test_parity_filtered_larger(engine):
    # 20k nodes x 256 rumors through a whole dissemination: live and complete
    # maps change every round, in-list tails and deep sibling walks (rank > 3)
    # under the skip flags, faults on; every 3rd round checked
    run_parity(engine, 20000, 256, "origins", check_every=3, faults=(0.02, 0.05, 0.05))


@pytest.mark.parametrize("n,R,filt", [(3000, 256, "1"), (3000, 256, "0"), (2000, 128, "1")])
def test_parity_round_kernel_wide(engine, monkeypatch, n, R, filt):
    # the 64-bit lane round_kernel on the wide 2P path, filtered and
    # unfiltered, with the 32-bit lane kernel explicitly off
    # (SAFE_GOSSIP_AMD_W32=0).  round_kernel is the default at R_pad 64..256
    # (every other wide 2P test runs it too); round_kernel_w32 is the default
    # at R_pad 32 only, and runs at R_pad 64..256 where test_parity_w32
    # forces it (SAFE_GOSSIP_AMD_W32=1)
    monkeypatch.setenv("SAFE_GOSSIP_AMD_W32", "0")
    monkeypatch.setenv("SAFE_GOSSIP_AMD_FILTER", filt)
    run_parity(engine, n, R, "origins", check_every=2)


@pytest.mark.parametrize("n,R,kind,faults", [
    (101, 32, "reinject", None),                   # R_pad 32: a lane per node, two nodes per unit word
    (777, 20, "origins", (0.05, 0.05, 0.05)),      # R_pad 32 with churn votes, an odd node count
    (300, 64, "trickle", None),                    # W32 = 2: 32 nodes per wave, u32 map stores
    (77, 100, "origins", None),                    # R_pad 128: W32 = 4
    (130, 256, "reinject", (0.1, 0.1, 0.2)),       # W32 = 8, churn votes in half words
    (1000, 200, "trickle", (0.05, 0.05, 0.05)),    # a partial last block
    (20000, 256, "origins", None),                 # deep in-lists and sibling walks
])
def test_parity_w32(engine, monkeypatch, n, R, kind, faults):
    # the 32-bit lane round kernel (gs_w32.hip), forced on explicitly
    monkeypatch.setenv("SAFE_GOSSIP_AMD_W32", "1")
    run_parity(engine, n, R, kind, faults=faults, check_every=1 if n < 5000 else 3)


@pytest.mark.parametrize("n,R,faults", [(400, 16, None), (300, 12, (0.05, 0.05, 0.05))])
def test_parity_long_run_stats_folds(engine, n, R, faults):
    # 200 rounds of a dissemination kept alive by re-sending: the delivery-
    # record engines keep Statistics deltas in 16 bits and fold them into the
    # u64 totals every 60 rounds (R_pad 16), so several folds happen here and
    # every counter must still equal the oracle's
    run_parity(engine, n, R, "steady", max_rounds=200, check_every=7, faults=faults)


@pytest.mark.parametrize("faults", [None, (0.1, 0.05, 0.05)])
def test_parity_two_epochs_wide(engine, faults):
    # R_pad 256 (W = 4, config 4's lane shape), a few rumors, so most nodes
    # hold all-zero planes for a while, then some; churn freezes some nodes;
    # two epochs (clear() zeroes both plane buffers): every round's state and
    # known sets, and the Statistics, are the oracle's.
    from oracle_lib import fault_threshold
    n, R = 3000, 200
    fk = dict(churn=faults[0], drop_push=faults[1], drop_pull=faults[2]) if faults else {}
    net = engine.Network(n, R, seed=SEED, **fk)
    orc = OracleNet(n, R, seed=SEED, faults=[fault_threshold(p) for p in faults] if faults else None)
    try:
        for epoch, rounds in ((0, 6), (3, 40)):
            if epoch:
                net.clear(epoch=epoch)
                orc.clear(epoch)
            for r in range(0, R, 7):  # a few rumors: most nodes stay all-zero for a while
                x = engine.origin_of(SEED, epoch, r, n)
                net.send_new(x, r)
                orc.send_new(x, r)
            for _ in range(rounds):
                net.next_round()
                orc.next_round(SCHED_2P)
                np.testing.assert_array_equal(net.dump_state(), orc.dump_state())
                np.testing.assert_array_equal(net.known_all(), orc.known_all())
            np.testing.assert_array_equal(net.statistics_all(), orc.statistics())
    finally:
        net.close()
        orc.close()
