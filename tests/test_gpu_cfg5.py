"""BASELINE config 5 at its full size: 10^8 nodes x 16 rumors (~6104 bins of
the binned in-list build, the R < 64 round kernel), with and without the
harness-injected faults (1 % churn, 1 % push-batch drop, 1 % pull-batch drop).

Too large for the oracle, so the check is by laws of the reference's
accounting that any lost, duplicated or misrouted edge breaks:
  * Statistics.rounds counts next_round calls (src/gossip.rs:80): summed over
    nodes it is the number of online node-rounds, recomputed here from the
    fault draws of the Philox stream (tests/philox_torch.py, independent of
    the engine);
  * every full copy sent is received when nothing is dropped
    (src/gossip.rs:103,139 vs :155); with drops, received <= sent;
  * the harness's `processed` flag (src/gossiper.rs:209-212) holds iff some
    online node pushed a live rumor, i.e. iff fewer online nodes than online
    ones sent an empty push this round (src/gossip.rs:105-106);
  * known sets (Gossip::messages, src/gossip.rs:66-68) only grow;
  * no device limit (in-degree, bin or tail capacity) is hit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5AFE6055
N5, R5 = 100_000_000, 16


@pytest.mark.parametrize("faults", [None, (0.01, 0.01, 0.01)])
def test_config5_full_size(engine, faults):
    import torch
    import philox_torch as pt
    fk = dict(churn=faults[0], drop_push=faults[1], drop_pull=faults[2]) if faults else {}
    net = engine.Network(N5, R5, seed=SEED, **fk)
    thr = [engine.fault_threshold(p) for p in faults] if faults else None
    nodes = torch.arange(N5, dtype=torch.int64, device="cuda")
    try:
        for r in range(R5):
            net.send_new(engine.origin_of(SEED, 0, r, N5), r)
        prev_known = net.known_all()
        prev = net.statistics_reduce("sum")
        online_total = 0
        prev_cnt = net.known_popcounts()
        for rnd in range(1, 23):
            rep = net.next_round()
            assert rep.round == rnd
            if thr:
                fb = pt.fault_bits(SEED, 0, rnd, nodes, *thr)
                online = N5 - int(((fb & 1) != 0).sum())
            else:
                online = N5
            online_total += online
            st = net.statistics_reduce("sum")
            assert st.rounds == online_total, f"round {rnd}: Statistics.rounds"
            d_empty_push = st.empty_push_sent - prev.empty_push_sent
            assert rep.any_live == (d_empty_push < online), f"round {rnd}: processed flag"
            if thr:
                assert st.full_message_received <= st.full_message_sent
                assert st.full_message_received > prev.full_message_received
            else:
                assert st.full_message_received == st.full_message_sent, f"round {rnd}"
            cnt = net.known_popcounts()
            assert np.all(cnt >= prev_cnt), f"round {rnd}: a node's known set shrank"
            if rnd % 7 == 0:  # whole known sets (800 MB) every 7th round
                known = net.known_all()
                assert not np.any(prev_known & ~known), f"round {rnd}: a known rumor was lost"
                prev_known = known
            tot, _ = net.known_counts(min_known=1)
            assert tot == int(cnt.sum(dtype=np.uint64)) and tot > 0
            prev_cnt, prev = cnt, st
        # 22 rounds: well past Karp's log3(n) + ln ln n ~ 19.7 rounds, so
        # nearly every node knows every rumor (exactly every one without faults)
        t, complete = net.known_counts()
        if thr:
            assert t > 0.99 * N5 * R5
        else:
            assert (t, complete) == (N5 * R5, N5)
        net.sync()   # no device limit hit in any round
    finally:
        net.close()
        del nodes
        torch.cuda.empty_cache()
