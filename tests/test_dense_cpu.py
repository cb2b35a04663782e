"""The dense bit-sliced OpenMP CPU program (oracle/gs_dense.c: the "best CPU"
baseline of bench.py, and the full-size checker of the GPU engine) equals the
reference-faithful oracle round by round under 2P: every (node, rumor) state,
record summary, |peers_in_this_round|, every Statistics counter, the
`processed` flag -- with and without the harness-injected faults of config 5
-- and its per-node digest (dn_digest) is the digest gs_state_digest defines
(tests/oracle_lib.py digest_of, over the oracle's own dumps)."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import SCHED_2P, DenseNet, OracleNet, digest_of


def _injections(L, kind, n, R, seed, rnd, rng, state):
    inj = []
    if kind == "origins" and rnd == 1:
        inj = [(L.or_origin(seed, 0, r, n), r) for r in range(R)]
    if kind == "reinject" and rnd in (1, 2, 4, 5):
        inj = [(int(rng.integers(n)), int(rng.integers(R))) for _ in range(max(1, R // 2))]
    if kind == "trickle":
        if rnd == 1:
            inj.append((L.or_origin(seed, 0, 0, n), 0))
            state["nxt"] = 1
        for x in range(n):
            if state["nxt"] >= R:
                break
            if L.or_coin(seed, 0, rnd, x):
                inj.append((x, state["nxt"]))
                state["nxt"] += 1
    return inj


@pytest.mark.parametrize("n,R,kind,faults", [
    (8, 3, "origins", None), (2, 1, "origins", None), (200, 1, "trickle", None), (97, 16, "origins", None),
    (300, 64, "trickle", None), (77, 100, "origins", None), (50, 256, "reinject", None),
    (1700, 3, "origins", None),
    # config-5 faults: churn, push-batch drop, pull-batch drop
    (600, 16, "origins", (0.05, 0.05, 0.05)), (300, 64, "reinject", (0.2, 0.1, 0.2)),
    (200, 1, "trickle", (0.1, 0.1, 0.1)), (77, 100, "origins", (0.3, 0.0, 0.3)),
    (1000, 5, "reinject", (0.01, 0.01, 0.01)),
])
def test_dense_equals_oracle(oracle, n, R, kind, faults):
    seed = 0x5AFE6055
    L = oracle_lib.lib()
    thr = [oracle_lib.fault_threshold(p) for p in faults] if faults else None
    orc, dn = OracleNet(n, R, seed=seed, faults=thr), DenseNet(n, R, seed=seed, faults=thr)
    rng = np.random.default_rng(n)
    state = {"nxt": 0}
    for rnd in range(1, 60):
        for x, r in _injections(L, kind, n, R, seed, rnd, rng, state):
            orc.send_new(x, r)
            dn.send_new(x, r)
        _, olive = orc.next_round(SCHED_2P)
        live, dg_before = dn.next_round(digest=True)
        assert live == olive, f"round {rnd}: any_live"
        if rnd > 1:  # the fused digest is the observation before this round's transition
            np.testing.assert_array_equal(dg_before, dg, err_msg=f"fused digest round {rnd}")
        codes, st = dn.dump()
        recs, ps = dn.dump_records()
        np.testing.assert_array_equal(codes, orc.dump_state(), err_msg=f"state round {rnd}")
        np.testing.assert_array_equal(st, orc.statistics(), err_msg=f"stats round {rnd}")
        orec, ops = orc.dump_records()
        # a node offline this round keeps stale peer_counters in the oracle and
        # only their two votes here (as on the GPU): compared once it returns
        on = ~orc.offline(rnd) if faults else np.ones(n, dtype=bool)
        np.testing.assert_array_equal(recs[on], orec[on], err_msg=f"records round {rnd}")
        np.testing.assert_array_equal(ps[on], ops[on], err_msg=f"|P| round {rnd}")
        dg = dn.digest()
        np.testing.assert_array_equal(dg, digest_of(codes, recs, ps, st), err_msg=f"digest round {rnd}")
        if not faults:
            np.testing.assert_array_equal(dg, digest_of(orc.dump_state(), orec, ops, orc.statistics()))
        if not olive:
            break
    orc.close()
    dn.close()
