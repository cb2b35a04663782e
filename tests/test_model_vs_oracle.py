"""The kernel's bit-sliced 2P algebra (tests/model_bitsliced.py, a line-by-line
Python model of gs_kernels.hip) equals the reference-faithful oracle, round by
round, on CPU.  Separates derivation errors from HIP-level errors."""
import numpy as np
import pytest

import oracle_lib
from model_bitsliced import Model
from oracle_lib import SCHED_2P, OracleNet


def run(n, R, params=None, seed=0x5AFE6055, epoch=0, kind="origins", max_rounds=40, faults=None,
        schedule=SCHED_2P):
    thr = [oracle_lib.fault_threshold(p) for p in faults] if faults else None
    orc = OracleNet(n, R, seed=seed, epoch=epoch, params=params, faults=thr)
    L = oracle_lib.lib()
    fault_fn = (lambda rnd, x: L.or_fault(seed, epoch, rnd, x, *thr)) if faults else None
    mdl = Model(n, R, seed, epoch, orc.params, L.or_peer, fault_fn, schedule)
    rng = np.random.default_rng(n * 31 + R)
    injected = []
    for rnd in range(1, max_rounds + 1):
        inj = []
        if kind == "origins" and rnd == 1:
            inj = [(L.or_origin(seed, epoch, r, n), r) for r in range(R)]
        if kind == "trickle":  # harness: first rumor at a Philox origin, then 50%/node/round
            if rnd == 1:
                inj.append((L.or_origin(seed, epoch, 0, n), 0))
            nxt = len(injected) + len(inj)
            for x in range(n):
                if nxt >= R:
                    break
                if L.or_coin(seed, epoch, rnd, x):
                    inj.append((x, nxt))
                    nxt += 1
            injected.extend(inj)
        if kind == "reinject" and rnd in (1, 2, 4, 5):
            inj = [(int(rng.integers(n)), int(rng.integers(R))) for _ in range(max(1, R // 2))]
        for x, r in inj:
            orc.send_new(x, r)
            mdl.send_new(x, r)
        _, olive = orc.next_round(schedule)
        mlive = mdl.next_round()
        assert mlive == olive, rnd
        codes, recs, psz, stats, known = mdl.observe()
        np.testing.assert_array_equal(np.array(codes, np.uint16), orc.dump_state(),
                                      err_msg=f"state round {rnd}")
        orec, ops = orc.dump_records()
        psz, recs = np.array(psz, np.uint32), np.array(recs, np.uint16)
        if faults:  # offline nodes: the oracle keeps stale records, the model only votes
            off = orc.offline(rnd)
            psz[off] = ops[off] = 0
            recs[off] = orec[off] = 0
        np.testing.assert_array_equal(psz, ops, err_msg=f"|P| round {rnd}")
        np.testing.assert_array_equal(recs, orec,
                                      err_msg=f"records round {rnd}")
        np.testing.assert_array_equal(np.array(stats, np.uint64), orc.statistics(),
                                      err_msg=f"stats round {rnd}")
        ok = orc.known_all()
        for x in range(n):
            got = known[x]
            exp = sum(int(w) << (64 * i) for i, w in enumerate(ok[x]))
            assert got == exp, (rnd, x)
        if not olive:
            break
    orc.close()


@pytest.mark.parametrize("n,R,params,kind", [
    (8, 3, None, "origins"),
    (2, 1, None, "origins"),
    (3, 2, None, "origins"),
    (20, 4, None, "reinject"),
    (60, 8, None, "origins"),
    (200, 5, None, "reinject"),
    (40, 7, (2, 3, 5), "origins"),
    (40, 7, (1, 1, 3), "reinject"),
    (300, 6, (3, 3, 14), "origins"),
    (400, 6, (3, 2, 9), "reinject"),
    (1700, 3, None, "origins"),
    (300, 64, None, "trickle"),
])
def test_model_equals_oracle(oracle, n, R, params, kind):
    run(n, R, params, kind=kind)


@pytest.mark.parametrize("n,R,kind,faults", [
    (8, 3, "origins", (0.2, 0.1, 0.1)),
    (60, 8, "origins", (0.1, 0.0, 0.0)),
    (60, 8, "origins", (0.0, 0.3, 0.0)),
    (60, 8, "origins", (0.0, 0.0, 0.3)),
    (200, 5, "reinject", (0.3, 0.1, 0.1)),
    (300, 6, "origins", (0.05, 0.05, 0.05)),
    (150, 4, "reinject", (0.6, 0.2, 0.2)),
])
def test_model_equals_oracle_faults(oracle, n, R, kind, faults):
    run(n, R, kind=kind, faults=faults)


@pytest.mark.parametrize("n,R,kind,params,faults", [
    (8, 3, "origins", None, None),
    (2, 1, "origins", None, None),
    (3, 2, "origins", None, None),
    (20, 4, "reinject", None, None),
    (60, 8, "origins", None, None),
    (200, 5, "reinject", None, None),
    (40, 7, "origins", (2, 3, 5), None),
    (40, 7, "reinject", (1, 1, 3), None),
    (300, 6, "origins", (3, 3, 14), None),
    (1700, 3, "origins", None, None),
    (300, 64, "trickle", None, None),   # mutual pairs: a pull overwritten per rumor
    (1000, 32, "trickle", None, None),
    (60, 8, "origins", None, (0.1, 0.1, 0.1)),
    (200, 5, "reinject", None, (0.3, 0.1, 0.2)),
    (300, 6, "origins", None, (0.0, 0.0, 0.4)),
])
def test_model_equals_oracle_seq(oracle, n, R, kind, params, faults):
    """The literal harness order (SEQ): pulls answered from the current state."""
    run(n, R, params, kind=kind, faults=faults, schedule=oracle_lib.SCHED_SEQ)
