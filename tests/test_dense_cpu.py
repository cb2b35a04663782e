"""The dense bit-sliced OpenMP CPU program (oracle/gs_dense.c, the "best CPU"
baseline of bench.py) equals the reference-faithful oracle round by round
under 2P: every (node, rumor) state, every Statistics counter, the
`processed` flag."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import SCHED_2P, DenseNet, OracleNet


@pytest.mark.parametrize("n,R,kind", [
    (8, 3, "origins"), (2, 1, "origins"), (200, 1, "trickle"), (97, 16, "origins"),
    (300, 64, "trickle"), (77, 100, "origins"), (50, 256, "reinject"), (1700, 3, "origins"),
])
def test_dense_equals_oracle(oracle, n, R, kind):
    seed = 0x5AFE6055
    L = oracle_lib.lib()
    orc, dn = OracleNet(n, R, seed=seed), DenseNet(n, R, seed=seed)
    rng = np.random.default_rng(n)
    nxt = 0
    for rnd in range(1, 60):
        inj = []
        if kind == "origins" and rnd == 1:
            inj = [(L.or_origin(seed, 0, r, n), r) for r in range(R)]
        if kind == "reinject" and rnd in (1, 2, 4, 5):
            inj = [(int(rng.integers(n)), int(rng.integers(R))) for _ in range(max(1, R // 2))]
        if kind == "trickle":
            if rnd == 1:
                inj.append((L.or_origin(seed, 0, 0, n), 0))
                nxt = 1
            for x in range(n):
                if nxt >= R:
                    break
                if L.or_coin(seed, 0, rnd, x):
                    inj.append((x, nxt))
                    nxt += 1
        for x, r in inj:
            orc.send_new(x, r)
            dn.send_new(x, r)
        _, olive = orc.next_round(SCHED_2P)
        assert dn.next_round() == olive, f"round {rnd}: any_live"
        codes, st = dn.dump()
        np.testing.assert_array_equal(codes, orc.dump_state(), err_msg=f"state round {rnd}")
        np.testing.assert_array_equal(st, orc.statistics(), err_msg=f"stats round {rnd}")
        if not olive:
            break
    orc.close()
    dn.close()
