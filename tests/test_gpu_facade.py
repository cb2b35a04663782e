"""The C++ host API (include/safe_gossip.hpp) -- the stand-in for the
reference crate's public surface (Gossiper / Statistics / Error,
src/lib.rs:62-65) -- exercised by the compiled examples/facade_check, every
value checked against the CPU oracle."""
import subprocess

import pytest

from oracle_lib import SCHED_2P, OracleNet, lib

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,R,seed", [(300, 16, 0x5AFE6055), (1000, 64, 7), (64, 130, 99)])
def test_facade_check(engine, n, R, seed):
    from safe_gossip_amd.build import REPO_DIR, build_examples
    exe = [e for e in build_examples() if e.endswith("facade_check")][0]
    out = subprocess.run([exe, str(n), str(R), hex(seed)], capture_output=True, text=True,
                         timeout=300, cwd=REPO_DIR)
    assert out.returncode == 0, out.stderr
    kv = {}
    for ln in out.stdout.splitlines():
        k, _, v = ln.partition(" ")
        kv[k] = v
    assert kv["lone_send_new"] == "NoPeers"                 # src/gossiper.rs:56-58
    assert kv["add_peer_after_send"] == "AlreadyStarted"    # src/gossiper.rs:45-48
    assert kv["add_peer_after_clear"] == "ok"
    assert kv["origin_knows_rumor0"] == "1"                 # src/gossip.rs:71-75
    orc = OracleNet(n, R, seed=seed)
    try:
        assert kv["params"] == " ".join(str(p) for p in orc.params)
        L = lib()
        for r in range(R):
            orc.send_new(L.or_origin(seed, 0, r, n), r)
        rounds = 0
        while True:
            _, live = orc.next_round(SCHED_2P)
            rounds += 1
            if not live:
                break
        assert int(kv["rounds"]) == rounds
        st = orc.statistics()
        fmt = lambda a: " ".join(str(int(v)) for v in a)
        assert kv["stats_sum"] == fmt(st.sum(axis=0)) == kv["view_sum"]
        assert kv["stats_min"] == fmt(st.min(axis=0)) == kv["view_min"]
        assert kv["stats_max"] == fmt(st.max(axis=0)) == kv["view_max"]
        assert int(kv["known_total"]) == orc.known_total()
    finally:
        orc.close()
