"""Engines created on memory that earlier engines filled.

A new engine's first rounds read buffers zeroed at creation (the in-list
counters, the SibRecs whose stale serials the filtered build leaves
unwritten, the state planes).  The engine streams are non-blocking, so that
zeroing must be ordered on them (gs_engine.cpp create_engine, DESIGN.md 7d
"Stream discipline"): here engines of alternating shapes are created and
destroyed back to back -- each on memory the one before left full of live
state -- and every round of each is compared with the oracle, on the gather
path (filtered), SEQ, the packed DLV path and in-process node shards.
"""
import pytest

from test_gpu_parity import run_parity

pytestmark = pytest.mark.gpu


def test_engines_on_reused_memory(engine):
    shapes = [(2000, 64, "trickle", "2P"), (200, 16, "trickle", "SEQ"), (1500, 16, "origins", "2P"),
              (3000, 256, "origins", "2P"), (400, 33, "trickle", "SEQ")]
    for rep in range(3):
        for n, R, kind, schedule in shapes:
            run_parity(engine, n, R, kind, max_rounds=12, schedule=schedule)


def test_shard_nets_on_reused_memory(engine):
    from safe_gossip_amd.net import Net
    from test_gpu_net import SEED, _net_vs_oracle
    for rep in range(3):
        for mode, world, n, R in [("shards", 2, 800, 100), ("shards", 3, 900, 16), ("slices", 2, 600, 40)]:
            net = Net(n, R, world, mode=mode, seed=SEED, transport="local", parts=2)
            try:
                _net_vs_oracle(engine, net, n, R)
            finally:
                net.close()
