"""Sharded engine (node range per rank) vs CPU oracle, bit-exact.

The sharded path moves push rows to the owner of each target and pull rows
back; here `world` shard engines share one GPU and the
two exchanges are device copies (transport "local").  The observable result
must equal the unsharded network's, which the oracle restates
(src/gossip.rs:95-151, src/message_state.rs).
"""
import numpy as np
import pytest

from oracle_lib import SCHED_2P, OracleNet
from test_gpu_parity import SEED, run_parity

pytestmark = pytest.mark.gpu


def _maker(world, parts=1):
    from safe_gossip_amd.sharded import ShardedNetwork

    def make(n, R, seed, epoch, params, **faults):
        return ShardedNetwork(n, R, world, seed=seed, epoch=epoch, params=params,
                              transport="local", parts=parts, **faults)
    return make


# (world, pipeline parts): parts cut each rank's node range; the exchanges
# are part-major and the round kernel runs part by part
@pytest.mark.parametrize("world,parts", [(2, 1), (3, 1), (4, 1), (2, 2), (3, 3), (4, 4)])
@pytest.mark.parametrize("n,R,kind,params", [
    (8, 3, "example", None),
    (5, 3, "trickle", None),
    (200, 1, "trickle", None),
    (97, 16, "origins", None),
    (101, 32, "reinject", None),
    (300, 64, "trickle", None),
    (77, 100, "origins", None),
    (130, 256, "reinject", None),
    (300, 16, "origins", (3, 3, 14)),
    (1619, 4, "origins", None),
    # every rank owns nodes (chunks are whole 256-node blocks)
    (700, 3, "trickle", None),
    (520, 100, "reinject", None),
    (1000, 256, "origins", None),
    (900, 7, "origins", (2, 3, 5)),
    (1100, 1, "trickle", (1, 1, 3)),
])
def test_sharded_parity(engine, world, parts, n, R, kind, params):
    run_parity(engine, n, R, kind, params, make_net=_maker(world, parts))


@pytest.mark.parametrize("world,parts", [(2, 1), (3, 1), (2, 2), (3, 4)])
@pytest.mark.parametrize("n,R,kind,faults", [
    (8, 3, "example", (0.2, 0.1, 0.1)),
    (700, 3, "trickle", (0.1, 0.1, 0.1)),
    (600, 16, "origins", (0.05, 0.05, 0.05)),   # config 5 shape
    (520, 100, "reinject", (0.3, 0.2, 0.2)),
    (1000, 256, "origins", (0.1, 0.0, 0.3)),
])
def test_sharded_parity_faults(engine, world, parts, n, R, kind, faults):
    run_parity(engine, n, R, kind, make_net=_maker(world, parts), faults=faults)


@pytest.mark.parametrize("parts", [1, 2])
def test_sharded_larger(engine, parts):
    # 3 shards whose chunk boundaries fall inside 256-node blocks' neighbours.
    run_parity(engine, 20000, 64, "origins", check_every=4, make_net=_maker(3, parts))


@pytest.mark.parametrize("parts", [1, 3])
def test_sharded_more_ranks_than_chunks(engine, parts):
    # world 8 over 600 nodes: chunk rounding leaves trailing ranks (and parts) empty.
    run_parity(engine, 600, 48, "origins", make_net=_maker(8, parts))


@pytest.mark.parametrize("R", [16, 256])
def test_sharded_parts_full_rank_parts(engine, R):
    # 2 ranks x 2 parts of 4096 nodes each: every part holds whole plan blocks
    # and receives rows from every (rank, part) sub-block.
    run_parity(engine, 16384, R, "origins", check_every=3, make_net=_maker(2, 2))


def test_sharded_clear(engine):
    from safe_gossip_amd.sharded import ShardedNetwork
    n, R = 500, 32
    net = ShardedNetwork(n, R, 2, transport="local", parts=2)
    orc = OracleNet(n, R)
    for epoch in (0, 5):
        for r in range(R):
            x = engine.origin_of(SEED, epoch, r, n)
            net.send_new(x, r)
            orc.send_new(x, r)
        for _ in range(4):
            net.next_round()
            orc.next_round(SCHED_2P)
        np.testing.assert_array_equal(net.dump_state(), orc.dump_state())
        np.testing.assert_array_equal(net.statistics_all(), orc.statistics())
        net.clear(epoch=5)
        orc.clear(5)
        assert net.known_counts() == (0, 0)
    net.close()
    orc.close()


# Code rows (R_pad <= 16, 2P): one u32 push / pull code per
# exchange row, the pull kernel writes delivery records, and the packed DLV
# round kernel (gs_dlv4.hip) runs each part; every R <= 16 case above runs them.
@pytest.mark.parametrize("world,parts,n,R,kind,faults", [
    (2, 2, 5000, 16, "origins", None),                # parts of 2048 / 512 nodes
    (3, 3, 20000, 16, "trickle", (0.05, 0.05, 0.05)),  # 3072 / 3072 / 768 nodes, faults
    (2, 4, 9000, 5, "reinject", (0.1, 0.1, 0.1)),     # R_pad 8: four nodes per lane
    (4, 2, 30000, 16, "origins", (0.01, 0.01, 0.01)),  # the config-5 shape
])
def test_sharded_code_rows_parts(engine, world, parts, n, R, kind, faults):
    run_parity(engine, n, R, kind, make_net=_maker(world, parts), faults=faults, check_every=2)


@pytest.mark.parametrize("pack", ["u64", "u32x1"])
def test_sharded_code_rows_packings(engine, monkeypatch, pack):
    # the other lane packings of the packed kernel on a code-row shard
    monkeypatch.setenv("SAFE_GOSSIP_AMD_DLV_PACK", pack)
    run_parity(engine, 5000, 16, "origins", make_net=_maker(3, 2), faults=(0.05, 0.05, 0.05))


@pytest.mark.parametrize("n,R,kind,faults", [
    (97, 16, "origins", None),
    (1619, 4, "origins", None),
    (600, 16, "origins", (0.05, 0.05, 0.05)),
])
def test_sharded_class_rows_small_r(engine, monkeypatch, n, R, kind, faults):
    # SAFE_GOSSIP_AMD_NO_DLV=1: class rows and the per-node shard kernel at
    # R_pad <= 16 (the layout before code rows)
    monkeypatch.setenv("SAFE_GOSSIP_AMD_NO_DLV", "1")
    run_parity(engine, n, R, kind, make_net=_maker(3, 2), faults=faults)
