"""Full-size configurations bit-exact against a CPU program that is itself
checked against the oracle: oracle/gs_dense.c (the dense bit-sliced OpenMP
2P round; tests/test_dense_cpu.py holds it equal to the reference-faithful
oracle round by round, faults included) runs beside the engine, and every
round the two are compared node by node through the per-node state digest
(gs_state_digest: every state code, record summary, |peers_in_this_round| and
Statistics counter of the node; dn_digest computes the same function), plus
the any-live flag and the Statistics sums.  Semantics: src/gossip.rs:79-166,
src/message_state.rs:86-171.

The small cases also pin the GPU digest to its definition (tests/oracle_lib.py
digest_of over the engine's own dumps)."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import DenseNet, digest_of

pytestmark = pytest.mark.gpu

SEED = 0x5AFE6055


def _first_bad(a, b):
    bad = np.flatnonzero(a != b)
    return None if bad.size == 0 else (int(bad[0]), bad.size)


# rounds to termination and first round of full spread at seed 0x5AFE6055,
# epoch 1, every rumor injected in round 1 at its Philox origin: the spread
# record bench.py prints for configs 3 and 4 (it times and spreads epoch 1)
SPREAD = {(1 << 20, 64): (22, 16), (1 << 24, 256): (34, 18)}


def _run(engine, nets, n, R, faults, max_rounds, every=1, epoch=0, dumps=False, spread=None, complete=None):
    """Inject every rumor at its Philox origin into every engine of `nets`
    (one network each) and into the dense program, then run them round by
    round; returns the rounds run.  An engine's digest after round t is
    compared with the one dense's round t+1 computes on the way (the same
    deliveries, before its transition)."""
    thr = [engine.fault_threshold(p) for p in faults] if faults else None
    dn = DenseNet(n, R, seed=SEED, epoch=epoch, faults=thr)

    def check(gs, c, rnd):
        for i, g in enumerate(gs):
            bad = _first_bad(g, c)
            assert bad is None, f"net {i}, round {rnd}: {bad[1]} nodes differ, first {bad[0]}"
    try:
        for r in range(R):
            x = engine.origin_of(SEED, epoch, r, n)
            for net in nets:
                net.send_new(x, r)
            dn.send_new(x, r)
        prev = None
        r_full = 0
        for rnd in range(1, max_rounds + 1):
            reps = [net.next_round() for net in nets]
            if spread is not None and not r_full and nets[0].known_counts()[1] == n:
                r_full = rnd
            if prev is not None:
                live, before = dn.next_round(digest=True)
                check(prev, before, rnd - 1)
            else:
                live = dn.next_round()
            for i, rep in enumerate(reps):
                assert rep.any_live == live, f"net {i}, round {rnd}: any_live"
            prev = None
            if rnd % every == 0 or not live or rnd == max_rounds:
                prev = [net.state_digest() for net in nets]
                if dumps:  # the GPU digest is the digest of its own dumps
                    for net, g in zip(nets, prev):
                        codes, st = net.dump_state(), net.statistics_all()
                        rec, ps = net.dump_records()
                        np.testing.assert_array_equal(g, digest_of(codes, rec, ps, st))
            if not live or rnd == max_rounds:
                check(prev, dn.digest(), rnd)
                if spread is not None:
                    full = n if complete is None else complete
                    for i, net in enumerate(nets):
                        kc = net.known_counts()
                        assert kc[1] == full, f"net {i}: {kc[1]} nodes complete at termination, not {full}"
                        if complete is None:
                            assert kc == (n * R, n), "full dissemination at termination"
                    assert (rnd, r_full) == spread, f"spread record {(rnd, r_full)}"
                return rnd
        return max_rounds
    finally:
        dn.close()


@pytest.mark.parametrize("n,R,faults", [
    (20000, 256, None),                    # the gather path, W = 4
    (5000, 16, (0.05, 0.05, 0.05)),        # DLV records, faults
    (3000, 64, (0.1, 0.1, 0.1)),           # R_pad 64
    (4000, 5, None),                       # four nodes per DLV lane
    (777, 20, (0.05, 0.05, 0.05)),         # 32-bit lanes
])
def test_digest_small(engine, n, R, faults):
    net = engine.Network(n, R, seed=SEED, **_fk(faults))
    try:
        _run(engine, [net], n, R, faults, 60, dumps=True)
    finally:
        net.close()


def _fk(faults):
    return dict(churn=faults[0], drop_push=faults[1], drop_pull=faults[2]) if faults else {}


@pytest.mark.parametrize("n,R", [(1 << 20, 64), (1 << 24, 256)])
def test_to_termination(engine, n, R):
    # configs 3 and 4 (the bench line) at the bench's epoch, every round until
    # no live push (the harness's termination, src/gossiper.rs:209-212); the
    # spread record is the one the bench prints
    net = engine.Network(n, R, seed=SEED, epoch=1)
    try:
        assert _run(engine, [net], n, R, None, 60, epoch=1, spread=SPREAD[(n, R)]) < 60
    finally:
        net.close()


def test_config5_faults_rounds(engine):
    # config 5: 10^8 x 16 with 1 % churn / push drop / pull drop, 8 rounds
    # against the dense program, on the single engine (the DLV build and the
    # packed round kernel) and on the layout `bench.py --gpus 8` runs: 8
    # code-row node shards of 12.5 M nodes with 4 pipeline parts each (one
    # GPU, device-copy exchanges)
    from safe_gossip_amd.sharded import ShardedNetwork
    n, R = 100_000_000, 16
    faults = (0.01, 0.01, 0.01)
    single = engine.Network(n, R, seed=SEED, **_fk(faults))
    shards = ShardedNetwork(n, R, 8, seed=SEED, transport="local", parts=4, **_fk(faults))
    try:
        assert shards.parts == 4 and shards.shards[0].codes
        _run(engine, [single, shards], n, R, faults, 8, every=2)
    finally:
        shards.close()
        single.close()


# config 5's spread record at the bench's epoch (bench.py prints it): 42
# rounds, churn keeps two nodes from some rumor, never a full spread
SPREAD5 = (42, 0, 99_999_998)


def test_config5_eight_shards_to_termination(engine):
    # config 5 to termination at full size in its 8-GPU layout: 8 code-row
    # shards (4 parts) against the single engine, node by node through the
    # state digest every 3rd round and the last, and the spread record on
    # both.  The late rounds are where churned nodes return with their frozen
    # votes and C / D transitions dominate.  (The dense program takes ~4.5 s
    # per round at this size; it checks rounds 1-8 above and a quarter-size
    # network to termination below.)
    from safe_gossip_amd.sharded import ShardedNetwork
    n, R = 100_000_000, 16
    fk = _fk((0.01, 0.01, 0.01))
    single = engine.Network(n, R, seed=SEED, epoch=1, **fk)
    shards = ShardedNetwork(n, R, 8, seed=SEED, epoch=1, transport="local", parts=4, **fk)
    try:
        for r in range(R):
            x = engine.origin_of(SEED, 1, r, n)
            single.send_new(x, r)
            shards.send_new(x, r)
        rnd = 0
        for rnd in range(1, 81):
            a, b = single.next_round(), shards.next_round()
            assert a.any_live == b.any_live, f"round {rnd}: any_live"
            if rnd % 3 == 0 or not a.any_live:
                bad = _first_bad(single.state_digest(), shards.state_digest())
                assert bad is None, f"round {rnd}: {bad[1]} nodes differ, first {bad[0]}"
            if not a.any_live:
                break
        assert rnd == SPREAD5[0], f"{rnd} rounds"
        for net in (single, shards):
            known, complete = net.known_counts()
            assert complete == SPREAD5[2] and known < n * R
    finally:
        shards.close()
        single.close()


def test_config5_quarter_to_termination(engine):
    # config 5's network at a quarter of its size (2.5 * 10^7 x 16, the same
    # faults) to termination against the dense program, every 3rd round and
    # the last, on the single engine and on 8 code-row shards with 4 parts
    from safe_gossip_amd.sharded import ShardedNetwork
    n, R = 25_000_000, 16
    faults = (0.01, 0.01, 0.01)
    single = engine.Network(n, R, seed=SEED, epoch=1, **_fk(faults))
    shards = ShardedNetwork(n, R, 8, seed=SEED, epoch=1, transport="local", parts=4, **_fk(faults))
    try:
        assert _run(engine, [single, shards], n, R, faults, 80, every=3, epoch=1) < 80
    finally:
        shards.close()
        single.close()


@pytest.mark.parametrize("n,R,world,faults", [
    (5000, 256, 8, None),                    # 32-rumor slices: R_pad 32 (32-bit lane kernel)
    (3000, 100, 3, (0.05, 0.05, 0.05)),      # ragged slices (33/33/34): words straddle slices
    (4000, 40, 5, None),                     # 8-rumor slices: delivery records
])
def test_sliced_digest_small(engine, n, R, world, faults):
    # the digest of a rumor-sliced network (each slice's word sums added on the
    # device, then mixed with |P| and the network Statistics) is the digest of
    # one engine holding every rumor: against the dense program every round
    from safe_gossip_amd.sliced import SlicedNetwork
    net = SlicedNetwork(n, R, world, seed=SEED, transport="local", **_fk(faults))
    try:
        _run(engine, [net], n, R, faults, 60)
    finally:
        net.close()


def test_config4_multi_gpu_shapes_to_termination(engine):
    # config 4 in the two 8-GPU layouts, on one GPU, to termination against the
    # dense program (every 4th round and the last): 8 rumor slices of 32 rumors
    # (round_kernel_w32 per slice, the empty counts MIN-combined on the
    # device, bench.py --gpus 8's slice mode) and 8 class-row node shards of
    # 2^21 nodes (device-copy exchanges, 2 pipeline parts each: --mode nodes)
    from safe_gossip_amd.sharded import ShardedNetwork
    from safe_gossip_amd.sliced import SlicedNetwork
    n, R = 1 << 24, 256
    slices = SlicedNetwork(n, R, 8, seed=SEED, epoch=1, transport="local")
    shards = ShardedNetwork(n, R, 8, seed=SEED, epoch=1, transport="local", parts=2)
    try:
        assert "w32" in slices.round_kernel_name()
        assert _run(engine, [slices, shards], n, R, None, 60, every=4, epoch=1,
                    spread=SPREAD[(n, R)]) == SPREAD[(n, R)][0]
    finally:
        shards.close()
        slices.close()
