"""The signature half of the wire path on the GPU (gs_verify.hip): SHA3-512
against hashlib, ed25519 over SHA3-512 (ed25519-dalek 0.6 sign / verify, as
src/messages.rs:28-44 uses it) against the CPU restatement
oracle/ed25519_sha3.py and the golden vectors it wrote
(tests/golden/ed25519_sha3_vectors.json; the oracle is pinned by RFC 8032's
SHA-512 vectors, the SHA3-512 curve results are parity unpinned against a
real ed25519-dalek run), and the signed forms of the engine's byte-level
entry points (gs_handle_received_signed, gs_push_batch_signed) end to end."""
import hashlib
import json
import os
import random
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import ed25519_sha3 as E  # noqa: E402

VEC = json.load(open(os.path.join(HERE, "golden", "ed25519_sha3_vectors.json")))
SEED = 0x5AFE6055


def test_sha3_512_batch(engine):
    rnd = random.Random(11)
    msgs = [bytes(rnd.randrange(256) for _ in range(n)) for n in list(range(0, 220)) + [575, 576, 577, 4000]]
    msgs += [bytes.fromhex(v["msg"]) for v in VEC["sha3_512"]]
    got = engine.sha3_512(msgs)
    assert got == [hashlib.sha3_512(m).digest() for m in msgs]


def test_ed25519_sign_batch(engine):
    seeds = [bytes.fromhex(k["seed"]) for k in VEC["sign"]]
    msgs = [bytes.fromhex(k["msg"]) for k in VEC["sign"]]
    pubs, sigs = engine.ed25519_sign(seeds, msgs)
    assert [p.hex() for p in pubs] == [k["pub"] for k in VEC["sign"]]
    assert [s.hex() for s in sigs] == [k["sig"] for k in VEC["sign"]]
    rnd = random.Random(12)
    seeds = [bytes(rnd.randrange(256) for _ in range(32)) for _ in range(70)]  # more than one wave
    msgs = [bytes(rnd.randrange(256) for _ in range(rnd.randrange(120))) for _ in range(70)]
    pubs, sigs = engine.ed25519_sign(seeds, msgs)
    for i in range(0, 70, 7):  # the pure-Python oracle is slow: a sample
        assert pubs[i] == E.public_key(seeds[i]) and sigs[i] == E.sign(seeds[i], msgs[i])
    assert all(engine.ed25519_verify(pubs, msgs, sigs))


def test_ed25519_verify_batch(engine):
    cases = VEC["verify"]
    got = engine.ed25519_verify([bytes.fromhex(v["pub"]) for v in cases], [bytes.fromhex(v["msg"]) for v in cases],
                                [bytes.fromhex(v["sig"]) for v in cases])
    assert got == [v["ok"] for v in cases], [v["what"] for v, g in zip(cases, got) if g != v["ok"]]


def _net(engine):
    net = engine.Network(100, 8, seed=SEED)
    for r in range(8):
        net.send_new(engine.origin_of(SEED, 0, r, 100), r)
    for _ in range(3):
        net.next_round()
    return net


def test_signed_wire_round_trip(engine):
    # an outside peer's signed Push to node 5 (src/gossiper.rs:82-99 on the
    # non-test path): verified on the GPU, applied exactly as the unsigned RPC
    # is on a twin network, answered with Pulls signed by node 5; a tampered
    # frame is refused (SigFailure) and changes nothing
    rnd = random.Random(13)
    peer_seed, node_seed = bytes(rnd.randrange(256) for _ in range(32)), bytes(rnd.randrange(256) for _ in range(32))
    peer_key, node_key = E.public_key(peer_seed), E.public_key(node_seed)
    a, b = _net(engine), _net(engine)
    try:
        rpc = engine.rpc_encode(False, a.rumor_key(6), 1)
        frame = engine.message_wrap(rpc, E.sign(peer_seed, rpc))
        bad = bytearray(frame)
        bad[9] ^= 1  # a byte of the signed payload
        with pytest.raises(engine.SigFailure):
            a.handle_received_signed(5, 200, peer_key, bytes(bad), node_seed)
        with pytest.raises(engine.SigFailure):  # signed by someone else
            a.handle_received_signed(5, 200, node_key, frame, node_seed)
        resp = a.handle_received_signed(5, 200, peer_key, frame, node_seed)
        want = b.handle_received(5, 200, rpc)
        assert len(resp) == len(want) >= 1
        for f, w in zip(resp, want):
            payload, sig = engine.message_unwrap(f)
            assert payload == w and E.verify(node_key, payload, sig)
        unsigned = a.handle_received_signed(5, 201, peer_key, frame)  # node_seed None: bare RPC frames
        assert unsigned == b.handle_received(5, 201, rpc)
        a.next_round()
        b.next_round()
        np.testing.assert_array_equal(a.dump_state(), b.dump_state())
        np.testing.assert_array_equal(a.statistics_all(), b.statistics_all())
        # the node's next Push RPCs, signed (Message::serialise)
        for node in (5, 17):
            pushes = a.push_batch_signed(node, node_seed)
            assert [engine.message_unwrap(f)[0] for f in pushes] == b.push_batch(node)
            pubs = [node_key] * len(pushes)
            msgs = [engine.message_unwrap(f)[0] for f in pushes]
            sigs = [engine.message_unwrap(f)[1] for f in pushes]
            assert all(engine.ed25519_verify(pubs, msgs, sigs))
    finally:
        a.close()
        b.close()


def test_signed_responses_larger_than_first_buffer(engine):
    # a node with 128 live rumors answers a first Push with 128 signed Pulls
    # (~14 KB, more than the wrapper's first 4 KB buffer, while the unsigned
    # frames, ~3.7 KB, fit it): the RPC must be applied exactly once (the
    # signed size is checked before anything is applied), so responses,
    # states and Statistics equal an unsigned twin's
    rnd = random.Random(14)
    peer_seed, node_seed = bytes(rnd.randrange(256) for _ in range(32)), bytes(rnd.randrange(256) for _ in range(32))
    peer_key, node_key = E.public_key(peer_seed), E.public_key(node_seed)
    nets = [engine.Network(64, 128, seed=SEED) for _ in range(2)]
    a, b = nets
    try:
        for net in nets:
            for r in range(128):
                net.send_new(5, r)
            net.next_round()
        rpc = engine.rpc_encode(False, a.rumor_key(3), 1)
        frame = engine.message_wrap(rpc, E.sign(peer_seed, rpc))
        resp = a.handle_received_signed(5, 300, peer_key, frame, node_seed)
        want = b.handle_received(5, 300, rpc)
        assert len(want) == 128 and sum(4 + len(w) for w in want) < 4096
        assert len(resp) == len(want)
        for f, w in zip(resp, want):
            payload, sig = engine.message_unwrap(f)
            assert payload == w and E.verify(node_key, payload, sig)
        # a second copy from the same peer: no responses, applied once more on both
        assert a.handle_received_signed(5, 300, peer_key, frame, node_seed) == b.handle_received(5, 300, rpc) == []
        np.testing.assert_array_equal(a.statistics_all(), b.statistics_all())
        a.next_round()
        b.next_round()
        np.testing.assert_array_equal(a.dump_state(), b.dump_state())
        np.testing.assert_array_equal(a.statistics_all(), b.statistics_all())
        np.testing.assert_array_equal(a.dump_records()[0], b.dump_records()[0])
    finally:
        a.close()
        b.close()
