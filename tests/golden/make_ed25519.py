"""Writes tests/golden/ed25519_sha3_vectors.json: SHA3-512 digests and
ed25519-over-SHA3-512 signatures / verification results for the signed wire
path (src/messages.rs:28-44), computed by the CPU restatement
oracle/ed25519_sha3.py (itself pinned by RFC 8032's SHA-512 vectors,
tests/test_ed25519_host.py) and hashlib.sha3_512.  The digests are pinned by
hashlib; the curve results are parity unpinned against a real ed25519-dalek
0.6.1 run (not available here).  Run: python tests/golden/make_ed25519.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import ed25519_sha3 as E  # noqa: E402


def main():
    rnd = random.Random(0x5AFE)
    rb = lambda n: bytes(rnd.randrange(256) for _ in range(n))  # noqa: E731
    sha = []
    for n in [0, 1, 31, 32, 64, 71, 72, 73, 100, 143, 144, 145, 300]:
        m = rb(n)
        sha.append(dict(msg=m.hex(), digest=hashlib.sha3_512(m).hexdigest()))
    keys = []
    for i in range(6):
        seed = rb(32)
        msg = rb([0, 1, 13, 45, 72, 200][i])  # bincode GossipRpc frames are 13 + len bytes
        pub, sig = E.public_key(seed), E.sign(seed, msg)
        assert E.verify(pub, msg, sig)
        keys.append(dict(seed=seed.hex(), msg=msg.hex(), pub=pub.hex(), sig=sig.hex()))
    # verification cases: valid, and each kind of corruption
    ver = []
    for k in keys:
        pub, msg, sig = bytes.fromhex(k["pub"]), bytes.fromhex(k["msg"]), bytes.fromhex(k["sig"])
        cases = [("valid", pub, msg, sig),
                 ("message changed", pub, msg + b"\x00", sig),
                 ("R bit flipped", pub, msg, bytes([sig[0] ^ 1]) + sig[1:]),
                 ("S bit flipped", pub, msg, sig[:40] + bytes([sig[40] ^ 4]) + sig[41:]),
                 ("S top bits set", pub, msg, sig[:63] + bytes([sig[63] | 0x20])),
                 ("other key", bytes.fromhex(keys[0]["pub"] if k is not keys[0] else keys[1]["pub"]), msg, sig)]
        for what, p, m, s in cases:
            ver.append(dict(what=what, pub=p.hex(), msg=m.hex(), sig=s.hex(), ok=E.verify(p, m, s)))
    # a public key that does not decompress (no square root for x^2)
    y = 2
    while E.decompress(int.to_bytes(y, 32, "little"), strict=False) is not None:
        y += 1
    k = keys[0]
    ver.append(dict(what="public key off the curve", pub=int.to_bytes(y, 32, "little").hex(), msg=k["msg"],
                    sig=k["sig"], ok=False))
    out = dict(source="oracle/ed25519_sha3.py + hashlib.sha3_512 (tests/golden/make_ed25519.py)",
               sha3_512=sha, sign=keys, verify=ver)
    with open(os.path.join(HERE, "ed25519_sha3_vectors.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(len(sha), "digests,", len(keys), "signatures,", len(ver), "verification cases")


if __name__ == "__main__":
    main()
