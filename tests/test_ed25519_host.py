"""The signature half of the wire path (src/messages.rs:28-44) on the CPU:

* the oracle (oracle/ed25519_sha3.py) is pinned by RFC 8032 section 7.1's
  Ed25519 test vectors when run with SHA-512 (same code, the hash is a
  parameter); with SHA3-512 it is the scheme the reference signs with
  (ed25519-dalek 0.6 Keypair::sign::<Sha3_512>), parity unpinned against a
  real ed25519-dalek run;
* the GPU arithmetic itself (safe_gossip_amd/csrc/gs_ed25519.h, compiled for
  the host by tests/ed_host.cpp) against hashlib.sha3_512, the oracle and the
  golden vectors of tests/golden/ed25519_sha3_vectors.json.
No GPU needed; tests/test_gpu_verify.py runs the same checks on the kernels."""
import ctypes
import hashlib
import json
import os
import random
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import ed25519_sha3 as E  # noqa: E402

VEC = json.load(open(os.path.join(HERE, "golden", "ed25519_sha3_vectors.json")))

# RFC 8032 section 7.1, TEST 1-3 (secret key, public key, message, signature)
RFC8032 = [
    ("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
     "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
     "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46b"
     "d25bf5f0595bbe24655141438e7a100b"),
    ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
     "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
     "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c"
     "387b2eaeb4302aeeb00d291612bb0c00"),
    ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
     "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
     "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc659"
     "4a7c15e9716ed28dc027beceea1ec40a"),
]


@pytest.mark.parametrize("sk,pk,msg,sig", RFC8032)
def test_oracle_rfc8032_vectors(sk, pk, msg, sig):
    sk, pk, msg, sig = (bytes.fromhex(v) for v in (sk, pk, msg, sig))
    assert E.public_key(sk, hashlib.sha512) == pk
    assert E.sign(sk, msg, hashlib.sha512) == sig
    for dalek in (True, False):
        assert E.verify(pk, msg, sig, hashlib.sha512, dalek=dalek)
        assert not E.verify(pk, msg + b"\x00", sig, hashlib.sha512, dalek=dalek)


def test_oracle_golden_vectors():
    for v in VEC["sha3_512"]:
        assert hashlib.sha3_512(bytes.fromhex(v["msg"])).hexdigest() == v["digest"]
    for k in VEC["sign"]:
        seed, msg = bytes.fromhex(k["seed"]), bytes.fromhex(k["msg"])
        assert E.public_key(seed).hex() == k["pub"] and E.sign(seed, msg).hex() == k["sig"]
    for v in VEC["verify"]:
        assert E.verify(*(bytes.fromhex(v[f]) for f in ("pub", "msg", "sig"))) == v["ok"], v["what"]


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("ed") / "ed_host.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-Wno-unknown-pragmas", "-shared",
                    "-fPIC", "-o", so, os.path.join(HERE, "ed_host.cpp")], check=True)
    return ctypes.CDLL(so)


def _sha(lib, m):
    o = (ctypes.c_uint8 * 64)()
    lib.ed_sha3_512(m, len(m), o)
    return bytes(o)


def test_host_sha3_512(host):
    rnd = random.Random(3)
    for n in list(range(0, 150)) + [215, 216, 217, 1000]:  # every position around the 72-byte rate
        m = bytes(rnd.randrange(256) for _ in range(n))
        assert _sha(host, m) == hashlib.sha3_512(m).digest(), n
    for v in VEC["sha3_512"]:
        assert _sha(host, bytes.fromhex(v["msg"])).hex() == v["digest"]


def test_host_sign_and_verify(host):
    for k in VEC["sign"]:
        seed, msg = bytes.fromhex(k["seed"]), bytes.fromhex(k["msg"])
        pub, sig = (ctypes.c_uint8 * 32)(), (ctypes.c_uint8 * 64)()
        host.ed_sign(seed, msg, len(msg), pub, sig)
        assert bytes(pub).hex() == k["pub"] and bytes(sig).hex() == k["sig"]
    for v in VEC["verify"]:
        p, m, s = (bytes.fromhex(v[f]) for f in ("pub", "msg", "sig"))
        assert host.ed_verify(p, s, m, len(m)) == int(v["ok"]), v["what"]
    rnd = random.Random(9)
    for _ in range(4):  # beyond the fixtures
        seed = bytes(rnd.randrange(256) for _ in range(32))
        msg = bytes(rnd.randrange(256) for _ in range(rnd.randrange(90)))
        pub, sig = (ctypes.c_uint8 * 32)(), (ctypes.c_uint8 * 64)()
        host.ed_sign(seed, msg, len(msg), pub, sig)
        assert bytes(pub) == E.public_key(seed) and bytes(sig) == E.sign(seed, msg)
