"""CPU restatement (test infrastructure only) of the signature half of
safe_gossip's wire path: ed25519 over a 64-byte digest, as the reference uses
it through ed25519-dalek ~0.6.1 with sha3 ~0.7.2 (neither vendored in
/root/reference; restated from their published algorithms):

  * Message::serialise   (src/messages.rs:30-34): keys.sign::<Sha3_512>(&rpc)
  * Message::deserialise (src/messages.rs:36-43): key.verify::<Sha3_512>(&msg, &sig)
  * Gossiper::handle_received_message (src/gossiper.rs:84-93): the peer's Id
    bytes are the public key; a failed verify drops the frame silently.

The curve arithmetic follows RFC 8032 section 5.1 (edwards25519, a = -1,
d = -121665/121666) with the hash as a parameter: ``hashlib.sha512`` gives
RFC 8032 Ed25519 (pinned by its section 7.1 test vectors in
tests/test_ed25519_oracle.py); ``hashlib.sha3_512`` gives the variant the
reference signs with (``Keypair::sign::<Sha3_512>`` hashes the secret-key
expansion, the nonce and the challenge with SHA3-512).  What the GPU path is
checked against is therefore pinned on the curve half only through the
SHA-512 vectors of the same code: the SHA3-512 curve results are parity
unpinned with respect to a real ed25519-dalek run.

Verification mirrors ed25519-dalek 0.6's ``PublicKey::verify``: reject when
the top three bits of S are set (signature[63] & 224), decompress A (reject
if y^2 - 1 over d y^2 + 1 has no square root), compute
R' = [S]B - [k]A with k = H(R || A || M) mod L, and accept iff the encoding of
R' equals the signature's R bytes.  Pure Python, for small batches only.
"""
from __future__ import annotations

import hashlib

P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)


def _inv(x: int) -> int:
    return pow(x, P - 2, P)


# Points in extended coordinates (X, Y, Z, T), x = X/Z, y = Y/Z, x*y = T/Z.
def _add(p, q):
    x1, y1, z1, t1 = p
    x2, y2, z2, t2 = q
    a = (y1 - x1) * (y2 - x2) % P
    b = (y1 + x1) * (y2 + x2) % P
    c = 2 * t1 * t2 * D % P
    dd = 2 * z1 * z2 % P
    e, f, g, h = b - a, dd - c, dd + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def _mul(s: int, p):
    q = (0, 1, 1, 0)  # neutral element
    while s > 0:
        if s & 1:
            q = _add(q, p)
        p = _add(p, p)
        s >>= 1
    return q


def _equal(p, q) -> bool:
    # x1 / z1 == x2 / z2 and y1 / z1 == y2 / z2
    return (p[0] * q[2] - q[0] * p[2]) % P == 0 and (p[1] * q[2] - q[1] * p[2]) % P == 0


def _recover_x(y: int, sign: int):
    if y >= P:
        return None
    x2 = (y * y - 1) * _inv(D * y * y + 1) % P
    if x2 == 0:
        return None if sign else 0
    x = pow(x2, (P + 3) // 8, P)
    if (x * x - x2) % P != 0:
        x = x * SQRT_M1 % P
    if (x * x - x2) % P != 0:
        return None
    if (x & 1) != sign:
        x = P - x
    return x


_GY = 4 * _inv(5) % P
_GX = _recover_x(_GY, 0)
G = (_GX, _GY, 1, _GX * _GY % P)


def compress(p) -> bytes:
    zi = _inv(p[2])
    x, y = p[0] * zi % P, p[1] * zi % P
    return int.to_bytes(y | ((x & 1) << 255), 32, "little")


def decompress(s: bytes, strict: bool = True):
    """RFC 8032 5.1.3 (strict: y >= p and x = 0 with the sign bit set are
    rejected).  strict=False is curve25519-dalek 0.x's decompression: the
    255-bit y is reduced mod p, and x = 0 keeps its sign bit (negating 0)."""
    if len(s) != 32:
        return None
    y = int.from_bytes(s, "little")
    sign = y >> 255
    y &= (1 << 255) - 1
    if not strict:
        y %= P
        x2 = (y * y - 1) * _inv(D * y * y + 1) % P
        x = pow(x2, (P + 3) // 8, P)
        if (x * x - x2) % P != 0:
            x = x * SQRT_M1 % P
        if (x * x - x2) % P != 0:
            return None
        if (x & 1) != sign:
            x = (P - x) % P
        return (x, y, 1, x * y % P)
    x = _recover_x(y, sign)
    if x is None:
        return None
    return (x, y, 1, x * y % P)


def _h(hashfn, *parts: bytes) -> bytes:
    h = hashfn()
    for p in parts:
        h.update(p)
    return h.digest()


def secret_expand(seed: bytes, hashfn=hashlib.sha3_512):
    if len(seed) != 32:
        raise ValueError("secret key seed is 32 bytes")
    h = _h(hashfn, seed)
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return a, h[32:]


def public_key(seed: bytes, hashfn=hashlib.sha3_512) -> bytes:
    a, _ = secret_expand(seed, hashfn)
    return compress(_mul(a, G))


def sign(seed: bytes, msg: bytes, hashfn=hashlib.sha3_512) -> bytes:
    a, prefix = secret_expand(seed, hashfn)
    A = compress(_mul(a, G))
    r = int.from_bytes(_h(hashfn, prefix, msg), "little") % L
    R = compress(_mul(r, G))
    k = int.from_bytes(_h(hashfn, R, A, msg), "little") % L
    s = (r + k * a) % L
    return R + int.to_bytes(s, 32, "little")


def verify(public: bytes, msg: bytes, sig: bytes, hashfn=hashlib.sha3_512, dalek: bool = True) -> bool:
    """dalek=True: ed25519-dalek 0.6 PublicKey::verify (see the module
    docstring); dalek=False: RFC 8032 5.1.7 (S < L, strict decoding,
    [S]B = R + [k]A)."""
    if len(public) != 32 or len(sig) != 64:
        return False
    Rb, Sb = sig[:32], sig[32:]
    s = int.from_bytes(Sb, "little")
    if dalek:
        if sig[63] & 224:
            return False
        A = decompress(public, strict=False)
        if A is None:
            return False
        k = int.from_bytes(_h(hashfn, Rb, public, msg), "little") % L
        negA = ((P - A[0]) % P, A[1], A[2], (P - A[3]) % P)
        Rp = _add(_mul(s, G), _mul(k, negA))
        return compress(Rp) == Rb
    if s >= L:
        return False
    A, R = decompress(public), decompress(Rb)
    if A is None or R is None:
        return False
    k = int.from_bytes(_h(hashfn, Rb, public, msg), "little") % L
    return _equal(_mul(s, G), _add(R, _mul(k, A)))
