"""Philox4x32-10 (Random123) as vectorised torch int64 arithmetic.

Test infrastructure: an implementation independent of both the engine
(gs_common.h) and the oracle (oracle/gs_oracle.c), used to recompute per-node
quantities of the injected schedule (peer choices, fault draws) for networks
too large for a per-node ctypes loop -- on the GPU when one is present.  Pinned
by the Random123 KATs and against the oracle in tests/test_philox.py.
"""
import torch

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def _mulhilo(a, m):
    """(hi, lo) of a * m for int64 tensors a < 2^32 and a constant m < 2^32,
    without int64 overflow (16-bit split)."""
    a0 = a & 0xFFFF
    a1 = a >> 16
    p0 = a0 * m            # < 2^48
    p1 = a1 * m            # < 2^48
    hi = (p1 + (p0 >> 16)) >> 16
    lo = (p0 + ((p1 & 0xFFFF) << 16)) & MASK
    return hi, lo


def philox4x32(c0, c1, c2, c3, seed):
    """Philox4x32-10 of the counter (c0..c3, int64 tensors or ints broadcast
    to the same shape) under key = seed (u64: k0 low word, k1 high word)."""
    k0, k1 = seed & MASK, (seed >> 32) & MASK
    shape = torch.broadcast_shapes(*[t.shape for t in (c0, c1, c2, c3) if torch.is_tensor(t)])
    dev = next(t.device for t in (c0, c1, c2, c3) if torch.is_tensor(t))

    def T(v):
        return (v if torch.is_tensor(v) else torch.full(shape, v, dtype=torch.int64, device=dev)).expand(shape)
    c0, c1, c2, c3 = (T(v).to(torch.int64) for v in (c0, c1, c2, c3))
    for _ in range(10):
        hi0, lo0 = _mulhilo(c0, M0)
        hi1, lo1 = _mulhilo(c2, M1)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0), lo1, (hi0 ^ c3 ^ k1), lo0
        k0 = (k0 + W0) & MASK
        k1 = (k1 + W1) & MASK
    return c0, c1, c2, c3


def fault_bits(seed, epoch, rnd, nodes, churn, drop_push, drop_pull):
    """gs_fault / or_fault of (rnd, node) for every node in `nodes` (int64):
    1 offline, 2 push batch dropped, 4 pull batch dropped (Philox stream 3)."""
    w0, w1, w2, _ = philox4x32(rnd, nodes, 3, epoch, seed)
    return ((w0 < churn).to(torch.int64) | ((w1 < drop_push).to(torch.int64) << 1)
            | ((w2 < drop_pull).to(torch.int64) << 2))


def peer_of(seed, epoch, rnd, nodes, n):
    """gs_peer / or_peer: node x's choice among its n-1 peers (stream 0)."""
    w0, w1, _, _ = philox4x32(rnd, nodes, 0, epoch, seed)
    # mulhi64((w1:w0), n-1) = floor(((w1 << 32) + w0) * (n-1) / 2^64)
    m = n - 1
    hi_lo, _ = _mulhilo(w0, m)
    hi_hi, lo_hi = _mulhilo(w1, m)
    u = hi_hi + ((lo_hi + hi_lo) >> 32)
    return u + (u >= nodes).to(torch.int64)
