"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker, never as the product.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")

SCHED_2P = 0
SCHED_SEQ = 1


class OrStats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in (
        "rounds", "empty_pull_sent", "empty_push_sent", "full_message_sent",
        "full_message_received")]


class OrMetrics(ctypes.Structure):
    _fields_ = [("nodes_missed", ctypes.c_uint64), ("msgs_missed", ctypes.c_uint64),
                ("stats", OrStats), ("rounds_run", ctypes.c_uint32),
                ("round_full", ctypes.c_uint32)]


_P = ctypes.c_void_p
_U8P = ctypes.POINTER(ctypes.c_uint8)
_U16P = ctypes.POINTER(ctypes.c_uint16)
_U32P = ctypes.POINTER(ctypes.c_uint32)
_U64P = ctypes.POINTER(ctypes.c_uint64)

_SIGS = {
    "or_create": (_P, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32]),
    "or_destroy": (None, [_P]),
    "or_set_params": (None, [_P, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8]),
    "or_get_params": (None, [_P, _U8P]),
    "or_send_new": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.c_uint32]),
    "or_next_round": (ctypes.c_int, [_P, ctypes.c_int, _U32P]),
    "or_clear": (None, [_P, ctypes.c_uint32]),
    "or_round": (ctypes.c_uint32, [_P]),
    "or_dump_state": (None, [_P, _U16P]),
    "or_dump_records": (None, [_P, _U16P, _U32P]),
    "or_statistics": (None, [_P, _U64P]),
    "or_messages": (None, [_P, ctypes.c_uint32, _U64P]),
    "or_known_total": (ctypes.c_uint64, [_P]),
    "or_known_all": (None, [_P, _U64P]),
    "or_send_messages": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.c_int,
                                         ctypes.POINTER(OrMetrics)]),
    "or_philox": (None, [_U32P, _U32P, _U32P]),
    "or_peer": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_uint32, ctypes.c_uint32]),
    "or_origin": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_uint32]),
    "or_coin": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_uint32]),
    "or_fault": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_uint32]),
    "or_set_faults": (None, [_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "or_push_list": (None, [_P, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int32),
                            ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint32)]),
    "or_receive": (None, [_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int32,
                          ctypes.c_uint8, ctypes.POINTER(ctypes.c_int32),
                          ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint32)]),
    "or_derive_params": (None, [ctypes.c_uint32, _U8P]),
    # gs_dense.c: the dense bit-sliced OpenMP CPU line
    "dn_create": (_P, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32]),
    "dn_destroy": (None, [_P]),
    "dn_send_new": (None, [_P, ctypes.c_uint32, ctypes.c_uint32]),
    "dn_next_round": (ctypes.c_int, [_P, _U32P]),
    "dn_dump_state": (None, [_P, _U16P, _U64P]),
    "dn_dump_records": (None, [_P, _U16P, _U32P]),
    "dn_set_faults": (None, [_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "dn_digest": (None, [_P, _U64P]),
    "dn_next_round_digest": (ctypes.c_int, [_P, _U32P, _U64P]),
    "dn_threads": (ctypes.c_int, []),
    "or_ms_step": (None, [_U8P, _U32P, _U8P, ctypes.c_uint32, _U32P, ctypes.c_uint32,
                          ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_int]),
    "or_ms_new": (None, [_U8P]),
    "or_ms_our_counter": (ctypes.c_int, [_U8P]),
}

_LIB = None


def build_oracle() -> str:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"], check=True)
    return ORACLE_LIB


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(ORACLE_LIB):
            build_oracle()
        _LIB = ctypes.CDLL(ORACLE_LIB)
        for name, (res, args) in _SIGS.items():
            f = getattr(_LIB, name)
            f.restype = res
            f.argtypes = args
    return _LIB


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().or_philox(c, k, o)
    return tuple(o)


def derive_params(n):
    o = (ctypes.c_uint8 * 3)()
    lib().or_derive_params(n, o)
    return tuple(o)


TAGS = {"A": 0, "B": 1, "C": 2, "D": 3}

FAULT_OFFLINE, FAULT_PUSH, FAULT_PULL = 1, 2, 4


def fault_threshold(p):
    """Probability -> threshold over 2^32 (the engine's and the oracle's unit)."""
    return min(int(round(p * 2.0 ** 32)), 0xFFFFFFFF)


def fault_bits(seed, epoch, rnd, node, faults):
    """or_fault bits of (round, node) for faults = (churn, drop_push, drop_pull) thresholds."""
    return lib().or_fault(seed, epoch, rnd, node, *faults)


def ms_step(state, records, pir, params, next_round=True):
    """state = (tag, round, our_counter, rib); records = [(peer, counter)]."""
    io = (ctypes.c_uint8 * 4)(*state)
    peers = (ctypes.c_uint32 * max(1, len(records)))(*[p for p, _ in records])
    vals = (ctypes.c_uint8 * max(1, len(records)))(*[v for _, v in records])
    pr = (ctypes.c_uint32 * max(1, len(pir)))(*sorted(pir))
    lib().or_ms_step(io, peers, vals, len(records), pr, len(pir), params[0], params[1],
                     params[2], 1 if next_round else 0)
    return tuple(io)


class OracleNet:
    """One oracle network (per-node ordered maps, reference-faithful)."""

    def __init__(self, n, R, seed=0x5AFE6055, epoch=0, params=None, faults=None):
        """faults = (churn, drop_push, drop_pull) thresholds over 2^32 (fault_threshold)."""
        self._l = lib()
        self.h = self._l.or_create(n, R, seed, epoch)
        self.n, self.R, self.seed, self.epoch = n, R, seed, epoch
        self.faults = tuple(faults) if faults else (0, 0, 0)
        if params is not None:
            self._l.or_set_params(self.h, *params)
        if faults:
            self._l.or_set_faults(self.h, *self.faults)

    def offline(self, rnd):
        """Boolean mask of the nodes offline in round `rnd` (churn)."""
        return np.array([bool(fault_bits(self.seed, self.epoch, rnd, x, self.faults) & FAULT_OFFLINE)
                         for x in range(self.n)])

    def close(self):
        if self.h:
            self._l.or_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def params(self):
        o = (ctypes.c_uint8 * 3)()
        self._l.or_get_params(self.h, o)
        return tuple(o)

    @property
    def round(self):
        return self._l.or_round(self.h)

    def send_new(self, node, rumor):
        return self._l.or_send_new(self.h, node, rumor)

    def next_round(self, schedule=SCHED_2P):
        live = ctypes.c_uint32()
        rc = self._l.or_next_round(self.h, schedule, ctypes.byref(live))
        return rc, bool(live.value)

    def clear(self, epoch):
        self._l.or_clear(self.h, epoch)
        self.epoch = epoch

    def dump_state(self):
        out = np.zeros((self.n, self.R), dtype=np.uint16)
        self._l.or_dump_state(self.h, out.ctypes.data_as(_U16P))
        return out

    def dump_records(self):
        rec = np.zeros((self.n, self.R), dtype=np.uint16)
        ps = np.zeros(self.n, dtype=np.uint32)
        self._l.or_dump_records(self.h, rec.ctypes.data_as(_U16P), ps.ctypes.data_as(_U32P))
        return rec, ps

    def statistics(self):
        out = np.zeros((self.n, 5), dtype=np.uint64)
        self._l.or_statistics(self.h, out.ctypes.data_as(_U64P))
        return out

    def known_all(self):
        kw = (self.R + 63) // 64
        out = np.zeros((self.n, kw), dtype=np.uint64)
        self._l.or_known_all(self.h, out.ctypes.data_as(_U64P))
        return out

    def known_total(self):
        return int(self._l.or_known_total(self.h))

    def push_list(self, node):
        """[(rumor or -1 for the empty Push, counter)] node pushes this round."""
        r = (ctypes.c_int32 * (self.R + 1))()
        c = (ctypes.c_uint8 * (self.R + 1))()
        m = ctypes.c_uint32()
        self._l.or_push_list(self.h, node, r, c, ctypes.byref(m))
        return [(r[i], c[i]) for i in range(m.value)]

    def receive(self, node, peer, push, rumor, counter):
        """Gossip::receive of one RPC (rumor -1 = empty) from `peer` on
        `node`; returns the Pull responses [(rumor or -1, counter)]."""
        r = (ctypes.c_int32 * (self.R + 1))()
        c = (ctypes.c_uint8 * (self.R + 1))()
        m = ctypes.c_uint32()
        self._l.or_receive(self.h, node, peer, 1 if push else 0, rumor, counter, r, c, ctypes.byref(m))
        return [(r[i], c[i]) for i in range(m.value)]

    def send_messages(self, num_msgs, schedule=SCHED_SEQ):
        m = OrMetrics()
        rc = self._l.or_send_messages(self.h, num_msgs, schedule, ctypes.byref(m))
        assert rc == 0
        return m


class DenseNet:
    """The dense bit-sliced OpenMP CPU program (oracle/gs_dense.c), 2P only;
    faults = (churn, drop_push, drop_pull) thresholds over 2^32."""

    def __init__(self, n, R, seed=0x5AFE6055, epoch=0, faults=None):
        self._l = lib()
        self.h = self._l.dn_create(n, R, seed, epoch)
        assert self.h
        self.n, self.R = n, R
        if faults:
            self._l.dn_set_faults(self.h, *faults)

    def close(self):
        if self.h:
            self._l.dn_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def send_new(self, node, rumor):
        self._l.dn_send_new(self.h, node, rumor)

    def next_round(self, digest=False):
        """One round; with digest=True returns (live, the digest of the state
        before it), computed in the same pass."""
        live = ctypes.c_uint32()
        if not digest:
            self._l.dn_next_round(self.h, ctypes.byref(live))
            return bool(live.value)
        out = np.zeros(self.n, dtype=np.uint64)
        self._l.dn_next_round_digest(self.h, ctypes.byref(live), out.ctypes.data_as(_U64P))
        return bool(live.value), out

    def dump(self):
        codes = np.zeros((self.n, self.R), dtype=np.uint16)
        st = np.zeros((self.n, 5), dtype=np.uint64)
        self._l.dn_dump_state(self.h, codes.ctypes.data_as(_U16P), st.ctypes.data_as(_U64P))
        return codes, st

    def dump_records(self):
        rec = np.zeros((self.n, self.R), dtype=np.uint16)
        ps = np.zeros(self.n, dtype=np.uint32)
        self._l.dn_dump_records(self.h, rec.ctypes.data_as(_U16P), ps.ctypes.data_as(_U32P))
        return rec, ps

    def digest(self):
        out = np.zeros(self.n, dtype=np.uint64)
        self._l.dn_digest(self.h, out.ctypes.data_as(_U64P))
        return out


def digest_of(codes, recs, psize, stats):
    """The per-node digest (gs_common.h digest_*, oracle/gs_dense.c dn_digest)
    of parity dumps, in numpy: pins both implementations to one definition."""
    def mix(z):
        z = np.asarray(z, dtype=np.uint64)
        with np.errstate(over="ignore"):
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))
    n, R = codes.shape
    W = (R + 63) // 64
    # the 20 planes: code bits 14, 15, 7, 8, 0..4, record bits 15, 0..4, 7..11
    bits = [(codes, 14), (codes, 15), (codes, 7), (codes, 8)] + [(codes, b) for b in range(5)] + \
        [(recs, 15)] + [(recs, b) for b in range(5)] + [(recs, b) for b in range(7, 12)]
    weights = np.uint64(1) << np.arange(64, dtype=np.uint64)
    h = np.zeros(n, dtype=np.uint64)
    acc = np.zeros((n, W), dtype=np.uint64)
    with np.errstate(over="ignore"):
        for p, (arr, b) in enumerate(bits):
            v = ((arr.astype(np.uint64) >> np.uint64(b)) & np.uint64(1))
            v = np.concatenate([v, np.zeros((n, W * 64 - R), dtype=np.uint64)], axis=1).reshape(n, W, 64)
            words = (v * weights).sum(axis=2, dtype=np.uint64)  # distinct bits: the sum is the OR
            acc = acc + words * np.uint64((0x9E3779B97F4A7C15 * (2 * p + 1)) % (1 << 64))
        for j in range(W):
            h = h + mix(acc[:, j] ^ mix(np.uint64(j + 0x632BE59BD9B4E019)))
        h = h + mix(np.uint64(1 << 63) | psize.astype(np.uint64))
        for i in range(5):
            h = h + mix(stats[:, i].astype(np.uint64) ^ np.uint64((0x9E3779B97F4A7C15 * (i + 1)) % (1 << 64)))
    return h
