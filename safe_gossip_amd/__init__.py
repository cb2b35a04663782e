"""safe_gossip_amd -- MI355X-native engine for safe_gossip's push-pull round.

Python host mirror of the reference crate's public surface
(``src/lib.rs:62-65``: ``Gossiper``, ``Statistics``, ``Error``) over the C ABI
in ``include/safe_gossip.h``.  One :class:`Network` is one simulated full-mesh
network resident on one MI355X; :meth:`Network.gossiper` returns the per-node
``Gossiper`` view (``send_new``, ``messages``, ``statistics``) and
:meth:`Network.next_round` runs ``Gossiper::next_round`` for every node plus the
delivery of every Push/Pull RPC (the reference harness round,
``src/gossiper.rs:198-235``, in the 2P schedule).

There is no CPU fallback: every call goes through ``libsafe_gossip_amd.so``
(hand-written gfx950 kernels) and raises :class:`DeviceError` when the library
or the GPU is unavailable.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from .build import LIB_PATH

__all__ = [
    "Network", "Gossiper", "Statistics", "RoundReport", "GossipError", "NoPeers",
    "AlreadyStarted", "DeviceError", "derive_params", "peer_of", "origin_of", "coin_of",
    "send_messages", "load_library", "SYMBOLS", "rpc_encode", "rpc_decode", "message_wrap",
    "message_unwrap", "split_frames", "SigFailure", "sha3_512", "ed25519_sign", "ed25519_verify",
    "default_rumor_key",
]

# ----------------------------------------------------------------- errors
class GossipError(Exception):
    """Mirror of ``enum Error`` (src/error.rs:23-51)."""

    code = None


class NoPeers(GossipError):
    """``Error::NoPeers``: there are no connected peers with which to gossip."""

    code = 1


class AlreadyStarted(GossipError):
    """``Error::AlreadyStarted``."""

    code = 2


class SigFailure(GossipError):
    """``Error::SigFailure``: a signed frame failed verification."""

    code = 3


class DeviceError(GossipError):
    """Engine-side failure (no library, no GPU, HIP error, device limit)."""


_ERRORS = {1: NoPeers, 2: AlreadyStarted, 3: SigFailure}

# ------------------------------------------------------------------ ctypes
class _Config(ctypes.Structure):
    _fields_ = [
        ("n_nodes", ctypes.c_uint32), ("n_rumors", ctypes.c_uint32),
        ("seed", ctypes.c_uint64), ("epoch", ctypes.c_uint32),
        ("counter_max", ctypes.c_uint8), ("max_c_rounds", ctypes.c_uint8),
        ("max_rounds", ctypes.c_uint8), ("schedule", ctypes.c_uint8),
        ("device", ctypes.c_int32), ("churn", ctypes.c_uint32),
        ("drop_push", ctypes.c_uint32), ("drop_pull", ctypes.c_uint32),
        ("rumor_slice", ctypes.c_uint32), ("reserved1", ctypes.c_uint32 * 3),
    ]


class _Stats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in (
        "rounds", "empty_pull_sent", "empty_push_sent", "full_message_sent",
        "full_message_received")]


class _Report(ctypes.Structure):
    _fields_ = [("round", ctypes.c_uint32), ("any_live", ctypes.c_uint32)]


_P = ctypes.c_void_p
_U8P = ctypes.POINTER(ctypes.c_uint8)
_U16P = ctypes.POINTER(ctypes.c_uint16)
_U32P = ctypes.POINTER(ctypes.c_uint32)
_U64P = ctypes.POINTER(ctypes.c_uint64)

# name -> (restype, argtypes): every symbol include/safe_gossip.h declares.
SYMBOLS = {
    "gs_create": (ctypes.c_int, [ctypes.POINTER(_Config), ctypes.POINTER(_P)]),
    "gs_destroy": (None, [_P]),
    "gs_get_params": (ctypes.c_int, [_P, _U8P]),
    "gs_send_new": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.c_uint32]),
    "gs_next_round": (ctypes.c_int, [_P, ctypes.POINTER(_Report)]),
    "gs_statistics": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.POINTER(_Stats)]),
    "gs_statistics_all": (ctypes.c_int, [_P, _U64P]),
    "gs_statistics_reduce": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(_Stats)]),
    "gs_messages": (ctypes.c_int, [_P, ctypes.c_uint32, _U64P]),
    "gs_known_all": (ctypes.c_int, [_P, _U64P]),
    "gs_known_counts": (ctypes.c_int, [_P, _U64P, _U64P]),
    "gs_known_counts_min": (ctypes.c_int, [_P, ctypes.c_uint32, _U64P, _U64P]),
    "gs_known_popcounts": (ctypes.c_int, [_P, _U32P]),
    "gs_set_params": (ctypes.c_int, [_P, _U8P]),
    "gs_rpc_encode": (ctypes.c_int, [ctypes.c_int, _U8P, ctypes.c_uint32, ctypes.c_uint8, _U8P,
                                     ctypes.c_uint32, _U32P]),
    "gs_rpc_decode": (ctypes.c_int, [_U8P, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int), _U32P, _U32P,
                                     _U8P]),
    "gs_message_wrap": (ctypes.c_int, [_U8P, ctypes.c_uint32, _U8P, _U8P, ctypes.c_uint32, _U32P]),
    "gs_message_unwrap": (ctypes.c_int, [_U8P, ctypes.c_uint32, _U32P, _U32P, _U32P]),
    "gs_set_rumor_key": (ctypes.c_int, [_P, ctypes.c_uint32, _U8P, ctypes.c_uint32]),
    "gs_rumor_key": (ctypes.c_int, [_P, ctypes.c_uint32, _U8P, ctypes.c_uint32, _U32P]),
    "gs_push_batch": (ctypes.c_int, [_P, ctypes.c_uint32, _U8P, ctypes.c_uint32, _U32P, _U32P]),
    "gs_handle_received": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.c_uint32, _U8P, ctypes.c_uint32,
                                          _U8P, ctypes.c_uint32, _U32P, _U32P]),
    "gs_handle_received_batch": (ctypes.c_int, [_P, ctypes.c_uint32, _U32P, _U32P, _U8P, _U32P, _U32P, _U8P,
                                                ctypes.c_uint32, _U32P, _U32P]),
    "gs_device": (ctypes.c_int, [_P]),
    "gs_sha3_512": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, _U8P, _U32P, _U32P, _U8P]),
    "gs_ed25519_verify": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, _U8P, _U8P, _U8P, _U32P, _U32P, _U8P]),
    "gs_ed25519_sign": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, _U8P, _U8P, _U32P, _U32P, _U8P, _U8P]),
    "gs_handle_received_signed": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.c_uint32, _U8P, _U8P, _U8P,
                                                 ctypes.c_uint32, _U8P, ctypes.c_uint32, _U32P, _U32P]),
    "gs_push_batch_signed": (ctypes.c_int, [_P, ctypes.c_uint32, _U8P, _U8P, ctypes.c_uint32, _U32P, _U32P]),
    "gs_dump_state": (ctypes.c_int, [_P, _U16P]),
    "gs_dump_records": (ctypes.c_int, [_P, _U16P, _U32P]),
    "gs_state_digest": (ctypes.c_int, [_P, _U64P]),
    "gs_state_digest_part": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]),
    "gs_digest_finish": (ctypes.c_int, [_P, ctypes.c_void_p, ctypes.c_uint32, _U64P, _U64P]),
    "gs_clear": (ctypes.c_int, [_P, ctypes.c_uint32]),
    "gs_sync": (ctypes.c_int, [_P]),
    "gs_round": (ctypes.c_uint32, [_P]),
    "gs_last_round_kernel_ms": (ctypes.c_float, [_P]),
    "gs_set_timing": (None, [_P, ctypes.c_int]),
    "gs_round_kernel_times": (ctypes.c_int32, [_P, ctypes.POINTER(ctypes.c_float), ctypes.c_uint32]),
    "gs_round_kernel_bytes": (ctypes.c_double, [_P]),
    "gs_round_kernel_name": (ctypes.c_char_p, [_P]),
    "gs_round_traffic": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), _U32P]),
    "gs_peer": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_uint32, ctypes.c_uint32]),
    "gs_origin": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_uint32]),
    "gs_coin": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_uint32]),
    "gs_fault": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_uint32]),
    "gs_derive_params": (None, [ctypes.c_uint32, _U8P]),
    "gs_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "gs_abi_version": (ctypes.c_uint32, []),
    "gs_build_id": (ctypes.c_char_p, []),
    # sharded engines (safe_gossip_amd.sharded)
    "gs_shard_create": (ctypes.c_int, [ctypes.POINTER(_Config), ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.POINTER(_P)]),
    "gs_shard_create_parts": (ctypes.c_int, [ctypes.POINTER(_Config), ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.POINTER(_P)]),
    "gs_shard_round_part": (ctypes.c_int, [_P, ctypes.c_uint32]),
    "gs_shard_info": (ctypes.c_int, [_P, _U32P]),
    "gs_shard_plan_info": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _U32P]),
    "gs_shard_bind": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P]),
    "gs_shard_pull": (ctypes.c_int, [_P]),
    "gs_stream": (ctypes.c_uint64, [_P]),
    # rumor-sliced engines (safe_gossip_amd.sliced)
    "gs_slice_bind": (ctypes.c_int, [_P, _P, _P, _P, _P]),
    "gs_slice_apply": (ctypes.c_int, [_P, ctypes.c_uint32]),
    "gs_slice_defer": (ctypes.c_int, [_P, ctypes.c_uint32]),
    "gs_slice_set_ext_limit": (ctypes.c_int, [_P, ctypes.c_uint32]),
    # the whole multi-GPU network behind the ABI (gs_net.cpp; C / C++ hosts)
    "gs_net_unique_id": (ctypes.c_int, [_U8P]),
    "gs_net_create": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _U8P,
                                     ctypes.POINTER(_P)]),
    "gs_net_create_local": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(_P)]),
    "gs_net_create_with": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _P,
                                          ctypes.POINTER(_P)]),
    "gs_net_destroy": (None, [_P]),
    "gs_net_send_new": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.c_uint32]),
    "gs_net_next_round": (ctypes.c_int, [_P, _P]),
    "gs_net_sync": (ctypes.c_int, [_P]),
    "gs_net_clear": (ctypes.c_int, [_P, ctypes.c_uint32]),
    "gs_net_known_counts": (ctypes.c_int, [_P, _U64P, _U64P]),
    "gs_net_statistics_all": (ctypes.c_int, [_P, _U64P]),
    "gs_net_dump_state": (ctypes.c_int, [_P, _U16P]),
    "gs_net_local_engines": (ctypes.c_uint32, [_P]),
    "gs_net_engine": (_P, [_P, ctypes.c_uint32]),
}

_LIB = None


def _share_torch_hip_runtime() -> None:
    """One HIP runtime per process.

    PyTorch-ROCm wheels carry their own ``libamdhip64.so`` (soname
    ``libamdhip64.so.7``, the engine's DT_NEEDED).  Loading it first makes the
    engine bind to the same runtime torch and its RCCL use, so the engine's
    streams and device pointers are valid for torch.distributed (the sharded
    transport) and the two never bring up the device twice.  Processes without
    torch use the system ROCm runtime.
    """
    if os.environ.get("SAFE_GOSSIP_AMD_HIP_RUNTIME") == "system":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    rt = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(rt):
        ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)


ABI_VERSION = 2  # include/safe_gossip.h GS_ABI_VERSION


def build_id() -> str:
    """The loaded library's provenance id (gs_build_id): the source hash of
    the tree it was built from (safe_gossip_amd/build.py source_hash)."""
    return load_library().gs_build_id().decode()


def load_library(path: Optional[str] = None):
    """Load ``libsafe_gossip_amd.so`` (built by ``__graft_entry__.build()``).

    Fails loudly when the library was built from other sources than the tree
    it is loaded from (its gs_build_id against build.source_hash()), or
    speaks another ABI version: a stale binary never runs silently."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or os.environ.get("SAFE_GOSSIP_AMD_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise DeviceError(f"engine library not built: {p} (run __graft_entry__.build())")
    _share_torch_hip_runtime()
    lib = ctypes.CDLL(p)
    for name, (res, args) in SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.gs_abi_version() != ABI_VERSION:
        raise DeviceError(f"{p}: C ABI version {lib.gs_abi_version()}, this binding speaks {ABI_VERSION}")
    from .build import source_hash
    have, want = lib.gs_build_id().decode(), source_hash()
    if have.split("+")[0] != want:
        raise DeviceError(f"{p} was built from other sources (build id {have}, tree {want}): "
                          "run __graft_entry__.build()")
    if path is None:
        _LIB = lib
    return lib


def _check(status: int) -> None:
    if status == 0:
        return
    lib = load_library()
    msg = lib.gs_status_string(status).decode()
    raise _ERRORS.get(status, DeviceError)(f"{msg} (status {status})")


# ------------------------------------------------------------------ values
@dataclass
class Statistics:
    """``struct Statistics`` (src/gossip.rs:209-264)."""

    rounds: int = 0
    empty_pull_sent: int = 0
    empty_push_sent: int = 0
    full_message_sent: int = 0
    full_message_received: int = 0

    FIELDS = ("rounds", "empty_pull_sent", "empty_push_sent", "full_message_sent",
              "full_message_received")

    @classmethod
    def new_max(cls) -> "Statistics":
        m = (1 << 64) - 1
        return cls(m, m, m, m, m)

    def add(self, other: "Statistics") -> None:
        for f in self.FIELDS:
            setattr(self, f, getattr(self, f) + getattr(other, f))

    def min(self, other: "Statistics") -> None:
        for f in self.FIELDS:
            setattr(self, f, min(getattr(self, f), getattr(other, f)))

    def max(self, other: "Statistics") -> None:
        for f in self.FIELDS:
            setattr(self, f, max(getattr(self, f), getattr(other, f)))

    def as_tuple(self):
        return tuple(getattr(self, f) for f in self.FIELDS)

    @classmethod
    def _from_c(cls, s: _Stats) -> "Statistics":
        return cls(s.rounds, s.empty_pull_sent, s.empty_push_sent, s.full_message_sent,
                   s.full_message_received)


@dataclass
class RoundReport:
    round: int
    any_live: bool


def derive_params(n: int):
    """``Gossip::add_peer`` parameters for network_size n (src/gossip.rs:59-64)."""
    out = (ctypes.c_uint8 * 3)()
    load_library().gs_derive_params(n, out)
    return tuple(out)


def peer_of(seed: int, epoch: int, rnd: int, node: int, n: int) -> int:
    return load_library().gs_peer(seed, epoch, rnd, node, n)


def origin_of(seed: int, epoch: int, rumor: int, n: int) -> int:
    return load_library().gs_origin(seed, epoch, rumor, n)


def fault_threshold(p: float) -> int:
    """Probability -> the engine's fault threshold over 2^32."""
    if not 0.0 <= p <= 1.0:
        raise ValueError(f"fault probability {p} outside [0, 1]")
    return min(int(round(p * 2.0 ** 32)), 0xFFFFFFFF)


FAULT_OFFLINE, FAULT_PUSH, FAULT_PULL = 1, 2, 4

# gs_schedule: "2P" (pulls after all pushes) or "SEQ" (the reference harness's
# literal order, src/gossiper.rs:217-234)
SCHEDULES = {"2P": 0, "SEQ": 1}


def fault_of(seed: int, epoch: int, rnd: int, node: int, faults) -> int:
    """Fault bits of (round, node); faults = (churn, drop_push, drop_pull) thresholds."""
    return load_library().gs_fault(seed, epoch, rnd, node, *faults)


def coin_of(seed: int, epoch: int, rnd: int, node: int) -> int:
    return load_library().gs_coin(seed, epoch, rnd, node)


# ------------------------------------------------------------ wire format
def _buf(data: bytes):
    return (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")


def rpc_encode(pull: bool, msg: bytes, counter: int) -> bytes:
    """``Message::serialise`` (cfg(test), src/messages.rs:48-50) of
    ``GossipRpc::{Push,Pull} { msg, counter }``: bincode."""
    lib = load_library()
    n = ctypes.c_uint32()
    lib.gs_rpc_encode(1 if pull else 0, _buf(msg), len(msg), counter, None, 0, ctypes.byref(n))
    out = (ctypes.c_uint8 * n.value)()
    _check(lib.gs_rpc_encode(1 if pull else 0, _buf(msg), len(msg), counter, out, n.value, ctypes.byref(n)))
    return bytes(out)


def rpc_decode(data: bytes):
    """``Message::deserialise`` (cfg(test), src/messages.rs:52-54) ->
    ``(pull, msg, counter)``; raises ``GossipError`` (Serialisation) on bad bytes."""
    lib = load_library()
    pull, off, ln, ctr = ctypes.c_int(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint8()
    _check(lib.gs_rpc_decode(_buf(data), len(data), ctypes.byref(pull), ctypes.byref(off), ctypes.byref(ln),
                             ctypes.byref(ctr)))
    return bool(pull.value), bytes(data[off.value:off.value + ln.value]), ctr.value


def message_wrap(payload: bytes, signature: bytes) -> bytes:
    """bincode of ``Message(payload, signature)`` (src/messages.rs:26-34); the
    signature is given (``ed25519_sign`` computes one)."""
    assert len(signature) == 64
    lib = load_library()
    n = ctypes.c_uint32()
    sig = _buf(signature)
    lib.gs_message_wrap(_buf(payload), len(payload), sig, None, 0, ctypes.byref(n))
    out = (ctypes.c_uint8 * n.value)()
    _check(lib.gs_message_wrap(_buf(payload), len(payload), sig, out, n.value, ctypes.byref(n)))
    return bytes(out)


def message_unwrap(data: bytes):
    """-> ``(payload, signature)`` of a bincode ``Message`` (framing only;
    ``ed25519_verify`` checks the signature)."""
    lib = load_library()
    po, pl, so = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib.gs_message_unwrap(_buf(data), len(data), ctypes.byref(po), ctypes.byref(pl), ctypes.byref(so)))
    return bytes(data[po.value:po.value + pl.value]), bytes(data[so.value:so.value + 64])


def _pack(msgs: Sequence[bytes]):
    off, ln, at = [], [], 0
    for m in msgs:
        off.append(at)
        ln.append(len(m))
        at += len(m)
    return (_buf(b"".join(msgs)), (ctypes.c_uint32 * max(1, len(msgs)))(*off),
            (ctypes.c_uint32 * max(1, len(msgs)))(*ln))


def sha3_512(msgs: Sequence[bytes], device: int = 0) -> List[bytes]:
    """SHA3-512 of each message, on the GPU (gs_verify.hip)."""
    lib = load_library()
    data, off, ln = _pack(msgs)
    out = (ctypes.c_uint8 * max(1, 64 * len(msgs)))()
    _check(lib.gs_sha3_512(device, len(msgs), data, off, ln, out))
    raw = bytes(out)
    return [raw[64 * i:64 * i + 64] for i in range(len(msgs))]


def ed25519_sign(seeds: Sequence[bytes], msgs: Sequence[bytes], device: int = 0):
    """``Keypair::sign::<Sha3_512>`` (ed25519-dalek 0.6, src/messages.rs:32) for
    32-byte secret seeds, on the GPU -> (public keys, 64-byte signatures)."""
    assert len(seeds) == len(msgs) and all(len(s) == 32 for s in seeds)
    lib = load_library()
    data, off, ln = _pack(msgs)
    k = len(msgs)
    pub, sig = (ctypes.c_uint8 * max(1, 32 * k))(), (ctypes.c_uint8 * max(1, 64 * k))()
    _check(lib.gs_ed25519_sign(device, k, _buf(b"".join(seeds)), data, off, ln, pub, sig))
    p, s = bytes(pub), bytes(sig)
    return [p[32 * i:32 * i + 32] for i in range(k)], [s[64 * i:64 * i + 64] for i in range(k)]


def ed25519_verify(pubs: Sequence[bytes], msgs: Sequence[bytes], sigs: Sequence[bytes],
                   device: int = 0) -> List[bool]:
    """``PublicKey::verify::<Sha3_512>`` (ed25519-dalek 0.6, the check of
    ``Message::deserialise``, src/messages.rs:38) of each (key, message,
    signature), on the GPU."""
    assert len(pubs) == len(msgs) == len(sigs)
    assert all(len(p) == 32 for p in pubs) and all(len(s) == 64 for s in sigs)
    lib = load_library()
    data, off, ln = _pack(msgs)
    k = len(msgs)
    ok = (ctypes.c_uint8 * max(1, k))()
    _check(lib.gs_ed25519_verify(device, k, _buf(b"".join(pubs)), _buf(b"".join(sigs)), data, off, ln, ok))
    return [bool(v) for v in bytes(ok)[:k]]


def split_frames(data: bytes) -> List[bytes]:
    """The RPCs of a u32-length-prefixed frame sequence (gs_push_batch,
    gs_handle_received)."""
    out, i = [], 0
    while i < len(data):
        m = int.from_bytes(data[i:i + 4], "little")
        out.append(bytes(data[i + 4:i + 4 + m]))
        i += 4 + m
    return out


def engine_push_batch(lib, h, node: int) -> List[bytes]:
    """gs_push_batch of one engine (a shard: ``node`` a global id it owns)."""
    n, c = ctypes.c_uint32(), ctypes.c_uint32()
    lib.gs_push_batch(h, node, None, 0, ctypes.byref(n), ctypes.byref(c))
    out = (ctypes.c_uint8 * max(1, n.value))()
    _check(lib.gs_push_batch(h, node, out, n.value, ctypes.byref(n), ctypes.byref(c)))
    return split_frames(bytes(out)[:n.value])


def engine_handle_received(lib, h, node: int, peer: int, message: bytes) -> List[bytes]:
    """gs_handle_received of one engine, the response buffer grown as needed."""
    cap = 4096
    while True:
        out = (ctypes.c_uint8 * cap)()
        n, c = ctypes.c_uint32(), ctypes.c_uint32()
        st = lib.gs_handle_received(h, node, peer, _buf(message), len(message), out, cap,
                                    ctypes.byref(n), ctypes.byref(c))
        if st == 5 and n.value > cap:  # responses larger than the buffer: nothing was applied
            cap = n.value
            continue
        _check(st)
        return split_frames(bytes(out)[:n.value])


def engine_handle_received_batch(lib, h, rpcs) -> List[List[bytes]]:
    """gs_handle_received_batch of one engine: (node, peer, message bytes) in order."""
    rpcs = list(rpcs)
    m = len(rpcs)
    nodes = np.array([r[0] for r in rpcs], dtype=np.uint32)
    peers = np.array([r[1] for r in rpcs], dtype=np.uint32)
    lens = np.array([len(r[2]) for r in rpcs], dtype=np.uint32)
    offs = np.zeros(m, dtype=np.uint32)
    if m:
        offs[1:] = np.cumsum(lens)[:-1]
    msgs = _buf(b"".join(r[2] for r in rpcs))
    resp = np.zeros(m + 1, dtype=np.uint32)
    cap = 4096
    while True:
        out = (ctypes.c_uint8 * cap)()
        n = ctypes.c_uint32()
        st = lib.gs_handle_received_batch(
            h, m, nodes.ctypes.data_as(_U32P), peers.ctypes.data_as(_U32P), msgs,
            offs.ctypes.data_as(_U32P), lens.ctypes.data_as(_U32P), out, cap, ctypes.byref(n),
            resp.ctypes.data_as(_U32P))
        if st == 5 and n.value > cap:  # responses larger than the buffer: nothing was applied
            cap = n.value
            continue
        _check(st)
        data = bytes(out)[:n.value]
        return [split_frames(data[resp[i]:resp[i + 1]]) for i in range(m)]


def default_rumor_key(rumor: int) -> bytes:
    """The message bytes a rumor slot has until ``set_rumor_key``: bincode of
    a 4-byte ``Vec<u8>`` holding the slot big-endian (so key order is slot
    order; gs_engine.cpp gs_create)."""
    return bytes([4, 0, 0, 0, 0, 0, 0, 0]) + int(rumor).to_bytes(4, "big")


# ---------------------------------------------------------------- network
class Network:
    """A simulated full-mesh network of ``n_nodes`` Gossipers on one MI355X.

    Equivalent to ``create_network(n)`` (src/gossiper.rs:157-171): every node
    knows every other node, so the protocol parameters are those of
    ``network_size == n``.  ``params`` overrides (counter_max, max_c_rounds,
    max_rounds).
    """

    def __init__(self, n_nodes: int, n_rumors: int, seed: int = 0x5AFE6055, epoch: int = 0,
                 params=None, device: int = 0, churn: float = 0.0, drop_push: float = 0.0,
                 drop_pull: float = 0.0, schedule: str = "2P", _rumor_slice: bool = False):
        self._lib = load_library()
        cfg = _Config()
        cfg.rumor_slice = 1 if _rumor_slice else 0  # safe_gossip_amd.sliced
        if schedule not in SCHEDULES:
            raise ValueError(f"schedule {schedule!r} not in {sorted(SCHEDULES)}")
        cfg.schedule = SCHEDULES[schedule]
        self.schedule = schedule
        # harness-injected faults (config 5): probabilities per (round, node)
        self.faults = (fault_threshold(churn), fault_threshold(drop_push), fault_threshold(drop_pull))
        cfg.churn, cfg.drop_push, cfg.drop_pull = self.faults
        cfg.n_nodes = n_nodes
        cfg.n_rumors = n_rumors
        cfg.seed = seed
        cfg.epoch = epoch
        if params is not None:
            cfg.counter_max, cfg.max_c_rounds, cfg.max_rounds = params
        cfg.device = device
        h = _P()
        _check(self._lib.gs_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.n = n_nodes
        self.R = n_rumors
        self.seed = seed
        self.epoch = epoch
        self.kw = (n_rumors + 63) // 64

    # lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.gs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # reference API
    def gossiper(self, node: int) -> "Gossiper":
        if not 0 <= node < self.n:
            raise IndexError(node)
        return Gossiper(self, node)

    @property
    def params(self):
        out = (ctypes.c_uint8 * 3)()
        _check(self._lib.gs_get_params(self._h, out))
        return tuple(out)

    @property
    def round(self) -> int:
        return self._lib.gs_round(self._h)

    def send_new(self, node: int, rumor: int) -> None:
        _check(self._lib.gs_send_new(self._h, node, rumor))

    def set_params(self, params=(0, 0, 0)) -> None:
        """``Gossiper::add_peer``'s parameter update (src/gossiper.rs:45-52):
        0 entries derive from n; raises :class:`AlreadyStarted` once a message
        was sent since the last clear."""
        p = (ctypes.c_uint8 * 3)(*params)
        _check(self._lib.gs_set_params(self._h, p))

    def next_round(self, report: bool = True) -> Optional[RoundReport]:
        if not report:
            _check(self._lib.gs_next_round(self._h, None))
            return None
        r = _Report()
        _check(self._lib.gs_next_round(self._h, ctypes.byref(r)))
        return RoundReport(r.round, bool(r.any_live))

    def statistics(self, node: int) -> Statistics:
        s = _Stats()
        _check(self._lib.gs_statistics(self._h, node, ctypes.byref(s)))
        return Statistics._from_c(s)

    def statistics_all(self) -> np.ndarray:
        out = np.zeros((self.n, 5), dtype=np.uint64)
        _check(self._lib.gs_statistics_all(self._h, out.ctypes.data_as(_U64P)))
        return out

    def statistics_reduce(self, op: str = "sum") -> Statistics:
        s = _Stats()
        _check(self._lib.gs_statistics_reduce(self._h, {"sum": 0, "min": 1, "max": 2}[op],
                                              ctypes.byref(s)))
        return Statistics._from_c(s)

    def messages(self, node: int) -> List[int]:
        w = np.zeros(self.kw, dtype=np.uint64)
        _check(self._lib.gs_messages(self._h, node, w.ctypes.data_as(_U64P)))
        bits = np.unpackbits(w.view(np.uint8), bitorder="little")[: self.R]
        return [int(i) for i in np.nonzero(bits)[0]]

    def known_all(self) -> np.ndarray:
        out = np.zeros((self.n, self.kw), dtype=np.uint64)
        _check(self._lib.gs_known_all(self._h, out.ctypes.data_as(_U64P)))
        return out

    def known_counts(self, min_known: Optional[int] = None):
        """(known node-rumor pairs, nodes knowing >= min_known rumors; default R)."""
        t = ctypes.c_uint64()
        c = ctypes.c_uint64()
        mk = self.R if min_known is None else min_known
        _check(self._lib.gs_known_counts_min(self._h, mk, ctypes.byref(t), ctypes.byref(c)))
        return int(t.value), int(c.value)

    # wire format (include/safe_gossip.h, src/messages.rs)
    def set_rumor_key(self, rumor: int, key: bytes) -> None:
        _check(self._lib.gs_set_rumor_key(self._h, rumor, _buf(key), len(key)))

    def rumor_key(self, rumor: int) -> bytes:
        n = ctypes.c_uint32()
        self._lib.gs_rumor_key(self._h, rumor, None, 0, ctypes.byref(n))
        out = (ctypes.c_uint8 * max(1, n.value))()
        _check(self._lib.gs_rumor_key(self._h, rumor, out, n.value, ctypes.byref(n)))
        return bytes(out)[:n.value]

    def push_batch(self, node: int) -> List[bytes]:
        """``Gossiper::next_round``'s Push RPCs of ``node`` this round (bytes)."""
        return engine_push_batch(self._lib, self._h, node)

    def handle_received(self, node: int, peer: int, message: bytes) -> List[bytes]:
        """``Gossiper::handle_received_message(peer, message)`` on ``node`` for a
        peer outside the simulated network (``peer >= n``): the Pull RPCs."""
        return engine_handle_received(self._lib, self._h, node, peer, message)

    def handle_received_batch(self, rpcs) -> List[List[bytes]]:
        """``handle_received`` for many (node, peer, message bytes) at once, in
        order (``gs_handle_received_batch``: one observation launch for all
        first Pushes); returns each RPC's Pull responses."""
        return engine_handle_received_batch(self._lib, self._h, rpcs)

    def handle_received_signed(self, node: int, peer: int, peer_key: bytes, message: bytes,
                               node_seed: Optional[bytes] = None) -> List[bytes]:
        """``handle_received`` for a signed ``Message`` frame (the reference's
        non-test path, src/messages.rs:36-43): verified on the GPU under
        ``peer_key`` (the peer's Id); raises ``SigFailure`` on a bad signature
        (the reference drops the frame).  With ``node_seed`` the Pull
        responses are signed by the node."""
        assert len(peer_key) == 32 and (node_seed is None or len(node_seed) == 32)
        cap = 4096
        while True:
            out = (ctypes.c_uint8 * cap)()
            n, c = ctypes.c_uint32(), ctypes.c_uint32()
            st = self._lib.gs_handle_received_signed(self._h, node, peer, _buf(peer_key),
                                                     _buf(node_seed) if node_seed else None, _buf(message),
                                                     len(message), out, cap, ctypes.byref(n), ctypes.byref(c))
            if st == 5 and n.value > cap:
                cap = n.value
                continue
            _check(st)
            return split_frames(bytes(out)[:n.value])

    def push_batch_signed(self, node: int, node_seed: bytes) -> List[bytes]:
        """``push_batch`` with every Push signed by the node (``Message::serialise``)."""
        assert len(node_seed) == 32
        n, c = ctypes.c_uint32(), ctypes.c_uint32()
        self._lib.gs_push_batch_signed(self._h, node, _buf(node_seed), None, 0, ctypes.byref(n), ctypes.byref(c))
        out = (ctypes.c_uint8 * max(1, n.value))()
        _check(self._lib.gs_push_batch_signed(self._h, node, _buf(node_seed), out, n.value, ctypes.byref(n),
                                              ctypes.byref(c)))
        return split_frames(bytes(out)[:n.value])

    def known_popcounts(self) -> np.ndarray:
        """``Gossiper::messages().len()`` of every node (device popcount)."""
        out = np.zeros(self.n, dtype=np.uint32)
        _check(self._lib.gs_known_popcounts(self._h, out.ctypes.data_as(_U32P)))
        return out

    def dump_state(self) -> np.ndarray:
        out = np.zeros((self.n, self.R), dtype=np.uint16)
        _check(self._lib.gs_dump_state(self._h, out.ctypes.data_as(_U16P)))
        return out

    def dump_records(self):
        rec = np.zeros((self.n, self.R), dtype=np.uint16)
        ps = np.zeros(self.n, dtype=np.uint32)
        _check(self._lib.gs_dump_records(self._h, rec.ctypes.data_as(_U16P),
                                         ps.ctypes.data_as(_U32P)))
        return rec, ps

    def state_digest(self) -> np.ndarray:
        """Per-node u64 digest of state codes, records, |P| and Statistics
        (``gs_state_digest``; oracle/gs_dense.c computes the same)."""
        out = np.zeros(self.n, dtype=np.uint64)
        _check(self._lib.gs_state_digest(self._h, out.ctypes.data_as(_U64P)))
        return out

    def clear(self, epoch: Optional[int] = None) -> None:
        """``Gossiper::clear`` for every node (src/gossiper.rs:111-115)."""
        self.epoch = self.epoch + 1 if epoch is None else epoch
        _check(self._lib.gs_clear(self._h, self.epoch))

    def sync(self) -> None:
        _check(self._lib.gs_sync(self._h))

    # measurement hooks
    def set_timing(self, on: bool) -> None:
        self._lib.gs_set_timing(self._h, 1 if on else 0)

    def last_round_kernel_ms(self) -> float:
        return float(self._lib.gs_last_round_kernel_ms(self._h))

    def round_kernel_times(self, max_n: int = 4096) -> np.ndarray:
        """Per-round device times (ms) of the round kernel since set_timing(True)."""
        out = np.zeros(max_n, dtype=np.float32)
        m = self._lib.gs_round_kernel_times(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                            max_n)
        if m < 0:
            raise DeviceError("kernel timing unavailable")
        return out[:m]

    def round_kernel_bytes(self) -> float:
        return float(self._lib.gs_round_kernel_bytes(self._h))

    def round_kernel_name(self) -> str:
        return self._lib.gs_round_kernel_name(self._h).decode()

    def round_traffic(self):
        """(algorithmic bytes per deliver+transition launch since set_timing(True),
        launches counted): the class rows the live filter leaves ungathered are
        not counted; launches = 0 means the static model (round_kernel_bytes)."""
        b, m = ctypes.c_double(), ctypes.c_uint32()
        _check(self._lib.gs_round_traffic(self._h, ctypes.byref(b), ctypes.byref(m)))
        return float(b.value), int(m.value)


class Gossiper:
    """Per-node view with the reference ``Gossiper`` methods (src/gossiper.rs:36-109)."""

    def __init__(self, net: Network, node: int):
        self._net = net
        self._node = node

    def id(self) -> int:
        """Node Id; Id order == index order."""
        return self._node

    def send_new(self, rumor: int) -> None:
        self._net.send_new(self._node, rumor)

    def messages(self) -> List[int]:
        return self._net.messages(self._node)

    def statistics(self) -> Statistics:
        return self._net.statistics(self._node)

    def push_batch(self) -> List[bytes]:
        """What ``Gossiper::next_round`` returned this round (its Push RPCs)."""
        return self._net.push_batch(self._node)

    def handle_received_message(self, peer: int, message: bytes) -> List[bytes]:
        """``Gossiper::handle_received_message`` (src/gossiper.rs:82-99) from a
        peer outside the simulated network; returns the Pull responses."""
        return self._net.handle_received(self._node, peer, message)


def send_messages(net: Network, num_of_msgs: int):
    """``send_messages`` (src/gossiper.rs:173-259) over the GPU engine.

    Philox-chosen first origin, then 50% per node per round while rumors
    remain, termination after a round in which no node pushed a live rumor.
    Returns ``(nodes_missed, msgs_missed, Statistics, rounds_run, round_full)``
    and clears the network (next epoch), like the reference.
    """
    assert num_of_msgs >= 1
    if num_of_msgs > net.R:
        raise ValueError(f"num_of_msgs {num_of_msgs} > rumor slots {net.R}")
    n = net.n
    next_rumor = 0
    net.send_new(origin_of(net.seed, net.epoch, 0, n), next_rumor)
    next_rumor += 1
    processed = True
    rounds_run = 0
    round_full = 0
    while processed:
        rnd = net.round + 1
        if next_rumor < num_of_msgs:
            for x in range(n):
                if next_rumor >= num_of_msgs:
                    break
                if coin_of(net.seed, net.epoch, rnd, x):
                    net.send_new(x, next_rumor)
                    next_rumor += 1
        rep = net.next_round()
        processed = rep.any_live
        rounds_run += 1
        if not round_full and next_rumor == num_of_msgs:
            # every node's messages().len() == num_of_msgs (only rumors
            # 0..num_of_msgs-1 are ever sent, so ">=" is "==")
            _, complete = net.known_counts(num_of_msgs)
            if complete == n:
                round_full = net.round
    # device reductions (src/gossiper.rs:241-256): Statistics::add over all
    # nodes, rounds = the last gossiper's, the final empty round subtracted
    tot = net.statistics_reduce("sum")
    stats = Statistics(net.statistics(n - 1).rounds, tot.empty_pull_sent - n,
                       tot.empty_push_sent - n, tot.full_message_sent, tot.full_message_received)
    counts = net.known_popcounts().astype(np.int64)
    missed = counts < num_of_msgs
    nodes_missed = int(missed.sum())
    msgs_missed = int((num_of_msgs - counts[missed]).sum())
    net.clear()
    return nodes_missed, msgs_missed, stats, rounds_run, round_full
