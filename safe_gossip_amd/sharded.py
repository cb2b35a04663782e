"""Sharded network: the node-id space split across ranks.

Each rank's engine (``gs_shard_create``) owns a contiguous node range.  Every
round moves two sets of rows between ranks, each as ONE fixed-size all-to-all
(equal splits: the engine sizes every block for the binomial row counts, so
no count is read back and a round runs without a host synchronisation):

* A -- push rows: the class code of each node's push batch goes to the owner
  of its target, plus the source ids of next round's edges (the receiver
  builds next round's in-lists from them on its side stream);
* B -- pull rows: the owner of each target returns, per pusher, the pull batch
  ``Gossip::receive`` built (``src/gossip.rs:124-151``), in the reverse layout.

Pipeline parts: a rank's node range is cut into ``parts`` parts and both
exchanges are stored part-major, so the rows of one part move in one
all-to-all of their own.  The round kernel runs part by part: part h starts
as soon as its pull rows (B_h) are in, and its push rows of the next round
(A_h) leave while the following part is updated -- with RCCL the collectives
run on the process group's stream, overlapped with the round kernel on the
engine's stream (``async_op`` works waited on the engine stream, never on the
host).

Transports:

* ``"dist"``  -- one shard per process, ``torch.distributed.all_to_all_single``
  on the engine's own HIP stream (backend ``nccl`` = RCCL over xGMI).  With the
  ``gloo`` backend the rows are staged through host memory.
* ``"local"`` -- all ``world`` shards in this process on one device, exchanged
  by device copies (used to test the sharded algorithm on a single GPU).

PyTorch is plumbing here (device buffers, streams, collectives); all protocol
work runs in the engine's gfx950 kernels.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import numpy as np

from . import (DeviceError, GossipError, NoPeers, RoundReport, _buf, _check, _Config, _Report,
               engine_handle_received_batch, engine_push_batch, fault_threshold, load_library, rpc_decode)

# RCCL's all_to_all_single is exact up to 2^30 bytes per rank (DESIGN.md
# section 7, "The single-part stall").
RCCL_MAX_BYTES = 1 << 30

_P = ctypes.c_void_p
_U32P = ctypes.POINTER(ctypes.c_uint32)
_U64P = ctypes.POINTER(ctypes.c_uint64)
_U16P = ctypes.POINTER(ctypes.c_uint16)


def _lib():
    return load_library()


def plan_info(n_nodes: int, n_rumors: int, world: int, rank: int = 0, parts: int = 4,
              schedule: int = 0) -> dict:
    """The exchange layout of one rank without creating an engine
    (``gs_shard_plan_info``, host only): node range, rows per sub-block, row
    size, buffer rows, and the largest single collective of a round (one
    part's all-to-all, bytes per rank)."""
    cfg = _Config()
    cfg.n_nodes, cfg.n_rumors, cfg.schedule = n_nodes, n_rumors, schedule
    info = (ctypes.c_uint32 * 14)()
    _check(_lib().gs_shard_plan_info(ctypes.byref(cfg), rank, world, parts, info))
    keys = ("lo", "m", "capP", "idrows", "row_words", "world", "rank", "chunk", "parts", "mP", "rowsA", "rowsB",
            "row_words_b", "codes")
    d = dict(zip(keys, list(info)))
    ra, rb = d["row_words"] * 4, d["row_words_b"] * 4
    d["row_bytes"], d["row_bytes_b"] = ra, rb
    # part h of A: world sub-blocks of capP rows (+ idrows for the last part); B: capP rows
    d["max_collective_bytes"] = max(world * (d["capP"] + d["idrows"]) * ra, world * d["capP"] * rb)
    d["bytes_per_round"] = d["rowsA"] * ra + d["rowsB"] * rb  # A + B sent per rank (self block included)
    return d


class _Shard:
    """One rank's engine plus its exchange buffers (torch device tensors)."""

    def __init__(self, lib, cfg, rank, world, parts, torch, device):
        self.lib = lib
        h = _P()
        _check(lib.gs_shard_create_parts(ctypes.byref(cfg), rank, world, parts, ctypes.byref(h)))
        self.h = h
        info = (ctypes.c_uint32 * 14)()
        _check(lib.gs_shard_info(h, info))
        (self.lo, self.m, self.capP, self.idrows, self.wa, self.world, self.rank, self.chunk,
         self.parts, self.mP, self.rowsA, self.rowsB, self.wb, self.codes) = list(info)
        dev = torch.device("cuda", device)
        # rows of wa (A) / wb (B) u32 words: the 2-plane class code (4W
        # words), or at R_pad <= 16 code rows (A: push code + target word, B:
        # pull code)
        i32 = torch.int32
        # exchange A: two buffer sets (round parity); B: one
        self.sendA = [torch.zeros(self.rowsA * self.wa, dtype=i32, device=dev) for _ in range(2)]
        self.recvA = [torch.zeros(self.rowsA * self.wa, dtype=i32, device=dev) for _ in range(2)]
        self.sendB = torch.zeros(self.rowsB * self.wb, dtype=i32, device=dev)
        self.recvB = torch.zeros(self.rowsB * self.wb, dtype=i32, device=dev)
        # (zeroed on torch's stream: done before the engine's non-blocking
        # streams, which do not wait for it, touch the buffers)
        torch.cuda.synchronize(dev)
        _check(lib.gs_shard_bind(h, self.sendA[0].data_ptr(), self.sendA[1].data_ptr(),
                                 self.recvA[0].data_ptr(), self.recvA[1].data_ptr(),
                                 self.sendB.data_ptr(), self.recvB.data_ptr()))
        self.stream = torch.cuda.ExternalStream(lib.gs_stream(h), device=dev)

    def region(self, which: str, h: int):
        """Part h of an exchange buffer: (first u32 word, u32 words per rank
        sub-block); the part's world sub-blocks are contiguous."""
        rows = self.capP + (self.idrows if which == "A" and h == self.parts - 1 else 0)
        w = self.wa if which == "A" else self.wb
        return h * self.world * self.capP * w, rows * w

    def close(self):
        if self.h:
            self.lib.gs_destroy(self.h)
            self.h = None


class ShardedNetwork:
    """A network of ``n_nodes`` gossipers sharded over ``world`` ranks.

    Mirrors :class:`safe_gossip_amd.Network`: ``send_new``, ``next_round``,
    ``statistics_all``, ``known_all``, ``dump_state``, ``dump_records``,
    ``known_counts`` and ``clear``.  With ``transport="dist"`` every rank makes
    the same calls (``send_new`` is ignored by ranks that do not own the node)
    and observers return the whole network on every rank (all-gathered in rank
    order).
    """

    def __init__(self, n_nodes: int, n_rumors: int, world: int, seed: int = 0x5AFE6055,
                 epoch: int = 0, params=None, device: int = 0, transport: str = "local",
                 group=None, churn: float = 0.0, drop_push: float = 0.0, drop_pull: float = 0.0,
                 parts: Optional[int] = None):
        import torch
        self.torch = torch
        self.lib = _lib()
        self.n, self.R, self.seed, self.epoch = n_nodes, n_rumors, seed, epoch
        self.world = world
        self.transport = transport
        self.group = group
        self.device = device
        self.kw = (n_rumors + 63) // 64
        cfg = _Config()
        cfg.n_nodes = n_nodes
        cfg.n_rumors = n_rumors
        cfg.seed = seed
        cfg.epoch = epoch
        if params is not None:
            cfg.counter_max, cfg.max_c_rounds, cfg.max_rounds = params
        cfg.device = device
        self.faults = (fault_threshold(churn), fault_threshold(drop_push), fault_threshold(drop_pull))
        cfg.churn, cfg.drop_push, cfg.drop_pull = self.faults
        self._cfg = cfg
        self.host_staged = False
        # largest RCCL collective issued at once (bytes per rank; tests lower it)
        self.max_collective_bytes = int(os.environ.get("SAFE_GOSSIP_AMD_RCCL_MAX_BYTES", RCCL_MAX_BYTES))
        if transport == "local":
            self.parts = 1 if parts is None else parts
            self.shards = [_Shard(self.lib, cfg, r, world, self.parts, torch, device) for r in range(world)]
        elif transport == "dist":
            import torch.distributed as dist
            self.dist = dist
            self.rank = dist.get_rank(group)
            assert dist.get_world_size(group) == world
            self.host_staged = dist.get_backend(group) == "gloo"
            # four parts overlap the RCCL exchanges with the round kernel
            self.parts = (1 if self.host_staged else 4) if parts is None else parts
            self.shards = [_Shard(self.lib, cfg, self.rank, world, self.parts, torch, device)]
            s = self.shards[0]
            biggest = max(world * s.region(which, h)[1] * 4 for which in "AB" for h in range(s.parts))
            if not self.host_staged and world > 1 and biggest > self.max_collective_bytes:
                for sh in self.shards:
                    sh.close()
                raise ValueError(f"an exchange of {biggest} B per rank exceeds the {self.max_collective_bytes} B "
                                 f"RCCL all_to_all limit; use more pipeline parts (parts={self.parts})")
        else:
            raise ValueError(transport)
        # parts that hold nodes (a small rank range holds fewer whole blocks
        # than asked: gs_shard_info reports the effective count)
        self.parts = self.shards[0].parts
        self.round = 0
        self._delivered = True
        self._pendA = []   # async works of exchange A of the current round
        self._pendB = {}   # part -> async work of exchange B of the current round

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "shards", []):
            self._wait_all()
        for s in getattr(self, "shards", []):
            s.close()
        self.shards = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def params(self):
        out = (ctypes.c_uint8 * 3)()
        _check(self.lib.gs_get_params(self.shards[0].h, out))
        return tuple(out)

    def owner(self, node: int) -> int:
        return node // self.shards[0].chunk

    # ------------------------------------------------------------ protocol
    def send_new(self, node: int, rumor: int) -> None:
        if self.n < 2:
            raise NoPeers("There are no connected peers with which to gossip.")
        if not 0 <= node < self.n:
            raise GossipError(f"node {node} out of range")
        for s in self.shards:
            if s.lo <= node < s.lo + s.m:
                _check(self.lib.gs_send_new(s.h, node, rumor))

    def _sync_all(self):
        for s in self.shards:
            _check(self.lib.gs_sync(s.h))

    # ------------------------------------------------------------ exchanges
    def _exchange(self, which, h, k=0):
        """Part h of exchange A (buffer set k) or B: sub-block d of every
        rank's send region -> sub-block (its rank) of rank d's receive region.
        Code rows: the engine also writes the rows of a rank's own sub-block
        (and the pulls answering them) straight into its receive buffer, so
        one rank exchanges nothing (no RCCL self-copy of the whole network).
        Returns an async work (RCCL) or None (done)."""
        own = self.shards[0].codes and self.world == 1  # own sub-blocks are not exchanged
        if self.transport == "local":
            self._sync_all()
            for d, dst in enumerate(self.shards):
                for r, src in enumerate(self.shards):
                    if own and r == d:
                        continue
                    off, w = src.region(which, h)
                    if which == "A":
                        sb, rb = src.sendA[k], dst.recvA[k]
                    else:
                        sb, rb = src.sendB, dst.recvB
                    rb[off + r * w:off + (r + 1) * w].copy_(sb[off + d * w:off + (d + 1) * w])
            self.torch.cuda.synchronize(self.device)
            return None
        s = self.shards[0]
        off, w = s.region(which, h)
        span = slice(off, off + self.world * w)
        send, recv = (s.sendA[k], s.recvA[k]) if which == "A" else (s.sendB, s.recvB)
        torch, dist = self.torch, self.dist
        if self.host_staged:  # gloo: rows through host memory, synchronously
            _check(self.lib.gs_sync(s.h))
            hout = torch.empty(self.world * w, dtype=torch.int32)
            dist.all_to_all_single(hout, send[span].cpu(), group=self.group)
            if own:  # (every sub-block but this rank's own)
                hdev = hout.to(recv.device)
                for r in range(self.world):
                    if r != self.rank:
                        recv[off + r * w:off + (r + 1) * w].copy_(hdev[r * w:(r + 1) * w])
            else:
                recv[span].copy_(hout.to(recv.device))
            torch.cuda.synchronize(self.device)
            return None
        if own:  # one rank, code rows: nothing moves
            return None
        # RCCL: the collective waits for the engine stream's work so far and
        # runs on the process group's stream; the engine stream waits for it
        # only when its rows are needed (_wait).  RCCL 2.26's all_to_all_single
        # returns wrong bytes past 2^30 per rank (measured on one rank,
        # exp/r3/rccl_size.py: 1024 MiB exact, 1025 MiB not), so a larger
        # exchange moves in pieces of at most RCCL_MAX_BYTES (one rank: the
        # span is its own single block, cut anywhere); with several ranks the
        # parts keep every exchange far below it (constructor check).
        limit = self.max_collective_bytes
        if self.world * w * 4 <= limit:
            with torch.cuda.stream(s.stream):
                return dist.all_to_all_single(recv[span], send[span], group=self.group, async_op=True)
        assert self.world == 1, "multi-rank exchange above the RCCL size limit (constructor check)"
        step = max(1, limit // 4)
        works = []
        with torch.cuda.stream(s.stream):
            for a in range(off, off + w, step):
                b = min(a + step, off + w)
                works.append(dist.all_to_all_single(recv[a:b], send[a:b], group=self.group, async_op=True))
        return works

    def _wait(self, work):
        if work is None:
            return
        with self.torch.cuda.stream(self.shards[0].stream):
            for wk in (work if isinstance(work, list) else [work]):
                wk.wait()

    def _wait_all(self):
        for w in self._pendA:
            self._wait(w)
        self._pendA = []
        for w in self._pendB.values():
            self._wait(w)
        self._pendB = {}

    def _deliver(self):
        """Exchange A of the current round complete (and, in round 1, the ids
        of round 1: part P-1 of buffer set 0), the pull rows, and every part
        of exchange B issued.  The parts of B are waited for by next_round part
        by part (observers wait for all)."""
        if self._delivered or self.round == 0:
            return
        t = self.round
        if t == 1 and not self.shards[0].codes:  # (code rows carry no ids)
            self._pendA.append(self._exchange("A", self.parts - 1, 0))
        for w in self._pendA:
            self._wait(w)
        self._pendA = []
        for s in self.shards:
            _check(self.lib.gs_shard_pull(s.h))
        self._pendB = {h: self._exchange("B", h) for h in range(self.parts)}
        self._delivered = True

    def next_round(self, report: bool = True) -> Optional[RoundReport]:
        """Deliver round t (pull rows, exchange B) and produce round t+1, part
        by part: part h's round kernel waits for B_h only, and A_h(t+1) leaves
        as soon as it is written."""
        self._deliver()
        t = self.round
        k = (t + 1) % 2
        for h in range(self.parts - 1):
            self._wait(self._pendB.pop(h, None))
            for s in self.shards:
                _check(self.lib.gs_shard_round_part(s.h, h))
            self._pendA.append(self._exchange("A", h, k))
        self._wait(self._pendB.pop(self.parts - 1, None))
        live = False
        for s in self.shards:
            if report:
                r = _Report()
                _check(self.lib.gs_next_round(s.h, ctypes.byref(r)))
                live |= bool(r.any_live)
            else:
                _check(self.lib.gs_next_round(s.h, None))
        self._pendA.append(self._exchange("A", self.parts - 1, k))
        self.round += 1
        self._delivered = False
        if not report:
            return None
        if self.transport == "dist":
            t = self.torch.tensor([1 if live else 0], dtype=self.torch.int32,
                                  device=("cpu" if self.host_staged else f"cuda:{self.device}"))
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
            live = bool(int(t.item()))
        return RoundReport(self.round, live)

    def clear(self, epoch: Optional[int] = None) -> None:
        self.epoch = self.epoch + 1 if epoch is None else epoch
        self._wait_all()  # no exchange of the old epoch may still write the buffers
        for s in self.shards:
            _check(self.lib.gs_clear(s.h, self.epoch))
        self.round = 0
        self._delivered = True

    def sync(self) -> None:
        self._wait_all()
        self._sync_all()

    # ------------------------------------------------------------ wire format
    # The byte boundary of src/gossiper.rs:70-99 on a sharded network: every
    # shard holds the rumor keys; an RPC goes to the shard owning its node (a
    # global id).  dist: every rank makes the same calls, the owner answers
    # and the answers are all-gathered.  Code-row shards (R_pad <= 16, 2P)
    # apply them through the EXT variant of the packed DLV kernel
    # (gs_dlv4.hip), class-row shards in their round kernel's n_ext block.
    def set_rumor_key(self, rumor: int, key: bytes) -> None:
        self._keys = None  # the key set _validate checks against, rebuilt on next use
        for s in self.shards:
            _check(self.lib.gs_set_rumor_key(s.h, rumor, _buf(key), len(key)))

    def rumor_key(self, rumor: int) -> bytes:
        h = self.shards[0].h
        n = ctypes.c_uint32()
        self.lib.gs_rumor_key(h, rumor, None, 0, ctypes.byref(n))
        out = (ctypes.c_uint8 * max(1, n.value))()
        _check(self.lib.gs_rumor_key(h, rumor, out, n.value, ctypes.byref(n)))
        return bytes(out)[:n.value]

    def _shard_of(self, node: int):
        for s in self.shards:
            if s.lo <= node < s.lo + s.m:
                return s
        return None

    def _share(self, mine):
        """dist: every rank's value (rank order); local: [mine]."""
        if self.transport == "local":
            return [mine]
        objs = [None] * self.world
        self.dist.all_gather_object(objs, mine, group=self.group)
        return objs

    def push_batch(self, node: int) -> List[bytes]:
        """``Gossiper::next_round``'s Push RPCs of ``node`` this round."""
        if not 0 <= node < self.n:
            _check(-1)
        self._wait_all()  # (the round kernel wrote the planes on the engine stream)
        s = self._shard_of(node)
        mine = engine_push_batch(self.lib, s.h, node) if s is not None else None
        return next(v for v in self._share(mine) if v is not None)

    def _validate(self, rpcs):
        """Every RPC checked before any shard applies one (the batch is whole
        or nothing across shards too): ids, then the frame (GossipError on
        bad bytes, src/gossiper.rs:89-94) and its rumor key."""
        if getattr(self, "_keys", None) is None:  # (2 FFI calls per rumor: built once per key change)
            self._keys = {self.rumor_key(r) for r in range(self.R)}
        keys = self._keys
        for node, peer, msg in rpcs:
            if not 0 <= node < self.n or peer < self.n:
                _check(-1)
            _, m, ctr = rpc_decode(msg)
            if (m or ctr) and m not in keys:
                _check(-1)

    def handle_received(self, node: int, peer: int, message: bytes) -> List[bytes]:
        """``Gossiper::handle_received_message(peer, message)`` on ``node`` for
        a peer outside the network: the Pull RPCs (after this round's
        deliveries, like the single engine)."""
        return self.handle_received_batch([(node, peer, message)])[0]

    def handle_received_batch(self, rpcs) -> List[List[bytes]]:
        """``handle_received`` for many (node, peer, message) in order; each
        shard takes its nodes' RPCs in one gs_handle_received_batch."""
        rpcs = list(rpcs)
        self._validate(rpcs)
        self._per_shard(lambda s: None)  # round delivered: pull rows in, exchange B waited for
        mine = {}
        for s in self.shards:
            idx = [i for i, r in enumerate(rpcs) if s.lo <= r[0] < s.lo + s.m]
            if idx:
                for i, resp in zip(idx, engine_handle_received_batch(self.lib, s.h, [rpcs[i] for i in idx])):
                    mine[i] = resp
        out = {}
        for d in self._share(mine):
            out.update(d)
        return [out[i] for i in range(len(rpcs))]

    # measurement hooks (this process's first shard)
    def set_timing(self, on: bool) -> None:
        for s in self.shards:
            self.lib.gs_set_timing(s.h, 1 if on else 0)

    def round_kernel_times(self, max_n: int = 4096) -> np.ndarray:
        out = np.zeros(max_n, dtype=np.float32)
        m = self.lib.gs_round_kernel_times(self.shards[0].h,
                                           out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), max_n)
        if m < 0:
            raise DeviceError("kernel timing unavailable")
        return out[:m]

    def round_kernel_bytes(self) -> float:
        return float(self.lib.gs_round_kernel_bytes(self.shards[0].h))

    def round_kernel_name(self) -> str:
        return self.lib.gs_round_kernel_name(self.shards[0].h).decode()

    # ------------------------------------------------------------ observers
    def _per_shard(self, fn):
        self._deliver()
        for w in self._pendB.values():
            self._wait(w)
        self._pendB = {}
        return [fn(s) for s in self.shards]

    def _gather_rows(self, parts):
        """Concatenate per-shard row blocks (dist: all-gather, rows in rank order)."""
        if self.transport == "local":
            return np.concatenate(parts, axis=0)
        torch, dist = self.torch, self.dist
        part = parts[0]
        objs = [None] * self.world
        dist.all_gather_object(objs, part, group=self.group)
        return np.concatenate(objs, axis=0)

    def statistics_all(self) -> np.ndarray:
        def f(s):
            out = np.zeros((s.m, 5), dtype=np.uint64)
            if s.m:
                _check(self.lib.gs_statistics_all(s.h, out.ctypes.data_as(_U64P)))
            return out
        return self._gather_rows(self._per_shard(f))

    def known_all(self) -> np.ndarray:
        def f(s):
            out = np.zeros((s.m, self.kw), dtype=np.uint64)
            if s.m:
                _check(self.lib.gs_known_all(s.h, out.ctypes.data_as(_U64P)))
            return out
        return self._gather_rows(self._per_shard(f))

    def dump_state(self) -> np.ndarray:
        def f(s):
            out = np.zeros((s.m, self.R), dtype=np.uint16)
            if s.m:
                _check(self.lib.gs_dump_state(s.h, out.ctypes.data_as(_U16P)))
            return out
        return self._gather_rows(self._per_shard(f))

    def dump_records(self):
        def f(s):
            rec = np.zeros((s.m, self.R), dtype=np.uint16)
            ps = np.zeros(s.m, dtype=np.uint32)
            if s.m:
                _check(self.lib.gs_dump_records(s.h, rec.ctypes.data_as(_U16P),
                                                ps.ctypes.data_as(_U32P)))
            return np.concatenate([rec.astype(np.uint32), ps[:, None]], axis=1)
        both = self._gather_rows(self._per_shard(f))
        return both[:, :-1].astype(np.uint16), both[:, -1].astype(np.uint32)

    def state_digest(self) -> np.ndarray:
        """Per-node digest (gs_state_digest) of the whole network, in node order."""
        def f(s):
            out = np.zeros(s.m, dtype=np.uint64)
            if s.m:
                _check(self.lib.gs_state_digest(s.h, out.ctypes.data_as(_U64P)))
            return out[:, None]
        return self._gather_rows(self._per_shard(f))[:, 0]

    def known_counts(self, min_known: Optional[int] = None):
        mk = self.R if min_known is None else min_known

        def f(s):
            if not s.m:
                return (0, 0)
            t, c = ctypes.c_uint64(), ctypes.c_uint64()
            _check(self.lib.gs_known_counts_min(s.h, mk, ctypes.byref(t), ctypes.byref(c)))
            return (int(t.value), int(c.value))
        parts = self._per_shard(f)
        tot = sum(p[0] for p in parts)
        comp = sum(p[1] for p in parts)
        if self.transport == "dist":
            t = self.torch.tensor([tot, comp], dtype=self.torch.int64,
                                  device=("cpu" if self.host_staged else f"cuda:{self.device}"))
            self.dist.all_reduce(t, group=self.group)
            tot, comp = int(t[0].item()), int(t[1].item())
        return tot, comp
