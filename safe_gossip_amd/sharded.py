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
from typing import Optional

import numpy as np

from . import (DeviceError, GossipError, NoPeers, RoundReport, _check, _Config, _Report,
               fault_threshold, load_library)

_P = ctypes.c_void_p
_U32P = ctypes.POINTER(ctypes.c_uint32)
_U64P = ctypes.POINTER(ctypes.c_uint64)
_U16P = ctypes.POINTER(ctypes.c_uint16)


def _lib():
    return load_library()


class _Shard:
    """One rank's engine plus its exchange buffers (torch device tensors)."""

    def __init__(self, lib, cfg, rank, world, torch, device):
        self.lib = lib
        h = _P()
        _check(lib.gs_shard_create(ctypes.byref(cfg), rank, world, ctypes.byref(h)))
        self.h = h
        info = (ctypes.c_uint32 * 12)()
        _check(lib.gs_shard_info(h, info))
        (self.lo, self.m, self.cap, self.capA, self.wa, self.world, self.rank, self.chunk,
         self.blockA, self.blockB) = list(info)[:10]
        dev = torch.device("cuda", device)
        i64 = torch.int64
        G = self.world
        # exchange A: two buffer sets (round parity); B: one
        self.sendA = [torch.zeros(G * self.blockA, dtype=i64, device=dev) for _ in range(2)]
        self.recvA = [torch.zeros(G * self.blockA, dtype=i64, device=dev) for _ in range(2)]
        self.sendB = torch.zeros(G * self.blockB, dtype=i64, device=dev)
        self.recvB = torch.zeros(G * self.blockB, dtype=i64, device=dev)
        _check(lib.gs_shard_bind(h, self.sendA[0].data_ptr(), self.sendA[1].data_ptr(),
                                 self.recvA[0].data_ptr(), self.recvA[1].data_ptr(),
                                 self.sendB.data_ptr(), self.recvB.data_ptr()))
        self.stream = torch.cuda.ExternalStream(lib.gs_stream(h), device=dev)

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
                 group=None, churn: float = 0.0, drop_push: float = 0.0, drop_pull: float = 0.0):
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
        if transport == "local":
            self.shards = [_Shard(self.lib, cfg, r, world, torch, device) for r in range(world)]
        elif transport == "dist":
            import torch.distributed as dist
            self.dist = dist
            self.rank = dist.get_rank(group)
            assert dist.get_world_size(group) == world
            self.shards = [_Shard(self.lib, cfg, self.rank, world, torch, device)]
            self.host_staged = dist.get_backend(group) == "gloo"
        else:
            raise ValueError(transport)
        self.round = 0
        self._delivered = True

    # ------------------------------------------------------------ lifecycle
    def close(self):
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

    def _deliver(self):
        """Exchange A (and A(0)'s ids in round 1), pull rows, exchange B of the
        current round, all ordered on the engine stream(s)."""
        if self._delivered or self.round == 0:
            return
        t = self.round
        sets = [0, 1] if t == 1 else [t % 2]
        if self.transport == "local":
            self._sync_all()
            for k in sets:
                self._local_exchange("A", k)
            for s in self.shards:
                _check(self.lib.gs_shard_pull(s.h))
            self._sync_all()
            self._local_exchange("B")
        else:
            s = self.shards[0]
            for k in sets:
                self._dist_exchange(s, s.sendA[k], s.recvA[k])
            _check(self.lib.gs_shard_pull(s.h))
            self._dist_exchange(s, s.sendB, s.recvB)
        self._delivered = True

    def _local_exchange(self, which, k=0):
        """Block d of every shard's send buffer -> block (its rank) of shard d's
        receive buffer (device copies; the shards share this GPU)."""
        G = self.world
        for d in range(G):
            dst = self.shards[d]
            for r in range(G):
                src = self.shards[r]
                if which == "A":
                    w = src.blockA
                    dst.recvA[k][r * w:(r + 1) * w].copy_(src.sendA[k][d * w:(d + 1) * w])
                else:
                    w = src.blockB
                    dst.recvB[r * w:(r + 1) * w].copy_(src.sendB[d * w:(d + 1) * w])
        self.torch.cuda.synchronize(self.device)

    def _dist_exchange(self, s, send, recv):
        """One equal-split all_to_all on the engine stream (RCCL), or staged
        through host memory (gloo)."""
        torch, dist = self.torch, self.dist
        if self.host_staged:
            _check(self.lib.gs_sync(s.h))
            hout = torch.empty(recv.numel(), dtype=torch.int64)
            dist.all_to_all_single(hout, send.cpu(), group=self.group)
            recv.copy_(hout.to(recv.device))
            torch.cuda.synchronize(self.device)
        else:
            with torch.cuda.stream(s.stream):
                dist.all_to_all_single(recv, send, group=self.group)

    def next_round(self, report: bool = True) -> Optional[RoundReport]:
        self._deliver()
        live = False
        for s in self.shards:
            if report:
                r = _Report()
                _check(self.lib.gs_next_round(s.h, ctypes.byref(r)))
                live |= bool(r.any_live)
            else:
                _check(self.lib.gs_next_round(s.h, None))
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
        for s in self.shards:
            _check(self.lib.gs_clear(s.h, self.epoch))
        self.round = 0
        self._delivered = True

    def sync(self) -> None:
        self._sync_all()

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

    # ------------------------------------------------------------ observers
    def _per_shard(self, fn):
        self._deliver()
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
