"""A multi-GPU network whose round loop runs in the library (``gs_net_*``,
DESIGN.md section 7d): the C++ driver of node shards and rumor slices that a
host without Python uses, bound here with ctypes so Python callers (the
bench) can run the same loop.

With ``transport="dist"`` every process of a ``torch.distributed`` group is
one rank (one GPU each): rank 0's RCCL id is broadcast over the group, then
the library joins its own RCCL communicator and issues every exchange on a
stream of its own, ordered against the engine stream with events.
``transport="host"``: the same, but the library calls back into this module
for every collective, on host buffers it staged (``gs_net_create_with``),
which runs them over the group's own backend (gloo: several ranks may share
one GPU -- the rehearsal of the multi-process loop on one box).
``transport="local"`` holds every rank in this process on one device.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import NoPeers, RoundReport, _check, _Config, _Report, fault_threshold, load_library

_U64P = ctypes.POINTER(ctypes.c_uint64)
_U16P = ctypes.POINTER(ctypes.c_uint16)
_U32P = ctypes.POINTER(ctypes.c_uint32)
MODES = {"slices": 0, "shards": 1}

_A2A = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)
_ARED = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int)


class _Collectives(ctypes.Structure):
    """include/safe_gossip.h gs_net_collectives."""
    _fields_ = [("ctx", ctypes.c_void_p), ("alltoall", _A2A), ("allreduce", _ARED), ("allgather", _A2A)]


def _host_bytes(ptr: int, n: int) -> np.ndarray:
    return np.ctypeslib.as_array((ctypes.c_uint8 * max(n, 1)).from_address(ptr))[:n]


def _group_collectives(group, world: int):
    """gs_net_collectives over a torch.distributed group, on CPU tensors (any
    backend that takes CPU tensors: gloo).  Exceptions become a nonzero
    status (GS_ERR_IO in the library)."""
    import torch
    import torch.distributed as dist
    dts = {0: (np.uint8, torch.int32), 1: (np.uint32, torch.int64), 2: (np.uint64, torch.int64)}
    ops = {0: dist.ReduceOp.SUM, 1: dist.ReduceOp.MIN, 2: dist.ReduceOp.MAX}

    def alltoall(_ctx, send, recv, nb):
        try:
            inp = torch.from_numpy(_host_bytes(send, nb * world).copy())
            out = torch.empty(nb * world, dtype=torch.uint8)
            dist.all_to_all_single(out, inp, group=group)
            _host_bytes(recv, nb * world)[:] = out.numpy()
            return 0
        except Exception:  # noqa: BLE001 -- reported as a status
            return 1

    def allreduce(_ctx, buf, count, dtype, op):
        try:
            npt, tt = dts[dtype]
            view = np.ctypeslib.as_array((ctypes.c_uint8 * max(count * np.dtype(npt).itemsize, 1))
                                         .from_address(buf)).view(npt)[:count]
            t = torch.from_numpy(view.astype(np.int64)).to(tt)
            dist.all_reduce(t, op=ops[op], group=group)
            view[:] = t.numpy().astype(npt)
            return 0
        except Exception:  # noqa: BLE001
            return 1

    def allgather(_ctx, send, recv, nb):
        try:
            inp = torch.from_numpy(_host_bytes(send, nb).copy())
            outs = [torch.empty(nb, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(outs, inp, group=group)
            _host_bytes(recv, nb * world)[:] = torch.cat(outs).numpy()
            return 0
        except Exception:  # noqa: BLE001
            return 1
    fns = (_A2A(alltoall), _ARED(allreduce), _A2A(allgather))
    return _Collectives(None, *fns), fns


class Net:
    """``n_nodes`` gossipers with ``n_rumors`` rumor slots over ``world``
    ranks, as rumor slices (``mode="slices"``) or node shards
    (``mode="shards"``).  Mirrors :class:`safe_gossip_amd.Network`'s round and
    observer calls; with ``transport="dist"`` every rank makes the same calls
    (observers are collective and return the whole network)."""

    def __init__(self, n_nodes: int, n_rumors: int, world: int, mode: str = "shards", seed: int = 0x5AFE6055,
                 epoch: int = 0, params=None, device: int = 0, transport: str = "local", group=None,
                 parts: int = 4, churn: float = 0.0, drop_push: float = 0.0, drop_pull: float = 0.0,
                 schedule: str = "2P"):
        self.lib = load_library()
        self.n, self.R, self.world, self.seed, self.epoch = n_nodes, n_rumors, world, seed, epoch
        self.mode, self.transport, self.device = mode, transport, device
        cfg = _Config()
        cfg.n_nodes, cfg.n_rumors, cfg.seed, cfg.epoch = n_nodes, n_rumors, seed, epoch
        if params is not None:
            cfg.counter_max, cfg.max_c_rounds, cfg.max_rounds = params
        cfg.schedule = 1 if schedule == "SEQ" else 0
        cfg.device = device
        cfg.churn, cfg.drop_push, cfg.drop_pull = (fault_threshold(churn), fault_threshold(drop_push),
                                                   fault_threshold(drop_pull))
        h = ctypes.c_void_p()
        if transport == "local":
            _check(self.lib.gs_net_create_local(ctypes.byref(cfg), MODES[mode], world, parts, ctypes.byref(h)))
        elif transport == "dist":
            import torch.distributed as dist
            rank = dist.get_rank(group)
            assert dist.get_world_size(group) == world
            ident = (ctypes.c_uint8 * 128)()
            if rank == 0:
                _check(self.lib.gs_net_unique_id(ident))
            box = [bytes(ident)]
            dist.broadcast_object_list(box, src=0, group=group)
            ident = (ctypes.c_uint8 * 128).from_buffer_copy(box[0])
            _check(self.lib.gs_net_create(ctypes.byref(cfg), MODES[mode], rank, world, parts, ident,
                                          ctypes.byref(h)))
        elif transport == "host":
            import torch.distributed as dist
            rank = dist.get_rank(group)
            assert dist.get_world_size(group) == world
            # (the callbacks must outlive the network: kept on self)
            self._coll, self._fns = _group_collectives(group, world)
            _check(self.lib.gs_net_create_with(ctypes.byref(cfg), MODES[mode], rank, world, parts,
                                               ctypes.byref(self._coll), ctypes.byref(h)))
        else:
            raise ValueError(transport)
        self.h = h
        self.round = 0

    def close(self):
        if getattr(self, "h", None):
            self.lib.gs_net_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ protocol
    def _engine(self, i: int = 0):
        return self.lib.gs_net_engine(self.h, i)

    @property
    def params(self):
        out = (ctypes.c_uint8 * 3)()
        _check(self.lib.gs_get_params(self._engine(), out))
        return tuple(out)

    @property
    def parts(self):
        if self.mode != "shards":
            return 1
        info = (ctypes.c_uint32 * 14)()
        _check(self.lib.gs_shard_info(self._engine(), info))
        return int(info[8])

    def send_new(self, node: int, rumor: int) -> None:
        if self.n < 2:
            raise NoPeers("There are no connected peers with which to gossip.")
        _check(self.lib.gs_net_send_new(self.h, node, rumor))

    def next_round(self, report: bool = True) -> Optional[RoundReport]:
        if report:
            r = _Report()
            _check(self.lib.gs_net_next_round(self.h, ctypes.byref(r)))
            self.round = r.round
            return RoundReport(r.round, bool(r.any_live))
        _check(self.lib.gs_net_next_round(self.h, None))
        self.round += 1
        return None

    def clear(self, epoch: Optional[int] = None) -> None:
        self.epoch = self.epoch + 1 if epoch is None else epoch
        _check(self.lib.gs_net_clear(self.h, self.epoch))
        self.round = 0

    def sync(self) -> None:
        _check(self.lib.gs_net_sync(self.h))

    # ------------------------------------------------------------ observers
    def known_counts(self):
        t, c = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self.lib.gs_net_known_counts(self.h, ctypes.byref(t), ctypes.byref(c)))
        return int(t.value), int(c.value)

    def statistics_all(self) -> np.ndarray:
        out = np.zeros((self.n, 5), dtype=np.uint64)
        _check(self.lib.gs_net_statistics_all(self.h, out.ctypes.data_as(_U64P)))
        return out

    def dump_state(self) -> np.ndarray:
        out = np.zeros((self.n, self.R), dtype=np.uint16)
        _check(self.lib.gs_net_dump_state(self.h, out.ctypes.data_as(_U16P)))
        return out

    # measurement hooks (this process's first engine)
    def set_timing(self, on: bool) -> None:
        for i in range(self.lib.gs_net_local_engines(self.h)):
            self.lib.gs_set_timing(self._engine(i), 1 if on else 0)

    def round_kernel_times(self, max_n: int = 4096) -> np.ndarray:
        buf = (ctypes.c_float * max_n)()
        k = self.lib.gs_round_kernel_times(self._engine(), buf, max_n)
        if k < 0:
            _check(-3)
        return np.array(buf[:k], dtype=np.float64)

    def round_kernel_bytes(self) -> float:
        return float(self.lib.gs_round_kernel_bytes(self._engine()))

    def round_kernel_name(self) -> str:
        return self.lib.gs_round_kernel_name(self._engine()).decode()

    def round_traffic(self):
        b, n = ctypes.c_double(), ctypes.c_uint32()
        _check(self.lib.gs_round_traffic(self._engine(), ctypes.byref(b), ctypes.byref(n)))
        return float(b.value), int(n.value)
