"""Rumor-sliced network: the rumor space split across ranks.

Every rank holds ALL ``n`` nodes and a slice of the rumors, ``[lo_g, lo_g +
R_g)`` with ``lo_g = g * R // world``, as a plain single-GPU engine of ``R_g``
rumor slots (``gs_config.rumor_slice = 1``; same seed, epoch and parameters on
every rank, so every rank draws the same Philox peer schedule and faults).

Why the slices exchange no state: a ``MessageState`` only ever sees copies of
its own rumor (``src/message_state.rs:73-84``, ``src/gossip.rs:153-163``), and
``peers_in_this_round`` counts RPCs (``src/gossip.rs:125``), which every node
sends whether its batch is empty or not (``src/gossip.rs:105-111``, the empty
Push; ``:143-148``, the empty Pull).  So rumor r's trajectory is the same
whichever other rumors the network carries.  The only coupling is in the
Statistics: a node's push is *empty* only when it is empty in every slice, and
the number of empty pulls a node sends (its answered pushers up to the first
one that creates an entry, none if it has a live entry) is a nondecreasing
function of that first creation, so the network's count is the MIN over the
slices of each slice's count.  Per round each engine writes these two counts
(2 bytes per node) instead of adding them to its Statistics; one
``all_reduce(MIN)`` over the ranks, and the next round kernel adds the
network's counts back (``gs_slice_defer``).  ``full_message_sent`` / ``full_message_received`` count messages
and are summed over the slices when observed.

Transports:

* ``"dist"``  -- one slice per process, ``torch.distributed`` (``nccl`` =
  RCCL over xGMI: the all-reduce of round t runs on the process group's stream
  while the engine runs round t+1, and round t+2's kernel adds it to the
  Statistics; ``gloo``: host-staged, synchronous).
* ``"local"`` -- all slices in this process on one device (tests).

PyTorch is plumbing here (device buffers, streams, collectives); all protocol
work runs in the engine's gfx950 kernels.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np

from . import (_U64P, GossipError, Network, NoPeers, RoundReport, Statistics, _check, default_rumor_key,
               rpc_decode, rpc_encode)


def merge_known(per, bounds, n: int, kw: int) -> np.ndarray:
    """Known-rumor words of the network (n x kw) from each slice's words
    (slice g: rumors [bounds[g], bounds[g+1]) as its bits 0..), each word
    shifted to its rumor offset -- no per-bit expansion."""
    out = np.zeros((n, kw), dtype=np.uint64)
    for k, lo in zip(per, bounds[:-1]):
        sh = np.uint64(lo % 64)
        for w in range(k.shape[1]):
            j = lo // 64 + w
            out[:, j] |= k[:, w] << sh
            if sh and j + 1 < kw:
                out[:, j + 1] |= k[:, w] >> (np.uint64(64) - sh)
    return out


def merge_answers(per_slice: List[List[bytes]]) -> List[bytes]:
    """One RPC's answers from every slice (frames of bincode GossipRpc): the
    non-empty frames in key order (the BTreeMap order a single Gossip
    iterates, src/gossip.rs:126-148), one empty frame if every slice
    answered empty, none if no slice answered."""
    frames = [f for fs in per_slice for f in fs]
    if not frames:
        return []
    full = []
    for f in frames:
        _, m, ctr = rpc_decode(f)
        if m or ctr:
            full.append((m, f))
    if not full:
        return [frames[0]]
    full.sort(key=lambda kv: kv[0])
    return [f for _, f in full]


def slice_ext_limit(n_rumors: int, world: int) -> int:
    """The network's bound on external first Pushes answered per node and
    round: min(200, 32 R_pad) of its smallest slice (gs_engine.cpp)."""
    r = n_rumors // world
    return min(200, 32 * (1 << (r - 1).bit_length()))


class _Slice:
    """One rank's engine (rumors [lo, hi)) and its empty-count buffers."""

    def __init__(self, torch, n, lo, hi, seed, epoch, params, device, faults, schedule="2P"):
        self.lo, self.hi = lo, hi
        self.net = Network(n, hi - lo, seed=seed, epoch=epoch, params=params, device=device,
                           churn=faults[0], drop_push=faults[1], drop_pull=faults[2], schedule=schedule,
                           _rumor_slice=True)
        self.lib, self.h = self.net._lib, self.net._h
        dev = torch.device("cuda", device)
        self.buf = [torch.zeros(2 * n, dtype=torch.uint8, device=dev) for _ in range(3)]
        self.obs = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        _check(self.lib.gs_slice_bind(self.h, *(b.data_ptr() for b in self.buf), self.obs.data_ptr()))
        self.stream = torch.cuda.ExternalStream(self.lib.gs_stream(self.h), device=dev)

    def close(self):
        self.net.close()


class SlicedNetwork:
    """A network of ``n_nodes`` gossipers whose ``n_rumors`` rumor slots are
    sliced over ``world`` ranks.

    Mirrors :class:`safe_gossip_amd.Network`: ``send_new``, ``next_round``,
    ``statistics_all``, ``statistics_reduce``, ``known_all``, ``known_counts``,
    ``dump_state``, ``dump_records``, ``clear`` and the measurement hooks.
    With ``transport="dist"`` every rank makes the same calls (``send_new`` is
    ignored by ranks that do not hold the rumor) and observers return the whole
    network on every rank.  Both schedules (2P and SEQ: the empty counts are
    the MIN over the slices under either, tests/test_sliced_gloo.py), and the
    wire boundary (``push_batch``, ``handle_received[_batch]``, rumor keys;
    see ``handle_received_batch``).
    """

    def __init__(self, n_nodes: int, n_rumors: int, world: int, seed: int = 0x5AFE6055,
                 epoch: int = 0, params=None, device: int = 0, transport: str = "local",
                 group=None, churn: float = 0.0, drop_push: float = 0.0, drop_pull: float = 0.0,
                 schedule: str = "2P"):
        import torch
        if world < 1 or n_rumors < world:
            raise ValueError(f"{n_rumors} rumors cannot be sliced over {world} ranks")
        self.torch = torch
        self.n, self.R, self.seed, self.epoch = n_nodes, n_rumors, seed, epoch
        self.world, self.transport, self.group, self.device = world, transport, group, device
        self.kw = (n_rumors + 63) // 64
        self.bounds = [g * n_rumors // world for g in range(world + 1)]
        faults = (churn, drop_push, drop_pull)
        if transport == "local":
            ranks = list(range(world))
            self.host_staged = False
        elif transport == "dist":
            import torch.distributed as dist
            self.dist = dist
            assert dist.get_world_size(group) == world
            ranks = [dist.get_rank(group)]
            self.host_staged = dist.get_backend(group) == "gloo"
        else:
            raise ValueError(transport)
        self.rank = ranks[0]
        self.schedule = schedule
        self.slices = [_Slice(torch, n_nodes, self.bounds[g], self.bounds[g + 1], seed, epoch, params,
                              device, faults, schedule) for g in ranks]
        self.faults = self.slices[0].net.faults
        # one bound on external first Pushes per node and round for the whole
        # network: the smallest slice's (floor(R / world) rumors), so every
        # slice refuses the same batches (gs_slice_set_ext_limit)
        self.ext_limit = slice_ext_limit(n_rumors, world)
        for s in self.slices:
            _check(s.lib.gs_slice_set_ext_limit(s.h, self.ext_limit))
        self.round = 0
        self._pend = []  # (async work, buffer) of all-reduces not applied yet (RCCL)
        # wire format: keys set by set_rumor_key (every rank tracks them all);
        # the slices' engines take the network's keys on first use
        self._key_of, self._rumor_of = {}, {}
        self._keys_ready = False

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "slices", []):
            self._flush()
        for s in getattr(self, "slices", []):
            s.close()
        self.slices = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def params(self):
        return self.slices[0].net.params

    @property
    def parts(self):
        return 1

    # ------------------------------------------------------------ protocol
    def send_new(self, node: int, rumor: int) -> None:
        if self.n < 2:
            raise NoPeers("There are no connected peers with which to gossip.")
        if not 0 <= rumor < self.R:
            raise GossipError(f"rumor {rumor} out of range")
        for s in self.slices:
            if s.lo <= rumor < s.hi:
                s.net.send_new(node, rumor - s.lo)

    def _min_local(self, bufs):
        """MIN over the slices of this process (local transport), into each."""
        for s in self.slices:
            _check(s.lib.gs_sync(s.h))
        m = bufs[0].clone()
        for b in bufs[1:]:
            self.torch.minimum(m, b, out=m)
        for b in bufs:
            b.copy_(m)
        self.torch.cuda.synchronize(self.device)

    def _min_dist_sync(self, t):
        """MIN over the ranks, synchronously (gloo: through host memory)."""
        s = self.slices[0]
        _check(s.lib.gs_sync(s.h))
        if self.host_staged:
            h = t.cpu()
            self.dist.all_reduce(h, op=self.dist.ReduceOp.MIN, group=self.group)
            t.copy_(h.to(t.device))
        else:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
        self.torch.cuda.synchronize(self.device)

    def _reduce_round(self, b: int):
        """Round t's empty counts (buffer b = t % 3): MIN over the slices, then
        added to every slice's Statistics.  RCCL: asynchronous; one round later
        the engine stream waits for it and round t+2's kernel adds it
        (gs_slice_defer, _apply_pending)."""
        if self.transport == "local":
            self._min_local([s.buf[b] for s in self.slices])
            for s in self.slices:  # added by the next round kernel (or an observer)
                _check(s.lib.gs_slice_defer(s.h, b))
            return
        s = self.slices[0]
        if self.host_staged:
            self._min_dist_sync(s.buf[b])
            _check(s.lib.gs_slice_defer(s.h, b))
            return
        with self.torch.cuda.stream(s.stream):
            w = self.dist.all_reduce(s.buf[b], op=self.dist.ReduceOp.MIN, group=self.group,
                                     async_op=True)
        self._pend.append((w, b))

    def _apply_pending(self, keep: int):
        s = self.slices[0] if self.slices else None
        while len(self._pend) > keep:
            w, b = self._pend.pop(0)
            with self.torch.cuda.stream(s.stream):
                w.wait()  # the engine stream waits, not the host
            if keep:  # folded into the next round kernel (no extra pass)
                _check(s.lib.gs_slice_defer(s.h, b))
            else:
                _check(s.lib.gs_slice_apply(s.h, b))

    def _flush(self):
        self._apply_pending(0)

    def next_round(self, report: bool = True) -> Optional[RoundReport]:
        """Round t on every slice; round t's empty counts all-reduced (RCCL: in
        flight during round t+1) and round t-1's applied."""
        live = False
        for s in self.slices:
            r = s.net.next_round(report=report)
            if r is not None:
                live |= r.any_live
        self.round += 1
        self._reduce_round(self.round % 3)
        self._apply_pending(1)
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
        self._flush()
        for s in self.slices:
            s.net.clear(self.epoch)
        self.round = 0

    def sync(self) -> None:
        self._flush()
        for s in self.slices:
            s.net.sync()

    # ------------------------------------------------------------ wire format
    # The byte boundary of src/gossiper.rs:70-99 on a sliced network.  A
    # rumor's Push / Pull RPC carries one message, held by one slice; but
    # peers_in_this_round and the answers to a first Push are node-level
    # (src/gossip.rs:125-148).  So every slice takes every RPC -- the owner
    # as sent, the others as the empty RPC of the same kind (which counts the
    # peer and asks for the slice's live entries but creates nothing) -- and
    # the answer is the slices' Pull responses merged in key order (one empty
    # Pull if no slice has a live entry).  A slice counts an empty answer
    # into its per-round empty count, so the network's count stays the MIN
    # over the slices (the first slice with a live entry ends the empty run,
    # a nondecreasing function of when that happens, as for the internal
    # pushes); the engine bounds those answers per node and round
    # (gs_engine.cpp slice_ext_limit).
    def _ensure_keys(self):
        """Each slice's engine keys := the network's (rumor lo+r for slot r),
        in descending slot order so no key is ever held twice."""
        if self._keys_ready:
            return
        for s in self.slices:
            if s.lo:
                for r in range(s.hi - s.lo - 1, -1, -1):
                    s.net.set_rumor_key(r, default_rumor_key(s.lo + r))
        self._keys_ready = True

    def rumor_key(self, rumor: int) -> bytes:
        if not 0 <= rumor < self.R:
            _check(-1)
        return self._key_of.get(rumor, default_rumor_key(rumor))

    def _rumor_by_key(self, key: bytes) -> Optional[int]:
        r = self._rumor_of.get(key)
        if r is not None:
            return r
        if len(key) == 12 and key[:8] == default_rumor_key(0)[:8]:
            q = int.from_bytes(key[8:], "big")
            if q < self.R and q not in self._key_of:
                return q
        return None

    def set_rumor_key(self, rumor: int, key: bytes) -> None:
        if not 0 <= rumor < self.R:
            _check(-1)
        held = self._rumor_by_key(key)
        if held is not None:
            if held != rumor:
                _check(-1)  # keys are distinct (gs_set_rumor_key)
            return
        self._ensure_keys()
        for s in self.slices:
            if s.lo <= rumor < s.hi:
                s.net.set_rumor_key(rumor - s.lo, key)
        old = self._key_of.pop(rumor, None)
        if old is not None:
            del self._rumor_of[old]
        self._key_of[rumor] = key
        self._rumor_of[key] = rumor

    def _merge(self, per_slice: List[List[bytes]]) -> List[bytes]:
        return merge_answers(per_slice)

    def _gather_lists(self, mine: List[List[List[bytes]]]) -> List[List[List[bytes]]]:
        """Per slice, per RPC answers of every slice (dist: all-gathered)."""
        if self.transport == "local":
            return mine
        objs = [None] * self.world
        self.dist.all_gather_object(objs, mine[0], group=self.group)
        return objs

    def push_batch(self, node: int) -> List[bytes]:
        """``Gossiper::next_round``'s Push RPCs of ``node`` this round, in key
        order across the slices (one empty Push if none has any)."""
        self._ensure_keys()
        per = self._gather_lists([[s.net.push_batch(node)] for s in self.slices])
        return self._merge([p[0] for p in per])

    def handle_received(self, node: int, peer: int, message: bytes) -> List[bytes]:
        """``Gossiper::handle_received_message(peer, message)`` on ``node``
        for a peer outside the network: the Pull RPCs."""
        return self.handle_received_batch([(node, peer, message)])[0]

    def handle_received_batch(self, rpcs) -> List[List[bytes]]:
        """``handle_received`` for many (node, peer, message) in order: every
        slice takes the whole batch (the owner's RPCs as sent, the others'
        emptied) in one gs_handle_received_batch."""
        rpcs = list(rpcs)
        self._ensure_keys()
        self._flush()
        split = []  # per RPC: (owning rumor or None, the empty RPC of its kind)
        for node, peer, msg in rpcs:
            pull, m, ctr = rpc_decode(msg)  # GossipError on bad bytes (src/gossiper.rs:89-94)
            if not 0 <= node < self.n or peer < self.n:
                _check(-1)
            r = None
            if m or ctr:
                r = self._rumor_by_key(m)
                if r is None:
                    _check(-1)  # no rumor slot for this message
            split.append((r, rpc_encode(pull, b"", 0)))
        mine = []
        for s in self.slices:
            batch = [(node, peer, msg if (r is not None and s.lo <= r < s.hi) else empty)
                     for (node, peer, msg), (r, empty) in zip(rpcs, split)]
            mine.append(s.net.handle_received_batch(batch))
        per = self._gather_lists(mine)
        return [self._merge([p[i] for p in per]) for i in range(len(rpcs))]

    # ------------------------------------------------------------ measurement (this rank's slice)
    def set_timing(self, on: bool) -> None:
        for s in self.slices:
            s.net.set_timing(on)

    def round_kernel_times(self, max_n: int = 4096) -> np.ndarray:
        return self.slices[0].net.round_kernel_times(max_n)

    def round_kernel_bytes(self) -> float:
        return self.slices[0].net.round_kernel_bytes()

    def round_kernel_name(self) -> str:
        return self.slices[0].net.round_kernel_name()

    def round_traffic(self):
        return self.slices[0].net.round_traffic()

    # ------------------------------------------------------------ observers
    def _gather(self, parts: List[np.ndarray]) -> List[np.ndarray]:
        """Per-slice arrays of every slice in rank order (dist: all-gathered)."""
        if self.transport == "local":
            return parts
        objs = [None] * self.world
        self.dist.all_gather_object(objs, parts[0], group=self.group)
        return objs

    def statistics_all(self) -> np.ndarray:
        self._flush()
        per = [s.net.statistics_all() for s in self.slices]
        # pending empty pulls of the last round: MIN over the slices
        if self.transport == "local":
            self._min_local([s.obs for s in self.slices])
        else:
            self._min_dist_sync(self.slices[0].obs)
        pend = self.slices[0].obs[:self.n].cpu().numpy().astype(np.uint64)
        full = [p[:, 3:5] for p in per]
        if self.transport == "dist":
            t = self.torch.from_numpy(full[0].astype(np.int64))
            if not self.host_staged:
                t = t.to(f"cuda:{self.device}")
            self.dist.all_reduce(t, group=self.group)
            full_sum = t.cpu().numpy().astype(np.uint64)
        else:
            full_sum = np.sum(full, axis=0, dtype=np.uint64)
        out = per[0].copy()
        out[:, 1] += pend
        out[:, 3:5] = full_sum
        return out

    def statistics(self, node: int) -> Statistics:
        return Statistics(*(int(v) for v in self.statistics_all()[node]))

    def statistics_reduce(self, op: str = "sum") -> Statistics:
        st = self.statistics_all()
        f = {"sum": lambda a: a.sum(axis=0, dtype=np.uint64), "min": lambda a: a.min(axis=0),
             "max": lambda a: a.max(axis=0)}[op]
        return Statistics(*(int(v) for v in f(st)))

    def dump_state(self) -> np.ndarray:
        self._flush()
        return np.concatenate(self._gather([s.net.dump_state() for s in self.slices]), axis=1)

    def dump_records(self):
        self._flush()
        both = [s.net.dump_records() for s in self.slices]
        recs = self._gather([b[0] for b in both])
        return np.concatenate(recs, axis=1), both[0][1]

    def state_digest(self) -> np.ndarray:
        """Per-node digest of the whole network (what gs_state_digest of one
        engine holding every rumor gives): each slice adds its word sums into
        one device buffer (gs_state_digest_part; dist: an all_reduce SUM),
        then gs_digest_finish mixes them with |P| and the network Statistics."""
        st = self.statistics_all()
        words = self.kw
        s0 = self.slices[0]
        dp = self.torch.zeros(self.n * words, dtype=self.torch.int64, device=f"cuda:{self.device}")
        self.torch.cuda.synchronize(self.device)  # (zeroed on torch's stream; the engines add on theirs)
        for s in self.slices:
            _check(s.lib.gs_state_digest_part(s.h, s.lo, words, dp.data_ptr()))
        if self.transport == "dist":
            if self.host_staged:
                h = dp.cpu()
                self.dist.all_reduce(h, group=self.group)
                dp.copy_(h.to(dp.device))
            else:
                self.dist.all_reduce(dp, group=self.group)
            self.torch.cuda.synchronize(self.device)
        out = np.zeros(self.n, dtype=np.uint64)
        stc = np.ascontiguousarray(st, dtype=np.uint64)
        _check(s0.lib.gs_digest_finish(s0.h, dp.data_ptr(), words, stc.ctypes.data_as(_U64P),
                                       out.ctypes.data_as(_U64P)))
        return out

    def known_all(self) -> np.ndarray:
        self._flush()
        per = self._gather([s.net.known_all() for s in self.slices])
        return merge_known(per, self.bounds, self.n, self.kw)

    def known_counts(self, min_known: Optional[int] = None):
        """(known node-rumor pairs, nodes knowing >= min_known rumors; default R)."""
        self._flush()
        mk = self.R if min_known is None else min_known
        per = [s.net.known_counts() for s in self.slices]
        tot = sum(p[0] for p in per)
        allc = all(p[1] == self.n for p in per)  # every node knows its whole slice
        loc = np.array([tot, 1 if allc else 0], dtype=np.int64)
        if self.transport == "dist":
            t = self.torch.from_numpy(loc.copy())
            if not self.host_staged:
                t = t.to(f"cuda:{self.device}")
            self.dist.all_reduce(t, group=self.group)
            tot, nall = int(t[0].item()), int(t[1].item())
            allc = nall == self.world
        if mk == self.R and allc:
            return tot, self.n
        cnt = [s.net.known_popcounts().astype(np.int64) for s in self.slices]
        if self.transport == "dist":
            t = self.torch.from_numpy(cnt[0])
            if not self.host_staged:
                t = t.to(f"cuda:{self.device}")
            self.dist.all_reduce(t, group=self.group)
            c = t.cpu().numpy()
        else:
            c = np.sum(cnt, axis=0)
        return tot, int((c >= mk).sum())
