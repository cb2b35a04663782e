"""Pure-Python model of the SHARDED round, test only.

Each rank owns the node range [lo, lo+m) (shard_plan in gs_shard.hip: chunk =
ceil(n/G) rounded up to 256 nodes) and runs, per round, the same two row
exchanges as the engine over a caller-supplied all-to-all of FIXED-SIZE
blocks ``a2a(blocks_per_dest, width) -> blocks_per_source`` (every block holds
``cap`` rows, the engine's capacity; empty slots carry id -1), so no row count
is exchanged or derived from other ranks' schedules:

  A  every owned node x whose push batch is delivered sends (x, isC, a0, a1)
     to owner(t(x)), rows per destination in ascending x, so each rank
     receives its pushers' rows in ascending source order (rank order = node
     order); the receiver recomputes each received source's target from the
     Philox stream (the engine's edge_keys) -- a rank computes the targets of
     its own sources only;
  B  the owner of z answers each received row, in the same order, with the pull
     batch z returned to that pusher (Model.pull_row: z's live set plus the
     entries z created from earlier pushers, as a 2-plane class code); a
     receiver whose pull batch is dropped ignores it.

Pipeline parts (gs_shard_create_parts): the owned range is cut into `parts`
parts of mP nodes and each part's rows move in an all-to-all of their own
(sub-blocks of capP rows); the receiver lists its pushers in (source rank,
part, index) order, which is ascending source order, and B answers part by
part in the same sub-blocks.

Code rows (R_pad <= 16, the engine's ShardPlan::codes): a push row carries
the pusher's push code and a pull row the pull batch's code, one u32 each
(b0 | b1 << 16: 01 counter 1, 10 counter 2, 11 counter 255), and parts are
whole 1024-node blocks; the receiver decodes a code into the class planes the
algebra reads (a C entry as C{round 0}, "none" as A).

Delivery and transition then use Model's bit-sliced algebra on the received
rows only, so a rank never reads another rank's state directly.  Faults follow
Model (flags of every edge derived locally from the Philox stream, like the
engine's plan).  Rumor sets are Python ints (R <= 62 so a plane fits one int64
of the gloo transport).
"""
from model_bitsliced import DEAD, NOPULL, OFF, Model


def shard_range(n, G, g):
    chunk = -(-n // G)
    chunk = -(-chunk // 256) * 256
    lo = min(g * chunk, n)
    return lo, min(lo + chunk, n) - lo, chunk


def part_nodes(n, G, parts, codes=False):
    """Nodes per pipeline part (shard_plan: whole 256-node plan blocks; code
    rows: whole 1024-node blocks)."""
    chunk = shard_range(n, G, 0)[2]
    align = 1024 if codes else 256
    return -(-(-(-chunk // parts)) // align) * align


def uses_codes(R):
    """Code rows at R_pad <= 16 (2P)."""
    return R <= 16


def push_code(qc, q0, q1, M):
    """Class planes -> the u32 push code (b0 | b1 << 16)."""
    vC = qc & ~(q0 & q1) & M
    vB = ~qc & (q0 | q1) & M
    return ((vB & q0 & ~q1) | vC) | (((vB & q1 & ~q0) | vC) << 16)


def decode_code(code):
    """u32 code -> class planes (gs_kernels.hip decode16)."""
    b0, b1 = code & 0xFFFF, code >> 16
    return b0 & b1, b0 & ~b1, b1 & ~b0


def part_count(n, G, parts, codes=False):
    """Parts that hold nodes (shard_plan): whole aligned blocks of mP nodes
    over the rank's chunk, at most `parts`."""
    chunk = shard_range(n, G, 0)[2]
    return max(1, -(-chunk // part_nodes(n, G, parts, codes)))


def shard_cap(n, G, W=1, parts=1, codes=False):
    """Row slots per (source rank, destination rank, part) sub-block (shard_plan)."""
    import math
    chunk = shard_range(n, G, 0)[2]
    mp = part_nodes(n, G, parts, codes)
    mean = mp * chunk / max(1.0, n - 1.0)
    cap = min(float(mp), mean + 16.0 * math.sqrt(mean + 1.0) + 64.0)
    q = max(64, 4 * W)
    return -(-math.ceil(cap) // q) * q


class ShardModel(Model):
    def __init__(self, n, R, seed, epoch, params, peer_fn, rank, world, a2a, fault_fn=None, parts=1):
        super().__init__(n, R, seed, epoch, params, peer_fn, fault_fn)
        assert R <= 62
        self.rank, self.world, self.a2a = rank, world, a2a
        self.lo, self.m, self.chunk = shard_range(n, world, rank)
        self.codes = uses_codes(R)
        self.parts = part_count(n, world, parts, self.codes)
        self.mP = part_nodes(n, world, parts, self.codes)
        self.cap = shard_cap(n, world, parts=parts, codes=self.codes)
        self.tg, self.fl = {}, {}
        self.P = {x: [0] * 8 for x in self.owned()}
        self.stats = {x: [0] * 5 for x in self.owned()}
        self.exchanged = False

    def owned(self):
        return range(self.lo, self.lo + self.m)

    def part(self, h):
        a = min(self.lo + h * self.mP, self.lo + self.m)
        return range(a, min(a + self.mP, self.lo + self.m))

    def owner(self, x):
        return x // self.chunk

    def exchange(self):
        """Exchanges A and B of the current round (needs self.tg of round t)."""
        if self.exchanged or not self.deliver_pending:
            return
        if self.codes:
            return self.exchange_codes()
        G, cap, P = self.world, self.cap, self.parts
        sendA, recvA = [], []  # [part][rank] sub-blocks
        for h in range(P):
            sa = [[] for _ in range(G)]
            for x in self.part(h):
                if not self.fl[x] & DEAD:
                    sa[self.owner(self.tg[x])].append([x] + list(self.cls(x)))
            for blk in sa:
                assert len(blk) <= cap, "block capacity exceeded (the engine flags a device limit)"
                blk.extend([[-1, 0, 0, 0]] * (cap - len(blk)))
            sendA.append(sa)
            recvA.append(self.a2a(sa, 4))
        # pushers in (source rank, part, index) order = ascending source order
        rows = [r for s in range(G) for h in range(P) for r in recvA[h][s] if r[0] >= 0]
        srcs = [r[0] for r in rows]
        assert srcs == sorted(srcs), "receive rows must be in ascending source order"
        # the receiver's own view of each source's target (Philox, edge_keys)
        rnd = self.round
        tgt = {s: self.peer_fn(self.seed, self.epoch, rnd, s, self.n) for s in srcs}
        ins = {z: [] for z in self.owned()}
        for s, qc, q0, q1 in rows:
            assert self.lo <= tgt[s] < self.lo + self.m, "row sent to a rank that does not own its target"
            ins[tgt[s]].append((s, (qc, q0, q1)))
        pull = {}
        for h in range(P):  # B_h answers A_h's rows in the same sub-blocks
            sendB = [[[r[0]] + list(self.pull_row(tgt[r[0]], r[0], ins[tgt[r[0]]]))
                      if r[0] >= 0 else [-1, 0, 0] for r in blk] for blk in recvA[h]]
            recvB = self.a2a(sendB, 3)
            for d in range(G):
                assert [r[0] for r in recvB[d]] == [r[0] for r in sendA[h][d]], "B order = A order"
                for x, b0, b1 in recvB[d]:
                    if x >= 0:
                        pull[x] = (b0, b1)
        self.ins, self.pull = ins, pull
        self.exchanged = True

    def exchange_codes(self):
        """Code rows: an A row is (push code, target local to the receiving
        rank | mutual << 31) -- no source id: the receiver orders a target's
        pushers by slot key (source rank, part, index), which is ascending
        source order, and knows t(z)'s pusher by the mutual bit the sender set
        (t(t(x)) == x); a B row is the pull code, in the same slot."""
        G, cap, P = self.world, self.cap, self.parts
        EMPTY = 0xFFFFFFFF
        sent = []  # [part][rank] -> the sources of the rows, in slot order (the plan's SPOSB)
        recvA = []
        for h in range(P):
            sa = [[] for _ in range(G)]
            xs = [[] for _ in range(G)]
            for x in self.part(h):
                if not self.fl[x] & DEAD:
                    t = self.tg[x]
                    d = self.owner(t)
                    mutual = self.peer_fn(self.seed, self.epoch, self.round, t, self.n) == x
                    sa[d].append([push_code(*self.cls(x), self.M), (t - d * self.chunk) | (mutual << 31)])
                    xs[d].append(x)
            for blk in sa:
                assert len(blk) <= cap, "block capacity exceeded (the engine flags a device limit)"
                blk.extend([[0, EMPTY]] * (cap - len(blk)))
            sent.append(xs)
            recvA.append(self.a2a([[[c, w - (1 << 32) if w >= 1 << 31 else w] for c, w in blk] for blk in sa], 2))
        ins = {z: [] for z in self.owned()}
        tz = {}  # the receiver's t(z), known only through the mutual bit
        for s in range(G):
            for h in range(P):
                for i, (code, w) in enumerate(recvA[h][s]):
                    w &= 0xFFFFFFFF
                    if w == EMPTY:
                        continue
                    z = self.lo + (w & 0x7FFFFFFF)
                    assert self.lo <= z < self.lo + self.m, "row sent to a rank that does not own its target"
                    key = (s * P + h) * cap + i
                    ins[z].append((key, w >> 31, decode_code(code & 0xFFFFFFFF)))
        pull = {}
        for h in range(P):  # B_h answers A_h's rows in the same sub-blocks
            sendB = []
            for s in range(G):
                blk = []
                for i, (code, w) in enumerate(recvA[h][s]):
                    w &= 0xFFFFFFFF
                    if w == EMPTY:
                        blk.append([0, 0])
                        continue
                    z, key = self.lo + (w & 0x7FFFFFFF), (s * P + h) * cap + i
                    b0, b1 = self.pull_row(z, key, [(k, c) for k, _, c in ins[z]])
                    blk.append([0, b0 | (b1 << 16)])
                sendB.append(blk)
            recvB = self.a2a(sendB, 2)
            for d in range(G):
                for x, r in zip(sent[h][d], recvB[d]):
                    pull[x] = (r[1] & 0xFFFF, r[1] >> 16)
        # deliveries see pushers by slot key; t(z)'s pusher carries z's own
        # target as its identity (the engine's zi from the mutual bit)
        self.ins = {z: [(self.tg_of(z) if m else -1 - k, c) for k, m, c in lst] for z, lst in ins.items()}
        self.pull = pull
        self.exchanged = True

    def tg_of(self, z):
        return self.tg[z]

    def deliver(self, x):
        pulled = not self.fl[x] & NOPULL
        return self.deliver_rows(x, self.tg[x], self.ins[x], self.pull[x] if pulled else (0, 0),
                                 pulled)

    def next_round(self):
        """Local part of the round; returns this shard's any-live flag."""
        self.exchange()
        rnd = self.round + 1
        inj = {x: 0 for x in self.owned()}
        for x, r in self.pending:
            inj[x] |= 1 << r
        self.pending = []
        zero = dict(crB=0, crC=0, anyC=0, c1=[0] * 5, c2=[0] * 5, psize=0, d_full=0,
                    d_empty_pull=0, d_recv=0)
        newP = {}
        live_any = False
        for x in self.owned():
            d = self.deliver(x) if self.deliver_pending else zero
            off_t = self.deliver_pending and bool(self.fl[x] & OFF)
            on_next = not self.offline(rnd, x)
            N, live = self.transition(x, d, inj[x], off_t, on_next)
            newP[x] = N
            st = self.stats[x]
            st[0] += 1 if on_next else 0
            st[1] += d["d_empty_pull"]
            st[4] += d["d_recv"]
            st[2] += 1 if on_next and live == 0 else 0
            st[3] += live + d["d_full"]
            live_any |= live > 0
        self.P = newP
        self.round = rnd
        # the plan of round t+1: targets and delivery flags of the OWNED
        # sources only (the engine's plan_count)
        self.plan_round(rnd)
        self.deliver_pending = True
        self.exchanged = False
        return live_any

    def plan_round(self, rnd):
        self.tg, self.fl = {}, {}
        for x in self.owned():
            t = self.peer_fn(self.seed, self.epoch, rnd, x, self.n)
            self.tg[x] = t
            f = 0
            if self.fault_fn:
                fb = self.fault_fn(rnd, x)
                if fb & 1:
                    f = OFF | DEAD | NOPULL
                elif fb & 2 or self.fault_fn(rnd, t) & 1:
                    f = DEAD | NOPULL
                elif fb & 4:
                    f = NOPULL
            self.fl[x] = f

    def observe_local(self):
        """(codes, records, psize, stats, known) rows of the owned nodes."""
        self.exchange()
        out = ([], [], [], [], [])
        for x in self.owned():
            for acc, v in zip(out, _Single(self, x).observe()):
                acc.append(v[0])
        return out


class _Single:
    """View of one owned node through Model.observe."""

    def __init__(self, sm, x):
        self.sm, self.x = sm, x
        self.n, self.R, self.M = 1, sm.R, sm.M
        self.P = [sm.P[x]]
        self.stats = [sm.stats[x]]
        self.deliver_pending = sm.deliver_pending

    def deliver(self, _):
        return self.sm.deliver(self.x)

    def observe(self):
        return Model.observe(self)
