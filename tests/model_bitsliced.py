"""Pure-Python model of the round kernel's bit-sliced algebra (test only).

Mirrors safe_gossip_amd/csrc/gs_kernels.hip formula by formula, with Python
integers as R-bit rumor sets, so the 2P derivation (creation by the first
carrier, records, z-dedupe, pull rows built from pushers ahead of x, median
rule as 2*ge > |P|, C/D transitions, statistics) can be checked against the
oracle on CPU independently of HIP.  Small sizes only.

Harness-injected faults follow the kernel too: delivery flags per edge
(dead push / dropped pull / offline), frozen pre-transition planes plus the
two votes (bump, anyC) of offline nodes, and a per-node offline count.
"""

OFF, DEAD, NOPULL = 1, 2, 4


def popc(v):
    return bin(v).count("1")


class Model:
    def __init__(self, n, R, seed, epoch, params, peer_fn, fault_fn=None, schedule=0):
        self.n, self.R, self.seed, self.epoch = n, R, seed, epoch
        self.cmax, self.maxc, self.maxr = params
        self.M = (1 << R) - 1
        self.P = [[0] * 8 for _ in range(n)]     # isC, a0, a1, b0..b4
        self.stats = [[0] * 5 for _ in range(n)]
        self.tg = [0] * n
        self.src = [[] for _ in range(n)]        # in-edges, ascending
        self.round = 0
        self.pending = []
        self.peer_fn = peer_fn
        self.fault_fn = fault_fn                 # (round, node) -> or_fault bits, or None
        self.fl = [0] * n                        # delivery flags of the round (OFF/DEAD/NOPULL)
        self.pend = [(0, 0)] * n                 # frozen votes (bump, anyC)
        self.deliver_pending = False
        self.schedule = schedule                 # 0 = 2P, 1 = SEQ
        self.W = None                            # SEQ: pull batch of every node

    def offline(self, rnd, x):
        return bool(self.fault_fn and self.fault_fn(rnd, x) & 1)

    def send_new(self, x, r):
        self.pending.append((x, r))

    @staticmethod
    def add5(c, v):
        for i in range(5):
            t = c[i] & v
            c[i] ^= v
            v = t

    def ge_k(self, x, nb, K):
        if K >= (1 << nb):
            return 0
        M = self.M
        gt, eq = 0, M
        for i in range(nb - 1, -1, -1):
            ki = M if (K >> i) & 1 else 0
            gt |= eq & x[i] & ~ki & M
            eq &= ~(x[i] ^ ki) & M
        return (gt | eq) & M

    def cls(self, s):
        p = self.P[s]
        return p[0], p[1], p[2]

    def pull_row(self, z, x, pushers):
        """Pull batch z returns to pusher x (src/gossip.rs:124-151) as the
        shard exchange's 2-plane class code (b0, b1): 01 counter 1, 10 counter
        2, 11 counter 255 (C).  `pushers` = (source, class) of z's in-edges."""
        M = self.M
        zc, z0, z1 = self.cls(z)
        zA = ~zc & ~z0 & ~z1 & M
        zB = ~zc & (z0 | z1) & M
        zC = zc & ~(z0 & z1) & M
        pB = pC = 0
        pnot = zA
        for s, (qc, q0, q1) in pushers:
            if not pnot or s >= x:
                break
            vC = qc & ~(q0 & q1) & M
            sl = (~qc & (q0 | q1) & M) | vC
            nc = pnot & sl
            pB |= nc & ~vC & M
            pC |= nc & vC
            pnot &= ~sl & M
        pcl = zC | pC
        return (zB & z0 & ~z1 & M) | pB | pcl, (zB & z1 & ~z0 & M) | pcl

    # ------------------------------------------------------------------ SEQ
    # The literal harness order (src/gossiper.rs:217-234): pair (x, t(x)) at
    # "time" x; t(x) answers x's push with its CURRENT live set (before
    # absorbing the push), which x absorbs at once.  So the pull x receives,
    # W(x) = S(z) + what z created before time x, depends on W(z) when z < x:
    # dependencies point to smaller ids, so ascending order (the engine: levels
    # of the chain x -> t(x) -> ... while ids decrease) resolves them.
    def got0(self, y):
        return not self.fl[y] & NOPULL

    def got(self, y):
        """y receives a pull at time y: its push was delivered and answered
        (t(y) had not heard from y already: the mutual pair processed second
        gets none, src/gossip.rs:125-126) and the pull was not dropped."""
        if not self.got0(y):
            return False
        z = self.tg[y]
        return not (self.tg[z] == y and z < y and self.got0(z))

    def seq_pulls(self):
        M = self.M
        W = [None] * self.n
        for y in range(self.n):
            if not self.got(y):
                continue
            z = self.tg[y]
            zc, z0, z1 = self.cls(z)
            notyet = ~zc & ~z0 & ~z1 & M
            zB = ~zc & (z0 | z1) & M
            zC = zc & ~(z0 & z1) & M
            cB = cC = 0
            ev = [(s, 0) for s in self.src[z] if s < y]
            if z < y and self.got(z):
                ev.append((z, 1))
            for t_, kind in sorted(ev):
                if kind == 0:
                    qc, q0, q1 = self.cls(t_)
                    vC = qc & ~(q0 & q1) & M
                    sl = (~qc & (q0 | q1) & M) | vC
                else:
                    b0, b1 = W[z]
                    vC = b0 & b1
                    sl = (b0 | b1) & M
                nc = notyet & sl
                cB |= nc & ~vC & M
                cC |= nc & vC
                notyet &= ~sl & M
            W[y] = ((zB & z0 & ~z1 & M) | cB | zC | cC, (zB & z1 & ~z0 & M) | zC | cC)
        self.W = W

    def deliver_seq(self, x):
        M = self.M
        isC, a0, a1 = self.cls(x)
        A = ~isC & ~a0 & ~a1 & M
        B = ~isC & (a0 | a1) & M
        C = isC & ~(a0 & a1) & M
        lc = popc(B | C)
        z = self.tg[x]
        gx = self.got(x)
        ins = self.src[x]
        zin = z in ins
        ev = [(s, 0) for s in ins] + ([(x, 1)] if gx else [])
        crB = crC = anyC = 0
        c1, c2 = [0] * 5, [0] * 5
        notyet = A
        recv = full = empty = created = 0
        for t_, kind in sorted(ev):
            rec_mask = M
            if kind == 0:
                s = t_
                if not (s == z and x < z and gx):      # x answers s's push
                    if lc + created:
                        full += lc + created
                    else:
                        empty += 1
                qc, q0, q1 = self.cls(s)
                vC = qc & ~(q0 & q1) & M
                vB = ~qc & (q0 | q1) & M
                v2 = vB & q1 & ~q0 & M
                rec_on = not (s == z and gx and z < x)  # superseded by the later pull
            else:
                b0, b1 = self.W[x]
                vC = b0 & b1
                vB = (b0 ^ b1) & M
                v2 = b1 & ~b0 & M
                rec_on = True
                if zin and z > x:  # z's later push overwrites the rumors it carries
                    qc, q0, q1 = self.cls(z)
                    rec_mask = ~((~qc & (q0 | q1)) | (qc & ~(q0 & q1))) & M
            sl = vB | vC
            newc = notyet & sl
            if rec_on:
                rec = (B | crB) & sl & rec_mask
                anyC |= rec & vC
                self.add5(c1, rec & vB)
                self.add5(c2, rec & v2)
            crB |= newc & ~vC & M
            crC |= newc & vC
            notyet &= ~sl & M
            created += popc(newc)
            recv += popc(sl)
        psize = len(ins) + (1 if gx and not zin else 0)
        return dict(crB=crB, crC=crC, anyC=anyC, c1=c1, c2=c2, psize=psize, d_full=full,
                    d_empty_pull=empty, d_recv=recv)

    def deliver(self, x):
        """Phases 1+2 of round t at x: returns the kernel's per-lane values."""
        if self.schedule == 1:
            if self.W is None:
                self.seq_pulls()
            return self.deliver_seq(x)
        z = self.tg[x]
        ins = [(s, self.cls(s)) for s in self.src[x]]
        pulled = not self.fl[x] & NOPULL
        pull = self.pull_row(z, x, [(s, self.cls(s)) for s in self.src[z]]) if pulled else (0, 0)
        return self.deliver_rows(x, z, ins, pull, pulled)

    def deliver_rows(self, x, z, ins, pull, pulled=True):
        """`ins` = (source, class planes) of x's pushers ascending; `pull` = the
        (b0, b1) code of the pull batch t(x) returned to x (none: not pulled)."""
        M = self.M
        isC, a0, a1 = self.cls(x)
        A = ~isC & ~a0 & ~a1 & M
        B = ~isC & (a0 | a1) & M
        C = isC & ~(a0 & a1) & M
        liveX = B | C
        crB = crC = anyC = 0
        c1 = [0] * 5
        c2 = [0] * 5
        k = len(ins)
        notyet = A
        zin = False
        part_cw = 0
        first = None
        recv = 0
        for i, (s, (qc, q0, q1)) in enumerate(ins):
            vC = qc & ~(q0 & q1) & M
            vB = ~qc & (q0 | q1) & M
            v2 = vB & q1 & ~q0 & M
            sl = vB | vC
            newc = notyet & sl
            zin |= s == z
            if not (pulled and s == z):  # t(x)'s push copy is superseded by its pull copy
                rec = (B | crB) & sl
                anyC |= rec & vC
                self.add5(c1, rec & vB)
                self.add5(c2, rec & v2)
            crB |= newc & ~vC & M
            crC |= newc & vC
            notyet &= ~sl & M
            pc = popc(newc)
            part_cw += (k - 1 - i) * pc
            if pc and first is None:
                first = i
            recv += popc(sl)
        b0, b1 = pull
        pv2 = b1 & ~b0 & M
        pvB = (b0 ^ b1) & M
        pCl = b0 & b1
        pl = pvB | pCl
        newc = notyet & pl
        rec = (B | crB) & pl
        anyC |= rec & pCl
        self.add5(c1, rec & pvB)
        self.add5(c2, rec & pv2)
        crB |= newc & ~pCl & M
        crC |= newc & pCl
        recv += popc(pl)
        psize = k + (1 if pulled and not zin else 0)
        lc = popc(liveX)
        d_full = k * lc + part_cw
        d_empty_pull = 0
        if k > 0 and lc == 0:
            d_empty_pull = k if first is None else first + 1
        return dict(crB=crB, crC=crC, anyC=anyC, c1=c1, c2=c2, psize=psize, d_full=d_full,
                    d_empty_pull=d_empty_pull, d_recv=recv)

    def transition(self, x, d, inj, off_t=False, on_next=True):
        M = self.M
        p = self.P[x]
        isC, a0, a1 = p[0], p[1], p[2]
        b = p[3:8]
        A = ~isC & ~a0 & ~a1 & M
        B = ~isC & (a0 | a1) & M
        C = isC & ~(a0 & a1) & M
        D = isC & a0 & a1 & M
        crB, crC, anyC, c1, c2, psize = d["crB"], d["crC"], d["anyC"], d["c1"], d["c2"], d["psize"]
        ninj = ~inj & M
        Bold, Cold, Dold = B & ninj, C & ninj, D & ninj
        cB, cC = crB & ninj, crC & ninj
        Bf = Bold | cB | inj
        Cf = Cold | cC
        oc1 = (Bold & a0 & ~a1 & M) | cB | inj
        oc2 = Bold & a1 & ~a0 & M
        thr = psize // 2 + 1
        if off_t:   # returning from offline: the votes frozen with the state
            bump = self.pend[x][0] & Bold
            anyCe = self.pend[x][1] & ninj
        else:
            bump = ((oc1 & self.ge_k(c1, 5, thr)) | (oc2 & self.ge_k(c2, 5, thr))) & ninj
            anyCe = anyC & ninj
        nr = [0] * 6
        carry = M
        for i in range(5):
            rb = b[i] & Bold
            nr[i] = (rb ^ carry) & M
            carry &= rb
        nr[5] = carry
        toD = self.ge_k(nr, 6, self.maxr)
        oc1n = oc1 & ~bump & M
        oc2n = (oc1 & bump) | (oc2 & ~bump & M)
        oc3n = oc2 & bump
        if self.cmax <= 1:
            ocge = M
        elif self.cmax == 2:
            ocge = oc2n | oc3n
        else:
            ocge = oc3n
        toC = anyCe | ocge
        BD = Bf & toD
        BC = Bf & ~toD & toC & M
        BB = Bf & ~toD & ~toC & M
        cr0, cr1 = a0 & Cold, a1 & Cold
        dd = [~cr0 & M, cr1 ^ cr0, cr1 & cr0]
        rib = [b[i] & Cold for i in range(5)]
        s = [0] * 6
        c = 0
        for i in range(5):
            di = dd[i] if i < 3 else 0
            s[i] = rib[i] ^ di ^ c
            c = (rib[i] & di) | (c & (rib[i] ^ di))
        s[5] = c
        CtoD = self.ge_k(s, 6, self.maxr) | self.ge_k(dd, 3, self.maxc)
        CD = Cf & CtoD
        CC = Cf & ~CtoD & M
        Dn = BD | CD | Dold
        Cn = BC | CC
        Bn = BB
        N = [0] * 8
        N[0] = Cn | Dn
        N[1] = (Bn & oc1n) | (CC & dd[0]) | Dn
        N[2] = (Bn & oc2n) | (CC & dd[1]) | Dn
        for i in range(5):
            N[3 + i] = ((Bn | BC) & nr[i]) | (CC & rib[i])
        if not on_next:  # offline next round: pre-transition planes + votes
            N = [(isC & ninj) | cC, (a0 & ninj) | cB | inj, a1 & ninj] + [v & ninj for v in b]
            self.pend[x] = (bump, anyCe & (Bold | cB))
            return [v & M for v in N], 0
        return [v & M for v in N], popc(Bn | Cn)

    def next_round(self):
        n = self.n
        rnd = self.round + 1
        inj = [0] * n
        for x, r in self.pending:
            inj[x] |= 1 << r
        self.pending = []
        dl = [None] * n
        zero = dict(crB=0, crC=0, anyC=0, c1=[0] * 5, c2=[0] * 5, psize=0, d_full=0,
                    d_empty_pull=0, d_recv=0)
        for x in range(n):
            dl[x] = self.deliver(x) if self.deliver_pending else zero
        newP = [None] * n
        live_any = False
        for x in range(n):
            off_t = self.deliver_pending and bool(self.fl[x] & OFF)
            on_next = not self.offline(rnd, x)
            N, live = self.transition(x, dl[x], inj[x], off_t, on_next)
            newP[x] = N
            st = self.stats[x]
            st[0] += 1 if on_next else 0
            st[1] += dl[x]["d_empty_pull"]
            st[4] += dl[x]["d_recv"]
            st[2] += 1 if on_next and live == 0 else 0
            st[3] += live + dl[x]["d_full"]
            live_any |= live > 0
        self.P = newP
        self.round = rnd
        self.W = None
        self.plan_round(rnd)
        self.deliver_pending = True
        return live_any

    def plan_round(self, rnd):
        """Targets, delivery flags and in-lists of round `rnd` (the in-list build)."""
        n = self.n
        self.tg = [self.peer_fn(self.seed, self.epoch, rnd, x, n) for x in range(n)]
        self.fl = [0] * n
        if self.fault_fn:
            fb = [self.fault_fn(rnd, x) for x in range(n)]
            for x in range(n):
                if fb[x] & 1:
                    self.fl[x] = OFF | DEAD | NOPULL
                elif fb[x] & 2 or fb[self.tg[x]] & 1:
                    self.fl[x] = DEAD | NOPULL
                elif fb[x] & 4:
                    self.fl[x] = NOPULL
        self.src = [[] for _ in range(n)]
        for x in range(n):
            if not self.fl[x] & DEAD:
                self.src[self.tg[x]].append(x)

    def observe(self):
        """(state codes, records, psize, stats, known) after deliveries."""
        n, R, M = self.n, self.R, self.M
        codes = [[0] * R for _ in range(n)]
        recs = [[0] * R for _ in range(n)]
        psz = [0] * n
        stats = []
        known = []
        for x in range(n):
            p = self.P[x]
            isC, a0, a1 = p[0], p[1], p[2]
            A = ~isC & ~a0 & ~a1 & M
            B = ~isC & (a0 | a1) & M
            C = isC & ~(a0 & a1) & M
            D = isC & a0 & a1 & M
            d = self.deliver(x) if self.deliver_pending else dict(
                crB=0, crC=0, anyC=0, c1=[0] * 5, c2=[0] * 5, psize=0, d_full=0,
                d_empty_pull=0, d_recv=0)
            psz[x] = d["psize"]
            st = list(self.stats[x])
            st[1] += d["d_empty_pull"]
            st[3] += d["d_full"]
            st[4] += d["d_recv"]
            stats.append(st)
            known.append((~A | d["crB"] | d["crC"]) & M)
            for r in range(R):
                bit = 1 << r
                bf = sum(((p[3 + i] >> r) & 1) << i for i in range(5))
                af = ((a0 >> r) & 1) | (((a1 >> r) & 1) << 1)
                if d["crB"] & bit:
                    code = (1 << 14) | (1 << 7)
                elif d["crC"] & bit:
                    code = 2 << 14
                elif B & bit:
                    code = (1 << 14) | (af << 7) | bf
                elif C & bit:
                    code = (2 << 14) | (af << 7) | bf
                elif D & bit:
                    code = 3 << 14
                else:
                    code = 0
                codes[x][r] = code
                if (B | d["crB"]) & bit:
                    v1 = sum(((d["c1"][i] >> r) & 1) << i for i in range(5))
                    v2 = sum(((d["c2"][i] >> r) & 1) << i for i in range(5))
                    recs[x][r] = (((d["anyC"] >> r) & 1) << 15) | (v2 << 7) | v1
        return codes, recs, psz, stats, known
