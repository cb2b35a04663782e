"""Packed vs one-node-per-lane DLV transition, side by side (debug)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import safe_gossip_amd as sg
from test_gpu_parity import _injections, SEED

n, R, kind = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
faults = tuple(float(v) for v in sys.argv[4:7]) if len(sys.argv) > 4 else (0, 0, 0)
fk = dict(churn=faults[0], drop_push=faults[1], drop_pull=faults[2])
os.environ["SAFE_GOSSIP_AMD_DLV_PACK"] = "1"
a = sg.Network(n, R, seed=SEED, **fk)
os.environ["SAFE_GOSSIP_AMD_DLV_PACK"] = "0"
b = sg.Network(n, R, seed=SEED, **fk)
L = sg.load_library()
thr = [sg.fault_threshold(p) for p in faults]
for rnd in range(1, 12):
    inj = list(_injections(kind, n, R, SEED, 0, rnd, sg))
    for x, r in inj:
        a.send_new(x, r); b.send_new(x, r)
    a.next_round(); b.next_round()
    sa, sb = a.dump_state(), b.dump_state()
    ta, tb = a.statistics_all(), b.statistics_all()
    bad = np.nonzero((sa != sb).any(axis=1) | (ta != tb).any(axis=1))[0]
    print(f"round {rnd}: inj {inj[:6]} differing nodes {len(bad)} {bad[:12].tolist()}", flush=True)
    for x in bad[:6]:
        fl = [L.gs_fault(SEED, 0, rr, int(x), *thr) for rr in (rnd - 1, rnd, rnd + 1)]
        print(f"   node {x}: packed {[hex(v) for v in sa[x][:4]]} {ta[x].tolist()} | per-node {[hex(v) for v in sb[x][:4]]} {tb[x].tolist()} faults(r-1,r,r+1)={fl} peer={L.gs_peer(SEED,0,rnd,int(x),n)}", flush=True)
    if len(bad):
        break
