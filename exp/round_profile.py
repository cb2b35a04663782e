"""Per-round profile of the bench workload (experiment): round-kernel time,
fraction of node-words (64 rumors) that are all-A (unknown), known pairs."""
import sys, time, json, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import safe_gossip_amd as sg
sys.path.insert(0, ".")
import bench

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
R = int(sys.argv[2]) if len(sys.argv) > 2 else 256
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 30
net = sg.Network(n, R, seed=0x5AFE6055)
bench.inject_all(net, 0)
net.set_timing(True)
for t in range(rounds):
    net.next_round(report=False)
net.sync()
kt = net.round_kernel_times()
net.set_timing(False)
net.clear(1)
bench.inject_all(net, 1)
rows = []
for t in range(rounds):
    rep = net.next_round()
    K = net.known_all()
    zero = float(np.mean(K == 0))
    full = float(np.mean(K == np.uint64(0xFFFFFFFFFFFFFFFF)))
    tot, comp = net.known_counts()
    rows.append(dict(round=t + 1, kernel_ms=float(kt[t]), words_all_unknown=zero, words_all_known=full,
                     known_frac=tot / (n * R), any_live=rep.any_live))
    print(json.dumps(rows[-1]), flush=True)
