"""A/B of round-kernel time per round (experiment): the bench workload
(cfg4 shape by default), library from SAFE_GOSSIP_AMD_LIB, mode from
SAFE_GOSSIP_AMD_SPARSE.  Prints one JSON line."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import safe_gossip_amd as sg
import bench

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
R = int(sys.argv[2]) if len(sys.argv) > 2 else 256
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 20
tag = sys.argv[4] if len(sys.argv) > 4 else ""
if tag == "head":  # the committed library predates this symbol
    sg.SYMBOLS.pop("gs_round_traffic", None)
net = sg.Network(n, R, seed=0x5AFE6055)
bench.inject_all(net, 0)
for _ in range(3):
    net.next_round(report=False)
net.clear(1)
bench.inject_all(net, 1)
net.set_timing(True)
for _ in range(rounds):
    net.next_round(report=False)
net.sync()
kt = net.round_kernel_times()
print(json.dumps({"tag": tag, "mode": os.environ.get("SAFE_GOSSIP_AMD_SPARSE", "auto"),
                  "sum_ms": float(np.sum(kt[1:])), "ms": [round(float(v), 3) for v in kt]}), flush=True)
