"""Per-kernel profile of the sharded engine: `world` shards on one GPU, local
(device-copy) transport, config 4 sizes (or config 5 with `cfg5` as the 4th
argument: 10^8 x 16, 1 % faults).  Run under rocprofv3 --kernel-trace."""
import sys
import time

import os
sys.path.insert(0, os.environ.get("GS_TREE") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import safe_gossip_amd as sg  # noqa: E402
from safe_gossip_amd.sharded import ShardedNetwork  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10   # timed rounds
W0 = int(sys.argv[3]) if len(sys.argv) > 3 else 3   # rounds before them
cfg5 = len(sys.argv) > 4 and sys.argv[4] == "cfg5"
n, R = (100_000_000, 16) if cfg5 else (1 << 24, 256)
fk = dict(churn=0.01, drop_push=0.01, drop_pull=0.01) if cfg5 else {}
torch.cuda.set_device(0)
net = ShardedNetwork(n, R, world, transport="local", parts=int(os.environ.get("PARTS", "1")), **fk)
for r in range(R):
    x = sg.origin_of(net.seed, 0, r, n)
    net.send_new(x, r)
for _ in range(W0):
    net.next_round(report=False)
net.sync()
t0 = time.perf_counter()
for _ in range(K):
    net.next_round(report=False)
net.sync()
print("world", world, "ms/round", (time.perf_counter() - t0) / K * 1e3)
net.close()
