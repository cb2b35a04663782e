"""Single-rank sharded engine (RCCL or gloo) at growing n: progress printed
per phase, to find where a full-size run stalls."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
import torch
import torch.distributed as dist
backend = sys.argv[1]
parts = int(sys.argv[2])
R = int(sys.argv[3])
torch.cuda.set_device(0)
dist.init_process_group(backend, rank=0, world_size=1)
import safe_gossip_amd as sg
from safe_gossip_amd.sharded import ShardedNetwork
for lg in [int(v) for v in sys.argv[4:]]:
    n = 1 << lg
    t0 = time.time()
    net = ShardedNetwork(n, R, 1, transport="dist", parts=parts)
    print(f"n=2^{lg} created {time.time()-t0:.1f}s", flush=True)
    for r in range(R):
        net.send_new(sg.origin_of(net.seed, 0, r, n), r)
    for rnd in range(4):
        t1 = time.time()
        net.next_round(report=False)
        print(f"  round {rnd} issued {time.time()-t1:.2f}s", flush=True)
        net.sync()
        torch.cuda.synchronize()
        print(f"  round {rnd} done {time.time()-t1:.2f}s", flush=True)
    print(f"  known {net.known_counts()}", flush=True)
    net.close()
dist.destroy_process_group()
