"""usage: rccl_p1.py log2(n) parts R [nccl|gloo]

The formerly stalling shape: one RCCL rank, node
shards with ONE pipeline part at 2^24 x 256, so each exchange is a single
~1.1 GB self all-to-all.  Phase by phase with host syncs first (where does it
stop?), then free-running rounds as the bench drives them."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")  # (tests pass a free port)
import torch
import torch.distributed as dist

lg, parts, R = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
backend = sys.argv[4] if len(sys.argv) > 4 else "nccl"
torch.cuda.set_device(0)
dist.init_process_group(backend, rank=0, world_size=1)
import safe_gossip_amd as sg  # noqa: E402
from safe_gossip_amd.sharded import ShardedNetwork  # noqa: E402

n = 1 << lg
t0 = time.time()
net = ShardedNetwork(n, R, 1, transport="dist", parts=parts)
s = net.shards[0]
print(f"n=2^{lg} R={R} parts={parts}: created in {time.time() - t0:.1f}s; exchange A {s.rowsA * s.wa * 4 / 1e9:.2f} GB, "
      f"B {s.rowsB * s.wa * 4 / 1e9:.2f} GB; engine stream {s.stream}", flush=True)
for r in range(R):
    net.send_new(sg.origin_of(net.seed, 0, r, n), r)


def step(what, fn):
    t = time.time()
    fn()
    print(f"    {what} issued {time.time() - t:.3f}s", flush=True)
    net._sync_all()
    torch.cuda.synchronize()
    print(f"    {what} done {time.time() - t:.3f}s", flush=True)


for rnd in range(3):  # phase by phase
    print(f"  round {rnd}", flush=True)
    if net.round > 0:
        t = net.round
        if t == 1:
            step("exchange A ids (round 1)", lambda: net._pendA.append(net._exchange("A", net.parts - 1, 0)))
        step("wait exchange A", lambda: [net._wait(w) for w in net._pendA])
        net._pendA = []
        step("pull kernel + edges", lambda: sg._check(net.lib.gs_shard_pull(s.h)))
        step("exchange B", lambda: net._pendB.update({h: net._exchange("B", h) for h in range(net.parts)}))
        net._delivered = True
    step("round kernel + exchange A", lambda: net.next_round(report=False))
t = time.time()
for rnd in range(6):  # as the bench drives it
    net.next_round(report=False)
    print(f"  free round {net.round} issued {time.time() - t:.3f}s", flush=True)
net.sync()
torch.cuda.synchronize()
print(f"  free rounds done {time.time() - t:.3f}s; known {net.known_counts()}", flush=True)
st = net.statistics_all()
assert int(st[:, 0].sum()) == net.round * n, "Statistics.rounds"
assert int(st[:, 4].sum()) == int(st[:, 3].sum()), "every full copy sent is received"
assert net.known_counts()[0] > R * 3 ** 6, "the rumors spread"
net.close()
dist.destroy_process_group()
print("ok", flush=True)
