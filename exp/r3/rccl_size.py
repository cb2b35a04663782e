"""One RCCL rank: all_to_all_single of growing sizes around 2^30 bytes on a
side stream, as the shard exchanges issue it (async_op, waited under another
stream), timed and checked (recv == send).  usage: rccl_size.py MB ..."""
import os
import sys
import time

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29547")
import torch
import torch.distributed as dist

torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1)
side = torch.cuda.Stream()
for mb in [float(v) for v in sys.argv[1:]]:
    words = int(mb * 2 ** 20) // 8
    send = torch.arange(words, dtype=torch.int64, device="cuda")
    recv = torch.zeros_like(send)
    torch.cuda.synchronize()
    t = time.time()
    with torch.cuda.stream(side):
        w = dist.all_to_all_single(recv, send, async_op=True)
    print(f"{mb:8.1f} MiB ({words * 8} B, {'>' if words * 8 > 2 ** 30 else '<='} 2^30): issued {time.time() - t:.3f}s",
          flush=True)
    with torch.cuda.stream(side):
        w.wait()
    side.synchronize()
    t1 = time.time() - t
    torch.cuda.synchronize()
    ok = bool(torch.equal(recv, send))
    print(f"    side stream done {t1:.3f}s, device sync {time.time() - t:.3f}s, recv == send: {ok}", flush=True)
    del send, recv
dist.destroy_process_group()
print("ok", flush=True)
