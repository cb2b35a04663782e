"""Host enqueue cost of a round against its device time (small networks).

For configs 2 and 3: K rounds enqueued without any sync (report=False), timed
on the host; then the sync.  If the enqueue alone takes about as long as the
whole, the round loop is host-bound and the device idles between kernels.
Also with the engine's timing events on (bench.py's setting)."""
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: F401
import safe_gossip_amd as sg

SEED = 0x5AFE6055
K = 200
for n, R in ((1 << 20, 1), (1 << 20, 64)):
    for timing in (False, True):
        net = sg.Network(n, R, seed=SEED, device=0)
        for r in range(R):
            net.send_new(sg.origin_of(SEED, 0, r, n), r)
        for _ in range(5):
            net.next_round(report=False)
        net.sync()
        net.set_timing(timing)
        t0 = time.perf_counter()
        for _ in range(K):
            net.next_round(report=False)
        t1 = time.perf_counter()
        net.sync()
        t2 = time.perf_counter()
        kt = net.round_kernel_times() if timing else []
        net.set_timing(False)
        net.close()
        print(json.dumps(dict(n=n, R=R, timing=timing, enqueue_us=(t1 - t0) / K * 1e6,
                              total_us=(t2 - t0) / K * 1e6,
                              kernel_us=float(sum(kt[1:]) / max(1, len(kt) - 1) * 1e3) if len(kt) else None)), flush=True)
