"""One DLV round at nb >= 512 bins with the quarter-bin variant library
(GS_DLV_SPLIT_LOG=2), to find which HIP call fails (AMD_LOG_LEVEL=1 set by
the caller prints the failing API and its error)."""
import sys
sys.path.insert(0, ".")
import safe_gossip_amd as sg

n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 23) + 1
net = sg.Network(n, 16, seed=0x5AFE6055, device=0)
net.send_new(0, 0)
for i in range(3):
    net.next_round(report=False)
    net.sync()
    print("round", i + 1, "ok", flush=True)
net.close()
