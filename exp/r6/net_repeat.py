"""Repeat GPU test functions K times in one process (mismatch hunting):
test_gpu_net.py's local-transport cases and test_gpu_harness.py's
fewer-rumors cases.  Usage: net_repeat.py K"""
import sys
import traceback

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import safe_gossip_amd as sg  # noqa: E402
import test_gpu_harness as th  # noqa: E402
import test_gpu_net as tn  # noqa: E402

sg.load_library()
print("library", sg.load_library().gs_build_id().decode(), flush=True)
K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
cases = [
    (tn.test_python_net_local, ("shards", 3, 900, 16, (0.05, 0.05, 0.05), "2P")),
    (tn.test_python_net_local, ("shards", 2, 800, 100, None, "2P")),
    (tn.test_python_net_local, ("slices", 3, 700, 30, (0.05, 0.05, 0.05), "SEQ")),
    (th.test_send_messages_fewer_rumors_than_slots, (200, 16, 10, "SEQ")),
    (th.test_send_messages_fewer_rumors_than_slots, (300, 70, 64, "2P")),
]
bad = 0
for k in range(K):
    for fn, args in cases:
        try:
            fn(sg, *args)
        except Exception as e:  # noqa: BLE001
            bad += 1
            print(f"rep {k} {fn.__name__}{args}: FAIL {type(e).__name__}: {str(e).splitlines()[0][:200]}", flush=True)
    print(f"rep {k} done, failures so far {bad}", flush=True)
print(f"TOTAL failures {bad} of {len(cases) * K}")
