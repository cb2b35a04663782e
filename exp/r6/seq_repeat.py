"""Repeat the SEQ harness case test_send_messages_fewer_rumors_than_slots
[200-16-10-SEQ] (and the R = 1 SEQ case) K times in one process against the
oracle: is a mismatch deterministic?  Usage: seq_repeat.py K"""
import sys
import traceback

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import safe_gossip_amd as sg  # noqa: E402
import test_gpu_harness as th  # noqa: E402

sg.load_library()
K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
bad = 0
for k in range(K):
    for args in [(200, 16, 10, "SEQ"), (150, 8, 3, "SEQ"), (300, 70, 64, "2P")]:
        try:
            th.test_send_messages_fewer_rumors_than_slots(sg, *args)
        except AssertionError as e:
            bad += 1
            print(f"rep {k} {args}: FAIL {str(e).splitlines()[0]}", flush=True)
    print(f"rep {k} done, failures so far {bad}", flush=True)
print(f"TOTAL failures {bad} of {3 * K}")
