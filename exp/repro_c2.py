import sys, ctypes
sys.path.insert(0, "/root/repo")
sys.path.insert(0, ".")
import safe_gossip_amd as sg
for n in [int(a) for a in sys.argv[1:]]:
    net = sg.Network(n, 1, seed=0x5AFE6055)
    net.send_new(sg.origin_of(0x5AFE6055, 0, 0, n), 0)
    try:
        for r in range(5):
            rep = net.next_round()
        print("ok", n, rep, flush=True)
    except Exception as e:
        print("FAIL", n, r, e, flush=True)
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipGetErrorString.restype = ctypes.c_char_p
        err = hip.hipPeekAtLastError()
        print("hip error", err, hip.hipGetErrorString(err), flush=True)
    net.close()
