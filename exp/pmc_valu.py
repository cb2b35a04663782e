"""Per-dispatch SQ counters of the round kernel (experiment)."""
import csv, collections, sys
for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    d = collections.defaultdict(dict); names = {}
    for r in rows:
        if "round_kernel" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        d[k][r["Counter_Name"]] = d[k].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
        names[k] = r["Kernel_Name"][:40]
    print(path)
    for k in sorted(d):
        v = d[k]; w = v.get("SQ_WAVES", 1)
        print(k, names[k], "valu/wave %.0f salu/wave %.0f vmem/wave %.1f wavecyc/wave %.0f" % (
            v["SQ_INSTS_VALU"] / w, v["SQ_INSTS_SALU"] / w, v["SQ_INSTS_VMEM_RD"] / w, v["SQ_WAVE_CYCLES"] / w))
