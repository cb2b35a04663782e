"""Per-dispatch SQ counters of a kernel from rocprofv3 --pmc CSVs (experiment)."""
import csv, collections, sys
pat = sys.argv[1]
for path in sys.argv[2:]:
    d = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
    for r in csv.DictReader(open(path)):
        if pat not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"][:30]
    print(path)
    keys = None
    for i, k in enumerate(sorted(d)):
        v = d[k]; w = v.get("SQ_WAVES", 1)
        if keys is None:
            keys = [c for c in sorted(v) if c != "SQ_WAVES"]
            print("disp waves " + " ".join(c.replace("SQ_", "") for c in keys))
        print(i, int(w), " ".join("%.1f" % (v[c] / w) for c in keys))
