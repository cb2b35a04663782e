"""Per-dispatch time and HBM traffic of a kernel from rocprofv3 CSVs (experiment).

usage: pmc_table.py <kernel substring> <dir with trace/ fetch/ write/>"""
import csv, collections, glob, sys
pat, d = sys.argv[1], sys.argv[2]
def rows(sub, name):
    return list(csv.DictReader(open(glob.glob(f"{d}/{sub}/**/{name}", recursive=True)[0])))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows("trace", "run_kernel_trace.csv") if pat in r["Kernel_Name"]]
def per_disp(sub, cname):
    acc = collections.defaultdict(float)
    for r in rows(sub, "run_counter_collection.csv"):
        if pat in r["Kernel_Name"] and r["Counter_Name"] == cname:
            acc[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return [acc[k] for k in sorted(acc)]
fe = per_disp("fetch", "FETCH_SIZE"); wr = per_disp("write", "WRITE_SIZE")
print("i ms  fetchGB(x2) writeGB  TB/s")
tot_b = tot_t = 0
for i, (t, f, w) in enumerate(zip(dur, fe, wr)):
    b = (2 * f + w) * 1e3  # FETCH_SIZE/WRITE_SIZE in KB
    print(i, "%.3f %.2f %.2f %.2f" % (t, 2 * f * 1e3 / 1e9, w * 1e3 / 1e9, b / (t * 1e-3) / 1e12))
    if i >= 4:
        tot_b += b; tot_t += t
print("rounds>=4 avg TB/s %.2f" % (tot_b / (tot_t * 1e-3) / 1e12))
