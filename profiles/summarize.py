"""Summarise a rocprofv3 run of bench.py (profiles/rocprof_r1.sh) into profiles/<tag>/.

Writes kernel_stats.csv (copied), summary.json and (for the default config 4
workload) pmc_latest.json (traffic of the dominant kernel per launch).
HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB units): FETCH_SIZE counts 64 B per
memory-side read request (TCC_EA0_RDREQ) and every request of the round
kernel moves a 128-B line -- calibrated with exp/gather_calib.hip on the
state's own layouts (coalesced 16-B streaming reads, and random 32-/96-B
class-row gathers: one request per gather, profiles/r2/pmc_calib_and_cfg5.json);
WRITE_SIZE is exact for our stores.

    python profiles/summarize.py gpurun_out/prof_r2 r2 --nodes 16777216 --rumors 256
"""
import argparse
import collections
import csv
import json
import os
import shutil

HERE = os.path.dirname(os.path.abspath(__file__))
DOMINANT = "round_kernel<false, 1"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("tag")
    ap.add_argument("--nodes", type=int, default=1 << 24)
    ap.add_argument("--rumors", type=int, default=256)
    ap.add_argument("--dominant", default=DOMINANT, help="substring of the dominant kernel's name")
    ap.add_argument("--no-latest", action="store_true", help="do not update profiles/pmc_latest.json")
    ap.add_argument("--commit", default=None,
                    help="commit of the profiled tree (default: this repository's HEAD, for a run "
                         "of a committed tree)")
    ap.add_argument("--skip-first", type=int, default=2,
                    help="dominant-kernel launches before the timed window (the bench's warmup "
                         "rounds that deliver: warmup 3 -> 2), left out of the PMC means")
    a = ap.parse_args()
    out = os.path.join(HERE, a.tag)
    os.makedirs(out, exist_ok=True)
    stats_csv = os.path.join(a.prof_dir, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(out, "kernel_stats.csv"))
    kernels = []
    for x in csv.DictReader(open(stats_csv)):
        kernels.append(dict(name=x["Name"], calls=int(x["Calls"]),
                            avg_ms=float(x["AverageNs"]) / 1e6, pct=float(x["Percentage"])))
    pmc = collections.defaultdict(dict)
    for sub, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        path = os.path.join(a.prof_dir, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        vals = collections.defaultdict(list)
        for x in sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"])):
            vals[x["Kernel_Name"]].append(float(x["Counter_Value"]))
        for k, v in vals.items():
            if a.dominant in k and len(v) > a.skip_first:
                v = v[a.skip_first:]  # the timed window's launches, as bench.py averages them
            pmc[k][counter + "_KiB_mean"] = sum(v) / len(v)
    dom = next((k for k in pmc if a.dominant in k), None)
    summary = dict(kernels=kernels, pmc=pmc)
    if dom and "FETCH_SIZE_KiB_mean" in pmc[dom] and "WRITE_SIZE_KiB_mean" in pmc[dom]:
        f = pmc[dom]["FETCH_SIZE_KiB_mean"] * 1024
        w = pmc[dom]["WRITE_SIZE_KiB_mean"] * 1024
        dom_ms = next(k["avg_ms"] for k in kernels if a.dominant in k["name"])
        commit = a.commit
        if commit is None:
            import subprocess
            commit = subprocess.run(["git", "-C", HERE, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                    text=True).stdout.strip() or None
        import sys
        sys.path.insert(0, os.path.dirname(HERE))
        from safe_gossip_amd.build import source_hash
        latest = dict(tag=a.tag, commit=commit, build_id=source_hash(), kernel=dom, nodes=a.nodes, rumors=a.rumors,
                      fetch_bytes_raw=f, write_bytes=w, hbm_bytes_per_launch=2 * f + w,
                      kernel_avg_ms_rocprof=dom_ms,
                      hbm_gbs=(2 * f + w) / (dom_ms * 1e-3) / 1e9,
                      note="hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE per launch (FETCH_SIZE = 64 B per "
                           "read request; each request moves a 128-B line, calibrated in "
                           "profiles/r2/pmc_calib_and_cfg5.json)")
        summary["dominant"] = latest
        json.dump(latest, open(os.path.join(HERE, f"pmc_n{a.nodes}_r{a.rumors}.json"), "w"), indent=1)
        if not a.no_latest:
            json.dump(latest, open(os.path.join(HERE, "pmc_latest.json"), "w"), indent=1)
    json.dump(summary, open(os.path.join(out, "summary.json"), "w"), indent=1)
    print(json.dumps(summary.get("dominant", {}), indent=1))


if __name__ == "__main__":
    main()
