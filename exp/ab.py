"""Interleaved A/B timing of bench.py variants on one box (the box-to-box
spread of one build is ~5 %, so a change is judged against its base run in
the same call, round-robin).

    python exp/ab.py --out gpurun_out/ab_<tag> --reps 3 \
        --variant "base:dir=exp/base_tree" --variant "head:dir=." \
        --variant "nofilt:env=SAFE_GOSSIP_AMD_FILTER=0" -- --config cfg5

A variant is `tag:key=value;key=value` with keys dir (the tree whose bench.py
and library run; default .), env (VAR=v,VAR=w) and lib (SAFE_GOSSIP_AMD_LIB).
Everything after `--` goes to bench.py (default args: --no-cpu-baseline
--no-spread --pmc off).  Writes <out>/runs.jsonl and prints per variant the
mean / min of ms_per_step and of the round kernel's mean ms.
(Replaces the per-experiment exp/r2-r4 shell recipes; they are in the
history at 677eb31.)"""
import argparse
import json
import os
import subprocess
import sys


def parse_variant(spec):
    tag, _, rest = spec.partition(":")
    v = {"tag": tag, "dir": ".", "env": {}, "lib": None}
    for kv in filter(None, rest.split(";")):
        k, _, val = kv.partition("=")
        if k == "env":
            for e in filter(None, val.split(",")):
                a, _, b = e.partition("=")
                v["env"][a] = b
        else:
            v[k] = val
    return v


def main():
    argv = sys.argv[1:]
    bench_args = []
    if "--" in argv:
        i = argv.index("--")
        argv, bench_args = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variant", action="append", required=True)
    ap.add_argument("--timeout", type=int, default=300)
    a = ap.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    vs = [parse_variant(s) for s in a.variant]
    res = {v["tag"]: [] for v in vs}
    with open(os.path.join(a.out, "runs.jsonl"), "a") as log:
        for rep in range(a.reps):
            for v in vs:
                d = os.path.join(root, v["dir"])
                env = dict(os.environ, **v["env"])
                if v["lib"]:
                    env["SAFE_GOSSIP_AMD_LIB"] = os.path.join(root, v["lib"])
                cmd = [sys.executable, os.path.join(d, "bench.py"), "--no-cpu-baseline", "--no-spread", "--pmc",
                       "off"] + bench_args
                r = subprocess.run(cmd, cwd=d, env=env, capture_output=True, text=True, timeout=a.timeout)
                if r.returncode != 0:
                    print(f"{v['tag']} rep {rep}: rc {r.returncode}\n{r.stderr[-2000:]}", flush=True)
                    sys.exit(1)
                line = json.loads(r.stdout.strip().splitlines()[-1])
                rec = {"variant": v["tag"], "rep": rep, "args": bench_args, "ms_per_step": line["ms_per_step"],
                       "kernel_ms": line["roofline"]["kernel_ms"], "line": line}
                log.write(json.dumps(rec) + "\n")
                log.flush()
                res[v["tag"]].append((line["ms_per_step"], line["roofline"]["kernel_ms"]))
                print(f"{v['tag']:>10s} rep {rep}: {line['ms_per_step']:.4f} ms/step, kernel "
                      f"{line['roofline']['kernel_ms']:.4f} ms", flush=True)
    for tag, xs in res.items():
        st = [x[0] for x in xs]
        kt = [x[1] for x in xs]
        print(f"{tag:>10s}: ms/step mean {sum(st) / len(st):.4f} min {min(st):.4f} | kernel mean "
              f"{sum(kt) / len(kt):.4f} min {min(kt):.4f}")


if __name__ == "__main__":
    main()
