"""Benchmark: node-rumor updates/sec of the safe_gossip push-pull round on MI355X.

A "step" is one round (phase 0 + push/pull delivery, 2P schedule) over the
whole simulated network.  Default workload (config 4 of BASELINE.json, which
fits one MI355X): n = 2^24 nodes x R = 256 rumors, all rumors injected in round
1 at Philox-chosen origins, seed 0x5AFE6055.  Inputs are synthetic and resident
in HBM (the state is created on the device; nothing crosses PCIe in the timed
region).

value  = n * R * K / wall seconds of K timed rounds (summed over ranks).
roofline: algorithmic HBM bytes of the round kernel (DESIGN.md "Roofline") per
          launch / its average duration measured with HIP events on the
          engine's stream over the timed rounds; peak 8.0 TB/s.  step_frac:
          the same bytes over the whole step (round kernel + in-list build).
traffic:  HBM bytes per launch of that kernel from PMC counters, measured in
          this run by two child rocprofv3 --pmc passes of the same workload
          (--pmc auto, N=1; else the committed profiles/pmc_n*_r*.json, marked
          with whether its build id is the loaded library's).
cpu_baseline: the CPU oracle (reference-faithful port: per-node ordered maps,
          one thread, same 2P schedule) on a bounded sample of the same
          workload (fewer nodes, same R and injection), rank 0 at N=1 only.

Other BASELINE configurations (--config): cfg2 (2^20 x 1), cfg3 (2^20 x 64) and
cfg5 (10^8 x 16 with harness-injected faults: 1% churn, 1% push-batch drop, 1%
pull-batch drop per node per round, Philox stream 3).  The default line is
cfg4, the configuration the metric is quoted on that fits one GPU.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N, or plain
`python bench.py --gpus N`, which starts that launcher itself): ONE network
of the same n x R over the N ranks, measured in both multi-GPU modes one after
the other, and the faster is the headline (the others under "alternative"):
rumor slices (every rank holds all n nodes and R/N of the rumors, DESIGN.md
section 7b; rumors evolve independently, so a round's only exchange is one
RCCL all_reduce(MIN) of 2 bytes per node, the empty-RPC Statistics,
overlapped with the next round) and node-range shards (DESIGN.md section 7:
push and pull rows exchanged by RCCL all-to-all every round).  Each mode runs
twice: with the round loop in the library (gs_net, safe_gossip_amd.net,
DESIGN.md section 7d: the C++ loop issues its own RCCL collectives; one RCCL
rank measured it 0.35-0.77 ms per round where the Python drivers took
0.36-1.19) and with the Python drivers (safe_gossip_amd.sliced / .sharded,
torch.distributed collectives).  --mode slices|nodes|slices-lib|nodes-lib
measures one.  Total work is fixed, so "scaling" is "strong".  Barrier +
synchronize around the timed region, time = max over ranks.  The roofline
line describes rank 0's round kernel.  A watchdog prints the line of the
modes finished so far and ends every rank if a mode overruns --deadline.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0
METRIC = "node-rumor updates/sec (whole node) + % HBM roofline; rounds-to-full-spread"


# BASELINE.json configs: (nodes, rumors, (churn, drop_push, drop_pull))
CONFIGS = {
    "cfg2": (1 << 20, 1, (0.0, 0.0, 0.0)),
    "cfg3": (1 << 20, 64, (0.0, 0.0, 0.0)),
    "cfg4": (1 << 24, 256, (0.0, 0.0, 0.0)),
    "cfg5": (100_000_000, 16, (0.01, 0.01, 0.01)),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="cfg4", choices=sorted(CONFIGS))
    p.add_argument("--nodes", type=int, default=None, help="override the config's node count")
    p.add_argument("--rumors", type=int, default=None)
    p.add_argument("--churn", type=float, default=None, help="P(node offline) per round")
    p.add_argument("--drop-push", type=float, default=None, help="P(push batch dropped)")
    p.add_argument("--drop-pull", type=float, default=None, help="P(pull batch dropped)")
    p.add_argument("--schedule", default="2P", choices=["2P", "SEQ"],
                   help="2P (default) or SEQ (the reference harness's literal order; N>1: rumor slices)")
    p.add_argument("--seed", type=lambda s: int(s, 0), default=0x5AFE6055)
    p.add_argument("--cpu-seconds", type=float, default=15.0,
                   help="budget of the CPU-oracle sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-spread", action="store_true", help="skip the rounds-to-full-spread run")
    p.add_argument("--parts", type=int, default=None,
                   help="pipeline parts per rank (N>1; default 4 with RCCL: the exchanges of one "
                        "part overlap the round kernel of another)")
    p.add_argument("--mode", default="both", choices=["both", "slices", "nodes", "slices-lib", "nodes-lib"],
                   help="N>1: measure both multi-GPU modes, each with the library's round loop (-lib) "
                        "and the Python drivers, and report the fastest (default), or only one; with "
                        "--sharded at N=1 the default is node shards")
    p.add_argument("--deadline", type=float, default=240.0,
                   help="N>1: seconds after which a watchdog reports the modes finished so far and "
                        "ends every rank")
    p.add_argument("--sharded", action="store_true",
                   help="run a multi-GPU mode even at N=1 (one RCCL rank: node-shard exchanges are "
                        "self-copies, the slice all-reduce a no-op; measures that path's overhead)")
    p.add_argument("--pmc", default="auto", choices=["auto", "off"],
                   help="auto (N=1, single engine): measure roofline.traffic live -- two child "
                        "rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of this same workload and "
                        "library; off: take it from the committed profiles/pmc_n*_r*.json")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (RCCL, one GPU per rank) or gloo (host-staged rows; rehearsal of "
                        "the N>1 path with several ranks on one GPU)")
    a = p.parse_args()
    n, R, f = CONFIGS[a.config]
    a.nodes = n if a.nodes is None else a.nodes
    a.rumors = R if a.rumors is None else a.rumors
    a.faults = (f[0] if a.churn is None else a.churn, f[1] if a.drop_push is None else a.drop_push,
                f[2] if a.drop_pull is None else a.drop_pull)
    return a


def inject_all(net, epoch):
    """Every rumor at its Philox origin (sharded: only the owner takes it)."""
    import safe_gossip_amd as sg
    for r in range(net.R):
        x = sg.origin_of(net.seed, epoch, r, net.n)
        if getattr(net, "transport", None) == "dist" and hasattr(net, "shards"):
            s = net.shards[0]
            if not s.lo <= x < s.lo + s.m:
                continue
        net.send_new(x, r)


def spread_run(net, epoch, max_rounds=200):
    """Untimed: rounds until termination and first round with full spread."""
    net.clear(epoch)
    inject_all(net, epoch)
    r_full = 0
    rounds = 0
    for _ in range(max_rounds):
        rep = net.next_round()
        rounds = rep.round
        if not r_full:
            _, complete = net.known_counts()
            if complete == net.n:
                r_full = rep.round
        if not rep.any_live:
            break
    known, complete = net.known_counts()
    return dict(rounds=rounds, round_full=r_full, nodes_complete=complete,
                known_fraction=known / float(net.n * net.R))


def cpu_baseline(R, seed, budget_s, faults=(0.0, 0.0, 0.0), schedule="2P"):
    """Time the CPU oracle (port) on a bounded sample: n_cpu nodes, same R."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    oracle_lib.build_oracle()
    n_cpu = 1 << 17  # (2^15 / 2^16 finished their whole dissemination in 4 / 8 s on the GPU box host; ~10-30 s is the aim)
    thr = [oracle_lib.fault_threshold(p) for p in faults] if any(faults) else None
    net = oracle_lib.OracleNet(n_cpu, R, seed=seed, faults=thr)
    L = oracle_lib.lib()
    for r in range(R):
        net.send_new(L.or_origin(seed, 0, r, n_cpu), r)
    t0 = time.perf_counter()
    rounds = 0
    while True:
        _, live = net.next_round(oracle_lib.SCHED_SEQ if schedule == "SEQ" else oracle_lib.SCHED_2P)
        rounds += 1
        el = time.perf_counter() - t0
        if not live or el > budget_s:
            break
    net.close()
    return dict(value=n_cpu * R * rounds / el, unit="node-rumor updates/s", cores=1,
                kind="port",
                sample=f"CPU oracle (per-node ordered maps, 1 thread, {schedule}), n={n_cpu}, R={R}, "
                       f"all rumors injected round 1, {rounds} rounds in {el:.1f}s"
                       + (f", faults {faults}" if thr else ""))


def cpu_best(R, seed, budget_s):
    """The dense bit-sliced OpenMP CPU program (oracle/gs_dense.c, checked
    against the oracle in tests/test_dense_cpu.py) on all its threads: the
    secondary "best CPU" line of SURVEY.md section 8d (2P, no faults)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    oracle_lib.build_oracle()
    L = oracle_lib.lib()
    n_cpu = 1 << 20
    net = oracle_lib.DenseNet(n_cpu, R, seed=seed)
    for r in range(R):
        net.send_new(L.or_origin(seed, 0, r, n_cpu), r)
    t0 = time.perf_counter()
    rounds = 0
    while True:
        live = net.next_round()
        rounds += 1
        el = time.perf_counter() - t0
        if not live or el > budget_s:
            break
    net.close()
    return dict(value=n_cpu * R * rounds / el, unit="node-rumor updates/s", cores=L.dn_threads(),
                kind="port (dense bit-sliced, OpenMP)",
                sample=f"oracle/gs_dense.c, n={n_cpu}, R={R}, all rumors injected round 1, "
                       f"{rounds} rounds in {el:.1f}s")


def rocprof_pattern(kernel_name):
    """The rocprofv3 (demangled) name prefix of an engine's deliver+transition
    kernel, e.g. "round_kernel<false,1> (...)" -> "round_kernel<false, 1,",
    "round_kernel_dlv4<1,u32,2>" -> "round_kernel_dlv4<1,",
    "round_kernel_w32<1> (...)" -> "round_kernel_w32<1>"."""
    base = kernel_name.split(" ")[0]
    fn, _, targs = base.partition("<")
    args = [a.strip() for a in targs.rstrip(">").split(",")]
    if fn == "round_kernel":
        return f"{fn}<{args[0]}, {args[1]},"
    if fn == "round_kernel_w32":
        return f"{fn}<{args[0]}>"
    return f"{fn}<{args[0]},"


def live_pmc(args, kernel_name, skip):
    """HBM bytes per launch of the dominant kernel, measured now: one child
    rocprofv3 run per counter group (FETCH_SIZE, then WRITE_SIZE -- they do
    not fit one pass, MI355X_MICROARCH.md), each running this same workload
    with this same library; bytes = 2 * FETCH_SIZE + WRITE_SIZE (FETCH_SIZE
    counts 64 B per 128-B read request on gfx950).  The launches of the
    child's timed window are averaged (its first `skip` deliver launches are
    warmup).  Returns (bytes, source dict) or (None, reason)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    pat = rocprof_pattern(kernel_name)
    child = [sys.executable, os.path.abspath(__file__), "--config", args.config, "--nodes", str(args.nodes),
             "--rumors", str(args.rumors), "--steps", str(args.steps), "--warmup", str(args.warmup),
             "--churn", str(args.faults[0]), "--drop-push", str(args.faults[1]), "--drop-pull",
             str(args.faults[2]), "--schedule", args.schedule, "--seed", hex(args.seed),
             "--no-cpu-baseline", "--no-spread", "--pmc", "off"]
    vals = {}
    tmp = tempfile.mkdtemp(prefix="gs_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = [prof, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--"] + child
            env = dict(os.environ, SAFE_GOSSIP_AMD_UNDER_PROFILER="1")
            try:
                r = subprocess.run(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                                   timeout=300, cwd=tmp)
            except subprocess.TimeoutExpired:
                return None, f"rocprofv3 --pmc {counter} timed out"
            path = os.path.join(d, "run_counter_collection.csv")
            if r.returncode != 0 or not os.path.exists(path):
                return None, f"rocprofv3 --pmc {counter} failed (rc {r.returncode}): {r.stderr[-300:]}"
            rows = sorted((x for x in csv.DictReader(open(path)) if pat in x["Kernel_Name"]),
                          key=lambda x: int(x["Dispatch_Id"]))
            v = [float(x["Counter_Value"]) for x in rows][skip:]
            if not v:
                return None, f"no {pat} launches in the {counter} pass"
            vals[counter] = (sum(v) / len(v) * 1024.0, len(v), rows[0]["Kernel_Name"])
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    f, w = vals["FETCH_SIZE"][0], vals["WRITE_SIZE"][0]
    return 2.0 * f + w, {"kind": "live", "kernel": vals["FETCH_SIZE"][2], "launches": vals["FETCH_SIZE"][1],
                         "fetch_bytes_raw": f, "write_bytes": w,
                         "note": "child rocprofv3 --pmc passes of this workload: 2*FETCH_SIZE + WRITE_SIZE "
                                 "per launch of the timed window"}


def self_launch(args):
    """`bench.py --gpus N` without a launcher: run torch.distributed.run with
    N ranks as a child process (before anything touches the GPU), relay its
    output and exit with its status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.run(cmd).returncode)


def run_mode(args, mode, world, rank, local, dist, sg, np, torch, with_spread):
    """Build the network for `mode` ("single", "slices" or "nodes"), run W
    warmup rounds of one dissemination, then time exactly K rounds of a fresh
    one (barrier + synchronize on both sides, max over ranks).  Returns the
    measurements; the network is closed."""
    n, R = args.nodes, args.rumors
    fk = dict(churn=args.faults[0], drop_push=args.faults[1], drop_pull=args.faults[2])
    if args.schedule != "2P":
        fk["schedule"] = args.schedule
    if mode in ("slices-lib", "nodes-lib"):
        from safe_gossip_amd.net import Net
        # RCCL, or (gloo rehearsal) the library calling back into the process group
        net = Net(n, R, world, mode="slices" if mode == "slices-lib" else "shards", seed=args.seed, epoch=0,
                  device=local, transport="dist" if args.dist_backend == "nccl" else "host",
                  parts=args.parts or 4, **fk)
    elif mode == "slices":
        from safe_gossip_amd.sliced import SlicedNetwork
        net = SlicedNetwork(n, R, world, seed=args.seed, epoch=0, device=local, transport="dist", **fk)
    elif mode == "nodes":
        from safe_gossip_amd.sharded import ShardedNetwork
        net = ShardedNetwork(n, R, world, seed=args.seed, epoch=0, device=local,
                             transport="dist", parts=args.parts, **fk)
    else:
        net = sg.Network(n, R, seed=args.seed, epoch=0, device=local, **fk)

    def barrier_sync():
        net.sync()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    # warmup: W rounds of a dissemination (epoch 0)
    inject_all(net, 0)
    for _ in range(args.warmup):
        net.next_round(report=False)
    # timed: K rounds of a fresh dissemination from round 1
    epoch = 1
    net.clear(epoch)
    inject_all(net, epoch)
    net.set_timing(True)
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        net.next_round(report=False)
    barrier_sync()   # net.sync() raises DeviceError if a device limit was hit
    elapsed = time.perf_counter() - t0
    ktimes = net.round_kernel_times()
    net.set_timing(False)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # rounds 2.. run the fused deliver+transition kernel (round 1 has nothing
    # to deliver); that is the dominant kernel the roofline describes.
    kt = ktimes[1:] if len(ktimes) > 1 else ktimes
    out = dict(mode=mode, elapsed=elapsed, kt=kt, name=net.round_kernel_name(),
               bytes_dense=net.round_kernel_bytes(), params=list(net.params),
               parts=getattr(net, "parts", None))
    # algorithmic bytes the timed launches had to move: with live-filtered
    # gathers, only the class rows the flags leave are gathered, so this is
    # counted by the kernels
    out["bytes_per"], out["launches"] = (net.round_traffic() if hasattr(net, "round_traffic")
                                         else (out["bytes_dense"], 0))
    out["spread"] = spread_run(net, epoch) if with_spread else None
    net.close()
    return out


def parallelism(args, mode, world, parts):
    backend = "RCCL" if args.dist_backend == "nccl" else args.dist_backend
    n, R = args.nodes, args.rumors
    if mode == "slices-lib":
        return (f"rumor slices x{world} (all {n} nodes, {R // world}-{-(-R // world)} rumors per rank), "
                "library round loop (gs_net): RCCL ncclAllReduce(MIN) of 2 B/node empty-RPC counts per round, "
                "overlapped with the next round")
    if mode == "nodes-lib":
        return (f"node-range shards x{world}, library round loop (gs_net): RCCL ncclAllToAll push/pull rows, "
                f"{parts} pipeline part(s) per rank")
    if mode == "slices":
        return (f"rumor slices x{world} (all {n} nodes, {R // world}-{-(-R // world)} rumors per rank), "
                + backend + " all_reduce(MIN) of 2 B/node empty-RPC counts per round"
                + (", overlapped with the next round" if args.dist_backend == "nccl" else ", host-staged"))
    if mode == "nodes":
        return (f"node-range shards x{world}, " + backend
                + f" all-to-all push/pull rows, {parts} pipeline part(s) per rank")
    return "single-gpu"


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        self_launch(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1 or args.sharded:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        import torch.distributed as dist
        if args.dist_backend == "gloo":
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)
        if dist.get_world_size() != args.gpus:
            print(f"bench.py: process group of {dist.get_world_size()} ranks, --gpus {args.gpus}",
                  file=sys.stderr)
            sys.exit(2)
    else:
        torch.cuda.set_device(0)

    import numpy as np
    import safe_gossip_amd as sg

    n, R = args.nodes, args.rumors
    # Modes measured: one GPU runs the single engine; several ranks run both
    # multi-GPU modes (rumor slices, node shards) one after the other and the
    # faster is the headline, unless --mode picks one;
    # --sharded at N = 1 runs the node shards (self-copy exchanges).
    if dist is None:
        modes = ["single"]
    elif args.mode != "both":
        modes = [args.mode]
    elif world == 1:
        modes = ["nodes"]
    else:
        # the Python drivers first (rehearsed with 8 ranks), then
        # the library's loop (over RCCL; with gloo, over the host collectives)
        modes = ["slices", "nodes", "slices-lib", "nodes-lib"]
    if R < world:  # fewer rumors than ranks: no rumor slices
        modes = [m for m in modes if not m.startswith("slices")] or ["nodes"]
    if args.schedule == "SEQ" and dist is not None:  # SEQ's pull chains cross node ranges: slices only
        modes = [m for m in modes if m.startswith("slices")] or ["slices"]
    runs, failed = [], []
    if dist is not None and world > 1:
        start_watchdog(args, runs, failed, world, rank, np, sg)
    for i, m in enumerate(modes):
        try:
            runs.append(run_mode(args, m, world, rank, local, dist, sg, np, torch,
                                 with_spread=(not runs and not args.no_spread)))
        except Exception as e:  # a later mode that cannot run here (e.g. no RCCL for gs_net)
            if not (runs and m.endswith("-lib")):
                raise
            failed.append(f"{m}: {type(e).__name__}: {e}")
            print(f"bench.py: mode {m} failed: {e}", file=sys.stderr)
    if rank == 0:
        report(args, runs, failed, world, rank, np, sg, None, dist is not None)
    if dist is not None:
        dist.destroy_process_group()


_REPORTED = []


def start_watchdog(args, runs, failed, world, rank, np, sg):
    """A mode that overruns --deadline (a stuck collective) must not cost the
    modes already measured: print their line (rank 0) and end this rank."""
    import threading

    def fire():
        if _REPORTED:
            return
        if rank == 0 and runs:
            report(args, list(runs), failed, world, rank, np, sg,
                   f"watchdog: a later mode overran the {args.deadline:.0f} s deadline", True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0 if runs else 1)
    t = threading.Timer(args.deadline, fire)
    t.daemon = True
    t.start()


def report(args, runs, failed, world, rank, np, sg, note, dist_on):
    """Rank 0: the JSON line of the fastest of `runs`."""
    _REPORTED.append(True)
    n, R = args.nodes, args.rumors
    best = min(runs, key=lambda r: r["elapsed"])
    spread = runs[0]["spread"]

    kt = best["kt"]
    kernel_ms = float(np.mean(kt)) if len(kt) else float("nan")
    achieved = best["bytes_per"] / (kernel_ms * 1e-3) / 1e9
    elapsed = best["elapsed"]
    ms_per_step = elapsed / args.steps * 1e3
    # the whole step's algorithmic bytes over its wall time: the round kernel's
    # bytes against the time of the round kernel AND the in-list build
    step_frac = best["bytes_per"] / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS

    # HBM traffic of the same kernel from PMC counters: measured live by child
    # rocprofv3 runs of this workload (N=1, single engine; rocprofv3 cannot
    # count the process it runs in), else from the committed rocprofv3 run of
    # this workload (profiles/summarize.py writes one file per (nodes,
    # rumors)), marked with whether it profiled this very library build
    traffic = traffic_src = None
    build_id = sg.build_id()
    if (rank == 0 and world == 1 and best["mode"] == "single" and args.pmc == "auto"
            and not os.environ.get("SAFE_GOSSIP_AMD_UNDER_PROFILER")):
        traffic, traffic_src = live_pmc(args, best["name"], skip=max(0, args.warmup - 1))
        if traffic is None:
            traffic_src = {"kind": "live", "failed": traffic_src}
    for name in (f"pmc_n{n}_r{R}.json", "pmc_latest.json"):
        pmc_path = os.path.join(REPO, "profiles", name)
        if traffic is None and os.path.exists(pmc_path) and world == 1 and best["mode"] == "single":
            try:
                pmc = json.load(open(pmc_path))
                if pmc.get("nodes") == n and pmc.get("rumors") == R:
                    traffic = pmc.get("hbm_bytes_per_launch")
                    traffic_src = {"kind": "committed", "file": "profiles/" + name, "profile": pmc.get("tag"),
                                   "commit": pmc.get("commit"), "build_id": pmc.get("build_id"),
                                   "build_id_match": pmc.get("build_id") == build_id,
                                   "kernel_avg_ms_rocprof": pmc.get("kernel_avg_ms_rocprof"),
                                   "live_failed": (traffic_src or {}).get("failed")}
            except Exception:
                traffic = None

    cpu = cpu_best_line = None
    if rank == 0 and world == 1 and not dist_on and not args.no_cpu_baseline:
        cpu = cpu_baseline(R, args.seed, args.cpu_seconds, args.faults, args.schedule)
        if args.schedule == "2P" and not any(args.faults):
            cpu_best_line = cpu_best(R, args.seed, args.cpu_seconds)

    if rank == 0:
        total_updates = float(n) * R * args.steps
        line = {
            "metric": METRIC,
            "value": total_updates / elapsed,
            "unit": "node-rumor updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {
                "workload": f"{args.config}: {n} nodes x {R} rumors, full mesh, all rumors injected in "
                            f"round 1 at Philox origins, {args.schedule} schedule, {args.steps} rounds"
                            + (", faults churn/drop_push/drop_pull = %g/%g/%g per node-round"
                               % args.faults if any(args.faults) else ""),
                "n_nodes": n, "n_rumors": R, "seed": hex(args.seed),
                "faults": {"churn": args.faults[0], "drop_push": args.faults[1],
                           "drop_pull": args.faults[2]},
                "params": best["params"],
                "parallelism": parallelism(args, best["mode"], world, best["parts"])
                               + (" (faster of: " + "; ".join(f"{r['mode']} {r['elapsed'] / args.steps * 1e3:.3f} ms/step"
                                                               for r in runs) + ")" if len(runs) > 1 else ""),
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                "step_frac": step_frac,
                "kernel": best["name"] + " (deliver round t + transition to t+1)",
                "kernel_ms": kernel_ms, "algorithmic_bytes_per_launch": best["bytes_per"],
                # the rest of a step: the next round's in-list build (the largest of
                # its kernels is smaller than the round kernel at every config) and
                # the launch gaps
                "rest_of_step_ms": ms_per_step - kernel_ms,
                "bytes_counted_by": ("kernels (rows actually gathered + every node's planes read and written, the stores all-A waves skip included), %d launches"
                                     % best["launches"]) if best["launches"] else "static model",
                "dense_model_bytes_per_launch": best["bytes_dense"],
                "kernel_ms_per_round": [round(float(v), 4) for v in kt],
            },
            "cpu_baseline": cpu,
            "cpu_best": cpu_best_line,
            "build": {"id": build_id, "abi": sg.ABI_VERSION,
                      "note": "gs_build_id: SHA-256 prefix of the library's sources (safe_gossip_amd/build.py)"},
            "spread": spread,
        }
        if len(runs) > 1:
            line["alternative"] = [{
                "mode": r["mode"], "parallelism": parallelism(args, r["mode"], world, r["parts"]),
                "value": total_updates / r["elapsed"], "ms_per_step": r["elapsed"] / args.steps * 1e3,
                "kernel": r["name"], "kernel_ms": float(np.mean(r["kt"])) if len(r["kt"]) else None,
            } for r in runs if r is not best]
        if failed:
            line["failed_modes"] = failed
        if note:
            line["note"] = note
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
