"""Build helpers: compile the gfx950 engine library and the C++ examples.

The engine is built in-tree (``safe_gossip_amd/libsafe_gossip_amd.so``) with an
explicit ``hipcc --offload-arch=gfx950`` line so the artefact travels with the
repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libsafe_gossip_amd.so")
SOURCES = [os.path.join(CSRC, "gs_kernels.hip"), os.path.join(CSRC, "gs_inlist.hip"),
           os.path.join(CSRC, "gs_shard.hip"), os.path.join(CSRC, "gs_seq.hip"), os.path.join(CSRC, "gs_dlv4.hip"), os.path.join(CSRC, "gs_w32.hip"), os.path.join(CSRC, "gs_verify.hip"),
           os.path.join(CSRC, "gs_engine.cpp"), os.path.join(CSRC, "gs_net.cpp"), os.path.join(CSRC, "gs_wire.cpp"),
           os.path.join(CSRC, "gs_sign.cpp")]
HEADERS = [os.path.join(CSRC, f) for f in ("gs_common.h", "gs_kernels.h", "gs_device.h", "gs_recv.h")] + [
    os.path.join(REPO_DIR, "include", "safe_gossip.h")
]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def source_hash(root: str = REPO_DIR) -> str:
    """Provenance id of a library built from the tree at `root`: the first 16
    hex digits of the SHA-256 over (relative path, contents) of every source
    and header, in path order.  Compiled into the library (gs_build_id) and
    compared by load_library with the tree it runs from."""
    import hashlib
    h = hashlib.sha256()
    for p in sorted(os.path.relpath(f, REPO_DIR) for f in SOURCES + HEADERS):
        h.update(p.encode() + b"\0")
        with open(os.path.join(root, p), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src: str, obj: str, flags: list[str], verbose: bool) -> None:
    cmd = [HIPCC] + flags + ["-c", "-o", obj + ".tmp", src]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(obj + ".tmp", obj)


def build_engine(force: bool = False, verbose: bool = False, defines=(), out: str = None) -> str:
    """Compile libsafe_gossip_amd.so for gfx950 (no-op when up to date).

    Each source is compiled to its own object in parallel (build/, one
    directory per define set), then linked.  ``defines``/``out`` build an
    experiment variant (timing-only flags such as GS_EXP_*) into another
    file; the product library never carries them.
    """
    from concurrent.futures import ThreadPoolExecutor
    target = out or LIB_PATH
    tag = "product" if not defines else "_".join(sorted(defines)).replace("=", "-")
    # the library's build id: the tree's source hash (+ the variant's defines)
    bid = source_hash() + ("" if not defines else "+" + tag)
    idfile = target + ".buildid"
    if not force and not _stale(target, SOURCES + HEADERS) and os.path.exists(idfile) and \
            open(idfile).read().strip() == bid:
        return target
    flags = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-Wall", "-Wextra", "-Werror"] + [
        f"-D{d}" for d in defines]
    bdir = os.path.join(PKG_DIR, "build", tag)
    os.makedirs(bdir, exist_ok=True)
    objs, jobs = [], []
    for src in SOURCES:
        obj = os.path.join(bdir, os.path.basename(src) + ".o")
        objs.append(obj)
        extra = []
        if src.endswith("gs_engine.cpp"):  # the build id lives here: rebuilt whenever it changes
            extra = [f'-DGS_BUILD_ID="{bid}"']
            stale_id = not os.path.exists(obj + ".buildid") or open(obj + ".buildid").read().strip() != bid
        else:
            stale_id = False
        if force or stale_id or _stale(obj, [src] + HEADERS):
            jobs.append((src, obj, extra))
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(max_workers=workers) as ex:
        for f in [ex.submit(_compile, s_, o_, flags + x_, verbose) for s_, o_, x_ in jobs]:
            f.result()
    for s_, o_, x_ in jobs:
        if x_:
            with open(o_ + ".buildid", "w") as f:
                f.write(bid)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", target + ".tmp"] + objs + ["-ldl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(target + ".tmp", target)
    with open(idfile, "w") as f:
        f.write(bid)
    return target


def build_examples(force: bool = False) -> list[str]:
    """Compile the C++ host examples (examples/*.cpp) against the C ABI."""
    out = []
    ex_dir = os.path.join(REPO_DIR, "examples")
    if not os.path.isdir(ex_dir):
        return out
    for name in sorted(os.listdir(ex_dir)):
        if not name.endswith(".cpp"):
            continue
        src = os.path.join(ex_dir, name)
        exe = os.path.join(ex_dir, name[:-4])
        deps = [src, LIB_PATH, os.path.join(REPO_DIR, "include", "safe_gossip.h"),
                os.path.join(REPO_DIR, "include", "safe_gossip.hpp")]
        if force or _stale(exe, [d for d in deps if os.path.exists(d)]):
            subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror",
                            "-I", os.path.join(REPO_DIR, "include"), "-o", exe, src,
                            "-L", PKG_DIR, "-lsafe_gossip_amd", f"-Wl,-rpath,{PKG_DIR}"],
                           check=True)
        out.append(exe)
    return out


if __name__ == "__main__":
    print(build_engine(force="--force" in sys.argv, verbose=True))
    for e in build_examples(force="--force" in sys.argv):
        print(e)
