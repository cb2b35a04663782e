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
           os.path.join(CSRC, "gs_engine.cpp"), os.path.join(CSRC, "gs_wire.cpp"),
           os.path.join(CSRC, "gs_sign.cpp")]
HEADERS = [os.path.join(CSRC, f) for f in ("gs_common.h", "gs_kernels.h", "gs_device.h", "gs_recv.h")] + [
    os.path.join(REPO_DIR, "include", "safe_gossip.h")
]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


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
    if not force and not defines and not _stale(target, SOURCES + HEADERS):
        return target
    flags = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-Wall", "-Wextra", "-Werror"] + [
        f"-D{d}" for d in defines]
    tag = "product" if not defines else "_".join(sorted(defines)).replace("=", "-")
    bdir = os.path.join(PKG_DIR, "build", tag)
    os.makedirs(bdir, exist_ok=True)
    objs, jobs = [], []
    for src in SOURCES:
        obj = os.path.join(bdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + HEADERS):
            jobs.append((src, obj))
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(max_workers=workers) as ex:
        for f in [ex.submit(_compile, s_, o_, flags, verbose) for s_, o_ in jobs]:
            f.result()
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", target + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(target + ".tmp", target)
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
