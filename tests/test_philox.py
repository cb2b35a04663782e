"""The injected peer schedule: Philox4x32-10 in the product and in the oracle.

Both are checked against the Random123 KATs and against rocrand's own
philox4x32_10 engine (compiled on the host from /opt/rocm/include), and the
product's host entry points (gs_peer / gs_origin / gs_coin) must equal the
oracle's on many counters.
"""
import ctypes
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle_lib

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "kat_reference.json")))

ROCRAND_PROBE = r"""
#include <hip/hip_runtime.h>
#include <rocrand/rocrand_philox4x32_10.h>
#include <cstdio>
#include <cstdlib>
struct probe : rocrand_device::philox4x32_10_engine {
  uint4 run(uint4 c, uint2 k) { return ten_rounds(c, k); }
};
int main(int argc, char** argv) {
  probe p;
  for (int i = 1; i + 5 < argc + 1; i += 6) {
    uint4 c = {(unsigned)strtoul(argv[i],0,0), (unsigned)strtoul(argv[i+1],0,0),
               (unsigned)strtoul(argv[i+2],0,0), (unsigned)strtoul(argv[i+3],0,0)};
    uint2 k = {(unsigned)strtoul(argv[i+4],0,0), (unsigned)strtoul(argv[i+5],0,0)};
    uint4 o = p.run(c, k);
    printf("%u %u %u %u\n", o.x, o.y, o.z, o.w);
  }
  return 0;
}
"""


def test_random123_kats(oracle):
    for case in GOLDEN["philox"]:
        assert list(oracle_lib.philox(case["ctr"], case["key"])) == case["expect"]


@pytest.fixture(scope="module")
def rocrand_probe(tmp_path_factory):
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    d = tmp_path_factory.mktemp("rocrand")
    src = d / "probe.cpp"
    src.write_text(ROCRAND_PROBE)
    exe = d / "probe"
    subprocess.run([hipcc, "-O1", "-x", "hip", "--offload-arch=gfx950", "-o", str(exe), str(src)],
                   check=True, capture_output=True)
    return str(exe)


def test_matches_rocrand(oracle, rocrand_probe):
    rng = np.random.default_rng(1234)
    vecs = [c["ctr"] + c["key"] for c in GOLDEN["philox"]]
    vecs += [list(map(int, rng.integers(0, 2**32, 6))) for _ in range(64)]
    args = [str(v) for vec in vecs for v in vec]
    try:
        out = subprocess.run([rocrand_probe] + args, check=True, capture_output=True, text=True,
                             timeout=60).stdout.split("\n")
    except (subprocess.CalledProcessError, OSError) as e:
        pytest.skip(f"host probe could not run: {e}")
    for vec, line in zip(vecs, out):
        got = [int(t) for t in line.split()]
        assert got == list(oracle_lib.philox(vec[:4], vec[4:])), vec


def test_engine_schedule_equals_oracle(oracle, engine):
    L = oracle_lib.lib()
    rng = np.random.default_rng(7)
    for _ in range(2000):
        seed = int(rng.integers(0, 2**63))
        epoch = int(rng.integers(0, 2**32))
        rnd = int(rng.integers(0, 2**32))
        n = int(rng.integers(2, 2**32 - 1))
        x = int(rng.integers(0, n))
        t = engine.peer_of(seed, epoch, rnd, x, n)
        assert t == L.or_peer(seed, epoch, rnd, x, n)
        assert t != x and 0 <= t < n
        assert engine.origin_of(seed, epoch, rnd, n) == L.or_origin(seed, epoch, rnd, n)
        assert engine.coin_of(seed, epoch, rnd, x) == L.or_coin(seed, epoch, rnd, x)


def test_peer_choice_is_uniform_over_others(engine):
    # choose(&peers) is uniform over the n-1 other nodes (src/gossiper.rs:71).
    n, trials = 7, 70000
    cnt = np.zeros((n, n), dtype=np.int64)
    for r in range(trials // n):
        for x in range(n):
            cnt[x, engine.peer_of(99, 0, r, x, n)] += 1
    assert np.all(np.diag(cnt) == 0)
    off = cnt[~np.eye(n, dtype=bool)]
    expect = trials / n / (n - 1)
    assert np.all(np.abs(off - expect) < 6 * np.sqrt(expect))


def test_torch_philox_matches_oracle():
    # the vectorised torch Philox (tests/philox_torch.py) used by the
    # full-size property tests equals the oracle's on KATs and random counters
    import numpy as np
    import torch
    import philox_torch as pt
    import oracle_lib
    L = oracle_lib.lib()
    rng = np.random.default_rng(5)
    for seed in (0, 0x5AFE6055, 0xFFFFFFFFFFFFFFFF, 2**63 + 5):
        ctr = rng.integers(0, 2**32, size=(64, 4), dtype=np.uint64)
        got = pt.philox4x32(*(torch.tensor(ctr[:, i].astype(np.int64)) for i in range(4)), seed)
        for i in range(64):
            exp = oracle_lib.philox([int(v) for v in ctr[i]], [seed & 0xFFFFFFFF, seed >> 32])
            assert [int(g[i]) for g in got] == list(exp)
    nodes = torch.arange(0, 5000, dtype=torch.int64)
    for n in (5000, 2**24):
        nn = nodes if n == 5000 else nodes * 3355
        peers = pt.peer_of(0x5AFE6055, 3, 7, nn, n)
        for x in range(0, 5000, 97):
            assert int(peers[x]) == L.or_peer(0x5AFE6055, 3, 7, int(nn[x]), n)
    thr = [oracle_lib.fault_threshold(p) for p in (0.3, 0.2, 0.1)]
    fb = pt.fault_bits(0x5AFE6055, 1, 4, nodes, *thr)
    for x in range(0, 5000, 13):
        assert int(fb[x]) == L.or_fault(0x5AFE6055, 1, 4, x, *thr)
