"""The C-ABI library: loads, exports every symbol include/safe_gossip.h
declares, host-side helpers agree with the oracle, and the product fails
loudly (no CPU fallback) when no GPU is present."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "safe_gossip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gs_[a-z_0-9]+)\s*\(", text)))


def test_header_symbols_exported(engine):
    lib = engine.load_library()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    # the Python binding declares a signature for every header symbol
    assert set(syms) == set(engine.SYMBOLS)


def test_exported_symbols_nm(engine):
    from safe_gossip_amd.build import LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gs_[a-z_0-9]+)\b", out))
    assert set(declared_symbols()) <= exported


def test_build_provenance(engine, tmp_path):
    # the library carries the hash of the sources it was built from and the
    # ABI version; load_library refuses a library built from other sources
    from safe_gossip_amd import build
    lib = engine.load_library()
    assert lib.gs_abi_version() == engine.ABI_VERSION == 2
    assert engine.build_id() == build.source_hash()
    assert open(build.LIB_PATH + ".buildid").read().strip() == build.source_hash()
    # a tree whose sources differ by one byte has another id
    root = tmp_path / "tree"
    for f in build.SOURCES + build.HEADERS:
        rel = os.path.relpath(f, REPO)
        (root / rel).parent.mkdir(parents=True, exist_ok=True)
        (root / rel).write_bytes(open(f, "rb").read())
    assert build.source_hash(str(root)) == build.source_hash()
    hdr = root / "include" / "safe_gossip.h"
    hdr.write_bytes(hdr.read_bytes() + b" ")
    assert build.source_hash(str(root)) != build.source_hash()


def test_derive_params_equal_oracle(engine, oracle):
    for n in list(range(1, 100)) + [1618, 1619, 2000, 5000, 10**4, 10**6, 2**24, 10**8,
                                    528491311, 2**32 - 2]:
        assert engine.derive_params(n) == oracle_lib.derive_params(n), n


def test_status_strings(engine):
    lib = engine.load_library()
    assert b"no connected peers" in lib.gs_status_string(1)
    assert b"before sending" in lib.gs_status_string(2)


def _has_gpu():
    return os.path.exists("/dev/kfd")


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure mode")
def test_fails_loudly_without_gpu(engine):
    with pytest.raises(engine.DeviceError):
        engine.Network(8, 3)


def test_invalid_config_rejected(engine):
    lib = engine.load_library()
    from safe_gossip_amd import _Config
    cfg = _Config()
    cfg.n_nodes = 10
    cfg.n_rumors = 0
    h = ctypes.c_void_p()
    assert lib.gs_create(ctypes.byref(cfg), ctypes.byref(h)) == -1
    cfg.n_rumors = 5000
    assert lib.gs_create(ctypes.byref(cfg), ctypes.byref(h)) == -1
    cfg.n_rumors = 8
    cfg.counter_max, cfg.max_c_rounds, cfg.max_rounds = 4, 3, 10
    assert lib.gs_create(ctypes.byref(cfg), ctypes.byref(h)) == -2   # unsupported layout
    cfg.counter_max, cfg.max_c_rounds, cfg.max_rounds = 3, 3, 33
    assert lib.gs_create(ctypes.byref(cfg), ctypes.byref(h)) == -2


def test_node_ids_beyond_target_word_rejected(engine):
    # t(x) is packed into 29 bits of the target word (gs_common.h kTgMask):
    # a network above 2^29 nodes is refused whatever the parameters, before
    # any device call (so this runs without a GPU).
    with pytest.raises(engine.DeviceError, match="status -2"):
        engine.Network((1 << 29) + 1, 1, params=(3, 3, 21))
    with pytest.raises(engine.DeviceError, match="status -2"):
        engine.Network(0xFFFFFFFE, 1, params=(3, 3, 21))


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure mode")
def test_net_fails_loudly_without_gpu(engine):
    # the library's multi-GPU loop has no CPU path either
    from safe_gossip_amd.net import Net
    with pytest.raises(engine.DeviceError):
        Net(64, 8, 2, mode="shards", transport="local")
    with pytest.raises(engine.DeviceError):
        Net(64, 8, 2, mode="slices", transport="local")


def test_net_invalid_arguments(engine):
    # argument checks run before any device call
    lib = engine.load_library()
    from safe_gossip_amd import _Config
    cfg = _Config()
    cfg.n_nodes, cfg.n_rumors = 100, 4
    h = ctypes.c_void_p()
    assert lib.gs_net_create_local(ctypes.byref(cfg), 0, 0, 1, ctypes.byref(h)) == -1   # no ranks
    assert lib.gs_net_create_local(ctypes.byref(cfg), 0, 5, 1, ctypes.byref(h)) == -1   # 4 rumors, 5 slices
    assert lib.gs_net_create_local(ctypes.byref(cfg), 7, 2, 1, ctypes.byref(h)) == -1   # no such mode
    cfg.schedule = 1
    assert lib.gs_net_create_local(ctypes.byref(cfg), 1, 2, 1, ctypes.byref(h)) == -2   # SEQ: slices only
    cfg.schedule, cfg.rumor_slice = 0, 1
    assert lib.gs_net_create_local(ctypes.byref(cfg), 1, 2, 1, ctypes.byref(h)) == -1   # a slice is not a network
    ident = (ctypes.c_uint8 * 128)()
    cfg.rumor_slice = 0
    assert lib.gs_net_create(ctypes.byref(cfg), 1, 2, 2, 1, ident, ctypes.byref(h)) == -1  # rank >= world
    assert lib.gs_net_send_new(None, 0, 0) == -1
    assert lib.gs_net_next_round(None, None) == -1
    assert lib.gs_net_local_engines(None) == 0
