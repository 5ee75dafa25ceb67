"""CPU: the C-ABI library builds for gfx950, loads, and exports every symbol that
include/merlin_hip.h declares.  Host-only entry points run here (no GPU calls)."""
import os
import re
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "merlin_hip.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(merlin_\w+)\s*\(", src, re.M)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    assert "merlin_env_step" in syms and "merlin_gae" in syms and len(syms) >= 15


def test_library_exports_every_declared_symbol():
    from merlin import _native as nat

    L = nat.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", nat.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (merlin_\w+)", out))
    assert set(declared_symbols()) <= exported
    assert set(nat.EXPORTED_SYMBOLS) <= exported


def test_library_has_gfx950_code_object():
    from merlin import _native as nat

    data = open(nat.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_atlas(golden):
    from merlin import _native as nat

    assert nat.lib().merlin_version() == nat.ABI_VERSION == 3
    # the library's own C++ restatement of render_tile == the numpy restatement golden
    assert (nat.tile_atlas() == golden("atlas")["atlas"]).all()


def test_errors_are_reported_not_thrown():
    import ctypes as C

    from merlin import _native as nat

    L = nat.lib()
    cfg = nat.EnvConfig(0, 16, 2, 0, 0, 3, -0.1, 0, 0.0)  # num_envs = 0 is invalid
    h = C.c_void_p()
    rc = L.merlin_env_create(C.byref(cfg), C.byref(h))
    assert rc == 1 and b"num_envs" in L.merlin_last_error()
    cfg = nat.EnvConfig(4, 40, 2, 0, 0, 3, -0.1, 0, 0.0)
    assert L.merlin_env_create(C.byref(cfg), C.byref(h)) == 4  # size > 32 unsupported


def test_act_heads_draw_requires_epoch_counter():
    """a sampled action without the epoch counter would repeat its draws every call."""
    import torch

    from merlin import _native as nat

    z = torch.zeros(2, 4, 8)
    b4 = torch.zeros(2, 8)
    wa, ba, wc, bc = torch.zeros(3, 8), torch.zeros(3), torch.zeros(1, 8), torch.zeros(1)
    with pytest.raises(ValueError, match="epoch"):
        nat.act_heads(z, b4, wa, ba, wc, bc, deterministic=False)


def test_env_config_binding_matches_the_c_struct():
    """VERDICT r1 boundary defect: the ctypes restatement of merlin_env_config (the one
    INTEGRATION.md tells a reference maintainer to paste) must have the C struct's size and field
    offsets; merlin_env_create reads every field."""
    import ctypes as C

    from merlin import _native as nat

    size, offs = nat.env_config_layout()
    assert size == C.sizeof(nat.EnvConfig)
    assert offs == [getattr(nat.EnvConfig, f).offset for f, _ in nat.EnvConfig._fields_]
    hdr = open(HEADER).read()
    assert int(re.search(r"#define MERLIN_ENV_CONFIG_FIELDS (\d+)", hdr).group(1)) == len(nat.EnvConfig._fields_)
    # the binding printed in INTEGRATION.md declares the same fields in the same order
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    block = doc[doc.index("class MerlinEnvConfig"):]
    block = block[:block.index("]")]
    assert re.findall(r'\("(\w+)"', block) == [f for f, _ in nat.EnvConfig._fields_]


def test_x6_gemm_argument_checks():
    """fc1's x6 GEMM entry points reject bad shapes on the host (no device work is queued)."""
    from merlin import _native as nat

    L = nat.lib()
    # K not a multiple of 32
    assert L.merlin_x6_gemm_nt(None, None, 0, 512, 33, 2, 0, 0, None, None, 0, 0, None) == 4
    # null operands with rows to do
    assert L.merlin_x6_gemm_nt(None, None, 10, 512, 576, 2, 0, 0, None, None, 0, 0, None) == 1
    assert L.merlin_x6_gemm_tn(None, None, 10, 512, 576, 2, 0, 0, 32, None, None, 0, None) == 1
    # planes need groups of 8 values
    assert L.merlin_x6_split(None, 7, None, None) == 1
    assert L.merlin_x6_tn_slab_floats(512, 576, 2, 32) == 32 * 2 * 512 * 576
    # colsum: rows of 4 x a divisor of 256 floats only
    assert L.merlin_tower_colsum(None, 0, 7, 7, 0, 1, None, None) == 1


def test_clip_adam_argument_checks():
    """merlin_clip_adam rejects bad tensor lists on the host (no device work is queued)."""
    import ctypes as C

    from merlin import _native as nat

    L = nat.lib()
    numel = (C.c_int64 * 3)(10, 4096, 5000)
    assert L.merlin_clip_adam_workspace(3, numel) == 1 + 4 + 5  # 1024-element blocks per tensor
    assert L.merlin_clip_adam_workspace(33, numel) == -1
    assert L.merlin_clip_adam(0, None, None, None, None, None, None, 1e-3, 0.9, 0.999, 1e-8, 0.5, None, None, None) == 1
    assert L.merlin_clip_adam(33, None, None, None, None, None, None, 1e-3, 0.9, 0.999, 1e-8, 0.5, None, None, None) == 1
    nul = (C.c_void_p * 3)()
    ws = (C.c_double * 4)()
    # null tensor pointers
    assert L.merlin_clip_adam(3, nul, nul, nul, nul, nul, numel, 1e-3, 0.9, 0.999, 1e-8, 0.5, None, ws, None) == 1
    # an empty tensor
    zero = (C.c_int64 * 3)(10, 0, 5)
    assert L.merlin_clip_adam(3, nul, nul, nul, nul, nul, zero, 1e-3, 0.9, 0.999, 1e-8, 0.5, None, ws, None) == 1
