"""CPU tests of the C-ABI boundary: the library loads, exports exactly what
include/marlsat.h declares, and rejects bad arguments through the error channel
(no GPU work is launched by these calls)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _header_symbols():
    import glob

    text = "".join(open(f).read() for f in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(msat_[a-z_0-9]+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    from marlsat import _lib

    syms = _header_symbols()
    assert len(syms) >= 11
    for s in syms:
        assert hasattr(_lib.lib, s), s
    assert sorted(_lib.EXPORTED) == syms
    assert _lib.lib.msat_version() == 3  # msat_env_state with reset_queue / reset_serial (include/marlsat.h)


def test_nm_lists_c_abi_symbols():
    from marlsat import _lib

    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for s in _header_symbols():
        assert re.search(rf"\bT {s}$", out, re.M), s


def _desc(**kw):
    from marlsat import _lib

    d = dict(num_envs=4, num_vars=20, num_clauses=91, clause_width=3, num_agents=2, max_vars_per_agent=10,
             max_steps=512, action_mode=0, reward_mode=0, obs_dtype=0, num_problems=1, r_clause=0.0, r_sat=1.0,
             gamma=0.99)
    d.update(kw)
    return _lib.EnvDesc(**d)


@pytest.mark.parametrize("bad,msg", [
    (dict(num_vars=0), "num_vars"),
    (dict(clause_width=4), "clause_width"),
    (dict(num_agents=1001), "num_agents"),
    (dict(max_vars_per_agent=9), "max_vars_per_agent"),
    (dict(action_mode=2), "action_mode"),
    (dict(obs_dtype=3), "obs_dtype"),
])
def test_bad_desc_is_rejected_with_message(bad, msg):
    from marlsat import _lib

    st = _lib.EnvStateC(*([1] * 7))  # never dereferenced: validation fails first
    pool = _lib.PoolC(1, 1, 1)
    rc = _lib.lib.msat_env_reset(ctypes.byref(_desc(**bad)), ctypes.byref(pool), ctypes.byref(st), None, None, None, 0,
                                 0, 1, None)
    assert rc == -1
    assert msg in _lib.lib.msat_last_error().decode()


def test_null_state_pointer_rejected():
    from marlsat import _lib

    st = _lib.EnvStateC(1, 1, None, 1, 1, 1, None)  # problem_idx missing
    pool = _lib.PoolC(1, 1, 1)
    rc = _lib.lib.msat_env_reset(ctypes.byref(_desc()), ctypes.byref(pool), ctypes.byref(st), None, None, None, 0, 0,
                                 1, None)
    assert rc == -1 and "NULL" in _lib.lib.msat_last_error().decode()
    st = _lib.EnvStateC(1, 1, None, 1, 1, 1, 1)
    pool = _lib.PoolC(1, None, 1)  # relation table missing
    rc = _lib.lib.msat_env_reset(ctypes.byref(_desc()), ctypes.byref(pool), ctypes.byref(st), None, None, None, 0, 0,
                                 1, None)
    assert rc == -1 and "pool" in _lib.lib.msat_last_error().decode()


def test_reset_queue_size_and_alignment():
    """msat_reset_queue_words: a pending token per env and parity; a queue pointer that is not 16-byte aligned is
    refused before any launch."""
    from marlsat import _lib

    for B in (0, 1, 1024, 4096):
        assert _lib.lib.msat_reset_queue_words(B) == 2 * B
    st = _lib.EnvStateC(8, 8, None, 8, 8, 8, 8, 12, 0)  # never dereferenced: the alignment check fails first
    out = _lib.StepOutC(8, 8, 8, None, None, None)
    rc = _lib.lib.msat_env_step(ctypes.byref(_desc()), ctypes.byref(_lib.PoolC(8, 8, 8)), ctypes.byref(st), 8, 1,
                                None, None, 0, 0, ctypes.byref(out), None, None)
    assert rc == -1 and "16-byte aligned" in _lib.lib.msat_last_error().decode()


def test_gae_bad_dims_rejected():
    from marlsat import _lib

    rc = _lib.lib.msat_gae(0, 4, 1, 1, 1, 1, 1, 0.99, 0.9, 1, 1, 1, 1, None)
    assert rc == -1 and "bad dims" in _lib.lib.msat_last_error().decode()
    assert _lib.lib.msat_gae_workspace_bytes(8, 1000) >= 16 * 4


def test_product_path_does_not_import_oracle():
    pkg = os.path.join(ROOT, "marl-sat_amd", "marlsat")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f


def test_ctypes_argtypes_match_header_prototypes():
    """Every ctypes binding in marlsat/_lib.py passes as many arguments as its include/*.h prototype
    declares (the compiler checks the prototypes against the extern "C" definitions: csrc/common.h
    includes both headers)."""
    import glob

    from marlsat import _lib

    text = "".join(open(f).read() for f in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    protos = dict(re.findall(r"\b(msat_[a-z_0-9]+)\s*\(([^)]*)\)\s*;", text))
    assert sorted(protos) == _header_symbols()
    for name, params in protos.items():
        params = params.strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        argtypes = getattr(_lib.lib, name).argtypes
        assert argtypes is not None and len(argtypes) == n, (name, n, argtypes)


def test_collective_entry_points_reject_bad_arguments():
    """msat_comm_init / msat_allreduce_sum argument checks run before any RCCL call."""
    from marlsat import _lib

    L = _lib.lib
    assert L.msat_comm_id_bytes() == 128
    h = ctypes.c_void_p()
    uid = (ctypes.c_uint8 * 128)()
    assert L.msat_comm_init(uid, 0, 0, ctypes.byref(h)) == -1
    assert b"world" in L.msat_last_error()
    assert L.msat_comm_init(uid, 2, 2, ctypes.byref(h)) == -1
    assert L.msat_allreduce_sum(None, None, 4, 0, None) == -1
    assert b"communicator" in L.msat_last_error()
    assert L.msat_comm_destroy(None) == 0


def test_library_does_not_link_rccl():
    """RCCL is opened lazily by msat_comm_* (comm.hip): a host that only steps environments loads
    libmarlsat.so without librccl installed."""
    import shutil
    import subprocess

    if shutil.which("readelf") is None:
        pytest.skip("readelf not available")
    lib = os.path.join(ROOT, "marl-sat_amd", "marlsat", "lib", "libmarlsat.so")
    out = subprocess.run(["readelf", "-d", lib], capture_output=True, text=True, check=True).stdout
    needed = [l for l in out.splitlines() if "(NEEDED)" in l]
    assert needed and not any("rccl" in l for l in needed), needed


def test_precision_entry_points_validate():
    """msat_set_precision / msat_get_precision (include/marlsat_net.h): the weight gradients' path is set
    once and validated; an unknown mode is MSAT_EBADARG with a message, not a silent fallback."""
    from marlsat import _lib
    from marlsat.learners import gnn

    L = _lib.lib
    assert L.msat_get_precision() == gnn.PRECISION_CODES[gnn.PRECISION]
    assert L.msat_set_precision(7) == -1
    assert b"unknown mode" in L.msat_last_error()
    assert L.msat_get_precision() == gnn.PRECISION_CODES[gnn.PRECISION]  # unchanged by the bad call
    try:
        for code in (2, 1, 0):
            assert L.msat_set_precision(code) == 0
            assert L.msat_get_precision() == code
    finally:
        L.msat_set_precision(gnn.PRECISION_CODES[gnn.PRECISION])


def test_unknown_precision_env_fails_loudly_in_a_c_host():
    """A C-ABI host that never calls msat_set_precision gets MARLSAT_PRECISION read once; a mistyped value
    makes msat_get_precision (and every weight gradient) return MSAT_EBADARG naming the value."""
    import subprocess
    import sys

    from marlsat import _lib

    code = ("import ctypes; L = ctypes.CDLL(%r); L.msat_last_error.restype = ctypes.c_char_p; "
            "rc = L.msat_get_precision(); print(rc, L.msat_last_error().decode())") % _lib.LIB_PATH
    for val, want in (("fp16X2", None), ("fp32", "2"), ("bf16x3", "1"), ("", "0")):
        env = dict(os.environ, MARLSAT_PRECISION=val)
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stderr
        rc, _, msg = out.stdout.strip().partition(" ")
        if want is None:
            assert rc == "-1" and "fp16X2" in msg, out.stdout
        else:
            assert rc == want, out.stdout
