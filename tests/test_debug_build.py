"""SURVEY.md section 5's debug target (marl-sat_amd/Makefile `debug`).

CPU: the C-ABI host glue built under AddressSanitizer (tests/capi_host_check.cpp linked against the library's
objects compiled with -Xarch_host -fsanitize=address) rejects bad arguments through the error channel, with no
ASan report.

GPU: libmarlsat_debug.so (every kernel with -DMSAT_DEBUG device bounds checks; each launch synchronised and
checked) runs the clause-cell GRU backward bitwise like the product library, and reports an undersized partial
buffer and an unwritten (NaN-poisoned) feature row as errors naming the check.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

LIBDIR = os.path.join(ROOT, "marl-sat_amd", "marlsat", "lib")
ASAN_BIN = os.path.join(ROOT, "marl-sat_amd", "build", "asan", "capi_host_check")


STATUS = os.path.join(LIBDIR, "debug_build_status.json")  # written by __graft_entry__.build()


def _require_built(path, what):
    """Skip only when no build ran here (no status record); a build() whose 'make debug' failed is a failure,
    not a skip, so a broken debug build cannot silently drop the device bounds checks' coverage."""
    if os.path.exists(path):
        return
    if os.path.exists(STATUS):
        import json

        st = json.load(open(STATUS))
        pytest.fail(f"{what} missing: __graft_entry__.build()'s 'make debug' exited {st.get('make_debug_rc')}")
    pytest.skip(f"{what} not built (make -C marl-sat_amd debug; __graft_entry__.build() does)")


def test_capi_host_glue_under_asan():
    _require_built(ASAN_BIN, "ASan driver build/asan/capi_host_check")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=23")
    r = subprocess.run([ASAN_BIN], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "capi_host_check: ok" in r.stdout
    assert "AddressSanitizer" not in r.stderr


def _bwd_args(torch, R, H, nfeat, feat, part):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(5)
    dy = torch.randn(R, H, device=dev, generator=g)
    g4 = torch.randn(R, 4 * H, device=dev, generator=g)
    hp = torch.randn(R, H, device=dev, generator=g)
    sc = torch.randn(H, device=dev, generator=g)
    D = torch.empty(R, 4 * H, device=dev)
    dh = torch.empty(R, H, device=dev)
    dln = torch.zeros(2 * H, device=dev)
    dbi = torch.zeros(3 * H, device=dev)
    dbh = torch.zeros(3 * H, device=dev)
    dfeat = torch.zeros(nfeat, 3 * H, device=dev)
    rexp = torch.empty(R, dtype=torch.int32, device=dev)
    keep = (dy, g4, hp, sc, D, dh, dln, dbi, dbh, dfeat, rexp, feat, part)
    args = (dy.data_ptr(), H, g4.data_ptr(), 4 * H, hp.data_ptr(), H, sc.data_ptr(), D.data_ptr(), 4 * H,
            D.data_ptr() + 4 * H, 4 * H, dh.data_ptr(), H, dln.data_ptr(), dln.data_ptr() + 4 * H, dbi.data_ptr(),
            dbh.data_ptr() + 4 * 2 * H, feat.data_ptr(), feat.shape[1], nfeat, dfeat.data_ptr(), part.data_ptr(), R, H,
            7, rexp.data_ptr())
    return args, {"D": D, "dh": dh, "dln": dln, "dbi": dbi, "dbh": dbh, "dfeat": dfeat, "rexp": rexp}, keep


@pytest.mark.gpu
def test_debug_library_checks_the_gru_backward():
    import torch

    from marlsat import _lib

    path = os.path.join(LIBDIR, "libmarlsat_debug.so")
    _require_built(path, "libmarlsat_debug.so")
    dbg = ctypes.CDLL(path)
    for lib in (dbg,):
        lib.msat_gru_ln_bwd_g4fe.restype = ctypes.c_int32
        lib.msat_gru_ln_bwd_g4fe.argtypes = _lib.lib.msat_gru_ln_bwd_g4fe.argtypes
        lib.msat_gru_ln_bwd_partial_floats.restype = ctypes.c_size_t
        lib.msat_gru_ln_bwd_partial_floats.argtypes = [ctypes.c_int32, ctypes.c_int32]
        lib.msat_last_error.restype = ctypes.c_char_p
    R, H, nfeat = 20000, 128, 2  # the clause cell's form (msat_gru_ln_bwd_g4fe, nfeat 2)
    s = _lib.stream_ptr()
    feat = torch.randint(0, 3, (R, 4), device="cuda").float()
    cap = int(dbg.msat_gru_ln_bwd_partial_floats(R, H))
    assert cap == int(_lib.lib.msat_gru_ln_bwd_partial_floats(R, H))
    part = torch.empty(cap, device="cuda")
    outs = {}
    for name, lib in (("product", _lib.lib), ("debug", dbg)):
        args, out, keep = _bwd_args(torch, R, H, nfeat, feat, part)
        assert lib.msat_gru_ln_bwd_g4fe(*args, s) == 0, lib.msat_last_error()
        torch.cuda.synchronize()
        outs[name] = {k: v.clone() for k, v in out.items()}
    for k in outs["product"]:
        assert torch.equal(outs["product"][k], outs["debug"][k]), k
    # an allocation smaller than msat_gru_ln_bwd_partial_floats: refused before the launch.  Allocated by
    # hipMalloc itself, so its extent is its own (a torch tensor may be carved from a larger cached segment)
    hip = ctypes.CDLL("libamdhip64.so")
    raw = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(raw), ctypes.c_size_t(4 * (cap // 2))) == 0

    class Small:  # the one attribute _bwd_args reads of the partial buffer
        def data_ptr(self):
            return raw.value

    try:
        args, _, keep = _bwd_args(torch, R, H, nfeat, feat, Small())
        assert dbg.msat_gru_ln_bwd_g4fe(*args, s) == -1
        assert b"partial buffer smaller" in dbg.msat_last_error()
    finally:
        torch.cuda.synchronize()
        hip.hipFree(raw)
    # an unwritten feature row (NaN, as MARLSAT_DEBUG=1 assembly poisons them): the device check names its row
    bad = feat.clone()
    bad[12345, 1] = float("nan")
    args, _, keep = _bwd_args(torch, R, H, nfeat, bad, part)
    assert dbg.msat_gru_ln_bwd_g4fe(*args, s) == -2
    msg = dbg.msat_last_error().decode()
    assert "MSAT_DEBUG: gru_ln_bwd_kernel" in msg and "index -12346 outside [0, 20000)" in msg, msg
    # the next call is clean again (the failure record is reset when reported)
    args, out, keep = _bwd_args(torch, R, H, nfeat, feat, part)
    assert dbg.msat_gru_ln_bwd_g4fe(*args, s) == 0, dbg.msat_last_error()
    torch.cuda.synchronize()
    assert np.array_equal(out["dfeat"].cpu().numpy(), outs["product"]["dfeat"].cpu().numpy())


TRAIN_SCRIPT = r"""
import sys, torch
sys.path[:0] = [{root!r}, {root!r} + '/marl-sat_amd']
from marlsat import _lib
assert _lib.LIB_PATH.endswith('libmarlsat_debug.so'), _lib.LIB_PATH
from marlsat import SATEnv
from marlsat.learners.gnn import GNNActorCritic
from marlsat.learners.mappo_gnn_sat_learner import MAPPOLearner
from marlsat.random import PRNGKey
from marlsat.utils.generate_cnf_dataset import generate_problem_pool
cfg = dict(NUM_ENVS=4, NUM_STEPS=2, NUM_UPDATES=10, UPDATE_EPOCHS=1, MINIBATCH_SIZE=4, LEARNING_RATE=3e-3,
           GAMMA=0.99, GAE_LAMBDA=0.95, CLIP_EPS=0.2, ENT_COEF=0.01, VF_COEF=0.5, VF_CLIP=0.2, ANNEAL_LR=True,
           LR_START_FACTOR=1.0, LR_END_FLOOR=1e-5, GNN_HIDDEN_DIM=128, GNN_NUM_MESSAGE_PASSING_STEPS=2, action_mode=0)
env = SATEnv(50, 218, max_steps=2, vars_per_agent=10)
pool = env.make_pool(generate_problem_pool(50, 218, 4, size_id=12, skip_isolated=True))
net = GNNActorCritic(128, 2, env.num_agents, env.max_vars_per_agent, 0, 50, device="cuda", seed=4)
learner = MAPPOLearner(cfg, env, net, pool)
rs = learner.init_runner_state(PRNGKey(1))
rs, metrics = learner.train_cycle(rs, 0, torch.Generator().manual_seed(7))
assert torch.isfinite(net.params).all()
print("debug train cycle ok", _lib.LIB_PATH)
"""


@pytest.mark.gpu
def test_debug_library_runs_a_train_cycle():
    """A small train cycle (uf50, H = 128, L = 2: env steps, batch assembly with NaN-poisoned feature rows,
    gathers, GRU forward / backward, reductions, GEMMs, Adam) on libmarlsat_debug.so with MARLSAT_DEBUG=1 (every
    launch synchronised and its device bounds checks read back; host-side planned-vs-actual totals), in a child
    process so that the library it loads is the debug one."""
    import sys

    path = os.path.join(LIBDIR, "libmarlsat_debug.so")
    _require_built(path, "libmarlsat_debug.so")
    env = dict(os.environ, MARLSAT_LIB=path, MARLSAT_DEBUG="1")
    r = subprocess.run([sys.executable, "-c", TRAIN_SCRIPT.format(root=ROOT)], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "debug train cycle ok" in r.stdout and "libmarlsat_debug.so" in r.stdout
