"""Diagnostic: where the dual data gradient's k steps spend their cycles.  Needs a library built from
gemm_x3.hip with the s_memtime stamps of profiles/archive_r03/dgrad_stamp.patch (MARLSAT_LIB=...), which adds
msat_debug_dgrad_stamps.  Runs profiles/dual_bench.py's clause-shape dual data gradient once more after its
timing and prints each phase's share of a wave's cycles (shares only: the stamps' waits forbid overlaps
the real kernel has).  usage: dgrad_stamps.py [rows]"""
import ctypes
import json
import os
import runpy
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = [sys.argv[0], sys.argv[1] if len(sys.argv) > 1 else "1316000", "2"]
g = runpy.run_path(os.path.join(ROOT, "profiles", "dual_bench.py"))
torch, L, fd, M = g["torch"], g["L"], g["fd"], g["M"]
L.msat_debug_dgrad_stamps.restype = ctypes.c_int
L.msat_debug_dgrad_stamps.argtypes = [ctypes.c_void_p]
SEG, CAP = 8, 16384 * 8
assert fd() == 0
torch.cuda.synchronize()
buf = np.zeros(CAP * SEG, dtype=np.uint64)
assert L.msat_debug_dgrad_stamps(buf.ctypes.data) == 0
st = buf.reshape(CAP, SEG).astype(np.float64)
st = st[st[:, 7] > 0]
total = st[:, 7]
names = ["prologue", "A split", "DMA issue + A loads", "MFMA blocks", "vmcnt wait", "barrier"]
share = {n: round(float((st[:, k] / total).mean()), 4) for k, n in enumerate(names)}
share["epilogue (rescale, stage, stores)"] = round(float(((total - st[:, 0] - st[:, 6]) / total).mean()), 4)
print(json.dumps({"what": "dual dgrad stamps", "rows": M, "waves": int(st.shape[0]),
                  "wave_cycles": float(total.mean()), "shares": share}), flush=True)
