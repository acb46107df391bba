"""Probe (not collected): msat_gru_ln_bwd_g4fe repeated on identical inputs (clause shape, nfeat 2; var
shape, nfeat 6); every output must be bitwise equal across repetitions.  Run two copies at once to load the
GPU.  usage: probe_bwd_determinism.py [rows] [reps]"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-sat_amd")]
import torch  # noqa: E402

from marlsat import _lib  # noqa: E402

L = _lib.lib
R = int(sys.argv[1]) if len(sys.argv) > 1 else 400000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
H = 128
torch.cuda.set_device(0)
g = torch.Generator(device="cuda").manual_seed(0)
s = _lib.stream_ptr()
for nfeat in (2, 6):
    dy = torch.randn(R, H, device="cuda", generator=g)
    g4 = torch.randn(R, 4 * H, device="cuda", generator=g)
    hp = torch.randn(R, H, device="cuda", generator=g)
    sc = torch.randn(H, device="cuda", generator=g)
    feat = torch.randn(R, 8, device="cuda", generator=g)
    part = torch.empty(int(L.msat_gru_ln_bwd_partial_floats(R, H)), device="cuda")
    ref = None
    for r in range(reps):
        D = torch.empty(R, 4 * H, device="cuda")
        dh = torch.empty(R, H, device="cuda")
        dln = torch.zeros(2 * H, device="cuda")
        dbi = torch.zeros(3 * H, device="cuda")
        dbh = torch.zeros(3 * H, device="cuda")
        dfeat = torch.zeros(nfeat, 3 * H, device="cuda")
        rexp = torch.empty(R, dtype=torch.int32, device="cuda")
        rc = L.msat_gru_ln_bwd_g4fe(dy.data_ptr(), H, g4.data_ptr(), 4 * H, hp.data_ptr(), H, sc.data_ptr(),
                                    D.data_ptr(), 4 * H, D.data_ptr() + 4 * H, 4 * H, dh.data_ptr(), H, dln.data_ptr(),
                                    dln.data_ptr() + 4 * H, dbi.data_ptr(), dbh.data_ptr() + 4 * 2 * H, feat.data_ptr(), 8,
                                    nfeat, dfeat.data_ptr(), part.data_ptr(), R, H, 7, rexp.data_ptr(), s)
        assert rc == 0
        out = {"D": D, "dh": dh, "dln": dln, "dbi": dbi, "dbh": dbh, "dfeat": dfeat, "rexp": rexp}
        torch.cuda.synchronize()
        if ref is None:
            ref = {k: v.clone() for k, v in out.items()}
            continue
        bad = {k: int((v != ref[k]).sum()) for k, v in out.items() if not torch.equal(v, ref[k])}
        if bad:
            rows = (dfeat != ref["dfeat"]).any(1).nonzero().flatten().tolist() if "dfeat" in bad else []
            print(f"nfeat {nfeat} rep {r}: differing {bad}; dfeat rows {rows}", flush=True)
    print(f"nfeat {nfeat}: {reps} reps done", flush=True)
