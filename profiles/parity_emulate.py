"""CPU emulation of the fp16x2 GRU forward's operand rounding inside the fp32 oracle (round 6, verdict r05 item 1).

Reloads a train-cycle dump (tests/test_mappo_gpu.py with MARLSAT_PARITY_DUMP) and recomputes one Adam step's
gradient with the fp32 oracle, the GRU cells' GEMM operands rounded the way the fp16x2 kernel represents them
(weights: hi + lo of 2^10 W; activations: hi + lo of ASC * a), the backward in plain fp32.  Compared with the
float64 oracle and the device's own gradient, it shows which rounding reproduces the device's error.

    ASC=<activation scale> python profiles/parity_emulate.py <dump.npz> <step> {w|a|a_h|a_x|w_hid|w_in|both}
"""
import os, sys, numpy as np, torch
ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, ROOT+'/marl-sat_amd', ROOT+'/tests', ROOT+'/profiles'): sys.path.insert(0,p)
from oracle import net as onet
from marlsat.learners import params as Pm
import parity_orderings as po
d=np.load(sys.argv[1]); s=int(sys.argv[2]); mode_=sys.argv[3]
V,C,vpa,H,L,mode,T,B,MB,E=(int(v) for v in d['shape']); A,M=d['av'].shape
cfg=po.cfg_of(d['shape'])
av=torch.from_numpy(d['av'].astype(np.int64)); am=torch.from_numpy(d['am'])
full={k[5:]:torch.from_numpy(d[k]) for k in d.files if k.startswith('full_')}
mb={k:v[d[f'idx_{s}']] for k,v in full.items()}
P=Pm.to_flax(d[f'params_{s}'].astype(np.float32),H,L,A,M,mode,16)
torch.set_num_threads(8)
g64_, _ = po.grads(P, mb, cfg, av, am, mode, L, torch.float64)
g32_, _ = po.grads(P, mb, cfg, av, am, mode, L, torch.float32)
gd_ = Pm.to_flax(d[f'grads_{s}'].astype(np.float32), H, L, A, M, mode, 16)
g = {**{'g64/' + k: v for k, v in g64_.items()}, **{'g32/' + k: v for k, v in g32_.items()},
     **{'dev/' + k: np.asarray(v, np.float64) for k, v in gd_.items()}}
def rnd_w(w):  # fp16x2 representation of w (scaled 2^10): hi + lo
    ws=(w*1024.0).float(); hi=ws.half().float(); lo=(ws-hi).half().float(); return (hi+lo)/1024.0
ASC=float(os.environ.get('ASC','1'))
def rnd_a(a):
    a2=a*ASC
    hi=a2.half().float(); lo=(a2-hi).half().float(); return (hi+lo)/ASC
class RD(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, rw, ra):
        ctx.save_for_backward(x, w)
        xx = rnd_a(x) if ra else x
        ww = rnd_w(w) if rw else w
        return xx @ ww
    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        return gy @ w.t(), x.transpose(-1,-2) @ gy, None, None
cells=('update_c','update_v_pos','update_v_neg')
orig=onet._dense
def dense(P_, name, x):
    parts=name.split('/')
    if len(parts)==3 and parts[1] in cells and x.dtype==torch.float32:
        hidden=parts[2][0]=='h'
        rw = mode_ in ('w','both') or (mode_=='w_in' and not hidden) or (mode_=='w_hid' and hidden)
        ra = mode_ in ('a','both') or (mode_=='a_h' and hidden) or (mode_=='a_x' and not hidden)
        y=RD.apply(x, P_[f'{name}/kernel'], rw, ra)
        b=P_.get(f'{name}/bias')
        return y+b if b is not None else y
    return orig(P_,name,x)
onet._dense=dense
g32,_=po.grads(P,mb,cfg,av,am,mode,L,torch.float32)
for k in ['encoder/update_v_neg/hn/bias','encoder/update_v_neg/in/bias','encoder/literal_neg_embed/bias','encoder/update_v_pos/hn/bias','encoder/update_c/hn/bias']:
    g64=g['g64/'+k]; de=np.abs(g['dev/'+k]-g64); fe=np.abs(g['g32/'+k]-g64); pe=np.abs(g32[k]-g64)
    print(f'{mode_:6s} {k}: dev max {de.max():.2g} med {np.median(de):.2g} | fp32 max {fe.max():.2g} med {np.median(fe):.2g} | emulated max {pe.max():.2g} med {np.median(pe):.2g}')
