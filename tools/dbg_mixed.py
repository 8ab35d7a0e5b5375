import sys, numpy as np
sys.path[:0]=['/root/repo','/root/repo/diffopt.jl_amd','/root/repo/tests']
from diffopt_amd.qp import QPBatch
from diffopt_amd.synthetic import qp_numpy
from oracle import qp as oqp
def relfro(a,b): return np.linalg.norm(a-b)/max(np.linalg.norm(b),1e-300)
lo=qp_numpy(3,60,80,4,0.2,31); hi=qp_numpy(3,60,80,4,0.8,32)
d={k: np.concatenate([np.stack([lo[k][i], hi[k][i]]) for i in range(3)]) for k in lo}
for fm in [100, 0, 512]:
    e=QPBatch(6,60,80,4); e.set_fast_max(fm)
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    rev,fwd=e.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    print('fast_max',fm,'sizes',e.system_size())
    for b in range(6):
        args=[d[k][b] for k in ["Q","G","h","A","z","lam","nu"]]
        r=np.concatenate(oqp.reverse_differentiate(*args, d["dl_dz"][b]))
        f=np.concatenate(oqp.forward_differentiate(*args, dq=d["dq"][b], dh=d["dh"][b], db=d["db"][b]))
        print(' b',b,'rev %.2e fwd %.2e'%(relfro(rev[b],r), relfro(fwd[b],f)))
