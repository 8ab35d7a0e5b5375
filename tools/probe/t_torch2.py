import sys, os
sys.path.insert(0, 'diffopt.jl_amd')
mode = sys.argv[1]
import numpy as np
if mode == 'torch_first':
    import torch
    x = torch.zeros(4, device='cuda')
    from diffopt_amd.qp import QPBatch
    from diffopt_amd.synthetic import qp_numpy
    d = qp_numpy(2, 5, 6, 1, 0.5, 1)
    t = {k: torch.tensor(v, device='cuda') for k, v in d.items()}
    e = QPBatch(2, 5, 6, 1)
    e.set(t["Q"], t["G"], t["h"], t["A"], t["z"], t["lam"], t["nu"])
    r, f = e.forward_reverse(t["dl_dz"], dq=t["dq"], dh=t["dh"], db=t["db"])
    e2 = QPBatch(2, 5, 6, 1)
    e2.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    r2, f2 = e2.forward_reverse(d["dl_dz"], dq=d["dq"], dh=d["dh"], db=d["db"])
    print('torch_first device-mode diff', float(abs(r.cpu().numpy() - r2).max()))
else:
    from diffopt_amd.qp import QPBatch
    e = QPBatch(1, 2, 0, 0)
    import torch
    print('lib_first torch avail', torch.cuda.is_available())
maps = open('/proc/self/maps').read().split('\n')
print(sorted(set(l.split()[-1] for l in maps if ('hsa' in l or 'amdhip' in l) and '/' in l)))
