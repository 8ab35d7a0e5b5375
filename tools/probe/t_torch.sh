python -c "import torch; print('torch-first', torch.cuda.is_available(), torch.version.hip, torch.cuda.device_count())"
python -c "
import sys; sys.path.insert(0,'diffopt.jl_amd')
from diffopt_amd import _lib; _lib.load()
import torch; print('lib-first', torch.cuda.is_available())"
python -c "
import sys; sys.path.insert(0,'diffopt.jl_amd')
import torch; print(torch.cuda.is_available())
from diffopt_amd.qp import QPBatch
import numpy as np
e = QPBatch(1, 2, 0, 0); print('engine ok after torch')
"
ldd diffopt.jl_amd/diffopt_amd/libdiffopt_mi355x.so | grep -i -E "hip|hsa|roc"
python -c "import torch, os; print([l for l in open('/proc/self/maps').read().split('\n') if 'amdhip' in l][:2])"
env | grep -i -E "HIP|ROC|HSA|CUDA" 
