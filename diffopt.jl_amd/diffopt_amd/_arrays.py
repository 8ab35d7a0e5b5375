"""Array staging between numpy (host) / torch-CUDA (device) and the C ABI.

The ABI wants column-major, batch-major float64 buffers (include header).  A
numpy/torch array of shape (B, r, c) in the usual C order is transposed to
(B, c, r) C-contiguous, which is exactly (B, r, c) column-major per problem.
Device tensors are passed zero-copy (DOPT_MEM_DEVICE) on torch's current
stream; host arrays are passed by pointer and copied by the library.
"""

import numpy as np

from . import _lib


def _is_torch(x):
    return x is not None and type(x).__module__.startswith("torch")


def _is_cuda(x):
    return _is_torch(x) and x.is_cuda


def colmajor(X, shape):
    """Batch of matrices (B, r, c) → per-problem column-major contiguous buffer."""
    if X is None:
        return None
    B, r, c = shape
    if _is_torch(X):
        import torch
        X = X.reshape(B, r, c).to(torch.float64)
        return X.transpose(1, 2).contiguous()
    X = np.asarray(X, dtype=np.float64).reshape(B, r, c)
    return np.ascontiguousarray(np.swapaxes(X, 1, 2))


def vector(x, shape):
    if x is None:
        return None
    if _is_torch(x):
        import torch
        return x.reshape(shape).to(torch.float64).contiguous()
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(shape))


class Staged:
    """Decides host vs device mode for one ABI call and yields raw pointers."""

    def __init__(self, arrays):
        present = [a for a in arrays if a is not None]
        cuda = [_is_cuda(a) for a in present]
        if any(cuda) and not all(cuda):
            raise TypeError("mix of host and device arrays in one call")
        self.mem = _lib.DOPT_MEM_DEVICE if (present and all(cuda)) else _lib.DOPT_MEM_HOST
        self.stream = None      # host mode: the handle's private stream
        self.set_stream = False
        if self.mem == _lib.DOPT_MEM_DEVICE:
            self.set_stream = True
            import torch
            self.stream = torch.cuda.current_stream(present[0].device).cuda_stream

    @staticmethod
    def ptr(a):
        if a is None:
            return None
        if _is_torch(a):
            return a.data_ptr()
        return a.ctypes.data

    @staticmethod
    def empty(shape, device):
        if device:
            import torch
            return torch.empty(shape, dtype=torch.float64, device="cuda")
        return np.empty(shape, dtype=np.float64)
