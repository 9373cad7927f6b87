"""Host-array plumbing for the reference's NumPy call surfaces.

The reference's Python functions take host ``[L, d]`` (or flat ``[L*d]``) NumPy arrays.  The
drop-in versions accept those too: the arrays are copied to the current ROCm device as
``[1, 1, L, d]``, the gfx950 kernel runs, and the result is copied back in the caller's
dtype.  torch device tensors pass through without copies.

Compute dtype for host arrays: float16 inputs run the fp16 kernels; float32 / float64
inputs run fp16 when every value fits in fp16's range (|x| <= 65504) and bf16 otherwise.
Accumulation is always fp32 (MFMA).  The PCIe copies are part of these host surfaces
only; bench.py times device-resident tensors.
"""
import numpy as np
import torch

FP16_MAX = 65504.0


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("exploring_flash_attention_amd needs a ROCm GPU (MI355X / gfx950); "
                           "there is no CPU fallback")


def compute_dtype(*arrays):
    if all(a.dtype == np.float16 for a in arrays):
        return torch.float16
    big = max(float(np.max(np.abs(a))) if a.size else 0.0 for a in arrays)
    return torch.float16 if big <= FP16_MAX else torch.bfloat16


def to_device(arrays, dtype):
    """Host [L, d] arrays -> contiguous [1, 1, L, d] device tensors of dtype."""
    require_gpu()
    dev = torch.device("cuda", torch.cuda.current_device())
    out = []
    for a in arrays:
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
        out.append(t.to(device=dev, dtype=dtype, non_blocking=False)[None, None].contiguous())
    return out


def to_host(t, like_dtype):
    """[1, 1, L, d] device tensor -> host [L, d] array of like_dtype."""
    return t[0, 0].float().cpu().numpy().astype(like_dtype, copy=False)


def is_device_tensor(x):
    return isinstance(x, torch.Tensor) and x.device.type == "cuda"
