"""FA-v1 fused forward -- drop-in surfaces of the reference's flash_attention_v1 family.

Reference surfaces mirrored (tyler-utah/exploring_flash_attention):

* ``flash_attention_tiled(Q, K, V, Bq=8, Bk=8) -> O``
      flash_attention_v1/numpy_basic.py:69  (host [L, d] arrays in, [L, d] out)
* ``flash_attention_tiled(Q, K, V, O, L, d, Bq=8, Bk=8)``
      flash_attention_v1/numpy_gpu_like_opt2.py:198  (flat [L*d] buffers, O written in place;
      also the signature of numpy_gpu_like.py:288 / _1D.py:320 / _opt1.py:320)
* ``flash_attention_v1(Q, K, V, O, B, H, L, d)`` and ``flash_attention_v1_opt1(...)``
      flash_attention_v1/CUDA/flash_attention_v1.h:251, flash_attention_v1_opt1.h:354
      (device [B, H, L, d] tensors, O written in place)
* ``flash_attention_v1(Q, K, V) -> O`` -- the ``naive_attention(Q, K, V)`` form
      (common/reference.py:7): NumPy [L, d] / [B, H, L, d] or torch device tensors

``Bq`` / ``Bk`` are the reference's tile sizes; they are accepted and validated (> 0) but
the gfx950 kernel uses its own tiles (128 query rows x 64 keys, see
``ops.kernel_geometry``) -- the result does not depend on them.
"""
import numpy as np

from . import _host, ops


def _check_tiles(Bq, Bk):
    assert isinstance(Bq, (int, np.integer)) and Bq > 0, "Bq must be a positive int"
    assert isinstance(Bk, (int, np.integer)) and Bk > 0, "Bk must be a positive int"


def _run_host(Q, K, V):
    Q, K, V = (np.asarray(x) for x in (Q, K, V))
    assert Q.ndim == 2 and Q.shape == K.shape == V.shape, "Q, K, V must have the same shape [L, d]"
    dt = _host.compute_dtype(Q, K, V)
    q, k, v = _host.to_device((Q, K, V), dt)
    return _host.to_host(ops.attention_v1(q, k, v), Q.dtype)


def flash_attention_tiled(Q, K, V, *args, Bq=8, Bk=8, **kw):
    """Both reference surfaces of ``flash_attention_tiled`` (see module docstring)."""
    if args or "O" in kw:  # C-style: (Q, K, V, O, L, d, Bq=8, Bk=8)
        names = ("O", "L", "d", "Bq", "Bk")
        vals = dict(zip(names, args))
        vals.update(kw)
        vals.setdefault("Bq", Bq)
        vals.setdefault("Bk", Bk)
        O, L, d = vals["O"], int(vals["L"]), int(vals["d"])
        _check_tiles(vals["Bq"], vals["Bk"])
        q2, k2, v2 = (np.asarray(x).reshape(L, d) for x in (Q, K, V))
        O[:L * d] = _run_host(q2, k2, v2).reshape(-1).astype(O.dtype, copy=False)
        return None
    if kw:
        raise TypeError(f"unexpected keyword arguments {sorted(kw)}")
    _check_tiles(Bq, Bk)
    if _host.is_device_tensor(Q):
        if Q.dim() == 2:
            return ops.attention_v1(Q[None, None], K[None, None], V[None, None])[0, 0]
        return ops.attention_v1(Q, K, V)
    return _run_host(Q, K, V)


def flash_attention_v1(Q, K, V, O=None, B=None, H=None, L=None, d=None):
    """``flash_attention_v1(Q, K, V) -> O`` (host or device), or the launcher form
    ``flash_attention_v1(Q, K, V, O, B, H, L, d)``: O[B,H,L,d] written in place,
    asynchronous on the current stream."""
    if O is None:
        return _host.run_qkv(ops.attention_v1, Q, K, V)
    assert B > 0 and H > 0 and L > 0 and d > 0, "All dimensions must be positive"
    assert tuple(Q.shape) == (B, H, L, d), f"Q shape {tuple(Q.shape)} != {(B, H, L, d)}"
    ops.attention_v1(Q, K, V, out=O)


flash_attention_v1_opt1 = flash_attention_v1
