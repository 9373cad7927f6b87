"""Device-tensor operators over the C ABI (torch tensors in HBM, zero-copy).

Every function takes ``[B, H, L, d]`` bf16 / fp16 (or fp64) tensors on a ROCm device --
contiguous, or for attention_v1 / _tiled_d / _v2 any view with a contiguous d (strided
kernels, no copy) --
launches on the current HIP stream of that device and returns without synchronising.
PyTorch is only the plumbing here (device memory, streams); the work is done by the
gfx950 kernels in libfa_mi355x.so.

Reference launchers these replace (tyler-utah/exploring_flash_attention):
  attention_v1       flash_attention_v1/CUDA/flash_attention_v1.h:251 (opt1 :354)
  attention_tiled_d  flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:312 (opt :448)
  attention_v2       flash_attention_v2/CUDA/flash_attention_v2.h:438 (opt :559)
  attention_partial  partial_attention_kernel, flash_attention_v2/CUDA/flash_attention_v2.h:243
  combine            reduction_kernel,         flash_attention_v2/CUDA/flash_attention_v2.h:356
"""
import contextlib
import ctypes
import threading

import torch

from . import _lib
from ._lib import (FA_BLOCKS_PER_WG_AUTO, FA_DTYPE_BF16, FA_DTYPE_FP16, FA_DTYPE_FP16_SCALED, FA_DTYPE_FP32,
                   FA_DTYPE_FP64, FA_KV_TILES_AUTO, check, lib)

# torch.float64 runs the fp64 kernels (the reference's USE_FP64 build): fp64 MFMA, softmax,
# partials and lse -- the bit-tight mode, not the fast one
_DTYPES = {torch.bfloat16: FA_DTYPE_BF16, torch.float16: FA_DTYPE_FP16, torch.float64: FA_DTYPE_FP64}
# split-KV partial formats: a torch dtype, or PARTIAL_FP16_SCALED (fp16 scaled per row by a
# power of two, exponent beside the lse: half the bytes of fp32, attention_v2 only)
PARTIAL_FP16_SCALED = "fp16_scaled"
_PDTYPES = {torch.float32: FA_DTYPE_FP32, torch.bfloat16: FA_DTYPE_BF16, torch.float16: FA_DTYPE_FP16,
            torch.float64: FA_DTYPE_FP64, PARTIAL_FP16_SCALED: FA_DTYPE_FP16_SCALED}


_klog = threading.local()


def _launched(status):
    """check() for a call that launches kernels; inside launched_kernels() also records what
    the library's launcher enqueued (fa_last_kernels)."""
    check(status)
    log = getattr(_klog, "log", None)
    if log is not None:
        log.append(_lib.last_kernels())


@contextlib.contextmanager
def launched_kernels():
    """Collect, in call order, the kernels (with grids) every operator of this module launches
    on this thread inside the block -- the library's own report (fa_last_kernels), so a caller
    such as bench.py names what ran instead of restating the launch rules."""
    prev = getattr(_klog, "log", None)
    _klog.log = []
    try:
        yield _klog.log
    finally:
        _klog.log = prev


def _default_pdtype(dtype, partial_dtype, fused=False):
    """Partial format when none is given: fp64 for fp64 inputs; the fused split-KV
    (attention_v2) keeps per-row scaled fp16 partials -- half the workspace traffic of fp32
    at C4 (4.73 -> 3.50 ms) and within a few output ulps of it (tests/test_gpu.py); the
    row-layout partials of the multi-GPU path stay fp32."""
    if partial_dtype is not None:
        return partial_dtype
    if dtype == torch.float64:
        return torch.float64
    return PARTIAL_FP16_SCALED if fused else torch.float32

SUPPORTED_HEAD_DIMS = (32, 64, 128, 256, 384, 512)  # head dims with a kernel
# head dims past one LDS tile: the d-tiled kernels (csrc/fa_fwd_dtiled.hip), contiguous tensors,
# FA-v1 / tiled-d / unsplit v2 only (no split-KV partial kernel, no multi-GPU path)
WIDE_HEAD_DIMS = (384, 512)
MAX_HEAD_DIM = 512


def kernel_head_dim(d):
    """Head dim of the kernel that serves head dim d: d itself when a kernel exists,
    otherwise the next larger one (the operators then zero-pad q, k, v to it and keep the
    softmax scale 1/sqrt(d); zero columns add nothing to q k^T and come out of P.V as zeros).
    The reference's Python functions take any d, e.g. d = 16 in its tests' shapes."""
    d = int(d)
    if d <= 0 or d > MAX_HEAD_DIM:
        raise ValueError(f"head dim d={d} unsupported (1 <= d <= {MAX_HEAD_DIM})")
    return next(D for D in SUPPORTED_HEAD_DIMS if D >= d)


def _pad_d(t, D):
    return t if t.shape[-1] == D else torch.nn.functional.pad(t, (0, D - t.shape[-1])).contiguous()


def _unpad_into(o_pad, o, d):
    if o_pad is not o:
        o.copy_(o_pad[..., :d])
    return o


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stride_args(q, k, v, o):
    """Stride arguments of the *_ex entry points for a mix of contiguous and strided
    [B, H, L, d] tensors: None when all four are contiguous, False when some view is not
    expressible (d not contiguous, strides not multiples of 8 elements, k and v strided
    differently, fp64), else three ctypes int64[3] arrays {batch, head, row} for q, k/v, o."""
    ts = (q, k, v, o)
    if all(t.is_contiguous() for t in ts):
        return None
    if q.dtype not in (torch.bfloat16, torch.float16) or k.stride() != v.stride():
        return False

    def ok(t):
        st = t.stride()
        return (st[3] == 1 and all(x > 0 and x % 8 == 0 for x in st[:3]) and st[2] >= t.shape[3]
                and t.data_ptr() % 16 == 0)

    if not all(ok(t) for t in ts):
        return False
    return tuple((ctypes.c_int64 * 3)(*t.stride()[:3]) for t in (q, k, o))


def _via_contiguous(fn, q, k, v, o, **kw):
    """Run fn on contiguous copies of views the strided kernels cannot address."""
    o.copy_(fn(q.contiguous(), k.contiguous(), v.contiguous(), **kw))
    return o


def _check_tensor(name, t, dtype=None, device=None, ndim=4, strided=False):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor, got {type(t).__name__}")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be a ROCm device tensor (got device {t.device}); "
                         "the MI355X path has no CPU fallback")
    if t.dim() != ndim:
        raise ValueError(f"{name} must be {ndim}-D, got shape {tuple(t.shape)}")
    if not strided and not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} has dtype {t.dtype}, expected {dtype}")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")


def _check_qkv(q, k, v, same_len=True, strided=False):
    _check_tensor("q", q, strided=strided)
    if q.dtype not in _DTYPES:
        raise ValueError(f"q dtype {q.dtype} unsupported (bfloat16, float16 or float64)")
    _check_tensor("k", k, q.dtype, q.device, strided=strided)
    _check_tensor("v", v, q.dtype, q.device, strided=strided)
    if k.shape != v.shape:
        raise ValueError(f"k {tuple(k.shape)} and v {tuple(v.shape)} must have the same shape")
    if q.shape[0] != k.shape[0] or q.shape[1] != k.shape[1] or q.shape[3] != k.shape[3]:
        raise ValueError(f"q {tuple(q.shape)} and k {tuple(k.shape)} disagree on B, H or d")
    if same_len and q.shape != k.shape:
        raise ValueError(f"q {tuple(q.shape)} and k {tuple(k.shape)} must have the same shape")


def _out(out, q, shape=None, dtype=None, strided=False):
    shape = tuple(q.shape) if shape is None else shape
    dtype = q.dtype if dtype is None else dtype
    if out is None:
        return torch.empty(shape, dtype=dtype, device=q.device)
    _check_tensor("out", out, dtype, q.device, ndim=len(shape), strided=strided)
    if tuple(out.shape) != shape:
        raise ValueError(f"out has shape {tuple(out.shape)}, expected {shape}")
    return out


def attention_v1(q, k, v, out=None):
    """FA-v1 fused forward: O = softmax(q k^T / sqrt(d)) v.  Any 1 <= d <= 256 (head dims
    without a kernel are zero-padded to the next one, see kernel_head_dim).  q, k, v and out
    may be strided [B, H, L, d] views with a contiguous d -- e.g. ``x.transpose(1, 2)`` of a
    [B, L, H, d] tensor -- which the kernel addresses in place (fa_fwd_v1_ex)."""
    _check_qkv(q, k, v, strided=True)
    o = _out(out, q, strided=True)
    B, H, L, d = q.shape
    D = kernel_head_dim(d)
    if q.numel() == 0:  # no rows: nothing to launch (the reference returns an empty O)
        return o
    st = _stride_args(q, k, v, o) if D == d else None
    if st is not None and D in WIDE_HEAD_DIMS:
        st = False  # the d-tiled kernels address contiguous tensors only
    if st is False:
        return _via_contiguous(attention_v1, q, k, v, o)
    if D == d:
        if st is None:
            _launched(lib().fa_fwd_v1(_ptr(q), _ptr(k), _ptr(v), _ptr(o), B, H, L, d, _DTYPES[q.dtype], _stream(q)))
        else:
            _launched(lib().fa_fwd_v1_ex(_ptr(q), _ptr(k), _ptr(v), _ptr(o), B, H, L, d, st[0], st[1], st[2],
                                     1.0 / d ** 0.5, _DTYPES[q.dtype], _stream(q)))
        return o
    qp, kp, vp = (_pad_d(t, D) for t in (q, k, v))
    op = torch.empty((B, H, L, D), dtype=q.dtype, device=q.device)
    _launched(lib().fa_fwd_v1_scaled(_ptr(qp), _ptr(kp), _ptr(vp), _ptr(op), B, H, L, D, 1.0 / d ** 0.5,
                                 _DTYPES[q.dtype], _stream(q)))
    return _unpad_into(op, o, d)


def _d_tiles(d, d_tile_qk, d_tile_v):
    """d tiles the caller left as None: min(32, d) up to d = 256 (the reference's D_TILE = 32
    where d allows it; there the tiles are only validated -- one LDS tile holds a whole row),
    128 above, where the d-tiled kernel streams K / V in tile-wide column chunks.  The output
    is bitwise the same for every tile choice, only the speed differs: d = 512 B32 H8 L1024,
    32/32 0.931 ms against 128/128 0.682 ms (24 chunk waits + barriers per 64-key tile against
    6; scripts/dtile_sweep.py, profiles/r05/dtile_sweep.txt)."""
    dflt = min(32, d) if d <= 256 else 128
    return (dflt if d_tile_qk is None else int(d_tile_qk),
            dflt if d_tile_v is None else int(d_tile_v))


def attention_tiled_d(q, k, v, d_tile_qk=None, d_tile_v=None, out=None):
    """FA-v1 d-tiled forward (O_acc in VGPRs); d tiles as in the reference launcher
    (0 < d_tile <= d; default min(32, d) up to d = 256, 128 above -- see _d_tiles).  d <= 256: one LDS tile holds a whole row and the
    fused kernel runs (tiles validated); 256 < d <= 512: the d-tiled kernel streams K and V
    through LDS in d_tile-wide column chunks (rounded down to 32, 64 or 128 columns)."""
    _check_qkv(q, k, v, strided=True)
    B, H, L, d = q.shape
    d_tile_qk, d_tile_v = _d_tiles(d, d_tile_qk, d_tile_v)
    # the tile arguments are validated against the true d, as the launcher does
    # (flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:326-327)
    for name, t in (("d_tile_qk", d_tile_qk), ("d_tile_v", d_tile_v)):
        if not 0 < int(t) <= d:
            raise _lib.FaArgumentError(1, f"{name}={int(t)} must satisfy 0 < {name} <= d={d}")
    D = kernel_head_dim(d)
    if D not in WIDE_HEAD_DIMS:
        if q.numel() == 0 or D != d or not all(t.is_contiguous() for t in (q, k, v)) or (
                out is not None and not out.is_contiguous()):
            # padded head dims and strided views run on fa_fwd_v1's paths (the same kernel)
            return attention_v1(q, k, v, out=out)
        o = _out(out, q)
        _launched(lib().fa_fwd_v1_tiled_d(_ptr(q), _ptr(k), _ptr(v), _ptr(o), B, H, L, d, int(d_tile_qk),
                                      int(d_tile_v), _DTYPES[q.dtype], _stream(q)))
        return o
    o = _out(out, q, strided=True)
    if q.numel() == 0:
        return o
    qc, kc, vc = (_pad_d(t.contiguous(), D) for t in (q, k, v))
    oc = o if D == d and o.is_contiguous() else torch.empty((B, H, L, D), dtype=q.dtype, device=q.device)
    _launched(lib().fa_fwd_v1_tiled_d_scaled(_ptr(qc), _ptr(kc), _ptr(vc), _ptr(oc), B, H, L, D, int(d_tile_qk),
                                         int(d_tile_v), 1.0 / d ** 0.5, _DTYPES[q.dtype], _stream(q)))
    if oc is not o:
        o.copy_(oc[..., :d])
    return o


def _kvtpb(kv_tiles_per_block):
    return FA_KV_TILES_AUTO if kv_tiles_per_block == "auto" else int(kv_tiles_per_block)


def _bpw(blocks_per_workgroup):
    g = FA_BLOCKS_PER_WG_AUTO if blocks_per_workgroup is None else int(blocks_per_workgroup)
    if g < 0:
        raise ValueError(f"blocks_per_workgroup={g} must be >= 1 (or None for the library's grouping)")
    return g


def v2_workspace_bytes(B, H, L, d, kv_tiles_per_block=4, dtype=torch.bfloat16,
                       partial_dtype=None, blocks_per_workgroup=None):
    """(bytes, num_splits) of the split-KV workspace: num_splits = the reference's key blocks;
    the bytes cover the partials actually combined through the workspace (v2_split_plan) in
    partial_dtype (per-row scaled fp16 by default; fp64 for fp64 inputs)."""
    pd = _default_pdtype(dtype, partial_dtype, fused=True)
    kv_tiles_per_block = _kvtpb(kv_tiles_per_block)
    nbytes = ctypes.c_size_t()
    ns = ctypes.c_int()
    d = kernel_head_dim(d)
    check(lib().fa_fwd_v2_workspace_size_ex(B, H, L, d, int(kv_tiles_per_block), _bpw(blocks_per_workgroup),
                                            _DTYPES[dtype], _PDTYPES[pd], ctypes.byref(nbytes), ctypes.byref(ns)))
    return nbytes.value, ns.value


def v2_split_plan(B, H, L, d, kv_tiles_per_block=4, dtype=torch.bfloat16, blocks_per_workgroup=None):
    """(key_blocks, blocks_per_workgroup, partials_per_tile) of fa_fwd_v2's schedule: the
    reference's key blocks of kv_tiles_per_block tiles, how many consecutive blocks one
    workgroup combines on chip, and how many partial workgroups per query tile are combined
    through the workspace.  ``blocks_per_workgroup`` None: the library's grouping; n >= 1 fixes
    it (1 = one workgroup and one HBM partial per key block, the reference's layout)."""
    kb, g, p = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    check(lib().fa_fwd_v2_split_plan(B, H, L, kernel_head_dim(d), int(_kvtpb(kv_tiles_per_block)),
                                     _bpw(blocks_per_workgroup), _DTYPES[dtype],
                                     ctypes.byref(kb), ctypes.byref(g), ctypes.byref(p)))
    return kb.value, g.value, p.value


def attention_v2(q, k, v, kv_tiles_per_block=4, d_tile_qk=None, d_tile_v=None, partial_dtype=None,
                 out=None, workspace=None, blocks_per_workgroup=None, workspace_zeroed=False):
    """FA-v2 split-KV forward (partial kernel + combine kernel).

    A split is ``kv_tiles_per_block`` KV tiles of the kernel's own tile size (64 keys;
    32 at d = 256); ``kv_tiles_per_block="auto"`` lets the library pick the split from the
    device's occupancy (no split when the query tiles already fill the GPU).
    ``blocks_per_workgroup`` (None: the library's grouping, v2_split_plan) fixes how many
    consecutive key blocks one workgroup combines on chip; 1 is the reference's layout (one
    HBM partial per key block).
    Partial outputs are kept as per-row scaled fp16 by default (``PARTIAL_FP16_SCALED``: half
    the workspace traffic of ``torch.float32``, 11 significant bits relative to each row's
    largest partial, no fp16 range limit); ``torch.float32`` or the input dtype on request.
    ``workspace`` (a uint8 device tensor) is allocated from torch's caching allocator when
    not given, so the call itself never reaches hipMalloc after warm-up.
    ``workspace_zeroed=True`` promises that the workspace came zeroed (``torch.zeros``) and has
    been used since only by attention_v2 calls of this same shape and plan (each leaves its
    counters zero): the per-call counter reset, a dispatch of its own, is skipped
    (fa_fwd_v2_ex2 with FA_V2_COUNTERS_ZERO; 1.6-1.8 us per call).
    """
    _check_qkv(q, k, v, strided=True)
    o = _out(out, q, strided=True)
    B, H, L, d = q.shape
    D = kernel_head_dim(d)
    d_tile_qk, d_tile_v = _d_tiles(d, d_tile_qk, d_tile_v)
    if q.numel() == 0:  # no rows: nothing to launch
        return o
    st = _stride_args(q, k, v, o) if D == d else None
    if st is not None and D in WIDE_HEAD_DIMS:
        st = False  # the d-tiled kernels address contiguous tensors only
    if st is False:
        return _via_contiguous(attention_v2, q, k, v, o, kv_tiles_per_block=kv_tiles_per_block,
                               d_tile_qk=d_tile_qk, d_tile_v=d_tile_v, partial_dtype=partial_dtype,
                               workspace=workspace, blocks_per_workgroup=blocks_per_workgroup,
                               workspace_zeroed=workspace_zeroed)
    pd = _default_pdtype(q.dtype, partial_dtype, fused=True)
    kv_tiles_per_block = _kvtpb(kv_tiles_per_block)
    bpw = _bpw(blocks_per_workgroup)
    nbytes, _ = v2_workspace_bytes(B, H, L, d, kv_tiles_per_block, q.dtype, pd, bpw)
    if workspace is None:
        workspace = torch.empty(nbytes, dtype=torch.uint8, device=q.device)
        workspace_zeroed = False
    elif workspace.numel() * workspace.element_size() < nbytes:
        raise ValueError(f"workspace too small: {nbytes} bytes needed")
    wsb = workspace.numel() * workspace.element_size()
    flags = _lib.FA_V2_COUNTERS_ZERO if workspace_zeroed else 0
    if D == d:
        sq, skv, so = (None, None, None) if st is None else st
        _launched(lib().fa_fwd_v2_ex2(_ptr(q), _ptr(k), _ptr(v), _ptr(o), B, H, L, d, int(d_tile_qk),
                                      int(d_tile_v), int(kv_tiles_per_block), bpw, _ptr(workspace), wsb, sq, skv,
                                      so, 1.0 / d ** 0.5, _DTYPES[q.dtype], _PDTYPES[pd], flags, _stream(q)))
        return o
    for name, t in (("d_tile_qk", d_tile_qk), ("d_tile_v", d_tile_v)):
        if not 0 < int(t) <= d:
            raise _lib.FaArgumentError(1, f"{name}={int(t)} must satisfy 0 < {name} <= d={d}")
    qp, kp, vp = (_pad_d(t, D) for t in (q, k, v))
    op = torch.empty((B, H, L, D), dtype=q.dtype, device=q.device)
    _launched(lib().fa_fwd_v2_ex2(_ptr(qp), _ptr(kp), _ptr(vp), _ptr(op), B, H, L, D, int(d_tile_qk),
                                  int(d_tile_v), int(kv_tiles_per_block), bpw, _ptr(workspace), wsb, None, None, None,
                                  1.0 / d ** 0.5, _DTYPES[q.dtype], _PDTYPES[pd], flags, _stream(q)))
    return _unpad_into(op, o, d)


def attention_partial(q, k, v, chunk_rows=None, partial_dtype=None, o_part=None, lse=None):
    """Split-KV partial over one whole key range (k, v: [B, H, Lk, d]).

    Returns ``(o_part, lse)`` with o_part ``[Lq/chunk_rows, B*H, chunk_rows, d]`` holding the
    normalised partial output and lse ``[Lq/chunk_rows, B*H, chunk_rows]`` its base-2
    log-sum-exp (of the scores times log2(e)/sqrt(d)); fp32 partials and lse by default,
    fp64 for fp64 inputs.  ``partial_dtype=PARTIAL_FP16_SCALED``: o_part is fp16 holding each
    row times 2^-e (the row's largest |value| just below 1) and lse gains a trailing dim of 2,
    ``{lse, e}`` per row -- ``combine`` recognises the format by that dim.
    """
    _check_qkv(q, k, v, same_len=False, strided=True)
    if not (k.is_contiguous() and v.is_contiguous()):
        k, v = k.contiguous(), v.contiguous()
    qst = None
    if not q.is_contiguous():  # a row range of a longer q (the multi-GPU chunks): in place
        st = _stride_args(q, k, v, q)
        if st is False:
            q = q.contiguous()
        else:
            qst = st[0]
    B, H, Lq, d = q.shape
    Lk = k.shape[2]
    cr = Lq if chunk_rows is None else int(chunk_rows)
    if cr <= 0 or Lq % cr:
        raise ValueError(f"chunk_rows={cr} must divide Lq={Lq}")
    nch = Lq // cr
    partial_dtype = _default_pdtype(q.dtype, partial_dtype)
    lse_dtype = torch.float64 if q.dtype == torch.float64 else torch.float32
    scaled = partial_dtype == PARTIAL_FP16_SCALED
    o_part = _out(o_part, q, (nch, B * H, cr, d), torch.float16 if scaled else partial_dtype)
    lse = _out(lse, q, (nch, B * H, cr, 2) if scaled else (nch, B * H, cr), lse_dtype)
    if qst is None:
        _launched(lib().fa_fwd_partial(_ptr(q), _ptr(k), _ptr(v), _ptr(o_part), _ptr(lse), B, H, Lq, Lk, d,
                                   cr, _DTYPES[q.dtype], _PDTYPES[partial_dtype], _stream(q)))
    else:
        _launched(lib().fa_fwd_partial_ex(_ptr(q), _ptr(k), _ptr(v), _ptr(o_part), _ptr(lse), B, H, Lq, Lk, d,
                                      cr, qst, _DTYPES[q.dtype], _PDTYPES[partial_dtype], _stream(q)))
    return o_part, lse


def combine(o_part, lse, B, H, dtype, out=None):
    """Combine ``S`` partials o_part ``[S, B*H, L, d]`` / lse ``[S, B*H, L]`` -> ``[B, H, L, d]``.

    An lse of shape ``[S, B*H, L, 2]`` marks fp16 per-row scaled partials (``attention_partial``
    with ``PARTIAL_FP16_SCALED``)."""
    _check_tensor("o_part", o_part, ndim=4)
    scaled = lse.dim() == 4
    _check_tensor("lse", lse, torch.float64 if o_part.dtype == torch.float64 else torch.float32,
                  o_part.device, ndim=4 if scaled else 3)
    S, BH, L, d = o_part.shape
    if BH != B * H or tuple(lse.shape) != ((S, BH, L, 2) if scaled else (S, BH, L)):
        raise ValueError(f"inconsistent shapes o_part {tuple(o_part.shape)} lse {tuple(lse.shape)} "
                         f"B={B} H={H}")
    if scaled and o_part.dtype != torch.float16:
        raise ValueError(f"scaled partials (lse [..., 2]) are fp16, got {o_part.dtype}")
    o = _out(out, o_part, (B, H, L, d), dtype)
    pd = PARTIAL_FP16_SCALED if scaled else o_part.dtype
    _launched(lib().fa_combine(_ptr(o_part), _ptr(lse), _ptr(o), S, B, H, L, d, _DTYPES[dtype],
                           _PDTYPES[pd], _stream(o_part)))
    return o


def kernel_geometry(d, dtype=torch.bfloat16):
    """(bq, bk, threads, lds_bytes) the library uses for head dim d."""
    return _lib.geometry(d, _DTYPES[dtype])
