"""CPU oracle for the flash-attention forward path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything in this package, and only as the checker (or the timed CPU baseline),
never as the thing measured or shipped.  The product path
(``exploring_flash_attention_amd``) never imports it and fails loudly when its HIP
library is missing.

Contents, each a restatement of the reference (tyler-utah/exploring_flash_attention,
paths relative to its root) -- see each function's docstring for file:line:

* ``reference``  -- ``naive_attention`` / ``check_accuracy`` (common/reference.py)
* ``fa_v1``      -- FA-v1 tiled forward: high-level form (flash_attention_v1/numpy_basic.py)
                    and the fused C-style form used as the CPU baseline
                    (flash_attention_v1/numpy_gpu_like_opt2.py)
* ``tiled_d``    -- d-tiled FA-v1 (flash_attention_v1_tiled_d/numpy_basic.py)
* ``splitkv``    -- FA-v2 split-KV partial + reduction (flash_attention_v2/numpy_gpu_like.py)
* ``batched``    -- vectorised fp64 attention over [B, H, L, d] for GPU parity checks
* ``standard_attention.c`` -- C/OpenMP restatement of standard_attention_cpu
                    (common/standard.h:28-102), built by ``oracle/Makefile``

Parity pinning: every restatement is checked against golden vectors generated in the
build container by importing the reference's own Python (``tests/golden/make_golden.py``),
see ``tests/test_oracle.py``.  The reference's C++ oracle ``common/standard.h`` includes
``cuda_runtime.h``/``cuda_fp16.h`` and is unbuildable in this image without stand-in
headers, so it is not compiled; its restatement is pinned against the
Python reference instead.
"""
