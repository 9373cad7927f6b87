"""exploring_flash_attention_amd -- MI355X (gfx950)-native flash-attention forward.

Drop-in for the attention-forward path of tyler-utah/exploring_flash_attention: the same
``Q, K, V -> O`` call surfaces (``v1``, ``tiled_d``, ``v2`` modules mirror the reference's
flash_attention_v1 / flash_attention_v1_tiled_d / flash_attention_v2 families), backed by
hand-written CDNA4 HIP kernels behind a C ABI (include/fa_mi355x.h,
``_lib/libfa_mi355x.so``).  ``ops`` has the zero-copy device-tensor operators and
``dist`` the split-KV forward sharded over the GPUs of a node with RCCL.

There is no CPU fallback: every entry point raises if the HIP library is not built or no
ROCm device is present.
"""
from . import ops  # noqa: F401
from .ops import (attention_partial, attention_tiled_d, attention_v1, attention_v2,  # noqa: F401
                  combine, kernel_geometry)
from .tiled_d import flash_attention_v1_tiled_d  # noqa: F401
from .v1 import flash_attention_v1  # noqa: F401
from .v2 import flash_attention_v2  # noqa: F401

__all__ = ["ops", "attention_v1", "attention_tiled_d", "attention_v2", "attention_partial",
           "combine", "kernel_geometry", "flash_attention_v1", "flash_attention_v1_tiled_d",
           "flash_attention_v2"]
__version__ = "0.1.0"
