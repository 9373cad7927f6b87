// Instantiates only the chained d = 128 kernels (final and fused walk, bf16) so that
// tests/test_vmcnt.py can compile them to ISA quickly and check their hand-counted vmcnt waits
// (scripts/check_vmcnt.py).  Not linked into anything.
#include "../../exploring_flash_attention_amd/csrc/fa_fwd_kernel.hpp"  // (FA_STAMP macros)
#include "../../exploring_flash_attention_amd/csrc/fa_fwd16_chain.hpp"

namespace fa {
template __global__ void fa_fwd16_chain_kernel<__bf16, kFinal>(FwdArgs, int);
template __global__ void fa_fwd16_chain_kernel<__bf16, kFused>(FwdArgs, int);
}  // namespace fa
