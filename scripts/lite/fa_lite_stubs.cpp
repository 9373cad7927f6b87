// Stubs of the launchers a "lite" A/B build leaves out (scripts/build_lite.sh): only the
// contiguous bf16 forward of fa_fwd.hip is compiled there, so that one kernel variant builds
// in seconds.  Never part of the product library.
#include "../../exploring_flash_attention_amd/csrc/fa_internal.hpp"
namespace fa {
hipError_t launch_fwd_strided(Elem, Elem, int, Mode, const FwdArgs&, hipStream_t) { return hipErrorInvalidValue; }
hipError_t launch_combine(Elem, Elem, int, const CombineArgs&, hipStream_t) { return hipErrorInvalidValue; }
hipError_t launch_fwd64(int, Mode, const FwdArgs&, hipStream_t) { return hipErrorInvalidValue; }
hipError_t launch_combine64(int, const CombineArgs&, hipStream_t) { return hipErrorInvalidValue; }
int fwd64_rows_per_block() { return 64; }
int fwd64_keys_per_tile() { return 16; }
// (weak: a lite build of the d-tiled kernel links fa_fwd_dtiled.hip's real definitions)
__attribute__((weak)) hipError_t launch_fwd_dtiled(Elem, int, const FwdArgs&, hipStream_t) { return hipErrorInvalidValue; }
hipError_t launch_fwd64_dtiled(int, const FwdArgs&, hipStream_t) { return hipErrorInvalidValue; }
__attribute__((weak)) int dtiled_rows_per_block() { return 64; }
__attribute__((weak)) int dtiled_lds_bytes(int d) { return (d <= 384 ? 3 : 4) * 16384; }
__attribute__((weak)) void dtiled_geometry(Elem, int d, int* rows, int* threads, int* lds) {
    *rows = 64;
    *threads = 256;
    *lds = dtiled_lds_bytes(d);
}
}  // namespace fa
