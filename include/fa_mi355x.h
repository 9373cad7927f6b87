/*
 * fa_mi355x.h -- C ABI of the MI355X (gfx950) flash-attention forward library
 * (libfa_mi355x.so, built from exploring_flash_attention_amd/csrc/).
 *
 * Computes the exact, non-causal attention forward O = softmax(Q K^T / sqrt(d)) V
 * over contiguous row-major [B, H, L, d] tensors held in device memory (HBM).
 * All entry points are asynchronous on the caller's HIP stream (pass NULL for the
 * null stream), never allocate, never synchronise the device, and return an
 * fa_status_t.  On failure fa_last_error() returns a thread-local message.
 *
 * Each entry point replaces one host launcher of the reference
 * (tyler-utah/exploring_flash_attention, paths relative to its root):
 *
 *   fa_fwd_v1          <- flash_attention_v1(Q,K,V,O,B,H,L,d)
 *                           flash_attention_v1/CUDA/flash_attention_v1.h:251
 *                         flash_attention_v1_opt1(Q,K,V,O,B,H,L,d)
 *                           flash_attention_v1/CUDA/flash_attention_v1_opt1.h:354
 *   fa_fwd_v1_tiled_d  <- flash_attention_v1(Q,K,V,O,B,H,L,d,d_tile_qk,d_tile_v)
 *                           flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:312
 *                         flash_attention_v1_opt(...)
 *                           flash_attention_v1_tiled_d/CUDA/flash_attention_v1_opt.h:448
 *   fa_fwd_v2_workspace_size + fa_fwd_v2
 *                      <- flash_attention_v2(Q,K,V,O,B,H,L,d,d_tile_qk,d_tile_v,kv_tiles_per_block)
 *                           flash_attention_v2/CUDA/flash_attention_v2.h:438 (opt: _opt.h:559)
 *                         The reference cudaMallocs/frees its workspace inside every call
 *                         (flash_attention_v2.h:461-463, :506-508); here the caller owns it.
 *   fa_fwd_partial     <- partial_attention_kernel  flash_attention_v2/CUDA/flash_attention_v2.h:243
 *   fa_combine         <- reduction_kernel          flash_attention_v2/CUDA/flash_attention_v2.h:356
 *                         (exposed separately so a multi-GPU caller can put an RCCL exchange
 *                         between the two kernels; the reference has no multi-GPU path)
 *
 * Differences from the reference contract, all deliberate:
 *   - the reference launchers return void, assert() on bad arguments and end with
 *     cudaDeviceSynchronize(); these return a status and never synchronise;
 *   - the reference element type is __half (or double under USE_FP64); here the
 *     element type is a runtime argument (FA_DTYPE_BF16, FA_DTYPE_FP16 or FA_DTYPE_FP64);
 *   - the reference fixes the head dim at compile time (assert(d == D),
 *     flash_attention_v1/CUDA/flash_attention_v1.h:264); here d is dispatched at run
 *     time to kernels for d in {32, 64, 128, 256} and, through fa_fwd_v1 / fa_fwd_v1_tiled_d
 *     and the unsplit fa_fwd_v2, the d-tiled kernels for d in {384, 512}; any other d returns
 *     FA_ERR_UNSUPPORTED (the *_scaled entry points let a caller zero-pad any d <= 512);
 *   - sizes are int64_t and every offset is 64-bit (the reference overflows int32 in
 *     its workspace index at L=4096, flash_attention_v2/CUDA/flash_attention_v2.h:324).
 */
#ifndef FA_MI355X_H
#define FA_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum fa_status {
    FA_OK = 0,
    FA_ERR_INVALID_ARG = 1,  /* null pointer, non-positive size, bad tile argument */
    FA_ERR_UNSUPPORTED = 2,  /* head dim / dtype without a kernel */
    FA_ERR_HIP = 3,          /* a HIP runtime call failed (launch, attribute) */
    FA_ERR_WORKSPACE = 4     /* workspace missing or smaller than fa_fwd_v2_workspace_size */
} fa_status_t;

typedef enum fa_dtype {
    FA_DTYPE_FP16 = 0,       /* IEEE binary16 storage, fp32 accumulate */
    FA_DTYPE_BF16 = 1,       /* bfloat16 storage, fp32 accumulate */
    FA_DTYPE_FP32 = 2,       /* only valid as the split-KV partial-output type */
    FA_DTYPE_FP16_SCALED = 4, /* only as a partial-output type (fa_fwd_v2, fa_fwd_partial,
                                 fa_combine): fp16 partials scaled per row by a power of two
                                 (the row's largest |value| below 1), the exponent kept beside
                                 the lse -- half the traffic of FA_DTYPE_FP32, 11 significant
                                 bits relative to each row's maximum, no fp16 range limit */
    FA_DTYPE_FP64 = 3        /* IEEE binary64 throughout (the reference's USE_FP64 build,
                                flash_attention_v1/CUDA/flash_attention_v1.h:29-41): fp64
                                MFMA, fp64 softmax, fp64 partials and lse */
} fa_dtype_t;

/* ABI version.  Callers built against one minor version must rebuild for another:
 *   0.2 -- fa_fwd_v2_ex and fa_fwd_v2_split_plan gained the int blocks_per_workgroup argument
 *          (inserted before workspace / dtype), fa_fwd_v2_workspace_size_ex was added;
 *   0.3 -- head dims 384 and 512 (the d-tiled kernels: fa_fwd_v1, fa_fwd_v1_tiled_d, and
 *          fa_fwd_v2 unsplit), fa_fwd_v1_tiled_d_scaled added;
 *   0.4 -- fa_last_kernels and fa_fwd_v2_ex2 (FA_V2_COUNTERS_ZERO) added (no signature changed).
 * fa_version() returns the library's (major << 16) | (minor << 8) | patch; check it against
 * these macros at load time. */
#define FA_MI355X_VERSION_MAJOR 0
#define FA_MI355X_VERSION_MINOR 4
int fa_version(void);

/* Thread-local message describing the last non-FA_OK status on this thread. */
const char* fa_last_error(void);

/* Thread-local description of the kernels the last launching call on this thread enqueued
 * (fa_fwd_v1*, fa_fwd_v1_tiled_d*, fa_fwd_v2*, fa_fwd_partial*, fa_combine), each with its
 * grid, joined by " + ", e.g. "fa_fwd16_chain_kernel<final> [grid 512]".  Valid after an FA_OK
 * return; the reference's launchers have no equivalent (a profiling aid: which of the
 * library's kernels and grids served the call, as the launcher chose them).  The grids of the
 * d = 128 persistent kernels are sized from the compute units of the device that owns
 * `stream`; the split-KV plan (fa_fwd_v2_split_plan, the workspace size) from the current
 * device's -- call them with the stream's device current. */
const char* fa_last_kernels(void);

/* Geometry the library uses for (d, dtype): query rows per workgroup (*bq),
 * keys per KV tile (*bk), threads per workgroup (*threads), LDS bytes per workgroup
 * (*lds_bytes).  Any output pointer may be NULL. */
int fa_kernel_geometry(int64_t d, int dtype, int* bq, int* bk, int* threads,
                       int* lds_bytes);

/* FA-v1 fused forward.  q, k, v, o: [B, H, L, d] contiguous, element type dtype.
 * d = 384 / 512 run the d-tiled kernel with 128-column tiles (fa_fwd_v1_tiled_d). */
int fa_fwd_v1(const void* q, const void* k, const void* v, void* o,
              int64_t B, int64_t H, int64_t L, int64_t d,
              int dtype, void* stream);

/* fa_fwd_v1 with an explicit softmax scale: O = softmax(softmax_scale * Q K^T) V.
 * softmax_scale > 0 and finite (else FA_ERR_INVALID_ARG); fa_fwd_v1 passes 1/sqrt(d).
 * Lets a caller run a head dim without its own kernel by zero-padding Q, K and V to a
 * supported d (zero columns add nothing to Q K^T; the padded O columns come out zero)
 * while keeping the scale of the true head dim -- the reference's Python functions take any
 * d (e.g. flash_attention_v1/numpy_gpu_like_opt2.py:198 with d = 16); the Python layer
 * (exploring_flash_attention_amd/ops.py) does exactly this. */
int fa_fwd_v1_scaled(const void* q, const void* k, const void* v, void* o,
                     int64_t B, int64_t H, int64_t L, int64_t d, double softmax_scale,
                     int dtype, void* stream);
/* fa_fwd_v1_scaled on strided tensors.  q_strides, kv_strides (shared by k and v) and
 * o_strides each point to three element strides {batch, head, row} of a [B, H, L, d] view
 * whose d is contiguous -- e.g. a [B, L, H, d] tensor is {L*H*d, d, H*d} -- or are NULL for
 * contiguous [B, H, L, d].  Strides must be positive multiples of 8 elements (16-byte row
 * starts), row strides >= d, and one head's rows must span < 2 GiB; bf16 / fp16 only
 * (FA_DTYPE_FP64 with strides: FA_ERR_UNSUPPORTED).  No copy is made. */
int fa_fwd_v1_ex(const void* q, const void* k, const void* v, void* o,
                 int64_t B, int64_t H, int64_t L, int64_t d,
                 const int64_t* q_strides, const int64_t* kv_strides, const int64_t* o_strides,
                 double softmax_scale, int dtype, void* stream);
/* FA-v1 d-tiled forward.  d_tile_qk / d_tile_v must satisfy 0 < d_tile <= d
 * (the reference's asserts, flash_attention_v1_tiled_d/CUDA/flash_attention_v1.h:326-327),
 * otherwise FA_ERR_INVALID_ARG.  d in {32, 64, 128, 256, 384, 512}.
 *   d <= 256: one LDS tile holds a whole row, and the fused kernel runs (its QK^T accumulates
 *   32-column k-steps, its O stays in VGPRs); the tiles are validated and do not change it.
 *   d = 384 / 512 (the head dims the variant exists for): the d-tiled kernel streams each
 *   64-key K tile through LDS in [64][d_tile_qk] column chunks and each V tile in
 *   [64][d_tile_v] chunks, O_acc in VGPRs for all d columns; a tile is honoured at the MFMA's
 *   granularity -- rounded down to 32, 64 or 128 columns (at least 32).  QK^T sums the same
 *   k-steps in the same order whatever the tiles, so the output does not depend on them.
 * FA_DTYPE_FP64 takes the same paths in fp64 (d = 384 / 512: 16-key tiles, Q chunks re-read
 * per tile as the reference does, :159-164). */
int fa_fwd_v1_tiled_d(const void* q, const void* k, const void* v, void* o,
                      int64_t B, int64_t H, int64_t L, int64_t d,
                      int d_tile_qk, int d_tile_v,
                      int dtype, void* stream);
/* fa_fwd_v1_tiled_d with an explicit softmax scale (as fa_fwd_v1_scaled: lets a caller zero-pad
 * a head dim without its own kernel, e.g. 257..511, to 384 or 512; the tiles are checked
 * against the d passed here). */
int fa_fwd_v1_tiled_d_scaled(const void* q, const void* k, const void* v, void* o,
                             int64_t B, int64_t H, int64_t L, int64_t d,
                             int d_tile_qk, int d_tile_v, double softmax_scale,
                             int dtype, void* stream);

/* kv_tiles_per_block value that lets the library choose the split from the device's
 * occupancy: no split when the query tiles alone number at least the device's compute units,
 * otherwise ceil(CUs / query tiles) splits (about one workgroup per CU) -- and, for d = 128
 * with 16-bit inputs, ceil(2 * CUs / query tiles) splits (two workgroups per CU) whenever
 * every split then still keeps at least 4096 keys (e.g. B1 H1 L16384: 128 query tiles on 256
 * CUs -> 4 splits, not 2).  The reference's README presets (flash_attention_v2/README.md:29-32)
 * made automatic. */
#define FA_KV_TILES_AUTO (-1)

/* blocks_per_workgroup value that lets the library group the key blocks of a query tile onto
 * workgroups itself (fa_fwd_v2_split_plan). */
#define FA_BLOCKS_PER_WG_AUTO 0

/* Bytes of device workspace fa_fwd_v2 needs for this problem.  A split (the reference's key
 * block) is kv_tiles_per_block * bk keys (bk from fa_kernel_geometry).  partial_dtype is
 * FA_DTYPE_FP32, the input dtype or FA_DTYPE_FP16_SCALED.  *num_splits (may be NULL)
 * receives the number of key blocks.  The size covers the partials fa_fwd_v2 actually moves
 * through the workspace (fa_fwd_v2_split_plan); it depends on the device's occupancy.
 * FA_ERR_UNSUPPORTED when the grid of (query tile, partial, b*h) workgroups exceeds 2^31 - 1
 * or a query tile would have more than 65535 partials (the in-kernel combine counts arrivals
 * and completions in 16-bit halves of one counter): raise kv_tiles_per_block. */
int fa_fwd_v2_workspace_size(int64_t B, int64_t H, int64_t L, int64_t d,
                             int kv_tiles_per_block, int dtype, int partial_dtype,
                             size_t* bytes, int* num_splits);
/* fa_fwd_v2_workspace_size for fa_fwd_v2_ex's blocks_per_workgroup (FA_BLOCKS_PER_WG_AUTO:
 * the library's grouping, as fa_fwd_v2_workspace_size). */
int fa_fwd_v2_workspace_size_ex(int64_t B, int64_t H, int64_t L, int64_t d,
                                int kv_tiles_per_block, int blocks_per_workgroup,
                                int dtype, int partial_dtype, size_t* bytes, int* num_splits);

/* How fa_fwd_v2 schedules the key blocks of a query tile: *key_blocks = ceil(L / (kv_tiles_per_block
 * * bk)) (the reference's partials), *blocks_per_wg_out consecutive blocks per workgroup
 * (combined on chip: the online softmax carried across them), *partials_per_tile partial
 * workgroups per query tile (combined through the workspace).  With blocks_per_workgroup =
 * FA_BLOCKS_PER_WG_AUTO the library cuts the blocks of a query tile into equal groups: none beyond
 * one when the query tiles alone number at least the device's compute units, otherwise
 * ceil(CUs / query tiles) groups (about one workgroup per CU) -- for d = 128 with 16-bit inputs
 * ceil(2 * CUs / query tiles) groups (two per CU) when each group then keeps >= 4096 keys
 * (B1 H1 L16384 on 256 CUs: 4 partials per tile); d = 384 / 512: always one group;
 * a positive value fixes the group size (1: one key block per group, the reference's layout;
 * clamped to the number of blocks).  *partials_per_tile counts the groups, i.e. the partials
 * of a tile; how they are scheduled: one workgroup per group (the one-shot grid), except at
 * d = 128 with 16-bit inputs and scaled-fp16 partials when the query tiles alone fill a grid
 * of two workgroups per CU (B*H*ceil(L/128) >= 2 * CUs), groups of a multiple of 128 keys (at
 * least 256) and L a multiple of 128 -- then a persistent grid of 2 workgroups per CU WALKS each query tile's
 * groups one after another on one workgroup (the "walk", fa_last_kernels:
 * "fa_fwd16_chain_kernel<fused walk>"), stores the first partials_per_tile - 1 partials and
 * combines them with the last one, still in its registers.  The plan depends only on the
 * arguments and the current device's compute-unit count.  Any output pointer may be NULL. */
int fa_fwd_v2_split_plan(int64_t B, int64_t H, int64_t L, int64_t d, int kv_tiles_per_block,
                         int blocks_per_workgroup, int dtype, int* key_blocks,
                         int* blocks_per_wg_out, int* partials_per_tile);

/* FA-v2 split-KV forward: per (q-tile, group of key blocks, b*h) the keys' normalised partial
 * O and log-sum-exp go into the workspace, and the tile's partials are combined with
 * fa_combine's formula inside the same launch (the reduction kernel's maths without its
 * separate pass over HBM) -- either by the last of the tile's workgroups to finish (one-shot
 * grid: one workgroup per group, an arrival counter per tile), or by the workgroup that walks
 * all of the tile's groups in turn (the persistent walk, see fa_fwd_v2_split_plan: no
 * counters, partials_per_tile - 1 partials through HBM).  One partial per q-tile
 * (fa_fwd_v2_split_plan): the plain FA-v1 kernel.  workspace: device buffer of at least fa_fwd_v2_workspace_size bytes,
 * 256-byte aligned, contents need not be initialised (a hipMemsetAsync of its counters
 * precedes the launch on `stream`).  d_tile_qk / d_tile_v as for fa_fwd_v1_tiled_d. */
int fa_fwd_v2(const void* q, const void* k, const void* v, void* o,
              int64_t B, int64_t H, int64_t L, int64_t d,
              int d_tile_qk, int d_tile_v, int kv_tiles_per_block,
              void* workspace, size_t workspace_bytes,
              int dtype, int partial_dtype, void* stream);

/* fa_fwd_v2 with an explicit softmax scale (as fa_fwd_v1_scaled). */
int fa_fwd_v2_scaled(const void* q, const void* k, const void* v, void* o,
                     int64_t B, int64_t H, int64_t L, int64_t d,
                     int d_tile_qk, int d_tile_v, int kv_tiles_per_block,
                     void* workspace, size_t workspace_bytes, double softmax_scale,
                     int dtype, int partial_dtype, void* stream);
/* fa_fwd_v2_scaled on strided q, k, v, o (strides as for fa_fwd_v1_ex), with an explicit key-block
 * grouping (blocks_per_workgroup as for fa_fwd_v2_split_plan; FA_BLOCKS_PER_WG_AUTO = the
 * library's); the workspace is sized by fa_fwd_v2_workspace_size_ex with the same value. */
int fa_fwd_v2_ex(const void* q, const void* k, const void* v, void* o,
                 int64_t B, int64_t H, int64_t L, int64_t d,
                 int d_tile_qk, int d_tile_v, int kv_tiles_per_block, int blocks_per_workgroup,
                 void* workspace, size_t workspace_bytes,
                 const int64_t* q_strides, const int64_t* kv_strides, const int64_t* o_strides,
                 double softmax_scale, int dtype, int partial_dtype, void* stream);
/* fa_fwd_v2_ex with flags (0, or FA_V2_COUNTERS_ZERO).  FA_V2_COUNTERS_ZERO: the caller
 * guarantees that the workspace's completion counters are zero -- it zeroed the whole
 * workspace once (hipMemset) and only fa_fwd_v2* calls with the same B, H, L, d,
 * kv_tiles_per_block, blocks_per_workgroup, dtype and partial_dtype (the same counter words)
 * have used it since, every one of which leaves its counters zero -- so the per-call counter
 * reset, a dispatch of its own on `stream`, is skipped.  A workspace with non-zero counters under this
 * flag gives wrong outputs or, for key blocks of >= 4096 keys, a kernel that never finishes:
 * pass 0 when in doubt.  The reference reallocates its workspace on every call
 * (flash_attention_v2/CUDA/flash_attention_v2.h:461-508). */
#define FA_V2_COUNTERS_ZERO 1u
int fa_fwd_v2_ex2(const void* q, const void* k, const void* v, void* o,
                  int64_t B, int64_t H, int64_t L, int64_t d,
                  int d_tile_qk, int d_tile_v, int kv_tiles_per_block, int blocks_per_workgroup,
                  void* workspace, size_t workspace_bytes,
                  const int64_t* q_strides, const int64_t* kv_strides, const int64_t* o_strides,
                  double softmax_scale, int dtype, int partial_dtype, unsigned flags, void* stream);
/* Split-KV partial forward over ONE key range (a whole KV shard, e.g. one GPU's
 * slice of the sequence).  q: [B, H, Lq, d]; k, v: [B, H, Lk, d].
 * Writes, for every query row, the normalised partial output and its log-sum-exp
 * (base 2, of the scaled scores: lse = log2(sum_j 2^(s_j * log2(e)/sqrt(d)))):
 *   o_part[(row / chunk_rows)][b*H + h][row % chunk_rows][:]   (partial_dtype)
 *   lse   [(row / chunk_rows)][b*H + h][row % chunk_rows]      (fp32; fp64 for FP64)
 * chunk_rows must divide Lq.  chunk_rows = Lq gives a plain [B,H,Lq,d] layout;
 * chunk_rows = Lq / world gives the all-to-all send layout of the multi-GPU path.
 * partial_dtype FA_DTYPE_FP16_SCALED: o_part holds O_row * 2^-e_row in fp16 and lse holds
 * two floats per row, {lse, e} (lse [...][row % chunk_rows][2]); fa_combine undoes the scale. */
int fa_fwd_partial(const void* q, const void* k, const void* v,
                   void* o_part, void* lse,
                   int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t d,
                   int64_t chunk_rows, int dtype, int partial_dtype, void* stream);

/* fa_fwd_partial with a strided q: q_strides = {batch, head, row} element strides of the
 * [B, H, Lq, d] query view (NULL = contiguous), e.g. rows [c*Lq, (c+1)*Lq) of a longer
 * [B, H, L, d] tensor -- the multi-GPU path computes one destination rank's chunk of the
 * partials per launch this way, so the exchange of one chunk overlaps the next one's
 * compute.  k, v contiguous; bf16 / fp16 only when strided. */
int fa_fwd_partial_ex(const void* q, const void* k, const void* v,
                      void* o_part, void* lse,
                      int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t d,
                      int64_t chunk_rows, const int64_t* q_strides,
                      int dtype, int partial_dtype, void* stream);
/* Combine num_splits partials: o_part [num_splits][B*H][L][d] (partial_dtype),
 * lse [num_splits][B*H][L] (fp32, base 2; fp64 for FA_DTYPE_FP64; [num_splits][B*H][L][2]
 * {lse, e} for FA_DTYPE_FP16_SCALED) -> o [B, H, L, d] (dtype), using
 * O = sum_s 2^(lse_s - M) O_s / sum_s 2^(lse_s - M), M = max_s lse_s
 * (the reference's formula, flash_attention_v2/numpy_gpu_like.py:269-288, on
 * normalised partials). */
int fa_combine(const void* o_part, const void* lse, void* o,
               int64_t num_splits, int64_t B, int64_t H, int64_t L, int64_t d,
               int dtype, int partial_dtype, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FA_MI355X_H */
