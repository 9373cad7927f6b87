/* fa_mi355x_dist.h -- C ABI of the multi-GPU split-KV forward (libfa_mi355x_dist.so).
 *
 * the north star's "split-KV two-kernel path sharded across the GPUs of
 * one node with an RCCL exchange for the combine step".  The reference has no multi-GPU
 * path; its single-GPU split-KV launcher is flash_attention_v2(Q,K,V,O,B,H,L,d,d_tile_qk,
 * d_tile_v,kv_tiles_per_block), flash_attention_v2/CUDA/flash_attention_v2.h:438, whose
 * partial_attention_kernel (:243) and reduction_kernel (:356) become, per rank:
 *
 *   1. the partial kernel (fa_fwd_partial_ex) over the rank's key shard, one launch per
 *      destination chunk of query rows (chunk p = the rows rank p will own), written in the
 *      send layout [W][B*H][L/W][d] (+ lse [W][B*H][L/W]);
 *   2. as soon as chunk p is queued, one RCCL send/recv step on the communicator's own
 *      stream: step s sends chunk rank+s to rank+s and receives chunk rank from rank-s -- a
 *      shifted exchange, every step a perfect matching (all xGMI links busy at once, where a
 *      ring reduce-scatter would serialise on one link per step) -- so the transfer of one
 *      chunk overlaps the next chunk's kernel; the rank's own chunk is computed last, straight
 *      into the receive buffer (it never crosses a link);
 *   3. fa_combine of the W partials -> the rank's rows [B, H, L/W, d] of O, once the exchange
 *      stream has finished (an event, no host wait);
 *   4. optionally an RCCL all-gather (+ a strided copy) -> the full [B, H, L, d] O.
 *
 * One process per GPU.  Kept in its own library so that processes that never shard (and
 * PyTorch's own RCCL) are not touched by it.  Same status codes and fa_last_error() as
 * fa_mi355x.h.
 */
#ifndef FA_MI355X_DIST_H
#define FA_MI355X_DIST_H

#include <stddef.h>
#include <stdint.h>

#include "fa_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

#define FA_DIST_UNIQUE_ID_BYTES 128 /* sizeof(ncclUniqueId) */
#define FA_ERR_RCCL 5               /* an RCCL call failed (message in fa_dist_last_error) */

const char* fa_dist_last_error(void);

/* Rank 0 creates the communicator id; the caller ships its 128 bytes to every rank. */
int fa_dist_get_unique_id(void* id);

/* Collective over all `world` ranks (each on its own device, set current beforehand).  The
 * handle owns the RCCL communicator plus the exchange stream and events the forward uses, all
 * created here so that fa_fwd_v2_dist itself never allocates. */
int fa_dist_comm_init(void** comm, int world, int rank, const void* id);
int fa_dist_comm_destroy(void* comm);

/* Workspace of fa_fwd_v2_dist: send + receive partials and lse, plus the all-gather
 * staging buffer.  L must be divisible by world.  partial_dtype (the exchanged format):
 * the input dtype, FA_DTYPE_FP32 or FA_DTYPE_FP16_SCALED (bf16's bytes, 11 significant
 * bits; fa_fwd_partial's layout, include/fa_mi355x.h); FA_DTYPE_FP64 for fp64 inputs. */
int fa_fwd_v2_dist_workspace_size(int64_t B, int64_t H, int64_t L, int64_t d, int world,
                                  int dtype, int partial_dtype, size_t* bytes);

/* q: [B, H, L, d] (identical on every rank); k_shard, v_shard: this rank's keys
 * [B, H, L/W, d] (rank r holds keys [r*L/W, (r+1)*L/W)); o: this rank's query rows
 * [B, H, L/W, d] of O, or the full [B, H, L, d] O when gather != 0.  Asynchronous on
 * `stream`: the kernels and the all-gather run on it, the send/recv steps on the handle's
 * exchange stream, ordered against it by events.  Every argument is checked before anything
 * is enqueued (a call that returns an error has posted nothing to the peers).  A failure that
 * strikes after the first exchange step was posted -- a kernel launch, an event record or
 * wait, a later step's RCCL enqueue, or, with gather, the combine or the all-gather -- leaves
 * the peers waiting on posts this rank will never make: it returns the error and marks the
 * handle unusable (later calls refuse with FA_ERR_RCCL; destroy it).  The schedule and this
 * latch are csrc/fa_dist_schedule.hpp, tested on the CPU with an in-process transport. */
int fa_fwd_v2_dist(const void* q, const void* k_shard, const void* v_shard, void* o,
                   int64_t B, int64_t H, int64_t L, int64_t d, void* comm, int gather,
                   void* workspace, size_t workspace_bytes, int dtype, int partial_dtype,
                   void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FA_MI355X_DIST_H */
