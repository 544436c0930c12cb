/*
 * zero_amd.h — C ABI of the MI355X-native ZeRO sharded-optimizer step.
 *
 * The reference (xo-toybox/distributed-training-sandbox, zero/zero{1,2,3}.py) has no native code:
 * its hot path is Python calling c10d collectives and torch.optim.Adam.  This library is what the
 * drop-in ShardedOptimizer (distributed-training-sandbox_amd/zero_amd/zero{1,2,3}.py) binds with
 * ctypes.  Every entry point below names the reference interface it replaces.
 *
 * Conventions
 *  - plain C types only: no torch types cross this boundary; device buffers are raw pointers
 *    (uint64_t / void*) owned by the caller (torch tensors); the library never frees caller memory.
 *  - every launch takes a hipStream_t passed as uintptr_t (torch.cuda.Stream.cuda_stream);
 *    nothing synchronises the host except *_create (table upload) and zs_comm_init.
 *  - every function returns int status: ZS_OK (0) or a ZS_ERR_* code; zs_last_error() returns a
 *    thread-local message for the most recent failure on the calling thread.
 *  - element counts are int64_t elements; byte counts say "bytes".
 */
#ifndef ZERO_AMD_H
#define ZERO_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Callers check zs_abi_version() == ZS_ABI_VERSION before any other call: version 7 kept the
 * names zs_plan_create / zs_adam_step but changed their argument lists (the version-6 forms are
 * the *_ex entry points), so a caller built against an older header links and then passes the
 * wrong arguments.  The Python binding (zero_amd/_lib.py) and tests/c/abi_host.c refuse a
 * mismatch. */
#define ZS_ABI_VERSION 13

enum zs_status {
  ZS_OK = 0,
  ZS_ERR_INVALID = 1,   /* bad argument / shape mismatch */
  ZS_ERR_HIP = 2,       /* hipError_t from the runtime */
  ZS_ERR_RCCL = 3,      /* ncclResult_t from RCCL */
  ZS_ERR_NOMEM = 4
};

enum zs_dtype {
  ZS_F32 = 0,
  ZS_BF16 = 1,
  ZS_U8 = 2,        /* raw bytes (fp8 payloads); collectives only */
  ZS_BF16_SPLIT = 3 /* zs_adamset_create p_dtype only: the fp32 master stored as the bf16 param
                       (its round-to-nearest-even high half) + a 16-bit residual, see zs_adam_seg */
};

/* Shard layouts (SURVEY.md §7 "Two shard layouts"). */
enum zs_layout {
  ZS_LAYOUT_R = 0,  /* reference owner-by-parameter-index (zero1.py:55-62, zero2.py:51-58) */
  ZS_LAYOUT_Z = 1,  /* dim-0 chunk of every parameter, torch.chunk semantics (zero3.py:105-110) */
  ZS_LAYOUT_F = 2   /* flat: one balanced contiguous 1/ws slice of the concatenated params */
};

/* Bucketing of the per-rank streams (see zs_plan_bucket). */
enum zs_bucket_mode {
  ZS_BUCKETS_RAGGED = 0, /* equal windows over the shortest stream, then per-owner ragged windows */
  ZS_BUCKETS_PADDED = 1  /* equal windows over the longest stream, shorter streams zero-padded */
};

int zs_abi_version(void);
const char* zs_last_error(void);

/* roctx range around a phase of step(), named like the reference's torch.profiler ranges
 * "all_reduce_gradients" / "optimizer_step" / "broadcast_parameters" (zero1.py:80-91), so
 * `rocprofv3 --marker-trace` shows which kernels and collectives each phase enqueued.  Host only;
 * no-ops unless a profiler is attached. */
int zs_range_push(const char* name);
int zs_range_pop(void);

/* ------------------------------------------------------------------------------------------ */
/* Layout planner (host only; callable without a GPU).                                         */
/* ------------------------------------------------------------------------------------------ */
typedef struct zs_plan zs_plan;

/* Replaces ShardedOptimizer.__init__'s ownership computation (zero1.py:44-62, zero2.py:39-58,
 * zero3.py:82-110).  numels[i] = params[i].numel(); dim0[i] = params[i].shape[0] (1 for 0-d;
 * only read for ZS_LAYOUT_Z, may be NULL otherwise).  SURVEY.md §8(b)'s signature: bucket_bytes
 * is the size of one bucket buffer in fp32 elements' bytes (a bf16 bucket of the same plan holds
 * the same elements in half the bytes; 0 = one bucket holding the whole longest stream); pieces
 * are 64-element aligned; ragged buckets (ZS_BUCKETS_RAGGED). */
int zs_plan_create(int64_t n_params, const int64_t* numels, const int64_t* dim0, int ws, int rank,
                   int layout, int64_t bucket_bytes, zs_plan** out);
/* The general form the Python engine uses: align_elems: every piece starts at a multiple of this
 * in its rank's stream (>=1).  window_elems: per-rank elements per bucket (0 = one bucket holding
 * the whole longest stream).  bucket_mode: ZS_BUCKETS_*. */
int zs_plan_create_ex(int64_t n_params, const int64_t* numels, const int64_t* dim0, int ws,
                      int rank, int layout, int64_t align_elems, int64_t window_elems,
                      int bucket_mode, zs_plan** out);
int zs_plan_destroy(zs_plan* plan);

/* info[0..9] = {n_params, ws, rank, layout, window_elems W, num_buckets K, max_stream_len M,
 *              arena_elems (all buckets, each starting align_elems-aligned), num_even_buckets,
 *              bucket_mode} */
int zs_plan_info(const zs_plan* plan, int64_t* info10);

/* Parameter-index ownership [start,end) of `rank` (zero1.py:55-62).  Same formula for every
 * layout: it is what the reference uses to filter the inner optimizer's param_groups. */
int zs_plan_owner_range(const zs_plan* plan, int rank, int64_t* start, int64_t* end);

/* Broadcast-source rank of parameter i (zero1.py:95-100, zero2.py:126-131). */
int zs_plan_owner_of(const zs_plan* plan, int64_t i, int* owner);

/* Length (elements, padded to align) of rank r's stream = its optimizer shard. */
int zs_plan_stream_len(const zs_plan* plan, int rank, int64_t* len);

/* Pieces of rank r's stream: param index, element offset inside the (flattened) param,
 * element offset inside the stream, length.  Arrays sized by zs_plan_num_pieces. */
int zs_plan_num_pieces(const zs_plan* plan, int rank, int64_t* n);
int zs_plan_pieces(const zs_plan* plan, int rank, int64_t* param, int64_t* param_off,
                   int64_t* stream_off, int64_t* len);

/* Bucket k: its offset and length (elements) in the arena, whether it is *even* (every window
 * the same length and window r at r*len: one equal-count reduce-scatter / all-gather moves it;
 * buckets 0..num_even-1) or *ragged* (one grouped reduce / broadcast per owner moves it), and per
 * rank r (arrays of ws): the window's offset inside the bucket, its length (0 = no data), and the
 * stream offset of its first element.  Replaces the per-tensor collective loop over
 * self.params (zero1.py:80-84, zero2.py:94-113) with a fixed bucket schedule. */
int zs_plan_bucket(const zs_plan* plan, int64_t bucket, int64_t* arena_off, int64_t* elems,
                   int* even, int64_t* win_off, int64_t* win_len, int64_t* win_stream);

/* Segments of bucket k (all ranks): param slices and where they sit in the bucket buffer.
 * buf_off is the element offset inside the bucket buffer (win_off[rank] + offset in window). */
int zs_plan_num_segments(const zs_plan* plan, int64_t bucket, int64_t* n);
int zs_plan_segments(const zs_plan* plan, int64_t bucket, int64_t* param, int64_t* rank,
                     int64_t* param_off, int64_t* buf_off, int64_t* len);

/* Number of buckets K (= info[5]) and the byte size of bucket k's buffer for dtype ZS_F32 /
 * ZS_BF16 (SURVEY.md §8(b) zs_plan_num_buckets / zs_plan_bucket_bytes). */
int zs_plan_num_buckets(const zs_plan* plan, int64_t* n);
int zs_plan_bucket_bytes(const zs_plan* plan, int64_t bucket, int dtype, int64_t* bytes);

/* Pack / unpack one bucket straight from the plan (SURVEY.md §8(b) zs_pack / zs_unpack).
 * grad_ptrs / param_ptrs: n_params device pointers indexed by parameter (flattened, dtype ZS_F32
 * or ZS_BF16); bucket_buf: the bucket's buffer (zs_plan_bucket_bytes long).  zs_pack copies every
 * segment of every rank's window (zero2.py:99-104 without the ws-fold torch.cat) — a NULL grad
 * is written as zeros; zs_unpack scatters every segment back into the params (the per-tensor
 * broadcast of zero2.py:122-133 after the all-gather).  Window padding is never written: zero
 * the buffer once.  The descriptor tables are built on the first call and reused while the
 * pointers are unchanged; tables replaced by new pointers are kept until zs_plan_destroy, which
 * must not be called while a pack / unpack of the plan may still run. */
int zs_pack(zs_plan* plan, int64_t bucket, const uint64_t* grad_ptrs, void* bucket_buf, int dtype,
            uintptr_t stream);
int zs_unpack(zs_plan* plan, int64_t bucket, const void* bucket_buf, const uint64_t* param_ptrs,
              int dtype, uintptr_t stream);

/* ------------------------------------------------------------------------------------------ */
/* Segment copy (pack / unpack).  Replaces the flatten + torch.cat([g]*ws) copies of            */
/* zero2.py:99-104, the chunk().contiguous() copies of zero3.py:44-51,107-108,142-143 and the   */
/* torch.cat of gathered shards (zero3.py:40).                                                  */
/* ------------------------------------------------------------------------------------------ */
typedef struct zs_copyset zs_copyset;

/* src[i]==0 means "write nbytes[i] zero bytes to dst[i]".  The table is uploaded once. */
int zs_copyset_create(const uint64_t* src, const uint64_t* dst, const int64_t* nbytes, int64_t n,
                      zs_copyset** out);
int zs_copyset_run(const zs_copyset* cs, uintptr_t stream);
int zs_copyset_destroy(zs_copyset* cs);
/* The same copy without a table (ABI v11): the segments travel in the kernel arguments, up to 64
 * per launch (more take more launches), so pointers that change on every call cost nothing to
 * set up — backward's fresh gradients copied into their flat-arena slots (zero2.py:99-104's
 * flatten, per overlap bucket).  src[i]==0: zero fill; empty segments are skipped. */
int zs_copy_direct(int64_t n, const uint64_t* src, const uint64_t* dst, const int64_t* nbytes,
                   uintptr_t stream);

/* In-place x[i] /= div over n elements (dtype ZS_F32 / ZS_BF16, x 16-byte aligned): the
 * `param.grad /= dist.get_world_size()` of DDP's sync_gradients (DDP/ddp.py:45-47), applied to a
 * whole all-reduced gradient bucket.  fp32: IEEE division (reciprocal multiply when div is a power
 * of two, which is exact); bf16: computed in fp32, rounded to nearest even. */
int zs_scale(void* x, int64_t n, int dtype, double div, uintptr_t stream);

/* n elements fp32 -> bf16 (round to nearest even, NaN stays NaN) or bf16 -> fp32 (exact).  The
 * bf16 gradient exchange of fp32-parameter models: the reference reduces fp32
 * grads (zero2.py:107); converting them first halves the bytes every collective moves.  16-B
 * vector path when both buffers are 16-byte aligned, scalar otherwise. */
int zs_convert(const void* src, int src_dtype, void* dst, int dst_dtype, int64_t n, uintptr_t stream);

/* Row-wise fp8 (OCP E4M3, the gfx950 format) quantisation for the low-precision parameter
 * all-gather (the reference's torchao float8 all-gather, fp8/fp8_benchmark.py:79-81).
 * Row r of src (row_len elements, dtype ZS_F32 / ZS_BF16): amax = max|x|, inv = 448/amax,
 * dst[r, i] = e4m3(RNE(clamp(x * inv, ±448))), scales[r] = amax/448 (amax == 0: inv = scale = 1).
 * Dequantise: dst[r, i] = (float(q) * scales[r]) rounded to dst_dtype.  Replaces gathering the
 * bf16/fp32 shard in zero3.py:36-41 with 1 byte/element + 4 bytes/row. */
int zs_fp8_quantize_rows(const void* src, int src_dtype, void* dst, float* scales, int64_t rows,
                         int64_t row_len, uintptr_t stream);
int zs_fp8_dequantize_rows(const void* src, const float* scales, void* dst, int dst_dtype,
                           int64_t rows, int64_t row_len, uintptr_t stream);

/* A ZeRO-3 gather group's fp8 send side in one launch per 16 matrices (the per-module
 * materialize of zero3.py:36-41 with every matrix of the module at once): matrix m's rows
 * [0, rows[m]) of src[m] (row_len[m] elements each, src_dtype) are quantised exactly as by
 * zs_fp8_quantize_rows into q[m] / scales[m]; rows [rows[m], cs[m]) — the dim-0 chunk's padding
 * beyond this rank's real rows — are written as q = 0, scale = 1.  row_len[m] a multiple of 8,
 * src 16-B and q 8-B aligned. */
int zs_fp8_quantize_rowset(int64_t n, const uint64_t* src, const uint64_t* q, const uint64_t* scales,
                           const int64_t* rows, const int64_t* cs, const int64_t* row_len,
                           int src_dtype, uintptr_t stream);
/* The group's receive side after ONE all-gather of every rank's concatenated q buffer
 * (q_rank_bytes per rank) and ONE of its scales (sc_rank_elems per rank): full row R < ws*cs[m] of
 * matrix m is rank k = R / cs[m]'s local row lr = R % cs[m], read from
 * q + k*q_rank_bytes + q_off[m] + lr*row_len[m] with scale scales[k*sc_rank_elems + sc_off[m] + lr],
 * and written, dequantised to dst_dtype, at dst[m] + R*row_len[m] (16-B aligned).  One launch per
 * 16 matrices. */
int zs_fp8_dequantize_gathered(int64_t n, const void* q, const float* scales, int ws,
                               int64_t q_rank_bytes, int64_t sc_rank_elems, const int64_t* q_off,
                               const int64_t* sc_off, const int64_t* cs, const int64_t* row_len,
                               const uint64_t* dst, int dst_dtype, uintptr_t stream);

/* ------------------------------------------------------------------------------------------ */
/* Fused Adam / AdamW.  Replaces torch.optim.Adam.step on the owned shard (zero1.py:88,          */
/* zero2.py:120, zero3.py:161; math of torch/optim/adam.py:457-547) plus the grad averaging     */
/* (zero1.py:84 `p.grad /= ws`, zero2.py:111 `output / ws`, zero3.py:147).                      */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  uint64_t g;          /* gradient (reduced SUM over ranks), dtype g_dtype; 0 = zero gradient */
  uint64_t master;     /* fp32 master / param read by the update */
  uint64_t master_out; /* fp32 destination of the updated master (may equal master, may be a
                          bucket slot; 0 = not written) */
  uint64_t p_out;      /* optional copy of the updated param in p_dtype (bf16); 0 = none */
  uint64_t m;          /* fp32 exp_avg, updated in place */
  uint64_t v;          /* fp32 exp_avg_sq, updated in place */
  uint64_t vmax;       /* fp32 max_exp_avg_sq (amsgrad) or 0 */
  uint64_t carry;      /* fp32 ZeRO-1 carried average A_{t-1}, rewritten with A_t; or 0 */
  int64_t n;           /* elements */
} zs_adam_seg;
/* p_dtype ZS_BF16_SPLIT (bf16 params; g must be bf16): the fp32 master is not stored as such.
 * Its bits u are the bf16 param hi = RNE(u) and the int16 residual lo = u - (hi << 16):
 *   master     = bf16 param read (hi), 8-byte aligned for the vector path
 *   master_out = int16 residual lo, read and rewritten in place
 *   p_out      = bf16 param written (hi of the updated master; may equal master)
 * u = (hi << 16) + sign_extend(lo) exactly, except an exact tie that rounds down to an even hi
 * (residual +0x8000, 1 in 2^17 of uniformly random masters): that master is stored 1 ulp toward
 * zero (lo = 0x7FFF), the bf16 param unchanged.  26 instead of 28 B/element per update. */

typedef struct {
  /* scalars exactly as torch computes them (double on host, rounded to f32 once) */
  float one_minus_beta1;  /* lerp weight 1-beta1 */
  float beta2;
  float one_minus_beta2;
  float neg_step_size;    /* -(lr / (1 - beta1^t)) */
  float bc2_sqrt;         /* sqrt(1 - beta2^t) */
  float eps;
  float weight_decay;     /* L2 (Adam) coefficient; 0 = off */
  float decay_mul;        /* AdamW: 1 - lr*wd; 1 = off */
  float grad_div;         /* divide the reduced sum by this (world size) */
  float carry_mul;        /* ZeRO-1: sum += carry_mul * carry (ws-1) */
  int32_t amsgrad;
  int32_t maximize;
} zs_adam_hparams;

/* Fill hp the way torch.optim.Adam/AdamW (non-capturable path) derives its scalars at step t. */
int zs_adam_hparams_init(double lr, double beta1, double beta2, double eps, double weight_decay,
                         int decoupled, int amsgrad, int maximize, int64_t step, double grad_div,
                         double carry_mul, zs_adam_hparams* hp);

typedef struct zs_adamset zs_adamset;
/* g_dtype: dtype of every seg's g; p_dtype: ZS_BF16 (fp32 master, optional bf16 p_out) or
 * ZS_BF16_SPLIT (split master, above). All fp32 pointers of a seg must be 16-byte aligned and
 * bf16 / int16 pointers 8-byte aligned for the vector path; other segments take a scalar path. */
int zs_adamset_create(const zs_adam_seg* segs, int64_t n, int g_dtype, int p_dtype,
                      zs_adamset** out);
int zs_adamset_run(const zs_adamset* as, const zs_adam_hparams* hp, uintptr_t stream);
/* Re-point the set's gradients (ABI v12): g[i] (0 = zero gradient) replaces the g of the i-th
 * segment given to zs_adamset_create (n = that count).  The new pointers travel in the arguments
 * of a small patch kernel enqueued on `stream`, which rewrites the device tables in stream order:
 * no upload, no host synchronisation, nothing launched when every pointer is unchanged.  Runs of
 * the set enqueued on `stream` afterwards read the new gradients; the set must not run on another
 * stream concurrently.  A segment with a vector part needs its new g aligned as at creation (8 B
 * bf16, 16 B fp32), else ZS_ERR_INVALID and nothing is changed.  The reference's `step()` reads
 * `p.grad` wherever backward left it after `zero_grad()` (zero2.py:94-120, 138-139): at world
 * size 1 the update reads those fresh gradient tensors in place instead of copying them into an
 * arena first. */
int zs_adamset_set_grads(zs_adamset* as, int64_t n, const uint64_t* g, uintptr_t stream);
int zs_adamset_destroy(zs_adamset* as);
/* total elements covered by the set and algorithmic HBM bytes one run moves (with the gradients
 * bound now) */
int zs_adamset_stats(const zs_adamset* as, int64_t* elems, int64_t* bytes);

/* Single-range form, SURVEY.md §8(b)'s signature: one torch.optim.Adam/AdamW step over n
 * contiguous elements — the update of one flat shard (zero1.py:88 on a flattened group) with no
 * table to build.  p: fp32 master/param, updated in place; p_bf16: optional bf16 copy of the
 * result (NULL = none); g: reduced gradient sum (g_dtype ZS_F32 or ZS_BF16; NULL = zero); m, v:
 * fp32 exp_avg / exp_avg_sq, in place; carry: ZeRO-1's A_{t-1}, READ AND REWRITTEN with A_t
 * (NULL = none; SURVEY.md §8(b) spells it const, but the kernel writes it, so it is declared
 * writable — same C calling convention); carry_scale: ws-1.  grad_scale = 1/ws: the update
 * divides by the float nearest to 1/grad_scale (the world size), as zero1.py:84 `p.grad /= ws`.
 * The float scalars are widened to double before torch's bias-correction arithmetic; torch
 * derives them from Python doubles (adam.py:508-515), so for torch's bits with hyper-parameters
 * not exactly representable in fp32 (lr=1e-3, betas 0.9 / 0.999) use zs_adam_step_ex.  Same
 * kernels as zs_adamset_run; amsgrad / maximize / the split master need an adamset.
 * Asynchronous on `stream`; its two-entry table is a stream-ordered allocation. */
int zs_adam_step(float* p, uint16_t* p_bf16, const void* g, int g_dtype, float* m, float* v,
                 int64_t n, float lr, float b1, float b2, float eps, float wd, int decoupled,
                 int64_t step, float grad_scale, float* carry, float carry_scale,
                 uintptr_t stream);
/* The same with torch's double scalars and the divisor itself (grad_div = ws; for a
 * non-power-of-two ws dividing is not multiplying by 1/ws): bit-exact with torch's arithmetic. */
int zs_adam_step_ex(float* p, uint16_t* p_bf16, const void* g, int g_dtype, float* m, float* v,
                    int64_t n, double lr, double beta1, double beta2, double eps,
                    double weight_decay, int decoupled, int64_t step, double grad_div, float* carry,
                    double carry_mul, uintptr_t stream);

/* ------------------------------------------------------------------------------------------ */
/* Device buffers outside the caller's caching allocator (ABI v10).  The placement probe          */
/* (zero_amd/engine.py probed_zeros) streams candidate allocations of a long-lived, bandwidth-    */
/* bound buffer and keeps the fastest; candidates come from here so a rejected one goes straight */
/* back to the device without emptying torch's cache (the caller's cached blocks stay).          */
/* ------------------------------------------------------------------------------------------ */
/* hipMalloc of `bytes` (> 0) into *out; ZS_ERR_NOMEM when the device is full. */
int zs_device_alloc(int64_t bytes, void** out);
/* hipFree (NULL is a no-op).  Synchronises the device as hipFree does: only for buffers no queued
 * work still uses.  Also frees a zs_device_alloc_chunked range (unmap, release, address free). */
int zs_device_free(void* p);
/* (v13) `bytes` rounded up to whole `chunk_bytes` chunks: physical chunks of their own
 * (hipMemCreate) mapped side by side into one reserved virtual range, read / write for this
 * device.  The placement probe's second route (zero_amd/engine.py probed_zeros): tried when no
 * plain allocation streams at the acceptance rate.  Freed with zs_device_free. */
int zs_device_alloc_chunked(int64_t bytes, int64_t chunk_bytes, void** out);

/* Diagnostic A/B knobs (process-wide; the defaults are the measured best, so a product caller
 * never needs this): "dq_unroll" (4 / 8 / 16 accesses in flight per lane of the fp8 dequantise),
 * "dq_nt_store" (0 / 1: non-temporal stores), "dq_wg_per_cu" (0 = one wave per row; k = at most k
 * workgroups per CU walking several rows each), "scale_nt" (zs_scale's cache policy: -1 by size,
 * non-temporal above 256 MiB; 0 default policy; 1 non-temporal), "convert_nt" (zs_convert's, the
 * same by source + destination bytes), "copy_nt" (zs_copyset_run's, by 2 x the set's bytes),
 * "adam_wg_per_cu" (0 = 128 workgroups per CU, the default grid of the fused Adam; k = at most k
 * per CU), "sync_host_flags" (1: flag syncs created from now on take words in pinned host
 * memory, whose satisfied waits the host skips; 0: device words, every wait enqueued — the
 * fallback the library takes by itself when pinned memory is refused), "sync_write_kernel" (1: a
 * flag sync's record is a one-wave kernel storing the epoch with a system-scope release; 0:
 * hipStreamWriteValue64 — same ordering, the runtime's stream-operation command costs more host
 * time), "sync_write_fence" (1: that store is a system-scope release; 0: relaxed), "sync_wait_kernel"
 * (1: a flag wait is a one-wave kernel polling the word with s_sleep between loads; 0:
 * hipStreamWaitValue64, on this stack a runtime kernel spinning without pause beside the compute
 * stream's kernels).  *previous (may be NULL) gets the old value;
 * ZS_ERR_INVALID for an unknown key or value. */
int zs_tune(const char* key, int64_t value, int64_t* previous);

/* ------------------------------------------------------------------------------------------ */
/* RCCL over xGMI.  Replaces the per-tensor dist.all_reduce (zero1.py:83, zero3.py:146),        */
/* dist.reduce_scatter_tensor (zero2.py:107), dist.broadcast (zero1.py:102, zero2.py:133) and   */
/* dist.all_gather (zero3.py:39) with bucketed collectives on a caller stream.                  */
/* ------------------------------------------------------------------------------------------ */
typedef struct zs_comm zs_comm;
#define ZS_UNIQUE_ID_BYTES 128
int zs_comm_unique_id(void* out128);
int zs_comm_init(const void* unique_id128, int ws, int rank, zs_comm** out);
int zs_comm_destroy(zs_comm* comm);
/* recv_count / send_count are elements per rank (NCCL convention). In-place is allowed:
 * recv == send + rank*recv_count (reduce-scatter), send == recv + rank*send_count (all-gather). */
int zs_reduce_scatter(zs_comm* comm, const void* send, void* recv, int64_t recv_count, int dtype,
                      uintptr_t stream);
int zs_all_gather(zs_comm* comm, const void* send, void* recv, int64_t send_count, int dtype,
                  uintptr_t stream);
int zs_all_reduce(zs_comm* comm, const void* send, void* recv, int64_t count, int dtype,
                  uintptr_t stream);
/* SUM-reduce count elements onto `root` (recv only read on root; in place when send == recv) and
 * broadcast count elements from `root`.  Issued once per owner inside zs_group_start/end they
 * form the reduce-scatter-v / all-gather-v of a ragged bucket (zero2.py:107 / zero2.py:133). */
int zs_reduce(zs_comm* comm, const void* send, void* recv, int64_t count, int dtype, int root,
              uintptr_t stream);
int zs_broadcast(zs_comm* comm, const void* send, void* recv, int64_t count, int dtype, int root,
                 uintptr_t stream);
/* One RCCL group of n SUM-reduces (entry i: send[i] -> recv[i] on root[i], count[i] elements;
 * recv[i] is only written on its root and may equal send[i]) or of n in-place broadcasts
 * (buf[i] from root[i]).  The reduce-scatter-v / all-gather-v of one round of the flat
 * parameter arena: each owner's contiguous window reduced to it (zero2.py:94-113) and its
 * updated parameters broadcast from it (zero2.py:122-133), one call per round. */
int zs_reduce_group(zs_comm* comm, int64_t n, const uint64_t* send, const uint64_t* recv,
                    const int64_t* count, const int32_t* root, int dtype, uintptr_t stream);
int zs_broadcast_group(zs_comm* comm, int64_t n, const uint64_t* buf, const int64_t* count,
                       const int32_t* root, int dtype, uintptr_t stream);
/* One RCCL group of n all-gathers (entry i: send_count[i] elements from send[i] on every rank
 * into recv[i], rank-major) or of n SUM reduce-scatters (entry i: ws * recv_count[i] elements at
 * send[i] reduced, this rank's recv_count[i] into recv[i]).  ZeRO-3's per-module gather of every
 * parameter's dim-0 chunk (Zero3ParamManager.materialize, zero3.py:36-41, one group per module)
 * and one backward bucket of gradient reduce-scatters into the chunk arena (the reduction of
 * zero3.py:131-147), each as ONE call instead of one per parameter. */
int zs_all_gather_group(zs_comm* comm, int64_t n, const uint64_t* send, const uint64_t* recv,
                        const int64_t* send_count, int dtype, uintptr_t stream);
int zs_reduce_scatter_group(zs_comm* comm, int64_t n, const uint64_t* send, const uint64_t* recv,
                            const int64_t* recv_count, int dtype, uintptr_t stream);
/* The same two groups with their stream ordering in the same call (a ZeRO-3 module gather or a
 * gradient bucket is otherwise four runtime calls from Python around one library call):
 * ready_event != 0: record it on after_stream (where the inputs were produced) and make `stream`
 * wait for it; then the group (comm may be NULL when n == 0: ordering only); done_event != 0:
 * record it on `stream` after the group.  Events are HIP events (hipEvent_t as uint64_t). */
int zs_all_gather_group_ordered(zs_comm* comm, int64_t n, const uint64_t* send,
                                const uint64_t* recv, const int64_t* send_count, int dtype,
                                uintptr_t after_stream, uint64_t ready_event, uintptr_t stream,
                                uint64_t done_event);
int zs_reduce_scatter_group_ordered(zs_comm* comm, int64_t n, const uint64_t* send,
                                    const uint64_t* recv, const int64_t* recv_count, int dtype,
                                    uintptr_t after_stream, uint64_t ready_event, uintptr_t stream,
                                    uint64_t done_event);
/* hipStreamWaitEvent(stream, event): the consumer side of the ordered groups. */
int zs_stream_wait_event(uintptr_t stream, uint64_t event);
/* Sync objects (ABI v12; v13: 64-bit epochs): a cross-stream ordering point that is either a HIP
 * event (ZS_SYNC_EVENT) or a stream memory operation on a flag word in pinned host-coherent memory
 * (ZS_SYNC_FLAG: the epoch stored on the producer — a one-wave store kernel with a system-scope
 * release, or hipStreamWriteValue64 (zs_tune "sync_write_kernel") — and a wait for >= it on the
 * consumer — a one-wave polling kernel, or hipStreamWaitValue64 (zs_tune "sync_wait_kernel"); epochs only grow and never wrap).  zs_sync_record enqueues the producer side on
 * `stream`; zs_sync_wait makes `stream` wait for the latest record (hipStreamWaitEvent's
 * semantics; a never-recorded sync, or one whose latest record has already executed — the host
 * reads the flag word — enqueues nothing).  A flag record from another stream than the previous
 * record's first waits for that record (v13), so any stream may record.  The ZeRO-3 gathers and
 * gradient buckets (zero3.py:36-41, 131-147; their torch.cuda.synchronize() after each collective
 * becomes this ordering) use the synced group forms: record `ready` on after_stream and wait for
 * it on `stream`, the RCCL group, record `done` on `stream` (either sync may be NULL). */
typedef struct zs_sync zs_sync;
enum zs_sync_kind { ZS_SYNC_EVENT = 0, ZS_SYNC_FLAG = 1 };
int zs_sync_create(int kind, zs_sync** out);
int zs_sync_destroy(zs_sync* sync);
int zs_sync_record(zs_sync* sync, uintptr_t stream);
int zs_sync_wait(zs_sync* sync, uintptr_t stream);
/* Test hook (v13): move a flag sync's epoch (and its word) forward to `epoch` — every record made
 * so far must have executed.  Lets a test cross an epoch boundary (2^32) without 2^32 records.
 * ZS_ERR_INVALID for an event sync, a smaller epoch or a pending record. */
int zs_sync_set_epoch(zs_sync* sync, uint64_t epoch);
/* Diagnostic (v13): a flag sync's latest recorded epoch and the current value of its word (the
 * word read through hipMemcpy when it lives in device memory); 0 / 0 for an event sync. */
int zs_sync_query(zs_sync* sync, uint64_t* epoch, uint64_t* word);
int zs_all_gather_group_synced(zs_comm* comm, int64_t n, const uint64_t* send,
                               const uint64_t* recv, const int64_t* send_count, int dtype,
                               uintptr_t after_stream, zs_sync* ready, uintptr_t stream,
                               zs_sync* done);
int zs_reduce_scatter_group_synced(zs_comm* comm, int64_t n, const uint64_t* send,
                                   const uint64_t* recv, const int64_t* recv_count, int dtype,
                                   uintptr_t after_stream, zs_sync* ready, uintptr_t stream,
                                   zs_sync* done);
int zs_group_start(void);
int zs_group_end(void);
/* RCCL version the library is bound to at run time (e.g. 22606). */
int zs_rccl_version(int* version);

#ifdef __cplusplus
}
#endif
#endif /* ZERO_AMD_H */
