// CDNA4 (gfx950) kernels of the ZeRO step: segment copy (pack / unpack) and the fused Adam.
//
// Both kernels are HBM-bound streaming kernels (no MFMA, no LDS): 64-wide waves, 256-thread
// workgroups, 16-byte-per-lane coalesced accesses, a grid of 128 workgroups per CU (16x the 8
// resident) that strides over fixed-size chunks of a segment table.  A workgroup finds the segment of its chunk with a forward
// scan from the previous one (chunks are visited in increasing order), so the lookup is a couple of
// scalar loads, not a per-chunk binary search.
//
// Tables (segment pointers + chunk prefix sums) are uploaded once per set and reused every step:
// the step itself only launches kernels (no host sync), so it can be captured into a hipGraph.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <vector>

#include "zs_common.h"

namespace {

constexpr int kThreads = 256;
// segment copy: U 16-byte accesses in flight per lane, a workgroup step moves 256 * 16 * U bytes
constexpr int kCopyUnrollDefault = 4;
constexpr int64_t copy_chunk_bytes(int u) { return int64_t(kThreads) * 16 * u; }
// float4 groups per thread: 2 (2048-element chunks); 4 (4096) for the split master, whose 26 B/elem
// stream has one fp32 array fewer in flight per group (+1 % measured, profiles/r01_adam_split_master.log)
constexpr int adam_groups(bool split) { return split ? 4 : 2; }
constexpr int64_t adam_chunk(bool split) { return int64_t(kThreads) * 4 * adam_groups(split); }

int grid_cap() {
  static int cap = 0;
  if (cap == 0) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t prop;
      if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
        cus = prop.multiProcessorCount;
    }
    // 128 workgroups per CU (16x the resident 8): the best of 32/64/128/512/one-per-chunk for the
    // Adam and copy kernels at C4 scale (profiles/r01_adam_variants2.log)
    cap = cus * 128;
  }
  return cap;
}

// Kernel pointers live in the global address space; a plain pointer loaded from a table would
// lower to flat_load/flat_store (which also count in lgkmcnt and complete out of order).
#if defined(__HIP_DEVICE_COMPILE__)
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
#else
template <typename T>
using gptr = T*;
#endif
template <typename T>
__device__ __forceinline__ gptr<T> glob(T* p) {
  return (gptr<T>)p;
}

// Streaming accesses carry the non-temporal hint (global_load/store ... nt): nothing these kernels
// touch is re-read while it could still be cached, and at C4 scale (86 GB per Adam launch) the hint
// measured +4-6 % over plain accesses, loads and stores alike (profiles/r01_adam_variants2.log).
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint4 nt_ld16(const void* p) {
  const u32x4 v = __builtin_nontemporal_load((gptr<const u32x4>)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_st16(void* p, uint4 x) {
  const u32x4 v = {x.x, x.y, x.z, x.w};
  __builtin_nontemporal_store(v, (gptr<u32x4>)p);
}
__device__ __forceinline__ uint2 nt_ld8(const void* p) {
  const u32x2 v = __builtin_nontemporal_load((gptr<const u32x2>)p);
  return make_uint2(v.x, v.y);
}
__device__ __forceinline__ void nt_st8(void* p, uint2 x) {
  const u32x2 v = {x.x, x.y};
  __builtin_nontemporal_store(v, (gptr<u32x2>)p);
}
// the same accesses with the cache policy chosen at compile time (NT: non-temporal hint)
template <bool NT>
__device__ __forceinline__ uint4 ld16(const void* p) {
  if constexpr (NT) return nt_ld16(p);
  else return *(gptr<const uint4>)p;
}
template <bool NT>
__device__ __forceinline__ void st16(void* p, uint4 x) {
  if constexpr (NT) nt_st16(p, x);
  else *(gptr<uint4>)p = x;
}
template <bool NT>
__device__ __forceinline__ uint2 ld8(const void* p) {
  if constexpr (NT) return nt_ld8(p);
  else return *(gptr<const uint2>)p;
}
template <bool NT>
__device__ __forceinline__ void st8(void* p, uint2 x) {
  if constexpr (NT) nt_st8(p, x);
  else *(gptr<uint2>)p = x;
}
// Above this many bytes a buffer cannot sit in the 256 MB MALL (Infinity Cache): the in-place scale
// and the conversions take the non-temporal policy there and the default policy below, where the
// buffer was usually just written (an all-reduce, a backward) and is read next (the collective).
constexpr int64_t kMallBytes = int64_t(256) << 20;

// ----------------------------------------------------------------------------------------------
// segment copy
// ----------------------------------------------------------------------------------------------
struct CopySeg {
  const unsigned char* src;  // nullptr = zero fill
  unsigned char* dst;
  int64_t nbytes;
  int64_t vec;  // 1 if src and dst are 16-byte aligned (or src is null and dst aligned)
};

// Cache policy by size (NT) as zs_scale / zs_convert: non-temporal when the set moves more than the
// MALL holds (a C4 pack group, a checkpoint), the default policy below (a 64 MB overlap bucket, read
// next by its collective); `zs_tune("copy_nt")` forces either.
// One chunk [b0, b1) of one segment, by the whole workgroup.
template <int U, bool NT>
__device__ __forceinline__ void copy_chunk(const unsigned char* s_src, unsigned char* s_dst, bool vec,
                                           int64_t b0, int64_t b1) {
  const gptr<const unsigned char> src = glob(s_src);
  const gptr<unsigned char> dst = glob(s_dst);
  if (vec) {
    uint4 val[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // all loads first: U x 16 B in flight per lane
      const int64_t off = b0 + (int64_t(u) * kThreads + threadIdx.x) * 16;
      val[u] = make_uint4(0, 0, 0, 0);
      if (s_src && off + 16 <= b1) val[u] = ld16<NT>(s_src + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t off = b0 + (int64_t(u) * kThreads + threadIdx.x) * 16;
      if (off + 16 <= b1) {
        st16<NT>(s_dst + off, val[u]);
      } else if (off < b1) {
        for (int64_t b = off; b < b1; ++b) dst[b] = s_src ? src[b] : 0;
      }
    }
  } else {
    for (int64_t b = b0 + threadIdx.x; b < b1; b += kThreads) dst[b] = s_src ? src[b] : 0;
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(kThreads) void copy_segments_kernel(
    const CopySeg* __restrict__ segs, const int64_t* __restrict__ chunk_prefix, int64_t nseg,
    int64_t total_chunks) {
  constexpr int64_t kChunk = copy_chunk_bytes(U);
  int64_t seg = 0;
  for (int64_t c = blockIdx.x; c < total_chunks; c += gridDim.x) {
    while (chunk_prefix[seg + 1] <= c) ++seg;  // uniform forward scan
    const CopySeg s = segs[seg];
    const int64_t b0 = (c - chunk_prefix[seg]) * kChunk;
    copy_chunk<U, NT>(s.src, s.dst, s.vec != 0, b0, min(b0 + kChunk, s.nbytes));
  }
}

// The same copy with up to kDirectMax segments passed BY VALUE in the kernel arguments: no
// descriptor table to allocate and upload, so a set whose pointers change every call (backward's
// fresh gradients into their arena slots) costs one launch and nothing else.
constexpr int kDirectMax = 64;
struct DirectSet {
  const unsigned char* src[kDirectMax];  // nullptr = zero fill
  unsigned char* dst[kDirectMax];
  int64_t nbytes[kDirectMax];
  int64_t prefix[kDirectMax + 1];  // chunk prefix over the segments
  uint64_t vec_mask;               // bit i: segment i is 16-byte aligned on both sides
  int n;
};

template <int U, bool NT>
__global__ __launch_bounds__(kThreads) void copy_direct_kernel(const DirectSet set) {
  constexpr int64_t kChunk = copy_chunk_bytes(U);
  const int64_t total = set.prefix[set.n];
  int seg = 0;
  for (int64_t c = blockIdx.x; c < total; c += gridDim.x) {
    while (set.prefix[seg + 1] <= c) ++seg;  // uniform forward scan
    const int64_t b0 = (c - set.prefix[seg]) * kChunk;
    copy_chunk<U, NT>(set.src[seg], set.dst[seg], (set.vec_mask >> seg) & 1, b0,
                      min(b0 + kChunk, set.nbytes[seg]));
  }
}

// ----------------------------------------------------------------------------------------------
// fused Adam
// ----------------------------------------------------------------------------------------------
struct AdamSeg {
  const void* g;
  const float* master;
  float* master_out;
  unsigned short* p_out;
  float* m;
  float* v;
  float* vmax;
  float* carry;
  int64_t n;
};

struct HP {
  float omb1, beta2, omb2, neg_step, bc2_sqrt, eps, wd, decay_mul, grad_div, inv_div, carry_mul;
  int div_pow2, maximize;
};

__device__ __forceinline__ float bf16_to_f32(unsigned short h) {
  return __uint_as_float(uint32_t(h) << 16);
}

__device__ __forceinline__ unsigned short f32_to_bf16(float f) {
  // round-to-nearest-even; NaN stays NaN (plain cast lowers to v_cvt_pk_bf16_f32 on gfx950)
  __bf16 h = static_cast<__bf16>(f);
  unsigned short r;
  __builtin_memcpy(&r, &h, 2);
  return r;
}

// Split master (ZS_BF16_SPLIT): the fp32 master's bits u live as hi = RNE-bf16(u) — the bf16 param
// itself — and the int16 residual lo = u - (hi << 16), so u = (hi << 16) + sext(lo).  The one
// residual int16 cannot hold, +0x8000 (an exact tie rounded down to an even hi), is stored as
// 0x7FFF: that master moves 1 ulp toward zero and its bf16 param stays the same.
__device__ __forceinline__ float join_master(uint32_t hi, uint32_t lo) {
  return __uint_as_float((hi << 16) + uint32_t(int32_t(int16_t(uint16_t(lo)))));
}
__device__ __forceinline__ uint32_t master_residual(float p, uint32_t hi) {
  const uint32_t d = __float_as_uint(p) - (hi << 16);
  return d == 0x8000u ? 0x7FFFu : (d & 0xFFFFu);
}

// One element of torch.optim.Adam's single-tensor update (adam.py:394-547), in the rounding order
// of torch's CPU kernels: lerp = fma(w, end-self, self) (ATen Lerp.h weight<0.5 branch),
// exp_avg_sq.mul_(b2).addcmul_(g,g,1-b2) = fma((1-b2)*g, g, v*b2), denom = sqrt(v)/bc2_sqrt + eps,
// param.addcdiv_(m, denom, -step_size) = p + (-step_size*m)/denom.  Only explicit fmaf() fuse;
// sqrt and '/' are IEEE correctly rounded (-fhip-fp32-correctly-rounded-divide-sqrt).
template <bool AMS, bool CARRY>
__device__ __forceinline__ void adam_elem(float gsum, float& p, float& m, float& v, float& vmax,
                                          float& carry, const HP& hp) {
#pragma clang fp contract(off)
  float s = gsum;
  if constexpr (CARRY) s = s + hp.carry_mul * carry;  // ZeRO-1: Σ G + (ws-1)·A_{t-1}
  // zero1.py:84 / zero2.py:111 `grad / ws`; a power-of-two divisor is an exact reciprocal multiply
  float g = hp.div_pow2 ? s * hp.inv_div : s / hp.grad_div;
  if constexpr (CARRY) carry = g;
  if (hp.maximize) g = -g;
  if (hp.wd != 0.0f) g = fmaf(hp.wd, p, g);  // grad.add(param, alpha=wd)
  p = p * hp.decay_mul;                       // AdamW: param.mul_(1 - lr*wd); 1.0 otherwise
  m = fmaf(hp.omb1, g - m, m);
  v = fmaf(hp.omb2 * g, g, v * hp.beta2);
  float vv = v;
  if constexpr (AMS) {
    vmax = fmaxf(vmax, v);
    vv = vmax;
  }
  const float denom = sqrtf(vv) / hp.bc2_sqrt + hp.eps;
  p = p + (hp.neg_step * m) / denom;
}

template <typename GT>
__device__ __forceinline__ float load_g1(const void* g, int64_t i) {
  if constexpr (sizeof(GT) == 4) return glob(static_cast<const float*>(g))[i];
  else return bf16_to_f32(glob(static_cast<const unsigned short*>(g))[i]);
}

// Scalar kernel: any alignment, any length (segment tails and unaligned segments; tiny).
template <typename GT, bool AMS, bool CARRY, bool SPLIT>
__global__ __launch_bounds__(kThreads) void adam_scalar_kernel(
    const AdamSeg* __restrict__ segs, const int64_t* __restrict__ chunk_prefix, int64_t nseg,
    int64_t total_chunks, HP hp) {
  int64_t seg = 0;
  for (int64_t c = blockIdx.x; c < total_chunks; c += gridDim.x) {
    while (chunk_prefix[seg + 1] <= c) ++seg;
    const AdamSeg s = segs[seg];
    const int64_t i = (c - chunk_prefix[seg]) * kThreads + threadIdx.x;
    if (i >= s.n) continue;
    float gs = s.g ? load_g1<GT>(s.g, i) : 0.0f;
    const gptr<unsigned short> lo = glob(reinterpret_cast<unsigned short*>(s.master_out));
    float p = SPLIT ? join_master(glob(reinterpret_cast<const unsigned short*>(s.master))[i], lo[i])
                    : glob(s.master)[i];
    float m = glob(s.m)[i], v = glob(s.v)[i];
    float vm = AMS ? glob(s.vmax)[i] : 0.0f;
    float cr = CARRY ? glob(s.carry)[i] : 0.0f;
    adam_elem<AMS, CARRY>(gs, p, m, v, vm, cr, hp);
    if constexpr (SPLIT) {
      const unsigned short h = f32_to_bf16(p);
      glob(s.p_out)[i] = h;
      lo[i] = (unsigned short)master_residual(p, h);
    } else {
      if (s.master_out) glob(s.master_out)[i] = p;
      if (s.p_out) glob(s.p_out)[i] = f32_to_bf16(p);
    }
    glob(s.m)[i] = m;
    glob(s.v)[i] = v;
    if constexpr (AMS) glob(s.vmax)[i] = vm;
    if constexpr (CARRY) glob(s.carry)[i] = cr;
  }
}

__device__ __forceinline__ float4 ld4(const float* p, int64_t i) {
  const uint4 r = nt_ld16(p + i);
  return make_float4(__uint_as_float(r.x), __uint_as_float(r.y), __uint_as_float(r.z),
                     __uint_as_float(r.w));
}
__device__ __forceinline__ void st4(float* p, int64_t i, float4 x) {
  nt_st16(p + i, make_uint4(__float_as_uint(x.x), __float_as_uint(x.y), __float_as_uint(x.z),
                            __float_as_uint(x.w)));
}

template <typename GT>
__device__ __forceinline__ float4 load_g4(const void* g, int64_t i) {
  if constexpr (sizeof(GT) == 4) {
    return ld4(static_cast<const float*>(g), i);
  } else {
    const uint2 r = nt_ld8(static_cast<const unsigned short*>(g) + i);
    return make_float4(__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
                       __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u));
  }
}

// Vector kernel: every segment 16-B aligned (8-B for bf16 arrays) with n % 4 == 0 (the host
// splits tails off into the scalar table).  adam_groups() float4 groups per thread, lane-contiguous
// (16 B per lane per access), so each wave instruction touches one contiguous 1 KiB (f32) /
// 512 B (bf16) run; every group's loads are issued before any math.
template <typename GT, bool AMS, bool CARRY, bool SPLIT>
__global__ __launch_bounds__(kThreads) void adam_segments_kernel(
    const AdamSeg* __restrict__ segs, const int64_t* __restrict__ chunk_prefix, int64_t nseg,
    int64_t total_chunks, HP hp) {
  int64_t seg = 0;
  for (int64_t c = blockIdx.x; c < total_chunks; c += gridDim.x) {
    while (chunk_prefix[seg + 1] <= c) ++seg;
    const AdamSeg s = segs[seg];
    constexpr int G = adam_groups(SPLIT);
    const int64_t e0 = (c - chunk_prefix[seg]) * adam_chunk(SPLIT);
    float4 g4[G], p4[G], m4[G], v4[G];
    float4 x4[G], c4[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int64_t i = e0 + (int64_t(u) * kThreads + threadIdx.x) * 4;
      if (i < s.n) {
        g4[u] = s.g ? load_g4<GT>(s.g, i) : make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (SPLIT) {
          const uint2 h = nt_ld8(reinterpret_cast<const unsigned short*>(s.master) + i);
          const uint2 l = nt_ld8(reinterpret_cast<const unsigned short*>(s.master_out) + i);
          p4[u] = make_float4(join_master(h.x & 0xFFFFu, l.x), join_master(h.x >> 16, l.x >> 16),
                              join_master(h.y & 0xFFFFu, l.y), join_master(h.y >> 16, l.y >> 16));
        } else {
          p4[u] = ld4(s.master, i);
        }
        m4[u] = ld4(s.m, i);
        v4[u] = ld4(s.v, i);
        if constexpr (AMS) x4[u] = ld4(s.vmax, i);
        if constexpr (CARRY) c4[u] = ld4(s.carry, i);
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int64_t i = e0 + (int64_t(u) * kThreads + threadIdx.x) * 4;
      if (i < s.n) {
        float* gp = reinterpret_cast<float*>(&g4[u]);
        float* pp = reinterpret_cast<float*>(&p4[u]);
        float* mp = reinterpret_cast<float*>(&m4[u]);
        float* vp = reinterpret_cast<float*>(&v4[u]);
        float* xp = reinterpret_cast<float*>(&x4[u]);
        float* cp = reinterpret_cast<float*>(&c4[u]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float xv = AMS ? xp[j] : 0.0f;
          float cv = CARRY ? cp[j] : 0.0f;
          adam_elem<AMS, CARRY>(gp[j], pp[j], mp[j], vp[j], xv, cv, hp);
          if constexpr (AMS) xp[j] = xv;
          if constexpr (CARRY) cp[j] = cv;
        }
        if constexpr (SPLIT) {
          uint32_t h[4], l[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            h[j] = f32_to_bf16(pp[j]);
            l[j] = master_residual(pp[j], h[j]);
          }
          nt_st8(s.p_out + i, make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16)));
          nt_st8(reinterpret_cast<unsigned short*>(s.master_out) + i,
                 make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16)));
        } else {
          if (s.master_out) st4(s.master_out, i, p4[u]);
          if (s.p_out) {
            uint2 r;
            r.x = uint32_t(f32_to_bf16(pp[0])) | (uint32_t(f32_to_bf16(pp[1])) << 16);
            r.y = uint32_t(f32_to_bf16(pp[2])) | (uint32_t(f32_to_bf16(pp[3])) << 16);
            nt_st8(s.p_out + i, r);
          }
        }
        st4(s.m, i, m4[u]);
        st4(s.v, i, v4[u]);
        if constexpr (AMS) st4(s.vmax, i, x4[u]);
        if constexpr (CARRY) st4(s.carry, i, c4[u]);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------------
// in-place scale: x /= div (DDP's `param.grad /= world_size`, ddp.py:45-47)
// ----------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ float to_f32(T x) {
  if constexpr (sizeof(T) == 4) return x;
  else return bf16_to_f32(x);
}
template <typename T>
__device__ __forceinline__ T from_f32(float x) {
  if constexpr (sizeof(T) == 4) return x;
  else return f32_to_bf16(x);
}

// In place, kScaleU 16-B accesses per lane in flight: a wave step covers kScaleU contiguous 1 KiB
// blocks (lane l of block u at 16-B chunk 64u + l), every load issued before the first store;
// grid-stride over wave steps; the tail (n % elements per step) by block 0.  Cache policy by size
// (NT): a DDP bucket (64 MiB) is scaled right after the all-reduce wrote it, while it is still in
// the 256 MB MALL — default policy; a buffer larger than the MALL cannot be there, so its loads
// and stores carry the non-temporal hint (kMallBytes; `zs_tune("scale_nt")` forces either).
// (Round 2's one access in flight per lane measured 0.61 of 8 TB/s on a 4 GiB buffer.)
// fp32: IEEE division (x / div), or an exact reciprocal multiply when div is a power of two;
// bf16: the same in fp32, rounded to bf16 (RNE) — torch's div_ on a bf16 tensor.
constexpr int kScaleU = 4;

template <typename T, bool NT>
__global__ __launch_bounds__(kThreads) void scale_kernel(T* __restrict__ x, int64_t n, float div,
                                                         float inv, int pow2) {
#pragma clang fp contract(off)
  constexpr int V = 16 / sizeof(T);
  constexpr int64_t kSpan = int64_t(64) * V * kScaleU;  // elements per wave step
  const gptr<T> gx = glob(x);
  const int64_t steps = n / kSpan;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = int64_t(gridDim.x) * (kThreads / 64);
  auto op = [&](float f) { return pow2 ? f * inv : f / div; };
  for (int64_t w = int64_t(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6); w < steps;
       w += nwaves) {
    T* base = x + w * kSpan + int64_t(lane) * V;
    uint4 raw[kScaleU];
#pragma unroll
    for (int u = 0; u < kScaleU; ++u) raw[u] = ld16<NT>(base + u * 64 * V);
#pragma unroll
    for (int u = 0; u < kScaleU; ++u) {
      T* e = reinterpret_cast<T*>(&raw[u]);
#pragma unroll
      for (int j = 0; j < V; ++j) e[j] = from_f32<T>(op(to_f32<T>(e[j])));
      st16<NT>(base + u * 64 * V, raw[u]);
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t i = steps * kSpan + threadIdx.x; i < n; i += kThreads)
      gx[i] = from_f32<T>(op(to_f32<T>(gx[i])));
  }
}

// ----------------------------------------------------------------------------------------------
// fp32 <-> bf16 conversion (the bf16 gradient exchange of fp32-parameter models)
// ----------------------------------------------------------------------------------------------
// Wave-dense accesses: a wave step covers kConvSpan elements in kConvU blocks of 256; in block u
// lane l converts elements [256u + 4l, +4) — one 16-B fp32 access and one 8-B bf16 access per
// block, so every wave instruction touches one contiguous 1 KiB (fp32) or 512 B (bf16) span.
// (Round 2's lane-contiguous 8 elements per lane gave each fp32 instruction a 32-B lane stride —
// half-dense — and measured 0.58 of 8 TB/s bf16 -> fp32, profiles/r03_kernels_table.json.)
// All kConvU loads are issued before the first store; grid-stride over wave steps; the n % kConvSpan
// tail by block 0.  Cache policy by size (NT), as zs_scale: non-temporal when source and destination
// together are larger than the MALL, the default policy below (a bucket's grads just written by
// backward, the bf16 bucket read next by the collective); `zs_tune("convert_nt")` forces either.
// Round 4 A/B on placed buffers (profiles/r04_policy_ab.json): 64 MiB fp32 side, bf16 -> fp32 0.80
// default vs 0.72 non-temporal (fp32 -> bf16 0.83 / 0.85); 256 MiB and above non-temporal wins
// (0.84 / 0.74 fp32 -> bf16, 0.75 / 0.72 bf16 -> fp32).
// fp32 -> bf16 rounds to nearest even (v_cvt_pk_bf16_f32), NaN stays NaN; bf16 -> fp32 is exact.
constexpr int kConvU = 4;
constexpr int64_t kConvSpan = 256 * kConvU;

template <bool TO_BF16, bool NT>
__global__ __launch_bounds__(kThreads) void convert_kernel(const void* __restrict__ src,
                                                           void* __restrict__ dst, int64_t n) {
  const int64_t steps = n / kConvSpan;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = int64_t(gridDim.x) * (kThreads / 64);
  for (int64_t w = int64_t(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6); w < steps;
       w += nwaves) {
    const int64_t base = w * kConvSpan + 4 * lane;
    if constexpr (TO_BF16) {
      const float* s = static_cast<const float*>(src) + base;
      float4 a[kConvU];
#pragma unroll
      for (int u = 0; u < kConvU; ++u) {
        const uint4 r = ld16<NT>(s + 256 * u);
        a[u] = make_float4(__uint_as_float(r.x), __uint_as_float(r.y), __uint_as_float(r.z),
                           __uint_as_float(r.w));
      }
      unsigned short* d = static_cast<unsigned short*>(dst) + base;
#pragma unroll
      for (int u = 0; u < kConvU; ++u) {
        const uint32_t lo = uint32_t(f32_to_bf16(a[u].x)) | (uint32_t(f32_to_bf16(a[u].y)) << 16);
        const uint32_t hi = uint32_t(f32_to_bf16(a[u].z)) | (uint32_t(f32_to_bf16(a[u].w)) << 16);
        st8<NT>(d + 256 * u, make_uint2(lo, hi));
      }
    } else {
      const unsigned short* s = static_cast<const unsigned short*>(src) + base;
      uint2 h[kConvU];
#pragma unroll
      for (int u = 0; u < kConvU; ++u) h[u] = ld8<NT>(s + 256 * u);
      float* d = static_cast<float*>(dst) + base;
#pragma unroll
      for (int u = 0; u < kConvU; ++u)
        st16<NT>(d + 256 * u, make_uint4(h[u].x << 16, h[u].x & 0xffff0000u, h[u].y << 16,
                                         h[u].y & 0xffff0000u));
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t i = steps * kConvSpan + threadIdx.x; i < n; i += kThreads) {
      if constexpr (TO_BF16)
        glob(static_cast<unsigned short*>(dst))[i] = f32_to_bf16(glob(static_cast<const float*>(src))[i]);
      else
        glob(static_cast<float*>(dst))[i] = bf16_to_f32(glob(static_cast<const unsigned short*>(src))[i]);
    }
  }
}

// scalar variant for unaligned buffers
template <bool TO_BF16>
__global__ __launch_bounds__(kThreads) void convert_scalar_kernel(const void* __restrict__ src,
                                                                  void* __restrict__ dst, int64_t n) {
  for (int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * kThreads) {
    if constexpr (TO_BF16)
      glob(static_cast<unsigned short*>(dst))[i] = f32_to_bf16(glob(static_cast<const float*>(src))[i]);
    else
      glob(static_cast<float*>(dst))[i] = bf16_to_f32(glob(static_cast<const unsigned short*>(src))[i]);
  }
}

// ----------------------------------------------------------------------------------------------
// row-wise fp8 (OCP E4M3) quantise / dequantise for the low-precision parameter all-gather
// ----------------------------------------------------------------------------------------------
constexpr float kE4M3Max = 448.0f;

__device__ __forceinline__ uint32_t e4m3x4(float a, float b, float c, float d) {
  // v_cvt_pk_fp8_f32: round to nearest even, OCP E4M3 on gfx950; inputs pre-clamped to ±448
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return uint32_t(w);
}
__device__ __forceinline__ float qclamp(float x, float inv) {
#pragma clang fp contract(off)
  return __builtin_amdgcn_fmed3f(x * inv, kE4M3Max, -kE4M3Max);
}

// Block-per-row fallback for any row length and alignment (scalar accesses): amax by wave
// shuffles + a 4-entry LDS exchange, then the row is re-read (L2-resident) and converted.
template <typename T>
__global__ __launch_bounds__(kThreads) void fp8_quantize_rows_kernel(
    const T* __restrict__ src, unsigned char* __restrict__ dst, float* __restrict__ scales,
    int64_t rows, int64_t row_len) {
#pragma clang fp contract(off)
  __shared__ float red[kThreads / 64];
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const gptr<const T> x = glob(src + r * row_len);
    const gptr<unsigned char> q = glob(dst + r * row_len);
    float amax = 0.0f;
    for (int64_t i = threadIdx.x; i < row_len; i += kThreads) amax = fmaxf(amax, fabsf(to_f32<T>(x[i])));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    const float inv = amax > 0.0f ? kE4M3Max / amax : 1.0f;
    if (threadIdx.x == 0) glob(scales)[r] = amax > 0.0f ? amax / kE4M3Max : 1.0f;
    for (int64_t i = threadIdx.x; i < row_len; i += kThreads) {
      const float c = qclamp(to_f32<T>(x[i]), inv);
      q[i] = (unsigned char)(__builtin_amdgcn_cvt_pk_fp8_f32(c, c, 0, false) & 0xff);
    }
  }
}

// Wave-per-row variant (the vector path): each 64-lane wave owns rows r = 4*block + wave (grid
// stride), reads the row as lane-contiguous 16-byte chunks (one wave instruction = 1 KiB), reduces
// amax with wave shuffles only (no LDS, no block barrier), and converts.  NREG > 0: the row's
// chunks stay in registers between the two passes (rows of at most 64 * NREG chunks: NREG = 8, 16
// or 32, i.e. up to 16384 bf16 / 8192 fp32 elements — every row of the C5 set) — one read of the
// row, all of its loads in flight at once; NREG == 0 (longer rows): both passes stream the row in
// batches of 8 loads in flight per lane, the second from L2 / MALL where it is still cached.  Same
// arithmetic, same bits as the block-per-row kernel: amax = max|x|, inv = 448/amax,
// e4m3(RNE(clamp(x*inv))), scale = amax/448.
// One row, one wave (lane = threadIdx.x & 63): x -> q (row_len elements), *scale.
template <typename T, int NREG>
__device__ __forceinline__ void fp8_quantize_row(const T* __restrict__ src_row,
                                                 unsigned char* __restrict__ dst_row,
                                                 float* __restrict__ scale, int64_t row_len,
                                                 int lane) {
#pragma clang fp contract(off)
  constexpr int E = 16 / int(sizeof(T));  // elements per 16-byte chunk
  constexpr int R = NREG > 0 ? NREG : 8;  // chunks in flight per lane
  auto unpack = [](const uint4& raw, float* v) {
    if constexpr (sizeof(T) == 2) {
      const unsigned short* h = reinterpret_cast<const unsigned short*>(&raw);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf16_to_f32(h[j]);
    } else {
      v[0] = __uint_as_float(raw.x); v[1] = __uint_as_float(raw.y);
      v[2] = __uint_as_float(raw.z); v[3] = __uint_as_float(raw.w);
    }
  };
  const gptr<const T> x = glob(src_row);
  const gptr<unsigned char> q = glob(dst_row);
  auto load = [&](int64_t i) {
    if (i >= row_len) return make_uint4(0, 0, 0, 0);
    if constexpr (NREG > 0) return nt_ld16(x + i);  // read once
    else return *reinterpret_cast<gptr<const uint4>>(x + i);  // read again in pass 2
  };
  float amax = 0.0f;
  uint4 keep[R];
  for (int64_t b0 = 0; b0 < row_len; b0 += int64_t(64) * R * E) {  // NREG > 0: one batch
#pragma unroll
    for (int u = 0; u < R; ++u) keep[u] = load(b0 + (int64_t(u) * 64 + lane) * E);
#pragma unroll
    for (int u = 0; u < R; ++u) {
      float v[E];
      unpack(keep[u], v);
#pragma unroll
      for (int j = 0; j < E; ++j) amax = fmaxf(amax, fabsf(v[j]));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  const float inv = amax > 0.0f ? kE4M3Max / amax : 1.0f;
  if (lane == 0) *glob(scale) = amax > 0.0f ? amax / kE4M3Max : 1.0f;
  auto emit = [&](int64_t i, const uint4& raw) {
    float v[E];
    unpack(raw, v);
    if constexpr (sizeof(T) == 2) {
      uint2 out;
      out.x = e4m3x4(qclamp(v[0], inv), qclamp(v[1], inv), qclamp(v[2], inv), qclamp(v[3], inv));
      out.y = e4m3x4(qclamp(v[4], inv), qclamp(v[5], inv), qclamp(v[6], inv), qclamp(v[7], inv));
      nt_st8(q + i, out);
    } else {
      *reinterpret_cast<gptr<uint32_t>>(q + i) =
          e4m3x4(qclamp(v[0], inv), qclamp(v[1], inv), qclamp(v[2], inv), qclamp(v[3], inv));
    }
  };
  if constexpr (NREG > 0) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int64_t i = (int64_t(u) * 64 + lane) * E;
      if (i < row_len) emit(i, keep[u]);
    }
  } else {
    for (int64_t b0 = 0; b0 < row_len; b0 += int64_t(64) * R * E) {
#pragma unroll
      for (int u = 0; u < R; ++u) keep[u] = load(b0 + (int64_t(u) * 64 + lane) * E);
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int64_t i = b0 + (int64_t(u) * 64 + lane) * E;
        if (i < row_len) emit(i, keep[u]);
      }
    }
  }
}

template <typename T, int NREG>
__global__ __launch_bounds__(kThreads) void fp8_quantize_rows_wave_kernel(
    const T* __restrict__ src, unsigned char* __restrict__ dst, float* __restrict__ scales,
    int64_t rows, int64_t row_len) {
  const int lane = threadIdx.x & 63;
  const int64_t wpb = kThreads / 64;
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  for (int64_t r = int64_t(blockIdx.x) * wpb + wave; r < rows; r += int64_t(gridDim.x) * wpb)
    fp8_quantize_row<T, NREG>(src + r * row_len, dst + r * row_len, scales + r, row_len, lane);
}

// A gather group's matrices in one launch (zs_fp8_quantize_rowset): global row g (one wave each,
// grid-stride, so g only grows and the matrix lookup is a forward scan) of matrix m, local row
// lr = g - prefix[m]; rows [rows[m], cs[m]) are the chunk's padding: q = 0, scale = 1.  The table
// travels in the kernel arguments (constant, uniform: scalar loads).
constexpr int kSetMax = 16;
struct QSet {
  const void* src[kSetMax];
  unsigned char* q[kSetMax];
  float* sc[kSetMax];
  int64_t rows[kSetMax], row_len[kSetMax], prefix[kSetMax + 1];  // prefix over cs
  int n;
};

template <typename T, int NREG>
__global__ __launch_bounds__(kThreads) void fp8_quantize_rowset_kernel(const QSet set) {
  const int lane = threadIdx.x & 63;
  const int64_t wpb = kThreads / 64;
  const int64_t total = set.prefix[set.n];
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));  // uniform: scalar math
  int m = 0;
  for (int64_t g = int64_t(blockIdx.x) * wpb + wave; g < total; g += int64_t(gridDim.x) * wpb) {
    while (set.prefix[m + 1] <= g) ++m;
    const int64_t lr = g - set.prefix[m], len = set.row_len[m];
    unsigned char* qrow = set.q[m] + lr * len;
    if (lr < set.rows[m]) {
      fp8_quantize_row<T, NREG>(static_cast<const T*>(set.src[m]) + lr * len, qrow, set.sc[m] + lr,
                                len, lane);
    } else {  // padding row of the chunk
      for (int64_t i = int64_t(lane) * 8; i < len; i += 64 * 8) nt_st8(qrow + i, make_uint2(0, 0));
      if (lane == 0) *glob(set.sc[m] + lr) = 1.0f;
    }
  }
}

// Dequantise (round 4): one wave walks whole rows.  The rows of a set of matrices are numbered
// over the set (a single matrix for zs_fp8_dequantize_rows; every matrix of a gather group, rank by
// rank, for zs_fp8_dequantize_gathered), and each wave takes rows g, g + nwaves, ... — so the matrix
// index only grows (uniform forward scan) and the row's rank, local row, scale and source /
// destination pointers are worked out ONCE per row, in scalar registers (one 32-bit division per
// row, none per access).  The wave then walks the row in batches of kDqU accesses per lane: 8-B fp8
// loads (512 B per wave instruction, dense) and 16-B bf16 stores (1 KiB, dense) for bf16 output,
// 4 B -> 16 B for fp32.  The loads of the NEXT batch — in the same row or the wave's next row — are
// issued before the stores of the current one, so on gfx950, whose vmcnt counts loads and stores
// together, waiting for a batch's data never waits for the previous batch's stores: each wave keeps
// one batch of loads and one of stores in flight throughout.
constexpr int kDqU = 4;  // default accesses in flight per lane (zs_tune "dq_unroll": 4 / 8 / 16;
                         // 4 measured best at ws = 1 and ws = 8, profiles/r04_dq_ab.json)

struct DqSet {
  const unsigned char* q;
  const float* sc;
  int64_t q_rank, sc_rank;  // per-rank strides of the gathered q (bytes) and scales (elements)
  int64_t q_off[kSetMax], sc_off[kSetMax], cs[kSetMax], row_len[kSetMax];
  int64_t prefix[kSetMax + 1];  // prefix over ws * cs[m] full rows
  void* dst[kSetMax];
  int n;
};

template <typename T>
struct DqRow {
  const unsigned char* q;
  T* y;
  float sc;
  int64_t len;
};

template <typename T, int U>
__device__ __forceinline__ void fp8_dq_load(const DqRow<T>& r, int64_t b0, int lane, uint2* raw) {
  constexpr int E = sizeof(T) == 2 ? 8 : 4;
  const gptr<const unsigned char> q = glob(r.q);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = b0 + (int64_t(u) * 64 + lane) * E;
    raw[u] = make_uint2(0, 0);
    if (i < r.len) {
      if constexpr (E == 8) raw[u] = nt_ld8(q + i);
      else raw[u].x = __builtin_nontemporal_load(reinterpret_cast<gptr<const uint32_t>>(q + i));
    }
  }
}

template <typename T, int U, bool NT>
__device__ __forceinline__ void fp8_dq_store(const DqRow<T>& r, int64_t b0, int lane,
                                             const uint2* raw) {
#pragma clang fp contract(off)
  constexpr int E = sizeof(T) == 2 ? 8 : 4;
  const gptr<T> y = glob(r.y);
  const float sc = r.sc;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = b0 + (int64_t(u) * 64 + lane) * E;
    if (i >= r.len) continue;
    const int lo = int(raw[u].x), hi = int(raw[u].y);
    const float a0 = __builtin_amdgcn_cvt_f32_fp8(lo, 0) * sc, a1 = __builtin_amdgcn_cvt_f32_fp8(lo, 1) * sc;
    const float a2 = __builtin_amdgcn_cvt_f32_fp8(lo, 2) * sc, a3 = __builtin_amdgcn_cvt_f32_fp8(lo, 3) * sc;
    if constexpr (E == 8) {
      const float b0_ = __builtin_amdgcn_cvt_f32_fp8(hi, 0) * sc, b1 = __builtin_amdgcn_cvt_f32_fp8(hi, 1) * sc;
      const float b2 = __builtin_amdgcn_cvt_f32_fp8(hi, 2) * sc, b3 = __builtin_amdgcn_cvt_f32_fp8(hi, 3) * sc;
      auto pk = [](float a, float b) { return uint32_t(f32_to_bf16(a)) | (uint32_t(f32_to_bf16(b)) << 16); };
      const uint4 v = make_uint4(pk(a0, a1), pk(a2, a3), pk(b0_, b1), pk(b2, b3));
      if constexpr (NT) nt_st16(y + i, v);
      else *reinterpret_cast<gptr<uint4>>(y + i) = v;
    } else {
      if constexpr (NT) st4(reinterpret_cast<float*>(r.y + i), 0, make_float4(a0, a1, a2, a3));
      else *reinterpret_cast<gptr<float4>>(y + i) = make_float4(a0, a1, a2, a3);
    }
  }
}

template <typename T, int U, bool NT>
__global__ __launch_bounds__(kThreads) void fp8_dequantize_gathered_kernel(const DqSet set) {
  constexpr int64_t B = int64_t(64) * (sizeof(T) == 2 ? 8 : 4) * U;  // elements per batch
  const int lane = threadIdx.x & 63;
  const int64_t total = set.prefix[set.n];
  const int64_t nwaves = int64_t(gridDim.x) * (kThreads / 64);
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));  // uniform: scalar math
  int m = 0;
  // row g of the set -> its pointers and scale (uniform; the host checks ws * cs[m] < 2^31)
  auto row_at = [&](int64_t g, DqRow<T>& r) {
    while (set.prefix[m + 1] <= g) ++m;
    const uint32_t R = uint32_t(g - set.prefix[m]), cs = uint32_t(set.cs[m]);
    const uint32_t rk = R / cs, lr = R - rk * cs;
    r.len = set.row_len[m];
    r.sc = glob(set.sc)[int64_t(rk) * set.sc_rank + set.sc_off[m] + lr];
    r.q = set.q + int64_t(rk) * set.q_rank + set.q_off[m] + int64_t(lr) * r.len;
    r.y = static_cast<T*>(set.dst[m]) + int64_t(R) * r.len;
  };
  int64_t g = int64_t(blockIdx.x) * (kThreads / 64) + wave;
  if (g >= total) return;
  DqRow<T> cur;
  row_at(g, cur);
  int64_t b0 = 0;
  uint2 raw[U];
  fp8_dq_load<T, U>(cur, b0, lane, raw);
  while (true) {
    DqRow<T> nxt = cur;
    int64_t nb0 = b0 + B;
    bool more = true;
    if (nb0 >= cur.len) {  // the wave's next row
      g += nwaves;
      more = g < total;
      if (more) row_at(g, nxt);
      nb0 = 0;
    }
    uint2 nraw[U];
    if (more) fp8_dq_load<T, U>(nxt, nb0, lane, nraw);  // next batch's loads before this one's stores
    fp8_dq_store<T, U, NT>(cur, b0, lane, raw);
    if (!more) break;
    cur = nxt;
    b0 = nb0;
#pragma unroll
    for (int u = 0; u < U; ++u) raw[u] = nraw[u];
  }
}

// Scalar fallback for any row length and alignment: grid-stride over elements.
template <typename T>
__global__ __launch_bounds__(kThreads) void fp8_dequantize_rows_kernel(
    const unsigned char* __restrict__ src, const float* __restrict__ scales, T* __restrict__ dst,
    int64_t n, int64_t row_len) {
#pragma clang fp contract(off)
  const gptr<const unsigned char> q = glob(src);
  const gptr<T> y = glob(dst);
  const int64_t stride = int64_t(gridDim.x) * kThreads;
  for (int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x; i < n; i += stride) {
    const float v = __builtin_amdgcn_cvt_f32_fp8(int(q[i]), 0) * glob(scales)[i / row_len];
    y[i] = from_f32<T>(v);
  }
}

inline bool aligned(uint64_t p, uint64_t a) { return p % a == 0; }

// Diagnostic tuning knobs of the dequantise kernel (zs_tune; defaults are the measured best):
// accesses in flight per lane, non-temporal stores, and a cap of workgroups per CU (0 = one wave
// per row up to the usual grid cap; k > 0 = at most k workgroups per CU, each wave walking several
// rows with the next row's loads issued before the current row's stores).
struct DqTune {
  int unroll = kDqU;
  int nt_store = 1;
  int wg_per_cu = 0;
};
DqTune& dq_tune() {
  static DqTune t;
  return t;
}

// Adam grid (zs_tune "adam_wg_per_cu", diagnostic A/B): 0 = grid_cap() (128 workgroups per CU),
// k = at most k workgroups per CU striding over the chunks
int& adam_wg_per_cu() {
  static int v = 0;
  return v;
}
int64_t adam_grid_cap() {
  const int k = adam_wg_per_cu();
  return k > 0 ? int64_t(grid_cap() / 128) * k : int64_t(grid_cap());
}

// zs_scale's / zs_convert's / zs_copyset_run's cache policy: -1 by size (kMallBytes), 0 default
// policy, 1 non-temporal
int& scale_nt_mode() {
  static int mode = -1;
  return mode;
}
int& convert_nt_mode() {
  static int mode = -1;
  return mode;
}
int& copy_nt_mode() {
  static int mode = -1;
  return mode;
}

int dq_grid(int64_t rows) {
  int64_t cap = grid_cap();
  const int per_cu = dq_tune().wg_per_cu;
  if (per_cu > 0) cap = std::max<int64_t>(1, cap / 128 * per_cu);
  return int(std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, cap)));
}

template <typename T>
void launch_dequantize_t(const DqSet& set, int grid, hipStream_t st) {
  const DqTune& t = dq_tune();
#define ZS_DQ(U, NT) hipLaunchKernelGGL((fp8_dequantize_gathered_kernel<T, U, NT>), dim3(grid), dim3(kThreads), 0, st, set)
  if (t.nt_store) {
    switch (t.unroll) { case 4: ZS_DQ(4, true); break; case 16: ZS_DQ(16, true); break; default: ZS_DQ(8, true); }
  } else {
    switch (t.unroll) { case 4: ZS_DQ(4, false); break; case 16: ZS_DQ(16, false); break; default: ZS_DQ(8, false); }
  }
#undef ZS_DQ
}

void launch_dequantize(const DqSet& set, int dst_dtype, int grid, hipStream_t st) {
  if (dst_dtype == ZS_F32) launch_dequantize_t<float>(set, grid, st);
  else launch_dequantize_t<unsigned short>(set, grid, st);
}

}  // namespace

struct zs_copyset {
  CopySeg* d_segs = nullptr;
  int64_t* d_prefix = nullptr;
  int64_t nseg = 0, total_chunks = 0;
  int64_t bytes = 0;                // copied per run (read + write: 2x this)
  int unroll = kCopyUnrollDefault;  // 16-B accesses in flight per lane (chunk = 4 KiB * unroll)
};

// ZERO_AMD_COPY_UNROLL (diagnostic A/B): 2, 4 (default) or 8 accesses in flight per lane.
static int copy_unroll() {
  static int u = 0;
  if (u == 0) {
    const char* e = std::getenv("ZERO_AMD_COPY_UNROLL");
    const int v = e ? std::atoi(e) : kCopyUnrollDefault;
    u = (v == 2 || v == 4 || v == 8) ? v : kCopyUnrollDefault;
  }
  return u;
}

struct zs_adamset {
  // vector table (aligned, n % 4 == 0) and scalar table (tails, unaligned segments)
  AdamSeg* d_vec = nullptr;
  int64_t* d_vec_prefix = nullptr;
  AdamSeg* d_sca = nullptr;
  int64_t* d_sca_prefix = nullptr;
  int64_t nvec = 0, vec_chunks = 0, nsca = 0, sca_chunks = 0, elems = 0, bytes = 0;
  int g_dtype = ZS_F32, p_dtype = ZS_BF16, has_carry = 0, has_vmax = 0;
  // zs_adamset_set_grads: which input segment each table entry came from (the scalar entries with
  // their byte offset into that input's gradient), the gradient each input is bound to now, its
  // elements, whether it has a vector part (then its gradient must keep the vector alignment), and
  // the algorithmic bytes of one run without any gradient read
  int32_t* d_vec_in = nullptr;
  int32_t* d_sca_in = nullptr;
  int64_t* d_sca_goff = nullptr;
  std::vector<uint64_t> in_g;
  std::vector<int64_t> in_n;
  std::vector<unsigned char> in_vec;
  int64_t bytes_no_g = 0;
};

namespace {
// zs_adamset_set_grads: new gradient pointers for inputs [k0, k0 + n) of a set, in the kernel
// arguments (no upload, no host synchronisation), patched into the device tables in stream order.
constexpr int kGradPatchMax = 224;
struct GradPatch {
  uint64_t g[kGradPatchMax];
  int64_t k0;
  int n;
};

__global__ __launch_bounds__(kThreads) void adam_patch_grads_kernel(
    AdamSeg* __restrict__ vec, const int32_t* __restrict__ vec_in, int64_t nvec,
    AdamSeg* __restrict__ sca, const int32_t* __restrict__ sca_in,
    const int64_t* __restrict__ sca_goff, int64_t nsca, const GradPatch p) {
  for (int64_t j = int64_t(blockIdx.x) * kThreads + threadIdx.x; j < nvec + nsca;
       j += int64_t(gridDim.x) * kThreads) {
    if (j < nvec) {
      const int64_t k = int64_t(vec_in[j]) - p.k0;
      if (k >= 0 && k < p.n) glob(&vec[j].g)[0] = reinterpret_cast<const void*>(p.g[k]);
    } else {
      const int64_t t = j - nvec;
      const int64_t k = int64_t(sca_in[t]) - p.k0;
      if (k >= 0 && k < p.n) {
        const uint64_t g = p.g[k];
        glob(&sca[t].g)[0] = reinterpret_cast<const void*>(g ? g + uint64_t(sca_goff[t]) : 0);
      }
    }
  }
}
}  // namespace

// zs_adam_step's one-range tables: [vector segment, tail segment], prefixes {0, vch, 0, sch}.
struct AdamTables {
  AdamSeg seg[2];
  int64_t prefix[4];
};

__global__ void write_tables_kernel(AdamTables* __restrict__ d, AdamTables t) { *d = t; }

// Table uploads run on a private non-blocking stream per device, so creating a set never
// synchronises with the legacy null stream (which may hold kernels waiting on collectives).
static hipStream_t upload_stream() {
  static std::mutex mu;
  static std::map<int, hipStream_t> streams;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto it = streams.find(dev);
  if (it != streams.end()) return it->second;
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return nullptr;
  streams[dev] = st;
  return st;
}

template <typename T>
static int upload(const std::vector<T>& h, T** d) {
  *d = nullptr;
  if (h.empty()) return ZS_OK;
  hipStream_t st = upload_stream();
  if (!st) return zs::fail(ZS_ERR_HIP, "table upload: no upload stream");
  ZS_HIP(hipMalloc(reinterpret_cast<void**>(d), h.size() * sizeof(T)));
  hipError_t e = hipMemcpyAsync(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    (void)hipFree(*d);
    *d = nullptr;
    return zs::fail(ZS_ERR_HIP, "table upload failed: %s", hipGetErrorString(e));
  }
  return ZS_OK;
}

static HP make_hp(const zs_adam_hparams* h) {
  HP hp;
  hp.omb1 = h->one_minus_beta1;
  hp.beta2 = h->beta2;
  hp.omb2 = h->one_minus_beta2;
  hp.neg_step = h->neg_step_size;
  hp.bc2_sqrt = h->bc2_sqrt;
  hp.eps = h->eps;
  hp.wd = h->weight_decay;
  hp.decay_mul = h->decay_mul;
  hp.grad_div = h->grad_div;
  hp.carry_mul = h->carry_mul;
  int exp2 = 0;
  hp.div_pow2 = std::frexp(double(h->grad_div), &exp2) == 0.5 ? 1 : 0;
  hp.inv_div = float(1.0 / double(h->grad_div));
  hp.maximize = h->maximize;
  return hp;
}

// Vector table (aligned, n % 4 == 0) then scalar table (tails, unaligned), each a segment array
// with its chunk prefix; the template instance is picked by grad dtype, split master, amsgrad
// and carry.
static int launch_adam_tables(const AdamSeg* vec, const int64_t* vpre, int64_t nvec, int64_t vch,
                              const AdamSeg* sca, const int64_t* spre, int64_t nsca, int64_t sch,
                              int g_dtype, bool split, bool ams, bool carry, const HP& hp,
                              hipStream_t st) {
#define ZS_LAUNCH(KERNEL, GT, A, C, S, TAB, PRE, NS, NCH)                                     \
  hipLaunchKernelGGL((KERNEL<GT, A, C, S>), dim3(int(std::min<int64_t>(NCH, adam_grid_cap()))), \
                     dim3(kThreads), 0, st, TAB, PRE, NS, NCH, hp)
#define ZS_DISPATCH_AC(KERNEL, GT, S, TAB, PRE, NS, NCH)                                      \
  do {                                                                                        \
    if (ams && carry) ZS_LAUNCH(KERNEL, GT, true, true, S, TAB, PRE, NS, NCH);                \
    else if (ams) ZS_LAUNCH(KERNEL, GT, true, false, S, TAB, PRE, NS, NCH);                   \
    else if (carry) ZS_LAUNCH(KERNEL, GT, false, true, S, TAB, PRE, NS, NCH);                 \
    else ZS_LAUNCH(KERNEL, GT, false, false, S, TAB, PRE, NS, NCH);                           \
  } while (0)
#define ZS_DISPATCH(KERNEL, TAB, PRE, NS, NCH)                                                \
  do {                                                                                        \
    if (g_dtype == ZS_F32) ZS_DISPATCH_AC(KERNEL, float, false, TAB, PRE, NS, NCH);          \
    else if (split) ZS_DISPATCH_AC(KERNEL, unsigned short, true, TAB, PRE, NS, NCH);         \
    else ZS_DISPATCH_AC(KERNEL, unsigned short, false, TAB, PRE, NS, NCH);                   \
  } while (0)
  if (vch) {
    ZS_DISPATCH(adam_segments_kernel, vec, vpre, nvec, vch);
    ZS_HIP(hipGetLastError());
  }
  if (sch) {
    ZS_DISPATCH(adam_scalar_kernel, sca, spre, nsca, sch);
    ZS_HIP(hipGetLastError());
  }
#undef ZS_DISPATCH
#undef ZS_DISPATCH_AC
#undef ZS_LAUNCH
  return ZS_OK;
}

extern "C" {

int zs_copyset_create(const uint64_t* src, const uint64_t* dst, const int64_t* nbytes, int64_t n,
                      zs_copyset** out) {
  ZS_REQUIRE(out != nullptr, "zs_copyset_create: out is NULL");
  *out = nullptr;
  ZS_REQUIRE(n >= 0, "zs_copyset_create: n < 0");
  ZS_REQUIRE(n == 0 || (src && dst && nbytes), "zs_copyset_create: NULL table");
  std::vector<CopySeg> segs;
  std::vector<int64_t> prefix(1, 0);
  int64_t bytes = 0;
  const int unroll = copy_unroll();
  const int64_t chunk = copy_chunk_bytes(unroll);
  for (int64_t i = 0; i < n; ++i) {
    ZS_REQUIRE(nbytes[i] >= 0, "zs_copyset_create: nbytes[%lld] < 0", (long long)i);
    if (nbytes[i] == 0) continue;
    ZS_REQUIRE(dst[i] != 0, "zs_copyset_create: dst[%lld] is NULL", (long long)i);
    CopySeg s;
    s.src = reinterpret_cast<const unsigned char*>(src[i]);
    s.dst = reinterpret_cast<unsigned char*>(dst[i]);
    s.nbytes = nbytes[i];
    s.vec = aligned(src[i], 16) && aligned(dst[i], 16) ? 1 : 0;
    segs.push_back(s);
    bytes += nbytes[i];
    prefix.push_back(prefix.back() + (nbytes[i] + chunk - 1) / chunk);
  }
  zs_copyset* cs = new (std::nothrow) zs_copyset();
  if (!cs) return zs::fail(ZS_ERR_NOMEM, "zs_copyset_create: out of memory");
  cs->nseg = int64_t(segs.size());
  cs->total_chunks = prefix.back();
  cs->bytes = bytes;
  cs->unroll = unroll;
  int rc = upload(segs, &cs->d_segs);
  if (rc == ZS_OK) rc = upload(prefix, &cs->d_prefix);
  if (rc != ZS_OK) {
    zs_copyset_destroy(cs);
    return rc;
  }
  *out = cs;
  return ZS_OK;
}

int zs_copyset_run(const zs_copyset* cs, uintptr_t stream) {
  ZS_REQUIRE(cs != nullptr, "zs_copyset_run: NULL set");
  if (cs->total_chunks == 0) return ZS_OK;
  const int grid = int(std::min<int64_t>(cs->total_chunks, grid_cap()));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int force = copy_nt_mode();
  const bool nt = force < 0 ? 2 * cs->bytes > kMallBytes : force == 1;
#define ZS_COPY(U, NT) hipLaunchKernelGGL((copy_segments_kernel<U, NT>), dim3(grid), dim3(kThreads), 0, st, \
                                          cs->d_segs, cs->d_prefix, cs->nseg, cs->total_chunks)
  if (nt) {
    switch (cs->unroll) { case 8: ZS_COPY(8, true); break; case 2: ZS_COPY(2, true); break; default: ZS_COPY(4, true); }
  } else {
    switch (cs->unroll) { case 8: ZS_COPY(8, false); break; case 2: ZS_COPY(2, false); break; default: ZS_COPY(4, false); }
  }
#undef ZS_COPY
  ZS_HIP(hipGetLastError());
  return ZS_OK;
}

int zs_copyset_destroy(zs_copyset* cs) {
  if (!cs) return ZS_OK;
  if (cs->d_segs) (void)hipFree(cs->d_segs);
  if (cs->d_prefix) (void)hipFree(cs->d_prefix);
  delete cs;
  return ZS_OK;
}

int zs_copy_direct(int64_t n, const uint64_t* src, const uint64_t* dst, const int64_t* nbytes,
                   uintptr_t stream) {
  ZS_REQUIRE(n >= 0, "zs_copy_direct: n < 0");
  if (n == 0) return ZS_OK;
  ZS_REQUIRE(src && dst && nbytes, "zs_copy_direct: NULL table");
  int64_t total_bytes = 0;
  for (int64_t i = 0; i < n; ++i) {
    ZS_REQUIRE(nbytes[i] >= 0, "zs_copy_direct: nbytes[%lld] < 0", (long long)i);
    ZS_REQUIRE(nbytes[i] == 0 || dst[i] != 0, "zs_copy_direct: dst[%lld] is NULL", (long long)i);
    total_bytes += nbytes[i];
  }
  const int force = copy_nt_mode();
  const bool nt = force < 0 ? 2 * total_bytes > kMallBytes : force == 1;
  constexpr int U = kCopyUnrollDefault;
  const int64_t chunk = copy_chunk_bytes(U);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int64_t i0 = 0; i0 < n;) {  // launches of up to kDirectMax non-empty segments
    DirectSet set{};
    int k = 0;
    for (; i0 < n && k < kDirectMax; ++i0) {
      if (nbytes[i0] == 0) continue;
      set.src[k] = reinterpret_cast<const unsigned char*>(src[i0]);
      set.dst[k] = reinterpret_cast<unsigned char*>(dst[i0]);
      set.nbytes[k] = nbytes[i0];
      set.prefix[k + 1] = set.prefix[k] + (nbytes[i0] + chunk - 1) / chunk;
      if (aligned(src[i0], 16) && aligned(dst[i0], 16)) set.vec_mask |= uint64_t(1) << k;
      ++k;
    }
    set.n = k;
    if (k == 0) break;
    for (int j = k; j < kDirectMax; ++j) set.prefix[j + 1] = set.prefix[k];
    const int grid = int(std::min<int64_t>(set.prefix[k], grid_cap()));
    if (nt) hipLaunchKernelGGL((copy_direct_kernel<U, true>), dim3(grid), dim3(kThreads), 0, st, set);
    else hipLaunchKernelGGL((copy_direct_kernel<U, false>), dim3(grid), dim3(kThreads), 0, st, set);
    ZS_HIP(hipGetLastError());
  }
  return ZS_OK;
}

int zs_scale(void* x, int64_t n, int dtype, double div, uintptr_t stream) {
  ZS_REQUIRE(n >= 0, "zs_scale: n < 0");
  ZS_REQUIRE(dtype == ZS_F32 || dtype == ZS_BF16, "zs_scale: bad dtype %d", dtype);
  ZS_REQUIRE(div != 0.0, "zs_scale: div == 0");
  if (n == 0) return ZS_OK;
  ZS_REQUIRE(x != nullptr && aligned(reinterpret_cast<uint64_t>(x), 16),
             "zs_scale: x must be non-NULL and 16-byte aligned");
  int e = 0;
  const int pow2 = std::frexp(div, &e) == 0.5 ? 1 : 0;
  const float fdiv = float(div), inv = float(1.0 / div);
  const int64_t span = int64_t(64) * kScaleU * (dtype == ZS_F32 ? 4 : 8);  // elements per wave step
  const int64_t blocks = std::max<int64_t>(1, (n / span + 3) / 4);
  const int grid = int(std::min<int64_t>(blocks, grid_cap()));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int force = scale_nt_mode();
  const bool nt = force < 0 ? n * (dtype == ZS_F32 ? 4 : 2) > kMallBytes : force == 1;
#define ZS_SCALE(T, NT) hipLaunchKernelGGL((scale_kernel<T, NT>), dim3(grid), dim3(kThreads), 0, st, \
                                           static_cast<T*>(x), n, fdiv, inv, pow2)
  if (dtype == ZS_F32) {
    if (nt) ZS_SCALE(float, true); else ZS_SCALE(float, false);
  } else {
    if (nt) ZS_SCALE(unsigned short, true); else ZS_SCALE(unsigned short, false);
  }
#undef ZS_SCALE
  ZS_HIP(hipGetLastError());
  return ZS_OK;
}

int zs_convert(const void* src, int src_dtype, void* dst, int dst_dtype, int64_t n,
               uintptr_t stream) {
  ZS_REQUIRE(n >= 0, "zs_convert: n < 0");
  ZS_REQUIRE((src_dtype == ZS_F32 && dst_dtype == ZS_BF16) ||
                 (src_dtype == ZS_BF16 && dst_dtype == ZS_F32),
             "zs_convert: only fp32 <-> bf16 (got %d -> %d)", src_dtype, dst_dtype);
  if (n == 0) return ZS_OK;
  ZS_REQUIRE(src && dst, "zs_convert: NULL buffer");
  const bool to_bf16 = src_dtype == ZS_F32;
  const bool vec = aligned(uint64_t(src), 16) && aligned(uint64_t(dst), 16);
  // vector path: one wave per kConvSpan-element step (4 waves per workgroup)
  const int64_t work = vec ? std::max<int64_t>(1, (n / kConvSpan + 3) / 4) : (n + kThreads - 1) / kThreads;
  const int grid = int(std::min<int64_t>(work, grid_cap()));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (vec) {
    const int force = convert_nt_mode();
    const bool nt = force < 0 ? n * 6 > kMallBytes : force == 1;  // by both sides' bytes
#define ZS_CONV(B, NT) hipLaunchKernelGGL((convert_kernel<B, NT>), dim3(grid), dim3(kThreads), 0, st, src, dst, n)
    if (to_bf16) {
      if (nt) ZS_CONV(true, true); else ZS_CONV(true, false);
    } else {
      if (nt) ZS_CONV(false, true); else ZS_CONV(false, false);
    }
#undef ZS_CONV
  } else {
    if (to_bf16) hipLaunchKernelGGL(convert_scalar_kernel<true>, dim3(grid), dim3(kThreads), 0, st, src, dst, n);
    else hipLaunchKernelGGL(convert_scalar_kernel<false>, dim3(grid), dim3(kThreads), 0, st, src, dst, n);
  }
  ZS_HIP(hipGetLastError());
  return ZS_OK;
}

int zs_fp8_quantize_rows(const void* src, int src_dtype, void* dst, float* scales, int64_t rows,
                         int64_t row_len, uintptr_t stream) {
  ZS_REQUIRE(rows >= 0 && row_len >= 0, "zs_fp8_quantize_rows: negative size");
  ZS_REQUIRE(src_dtype == ZS_F32 || src_dtype == ZS_BF16, "zs_fp8_quantize_rows: bad dtype %d",
             src_dtype);
  if (rows == 0 || row_len == 0) return ZS_OK;
  ZS_REQUIRE(src && dst && scales, "zs_fp8_quantize_rows: NULL buffer");
  const bool vec = row_len % 8 == 0 && aligned(uint64_t(src), 16) && aligned(uint64_t(dst), 8);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  unsigned char* q = static_cast<unsigned char*>(dst);
  if (vec) {  // wave per row, 4 rows per workgroup
    const int grid = int(std::min<int64_t>((rows + 3) / 4, grid_cap()));
    // 16-B chunks per lane the row needs: the smallest register-resident variant that holds it
    const int64_t chunks = (row_len + 64 * (src_dtype == ZS_F32 ? 4 : 8) - 1) / (64 * (src_dtype == ZS_F32 ? 4 : 8));
    const int nreg = chunks <= 8 ? 8 : chunks <= 16 ? 16 : chunks <= 32 ? 32 : 0;
#define ZS_Q(T, N, X) hipLaunchKernelGGL((fp8_quantize_rows_wave_kernel<T, N>), dim3(grid), dim3(kThreads), 0, st, X, q, scales, rows, row_len)
#define ZS_QSEL(T, X) \
    switch (nreg) { case 8: ZS_Q(T, 8, X); break; case 16: ZS_Q(T, 16, X); break; \
                    case 32: ZS_Q(T, 32, X); break; default: ZS_Q(T, 0, X); }
    if (src_dtype == ZS_F32) {
      const float* x = static_cast<const float*>(src);
      ZS_QSEL(float, x)
    } else {
      const unsigned short* x = static_cast<const unsigned short*>(src);
      ZS_QSEL(unsigned short, x)
    }
#undef ZS_QSEL
#undef ZS_Q
  } else {  // any row length / alignment: block per row, scalar accesses
    const int grid = int(std::min<int64_t>(rows, grid_cap()));
    if (src_dtype == ZS_F32)
      hipLaunchKernelGGL((fp8_quantize_rows_kernel<float>), dim3(grid), dim3(kThreads), 0, st, static_cast<const float*>(src), q, scales, rows, row_len);
    else
      hipLaunchKernelGGL((fp8_quantize_rows_kernel<unsigned short>), dim3(grid), dim3(kThreads), 0, st, static_cast<const unsigned short*>(src), q, scales, rows, row_len);
  }
  ZS_HIP(hipGetLastError());
  return ZS_OK;
}

int zs_fp8_dequantize_rows(const void* src, const float* scales, void* dst, int dst_dtype,
                           int64_t rows, int64_t row_len, uintptr_t stream) {
  ZS_REQUIRE(rows >= 0 && row_len >= 0, "zs_fp8_dequantize_rows: negative size");
  ZS_REQUIRE(dst_dtype == ZS_F32 || dst_dtype == ZS_BF16, "zs_fp8_dequantize_rows: bad dtype %d",
             dst_dtype);
  if (rows == 0 || row_len == 0) return ZS_OK;
  ZS_REQUIRE(src && dst && scales, "zs_fp8_dequantize_rows: NULL buffer");
  const int64_t n = rows * row_len;
  const bool vec = row_len % 8 == 0 && aligned(uint64_t(src), 8) && aligned(uint64_t(dst), 16);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const unsigned char* q = static_cast<const unsigned char*>(src);
  if (vec) {  // the gathered kernel over one matrix of one rank: one wave per row
    ZS_REQUIRE(rows < (int64_t(1) << 31), "zs_fp8_dequantize_rows: %lld rows (max 2^31 - 1)",
               (long long)rows);
    DqSet set{};
    set.q = q;
    set.sc = scales;
    set.n = 1;
    set.cs[0] = rows;
    set.row_len[0] = row_len;
    set.dst[0] = dst;
    set.prefix[0] = 0;
    for (int k = 1; k <= kSetMax; ++k) set.prefix[k] = rows;
    const int grid = dq_grid(rows);
    launch_dequantize(set, dst_dtype, grid, st);
  } else {
    const int grid = int(std::min<int64_t>(std::max<int64_t>(1, (n + kThreads - 1) / kThreads), grid_cap()));
    if (dst_dtype == ZS_F32)
      hipLaunchKernelGGL((fp8_dequantize_rows_kernel<float>), dim3(grid), dim3(kThreads), 0, st, q, scales, static_cast<float*>(dst), n, row_len);
    else
      hipLaunchKernelGGL((fp8_dequantize_rows_kernel<unsigned short>), dim3(grid), dim3(kThreads), 0, st, q, scales, static_cast<unsigned short*>(dst), n, row_len);
  }
  ZS_HIP(hipGetLastError());
  return ZS_OK;
}

int zs_fp8_quantize_rowset(int64_t n, const uint64_t* src, const uint64_t* q, const uint64_t* scales,
                           const int64_t* rows, const int64_t* cs, const int64_t* row_len,
                           int src_dtype, uintptr_t stream) {
  ZS_REQUIRE(n >= 0, "zs_fp8_quantize_rowset: n < 0");
  ZS_REQUIRE(src_dtype == ZS_F32 || src_dtype == ZS_BF16, "zs_fp8_quantize_rowset: bad dtype %d",
             src_dtype);
  if (n == 0) return ZS_OK;
  ZS_REQUIRE(src && q && scales && rows && cs && row_len, "zs_fp8_quantize_rowset: NULL table");
  const int E = src_dtype == ZS_F32 ? 4 : 8;
  for (int64_t m = 0; m < n; ++m) {
    ZS_REQUIRE(rows[m] >= 0 && cs[m] >= rows[m] && row_len[m] > 0 && row_len[m] % 8 == 0,
               "zs_fp8_quantize_rowset: matrix %lld: rows %lld, cs %lld, row_len %lld (needs "
               "0 <= rows <= cs, row_len a positive multiple of 8)", (long long)m,
               (long long)rows[m], (long long)cs[m], (long long)row_len[m]);
    ZS_REQUIRE((rows[m] == 0 || (src[m] && aligned(src[m], 16))) && (cs[m] == 0 || (q[m] &&
               aligned(q[m], 8) && scales[m] && aligned(scales[m], 4))),
               "zs_fp8_quantize_rowset: matrix %lld: src must be 16-B and q 8-B aligned",
               (long long)m);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // one launch per register class (8 / 16 / 32 resident chunks per lane, or streamed) and per
  // kSetMax matrices: a long-row matrix does not push the others into its low-occupancy variant
  auto nreg_of = [&](int64_t len) {
    const int64_t chunks = (len + 64 * E - 1) / (64 * E);
    return chunks <= 8 ? 8 : chunks <= 16 ? 16 : chunks <= 32 ? 32 : 0;
  };
  for (int cls : {8, 16, 32, 0}) {
    std::vector<int64_t> ms;
    for (int64_t m = 0; m < n; ++m)
      if (nreg_of(row_len[m]) == cls && cs[m] > 0) ms.push_back(m);
    for (size_t k0 = 0; k0 < ms.size(); k0 += kSetMax) {
      QSet set{};
      set.n = int(std::min<size_t>(kSetMax, ms.size() - k0));
      set.prefix[0] = 0;
      for (int k = 0; k < set.n; ++k) {
        const int64_t m = ms[k0 + k];
        set.src[k] = reinterpret_cast<const void*>(src[m]);
        set.q[k] = reinterpret_cast<unsigned char*>(q[m]);
        set.sc[k] = reinterpret_cast<float*>(scales[m]);
        set.rows[k] = rows[m];
        set.row_len[k] = row_len[m];
        set.prefix[k + 1] = set.prefix[k] + cs[m];
      }
      for (int k = set.n; k < kSetMax; ++k) set.prefix[k + 1] = set.prefix[set.n];
      const int64_t total = set.prefix[set.n];
      const int grid = int(std::min<int64_t>((total + 3) / 4, grid_cap()));
#define ZS_QS(T, N) hipLaunchKernelGGL((fp8_quantize_rowset_kernel<T, N>), dim3(grid), dim3(kThreads), 0, st, set)
#define ZS_QSSEL(T) \
      switch (cls) { case 8: ZS_QS(T, 8); break; case 16: ZS_QS(T, 16); break; \
                     case 32: ZS_QS(T, 32); break; default: ZS_QS(T, 0); }
      if (src_dtype == ZS_F32) { ZS_QSSEL(float) } else { ZS_QSSEL(unsigned short) }
#undef ZS_QSSEL
#undef ZS_QS
      ZS_HIP(hipGetLastError());
    }
  }
  return ZS_OK;
}

int zs_fp8_dequantize_gathered(int64_t n, const void* q, const float* scales, int ws,
                               int64_t q_rank_bytes, int64_t sc_rank_elems, const int64_t* q_off,
                               const int64_t* sc_off, const int64_t* cs, const int64_t* row_len,
                               const uint64_t* dst, int dst_dtype, uintptr_t stream) {
  ZS_REQUIRE(n >= 0 && ws >= 1, "zs_fp8_dequantize_gathered: n %lld, ws %d", (long long)n, ws);
  ZS_REQUIRE(dst_dtype == ZS_F32 || dst_dtype == ZS_BF16,
             "zs_fp8_dequantize_gathered: bad dtype %d", dst_dtype);
  if (n == 0) return ZS_OK;
  ZS_REQUIRE(q && scales && q_off && sc_off && cs && row_len && dst,
             "zs_fp8_dequantize_gathered: NULL buffer or table");
  ZS_REQUIRE(aligned(uint64_t(q), 8) && aligned(uint64_t(scales), 4) && q_rank_bytes % 8 == 0 &&
                 q_rank_bytes >= 0 && sc_rank_elems >= 0,
             "zs_fp8_dequantize_gathered: q must be 8-B aligned with an 8-B multiple rank stride");
  for (int64_t m = 0; m < n; ++m)
    ZS_REQUIRE(cs[m] >= 0 && row_len[m] > 0 && row_len[m] % 8 == 0 && q_off[m] % 8 == 0 &&
                   q_off[m] >= 0 && sc_off[m] >= 0 && (cs[m] == 0 || (dst[m] && aligned(dst[m], 16))),
               "zs_fp8_dequantize_gathered: matrix %lld: cs %lld, row_len %lld, q_off %lld (needs "
               "row_len and q_off multiples of 8, dst 16-B aligned)", (long long)m,
               (long long)cs[m], (long long)row_len[m], (long long)q_off[m]);
  for (int64_t m = 0; m < n; ++m)  // the kernel's row arithmetic is 32-bit
    ZS_REQUIRE(int64_t(ws) * cs[m] < (int64_t(1) << 31),
               "zs_fp8_dequantize_gathered: matrix %lld too large (%lld rows x %d ranks)",
               (long long)m, (long long)cs[m], ws);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int64_t m0 = 0; m0 < n; m0 += kSetMax) {
    DqSet set{};
    set.q = static_cast<const unsigned char*>(q);
    set.sc = scales;
    set.q_rank = q_rank_bytes;
    set.sc_rank = sc_rank_elems;
    set.n = int(std::min<int64_t>(kSetMax, n - m0));
    set.prefix[0] = 0;
    for (int k = 0; k < set.n; ++k) {
      const int64_t m = m0 + k;
      set.q_off[k] = q_off[m];
      set.sc_off[k] = sc_off[m];
      set.cs[k] = cs[m];
      set.row_len[k] = row_len[m];
      set.dst[k] = reinterpret_cast<void*>(dst[m]);
      set.prefix[k + 1] = set.prefix[k] + int64_t(ws) * cs[m];
    }
    for (int k = set.n; k < kSetMax; ++k) set.prefix[k + 1] = set.prefix[set.n];
    const int64_t total = set.prefix[set.n];
    if (total == 0) continue;
    const int grid = dq_grid(total);
    launch_dequantize(set, dst_dtype, grid, st);
    ZS_HIP(hipGetLastError());
  }
  return ZS_OK;
}

int zs_adam_hparams_init(double lr, double beta1, double beta2, double eps, double weight_decay,
                         int decoupled, int amsgrad, int maximize, int64_t step, double grad_div,
                         double carry_mul, zs_adam_hparams* hp) {
  ZS_REQUIRE(hp != nullptr, "zs_adam_hparams_init: hp is NULL");
  ZS_REQUIRE(step >= 1, "zs_adam_hparams_init: step must be >= 1");
  ZS_REQUIRE(grad_div > 0.0, "zs_adam_hparams_init: grad_div must be > 0");
  // adam.py:508-515 (non-capturable): Python-float (double) scalars.
  const double t = double(step);
  const double bc1 = 1.0 - std::pow(beta1, t);
  const double bc2 = 1.0 - std::pow(beta2, t);
  hp->one_minus_beta1 = float(1.0 - beta1);
  hp->beta2 = float(beta2);
  hp->one_minus_beta2 = float(1.0 - beta2);
  hp->neg_step_size = float(-(lr / bc1));
  hp->bc2_sqrt = float(std::pow(bc2, 0.5));
  hp->eps = float(eps);
  hp->weight_decay = decoupled ? 0.0f : float(weight_decay);
  hp->decay_mul = decoupled ? float(1.0 - lr * weight_decay) : 1.0f;
  hp->grad_div = float(grad_div);
  hp->carry_mul = float(carry_mul);
  hp->amsgrad = amsgrad ? 1 : 0;
  hp->maximize = maximize ? 1 : 0;
  return ZS_OK;
}

int zs_adamset_create(const zs_adam_seg* in, int64_t n, int g_dtype, int p_dtype,
                      zs_adamset** out) {
  ZS_REQUIRE(out != nullptr, "zs_adamset_create: out is NULL");
  *out = nullptr;
  ZS_REQUIRE(n >= 0 && (n == 0 || in), "zs_adamset_create: bad table");
  ZS_REQUIRE(g_dtype == ZS_F32 || g_dtype == ZS_BF16, "zs_adamset_create: bad g_dtype %d", g_dtype);
  ZS_REQUIRE(p_dtype == ZS_BF16 || p_dtype == ZS_BF16_SPLIT,
             "zs_adamset_create: p_dtype must be ZS_BF16 or ZS_BF16_SPLIT (got %d)", p_dtype);
  const bool split = p_dtype == ZS_BF16_SPLIT;
  ZS_REQUIRE(!split || g_dtype == ZS_BF16, "zs_adamset_create: ZS_BF16_SPLIT needs bf16 grads");
  const int64_t msz = split ? 2 : 4;  // bytes per element of master / master_out
  const int64_t gsz = g_dtype == ZS_F32 ? 4 : 2;
  ZS_REQUIRE(n < (int64_t(1) << 31), "zs_adamset_create: %lld segments (max 2^31 - 1)",
             (long long)n);
  std::vector<AdamSeg> vec, sca;
  std::vector<int64_t> vpre(1, 0), spre(1, 0);
  std::vector<int32_t> vec_in, sca_in;
  std::vector<int64_t> sca_goff;
  std::vector<uint64_t> in_g(size_t(n), 0);
  std::vector<int64_t> in_n(size_t(n), 0);
  std::vector<unsigned char> in_vec(size_t(n), 0);
  int carry_state = -1, vmax_state = -1;
  int64_t elems = 0, bytes = 0, bytes_no_g = 0;
  for (int64_t i = 0; i < n; ++i) {
    const zs_adam_seg& s = in[i];
    ZS_REQUIRE(s.n >= 0, "zs_adamset_create: seg %lld n < 0", (long long)i);
    in_g[size_t(i)] = s.g;
    in_n[size_t(i)] = s.n;
    if (s.n == 0) continue;
    ZS_REQUIRE(s.master && s.m && s.v, "zs_adamset_create: seg %lld missing master/m/v",
               (long long)i);
    ZS_REQUIRE(!split || (s.master_out && s.p_out),
               "zs_adamset_create: seg %lld: a split master needs master_out (residual) and p_out",
               (long long)i);
    const int c = s.carry ? 1 : 0;
    ZS_REQUIRE(carry_state < 0 || carry_state == c,
               "zs_adamset_create: carry must be set on all segments or none");
    carry_state = c;
    const int x = s.vmax ? 1 : 0;
    ZS_REQUIRE(vmax_state < 0 || vmax_state == x,
               "zs_adamset_create: vmax must be set on all segments or none");
    vmax_state = x;
    AdamSeg d;
    d.g = reinterpret_cast<const void*>(s.g);
    d.master = reinterpret_cast<const float*>(s.master);
    d.master_out = reinterpret_cast<float*>(s.master_out);
    d.p_out = reinterpret_cast<unsigned short*>(s.p_out);
    d.m = reinterpret_cast<float*>(s.m);
    d.v = reinterpret_cast<float*>(s.v);
    d.vmax = reinterpret_cast<float*>(s.vmax);
    d.carry = reinterpret_cast<float*>(s.carry);
    const bool ok = aligned(s.g, uint64_t(gsz) * 4) && aligned(s.master, uint64_t(msz) * 4) &&
                    aligned(s.master_out, uint64_t(msz) * 4) && aligned(s.p_out, 8) && aligned(s.m, 16) &&
                    aligned(s.v, 16) && aligned(s.vmax, 16) && aligned(s.carry, 16);
    const int64_t nv = ok ? (s.n & ~int64_t(3)) : 0;
    if (nv) {
      d.n = nv;
      vec.push_back(d);
      vec_in.push_back(int32_t(i));
      in_vec[size_t(i)] = 1;
      vpre.push_back(vpre.back() + (nv + adam_chunk(split) - 1) / adam_chunk(split));
    }
    if (nv < s.n) {  // tail (or the whole unaligned segment) through the scalar kernel
      AdamSeg t = d;
      auto adv = [nv](auto* p, int64_t es) {
        using P = decltype(p);
        return p ? reinterpret_cast<P>(reinterpret_cast<uintptr_t>(p) + uintptr_t(nv * es)) : p;
      };
      t.g = s.g ? reinterpret_cast<const void*>(s.g + uint64_t(nv * gsz)) : nullptr;
      t.master = adv(d.master, msz);
      t.master_out = adv(d.master_out, msz);
      t.p_out = adv(d.p_out, 2);
      t.m = adv(d.m, 4);
      t.v = adv(d.v, 4);
      t.vmax = adv(d.vmax, 4);
      t.carry = adv(d.carry, 4);
      t.n = s.n - nv;
      sca.push_back(t);
      sca_in.push_back(int32_t(i));
      sca_goff.push_back(nv * gsz);
      spre.push_back(spre.back() + (t.n + kThreads - 1) / kThreads);
    }
    elems += s.n;
    int64_t b = msz /*master*/ + 8 /*m*/ + 8 /*v*/;
    if (s.master_out) b += split ? 4 /*residual read + write*/ : 4;
    if (s.p_out) b += 2;
    if (s.vmax) b += 8;
    if (s.carry) b += 8;
    bytes_no_g += b * s.n;
    bytes += (b + (s.g ? gsz : 0)) * s.n;
  }
  zs_adamset* as = new (std::nothrow) zs_adamset();
  if (!as) return zs::fail(ZS_ERR_NOMEM, "zs_adamset_create: out of memory");
  as->nvec = int64_t(vec.size());
  as->vec_chunks = vpre.back();
  as->nsca = int64_t(sca.size());
  as->sca_chunks = spre.back();
  as->elems = elems;
  as->bytes = bytes;
  as->g_dtype = g_dtype;
  as->p_dtype = p_dtype;
  as->has_carry = carry_state > 0 ? 1 : 0;
  as->has_vmax = vmax_state > 0 ? 1 : 0;
  as->in_g = std::move(in_g);
  as->in_n = std::move(in_n);
  as->in_vec = std::move(in_vec);
  as->bytes_no_g = bytes_no_g;
  int rc = ZS_OK;
  if (as->nvec) {
    rc = upload(vec, &as->d_vec);
    if (rc == ZS_OK) rc = upload(vpre, &as->d_vec_prefix);
    if (rc == ZS_OK) rc = upload(vec_in, &as->d_vec_in);
  }
  if (rc == ZS_OK && as->nsca) {
    rc = upload(sca, &as->d_sca);
    if (rc == ZS_OK) rc = upload(spre, &as->d_sca_prefix);
    if (rc == ZS_OK) rc = upload(sca_in, &as->d_sca_in);
    if (rc == ZS_OK) rc = upload(sca_goff, &as->d_sca_goff);
  }
  if (rc != ZS_OK) {
    zs_adamset_destroy(as);
    return rc;
  }
  *out = as;
  return ZS_OK;
}

int zs_adamset_run(const zs_adamset* as, const zs_adam_hparams* h, uintptr_t stream) {
  ZS_REQUIRE(as && h, "zs_adamset_run: NULL argument");
  const bool ams = h->amsgrad != 0;
  ZS_REQUIRE(!ams || as->has_vmax || (as->nvec + as->nsca) == 0,
             "zs_adamset_run: amsgrad needs vmax segments");
  return launch_adam_tables(as->d_vec, as->d_vec_prefix, as->nvec, as->vec_chunks, as->d_sca,
                            as->d_sca_prefix, as->nsca, as->sca_chunks, as->g_dtype,
                            as->p_dtype == ZS_BF16_SPLIT, ams, as->has_carry != 0, make_hp(h),
                            reinterpret_cast<hipStream_t>(stream));
}

// zs_adam_step: one contiguous range through the same kernels.  Its two one-entry tables
// (vector part + tail) are written on the caller's stream by a one-thread kernel into a
// stream-ordered allocation, so the call neither synchronises nor keeps state between calls.
int zs_adam_step_ex(float* p, uint16_t* p_bf16, const void* g, int g_dtype, float* m, float* v,
                    int64_t n, double lr, double beta1, double beta2, double eps,
                    double weight_decay, int decoupled, int64_t step, double grad_div, float* carry,
                    double carry_mul, uintptr_t stream) {
  ZS_REQUIRE(n >= 0, "zs_adam_step_ex: n < 0");
  ZS_REQUIRE(g_dtype == ZS_F32 || g_dtype == ZS_BF16, "zs_adam_step_ex: bad g_dtype %d", g_dtype);
  ZS_REQUIRE(n == 0 || (p && m && v), "zs_adam_step_ex: p, m and v must be non-NULL");
  zs_adam_hparams h;
  int rc = zs_adam_hparams_init(lr, beta1, beta2, eps, weight_decay, decoupled, 0, 0, step,
                                grad_div, carry_mul, &h);
  if (rc != ZS_OK) return rc;
  if (n == 0) return ZS_OK;
  const int64_t gsz = g_dtype == ZS_F32 ? 4 : 2;
  const uint64_t up = reinterpret_cast<uint64_t>(p), ug = reinterpret_cast<uint64_t>(g);
  const uint64_t ub = reinterpret_cast<uint64_t>(p_bf16), um = reinterpret_cast<uint64_t>(m);
  const uint64_t uv = reinterpret_cast<uint64_t>(v), uc = reinterpret_cast<uint64_t>(carry);
  const bool ok = aligned(ug, uint64_t(gsz) * 4) && aligned(up, 16) && aligned(ub, 8) &&
                  aligned(um, 16) && aligned(uv, 16) && aligned(uc, 16);
  const int64_t nv = ok ? (n & ~int64_t(3)) : 0;
  AdamTables t;
  AdamSeg& a = t.seg[0];
  a.g = g;
  a.master = p;
  a.master_out = p;
  a.p_out = reinterpret_cast<unsigned short*>(p_bf16);
  a.m = m;
  a.v = v;
  a.vmax = nullptr;
  a.carry = carry;
  a.n = nv;
  AdamSeg& b = t.seg[1];
  b = a;
  b.g = g ? reinterpret_cast<const void*>(ug + uint64_t(nv * gsz)) : nullptr;
  b.master = p + nv;
  b.master_out = p + nv;
  b.p_out = p_bf16 ? reinterpret_cast<unsigned short*>(p_bf16 + nv) : nullptr;
  b.m = m + nv;
  b.v = v + nv;
  b.carry = carry ? carry + nv : nullptr;
  b.n = n - nv;
  const int64_t vch = (nv + adam_chunk(false) - 1) / adam_chunk(false);
  const int64_t sch = (b.n + kThreads - 1) / kThreads;
  t.prefix[0] = 0;
  t.prefix[1] = vch;
  t.prefix[2] = 0;
  t.prefix[3] = sch;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  AdamTables* d = nullptr;
  ZS_HIP(hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(AdamTables), st));
  hipLaunchKernelGGL(write_tables_kernel, dim3(1), dim3(1), 0, st, d, t);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) {
    rc = launch_adam_tables(d->seg, d->prefix, 1, vch, d->seg + 1, d->prefix + 2, 1, sch, g_dtype,
                            false, false, carry != nullptr, make_hp(&h), st);
  }
  const hipError_t ef = hipFreeAsync(d, st);  // after the launches, in stream order
  if (e != hipSuccess)
    return zs::fail(ZS_ERR_HIP, "zs_adam_step_ex: table kernel: %s", hipGetErrorString(e));
  if (rc != ZS_OK) return rc;
  ZS_HIP(ef);
  return ZS_OK;
}

// SURVEY.md §8(b)'s literal signature: float scalars and grad_scale = 1/ws.  The divisor is the
// integer nearest to 1/grad_scale when that is within float(1/ws)'s rounding (2^-24 relative) —
// the world size, so the update divides as zero1.py:84 `p.grad /= ws` does — else 1/grad_scale;
// the scalars are widened to double before torch's bias-correction arithmetic.  carry is read and
// rewritten (A_{t-1} -> A_t) although the reference signature spells it const.
int zs_adam_step(float* p, uint16_t* p_bf16, const void* g, int g_dtype, float* m, float* v,
                 int64_t n, float lr, float b1, float b2, float eps, float wd, int decoupled,
                 int64_t step, float grad_scale, float* carry, float carry_scale,
                 uintptr_t stream) {
  ZS_REQUIRE(grad_scale > 0.0f && std::isfinite(grad_scale), "zs_adam_step: grad_scale must be > 0");
  const double r = 1.0 / double(grad_scale), k = std::nearbyint(r);
  const double div = (k >= 1.0 && std::fabs(r - k) <= 1e-6 * k) ? k : r;
  return zs_adam_step_ex(p, p_bf16, g, g_dtype, m, v, n, lr, b1, b2, eps, wd, decoupled, step, div,
                         carry, carry_scale, stream);
}

int zs_adamset_set_grads(zs_adamset* as, int64_t n, const uint64_t* g, uintptr_t stream) {
  ZS_REQUIRE(as != nullptr, "zs_adamset_set_grads: NULL set");
  ZS_REQUIRE(n == int64_t(as->in_g.size()),
             "zs_adamset_set_grads: %lld gradients for a set of %lld segments", (long long)n,
             (long long)as->in_g.size());
  ZS_REQUIRE(n == 0 || g != nullptr, "zs_adamset_set_grads: NULL table");
  const uint64_t galign = as->g_dtype == ZS_F32 ? 16 : 8;
  int64_t lo = n, hi = -1, g_elems = 0;
  for (int64_t i = 0; i < n; ++i) {
    // the set's vector / scalar split was made on the create-time alignment: a gradient of an
    // input with a vector part must keep it (torch allocations are 512-B aligned)
    ZS_REQUIRE(!as->in_vec[size_t(i)] || aligned(g[i], galign),
               "zs_adamset_set_grads: g[%lld] = %#llx is not %llu-byte aligned", (long long)i,
               (unsigned long long)g[i], (unsigned long long)galign);
    if (g[i] != as->in_g[size_t(i)]) {
      lo = std::min(lo, i);
      hi = i;
    }
    if (g[i]) g_elems += as->in_n[size_t(i)];
  }
  if (hi < lo) return ZS_OK;  // bound to these gradients already: nothing to launch
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t nseg = as->nvec + as->nsca;
  const int grid = int(std::max<int64_t>(1, std::min<int64_t>((nseg + kThreads - 1) / kThreads, 64)));
  for (int64_t k0 = lo; k0 <= hi; k0 += kGradPatchMax) {
    GradPatch p{};
    p.k0 = k0;
    p.n = int(std::min<int64_t>(kGradPatchMax, hi + 1 - k0));
    for (int k = 0; k < p.n; ++k) p.g[k] = g[k0 + k];
    if (nseg)
      hipLaunchKernelGGL(adam_patch_grads_kernel, dim3(grid), dim3(kThreads), 0, st, as->d_vec,
                         as->d_vec_in, as->nvec, as->d_sca, as->d_sca_in, as->d_sca_goff, as->nsca,
                         p);
    ZS_HIP(hipGetLastError());
  }
  std::copy(g, g + n, as->in_g.begin());
  const int64_t gsz = as->g_dtype == ZS_F32 ? 4 : 2;
  as->bytes = as->bytes_no_g + gsz * g_elems;
  return ZS_OK;
}

int zs_adamset_destroy(zs_adamset* as) {
  if (!as) return ZS_OK;
  if (as->d_vec) (void)hipFree(as->d_vec);
  if (as->d_vec_prefix) (void)hipFree(as->d_vec_prefix);
  if (as->d_sca) (void)hipFree(as->d_sca);
  if (as->d_sca_prefix) (void)hipFree(as->d_sca_prefix);
  if (as->d_vec_in) (void)hipFree(as->d_vec_in);
  if (as->d_sca_in) (void)hipFree(as->d_sca_in);
  if (as->d_sca_goff) (void)hipFree(as->d_sca_goff);
  delete as;
  return ZS_OK;
}

int zs_adamset_stats(const zs_adamset* as, int64_t* elems, int64_t* bytes) {
  ZS_REQUIRE(as && elems && bytes, "zs_adamset_stats: NULL argument");
  *elems = as->elems;
  *bytes = as->bytes;
  return ZS_OK;
}

}  // extern "C"

// A stream-flag record (zs_comm.cpp zs_sync_record): one wave whose lane 0 stores the epoch with a
// system-scope release (a vector store: global_store … sc0 sc1).  In stream order like any launch
// (the dispatch waits for the stream's earlier work, whose writes its end-of-kernel release made
// visible), so the word reaches `value` only after everything recorded before it — what
// hipStreamWriteValue64 does, without the runtime's stream-operation command: on this stack that
// command costs a HIP runtime thread ~20 us of CPU per record (profiles/r06_z3_thr_*.json: 1.5 ms
// of the simulated ws = 8 C5 iteration's 102 records), a kernel launch does not.
template <bool kFence>
__global__ __launch_bounds__(64) void flag_write_kernel(uint64_t* flag, uint64_t value) {
  // kFence: a system-scope release (an L2 write-back first); without it a relaxed store straight
  // to memory (sc0 sc1) — the stream's earlier kernels made their writes visible at their own end
  if (threadIdx.x == 0) {
    if (kFence)
      __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// A stream-flag wait as one wave that polls the word with s_sleep between loads (zs_tune
// "sync_wait_kernel" 1).  hipStreamWaitValue64 on this stack is a runtime kernel
// (__amd_rocclr_streamOpsWait) spinning without pause: a side stream waiting for the compute stream
// keeps it busy for milliseconds beside the compute stream's GEMMs (profiles/r06_sm3_sim8 kernel
// stats).  Gives up after ~2^24 polls (about a minute) rather than hold the GPU forever, and then
// stores 1 into `timed_out` (a pinned host word): the next sync call on the host fails loudly
// (zs_comm.cpp flag_wait_check) instead of the lost ordering passing silently.
__global__ __launch_bounds__(64) void flag_wait_kernel(const uint64_t* flag, uint64_t value,
                                                       uint32_t* timed_out) {
  if (threadIdx.x == 0) {
    uint32_t i = 0;
    for (; i < (1u << 24); ++i) {
      if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= value) break;
      __builtin_amdgcn_s_sleep(64);
    }
    if (i == (1u << 24) && timed_out != nullptr)
      __hip_atomic_store(timed_out, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

namespace zs {
int& sync_write_kernel() {  // zs_tune("sync_write_kernel"): 1 = flag_write_kernel, 0 = hipStreamWriteValue64
  static int v = 1;
  return v;
}
int& sync_write_fence() {  // zs_tune("sync_write_fence"): 1 = release store, 0 = relaxed store
  static int v = 1;
  return v;
}
int& sync_wait_kernel() {  // zs_tune("sync_wait_kernel"): 1 = flag_wait_kernel, 0 = hipStreamWaitValue64
  static int v = 1;
  return v;
}

hipError_t flag_write(uint64_t* flag, uint64_t value, hipStream_t st) {
  if (sync_write_fence())
    hipLaunchKernelGGL(flag_write_kernel<true>, dim3(1), dim3(64), 0, st, flag, value);
  else
    hipLaunchKernelGGL(flag_write_kernel<false>, dim3(1), dim3(64), 0, st, flag, value);
  return hipGetLastError();
}

// the pinned host word flag_wait_kernel marks on a timeout (nullptr when pinned memory is refused)
uint32_t* wait_timeout_word() {
  static uint32_t* w = [] {
    void* p = nullptr;
    if (hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocPortable | hipHostMallocMapped) !=
        hipSuccess) {
      (void)hipGetLastError();
      return static_cast<uint32_t*>(nullptr);
    }
    *static_cast<volatile uint32_t*>(p) = 0;
    return static_cast<uint32_t*>(p);
  }();
  return w;
}

hipError_t flag_wait_launch(const uint64_t* flag, uint64_t value, hipStream_t st) {
  hipLaunchKernelGGL(flag_wait_kernel, dim3(1), dim3(64), 0, st, flag, value, wait_timeout_word());
  return hipGetLastError();
}
}  // namespace zs

extern "C" {

int zs_tune(const char* key, int64_t value, int64_t* previous) {
  ZS_REQUIRE(key != nullptr, "zs_tune: key is NULL");
  int* slot = nullptr;
  bool ok = false;
  if (std::strcmp(key, "dq_unroll") == 0) {
    slot = &dq_tune().unroll;
    ok = value == 4 || value == 8 || value == 16;
  } else if (std::strcmp(key, "dq_nt_store") == 0) {
    slot = &dq_tune().nt_store;
    ok = value == 0 || value == 1;
  } else if (std::strcmp(key, "dq_wg_per_cu") == 0) {
    slot = &dq_tune().wg_per_cu;
    ok = value >= 0 && value <= 128;
  } else if (std::strcmp(key, "scale_nt") == 0) {
    slot = &scale_nt_mode();
    ok = value >= -1 && value <= 1;
  } else if (std::strcmp(key, "convert_nt") == 0) {
    slot = &convert_nt_mode();
    ok = value >= -1 && value <= 1;
  } else if (std::strcmp(key, "copy_nt") == 0) {
    slot = &copy_nt_mode();
    ok = value >= -1 && value <= 1;
  } else if (std::strcmp(key, "adam_wg_per_cu") == 0) {
    slot = &adam_wg_per_cu();
    ok = value >= 0 && value <= 1024;
  } else if (std::strcmp(key, "sync_host_flags") == 0) {
    slot = &zs::sync_host_flags();
    ok = value == 0 || value == 1;
  } else if (std::strcmp(key, "sync_write_kernel") == 0) {
    slot = &zs::sync_write_kernel();
    ok = value == 0 || value == 1;
  } else if (std::strcmp(key, "sync_write_fence") == 0) {
    slot = &zs::sync_write_fence();
    ok = value == 0 || value == 1;
  } else if (std::strcmp(key, "sync_wait_kernel") == 0) {
    slot = &zs::sync_wait_kernel();
    ok = value == 0 || value == 1;
  } else {
    return zs::fail(ZS_ERR_INVALID, "zs_tune: unknown key '%s'", key);
  }
  ZS_REQUIRE(ok, "zs_tune: value %lld out of range for '%s'", (long long)value, key);
  if (previous) *previous = *slot;
  *slot = int(value);
  return ZS_OK;
}

int zs_device_alloc(int64_t bytes, void** out) {
  ZS_REQUIRE(out != nullptr, "zs_device_alloc: out is NULL");
  ZS_REQUIRE(bytes > 0, "zs_device_alloc: bytes must be > 0 (got %lld)", (long long)bytes);
  *out = nullptr;
  void* p = nullptr;
  const hipError_t e = hipMalloc(&p, size_t(bytes));
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();  // clear the sticky-looking error state of the runtime
    return zs::fail(ZS_ERR_NOMEM, "zs_device_alloc: %lld bytes: out of device memory",
                    (long long)bytes);
  }
  ZS_HIP(e);
  *out = p;
  return ZS_OK;
}

}  // extern "C"

namespace {
// Chunked allocations (zs_device_alloc_chunked): the physical handles behind each reserved range.
struct ChunkedAlloc {
  size_t bytes = 0;
  std::vector<hipMemGenericAllocationHandle_t> handles;
};
std::mutex g_chunked_mu;
std::map<void*, ChunkedAlloc> g_chunked;

void chunked_release(void* p, ChunkedAlloc& a) {  // (every chunk of a live range is mapped)
  (void)hipMemUnmap(p, a.bytes);
  for (auto h : a.handles) (void)hipMemRelease(h);
  (void)hipMemAddressFree(p, a.bytes);
}
}  // namespace

extern "C" {

int zs_device_alloc_chunked(int64_t bytes, int64_t chunk_bytes, void** out) {
  ZS_REQUIRE(out != nullptr, "zs_device_alloc_chunked: out is NULL");
  ZS_REQUIRE(bytes > 0 && chunk_bytes > 0, "zs_device_alloc_chunked: bytes and chunk_bytes must be > 0");
  *out = nullptr;
  int dev = 0;
  ZS_HIP(hipGetDevice(&dev));
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  ZS_HIP(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  ZS_REQUIRE(gran > 0 && size_t(chunk_bytes) % gran == 0,
             "zs_device_alloc_chunked: chunk_bytes %lld is not a multiple of the granularity %zu",
             (long long)chunk_bytes, gran);
  const size_t chunk = size_t(chunk_bytes);
  const size_t total = (size_t(bytes) + chunk - 1) / chunk * chunk;
  ChunkedAlloc a;
  a.bytes = total;
  void* p = nullptr;
  hipError_t e = hipMemAddressReserve(&p, total, 0, nullptr, 0);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return zs::fail(ZS_ERR_HIP, "zs_device_alloc_chunked: hipMemAddressReserve(%zu): %s", total,
                    hipGetErrorString(e));
  }
  for (size_t off = 0; off < total && e == hipSuccess; off += chunk) {
    hipMemGenericAllocationHandle_t h;
    e = hipMemCreate(&h, chunk, &prop, 0);
    if (e != hipSuccess) break;
    e = hipMemMap(static_cast<char*>(p) + off, chunk, 0, h, 0);
    if (e != hipSuccess) {
      (void)hipMemRelease(h);
      break;
    }
    a.handles.push_back(h);
  }
  if (e == hipSuccess) {
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    e = hipMemSetAccess(p, total, &acc, 1);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    const size_t n = a.handles.size();
    if (n) (void)hipMemUnmap(p, n * chunk);
    for (auto h : a.handles) (void)hipMemRelease(h);
    (void)hipMemAddressFree(p, total);
    (void)hipGetLastError();
    return zs::fail(e == hipErrorOutOfMemory ? ZS_ERR_NOMEM : ZS_ERR_HIP,
                    "zs_device_alloc_chunked: %lld bytes in %lld-byte chunks: %s", (long long)bytes,
                    (long long)chunk_bytes, hipGetErrorString(e));
  }
  {
    std::lock_guard<std::mutex> lk(g_chunked_mu);
    g_chunked[p] = std::move(a);
  }
  *out = p;
  return ZS_OK;
}

int zs_device_free(void* p) {
  if (p == nullptr) return ZS_OK;
  {
    std::unique_lock<std::mutex> lk(g_chunked_mu);
    auto it = g_chunked.find(p);
    if (it != g_chunked.end()) {
      ChunkedAlloc a = std::move(it->second);
      g_chunked.erase(it);
      lk.unlock();
      // hipFree waits for the device; an unmap does not: no queued work may still use the range
      ZS_HIP(hipDeviceSynchronize());
      chunked_release(p, a);
      return ZS_OK;
    }
  }
  ZS_HIP(hipFree(p));
  return ZS_OK;
}

}  // extern "C"
