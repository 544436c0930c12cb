// Microbenchmark: the C4 fused Adam with the fp32 master stored as (bf16 param, 16-bit residual)
// instead of a separate fp32 array next to the bf16 param: 26 instead of 28 B/elem (reads g 2 +
// hi 2 + lo 2 + m 4 + v 4, writes hi 2 + lo 2 + m 4 + v 4).  Same arithmetic; the residual
// encoding itself is tested in the library, this only times the access pattern.
// Dev tool only: hipcc --offload-arch=gfx950 -O3 tools/adam_split.hip -o tools/adam_split
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("%s failed: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u2 __attribute__((ext_vector_type(2)));

struct HP {
  float omb1, beta2, omb2, neg_step, bc2_sqrt, eps;
};

__device__ __forceinline__ f4 ld4(const float* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
}
__device__ __forceinline__ void st4(float* p, f4 x) {
  __builtin_nontemporal_store(x, reinterpret_cast<f4*>(p));
}
__device__ __forceinline__ u2 ld2(const unsigned short* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u2*>(p));
}
__device__ __forceinline__ void st2(unsigned short* p, u2 x) {
  __builtin_nontemporal_store(x, reinterpret_cast<u2*>(p));
}
__device__ __forceinline__ unsigned short bf(float f) {
  __bf16 h = static_cast<__bf16>(f);
  unsigned short r;
  __builtin_memcpy(&r, &h, 2);
  return r;
}
__device__ __forceinline__ f4 unbf(u2 r) {
  return f4{__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
            __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u)};
}
__device__ __forceinline__ u2 tobf(f4 p) {
  u2 r;
  r.x = unsigned(bf(p[0])) | (unsigned(bf(p[1])) << 16);
  r.y = unsigned(bf(p[2])) | (unsigned(bf(p[3])) << 16);
  return r;
}
__device__ __forceinline__ void elem4(f4 g, f4& p, f4& m, f4& v, const HP& hp) {
#pragma clang fp contract(off)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m[j] = fmaf(hp.omb1, g[j] - m[j], m[j]);
    v[j] = fmaf(hp.omb2 * g[j], g[j], v[j] * hp.beta2);
    const float denom = sqrtf(v[j]) / hp.bc2_sqrt + hp.eps;
    p[j] = p[j] + (hp.neg_step * m[j]) / denom;
  }
}

// SoA: the library's layout (separate master / m / v arrays)
template <int G>
__global__ __launch_bounds__(256) void adam_soa(const unsigned short* __restrict__ g,
                                                float* __restrict__ p, float* __restrict__ m,
                                                float* __restrict__ v,
                                                unsigned short* __restrict__ po, long n, HP hp) {
  const long chunk = 256L * 4 * G;
  const long nchunks = n / chunk;
  for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
    f4 gg[G], pp[G], mm[G], vv[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long i = c * chunk + (long(u) * 256 + threadIdx.x) * 4;
      gg[u] = unbf(ld2(g + i));
      pp[u] = ld4(p + i);
      mm[u] = ld4(m + i);
      vv[u] = ld4(v + i);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long i = c * chunk + (long(u) * 256 + threadIdx.x) * 4;
      elem4(gg[u], pp[u], mm[u], vv[u], hp);
      st4(p + i, pp[u]);
      st4(m + i, mm[u]);
      st4(v + i, vv[u]);
      st2(po + i, tobf(pp[u]));
    }
  }
}


// split master: u = fp32 bits of the master, hi = RNE bf16 (the param), lo = int16(u - hi<<16)
__device__ __forceinline__ f4 join(u2 hi, u2 lo) {
  f4 r;
  r[0] = __uint_as_float((hi.x << 16) + int(short(lo.x & 0xffff)));
  r[1] = __uint_as_float((hi.x & 0xffff0000u) + int(short(lo.x >> 16)));
  r[2] = __uint_as_float((hi.y << 16) + int(short(lo.y & 0xffff)));
  r[3] = __uint_as_float((hi.y & 0xffff0000u) + int(short(lo.y >> 16)));
  return r;
}
__device__ __forceinline__ void split(f4 p, u2& hi, u2& lo) {
  hi = tobf(p);
  unsigned d[4];
  d[0] = __float_as_uint(p[0]) - ((hi.x & 0xffffu) << 16);
  d[1] = __float_as_uint(p[1]) - (hi.x & 0xffff0000u);
  d[2] = __float_as_uint(p[2]) - ((hi.y & 0xffffu) << 16);
  d[3] = __float_as_uint(p[3]) - (hi.y & 0xffff0000u);
  lo.x = (d[0] & 0xffffu) | (d[1] << 16);
  lo.y = (d[2] & 0xffffu) | (d[3] << 16);
}

template <int G>
__global__ __launch_bounds__(256) void adam_split(const unsigned short* __restrict__ g,
                                                  unsigned short* __restrict__ hi,
                                                  unsigned short* __restrict__ lo,
                                                  float* __restrict__ m, float* __restrict__ v,
                                                  long n, HP hp) {
  const long chunk = 256L * 4 * G;
  const long nchunks = n / chunk;
  for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
    f4 gg[G], pp[G], mm[G], vv[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long i = c * chunk + (long(u) * 256 + threadIdx.x) * 4;
      gg[u] = unbf(ld2(g + i));
      pp[u] = join(ld2(hi + i), ld2(lo + i));
      mm[u] = ld4(m + i);
      vv[u] = ld4(v + i);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long i = c * chunk + (long(u) * 256 + threadIdx.x) * 4;
      elem4(gg[u], pp[u], mm[u], vv[u], hp);
      u2 h, l;
      split(pp[u], h, l);
      st2(hi + i, h);
      st2(lo + i, l);
      st4(m + i, mm[u]);
      st4(v + i, vv[u]);
    }
  }
}

// 8 consecutive elements per lane and group: the three 2-byte streams move 16 B per lane (1 KiB
// per wave instruction, like the fp32 streams' float4), the fp32 streams two float4 per lane.
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u4 ld16(const unsigned short* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u4*>(p));
}
__device__ __forceinline__ void st16(unsigned short* p, u4 x) {
  __builtin_nontemporal_store(x, reinterpret_cast<u4*>(p));
}
template <int G>
__global__ __launch_bounds__(256) void adam_split8(const unsigned short* __restrict__ g,
                                                   unsigned short* __restrict__ hi,
                                                   unsigned short* __restrict__ lo,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   long n, HP hp) {
  const long chunk = 256L * 8 * G;
  const long nchunks = n / chunk;
  for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
    u4 gg[G], hh[G], ll[G];
    f4 m0[G], m1[G], v0[G], v1[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long i = c * chunk + (long(u) * 256 + threadIdx.x) * 8;
      gg[u] = ld16(g + i);
      hh[u] = ld16(hi + i);
      ll[u] = ld16(lo + i);
      m0[u] = ld4(m + i);
      m1[u] = ld4(m + i + 4);
      v0[u] = ld4(v + i);
      v1[u] = ld4(v + i + 4);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long i = c * chunk + (long(u) * 256 + threadIdx.x) * 8;
      f4 g0 = unbf(u2{gg[u].x, gg[u].y}), g1 = unbf(u2{gg[u].z, gg[u].w});
      f4 p0 = join(u2{hh[u].x, hh[u].y}, u2{ll[u].x, ll[u].y});
      f4 p1 = join(u2{hh[u].z, hh[u].w}, u2{ll[u].z, ll[u].w});
      elem4(g0, p0, m0[u], v0[u], hp);
      elem4(g1, p1, m1[u], v1[u], hp);
      u2 h0, l0, h1, l1;
      split(p0, h0, l0);
      split(p1, h1, l1);
      st16(hi + i, u4{h0.x, h0.y, h1.x, h1.y});
      st16(lo + i, u4{l0.x, l0.y, l1.x, l1.y});
      st4(m + i, m0[u]);
      st4(m + i + 4, m1[u]);
      st4(v + i, v0[u]);
      st4(v + i + 4, v1[u]);
    }
  }
}

// 16 B per lane for the three 2-byte streams (8 consecutive elements per lane: 1 KiB per wave
// instruction) AND dense float4 accesses for m / v: the fp32 streams are loaded lane-contiguous
// (lane l: elements 4l.. of each 256-element half of the wave's 512-element span) and transposed
// through a wave-private LDS area to 8 consecutive elements per lane, and back before the stores.
template <int G>
__global__ __launch_bounds__(256) void adam_split8t(const unsigned short* __restrict__ g,
                                                    unsigned short* __restrict__ hi,
                                                    unsigned short* __restrict__ lo,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    long n, HP hp) {
  __shared__ f4 lds[4][2][128];  // per wave: m and v, 512 floats each
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  f4* lm = lds[wv][0];
  f4* lv = lds[wv][1];
  const long chunk = 256L * 8 * G;
  const long nchunks = n / chunk;
  for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
    u4 gg[G], hh[G], ll[G];
    f4 ma[G], mb[G], va[G], vb[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {  // every load first
      const long base = c * chunk + long(u * 4 + wv) * 512;
      gg[u] = ld16(g + base + 8 * lane);
      hh[u] = ld16(hi + base + 8 * lane);
      ll[u] = ld16(lo + base + 8 * lane);
      ma[u] = ld4(m + base + 4 * lane);
      mb[u] = ld4(m + base + 256 + 4 * lane);
      va[u] = ld4(v + base + 4 * lane);
      vb[u] = ld4(v + base + 256 + 4 * lane);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long base = c * chunk + long(u * 4 + wv) * 512;
      lm[lane] = ma[u];
      lm[64 + lane] = mb[u];
      lv[lane] = va[u];
      lv[64 + lane] = vb[u];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      f4 m0 = lm[2 * lane], m1 = lm[2 * lane + 1], v0 = lv[2 * lane], v1 = lv[2 * lane + 1];
      f4 g0 = unbf(u2{gg[u].x, gg[u].y}), g1 = unbf(u2{gg[u].z, gg[u].w});
      f4 p0 = join(u2{hh[u].x, hh[u].y}, u2{ll[u].x, ll[u].y});
      f4 p1 = join(u2{hh[u].z, hh[u].w}, u2{ll[u].z, ll[u].w});
      elem4(g0, p0, m0, v0, hp);
      elem4(g1, p1, m1, v1, hp);
      u2 h0, l0, h1, l1;
      split(p0, h0, l0);
      split(p1, h1, l1);
      st16(hi + base + 8 * lane, u4{h0.x, h0.y, h1.x, h1.y});
      st16(lo + base + 8 * lane, u4{l0.x, l0.y, l1.x, l1.y});
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      lm[2 * lane] = m0;
      lm[2 * lane + 1] = m1;
      lv[2 * lane] = v0;
      lv[2 * lane + 1] = v1;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      st4(m + base + 4 * lane, lm[lane]);
      st4(m + base + 256 + 4 * lane, lm[64 + lane]);
      st4(v + base + 4 * lane, lv[lane]);
      st4(v + base + 256 + 4 * lane, lv[64 + lane]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

__global__ __launch_bounds__(256) void copy_nt(const float* __restrict__ a, float* __restrict__ b,
                                               long n) {
  for (long i = (long(blockIdx.x) * 256 + threadIdx.x) * 4; i < n; i += long(gridDim.x) * 256 * 4)
    st4(b + i, ld4(a + i));
}

template <typename F>
float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a, 0));
    f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  CK(hipGetLastError());
  return best;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 3075276800L;  // C4, a multiple of 256*4*4
  const int rounds = argc > 2 ? atoi(argv[2]) : 2;
  const int allocs = argc > 3 ? atoi(argv[3]) : 3;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 128;
  printf("CUs %d, n = %ld, grid %d\n", cus, n, grid);
  unsigned short *g, *po;
  CK(hipMalloc(&g, n * 2));
  CK(hipMalloc(&po, n * 2));  // the bf16 param (= hi of the split master)
  CK(hipMemset(g, 0x3c, n * 2));
  CK(hipMemset(po, 0, n * 2));
  HP hp{0.1f, 0.999f, 0.001f, -1e-3f, 0.03f, 1e-8f};
  // the same 12 B/elem state allocation serves both: SoA master | m | v, split lo | m | v
  for (int a = 0; a < allocs; ++a) {
    float* s;
    CK(hipMalloc(&s, n * 12));
    CK(hipMemset(s, 0, n * 12));
    float *p = s, *m = s + n, *v = s + 2 * n;
    unsigned short* lo = reinterpret_cast<unsigned short*>(s);
    for (int r = 0; r < rounds; ++r) {
      float ms = time_ms([&] { adam_soa<2><<<grid, 256>>>(g, p, m, v, po, n, hp); }, 5);
      printf("alloc %d round %d adam fp32-master  28 B %8.3f ms %7.1f GB/s %.4g elem/s\n", a, r, ms,
             28.0 * n / ms / 1e6, n / ms * 1e3);
      ms = time_ms([&] { adam_split<2><<<grid, 256>>>(g, po, lo, m, v, n, hp); }, 5);
      printf("alloc %d round %d adam split-master 26 B %8.3f ms %7.1f GB/s %.4g elem/s\n", a, r, ms,
             26.0 * n / ms / 1e6, n / ms * 1e3);
      ms = time_ms([&] { adam_split<4><<<grid, 256>>>(g, po, lo, m, v, n, hp); }, 5);
      printf("alloc %d round %d adam split G=4    26 B %8.3f ms %7.1f GB/s %.4g elem/s\n", a, r, ms,
             26.0 * n / ms / 1e6, n / ms * 1e3);
      ms = time_ms([&] { adam_split8<1><<<grid, 256>>>(g, po, lo, m, v, n, hp); }, 5);
      printf("alloc %d round %d adam split8 G=1   26 B %8.3f ms %7.1f GB/s %.4g elem/s\n", a, r, ms,
             26.0 * n / ms / 1e6, n / ms * 1e3);
      ms = time_ms([&] { adam_split8<2><<<grid, 256>>>(g, po, lo, m, v, n, hp); }, 5);
      printf("alloc %d round %d adam split8 G=2   26 B %8.3f ms %7.1f GB/s %.4g elem/s\n", a, r, ms,
             26.0 * n / ms / 1e6, n / ms * 1e3);
      ms = time_ms([&] { adam_split8t<1><<<grid, 256>>>(g, po, lo, m, v, n, hp); }, 5);
      printf("alloc %d round %d adam split8t G=1  26 B %8.3f ms %7.1f GB/s %.4g elem/s\n", a, r, ms,
             26.0 * n / ms / 1e6, n / ms * 1e3);
      ms = time_ms([&] { adam_split8t<2><<<grid, 256>>>(g, po, lo, m, v, n, hp); }, 5);
      printf("alloc %d round %d adam split8t G=2  26 B %8.3f ms %7.1f GB/s %.4g elem/s\n", a, r, ms,
             26.0 * n / ms / 1e6, n / ms * 1e3);
      ms = time_ms([&] { copy_nt<<<grid, 256>>>(m, v, n); }, 5);
      printf("alloc %d round %d copy_nt           8 B %8.3f ms %7.1f GB/s\n", a, r, ms,
             8.0 * n / ms / 1e6);
    }
    // keep s allocated so the next iteration gets new memory
  }
  return 0;
}
