// Microbenchmark: does interleaving the fp32 optimizer state (array-of-structs) beat separate
// exp_avg / exp_avg_sq / master arrays for the C4 fused Adam (bf16 grad in, bf16 param out)?
// SoA = 5 read + 4 write address streams per element; AoS = 2 read + 2 write (grad, state in;
// state, param out).  Same arithmetic, same 28 B/elem, same grid policy (128 WG/CU).
// Dev tool only: hipcc --offload-arch=gfx950 -O3 tools/adam_aos.hip -o tools/adam_aos
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

// AoS: state[q] = {m[4], v[4], master[4]} for element quad q (48 B, three 16-B accesses)
template <int G>
__global__ __launch_bounds__(256) void adam_aos(const unsigned short* __restrict__ g,
                                                float* __restrict__ s,
                                                unsigned short* __restrict__ po, long n, HP hp) {
  const long chunk = 256L * 4 * G;
  const long nchunks = n / chunk;
  for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
    f4 gg[G], pp[G], mm[G], vv[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long q = c * (256L * G) + long(u) * 256 + threadIdx.x;  // element quad
      gg[u] = unbf(ld2(g + q * 4));
      mm[u] = ld4(s + q * 12);
      vv[u] = ld4(s + q * 12 + 4);
      pp[u] = ld4(s + q * 12 + 8);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long q = c * (256L * G) + long(u) * 256 + threadIdx.x;
      elem4(gg[u], pp[u], mm[u], vv[u], hp);
      st4(s + q * 12, mm[u]);
      st4(s + q * 12 + 4, vv[u]);
      st4(s + q * 12 + 8, pp[u]);
      st2(po + q * 4, tobf(pp[u]));
    }
  }
}

// AoS-T: lane-transposed blocks — a block of 256 quads stores m for all 256 quads (4 KiB), then v,
// then master, so every wave access is 1 KiB contiguous (the SoA pattern) inside one 12 KiB block
template <int G>
__global__ __launch_bounds__(256) void adam_aost(const unsigned short* __restrict__ g,
                                                 float* __restrict__ s,
                                                 unsigned short* __restrict__ po, long n, HP hp) {
  const long chunk = 256L * 4 * G;
  const long nchunks = n / chunk;
  for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
    f4 gg[G], pp[G], mm[G], vv[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long blk = c * G + u;  // 256-quad block
      float* b = s + blk * 3072;
      gg[u] = unbf(ld2(g + (blk * 256 + threadIdx.x) * 4));
      mm[u] = ld4(b + threadIdx.x * 4);
      vv[u] = ld4(b + 1024 + threadIdx.x * 4);
      pp[u] = ld4(b + 2048 + threadIdx.x * 4);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long blk = c * G + u;
      float* b = s + blk * 3072;
      elem4(gg[u], pp[u], mm[u], vv[u], hp);
      st4(b + threadIdx.x * 4, mm[u]);
      st4(b + 1024 + threadIdx.x * 4, vv[u]);
      st4(b + 2048 + threadIdx.x * 4, pp[u]);
      st2(po + (blk * 256 + threadIdx.x) * 4, tobf(pp[u]));
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
  return best;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 3075276800L;  // C4, a multiple of 256*4*4
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 128;
  printf("CUs %d, n = %ld (%.1f GB algorithmic per step), grid %d\n", cus, n, 28.0 * n / 1e9, grid);
  const int allocs = argc > 3 ? atoi(argv[3]) : 3;
  unsigned short *g, *po;
  CK(hipMalloc(&g, n * 2));
  CK(hipMalloc(&po, n * 2));
  CK(hipMemset(g, 0x3c, n * 2));
  HP hp{0.1f, 0.999f, 0.001f, -1e-3f, 0.03f, 1e-8f};
  // Every variant runs over the SAME 12 B/elem allocation (SoA: master | m | v as three arrays in
  // it, as the library's single state allocation; AoS: interleaved), and the comparison is
  // repeated on several allocations, since placement alone moves the rate by up to 20 %.
  std::vector<float*> keep;
  for (int a = 0; a < allocs; ++a) {
    float* s;
    CK(hipMalloc(&s, n * 12));
    CK(hipMemset(s, 0, n * 12));
    keep.push_back(s);
    float *p = s, *m = s + n, *v = s + 2 * n;
    for (int r = 0; r < rounds; ++r) {
      float ms = time_ms([&] { copy_nt<<<cus * 64, 256>>>(m, v, n); }, 5);
      printf("alloc %d round %d copy-nt (m->v)  %8.3f ms %7.1f GB/s\n", a, r, ms, 8.0 * n / ms / 1e6);
      ms = time_ms([&] { adam_soa<2><<<grid, 256>>>(g, p, m, v, po, n, hp); }, 5);
      printf("alloc %d round %d adam SoA  G=2   %8.3f ms %7.1f GB/s\n", a, r, ms, 28.0 * n / ms / 1e6);
      ms = time_ms([&] { adam_aos<2><<<grid, 256>>>(g, s, po, n, hp); }, 5);
      printf("alloc %d round %d adam AoS  G=2   %8.3f ms %7.1f GB/s\n", a, r, ms, 28.0 * n / ms / 1e6);
      ms = time_ms([&] { adam_aos<1><<<grid, 256>>>(g, s, po, n, hp); }, 5);
      printf("alloc %d round %d adam AoS  G=1   %8.3f ms %7.1f GB/s\n", a, r, ms, 28.0 * n / ms / 1e6);
      ms = time_ms([&] { adam_aost<2><<<grid, 256>>>(g, s, po, n, hp); }, 5);
      printf("alloc %d round %d adam AoST G=2   %8.3f ms %7.1f GB/s\n", a, r, ms, 28.0 * n / ms / 1e6);
      ms = time_ms([&] { adam_aost<4><<<grid, 256>>>(g, s, po, n, hp); }, 5);
      printf("alloc %d round %d adam AoST G=4   %8.3f ms %7.1f GB/s\n", a, r, ms, 28.0 * n / ms / 1e6);
    }
  }
  for (float* s : keep) CK(hipFree(s));
  return 0;
}
