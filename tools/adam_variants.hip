// Microbenchmark: memory-access variants of the fused Adam update at C4 scale (3.075e9 elems,
// bf16 grads/params + fp32 master/m/v = 28 B/elem) plus copy / read roofline calibrations.
// Dev tool only (not part of the library): hipcc --offload-arch=gfx950 -O3 tools/adam_variants.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("%s failed: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__);        \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u2 __attribute__((ext_vector_type(2)));

struct HP {
  float omb1, beta2, omb2, neg_step, bc2_sqrt, eps;
};

template <bool NT>
__device__ __forceinline__ f4 ld4(const float* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
  else return *reinterpret_cast<const f4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st4(float* p, f4 x) {
  if constexpr (NT) __builtin_nontemporal_store(x, reinterpret_cast<f4*>(p));
  else *reinterpret_cast<f4*>(p) = x;
}
template <bool NT>
__device__ __forceinline__ u2 ld2(const unsigned short* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u2*>(p));
  else return *reinterpret_cast<const u2*>(p);
}
template <bool NT>
__device__ __forceinline__ void st2(unsigned short* p, u2 x) {
  if constexpr (NT) __builtin_nontemporal_store(x, reinterpret_cast<u2*>(p));
  else *reinterpret_cast<u2*>(p) = x;
}

__device__ __forceinline__ unsigned short bf(float f) {
  __bf16 h = static_cast<__bf16>(f);
  unsigned short r;
  __builtin_memcpy(&r, &h, 2);
  return r;
}

__device__ __forceinline__ void elem(float g, float& p, float& m, float& v, const HP& hp) {
#pragma clang fp contract(off)
  m = fmaf(hp.omb1, g - m, m);
  v = fmaf(hp.omb2 * g, g, v * hp.beta2);
  const float denom = sqrtf(v) / hp.bc2_sqrt + hp.eps;
  p = p + (hp.neg_step * m) / denom;
}

template <int G, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void adam_v(const unsigned short* __restrict__ g,
                                              float* __restrict__ p, float* __restrict__ m,
                                              float* __restrict__ v, unsigned short* __restrict__ po,
                                              long n, HP hp) {
  const long chunk = 256L * 4 * G;
  const long nchunks = n / chunk;  // n is a multiple of chunk in this tool
  for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
    f4 gg[G], pp[G], mm[G], vv[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long i = c * chunk + (long(u) * 256 + threadIdx.x) * 4;
      u2 r = ld2<NTL>(g + i);
      gg[u] = f4{__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u),
                 __uint_as_float(r.y << 16), __uint_as_float(r.y & 0xffff0000u)};
      pp[u] = ld4<NTL>(p + i);
      mm[u] = ld4<NTL>(m + i);
      vv[u] = ld4<NTL>(v + i);
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const long i = c * chunk + (long(u) * 256 + threadIdx.x) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a = pp[u][j], b = mm[u][j], c = vv[u][j];
        elem(gg[u][j], a, b, c, hp);
        pp[u][j] = a;
        mm[u][j] = b;
        vv[u][j] = c;
      }
      st4<NTS>(p + i, pp[u]);
      st4<NTS>(m + i, mm[u]);
      st4<NTS>(v + i, vv[u]);
      u2 r;
      r.x = unsigned(bf(pp[u][0])) | (unsigned(bf(pp[u][1])) << 16);
      r.y = unsigned(bf(pp[u][2])) | (unsigned(bf(pp[u][3])) << 16);
      st2<NTS>(po + i, r);
    }
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void copy_v(const float* __restrict__ a, float* __restrict__ b,
                                              long n) {
  for (long i = (long(blockIdx.x) * 256 + threadIdx.x) * 4; i < n; i += long(gridDim.x) * 256 * 4)
    st4<NT>(b + i, ld4<NT>(a + i));
}

__global__ __launch_bounds__(256) void read_v(const float* __restrict__ a, float* out, long n) {
  f4 acc = {0, 0, 0, 0};
  for (long i = (long(blockIdx.x) * 256 + threadIdx.x) * 4; i < n; i += long(gridDim.x) * 256 * 4)
    acc += ld4<false>(a + i);
  if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
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
  return best;
}

template <int G, bool NTL, bool NTS>
void run_adam(const char* name, unsigned short* g, float* p, float* m, float* v, unsigned short* po,
              long n, int cus) {
  HP hp{0.1f, 0.999f, 0.001f, -1e-3f, 0.03f, 1e-8f};
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, adam_v<G, NTL, NTS>, 256, 0));
  const long nchunks = n / (256L * 4 * G);
  for (long mult : {4L, 8L, 16L, 64L, 0L}) {  // 0 = one workgroup per chunk (non-persistent)
    const int grid = int(mult ? std::min<long>(cus * occ * mult, nchunks) : nchunks);
    float ms = time_ms([&] { adam_v<G, NTL, NTS><<<grid, 256>>>(g, p, m, v, po, n, hp); }, 5);
    printf("adam %-12s G=%d occ=%d grid=%6d  %8.3f ms  %7.1f GB/s\n", name, G, occ, grid, ms,
           28.0 * n / ms / 1e6);
  }
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 3075276800L;  // C4 rounded to 16384 multiples
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  printf("CUs %d, n = %ld elements (%.1f GB algorithmic per Adam step)\n", cus, n, 28.0 * n / 1e9);
  unsigned short *g, *po;
  float *p, *m, *v;
  CK(hipMalloc(&g, n * 2));
  CK(hipMalloc(&po, n * 2));
  CK(hipMalloc(&p, n * 4));
  CK(hipMalloc(&m, n * 4));
  CK(hipMalloc(&v, n * 4));
  CK(hipMemset(g, 0x3c, n * 2));
  CK(hipMemset(p, 0, n * 4));
  CK(hipMemset(m, 0, n * 4));
  CK(hipMemset(v, 0, n * 4));
  // rooflines: copy (R+W) and read-only over 4*n floats... use m -> v (n floats each)
  for (int mult : {8, 32}) {
    const int grid = cus * 8 * mult;
    float ms = time_ms([&] { copy_v<false><<<grid, 256>>>(m, v, n); }, 5);
    printf("copy  plain grid=%6d %8.3f ms %7.1f GB/s\n", grid, ms, 8.0 * n / ms / 1e6);
    ms = time_ms([&] { copy_v<true><<<grid, 256>>>(m, v, n); }, 5);
    printf("copy  nt    grid=%6d %8.3f ms %7.1f GB/s\n", grid, ms, 8.0 * n / ms / 1e6);
    ms = time_ms([&] { read_v<<<grid, 256>>>(m, v, n); }, 5);
    printf("read        grid=%6d %8.3f ms %7.1f GB/s\n", grid, ms, 4.0 * n / ms / 1e6);
  }
  run_adam<1, false, false>("plain", g, p, m, v, po, n, cus);
  run_adam<2, false, false>("plain", g, p, m, v, po, n, cus);
  run_adam<4, false, false>("plain", g, p, m, v, po, n, cus);
  run_adam<2, true, true>("nt-ld-st", g, p, m, v, po, n, cus);
  run_adam<4, true, true>("nt-ld-st", g, p, m, v, po, n, cus);
  run_adam<2, false, true>("nt-st", g, p, m, v, po, n, cus);
  return 0;
}
