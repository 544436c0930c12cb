// Dev tool: for several fresh allocations of the Adam streams (older ones kept alive so each trial
// gets new memory), time the same fused update at different grid sizes.  Question: is the
// allocation-dependent slowdown (profiles/r01_alloc_probe.log) sensitive to how far apart the
// concurrently active chunks are (i.e. TLB reach), which the grid size controls?
// hipcc --offload-arch=gfx950 -O3 tools/alloc_grid.hip -o tools/alloc_grid
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) {                                                                     \
      printf("%s failed: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__);                 \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned short bf(float f) {
  __bf16 h = static_cast<__bf16>(f);
  unsigned short r;
  __builtin_memcpy(&r, &h, 2);
  return r;
}

// same access pattern as the library kernel: 2 x 16-B groups per thread, nt loads/stores,
// grid-stride over 2048-element chunks
__global__ __launch_bounds__(256) void adam(const unsigned short* g, float* p, float* m, float* v,
                                            unsigned short* po, long n) {
  const long chunk = 2048, nch = n / chunk;
  for (long c = blockIdx.x; c < nch; c += gridDim.x) {
    u4 pp[2], mm[2], vv[2];
    u2 gg[2];
    for (int u = 0; u < 2; ++u) {
      const long i = c * chunk + (long(u) * 256 + threadIdx.x) * 4;
      gg[u] = __builtin_nontemporal_load(reinterpret_cast<const u2*>(g + i));
      pp[u] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(p + i));
      mm[u] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(m + i));
      vv[u] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(v + i));
    }
    for (int u = 0; u < 2; ++u) {
      const long i = c * chunk + (long(u) * 256 + threadIdx.x) * 4;
      u2 o;
      unsigned short h[4];
      for (int j = 0; j < 4; ++j) {
        float gf = __uint_as_float(j & 1 ? (gg[u][j / 2] & 0xffff0000u) : (gg[u][j / 2] << 16));
        float a = __uint_as_float(pp[u][j]), b = __uint_as_float(mm[u][j]), q = __uint_as_float(vv[u][j]);
        b = fmaf(0.1f, gf - b, b);
        q = fmaf(0.001f * gf, gf, q * 0.999f);
        a = a + (-1e-3f * b) / (sqrtf(q) / 0.03f + 1e-8f);
        pp[u][j] = __float_as_uint(a);
        mm[u][j] = __float_as_uint(b);
        vv[u][j] = __float_as_uint(q);
        h[j] = bf(a);
      }
      o.x = h[0] | (unsigned(h[1]) << 16);
      o.y = h[2] | (unsigned(h[3]) << 16);
      __builtin_nontemporal_store(pp[u], reinterpret_cast<u4*>(p + i));
      __builtin_nontemporal_store(mm[u], reinterpret_cast<u4*>(m + i));
      __builtin_nontemporal_store(vv[u], reinterpret_cast<u4*>(v + i));
      __builtin_nontemporal_store(o, reinterpret_cast<u2*>(po + i));
    }
  }
}

int main(int argc, char** argv) {
  const long n = 3075276800L;
  const int trials = argc > 1 ? atoi(argv[1]) : 4;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int t = 0; t < trials; ++t) {
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
    printf("trial %d:", t);
    for (int per_cu : {8, 32, 128}) {
      const int grid = cus * per_cu;
      adam<<<grid, 256>>>(g, p, m, v, po, n);
      CK(hipEventRecord(a, 0));
      for (int r = 0; r < 5; ++r) adam<<<grid, 256>>>(g, p, m, v, po, n);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= 5;
      printf("  %3d/CU %7.3f ms %6.0f GB/s", per_cu, ms, 28.0 * n / ms / 1e6);
    }
    printf("\n");
    fflush(stdout);
    if (t % 2 == 1) {  // free every other trial's buffers: later trials reuse a mix
      CK(hipFree(g));
      CK(hipFree(po));
      CK(hipFree(p));
      CK(hipFree(m));
      CK(hipFree(v));
    }
  }
  return 0;
}
