// Dev tool: map streaming bandwidth against allocation order at fine granularity.  Allocates
// successive buffers of B GiB (each kept, so each is new memory) until the device is nearly full,
// times an in-place 16-B non-temporal copy over each, prints one line per buffer; then frees
// everything and repeats (does the same allocation index land in equally fast memory again?).
// hipcc --offload-arch=gfx950 -O3 tools/vram_map.hip -o tools/vram_map
// usage: tools/vram_map [GiB per buffer] [passes] [reserve GiB]
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

__global__ __launch_bounds__(256) void copy_inplace(u4* buf, long nch) {
  for (long c = blockIdx.x; c < nch; c += gridDim.x) {
    u4 x[4];
    u4* q = buf + c * 1024;
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = __builtin_nontemporal_load(q + u * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      x[u] += 1u;
      __builtin_nontemporal_store(x[u], q + u * 256 + threadIdx.x);
    }
  }
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 1.0;
  const int passes = argc > 2 ? atoi(argv[2]) : 2;
  const double reserve = argc > 3 ? atof(argv[3]) : 4.0;
  const size_t bytes = size_t(gib * (1ull << 30)) / 16384 * 16384;
  const long nch = long(bytes / 16384);
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int pass = 0; pass < passes; ++pass) {
    std::vector<void*> keep;
    printf("{\"pass\": %d, \"gib\": %.2f, \"gbs\": [", pass, gib);
    for (int a = 0;; ++a) {
      size_t fr = 0, tot = 0;
      CK(hipMemGetInfo(&fr, &tot));
      if (double(fr) < double(bytes) + reserve * double(1ull << 30)) break;
      void* b = nullptr;
      if (hipMalloc(&b, bytes) != hipSuccess) break;
      keep.push_back(b);
      copy_inplace<<<128 * cus, 256>>>(static_cast<u4*>(b), nch);  // first touch / warm
      float best = 1e30f;
      for (int r = 0; r < 2; ++r) {
        CK(hipEventRecord(e0));
        copy_inplace<<<128 * cus, 256>>>(static_cast<u4*>(b), nch);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      printf("%s%.0f", a ? ", " : "", 2.0 * bytes / (best / 1e3) / 1e9);
      fflush(stdout);
    }
    printf("]}\n");
    fflush(stdout);
    for (void* b : keep) CK(hipFree(b));
  }
  return 0;
}
