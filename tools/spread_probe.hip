// Dev tool: does the streaming bandwidth of a "slow" allocation depend on how far apart the
// chunks that are in flight at the same time lie?  The library kernels sweep a buffer linearly
// (chunk c = blockIdx.x + k * gridDim.x), so at any moment the ~32K resident workgroups work on one
// contiguous window of the buffer.  Mode P splits the buffer into P equal parts and deals the
// workgroups round-robin over them, so the in-flight chunks are spread over P distant regions.
// An in-place 16-B non-temporal copy (read + write, the Adam traffic mix) is timed for each mode on
// successive fresh allocations (earlier ones kept, so each is new memory), interleaved.
// hipcc --offload-arch=gfx950 -O3 tools/spread_probe.hip -o tools/spread_probe
// usage: tools/spread_probe [GiB per buffer] [allocations] [reps]
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

// 4096-byte... chunks of 4 x 16-B groups per thread (256 threads): 16 KiB per chunk
__global__ __launch_bounds__(256) void copy_spread(u4* buf, long nch, int parts) {
  const long per = nch / parts;                 // chunks per part (nch % parts handled below)
  const long wg_per_part = gridDim.x / parts;   // grid is a multiple of parts
  const int part = blockIdx.x % parts;
  const long w = blockIdx.x / parts;
  const long base = part * per;
  const long end = (part == parts - 1) ? nch : base + per;
  for (long c = base + w; c < end; c += wg_per_part) {
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
  const double gib = argc > 1 ? atof(argv[1]) : 8.0;
  const int nalloc = argc > 2 ? atoi(argv[2]) : 12;
  const int reps = argc > 3 ? atoi(argv[3]) : 3;
  const size_t bytes = size_t(gib * (1ull << 30)) / (16384) * 16384;
  const long nch = long(bytes / 16384);
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int modes[] = {1, 2, 8, 32, 256};
  const int grid = 128 * cus;  // multiple of every mode
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<void*> keep;
  printf("{\"gib\": %.2f, \"cus\": %d, \"grid\": %d}\n", gib, cus, grid);
  for (int a = 0; a < nalloc; ++a) {
    void* b = nullptr;
    if (hipMalloc(&b, bytes) != hipSuccess) break;
    keep.push_back(b);
    CK(hipMemset(b, 0, bytes));
    printf("{\"alloc\": %d", a);
    for (int mi = 0; mi < 5; ++mi) {
      const int parts = modes[mi];
      copy_spread<<<grid, 256>>>(static_cast<u4*>(b), nch, parts);  // warm
      float best = 1e30f;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        copy_spread<<<grid, 256>>>(static_cast<u4*>(b), nch, parts);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      printf(", \"p%d\": %.1f", parts, 2.0 * bytes / (best / 1e3) / 1e9);
    }
    printf("}\n");
    fflush(stdout);
  }
  for (void* b : keep) CK(hipFree(b));
  return 0;
}
