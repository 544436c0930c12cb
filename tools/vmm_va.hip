// Is streaming bandwidth a property of the VIRTUAL address range? (placement study)
//
// One physical handle of `gib` GiB (hipMemCreate) is mapped, in turn, at offsets 0, step, 2*step,
// ... of one large reserved virtual range (hipMemAddressReserve of `span_gib`), and an in-place
// 16-byte streaming pass (read + write every byte) is timed at each offset: the physical memory
// is the same every time, only the virtual address changes.  Then `copies` further handles are
// mapped side by side at the start of a second reservation and timed one by one.
//
//   hipcc --offload-arch=gfx950 -O3 tools/vmm_va.hip -o tools/vmm_va
//   tools/vmm_va <gib> <span_gib> <step_gib> <copies>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) stream_inplace(u32x4* p, size_t n, unsigned key) {
  size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x;
  size_t stride = size_t(gridDim.x) * blockDim.x;
  for (; i < n; i += stride) {
    u32x4 v = __builtin_nontemporal_load(p + i);
    v ^= key;
    __builtin_nontemporal_store(v, p + i);
  }
}

static double time_pass(void* ptr, size_t bytes, hipStream_t st, int reps) {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  dim3 grid(cus * 64), block(256);
  size_t n = bytes / 16;
  hipLaunchKernelGGL(stream_inplace, grid, block, 0, st, (u32x4*)ptr, n, 0u);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, st));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(stream_inplace, grid, block, 0, st, (u32x4*)ptr, n, 0u);
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 2.0 * bytes * reps / (ms / 1e3) / 1e9;
}

int main(int argc, char** argv) {
  size_t bytes = size_t(argc > 1 ? std::atoll(argv[1]) : 8) << 30;
  size_t span = size_t(argc > 2 ? std::atoll(argv[2]) : 128) << 30;
  size_t step = size_t(argc > 3 ? std::atoll(argv[3]) : 8) << 30;
  int copies = argc > 4 ? std::atoi(argv[4]) : 8;
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipMemAllocationProp pr = {};
  pr.type = hipMemAllocationTypePinned;
  pr.location.type = hipMemLocationTypeDevice;
  pr.location.id = 0;
  hipMemAccessDesc acc = {};
  acc.location = pr.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;

  hipMemGenericAllocationHandle_t h;
  CK(hipMemCreate(&h, bytes, &pr, 0));
  void* base = nullptr;
  CK(hipMemAddressReserve(&base, span, size_t(1) << 30, nullptr, 0));
  for (size_t off = 0; off + bytes <= span; off += step) {
    void* p = (char*)base + off;
    CK(hipMemMap(p, bytes, 0, h, 0));
    CK(hipMemSetAccess(p, bytes, &acc, 1));
    double g = time_pass(p, bytes, st, 5);
    CK(hipStreamSynchronize(st));
    std::printf("{\"same_physical\": true, \"va_off_gib\": %zu, \"va_mod_1g_mib\": %zu, \"gbs\": %.1f}\n",
                off >> 30, ((size_t)p % (size_t(1) << 30)) >> 20, g);
    std::fflush(stdout);
    CK(hipMemUnmap(p, bytes));
  }
  CK(hipMemAddressFree(base, span));
  CK(hipMemRelease(h));

  // different physical handles side by side in one reservation
  std::vector<hipMemGenericAllocationHandle_t> hs(copies);
  void* b2 = nullptr;
  CK(hipMemAddressReserve(&b2, bytes * copies, size_t(1) << 30, nullptr, 0));
  for (int k = 0; k < copies; ++k) {
    CK(hipMemCreate(&hs[k], bytes, &pr, 0));
    CK(hipMemMap((char*)b2 + k * bytes, bytes, 0, hs[k], 0));
  }
  CK(hipMemSetAccess(b2, bytes * copies, &acc, 1));
  for (int k = 0; k < copies; ++k) {
    double g = time_pass((char*)b2 + k * bytes, bytes, st, 5);
    std::printf("{\"same_physical\": false, \"handle\": %d, \"va_off_gib\": %zu, \"gbs\": %.1f}\n", k,
                (k * bytes) >> 30, g);
    std::fflush(stdout);
  }
  CK(hipStreamSynchronize(st));
  CK(hipMemUnmap(b2, bytes * copies));
  for (auto x : hs) CK(hipMemRelease(x));
  CK(hipMemAddressFree(b2, bytes * copies));
  CK(hipStreamDestroy(st));
  return 0;
}
