// Is a buffer's streaming bandwidth a property of HOW it is mapped? (placement study)
//
// tools/vmm_probe showed the same physical 1-GiB chunks streaming at 5.3-5.6 TB/s mapped one per
// virtual range and at 6.2 TB/s mapped side by side into one large range.  This compares, in one
// process and interleaved over `rounds`, buffers of `gib` GiB obtained as:
//   hipmalloc — plain hipMalloc (what torch's caching allocator does);
//   vmm1      — ONE physical handle (hipMemCreate) of the whole size, mapped into one range;
//   vmmN      — `chunk_mib` physical handles mapped side by side into one reserved range.
// For each: GB/s of an in-place 16-byte streaming pass (read + write every byte) over the whole
// buffer and over an 8-GiB slice from its middle.
//
//   hipcc --offload-arch=gfx950 -O3 tools/vmm_modes.hip -o tools/vmm_modes
//   tools/vmm_modes <gib> <chunk_mib> <rounds>
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

struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
  std::vector<hipMemGenericAllocationHandle_t> h;
  bool vmm = false;
};

static hipMemAllocationProp prop() {
  hipMemAllocationProp pr = {};
  pr.type = hipMemAllocationTypePinned;
  pr.location.type = hipMemLocationTypeDevice;
  pr.location.id = 0;
  return pr;
}

static Buf make(const char* mode, size_t bytes, size_t chunk) {
  Buf b;
  b.bytes = bytes;
  if (mode[0] == 'h') {
    CK(hipMalloc(&b.p, bytes));
    return b;
  }
  b.vmm = true;
  hipMemAllocationProp pr = prop();
  size_t piece = mode[3] == '1' ? bytes : chunk;
  CK(hipMemAddressReserve(&b.p, bytes, 0, nullptr, 0));
  for (size_t off = 0; off < bytes; off += piece) {
    hipMemGenericAllocationHandle_t hh;
    CK(hipMemCreate(&hh, piece, &pr, 0));
    CK(hipMemMap((char*)b.p + off, piece, 0, hh, 0));
    b.h.push_back(hh);
  }
  hipMemAccessDesc acc = {};
  acc.location = pr.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(b.p, bytes, &acc, 1));
  return b;
}

static void drop(Buf& b) {
  CK(hipDeviceSynchronize());
  if (!b.vmm) {
    CK(hipFree(b.p));
    return;
  }
  CK(hipMemUnmap(b.p, b.bytes));
  for (auto hh : b.h) CK(hipMemRelease(hh));
  CK(hipMemAddressFree(b.p, b.bytes));
}

int main(int argc, char** argv) {
  size_t bytes = size_t(argc > 1 ? std::atoll(argv[1]) : 40) << 30;
  size_t chunk = size_t(argc > 2 ? std::atoll(argv[2]) : 1024) << 20;
  int rounds = argc > 3 ? std::atoi(argv[3]) : 3;
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  size_t slice = size_t(8) << 30;
  const char* modes[] = {"hipmalloc", "vmm1", "vmmN"};
  for (int r = 0; r < rounds; ++r) {
    for (const char* m : modes) {
      Buf b = make(m, bytes, chunk);
      CK(hipMemsetAsync(b.p, 0, bytes, st));
      double whole = time_pass(b.p, bytes, st, 5);
      size_t mid = (bytes / 2 - slice / 2) / (size_t(2) << 20) * (size_t(2) << 20);
      double part = slice <= bytes ? time_pass((char*)b.p + mid, slice, st, 10) : 0.0;
      std::printf("{\"round\": %d, \"mode\": \"%s\", \"gib\": %zu, \"chunk_mib\": %zu, \"whole_gbs\": %.1f, "
                  "\"mid8g_gbs\": %.1f, \"va_mod_1g_mib\": %zu}\n",
                  r, m, bytes >> 30, chunk >> 20, whole, part, ((size_t)b.p % (size_t(1) << 30)) >> 20);
      std::fflush(stdout);
      drop(b);
    }
  }
  CK(hipStreamDestroy(st));
  return 0;
}
