// Does picking fast PHYSICAL chunks make a fast buffer? (placement study)
//
// Streaming bandwidth depends on where in VRAM an allocation lands (profiles/r02_alloc/).  This
// probe uses the HIP virtual-memory API: it creates `count` physical chunks of `chunk_mib` each
// (hipMemCreate), maps each at its own address and times an in-place 16-byte streaming pass over
// it (read + write every byte, the Adam kernel's access shape), then maps the `pick` fastest
// chunks — and, for contrast, the `pick` slowest and the first `pick` — contiguously into one
// reserved range each and times a pass over the whole range.
//
//   hipcc --offload-arch=gfx950 -O3 tools/vmm_probe.hip -o tools/vmm_probe
//   tools/vmm_probe <chunk_mib> <count> <pick> [va_align_mib]
// va_align_mib: alignment of every virtual range reserved (0 = the runtime's default).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

// in-place pass: every 16-B word read and written back XOR key (key = 0 at run time)
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
  size_t n = bytes / 16;
  dim3 grid(cus * 64), block(256);
  hipLaunchKernelGGL(stream_inplace, grid, block, 0, st, (u32x4*)ptr, n, 0u);  // warm
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
  size_t chunk = (argc > 1 ? std::atoll(argv[1]) : 1024) << 20;
  int count = argc > 2 ? std::atoi(argv[2]) : 64;
  int pick = argc > 3 ? std::atoi(argv[3]) : 16;
  size_t align = (argc > 4 ? std::atoll(argv[4]) : 0) << 20;
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gran = 0;
  CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
  chunk = (chunk + gran - 1) / gran * gran;
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  std::printf("{\"granularity\": %zu, \"chunk_bytes\": %zu, \"count\": %d, \"pick\": %d, \"va_align\": %zu}\n",
              gran, chunk, count, pick, align);
  std::vector<hipMemGenericAllocationHandle_t> h;
  std::vector<void*> va;
  std::vector<double> gbs;
  for (int k = 0; k < count; ++k) {
    size_t freeb = 0, totalb = 0;
    CK(hipMemGetInfo(&freeb, &totalb));
    if (freeb < chunk + (size_t(16) << 30)) break;  // leave room for the contiguous maps' VA only
    hipMemGenericAllocationHandle_t hh;
    if (hipMemCreate(&hh, chunk, &prop, 0) != hipSuccess) break;
    void* p = nullptr;
    CK(hipMemAddressReserve(&p, chunk, align, nullptr, 0));
    CK(hipMemMap(p, chunk, 0, hh, 0));
    CK(hipMemSetAccess(p, chunk, &acc, 1));
    CK(hipMemsetAsync(p, 0, chunk, st));
    double g = time_pass(p, chunk, st, 3);
    // one mapping per handle at a time: the contiguous maps below re-map these handles
    CK(hipStreamSynchronize(st));
    CK(hipMemUnmap(p, chunk));
    CK(hipMemAddressFree(p, chunk));
    h.push_back(hh);
    va.push_back(p);
    gbs.push_back(g);
    std::printf("{\"chunk\": %d, \"gbs\": %.1f, \"va_mod_1g\": %zu}\n", k, g,
                (size_t)p % (size_t(1) << 30));
    std::fflush(stdout);
  }
  int nchunks = int(h.size());
  pick = std::min(pick, nchunks);
  std::vector<int> order(nchunks);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int a, int b) { return gbs[a] > gbs[b]; });
  auto contiguous = [&](const char* name, std::vector<int> sel) {
    void* base = nullptr;
    size_t total = chunk * sel.size();
    CK(hipMemAddressReserve(&base, total, align, nullptr, 0));
    for (size_t j = 0; j < sel.size(); ++j)
      CK(hipMemMap((char*)base + j * chunk, chunk, 0, h[sel[j]], 0));
    CK(hipMemSetAccess(base, total, &acc, 1));
    double g = time_pass(base, total, st, 3);
    // the same mapping, passes over its first 1, 2, 4, ... GiB: pass length or placement?
    for (size_t sub = size_t(1) << 30; sub < total; sub *= 2) {
      double gs = time_pass(base, sub, st, 3);
      double gl = time_pass(base, sub, st, 30);
      std::printf("{\"contiguous\": \"%s\", \"prefix_gib\": %zu, \"gbs_3reps\": %.1f, \"gbs_30reps\": %.1f}\n",
                  name, sub >> 30, gs, gl);
    }
    double mean = 0;
    for (int s : sel) mean += gbs[s];
    mean /= sel.size();
    std::printf("{\"contiguous\": \"%s\", \"chunks\": %zu, \"gbs\": %.1f, \"mean_chunk_gbs\": %.1f, "
                "\"va_mod_1g\": %zu}\n", name, sel.size(), g, mean, (size_t)base % (size_t(1) << 30));
    std::fflush(stdout);
    CK(hipStreamSynchronize(st));
    CK(hipMemUnmap(base, total));
    CK(hipMemAddressFree(base, total));
  };
  if (pick > 0) {
    contiguous("fastest", std::vector<int>(order.begin(), order.begin() + pick));
    contiguous("slowest", std::vector<int>(order.end() - pick, order.end()));
    std::vector<int> first(pick);
    std::iota(first.begin(), first.end(), 0);
    contiguous("first", first);
  }
  // single chunks again, each at a fresh range (is a chunk's speed its own, or its mapping's?)
  for (int k = 0; k < std::min(nchunks, 8); ++k) {
    void* p = nullptr;
    CK(hipMemAddressReserve(&p, chunk, align, nullptr, 0));
    CK(hipMemMap(p, chunk, 0, h[order[k]], 0));
    CK(hipMemSetAccess(p, chunk, &acc, 1));
    double g = time_pass(p, chunk, st, 3);
    CK(hipStreamSynchronize(st));
    std::printf("{\"remap_fast_chunk\": %d, \"was_gbs\": %.1f, \"gbs\": %.1f, \"va_mod_1g\": %zu}\n", order[k],
                gbs[order[k]], g, (size_t)p % (size_t(1) << 30));
    CK(hipMemUnmap(p, chunk));
    CK(hipMemAddressFree(p, chunk));
  }
  for (int k = 0; k < nchunks; ++k) CK(hipMemRelease(h[k]));
  CK(hipStreamDestroy(st));
  return 0;
}
