// Microbenchmark: HBM read path ceilings on gfx950 — ordinary 16-B vector loads vs LDS-DMA
// (global_load_lds_dwordx4, "glds") — for read-only and copy streams, to decide whether the fused
// Adam's five read streams could go faster through LDS.  Dev tool only:
//   hipcc --offload-arch=gfx950 -O3 tools/glds_probe.hip -o tools/glds_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("%s failed: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const void* gcptr;
typedef __attribute__((address_space(3))) void* lptr;

constexpr int kT = 256;  // threads per workgroup (4 waves)

__global__ __launch_bounds__(kT) void read_nt(const float* __restrict__ a, float* out, long n) {
  f4 acc = {0, 0, 0, 0};
  for (long i = (long(blockIdx.x) * kT + threadIdx.x) * 4; i < n; i += long(gridDim.x) * kT * 4)
    acc += __builtin_nontemporal_load(reinterpret_cast<const f4*>(a + i));
  if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
}

__global__ __launch_bounds__(kT) void copy_nt(const float* __restrict__ a, float* __restrict__ b,
                                              long n) {
  for (long i = (long(blockIdx.x) * kT + threadIdx.x) * 4; i < n; i += long(gridDim.x) * kT * 4)
    __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const f4*>(a + i)),
                                reinterpret_cast<f4*>(b + i));
}

// B glds per wave in flight: each wave owns B KiB of LDS; a workgroup step covers kT*4*B floats.
template <int B, int AUX, bool COPY>
__global__ __launch_bounds__(kT) void glds_stream(const float* __restrict__ a, float* __restrict__ b,
                                                  float* out, long n) {
  __shared__ f4 lds[kT * B];  // 4 waves x B slots x 64 lanes x 16 B
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  f4 acc = {0, 0, 0, 0};
  const long step = long(kT) * 4 * B;
  for (long base = long(blockIdx.x) * step; base < n; base += long(gridDim.x) * step) {
#pragma unroll
    for (int k = 0; k < B; ++k) {
      // slot k of this wave: 64 lanes x 16 B contiguous in global and in LDS
      const long i = base + (long(k) * kT + wave * 64 + lane) * 4;
      __builtin_amdgcn_global_load_lds((gcptr)(a + i), (lptr)&lds[(wave * B + k) * 64], 16, 0, AUX);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0); expcnt, lgkmcnt at max (no wait)
#pragma unroll
    for (int k = 0; k < B; ++k) {
      const f4 x = lds[(wave * B + k) * 64 + lane];
      const long i = base + (long(k) * kT + wave * 64 + lane) * 4;
      if constexpr (COPY) __builtin_nontemporal_store(x, reinterpret_cast<f4*>(b + i));
      else acc += x;
    }
  }
  if (!COPY && acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
}

template <typename F>
float time_ms(F f, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  f();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0, 0));
    f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  CK(hipGetLastError());
  return best;
}

template <int B, int AUX>
void run_glds(const float* a, float* b, float* out, long n, int cus) {
  for (int per_cu : {2, 8, 32}) {
    const int grid = cus * per_cu;
    float ms = time_ms([&] { glds_stream<B, AUX, false><<<grid, kT>>>(a, b, out, n); }, 5);
    printf("glds read  B=%d aux=%d grid=%6d %8.3f ms %7.1f GB/s\n", B, AUX, grid, ms, 4.0 * n / ms / 1e6);
    ms = time_ms([&] { glds_stream<B, AUX, true><<<grid, kT>>>(a, b, out, n); }, 5);
    printf("glds copy  B=%d aux=%d grid=%6d %8.3f ms %7.1f GB/s\n", B, AUX, grid, ms, 8.0 * n / ms / 1e6);
  }
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : (4L << 30);  // floats per buffer (16 GiB)
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float *a, *b, *out;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 0, n * 4));
  CK(hipMemset(b, 0, n * 4));
  printf("CUs %d, n = %ld floats per buffer\n", cus, n);
  for (int per_cu : {8, 64}) {
    const int grid = cus * per_cu;
    float ms = time_ms([&] { read_nt<<<grid, kT>>>(a, out, n); }, 5);
    printf("vec  read  nt       grid=%6d %8.3f ms %7.1f GB/s\n", grid, ms, 4.0 * n / ms / 1e6);
    ms = time_ms([&] { copy_nt<<<grid, kT>>>(a, b, n); }, 5);
    printf("vec  copy  nt       grid=%6d %8.3f ms %7.1f GB/s\n", grid, ms, 8.0 * n / ms / 1e6);
  }
  run_glds<4, 0>(a, b, out, n, cus);
  run_glds<4, 2>(a, b, out, n, cus);
  run_glds<8, 2>(a, b, out, n, cus);
  run_glds<16, 2>(a, b, out, n, cus);
  return 0;
}
