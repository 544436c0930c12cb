// How far can the host enqueue kernel launches ahead of a busy GPU before hipLaunchKernel blocks,
// and does the depth depend on the size of the launch's kernel arguments?  (the
// default gradient hand-off's host runs ~200 steps ahead and then waits; round 5 guessed "the
// kernel-argument pool" because each step's gradient-pointer patch carries a 1,808-byte argument
// struct, zs_kernels.hip GradPatch.)
//
// Per variant: one kernel spins for `spin_ms` on the GPU, then the host launches `n` empty kernels
// whose argument struct is `bytes` long (`per_step` launches per "step": the C4 default hand-off
// step is 2 patch launches of 1,808 B + 1 Adam launch of ~100 B), timing each launch call; the
// first call that takes > 1 ms is where the host had to wait.  If the depth in launches is the same
// for every argument size, the bound is the queue (packets), not the argument pool.
//
//   hipcc --offload-arch=gfx950 -O3 tools/queue_depth_probe.hip -o tools/queue_depth_probe
//   tools/queue_depth_probe [spin_ms] [n]     -> one JSON line per variant
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

// spins for `ticks` of the 100 MHz wall clock; writes nothing
__global__ void spin(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

template <int B>
struct Args {
  unsigned char b[B];
};

// an empty kernel whose argument segment is B bytes
template <int B>
__global__ void empty_kernel(const Args<B> a) {}

template <int B>
static void variant(const char* name, hipStream_t st, double spin_ms, int n, int per_step, int small_every) {
  const unsigned long long ticks = (unsigned long long)(spin_ms * 1e5);  // 100 MHz
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st, ticks);
  Args<B> a{};
  Args<16> s{};
  int first_blocked = -1, launches = 0;
  double before_us = 0.0, max_ms = 0.0;
  for (int i = 0; i < n; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    if (small_every > 0 && i % small_every == small_every - 1)
      hipLaunchKernelGGL(empty_kernel<16>, dim3(1), dim3(64), 0, st, s);
    else
      hipLaunchKernelGGL(empty_kernel<B>, dim3(1), dim3(64), 0, st, a);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ++launches;
    if (ms > max_ms) max_ms = ms;
    if (first_blocked < 0) {
      if (ms > 1.0)
        first_blocked = i;
      else
        before_us += ms * 1e3;
    }
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const int k = first_blocked < 0 ? n : first_blocked;
  std::printf("{\"variant\": \"%s\", \"arg_bytes\": %d, \"small_every\": %d, \"launches\": %d, "
              "\"first_blocked_launch\": %d, \"first_blocked_step\": %d, \"us_per_launch_before\": %.2f, "
              "\"max_launch_ms\": %.1f, \"per_step\": %d}\n",
              name, B, small_every, launches, first_blocked, first_blocked < 0 ? -1 : first_blocked / per_step,
              k ? before_us / k : 0.0, max_ms, per_step);
  std::fflush(stdout);
}

int main(int argc, char** argv) {
  const double spin_ms = argc > 1 ? std::atof(argv[1]) : 3000.0;
  const int n = argc > 2 ? std::atoi(argv[2]) : 3000;
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (int rep = 0; rep < 2; ++rep) {
    variant<16>("args 16 B", st, spin_ms, n, 1, 0);
    variant<256>("args 256 B", st, spin_ms, n, 1, 0);
    variant<1024>("args 1 KiB", st, spin_ms, n, 1, 0);
    variant<1808>("args 1808 B (GradPatch)", st, spin_ms, n, 1, 0);
    variant<4000>("args 4000 B", st, spin_ms, n, 1, 0);
    // the default hand-off's mix: two 1808-B patch launches and one small Adam launch per step
    variant<1808>("C4 default-step mix (2 x 1808 B + 1 x 16 B)", st, spin_ms, n, 3, 3);
  }
  CK(hipStreamDestroy(st));
  return 0;
}
