// Which cross-stream ordering makes a HIP runtime thread poll?  (round 4, ZeRO-3 host time)
//
// A bounded "busy" kernel (~T ms of s_sleep loops, one workgroup) runs on stream A; an event is
// recorded after it; stream B waits on that event (hipStreamWaitEvent) and records its own event;
// the host then waits on B's event.  For each variant the CPU time of every thread of this process
// over the span is read from /proc/self/task/<tid>/stat (utime + stime, clock ticks), so the
// runtime's own threads show up beside the main thread.  Variants: event flags (timing / disable
// timing / disable system fence), stream flags (default / non-blocking), host wait by
// hipEventSynchronize vs a hipEventQuery sleep loop, and no cross-stream wait at all.
// Round 5: stream memory operations as the ordering — hipStreamWriteValue32 of an
// epoch on stream A after the busy kernel, hipStreamWaitValue32(>= epoch) on stream B — with the
// flag word in device memory (hipMalloc), in signal memory (hipExtMallocWithFlags
// hipMallocSignalMemory) and in pinned host memory (hipHostMalloc).
//
// build: hipcc --offload-arch=gfx950 -O2 tools/event_poll_probe.hip -o tools/event_poll_probe
// run:   tools/event_poll_probe [ms]
#include <hip/hip_runtime.h>

#include <dirent.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,              \
                   hipGetErrorString(e_));                                         \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

// bounded busy kernel: `iters` rounds of s_sleep; each lane writes one word at the end
__global__ void busy_kernel(int iters, int* out) {
  for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(127);
  out[threadIdx.x] = iters + int(threadIdx.x);  // a per-lane (vector) store
}

static std::map<long, long> thread_ticks() {
  std::map<long, long> out;
  DIR* d = opendir("/proc/self/task");
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    char path[256];
    std::snprintf(path, sizeof path, "/proc/self/task/%s/stat", e->d_name);
    FILE* f = std::fopen(path, "r");
    if (!f) continue;
    char buf[2048];
    size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    // fields after the ") " of the comm: state(3) ... utime(14) stime(15)
    char* p = std::strrchr(buf, ')');
    if (!p) continue;
    long ut = 0, st = 0;
    int field = 2;
    for (char* tok = std::strtok(p + 2, " "); tok; tok = std::strtok(nullptr, " ")) {
      ++field;
      if (field == 14) ut = std::atol(tok);
      if (field == 15) {
        st = std::atol(tok);
        break;
      }
    }
    out[std::atol(e->d_name)] = ut + st;
  }
  closedir(d);
  return out;
}

enum Flag { kNoFlag = 0, kDeviceFlag, kSignalFlag, kHostFlag };

struct Variant {
  const char* name;
  unsigned ev_flags;
  unsigned st_flags;
  bool cross_wait;
  bool query_loop;
  Flag flag = kNoFlag;  // != kNoFlag: the cross-stream ordering is a write / wait of this word
};

int main(int argc, char** argv) {
  const double ms = argc > 1 ? std::atof(argv[1]) : 200.0;
  const long hz = sysconf(_SC_CLK_TCK);
  int* out = nullptr;
  CHECK(hipMalloc(&out, 64 * sizeof(int)));
  // calibrate: iterations per ms of the busy kernel
  hipStream_t s0;
  CHECK(hipStreamCreate(&s0));
  hipEvent_t c0, c1;
  CHECK(hipEventCreate(&c0));
  CHECK(hipEventCreate(&c1));
  const int probe_iters = 20000;
  hipLaunchKernelGGL(busy_kernel, dim3(1), dim3(64), 0, s0, probe_iters, out);
  CHECK(hipEventRecord(c0, s0));
  hipLaunchKernelGGL(busy_kernel, dim3(1), dim3(64), 0, s0, probe_iters, out);
  CHECK(hipEventRecord(c1, s0));
  CHECK(hipEventSynchronize(c1));
  float pms = 0;
  CHECK(hipEventElapsedTime(&pms, c0, c1));
  const int iters = int(probe_iters * ms / (pms > 0 ? pms : 1.0f));
  std::printf("{\"calibration\": {\"iters_per_ms\": %.1f, \"span_ms\": %.1f}}\n", probe_iters / pms, ms);
  const Variant vs[] = {
      {"no cross-stream wait (event sync on A)", hipEventDisableTiming, hipStreamDefault, false, false},
      {"cross wait, DisableTiming events", hipEventDisableTiming, hipStreamDefault, true, false},
      {"cross wait, timing events", hipEventDefault, hipStreamDefault, true, false},
      {"cross wait, DisableTiming|DisableSystemFence", hipEventDisableTiming | hipEventDisableSystemFence,
       hipStreamDefault, true, false},
      {"cross wait, non-blocking streams", hipEventDisableTiming, hipStreamNonBlocking, true, false},
      {"cross wait, host polls hipEventQuery + sleep", hipEventDisableTiming, hipStreamDefault, true, true},
      {"no cross wait, host polls hipEventQuery + sleep", hipEventDisableTiming, hipStreamDefault, false, true},
      {"stream write/wait value32, flag in hipMalloc memory", hipEventDisableTiming, hipStreamDefault, true,
       false, kDeviceFlag},
      {"stream write/wait value32, flag in signal memory", hipEventDisableTiming, hipStreamDefault, true,
       false, kSignalFlag},
      {"stream write/wait value32, flag in pinned host memory", hipEventDisableTiming, hipStreamDefault, true,
       false, kHostFlag},
      {"stream write/wait value32 (hipMalloc), host polls hipEventQuery + sleep", hipEventDisableTiming,
       hipStreamDefault, true, true, kDeviceFlag},
  };
  // the flag words (one per kind); epochs only grow, so a wait never sees a stale value as done
  uint32_t* flags[4] = {nullptr, nullptr, nullptr, nullptr};
  CHECK(hipMalloc(&flags[kDeviceFlag], 64));
  CHECK(hipMemset(flags[kDeviceFlag], 0, 64));
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&flags[kSignalFlag]), 64, hipMallocSignalMemory) != hipSuccess) {
    (void)hipGetLastError();
    flags[kSignalFlag] = nullptr;
    std::printf("{\"note\": \"hipMallocSignalMemory refused: signal-memory variant skipped\"}\n");
  } else {
    CHECK(hipMemset(flags[kSignalFlag], 0, 8));
  }
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&flags[kHostFlag]), 64, hipHostMallocCoherent));
  std::memset(flags[kHostFlag], 0, 64);
  uint32_t epoch = 0;
  const long self_tid = long(gettid());
  for (const Variant& v : vs) {
    if (v.flag != kNoFlag && flags[v.flag] == nullptr) continue;
    for (int rep = 0; rep < 2; ++rep) {
      hipStream_t a, b;
      CHECK(hipStreamCreateWithFlags(&a, v.st_flags));
      CHECK(hipStreamCreateWithFlags(&b, v.st_flags));
      hipEvent_t ea, eb;
      CHECK(hipEventCreateWithFlags(&ea, v.ev_flags));
      CHECK(hipEventCreateWithFlags(&eb, v.ev_flags));
      CHECK(hipDeviceSynchronize());
      auto t0 = thread_ticks();
      auto w0 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(busy_kernel, dim3(1), dim3(64), 0, a, iters, out);
      CHECK(hipEventRecord(ea, a));
      hipEvent_t last = ea;
      if (v.cross_wait && v.flag != kNoFlag) {
        ++epoch;
        CHECK(hipStreamWriteValue32(a, flags[v.flag], epoch, 0));
        CHECK(hipStreamWaitValue32(b, flags[v.flag], epoch, hipStreamWaitValueGte, 0xFFFFFFFFu));
        CHECK(hipEventRecord(eb, b));
        last = eb;
      } else if (v.cross_wait) {
        CHECK(hipStreamWaitEvent(b, ea, 0));
        CHECK(hipEventRecord(eb, b));
        last = eb;
      }
      if (v.query_loop) {
        while (hipEventQuery(last) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(200));
      } else {
        CHECK(hipEventSynchronize(last));
      }
      const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
      auto t1 = thread_ticks();
      double main_ms = 0, other_ms = 0, busiest = 0;
      for (auto& [tid, tk] : t1) {
        const double d = double(tk - (t0.count(tid) ? t0[tid] : 0)) * 1e3 / double(hz);
        if (tid == self_tid) main_ms += d;
        else {
          other_ms += d;
          if (d > busiest) busiest = d;
        }
      }
      std::printf("{\"variant\": \"%s\", \"rep\": %d, \"wall_ms\": %.1f, \"main_thread_ms\": %.1f, "
                  "\"other_threads_ms\": %.1f, \"busiest_other_ms\": %.1f, \"threads\": %zu}\n",
                  v.name, rep, wall, main_ms, other_ms, busiest, t1.size());
      std::fflush(stdout);
      CHECK(hipEventDestroy(ea));
      CHECK(hipEventDestroy(eb));
      CHECK(hipStreamDestroy(a));
      CHECK(hipStreamDestroy(b));
    }
  }
  CHECK(hipDeviceSynchronize());
  CHECK(hipFree(flags[kDeviceFlag]));
  if (flags[kSignalFlag]) CHECK(hipFree(flags[kSignalFlag]));
  CHECK(hipHostFree(flags[kHostFlag]));
  CHECK(hipFree(out));
  return 0;
}
