// RCCL over xGMI: one communicator per ShardedOptimizer, bucketed collectives on a caller stream.
//
// The reference issues one blocking c10d collective per parameter tensor (zero1.py:81-84,
// zero1.py:95-102, zero2.py:94-113, zero2.py:126-133, zero3.py:38-39, zero3.py:146) followed by
// torch.cuda.synchronize().  Here every collective moves a whole bucket and is only enqueued:
// ordering against the pack / Adam / unpack kernels is by stream and event, never by host sync.
//
// Binding: the library links librccl.so.1 / libamdhip64.so.7 by SONAME; the Python loader imports
// torch first so both resolve to torch's already-loaded copies (one HIP runtime, one RCCL).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <vector>

#include "zs_common.h"

struct zs_comm {
  ncclComm_t comm = nullptr;
  int ws = 1, rank = 0;
};

static_assert(sizeof(ncclUniqueId) == ZS_UNIQUE_ID_BYTES, "ncclUniqueId size changed");

#define ZS_NCCL(expr)                                                                   \
  do {                                                                                  \
    ncclResult_t r_ = (expr);                                                           \
    if (r_ != ncclSuccess)                                                              \
      return zs::fail(ZS_ERR_RCCL, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(r_), \
                      __FILE__, __LINE__);                                              \
  } while (0)

static int to_nccl(int dtype, ncclDataType_t* t) {
  switch (dtype) {
    case ZS_F32: *t = ncclFloat32; return ZS_OK;
    case ZS_BF16: *t = ncclBfloat16; return ZS_OK;
    case ZS_U8: *t = ncclUint8; return ZS_OK;
    default: return zs::fail(ZS_ERR_INVALID, "unsupported dtype %d", dtype);
  }
}

int& zs::sync_host_flags() {  // (zs_tune "sync_host_flags"; zs_common.h)
  static int mode = 1;
  return mode;
}

namespace zs {
hipError_t flag_write(uint64_t* flag, uint64_t value, hipStream_t st);  // zs_kernels.hip
hipError_t flag_wait_launch(const uint64_t* flag, uint64_t value, hipStream_t st);  // zs_kernels.hip
uint32_t* wait_timeout_word();  // zs_kernels.hip: set by a flag wait kernel that gave up
}

extern "C" {

int zs_comm_unique_id(void* out128) {
  ZS_REQUIRE(out128 != nullptr, "zs_comm_unique_id: out is NULL");
  ncclUniqueId id;
  ZS_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out128, &id, sizeof id);
  return ZS_OK;
}

int zs_comm_init(const void* uid, int ws, int rank, zs_comm** out) {
  ZS_REQUIRE(uid && out, "zs_comm_init: NULL argument");
  *out = nullptr;
  ZS_REQUIRE(ws >= 1 && rank >= 0 && rank < ws, "zs_comm_init: bad ws/rank %d/%d", ws, rank);
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof id);
  zs_comm* c = new (std::nothrow) zs_comm();
  if (!c) return zs::fail(ZS_ERR_NOMEM, "zs_comm_init: out of memory");
  ncclResult_t r = ncclCommInitRank(&c->comm, ws, id, rank);
  if (r != ncclSuccess) {
    delete c;
    return zs::fail(ZS_ERR_RCCL, "ncclCommInitRank(ws=%d, rank=%d) failed: %s", ws, rank,
                    ncclGetErrorString(r));
  }
  c->ws = ws;
  c->rank = rank;
  *out = c;
  return ZS_OK;
}

int zs_comm_destroy(zs_comm* c) {
  if (!c) return ZS_OK;
  ncclResult_t r = c->comm ? ncclCommDestroy(c->comm) : ncclSuccess;
  delete c;
  if (r != ncclSuccess)
    return zs::fail(ZS_ERR_RCCL, "ncclCommDestroy failed: %s", ncclGetErrorString(r));
  return ZS_OK;
}

int zs_reduce_scatter(zs_comm* c, const void* send, void* recv, int64_t recv_count, int dtype,
                      uintptr_t stream) {
  ZS_REQUIRE(c && c->comm, "zs_reduce_scatter: NULL communicator");
  ZS_REQUIRE(recv_count >= 0, "zs_reduce_scatter: recv_count < 0");
  if (recv_count == 0) return ZS_OK;
  ZS_REQUIRE(send && recv, "zs_reduce_scatter: NULL buffer");
  ncclDataType_t t;
  int rc = to_nccl(dtype, &t);
  if (rc) return rc;
  ZS_NCCL(ncclReduceScatter(send, recv, size_t(recv_count), t, ncclSum, c->comm,
                            reinterpret_cast<hipStream_t>(stream)));
  return ZS_OK;
}

int zs_all_gather(zs_comm* c, const void* send, void* recv, int64_t send_count, int dtype,
                  uintptr_t stream) {
  ZS_REQUIRE(c && c->comm, "zs_all_gather: NULL communicator");
  ZS_REQUIRE(send_count >= 0, "zs_all_gather: send_count < 0");
  if (send_count == 0) return ZS_OK;
  ZS_REQUIRE(send && recv, "zs_all_gather: NULL buffer");
  ncclDataType_t t;
  int rc = to_nccl(dtype, &t);
  if (rc) return rc;
  ZS_NCCL(ncclAllGather(send, recv, size_t(send_count), t, c->comm,
                        reinterpret_cast<hipStream_t>(stream)));
  return ZS_OK;
}

int zs_all_reduce(zs_comm* c, const void* send, void* recv, int64_t count, int dtype,
                  uintptr_t stream) {
  ZS_REQUIRE(c && c->comm, "zs_all_reduce: NULL communicator");
  ZS_REQUIRE(count >= 0, "zs_all_reduce: count < 0");
  if (count == 0) return ZS_OK;
  ZS_REQUIRE(send && recv, "zs_all_reduce: NULL buffer");
  ncclDataType_t t;
  int rc = to_nccl(dtype, &t);
  if (rc) return rc;
  ZS_NCCL(ncclAllReduce(send, recv, size_t(count), t, ncclSum, c->comm,
                        reinterpret_cast<hipStream_t>(stream)));
  return ZS_OK;
}

int zs_reduce(zs_comm* c, const void* send, void* recv, int64_t count, int dtype, int root,
              uintptr_t stream) {
  ZS_REQUIRE(c && c->comm, "zs_reduce: NULL communicator");
  ZS_REQUIRE(count >= 0, "zs_reduce: count < 0");
  ZS_REQUIRE(root >= 0 && root < c->ws, "zs_reduce: root %d out of range", root);
  if (count == 0) return ZS_OK;
  ZS_REQUIRE(send && (recv || c->rank != root), "zs_reduce: NULL buffer");
  ncclDataType_t t;
  int rc = to_nccl(dtype, &t);
  if (rc) return rc;
  ZS_NCCL(ncclReduce(send, recv, size_t(count), t, ncclSum, root, c->comm,
                     reinterpret_cast<hipStream_t>(stream)));
  return ZS_OK;
}

int zs_broadcast(zs_comm* c, const void* send, void* recv, int64_t count, int dtype, int root,
                 uintptr_t stream) {
  ZS_REQUIRE(c && c->comm, "zs_broadcast: NULL communicator");
  ZS_REQUIRE(count >= 0, "zs_broadcast: count < 0");
  ZS_REQUIRE(root >= 0 && root < c->ws, "zs_broadcast: root %d out of range", root);
  if (count == 0) return ZS_OK;
  ZS_REQUIRE(recv && (send || c->rank != root), "zs_broadcast: NULL buffer");
  ncclDataType_t t;
  int rc = to_nccl(dtype, &t);
  if (rc) return rc;
  ZS_NCCL(ncclBroadcast(send, recv, size_t(count), t, root, c->comm,
                        reinterpret_cast<hipStream_t>(stream)));
  return ZS_OK;
}

// One RCCL group of n reduces / in-place broadcasts: the reduce-scatter-v and all-gather-v of a
// flat-arena round (each owner's contiguous window reduced to it, then broadcast from it).  One
// call per round instead of one per owner; the group launches every transfer together, so each
// rank is the root of one and forwards for the others.
int zs_reduce_group(zs_comm* c, int64_t n, const uint64_t* send, const uint64_t* recv,
                    const int64_t* count, const int32_t* root, int dtype, uintptr_t stream) {
  ZS_REQUIRE(c && c->comm, "zs_reduce_group: NULL communicator");
  ZS_REQUIRE(n >= 0 && (n == 0 || (send && recv && count && root)), "zs_reduce_group: bad table");
  ncclDataType_t t;
  int rc = to_nccl(dtype, &t);
  if (rc) return rc;
  for (int64_t i = 0; i < n; ++i) {
    ZS_REQUIRE(count[i] >= 0 && root[i] >= 0 && root[i] < c->ws,
               "zs_reduce_group: entry %lld: count %lld root %d", (long long)i,
               (long long)count[i], root[i]);
    ZS_REQUIRE(count[i] == 0 || (send[i] && (recv[i] || root[i] != c->rank)),
               "zs_reduce_group: entry %lld: NULL buffer", (long long)i);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  ZS_NCCL(ncclGroupStart());
  for (int64_t i = 0; i < n; ++i) {
    if (count[i] == 0) continue;
    ncclResult_t r = ncclReduce(reinterpret_cast<const void*>(send[i]),
                                reinterpret_cast<void*>(recv[i]), size_t(count[i]), t, ncclSum,
                                root[i], c->comm, st);
    if (r != ncclSuccess) {
      (void)ncclGroupEnd();
      return zs::fail(ZS_ERR_RCCL, "ncclReduce (group entry %lld) failed: %s", (long long)i,
                      ncclGetErrorString(r));
    }
  }
  ZS_NCCL(ncclGroupEnd());
  return ZS_OK;
}

int zs_broadcast_group(zs_comm* c, int64_t n, const uint64_t* buf, const int64_t* count,
                       const int32_t* root, int dtype, uintptr_t stream) {
  ZS_REQUIRE(c && c->comm, "zs_broadcast_group: NULL communicator");
  ZS_REQUIRE(n >= 0 && (n == 0 || (buf && count && root)), "zs_broadcast_group: bad table");
  ncclDataType_t t;
  int rc = to_nccl(dtype, &t);
  if (rc) return rc;
  for (int64_t i = 0; i < n; ++i)
    ZS_REQUIRE(count[i] >= 0 && root[i] >= 0 && root[i] < c->ws && (count[i] == 0 || buf[i]),
               "zs_broadcast_group: entry %lld: count %lld root %d", (long long)i,
               (long long)count[i], root[i]);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  ZS_NCCL(ncclGroupStart());
  for (int64_t i = 0; i < n; ++i) {
    if (count[i] == 0) continue;
    void* p = reinterpret_cast<void*>(buf[i]);
    ncclResult_t r = ncclBroadcast(p, p, size_t(count[i]), t, root[i], c->comm, st);
    if (r != ncclSuccess) {
      (void)ncclGroupEnd();
      return zs::fail(ZS_ERR_RCCL, "ncclBroadcast (group entry %lld) failed: %s", (long long)i,
                      ncclGetErrorString(r));
    }
  }
  ZS_NCCL(ncclGroupEnd());
  return ZS_OK;
}

int zs_all_gather_group(zs_comm* c, int64_t n, const uint64_t* send, const uint64_t* recv,
                        const int64_t* send_count, int dtype, uintptr_t stream) {
  ZS_REQUIRE(c && c->comm, "zs_all_gather_group: NULL communicator");
  ZS_REQUIRE(n >= 0 && (n == 0 || (send && recv && send_count)), "zs_all_gather_group: bad table");
  ncclDataType_t t;
  int rc = to_nccl(dtype, &t);
  if (rc) return rc;
  for (int64_t i = 0; i < n; ++i)
    ZS_REQUIRE(send_count[i] >= 0 && (send_count[i] == 0 || (send[i] && recv[i])),
               "zs_all_gather_group: entry %lld: count %lld", (long long)i,
               (long long)send_count[i]);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  ZS_NCCL(ncclGroupStart());
  for (int64_t i = 0; i < n; ++i) {
    if (send_count[i] == 0) continue;
    ncclResult_t r = ncclAllGather(reinterpret_cast<const void*>(send[i]),
                                   reinterpret_cast<void*>(recv[i]), size_t(send_count[i]), t,
                                   c->comm, st);
    if (r != ncclSuccess) {
      (void)ncclGroupEnd();
      return zs::fail(ZS_ERR_RCCL, "ncclAllGather (group entry %lld) failed: %s", (long long)i,
                      ncclGetErrorString(r));
    }
  }
  ZS_NCCL(ncclGroupEnd());
  return ZS_OK;
}

int zs_reduce_scatter_group(zs_comm* c, int64_t n, const uint64_t* send, const uint64_t* recv,
                            const int64_t* recv_count, int dtype, uintptr_t stream) {
  ZS_REQUIRE(c && c->comm, "zs_reduce_scatter_group: NULL communicator");
  ZS_REQUIRE(n >= 0 && (n == 0 || (send && recv && recv_count)),
             "zs_reduce_scatter_group: bad table");
  ncclDataType_t t;
  int rc = to_nccl(dtype, &t);
  if (rc) return rc;
  for (int64_t i = 0; i < n; ++i)
    ZS_REQUIRE(recv_count[i] >= 0 && (recv_count[i] == 0 || (send[i] && recv[i])),
               "zs_reduce_scatter_group: entry %lld: count %lld", (long long)i,
               (long long)recv_count[i]);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  ZS_NCCL(ncclGroupStart());
  for (int64_t i = 0; i < n; ++i) {
    if (recv_count[i] == 0) continue;
    ncclResult_t r = ncclReduceScatter(reinterpret_cast<const void*>(send[i]),
                                       reinterpret_cast<void*>(recv[i]), size_t(recv_count[i]), t,
                                       ncclSum, c->comm, st);
    if (r != ncclSuccess) {
      (void)ncclGroupEnd();
      return zs::fail(ZS_ERR_RCCL, "ncclReduceScatter (group entry %lld) failed: %s",
                      (long long)i, ncclGetErrorString(r));
    }
  }
  ZS_NCCL(ncclGroupEnd());
  return ZS_OK;
}

// Ordering around a group in the same call: record `ready` where the inputs were produced, make
// the collective stream wait for it, issue the group, record `done` after it.
static int ordered_prologue(uintptr_t after_stream, uint64_t ready_event, uintptr_t stream) {
  if (ready_event) {
    hipEvent_t ev = reinterpret_cast<hipEvent_t>(ready_event);
    ZS_HIP(hipEventRecord(ev, reinterpret_cast<hipStream_t>(after_stream)));
    ZS_HIP(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ev, 0));
  }
  return ZS_OK;
}

static int ordered_epilogue(uintptr_t stream, uint64_t done_event) {
  if (done_event)
    ZS_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(done_event),
                          reinterpret_cast<hipStream_t>(stream)));
  return ZS_OK;
}

int zs_all_gather_group_ordered(zs_comm* c, int64_t n, const uint64_t* send, const uint64_t* recv,
                                const int64_t* send_count, int dtype, uintptr_t after_stream,
                                uint64_t ready_event, uintptr_t stream, uint64_t done_event) {
  ZS_REQUIRE(n == 0 || (c && c->comm), "zs_all_gather_group_ordered: NULL communicator");
  int rc = ordered_prologue(after_stream, ready_event, stream);
  if (rc == ZS_OK && n > 0) rc = zs_all_gather_group(c, n, send, recv, send_count, dtype, stream);
  if (rc == ZS_OK) rc = ordered_epilogue(stream, done_event);
  return rc;
}

int zs_reduce_scatter_group_ordered(zs_comm* c, int64_t n, const uint64_t* send,
                                    const uint64_t* recv, const int64_t* recv_count, int dtype,
                                    uintptr_t after_stream, uint64_t ready_event, uintptr_t stream,
                                    uint64_t done_event) {
  ZS_REQUIRE(n == 0 || (c && c->comm), "zs_reduce_scatter_group_ordered: NULL communicator");
  int rc = ordered_prologue(after_stream, ready_event, stream);
  if (rc == ZS_OK && n > 0)
    rc = zs_reduce_scatter_group(c, n, send, recv, recv_count, dtype, stream);
  if (rc == ZS_OK) rc = ordered_epilogue(stream, done_event);
  return rc;
}

int zs_stream_wait_event(uintptr_t stream, uint64_t event) {
  ZS_REQUIRE(event != 0, "zs_stream_wait_event: NULL event");
  ZS_HIP(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream),
                            reinterpret_cast<hipEvent_t>(event), 0));
  return ZS_OK;
}

// ---------------------------------------------------------------------------------------------
// Sync objects (ABI v12; 64-bit words since v13): the cross-stream ordering of the engines as either
// a HIP event or a stream memory operation on a flag word (a one-wave release-store kernel —
// round 6; hipStreamWriteValue64 with zs_tune "sync_write_kernel" 0 — after the producer's work, hipStreamWaitValue64 >= the recorded epoch before the consumer's).  A record
// bumps the object's epoch on the host and enqueues its write; a wait enqueues a wait for the epoch
// of the latest record, the semantics of hipStreamWaitEvent.  Epochs are 64-bit and only grow: at
// one record per microsecond a word wraps after 584,000 years, so the unsigned >= of the GPU wait
// and the host's skip test agree for the life of any process (v12's 32-bit epoch wrapped after
// 2^32 records, where the GPU's unsigned compare and the host's modulo compare disagree).
// A record from a different stream than the previous one first makes its stream wait for the
// previous epoch, so the words reach the flag in epoch order whichever streams record.
struct zs_sync {
  int kind = ZS_SYNC_EVENT;
  int device = 0;
  hipEvent_t event = nullptr;
  uint64_t* flag = nullptr;
  bool host_word = false;  // the flag word is host-readable (pinned): satisfied waits are skipped
  uint64_t epoch = 0;
  hipStream_t last_stream = nullptr;  // the stream of the latest record (flag kind)
};

namespace {
// Flag words come from slabs of pinned, host-coherent memory (one hipHostMalloc per 4096 flags, 64 B
// apart: one cache line each; engines create a few hundred syncs, not a few hundred tiny
// allocations).  The GPU writes and polls them like device memory, and the host can read them: a
// wait whose epoch has already been written is skipped on the host, as the HIP runtime skips a wait
// on a completed event — the enqueue of a stream wait costs ~3-5 us of the caller
// (profiles/r05_sync_cost.json), and a prefetched gather has usually finished when its consumer
// asks for it whenever the host, not the GPU, is the bottleneck.  Zero-filled by the host before
// any word is handed out (no device work a record could race with).
// (Should pinned memory be refused, the words come from device slabs instead — zeroed to
// completion on the device before any word is handed out, so no record can be overtaken by the
// fill — and every wait is enqueued.)
constexpr int kFlagsPerSlab = 4096;
constexpr size_t kFlagStride = 64;
std::mutex g_flag_mu;
std::vector<uint64_t*> g_flag_free;                      // host-coherent words
std::map<int, std::vector<uint64_t*>> g_flag_dev_free;  // device words, per device (fallback)
bool g_host_flags = true;

void carve(unsigned char* slab, std::vector<uint64_t*>& fl) {
  for (int i = kFlagsPerSlab - 1; i >= 0; --i)
    fl.push_back(reinterpret_cast<uint64_t*>(slab + size_t(i) * kFlagStride));
}

hipError_t flag_take(int device, uint64_t** out, bool* host_word) {
  std::lock_guard<std::mutex> lk(g_flag_mu);
  const bool host = g_host_flags && zs::sync_host_flags();
  if (host && g_flag_free.empty()) {
    void* slab = nullptr;
    if (hipHostMalloc(&slab, kFlagsPerSlab * kFlagStride,
                      hipHostMallocCoherent | hipHostMallocPortable | hipHostMallocMapped) ==
        hipSuccess) {
      std::memset(slab, 0, kFlagsPerSlab * kFlagStride);
      carve(static_cast<unsigned char*>(slab), g_flag_free);
    } else {
      (void)hipGetLastError();
      g_host_flags = false;
    }
  }
  if (host && g_host_flags) {
    *out = g_flag_free.back();
    g_flag_free.pop_back();
    *host_word = true;
    return hipSuccess;
  }
  auto& fl = g_flag_dev_free[device];
  if (fl.empty()) {
    unsigned char* slab = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&slab), kFlagsPerSlab * kFlagStride);
    if (e == hipSuccess) e = hipMemsetAsync(slab, 0, kFlagsPerSlab * kFlagStride, nullptr);
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    if (e != hipSuccess) return e;
    carve(slab, fl);
  }
  *out = fl.back();
  fl.pop_back();
  *host_word = false;
  return hipSuccess;
}

// the word has reached epoch `e` (epochs only grow; 64-bit, so they never wrap)
bool flag_reached(const uint64_t* w, uint64_t e) { return __atomic_load_n(w, __ATOMIC_ACQUIRE) >= e; }

// `st` waits for the word to reach `e` unless the host already sees it there
hipError_t flag_wait(const zs_sync* s, hipStream_t st, uint64_t e) {
  if (e == 0 || (s->host_word && flag_reached(s->flag, e))) return hipSuccess;
  if (zs::sync_wait_kernel()) return zs::flag_wait_launch(s->flag, e, st);
  return hipStreamWaitValue64(st, s->flag, e, hipStreamWaitValueGte, ~uint64_t(0));
}
}  // namespace

int zs_sync_create(int kind, zs_sync** out) {
  ZS_REQUIRE(out != nullptr, "zs_sync_create: out is NULL");
  ZS_REQUIRE(kind == ZS_SYNC_EVENT || kind == ZS_SYNC_FLAG, "zs_sync_create: bad kind %d", kind);
  *out = nullptr;
  zs_sync* s = new (std::nothrow) zs_sync();
  if (!s) return zs::fail(ZS_ERR_NOMEM, "zs_sync_create: out of memory");
  s->kind = kind;
  hipError_t e = hipGetDevice(&s->device);
  if (e == hipSuccess) {
    if (kind == ZS_SYNC_EVENT) {
      e = hipEventCreateWithFlags(&s->event, hipEventDisableTiming);
    } else {
      e = flag_take(s->device, &s->flag, &s->host_word);  // (zeroed with its slab: epoch 0)
    }
  }
  if (e != hipSuccess) {
    zs_sync_destroy(s);
    return zs::fail(ZS_ERR_HIP, "zs_sync_create: %s", hipGetErrorString(e));
  }
  *out = s;
  return ZS_OK;
}

int zs_sync_destroy(zs_sync* s) {
  if (!s) return ZS_OK;
  if (s->event) (void)hipEventDestroy(s->event);
  // a flag word may still be written by a queued record or read by a queued wait, and finding
  // out would synchronise the device from a destructor: the word is abandoned, not recycled
  // (64 B; a destroyed sync is rare — an engine going away)
  delete s;
  return ZS_OK;
}

// a flag wait kernel gave up (about a minute without its record): its stream went on unordered
static int flag_wait_check() {
  const uint32_t* w = zs::wait_timeout_word();
  if (w != nullptr && __atomic_load_n(w, __ATOMIC_ACQUIRE) != 0)
    return zs::fail(ZS_ERR_HIP, "a stream-flag wait timed out on the GPU (no record within ~1 min): "
                    "cross-stream ordering was lost; results since then are not trustworthy");
  return ZS_OK;
}

int zs_sync_record(zs_sync* s, uintptr_t stream) {
  ZS_REQUIRE(s != nullptr, "zs_sync_record: NULL sync");
  if (int rc = flag_wait_check()) return rc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (s->kind == ZS_SYNC_EVENT) {
    ZS_HIP(hipEventRecord(s->event, st));
  } else {
    // another stream than the last record's: order this write after that one's, or the word
    // could go back from epoch + 1 to epoch when the two streams run in the other order
    if (s->epoch > 0 && st != s->last_stream) ZS_HIP(flag_wait(s, st, s->epoch));
    if (zs::sync_write_kernel())
      ZS_HIP(zs::flag_write(s->flag, s->epoch + 1, st));
    else
      ZS_HIP(hipStreamWriteValue64(st, s->flag, s->epoch + 1, 0));
    ++s->epoch;
    s->last_stream = st;
  }
  return ZS_OK;
}

int zs_sync_wait(zs_sync* s, uintptr_t stream) {
  ZS_REQUIRE(s != nullptr, "zs_sync_wait: NULL sync");
  if (int rc = flag_wait_check()) return rc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (s->kind == ZS_SYNC_EVENT) {
    ZS_HIP(hipStreamWaitEvent(st, s->event, 0));
  } else {
    // (epoch 0: never recorded, nothing to wait for; a record that already executed: skipped)
    ZS_HIP(flag_wait(s, st, s->epoch));
  }
  return ZS_OK;
}

int zs_sync_set_epoch(zs_sync* s, uint64_t epoch) {
  ZS_REQUIRE(s != nullptr, "zs_sync_set_epoch: NULL sync");
  ZS_REQUIRE(s->kind == ZS_SYNC_FLAG, "zs_sync_set_epoch: not a flag sync");
  ZS_REQUIRE(epoch >= s->epoch, "zs_sync_set_epoch: epochs only grow (%llu < %llu)",
             (unsigned long long)epoch, (unsigned long long)s->epoch);
  // every record enqueued so far has executed (the caller's contract); then the word and the
  // host epoch move together
  if (s->host_word) {
    ZS_REQUIRE(flag_reached(s->flag, s->epoch), "zs_sync_set_epoch: a record is still pending");
    __atomic_store_n(s->flag, epoch, __ATOMIC_RELEASE);
  } else {
    ZS_HIP(hipMemcpy(s->flag, &epoch, sizeof(epoch), hipMemcpyHostToDevice));
  }
  s->epoch = epoch;
  return ZS_OK;
}

int zs_sync_query(zs_sync* s, uint64_t* epoch, uint64_t* word) {
  ZS_REQUIRE(s != nullptr, "zs_sync_query: NULL sync");
  if (epoch) *epoch = s->kind == ZS_SYNC_FLAG ? s->epoch : 0;
  if (word) {
    *word = 0;
    if (s->kind == ZS_SYNC_FLAG) {
      if (s->host_word)
        *word = __atomic_load_n(s->flag, __ATOMIC_ACQUIRE);
      else
        ZS_HIP(hipMemcpy(word, s->flag, sizeof(*word), hipMemcpyDeviceToHost));
    }
  }
  return ZS_OK;
}

// `stream` after everything enqueued so far on `after_stream`.  (Not skipped when after_stream is
// idle: tried with a hipStreamQuery per call, ~0.2 us for the caller, the process CPU of the
// simulated C5 iteration rose from 7.2 to 11.1 ms against 11.7 ms with events — other threads'
// time, as a pending event wait costs — profiles/r05_z3_host_ab_query.json.)
static int synced_prologue(uintptr_t after_stream, zs_sync* ready, uintptr_t stream) {
  if (ready) {
    int rc = zs_sync_record(ready, after_stream);
    if (rc == ZS_OK) rc = zs_sync_wait(ready, stream);
    return rc;
  }
  return ZS_OK;
}

int zs_all_gather_group_synced(zs_comm* c, int64_t n, const uint64_t* send, const uint64_t* recv,
                               const int64_t* send_count, int dtype, uintptr_t after_stream,
                               zs_sync* ready, uintptr_t stream, zs_sync* done) {
  ZS_REQUIRE(n == 0 || (c && c->comm), "zs_all_gather_group_synced: NULL communicator");
  int rc = synced_prologue(after_stream, ready, stream);
  if (rc == ZS_OK && n > 0) rc = zs_all_gather_group(c, n, send, recv, send_count, dtype, stream);
  if (rc == ZS_OK && done) rc = zs_sync_record(done, stream);
  return rc;
}

int zs_reduce_scatter_group_synced(zs_comm* c, int64_t n, const uint64_t* send,
                                   const uint64_t* recv, const int64_t* recv_count, int dtype,
                                   uintptr_t after_stream, zs_sync* ready, uintptr_t stream,
                                   zs_sync* done) {
  ZS_REQUIRE(n == 0 || (c && c->comm), "zs_reduce_scatter_group_synced: NULL communicator");
  int rc = synced_prologue(after_stream, ready, stream);
  if (rc == ZS_OK && n > 0)
    rc = zs_reduce_scatter_group(c, n, send, recv, recv_count, dtype, stream);
  if (rc == ZS_OK && done) rc = zs_sync_record(done, stream);
  return rc;
}

int zs_group_start(void) {
  ZS_NCCL(ncclGroupStart());
  return ZS_OK;
}

int zs_group_end(void) {
  ZS_NCCL(ncclGroupEnd());
  return ZS_OK;
}

int zs_rccl_version(int* version) {
  ZS_REQUIRE(version != nullptr, "zs_rccl_version: NULL argument");
  ZS_NCCL(ncclGetVersion(version));
  return ZS_OK;
}

}  // extern "C"
