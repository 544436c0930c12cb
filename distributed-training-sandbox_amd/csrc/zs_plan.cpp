// Layout planner: parameter ownership, per-rank optimizer-shard streams and bucket segments.
//
// Host-only (no HIP calls of its own: zs_pack / zs_unpack launch through the copy-set API), so
// the planner runs in the CPU test suite.  Ownership follows the reference's
// ShardedOptimizer.__init__ exactly (zero1.py:55-62, zero2.py:51-58, zero3.py:93-100):
//     ppr = n // ws, rem = n % ws
//     start_r = r*ppr + min(r, rem), end_r = start_r + ppr + (r < rem)
// and the broadcast owner of index i (zero1.py:95-100, zero2.py:126-131):
//     i < (ppr+1)*rem ? i // (ppr+1) : (i - rem) // ppr
//
// A rank's *stream* is the ordered list of pieces whose optimizer state it owns; pieces start at
// multiples of align_elems so that every device access can be 16-byte vectorised.  A bucket
// concatenates, rank-major, one *window* of every rank's stream:
//   * even buckets cover stream positions [0, Lmin) (Lmin = the shortest stream) with equal windows
//     of <= W elements: exactly the buffer one equal-count reduce-scatter / all-gather moves;
//   * ragged buckets (ZS_BUCKETS_RAGGED) cover the rest, [Lmin, L_r) of each longer stream, with
//     per-rank windows of different length, moved by one grouped reduce / broadcast per owner.
// Layout R's ownership is uneven (SmolLM3-3B at ws=8: 585.6M vs 335.0M elements), so padding every
// window to the longest stream (ZS_BUCKETS_PADDED, the simple scheme) makes each equal-count
// collective move 1.52x the data; the ragged tail moves only the bytes that exist.
#include <algorithm>
#include <cstring>
#include <map>
#include <new>
#include <utility>
#include <vector>

#include "zs_common.h"

namespace {

struct Piece {
  int64_t param, param_off, stream_off, len;
};
struct Seg {
  int64_t param, rank, param_off, buf_off, len;
};
struct Bucket {
  int64_t arena_off = 0, elems = 0;
  int even = 1;
  std::vector<int64_t> win_off, win_len, win_stream;  // per rank: offset in bucket, length,
                                                      // offset in the rank's stream
};

inline int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// zs_pack / zs_unpack descriptor tables of one bucket, keyed by the pointers they were built for.
struct CopyCache {
  std::vector<uint64_t> sig;
  zs_copyset* cs = nullptr;
};

}  // namespace

struct zs_plan {
  int64_t n = 0;
  int ws = 1, rank = 0, layout = 0;
  int64_t align = 1, W = 0, K = 0, M = 0, Lmin = 0, arena = 0, K_even = 0;
  int mode = ZS_BUCKETS_RAGGED;
  std::vector<int64_t> numel;
  std::vector<std::vector<Piece>> pieces;  // per rank
  std::vector<int64_t> stream_len;         // per rank
  std::vector<Bucket> buckets;
  std::vector<std::vector<Seg>> segs;      // per bucket
  std::map<std::pair<int64_t, int>, CopyCache> copy_cache;  // (bucket, 0 = pack / 1 = unpack)
  std::vector<zs_copyset*> retired;  // tables replaced while a copy might still read them
  ~zs_plan() {
    for (auto& kv : copy_cache) zs_copyset_destroy(kv.second.cs);
    for (zs_copyset* cs : retired) zs_copyset_destroy(cs);
  }
};

static void owner_range(int64_t n, int ws, int r, int64_t* s, int64_t* e) {
  const int64_t ppr = n / ws, rem = n % ws;
  *s = r * ppr + std::min<int64_t>(r, rem);
  *e = *s + ppr + (r < rem ? 1 : 0);
}

static int owner_of(int64_t n, int ws, int64_t i) {
  const int64_t ppr = n / ws, rem = n % ws;
  if (i < (ppr + 1) * rem) return int(i / (ppr + 1));
  return int((i - rem) / ppr);
}

// zs_pack (unpack = 0: param grads -> bucket) / zs_unpack (unpack = 1: bucket -> params) of every
// segment of `bucket`, through a cached copy set (host work only when the pointers change).
static int bucket_copy(zs_plan* p, int64_t bucket, int unpack, const uint64_t* ptrs, uint64_t buf,
                       int dtype, uintptr_t stream, const char* fn) {
  ZS_REQUIRE(p && ptrs, "%s: NULL argument", fn);
  ZS_REQUIRE(bucket >= 0 && bucket < p->K, "%s: bucket %lld out of range", fn, (long long)bucket);
  ZS_REQUIRE(dtype == ZS_F32 || dtype == ZS_BF16, "%s: dtype must be ZS_F32 or ZS_BF16 (got %d)",
             fn, dtype);
  ZS_REQUIRE(buf != 0, "%s: bucket buffer is NULL", fn);
  const uint64_t es = dtype == ZS_F32 ? 4 : 2;
  const auto& v = p->segs[bucket];
  const size_t n = v.size();
  std::vector<uint64_t> sig(2 * n + 1);  // src[n] | dst[n] | element size
  std::vector<int64_t> nb(n);
  for (size_t j = 0; j < n; ++j) {
    const Seg& s = v[j];
    const uint64_t prm = ptrs[s.param];
    const uint64_t q = prm ? prm + uint64_t(s.param_off) * es : 0;
    const uint64_t b = buf + uint64_t(s.buf_off) * es;
    ZS_REQUIRE(!unpack || q != 0 || s.len == 0, "%s: param_ptrs[%lld] is NULL", fn,
               (long long)s.param);
    sig[j] = unpack ? b : q;  // a NULL grad source zero-fills its slot
    sig[n + j] = unpack ? q : b;
    nb[j] = s.len * int64_t(es);
  }
  sig[2 * n] = es;
  CopyCache& c = p->copy_cache[{bucket, unpack}];
  if (!c.cs || c.sig != sig) {
    zs_copyset* cs = nullptr;
    const int rc = zs_copyset_create(sig.data(), sig.data() + n, nb.data(), int64_t(n), &cs);
    if (rc != ZS_OK) return rc;
    if (c.cs) p->retired.push_back(c.cs);
    c.cs = cs;
    c.sig = std::move(sig);
  }
  return zs_copyset_run(c.cs, stream);
}

// Buckets over the per-rank streams, then the segments (param slices) of every bucket.
static void plan_buckets(zs_plan* p) {
  const int ws = p->ws;
  const int64_t W = p->W, A = p->align;
  auto add = [&](Bucket&& b) {
    b.arena_off = p->arena;
    p->arena += round_up(b.elems, A);
    p->buckets.push_back(std::move(b));
  };
  // even part: equal windows over [0, Lmin) (all of [0, M) with padding in ZS_BUCKETS_PADDED)
  const int64_t even_end = p->mode == ZS_BUCKETS_PADDED ? p->M : p->Lmin;
  for (int64_t pos = 0; pos < even_end; pos += W) {
    const int64_t wk = std::min(W, even_end - pos);  // multiple of A: every stream length is
    Bucket b;
    b.even = 1;
    for (int r = 0; r < ws; ++r) {
      b.win_off.push_back(int64_t(r) * wk);
      b.win_len.push_back(wk);
      b.win_stream.push_back(pos);
    }
    b.elems = int64_t(ws) * wk;
    add(std::move(b));
  }
  p->K_even = int64_t(p->buckets.size());
  // ragged tail: per-rank cursors from Lmin; each bucket holds at most ws*W elements, shared
  // equally by the ranks that still have stream left (a rank with a short tail leaves its share
  // to the others in the next bucket)
  std::vector<int64_t> cur(ws, even_end);
  const int64_t cap = int64_t(ws) * W;
  for (;;) {
    int active = 0;
    for (int r = 0; r < ws; ++r) active += cur[r] < p->stream_len[r];
    if (active == 0) break;
    const int64_t share = std::max(A, cap / active / A * A);
    Bucket b;
    b.even = 0;
    int64_t off = 0;
    for (int r = 0; r < ws; ++r) {
      const int64_t len = std::min(share, p->stream_len[r] - cur[r]);  // <= 0: rank is done
      b.win_off.push_back(off);
      b.win_len.push_back(std::max<int64_t>(len, 0));
      b.win_stream.push_back(cur[r]);
      if (len > 0) {
        off += round_up(len, A);
        cur[r] += len;
      }
    }
    b.elems = off;
    add(std::move(b));
  }
  p->K = int64_t(p->buckets.size());
  // segments: walk each rank's windows (monotone in its stream) against its pieces
  p->segs.assign(p->K, {});
  for (int r = 0; r < ws; ++r) {
    for (const Piece& pc : p->pieces[r]) {
      if (pc.len == 0) continue;
      const int64_t a = pc.stream_off, e = pc.stream_off + pc.len;
      for (int64_t k = 0; k < p->K; ++k) {
        const Bucket& b = p->buckets[k];
        const int64_t lo = std::max(a, b.win_stream[r]);
        const int64_t hi = std::min(e, b.win_stream[r] + b.win_len[r]);
        if (lo >= hi) continue;
        p->segs[k].push_back({pc.param, r, pc.param_off + (lo - a),
                              b.win_off[r] + (lo - b.win_stream[r]), hi - lo});
      }
    }
  }
}

extern "C" {

int zs_plan_create_ex(int64_t n_params, const int64_t* numels, const int64_t* dim0, int ws,
                      int rank, int layout, int64_t align_elems, int64_t window_elems,
                      int bucket_mode, zs_plan** out) {
  ZS_REQUIRE(out != nullptr, "zs_plan_create_ex: out is NULL");
  *out = nullptr;
  ZS_REQUIRE(n_params >= 0, "zs_plan_create_ex: n_params < 0");
  ZS_REQUIRE(n_params == 0 || numels != nullptr, "zs_plan_create_ex: numels is NULL");
  ZS_REQUIRE(ws >= 1, "zs_plan_create_ex: ws must be >= 1 (got %d)", ws);
  ZS_REQUIRE(rank >= 0 && rank < ws, "zs_plan_create_ex: rank %d out of [0,%d)", rank, ws);
  ZS_REQUIRE(layout == ZS_LAYOUT_R || layout == ZS_LAYOUT_Z || layout == ZS_LAYOUT_F,
             "zs_plan_create_ex: unknown layout %d", layout);
  ZS_REQUIRE(align_elems >= 1, "zs_plan_create_ex: align_elems must be >= 1");
  ZS_REQUIRE(window_elems >= 0, "zs_plan_create_ex: window_elems < 0");
  ZS_REQUIRE(bucket_mode == ZS_BUCKETS_RAGGED || bucket_mode == ZS_BUCKETS_PADDED,
             "zs_plan_create_ex: unknown bucket_mode %d", bucket_mode);
  ZS_REQUIRE(layout != ZS_LAYOUT_Z || dim0 != nullptr, "zs_plan_create_ex: layout Z needs dim0");
  for (int64_t i = 0; i < n_params; ++i) {
    ZS_REQUIRE(numels[i] >= 0, "zs_plan_create_ex: numel[%lld] < 0", (long long)i);
    if (layout == ZS_LAYOUT_Z) {
      ZS_REQUIRE((dim0[i] == 0 && numels[i] == 0) || (dim0[i] >= 1 && numels[i] % dim0[i] == 0),
                 "zs_plan_create_ex: param %lld numel %lld not divisible by dim0 %lld", (long long)i,
                 (long long)numels[i], (long long)dim0[i]);
    }
  }

  zs_plan* p = new (std::nothrow) zs_plan();
  if (!p) return zs::fail(ZS_ERR_NOMEM, "zs_plan_create_ex: out of memory");
  p->n = n_params;
  p->ws = ws;
  p->rank = rank;
  p->layout = layout;
  p->align = align_elems;
  p->numel.assign(numels, numels + n_params);
  p->pieces.assign(ws, {});
  p->stream_len.assign(ws, 0);

  if (layout == ZS_LAYOUT_R) {
    for (int r = 0; r < ws; ++r) {
      int64_t s, e, off = 0;
      owner_range(n_params, ws, r, &s, &e);
      for (int64_t i = s; i < e; ++i) {
        p->pieces[r].push_back({i, 0, off, numels[i]});
        off = round_up(off + numels[i], align_elems);
      }
      p->stream_len[r] = off;
    }
  } else if (layout == ZS_LAYOUT_Z) {
    std::vector<int64_t> off(ws, 0);
    for (int64_t i = 0; i < n_params; ++i) {
      const int64_t d0 = dim0[i], row = d0 ? numels[i] / d0 : 0;
      const int64_t cs = (d0 + ws - 1) / ws;  // torch.chunk: ceil(d0/ws) rows per chunk
      for (int r = 0; r < ws; ++r) {
        const int64_t r0 = std::min<int64_t>(int64_t(r) * cs, d0);
        const int64_t r1 = std::min<int64_t>(int64_t(r + 1) * cs, d0);
        const int64_t len = (r1 - r0) * row;
        p->pieces[r].push_back({i, r0 * row, off[r], len});  // zero-length kept: index = param
        off[r] = round_up(off[r] + len, align_elems);
      }
    }
    for (int r = 0; r < ws; ++r) p->stream_len[r] = off[r];
  } else {  // ZS_LAYOUT_F: balanced contiguous slices of the aligned concatenation
    std::vector<int64_t> goff(n_params);
    int64_t T = 0;
    for (int64_t i = 0; i < n_params; ++i) {
      goff[i] = T;
      T = round_up(T + numels[i], align_elems);
    }
    const int64_t S = round_up((T + ws - 1) / ws, align_elems);
    for (int r = 0; r < ws; ++r) {
      const int64_t lo = int64_t(r) * S, hi = lo + S;
      for (int64_t i = 0; i < n_params; ++i) {
        const int64_t a = std::max(lo, goff[i]), b = std::min(hi, goff[i] + numels[i]);
        if (a < b) p->pieces[r].push_back({i, a - goff[i], a - lo, b - a});
      }
      p->stream_len[r] = S;
    }
  }

  p->M = 0;
  p->Lmin = ws > 0 ? p->stream_len[0] : 0;
  for (int r = 0; r < ws; ++r) {
    p->M = std::max(p->M, p->stream_len[r]);
    p->Lmin = std::min(p->Lmin, p->stream_len[r]);
  }
  int64_t W = window_elems == 0 ? p->M : round_up(window_elems, align_elems);
  if (W > p->M) W = p->M;
  p->W = W;
  p->mode = bucket_mode;
  if (W > 0) plan_buckets(p);
  *out = p;
  return ZS_OK;
}

// SURVEY.md §8(b)'s literal signature: the bucket size in bytes of fp32 elements (a bf16 bucket of
// the same plan holds the same elements in half the bytes), 64-element alignment, ragged buckets.
int zs_plan_create(int64_t n_params, const int64_t* numels, const int64_t* dim0, int ws, int rank,
                   int layout, int64_t bucket_bytes, zs_plan** out) {
  ZS_REQUIRE(bucket_bytes >= 0, "zs_plan_create: bucket_bytes < 0");
  ZS_REQUIRE(ws >= 1, "zs_plan_create: ws must be >= 1 (got %d)", ws);
  constexpr int64_t kAlign = 64;
  int64_t window = 0;
  if (bucket_bytes > 0 && ws > 1)
    window = std::max<int64_t>(kAlign, bucket_bytes / (int64_t(ws) * 4) / kAlign * kAlign);
  return zs_plan_create_ex(n_params, numels, dim0, ws, rank, layout, kAlign, window,
                           ZS_BUCKETS_RAGGED, out);
}

int zs_plan_destroy(zs_plan* plan) {
  delete plan;
  return ZS_OK;
}

int zs_plan_info(const zs_plan* p, int64_t* info) {
  ZS_REQUIRE(p && info, "zs_plan_info: NULL argument");
  info[0] = p->n;
  info[1] = p->ws;
  info[2] = p->rank;
  info[3] = p->layout;
  info[4] = p->W;
  info[5] = p->K;
  info[6] = p->M;
  info[7] = p->arena;
  info[8] = p->K_even;
  info[9] = p->mode;
  return ZS_OK;
}

int zs_plan_bucket(const zs_plan* p, int64_t bucket, int64_t* arena_off, int64_t* elems,
                   int* even, int64_t* win_off, int64_t* win_len, int64_t* win_stream) {
  ZS_REQUIRE(p && arena_off && elems && even && win_off && win_len && win_stream,
             "zs_plan_bucket: NULL argument");
  ZS_REQUIRE(bucket >= 0 && bucket < p->K, "zs_plan_bucket: bucket %lld out of range",
             (long long)bucket);
  const Bucket& b = p->buckets[bucket];
  *arena_off = b.arena_off;
  *elems = b.elems;
  *even = b.even;
  for (int r = 0; r < p->ws; ++r) {
    win_off[r] = b.win_off[r];
    win_len[r] = b.win_len[r];
    win_stream[r] = b.win_stream[r];
  }
  return ZS_OK;
}

int zs_plan_owner_range(const zs_plan* p, int rank, int64_t* start, int64_t* end) {
  ZS_REQUIRE(p && start && end, "zs_plan_owner_range: NULL argument");
  ZS_REQUIRE(rank >= 0 && rank < p->ws, "zs_plan_owner_range: rank %d out of range", rank);
  owner_range(p->n, p->ws, rank, start, end);
  return ZS_OK;
}

int zs_plan_owner_of(const zs_plan* p, int64_t i, int* owner) {
  ZS_REQUIRE(p && owner, "zs_plan_owner_of: NULL argument");
  ZS_REQUIRE(i >= 0 && i < p->n, "zs_plan_owner_of: index %lld out of range", (long long)i);
  *owner = owner_of(p->n, p->ws, i);
  return ZS_OK;
}

int zs_plan_stream_len(const zs_plan* p, int rank, int64_t* len) {
  ZS_REQUIRE(p && len, "zs_plan_stream_len: NULL argument");
  ZS_REQUIRE(rank >= 0 && rank < p->ws, "zs_plan_stream_len: rank %d out of range", rank);
  *len = p->stream_len[rank];
  return ZS_OK;
}

int zs_plan_num_pieces(const zs_plan* p, int rank, int64_t* n) {
  ZS_REQUIRE(p && n, "zs_plan_num_pieces: NULL argument");
  ZS_REQUIRE(rank >= 0 && rank < p->ws, "zs_plan_num_pieces: rank %d out of range", rank);
  *n = int64_t(p->pieces[rank].size());
  return ZS_OK;
}

int zs_plan_pieces(const zs_plan* p, int rank, int64_t* param, int64_t* param_off,
                   int64_t* stream_off, int64_t* len) {
  ZS_REQUIRE(p && param && param_off && stream_off && len, "zs_plan_pieces: NULL argument");
  ZS_REQUIRE(rank >= 0 && rank < p->ws, "zs_plan_pieces: rank %d out of range", rank);
  const auto& v = p->pieces[rank];
  for (size_t j = 0; j < v.size(); ++j) {
    param[j] = v[j].param;
    param_off[j] = v[j].param_off;
    stream_off[j] = v[j].stream_off;
    len[j] = v[j].len;
  }
  return ZS_OK;
}

int zs_plan_num_buckets(const zs_plan* p, int64_t* n) {
  ZS_REQUIRE(p && n, "zs_plan_num_buckets: NULL argument");
  *n = p->K;
  return ZS_OK;
}

int zs_plan_bucket_bytes(const zs_plan* p, int64_t bucket, int dtype, int64_t* bytes) {
  ZS_REQUIRE(p && bytes, "zs_plan_bucket_bytes: NULL argument");
  ZS_REQUIRE(bucket >= 0 && bucket < p->K, "zs_plan_bucket_bytes: bucket %lld out of range",
             (long long)bucket);
  ZS_REQUIRE(dtype == ZS_F32 || dtype == ZS_BF16, "zs_plan_bucket_bytes: bad dtype %d", dtype);
  *bytes = p->buckets[bucket].elems * (dtype == ZS_F32 ? 4 : 2);
  return ZS_OK;
}

int zs_pack(zs_plan* p, int64_t bucket, const uint64_t* grad_ptrs, void* bucket_buf, int dtype,
            uintptr_t stream) {
  return bucket_copy(p, bucket, 0, grad_ptrs, reinterpret_cast<uint64_t>(bucket_buf), dtype,
                     stream, "zs_pack");
}

int zs_unpack(zs_plan* p, int64_t bucket, const void* bucket_buf, const uint64_t* param_ptrs,
              int dtype, uintptr_t stream) {
  return bucket_copy(p, bucket, 1, param_ptrs, reinterpret_cast<uint64_t>(bucket_buf), dtype,
                     stream, "zs_unpack");
}

int zs_plan_num_segments(const zs_plan* p, int64_t bucket, int64_t* n) {
  ZS_REQUIRE(p && n, "zs_plan_num_segments: NULL argument");
  ZS_REQUIRE(bucket >= 0 && bucket < p->K, "zs_plan_num_segments: bucket %lld out of range",
             (long long)bucket);
  *n = int64_t(p->segs[bucket].size());
  return ZS_OK;
}

int zs_plan_segments(const zs_plan* p, int64_t bucket, int64_t* param, int64_t* rank,
                     int64_t* param_off, int64_t* buf_off, int64_t* len) {
  ZS_REQUIRE(p && param && rank && param_off && buf_off && len, "zs_plan_segments: NULL argument");
  ZS_REQUIRE(bucket >= 0 && bucket < p->K, "zs_plan_segments: bucket %lld out of range",
             (long long)bucket);
  const auto& v = p->segs[bucket];
  for (size_t j = 0; j < v.size(); ++j) {
    param[j] = v[j].param;
    rank[j] = v[j].rank;
    param_off[j] = v[j].param_off;
    buf_off[j] = v[j].buf_off;
    len[j] = v[j].len;
  }
  return ZS_OK;
}

}  // extern "C"
