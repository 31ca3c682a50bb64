// Internal definitions shared by the libblp.so translation units (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "blp.h"

namespace blp {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what, const char* file, int line);

// BLP_SLOW_HIP_MS=t (profiling): every HIP call made through BLP_HIP / BLP_HIP_OR that takes
// longer than t ms is reported on stderr (call, file:line, thread, start time); 0 / unset = off,
// one relaxed load per call.
int64_t slow_clock();  // ns since the first traced call, or 0 when tracing is off
void slow_check(int64_t t0, const char* what, const char* file, int line);

#define BLP_HIP(call)                                                         \
  do {                                                                        \
    const int64_t _t0 = ::blp::slow_clock();                                  \
    hipError_t _e = (call);                                                   \
    if (_t0) ::blp::slow_check(_t0, #call, __FILE__, __LINE__);               \
    if (_e != hipSuccess) return ::blp::hip_fail(_e, #call, __FILE__, __LINE__); \
  } while (0)

#define BLP_HIP_OR(call, handler)                                              \
  do {                                                                          \
    const int64_t _t0 = ::blp::slow_clock();                                    \
    hipError_t _e = (call);                                                     \
    if (_t0) ::blp::slow_check(_t0, #call, __FILE__, __LINE__);                 \
    if (_e != hipSuccess) return handler(::blp::hip_fail(_e, #call, __FILE__, __LINE__)); \
  } while (0)

#define BLP_CHECK(cond, code, msg)       \
  do {                                   \
    if (!(cond)) return ::blp::fail((code), (msg)); \
  } while (0)

// Device scratch buffer that grows on demand (never shrinks while the handle lives).
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int dev = -1;  // the device the block belongs to (release returns it to that device's cache)
  int reserve(size_t want);
  // back to the device scratch cache after a device sync, or freed; a failed sync (a fault in
  // work queued earlier) is recorded as the last error and returned, and the block is then freed,
  // never cached
  int release();
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};
// empty the device scratch cache of `device` (DevBuf blocks kept for reuse; graph.hip)
void dev_cache_flush(int device);
// bytes the scratch cache of `device` holds (free for any allocation that flushes it)
size_t dev_cache_bytes(int device);
// hipMalloc on the current device; out of memory empties the device scratch cache and tries once
// more (every raw device allocation goes through it: cached blocks must not starve them)
hipError_t dev_malloc(void** p, size_t bytes);
template <class T>
hipError_t dev_malloc(T** p, size_t bytes) {
  return dev_malloc(reinterpret_cast<void**>(p), bytes);
}
// A DevBuf freed when it leaves scope (temporaries on paths with early returns).
struct ScopedBuf : DevBuf {
  ScopedBuf() = default;
  ScopedBuf(const ScopedBuf&) = delete;
  ScopedBuf& operator=(const ScopedBuf&) = delete;
  ~ScopedBuf() { release(); }
};

// Adamic-Adar sums are EXACT. A term w = (log deg)^-1 (similarity.py:121-125) is a double in
// [2^-5, 2) for any degree an int32 CSR can hold, so W = w * 2^58 is an integer below 2^59 with
// no rounding at all. A pair's sum S = Σ W over its CN common neighbours is carried in two u64
// words that any order of addition leaves identical:
//   lo = Σ W mod 2^64 (wrapping adds)      hi = Σ (W >> 32) (exact: < CN * 2^27 < 2^58)
// S - hi * 2^32 = Σ (W mod 2^32) < CN * 2^32 < 2^63, so S = hi * 2^32 + (lo - hi * 2^32 mod 2^64)
// exactly (aa_exact below), and the score is S * 2^-58 rounded once to the nearest double:
// the correctly rounded sum of the reference's own terms, which is what math.fsum returns. The
// reference adds the same terms in Python set order (one rounding per add), so it agrees to a
// few ulps; the oracle's fsum agrees bit for bit, and so do the AUCs computed from them.
constexpr int AA_SHIFT = 58;
constexpr double AA_WMAX = 2.0;  // custom weight tables: [0, 2) keeps W < 2^59 (the scorers' 32-bit step sums of W >> 32)

// S = hi * 2^32 + r as a 128-bit integer (hi64:lo64), from the two accumulator words. More
// generally the high word may count units of 2^hs (hs in [32, 63]) as long as hi * 2^hs <= S and
// S - hi * 2^hs < 2^64: the packed layout of the row-chunk scan (pairs.hip rc_scan) uses hs = 40.
__host__ __device__ inline void aa_exact(unsigned long long lo, unsigned long long hi, unsigned long long* s_hi,
                                         unsigned long long* s_lo, int hs = 32) {
  const unsigned long long a = hi << hs;  // hi * 2^hs mod 2^64; the 128-bit low word of S is lo itself
  *s_lo = lo;
  *s_hi = (hi >> (64 - hs)) + (lo < a ? 1ull : 0ull);
}

// Correctly rounded (nearest-even) conversion of the 128-bit integer hi64:lo64 to double.
__host__ __device__ inline double u128_to_double(unsigned long long h, unsigned long long l) {
  if (h == 0) return (double)l;  // u64 -> f64 rounds once
  const int lz = __builtin_clzll(h);
  unsigned long long m = lz ? (h << lz) | (l >> (64 - lz)) : h;  // top 64 significant bits
  const unsigned long long rest = lz ? l << lz : l;                // bits below them
  m |= rest != 0 ? 1ull : 0ull;  // sticky: bit 0 lies far below the rounding position (bit 10)
  return __builtin_ldexp((double)m, 64 - lz);
}

// Adamic-Adar score of one accumulator pair: S * 2^-58, correctly rounded.
__host__ __device__ inline double aa_value(unsigned long long lo, unsigned long long hi, int hs = 32) {
  unsigned long long sh, sl;
  aa_exact(lo, hi, &sh, &sl, hs);
  return __builtin_ldexp(u128_to_double(sh, sl), -AA_SHIFT);
}

enum KernelId { K_SCORE = 0, K_GROUP = 1, K_SVD_PAIRS = 2, K_SVD_TOPK = 3, K_WALK = 4, K_HOP3 = 5, K_COUNT = 6 };

// Event-pair timer on the graph stream; accumulated lazily when the stats are read.
struct KernelTimer {
  std::vector<hipEvent_t> pending_start, pending_stop;
  std::vector<hipEvent_t> free_events;
  double total_ms = 0.0;
  int64_t launches = 0;
  // a batch's timer also counts into its graph's timer of the same kind (under mirror_mu), so
  // the graph totals need no timing events of their own on the batch's stream
  KernelTimer* mirror = nullptr;
  std::mutex* mirror_mu = nullptr;
};

}  // namespace blp

namespace blp {
constexpr int64_t CI_PAD = 16;  // ids of zero padding before and after d_ci / d_ci_w

// The id sets of a graph's long wedge rows over [lo, hi): bit i of a slot = id lo + i; words
// rounded to whole 16-byte vectors; slot[x] (device, and its host copy) = x's slot or -1.
struct WedgeBitmaps {
  int64_t lo = 0, hi = 0, words = 0, slots = 0;
  int32_t* d_slot = nullptr;
  uint32_t* d_pool = nullptr;
  std::vector<int32_t> h_slot;
};
// The dense wedge-set index over [lo, hi) (round 6, hop3.hip wedge_sets): for EVERY node c of the
// range, W(c) = N(N(c)) ∩ [lo, hi) as a bitmap of `words` u32 at d_pool + (c - lo) * words, and
// d_h2[c - lo] = |W(c) \ {c}| (in a bipartite graph: |H2(c)|, the exact distance-2 set). Built from
// the wedge rows; needs every node of the range with neighbours to hold one.
struct WedgeSets {
  int64_t lo = 0, hi = 0, words = 0;
  uint32_t* d_pool = nullptr;
  int32_t* d_h2 = nullptr;
};
}

struct blp_graph {
  int device = 0;
  int n_cu = 256;
  hipStream_t stream = nullptr;
  int64_t n = 0;    // nodes
  int64_t nnz = 0;  // stored CSR entries (both directions, no self-loops)
  int64_t max_row = 0;  // longest CSR row (graph_finish)
  int64_t* d_rp = nullptr;   // [n+1]
  int32_t* d_ci = nullptr;   // [nnz], CI_PAD readable ids on each side
  long long* d_aaw_fx = nullptr;  // [n] Adamic-Adar weight per node, W = w * 2^58 (exact; or null)
  // weight-coded copy of d_ci for the scorers: ci | code(ci) << id_bits, code 1..255 naming
  // one of the graph's most used weights (d_wtab[code]), 0 = look up d_aaw_fx (or null)
  int32_t* d_ci_w = nullptr;
  int id_bits = 31;
  long long* d_wtab = nullptr;  // [256]; d_wtab[0] = 0
  // dense-row index: rows dense enough in their id range also stored as bitmaps (hot.hip)
  int32_t* d_hot_idx = nullptr;  // [n] hot row number or -1
  void* d_hot_tab = nullptr;     // [n_hot] blp::HotRow
  uint32_t* d_hot_pool = nullptr;
  int64_t n_hot = 0, hot_pool_words = 0;
  std::vector<int32_t> h_hot_idx;
  // wedge rows (wedge.hip): for every node x whose neighbours' rows all hold <= SHORT_ROW_MAX
  // ids, the rows N(z), z in N(x), back to back (d_wedge[4 d_wp[x] .. 4 d_wp[x + 1]), padded to
  // whole 16-byte vectors with a repeat of the row's last id); null when over budget
  int64_t* d_wp = nullptr;    // [n + 1], in 16-byte vectors
  int32_t* d_wedge = nullptr;
  int64_t wedge_vecs = 0;
  std::vector<int64_t> h_wp;  // host copy of d_wp (heavy-source planning)
  // per-node two-hop statistics over N(x) (node2.hip, built on the device): sum of |N(z)|, the id
  // range of N(N(x)) ([lo2, hi2), lo2 = INT32_MAX when empty), max |N(z)|, bit 0: some z is dense
  std::vector<unsigned long long> h_w2;
  std::vector<int32_t> h_lo2, h_hi2, h_maxd;
  std::vector<uint8_t> h_flag2;
  // ... and their device arrays, kept for blp_batch_create's device planning pass (k_plan_pairs)
  unsigned long long* d_w2 = nullptr;
  int32_t *d_lo2 = nullptr, *d_hi2 = nullptr, *d_maxd = nullptr;
  uint8_t* d_flag2 = nullptr;

  // wedge-row bitmaps (hop3.hip, blp::wedge_bitmaps): the SET of ids of each long wedge row over
  // an id range [lo, hi), built on first use per range (the hop-3 mark range; the business
  // batch's universe) and kept with the graph (at most 4 ranges)
  std::vector<blp::WedgeBitmaps> wbm;
  blp::WedgeSets* wset = nullptr;  // the dense wedge-set index (one range; built on first use, under wbm_mu)
  int wedge_users = 0;  // live batches whose plan reads the wedge index or its bitmaps (under wbm_mu)
  std::mutex wbm_mu;  // held across wedge_bitmaps' lookup-or-build (batches are created concurrently)
  // host mirrors used for launch planning (bitmap universe bounds) and the host-built indexes:
  // owned copies (blp_graph_create), or the caller's buffers (blp_graph_create_from_csr, which
  // requires them to outlive the handle)
  std::vector<int64_t> h_rp;
  std::vector<int32_t> h_ci;
  const int64_t* hrp = nullptr;
  const int32_t* hci = nullptr;  // null until first needed when the graph was created without it (host_col_idx)
  std::mutex mirror_mu;          // held while host_col_idx fetches the column mirror
  blp::KernelTimer timers[blp::K_COUNT];
  // the live batches' score / group timers (their pending events are collected into timers[]
  // when the graph's totals are read) and the lock of both
  std::vector<blp::KernelTimer*> live_timers;
  std::mutex timer_mu;
};

namespace blp {
// One dense row: bits [128 * vlo, 128 * (vlo + nvec)) of N(v) at pool words [4*vec_off, ...).
struct HotRow {
  int64_t vec_off;
  int32_t vlo;
  int32_t nvec;
};
// Four consecutive column ids loaded as one 16-byte vector at 4-byte alignment (gfx950 global
// loads accept unaligned dwordx4).
struct __attribute__((aligned(4))) U4a {
  int32_t x, y, z, w;
};
constexpr int SHORT_ROW_MAX = 32;  // the short-row scorer's row bound (pairs.hip SHORT_MAX)
int build_hot_index(blp_graph* g);
int graph_finish(blp_graph* g, const double* aaw);
int build_wedge_index(blp_graph* g);
int build_node2(blp_graph* g);  // after build_hot_index (the dense-row flag)
// Non-blocking streams kept across handles, per device. hipStreamCreate costs milliseconds (it
// sets up a hardware queue); similarity.main would pay it for the parse, the CSR build, the graph
// and each batch. stream_take returns a pooled stream of `device` (the current device) or a new
// one (null on failure, the HIP error recorded); stream_give synchronizes it and pools it (a few
// per device; the rest are destroyed). blp_stream_prewarm fills the pool ahead of time.
// hi: the highest-priority pool -- a stream of the highest priority is never placed on a
// hardware queue of normal-priority streams (blp_batch_create_pair's first batch, so the two
// co-scheduled passes cannot serialize on one queue; with 4 queues per process two pooled
// streams did, config-2 step 3.4 instead of 2.27 ms, r05 call O)
hipStream_t stream_take(int device, bool hi = false);
void stream_give(int device, hipStream_t s, bool hi = false);
hipStream_t stream_new(bool hi);  // a new non-blocking stream (null + error recorded on failure)

// The host column-id mirror, fetched from the device on first use when the graph was created
// without one (blp_graph_create_from_csr with col_idx = NULL: similarity.main's path, whose
// scoring plans on the device and never reads it). Null + error set on failure.
const int32_t* host_col_idx(blp_graph* g);
void free_node2(blp_graph* g);
// per translation unit: load its GPU code object now (hipFuncGetAttributes on one of its kernels)
int preload_ingest();
int preload_staging(int device);  // the graph.txt staging ring of `device` (ingest.hip), allocated once
int preload_csr();
int preload_graph();
int preload_hot();
int preload_node2();
int preload_wedge();
int preload_pairs();
int preload_hop3();
int preload_repr();
constexpr int REPR_SLOT_BYTES = 24;  // repr.h REPR_SLOT
// repr(v) of n device doubles into 24-byte slots at d_out (repr.hip); enqueued on s
int repr_launch(const double* d_v, int64_t n, bool zero_int, char* d_out, int n_cu, hipStream_t s);
// the graph's wedge-row bitmaps over [lo, hi) (built and cached on first use); null with *rc == 0
// when there is no wedge index or no cache slot left
const WedgeBitmaps* wedge_bitmaps(blp_graph* g, int64_t lo, int64_t hi, int* rc);
// the graph's dense wedge-set index over [lo, hi) (built and cached on first use; one range per
// graph); null with *rc == 0 when it cannot be built (no wedge rows, a node of the range with
// neighbours but no wedge row, over the HBM budget BLP_WSET_MB / 25 % of free HBM, or another range cached)
const WedgeSets* wedge_sets(blp_graph* g, int64_t lo, int64_t hi, int* rc);
void free_wedge_index(blp_graph* g);
void free_hot_index(blp_graph* g);
int timer_begin(blp_graph* g, int k, hipEvent_t* start);
int timer_end(blp_graph* g, int k, hipEvent_t start);
int timers_collect(blp_graph* g);
int timer_begin(KernelTimer& t, hipStream_t s, hipEvent_t* start);
int timer_end(KernelTimer& t, hipStream_t s, hipEvent_t start);
int timer_collect(KernelTimer& t);
void timer_release(KernelTimer& t);
int set_device(const blp_graph* g);
// touch every page of a fresh host buffer (>= 8 MB) from up to 16 threads before a pageable
// device-to-host copy into it (graph.hip)
void prefault_host(void* p, size_t bytes);
// Large host buffers (score files, examples, fetched scores): at >= 4 MiB an anonymous mapping,
// 2 MiB aligned, advised as transparent huge pages (the GPU boxes run THP in madvise mode), so
// first touch takes one fault per 2 MiB instead of per 4 KiB and the release is one munmap of a
// few hundred pages. Smaller sizes (and BLP_NO_THP=1) use malloc. Null on failure.
void* host_alloc(size_t bytes);
// A host<->device copy of `bytes` on stream st, complete on return.
int copy_sync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t st);
void host_free(void* p, size_t bytes);
// std allocator over host_alloc that leaves elements uninitialised on resize()
template <class T>
struct HostAlloc {
  using value_type = T;
  HostAlloc() = default;
  template <class U>
  HostAlloc(const HostAlloc<U>&) noexcept {}
  T* allocate(size_t n) {
    void* p = host_alloc(n * sizeof(T));
    if (!p) throw std::bad_alloc();
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t n) noexcept { host_free(p, n * sizeof(T)); }
  template <class U>
  void construct(U* p) noexcept {
    ::new ((void*)p) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new ((void*)p) U(std::forward<A>(a)...);
  }
  template <class U>
  bool operator==(const HostAlloc<U>&) const noexcept { return true; }
  template <class U>
  bool operator!=(const HostAlloc<U>&) const noexcept { return false; }
};
template <class T>
using HostVec = std::vector<T, HostAlloc<T>>;
// the device CSR of m dense endpoint pairs already in HBM on `device` (csr.hip; blp_csr_build_device
// with sync_device, which first waits for all work queued on the device)
int csr_build(int device, const int32_t* d_a, const int32_t* d_b, int64_t m, int64_t n, blp_csr** out,
              bool sync_device);
// d_idx = 0..n-1 ordered by d_keys descending, ties by index (csr.hip; enqueued on st, then synced)
int order_desc_u64(const uint64_t* d_keys, int64_t n, int32_t* d_idx, hipStream_t st);
}  // namespace blp
