// Graph handle, host CSR builder, errors, timers (libblp.so).
//
// Replaces snap.LoadEdgeList(snap.PUNGraph, ...) (similarity.py:16) and SNAP's degree
// lookups (similarity.py:121): the undirected simple graph lives in HBM as one CSR over
// dense node ids, both directions stored, rows sorted ascending, int64 row offsets and
// int32 column ids.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cmath>
#include <cstring>
#include <mutex>
#include <thread>
#include <map>
#include <unordered_map>

#include <sys/mman.h>

#include <chrono>

#include "blp_internal.h"

namespace {

__global__ void k_code_ids(const int32_t* __restrict__ ci, int64_t nnz, const uint8_t* __restrict__ ncode, int bits,
                           int32_t* __restrict__ out) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz; e += (int64_t)gridDim.x * blockDim.x) {
    const int32_t v = ci[e];
    out[e] = v | (int32_t)((uint32_t)ncode[v] << bits);
  }
}

__global__ void k_noop() {}  // blp_stream_prewarm: the first work of a new stream

}  // namespace

namespace blp {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

int hip_fail(hipError_t e, const char* what, const char* file, int line) {
  char buf[512];
  snprintf(buf, sizeof(buf), "%s failed: %s (%d) at %s:%d", what, hipGetErrorString(e), (int)e, file, line);
  set_error(buf);
  return BLP_E_HIP_BASE - (int)e;
}

namespace {
std::atomic<int> g_slow_state{-1};  // -1 unread, 0 off, else the threshold in microseconds
std::chrono::steady_clock::time_point g_slow_t0;
std::mutex g_slow_mu;
}  // namespace

int64_t slow_clock() {
  int st = g_slow_state.load(std::memory_order_relaxed);
  if (st == 0) return 0;
  if (st < 0) {
    std::lock_guard<std::mutex> lk(g_slow_mu);
    st = g_slow_state.load();
    if (st < 0) {
      const char* e = getenv("BLP_SLOW_HIP_MS");
      const double ms = e ? atof(e) : 0.0;
      g_slow_t0 = std::chrono::steady_clock::now();
      st = ms > 0 ? std::max(1, (int)(ms * 1000)) : 0;
      g_slow_state.store(st);
    }
    if (st == 0) return 0;
  }
  return std::max<int64_t>(1, std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                                                     g_slow_t0).count());
}

void slow_check(int64_t t0, const char* what, const char* file, int line) {
  const int64_t t1 = slow_clock();
  if (t1 && (t1 - t0) / 1000 >= g_slow_state.load(std::memory_order_relaxed)) {
    const char* f = strrchr(file, '/');
    fprintf(stderr, "[blp slow hip] %8.3f ms at t=%9.3f ms tid %zx %s:%d %s\n", (t1 - t0) * 1e-6, t0 * 1e-6,
            (size_t)std::hash<std::thread::id>()(std::this_thread::get_id()) & 0xffff, f ? f + 1 : file, line, what);
  }
}

// Device scratch cache (round 5). Freeing a large device buffer and allocating a new one made the
// next kernels wait 16-26 ms in similarity.main (the driver clears released VRAM before it is
// handed out again; profiles/r05_e2e_*slow_calls.txt). Released DevBuf blocks are kept per device
// (after a device sync, which hipFree implied) up to a budget (BLP_DEV_CACHE_MB, default 8192; 0
// disables) and handed back to a later reservation of at most the same size and at least half;
// an allocation that runs out of memory empties the cache and tries again.
namespace {
struct DevCache {
  std::multimap<size_t, void*> blocks;
  size_t bytes = 0;
};
std::mutex g_dc_mu;
std::vector<DevCache> g_dc;  // [device]
size_t dc_budget() {
  static const size_t b = getenv("BLP_DEV_CACHE_MB") ? (size_t)std::max(0ll, atoll(getenv("BLP_DEV_CACHE_MB"))) << 20
                                                       : size_t(8192) << 20;
  return b;
}
int current_device() {
  int d = 0;
  return hipGetDevice(&d) == hipSuccess ? d : 0;
}
}  // namespace

void dev_cache_flush(int device) {
  std::vector<void*> drop;
  {
    std::lock_guard<std::mutex> lk(g_dc_mu);
    if ((size_t)device >= g_dc.size()) return;
    for (auto& kv : g_dc[device].blocks) drop.push_back(kv.second);
    g_dc[device].blocks.clear();
    g_dc[device].bytes = 0;
  }
  for (void* q : drop) (void)hipFree(q);
}

int DevBuf::reserve(size_t want) {
  if (want <= bytes && p) return BLP_OK;
  if (p) release();
  const size_t sz = std::max<size_t>(want, 256);
  const int dev = current_device();
  if (dc_budget()) {
    std::lock_guard<std::mutex> lk(g_dc_mu);
    if ((size_t)dev < g_dc.size()) {
      DevCache& c = g_dc[dev];
      auto it = c.blocks.lower_bound(sz);
      if (it != c.blocks.end() && it->first <= 2 * sz) {
        p = it->second;
        bytes = it->first;
        this->dev = dev;
        c.bytes -= it->first;
        c.blocks.erase(it);
        return BLP_OK;
      }
    }
  }
  hipError_t e = hipMalloc(&p, sz);
  if (e == hipErrorOutOfMemory && dc_budget()) {
    (void)hipGetLastError();
    dev_cache_flush(dev);
    e = hipMalloc(&p, sz);
  }
  if (e != hipSuccess) {
    p = nullptr;
    this->dev = -1;
    return hip_fail(e, "hipMalloc (DevBuf)", __FILE__, __LINE__);
  }
  bytes = sz;
  this->dev = dev;
  return BLP_OK;
}

int DevBuf::release() {
  int rc = BLP_OK;
  if (p) {
    const int64_t t0 = slow_clock();
    bool kept = false;
    const size_t budget = dc_budget();
    if (budget && bytes <= budget && dev >= 0) {
      // what hipFree implied: nothing queued on the device still reads the block (the block's
      // own device: the caller may have another one current)
      int cur = -1;
      (void)hipGetDevice(&cur);
      if (cur != dev) (void)hipSetDevice(dev);
      const hipError_t se = hipDeviceSynchronize();
      if (cur != dev && cur >= 0) (void)hipSetDevice(cur);
      if (se != hipSuccess) {
        rc = hip_fail(se, "hipDeviceSynchronize (DevBuf::release: work queued before the release failed)", __FILE__,
                      __LINE__);
      } else {
        std::lock_guard<std::mutex> lk(g_dc_mu);
        if ((size_t)dev >= g_dc.size()) g_dc.resize((size_t)dev + 1);
        DevCache& c = g_dc[dev];
        if (c.bytes + bytes <= budget) {
          c.blocks.emplace(bytes, p);
          c.bytes += bytes;
          kept = true;
        }
      }
    }
    if (!kept) (void)hipFree(p);
    if (t0) slow_check(t0, "DevBuf::release", __FILE__, __LINE__);
  }
  p = nullptr;
  bytes = 0;
  dev = -1;
  return rc;
}

size_t dev_cache_bytes(int device) {
  std::lock_guard<std::mutex> lk(g_dc_mu);
  return (size_t)device < g_dc.size() ? g_dc[device].bytes : 0;
}

hipError_t dev_malloc(void** p, size_t bytes) {
  hipError_t e = hipMalloc(p, bytes);
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();
    const int dev = current_device();
    if (dev_cache_bytes(dev)) {
      dev_cache_flush(dev);
      e = hipMalloc(p, bytes);
    }
  }
  if (e != hipSuccess) *p = nullptr;
  return e;
}

int set_device(const blp_graph* g) {
  BLP_HIP(hipSetDevice(g->device));
  return BLP_OK;
}

// Touch every page of a fresh host buffer from up to 16 threads: a pageable device-to-host copy
// into never-touched memory takes its page faults one by one on the copying thread (80 MB of
// col_idx at config 2: ~20 ms serial, a few ms spread over the threads). Buffers under 8 MB are
// left alone.
void prefault_host(void* p, size_t bytes) {
  if (!p || bytes < (size_t(8) << 20)) return;
  const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([=]() {
      volatile char* q = static_cast<volatile char*>(p);
      for (size_t o = bytes * t / nt / 4096 * 4096; o < bytes * (t + 1) / nt; o += 4096) q[o] = 0;
    });
  for (auto& x : th) x.join();
}

namespace {
constexpr size_t HUGE_MIN = size_t(4) << 20, HUGE_PAGE = size_t(2) << 20;
bool thp_on() {
  static const bool on = !getenv("BLP_NO_THP");
  return on;
}
}  // namespace

void* host_alloc(size_t bytes) {
  if (bytes < HUGE_MIN || !thp_on()) return malloc(std::max<size_t>(bytes, 1));
  // over-map by one huge page, then trim to a 2 MiB aligned span (the kernel backs only aligned
  // 2 MiB ranges with huge pages)
  const size_t len = (bytes + HUGE_PAGE - 1) / HUGE_PAGE * HUGE_PAGE;
  void* m = mmap(nullptr, len + HUGE_PAGE, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (m == MAP_FAILED) return nullptr;
  const uintptr_t b = (uintptr_t)m, a = (b + HUGE_PAGE - 1) / HUGE_PAGE * HUGE_PAGE;
  if (a > b) munmap(m, a - b);
  if (b + HUGE_PAGE > a) munmap((void*)(a + len), b + HUGE_PAGE - a);
  madvise((void*)a, len, MADV_HUGEPAGE);
  return (void*)a;
}

int copy_sync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t st) {
  if (!bytes) return BLP_OK;
  hipError_t err = hipMemcpyAsync(dst, src, bytes, kind, st);
  if (err == hipSuccess) err = hipStreamSynchronize(st);
  if (err != hipSuccess) return hip_fail(err, "copy_sync", __FILE__, __LINE__);
  return BLP_OK;
}

void host_free(void* p, size_t bytes) {
  if (!p) return;
  if (bytes < HUGE_MIN || !thp_on()) {
    free(p);
    return;
  }
  munmap(p, (bytes + HUGE_PAGE - 1) / HUGE_PAGE * HUGE_PAGE);
}

// A batch's timers (mirror_mu set: the graph's lock) are also read by the graph's stats calls,
// which may come from another host thread: their lists are touched under that lock. The graph's
// own timers (mirror_mu null) belong to the graph's calls.
namespace {
struct TimerLock {
  std::mutex* m;
  explicit TimerLock(const KernelTimer& t) : m(t.mirror_mu) {
    if (m) m->lock();
  }
  ~TimerLock() {
    if (m) m->unlock();
  }
};

int timer_collect_locked(KernelTimer& t) {
  double added = 0.0;
  int rc = BLP_OK;
  size_t i = 0;
  for (; i < t.pending_stop.size(); ++i) {
    hipError_t e = hipEventSynchronize(t.pending_stop[i]);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, t.pending_start[i], t.pending_stop[i]);
    if (e != hipSuccess) {
      rc = hip_fail(e, "timer_collect", __FILE__, __LINE__);
      break;
    }
    t.total_ms += ms;
    added += ms;
    t.free_events.push_back(t.pending_start[i]);
    t.free_events.push_back(t.pending_stop[i]);
  }
  t.pending_start.erase(t.pending_start.begin(), t.pending_start.begin() + i);
  t.pending_stop.erase(t.pending_stop.begin(), t.pending_stop.begin() + i);
  if (t.mirror) t.mirror->total_ms += added;  // (the mirror is guarded by the same lock)
  return rc;
}
}  // namespace

int timer_begin(KernelTimer& t, hipStream_t s, hipEvent_t* start) {
  TimerLock lk(t);
  if (t.free_events.empty()) {
    hipEvent_t e;
    BLP_HIP(hipEventCreate(&e));
    t.free_events.push_back(e);
  }
  *start = t.free_events.back();
  t.free_events.pop_back();
  BLP_HIP(hipEventRecord(*start, s));
  return BLP_OK;
}

int timer_end(KernelTimer& t, hipStream_t s, hipEvent_t start) {
  TimerLock lk(t);
  hipEvent_t stop;
  if (t.free_events.empty()) {
    BLP_HIP(hipEventCreate(&stop));
  } else {
    stop = t.free_events.back();
    t.free_events.pop_back();
  }
  BLP_HIP(hipEventRecord(stop, s));
  t.pending_start.push_back(start);
  t.pending_stop.push_back(stop);
  t.launches++;
  if (t.mirror) t.mirror->launches++;
  // keep the pending list bounded: fold finished pairs in as we go
  if (t.pending_stop.size() > 4096) return timer_collect_locked(t);
  return BLP_OK;
}

int timer_collect(KernelTimer& t) {
  TimerLock lk(t);
  return timer_collect_locked(t);
}

void timer_release(KernelTimer& t) {
  for (auto e : t.pending_start) (void)hipEventDestroy(e);
  for (auto e : t.pending_stop) (void)hipEventDestroy(e);
  for (auto e : t.free_events) (void)hipEventDestroy(e);
  t.pending_start.clear();
  t.pending_stop.clear();
  t.free_events.clear();
}

int timer_begin(blp_graph* g, int k, hipEvent_t* start) { return timer_begin(g->timers[k], g->stream, start); }

int timer_end(blp_graph* g, int k, hipEvent_t start) { return timer_end(g->timers[k], g->stream, start); }

int timers_collect(blp_graph* g) {
  std::vector<KernelTimer*> live;
  {
    std::lock_guard<std::mutex> lk(g->timer_mu);
    live = g->live_timers;
  }
  for (KernelTimer* t : live) {  // (the batches' own calls are not concurrent with this one)
    int rc = timer_collect(*t);
    if (rc) return rc;
  }
  for (int k = 0; k < K_COUNT; ++k) {
    int rc = timer_collect(g->timers[k]);
    if (rc) return rc;
  }
  return BLP_OK;
}

// Weight-coded column ids: the scorers' Adamic-Adar term of a common neighbour w is a
// per-node weight (similarity.py:121-125, a function of deg(w)). Instead of gathering aaw[w]
// per hit, the id stream itself carries a code in its free high bits: codes 1..255 go to the
// distinct weights with the most occurrences in col_idx (on a review graph the few distinct
// user degrees cover every user), code 0 means "gather aaw". Only when the ids leave at least
// one free bit below the sign bit.
int build_weight_codes(blp_graph* g, const int64_t* row_ptr, const std::vector<long long>& fx) {
  const int64_t n = g->n, nnz = g->nnz;
  int bits = 1;
  while (bits < 31 && (int64_t(1) << bits) < n) ++bits;
  const int cbits = std::min(8, 31 - bits);
  int max_codes = (1 << cbits) - 1;
  if (const char* e = getenv("BLP_WCODES")) max_codes = std::min(max_codes, std::max(0, atoi(e)));  // test knob
  std::vector<long long> wtab(256, 0);
  BLP_HIP(dev_malloc(&g->d_wtab, sizeof(long long) * 256));  // always: code 0 reads wtab[0]
  BLP_HIP(hipMemcpy(g->d_wtab, wtab.data(), sizeof(long long) * 256, hipMemcpyHostToDevice));
  if (max_codes <= 0 || nnz == 0) return BLP_OK;
  const bool gprof = getenv("BLP_GRAPH_PROF") != nullptr;
  auto t_prev = std::chrono::steady_clock::now();
  auto stage = [&](const char* what) {
    if (!gprof) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "  codes %-8s %.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t_prev).count());
    t_prev = t;
  };
  // occurrences per distinct weight, node slices on up to 16 threads (a handful of distinct
  // weights: each thread's table stays small), then merged
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({16, (int64_t)std::thread::hardware_concurrency(), n >> 16}));
  std::vector<std::unordered_map<long long, int64_t>> part_uses((size_t)nt);
  auto par = [&](auto fn) {
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(fn, t);
    fn(0);
    for (auto& h : th) h.join();
  };
  par([&](int t) {
    auto& m = part_uses[t];
    for (int64_t i = n * t / nt, e = n * (t + 1) / nt; i < e; ++i) m[fx[i]] += row_ptr[i + 1] - row_ptr[i];
  });
  std::unordered_map<long long, int64_t> uses;
  for (const auto& m : part_uses)
    for (const auto& kv : m) uses[kv.first] += kv.second;
  std::vector<std::pair<int64_t, long long>> order;
  order.reserve(uses.size());
  for (const auto& kv : uses)
    if (kv.second > 0) order.emplace_back(-kv.second, kv.first);
  std::sort(order.begin(), order.end());
  std::unordered_map<long long, int> code;
  for (size_t j = 0; j < order.size() && (int)j < max_codes; ++j) {
    wtab[j + 1] = order[j].second;
    code[order[j].second] = (int)j + 1;
  }
  stage("uses");
  std::vector<uint8_t> ncode((size_t)n, 0);
  par([&](int t) {
    for (int64_t i = n * t / nt, e = n * (t + 1) / nt; i < e; ++i) {
      const auto it = code.find(fx[i]);
      if (it != code.end()) ncode[i] = (uint8_t)it->second;
    }
  });
  stage("ncode");
  uint8_t* d_ncode = nullptr;
  BLP_HIP(hipMemcpy(g->d_wtab, wtab.data(), sizeof(long long) * 256, hipMemcpyHostToDevice));
  BLP_HIP(dev_malloc(&g->d_ci_w, sizeof(int32_t) * (nnz + 2 * CI_PAD)));
  BLP_HIP(hipMemset(g->d_ci_w, 0, sizeof(int32_t) * (nnz + 2 * CI_PAD)));
  g->d_ci_w += CI_PAD;
  stage("alloc");
  BLP_HIP(dev_malloc(&d_ncode, (size_t)n));
  BLP_HIP(hipMemcpy(d_ncode, ncode.data(), (size_t)n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_code_ids, dim3((unsigned)std::min<int64_t>((nnz + 255) / 256, 1 << 20)), dim3(256), 0, g->stream,
                     g->d_ci, nnz, d_ncode, bits, g->d_ci_w);
  BLP_HIP(hipGetLastError());
  BLP_HIP(hipStreamSynchronize(g->stream));
  BLP_HIP(hipFree(d_ncode));
  stage("kernel");
  g->id_bits = bits;
  return BLP_OK;
}

// Adamic-Adar weights as integers W = w * 2^58 (blp_internal.h). Every weight the reference
// produces, (log d)^-1 for 2 <= d < 2^31, lies in [2^-5, 2) and converts exactly; a custom table
// must hold weights in [0, 2) (smaller weights than 2^-6 round to the 2^-58 grid once, here).
int aa_weights_fixed(const double* aaw, int64_t n, std::vector<long long>& fx) {
  const double scale = std::ldexp(1.0, AA_SHIFT);
  fx.resize((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    const double w = aaw[i];
    if (!(w >= 0.0 && w < AA_WMAX))
      return fail(BLP_E_ARG, "blp_graph_create: aa_weight entries must lie in [0, 2) (node " + std::to_string(i) + ")");
    fx[i] = (long long)(unsigned long long)std::nearbyint(w * scale);
  }
  return BLP_OK;
}

// Everything a graph handle derives from its CSR once g->d_rp / g->d_ci (device) and
// g->hrp / g->hci (host mirrors) are in place: stream, CU count, fixed-point Adamic-Adar
// weights and the weight-coded id stream, the dense-row index and the wedge rows.
int graph_finish(blp_graph* g, const double* aaw) {
  // BLP_GRAPH_PROF: stage wall times on stderr (profiling only; the stages run either way)
  const bool gprof = getenv("BLP_GRAPH_PROF") != nullptr;
  auto t_prev = std::chrono::steady_clock::now();
  auto stage = [&](const char* what) {
    if (!gprof) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "graph_finish %-8s %.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t_prev).count());
    t_prev = t;
  };
  int n_cu = 0;  // one attribute, not hipGetDeviceProperties' full query (~5 ms)
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, g->device) == hipSuccess && n_cu > 0)
    g->n_cu = n_cu;
  if (!g->stream && !(g->stream = stream_take(g->device))) return BLP_E_HIP_BASE;
  const int64_t n = g->n;
  g->max_row = 0;
  for (int64_t v = 0; v < n; ++v) g->max_row = std::max<int64_t>(g->max_row, g->hrp[v + 1] - g->hrp[v]);
  stage("setup");
  if (aaw) {
    std::vector<long long> fx;
    if (int rc = aa_weights_fixed(aaw, n, fx)) return rc;
    BLP_HIP(dev_malloc(&g->d_aaw_fx, sizeof(long long) * std::max<int64_t>(n, 1)));
    if (n) {
      if (int rc = copy_sync(g->d_aaw_fx, fx.data(), sizeof(long long) * n, hipMemcpyHostToDevice, g->stream)) return rc;
    }
    stage("weights");
    int rc = build_weight_codes(g, g->hrp, fx);
    if (rc != BLP_OK) return rc;
    stage("codes");
  }
  int rc = build_hot_index(g);
  if (rc != BLP_OK) return rc;
  stage("hot");
  if ((rc = build_node2(g)) != BLP_OK) return rc;
  stage("node2");
  rc = build_wedge_index(g);
  stage("wedge");
  return rc;
}

}  // namespace blp

namespace blp {
namespace {
std::mutex g_stream_mu;
std::condition_variable g_stream_cv;
int g_prewarming = 0;  // blp_stream_prewarm calls creating streams (under g_stream_mu)
std::vector<std::vector<hipStream_t>> g_stream_pool;     // [device]
std::vector<std::vector<hipStream_t>> g_stream_pool_hi;  // [device] highest-priority streams
constexpr size_t STREAM_POOL_CAP = 16;
}  // namespace

hipStream_t stream_take(int device, bool hi) {
  {
    std::unique_lock<std::mutex> lk(g_stream_mu);
    // a prewarm creating streams: wait for them rather than overlap this caller's first GPU work
    // with the stream creation (that overlap preceded 27-39 ms stalls, r05_e2e_final_ab)
    g_stream_cv.wait(lk, [] { return g_prewarming == 0; });
    auto& pool = hi ? g_stream_pool_hi : g_stream_pool;
    if ((size_t)device < pool.size() && !pool[device].empty()) {
      hipStream_t s = pool[device].back();
      pool[device].pop_back();
      return s;
    }
  }
  return stream_new(hi);
}

hipStream_t stream_new(bool hi) {
  hipStream_t s = nullptr;
  hipError_t e;
  if (hi) {
    int least = 0, greatest = 0;
    e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest);
  } else {
    e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  }
  if (e != hipSuccess) {
    hip_fail(e, "hipStreamCreate", __FILE__, __LINE__);
    return nullptr;
  }
  return s;
}

void stream_give(int device, hipStream_t s, bool hi) {
  if (!s) return;
  (void)hipStreamSynchronize(s);
  {
    std::lock_guard<std::mutex> lk(g_stream_mu);
    auto& pool = hi ? g_stream_pool_hi : g_stream_pool;
    if ((size_t)device >= pool.size()) pool.resize((size_t)device + 1);
    if (pool[device].size() < STREAM_POOL_CAP) {
      pool[device].push_back(s);
      return;
    }
  }
  (void)hipStreamDestroy(s);
}

const int32_t* host_col_idx(blp_graph* g) {
  std::lock_guard<std::mutex> lk(g->mirror_mu);
  static const int32_t none = 0;  // an empty graph's mirror: nothing to read
  if (g->hci || g->nnz == 0) return g->hci ? g->hci : &none;
  try {
    g->h_ci.resize((size_t)g->nnz);
  } catch (...) {
    fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "host_col_idx: host mirror allocation");
    return nullptr;
  }
  prefault_host(g->h_ci.data(), 4 * (size_t)g->nnz);
  if (hipSetDevice(g->device) != hipSuccess ||
      hipMemcpy(g->h_ci.data(), g->d_ci, 4 * (size_t)g->nnz, hipMemcpyDeviceToHost) != hipSuccess) {
    fail(BLP_E_HIP_BASE, "host_col_idx: fetch of the column ids failed");
    return nullptr;
  }
  g->hci = g->h_ci.data();
  return g->hci;
}
}  // namespace blp

using namespace blp;

extern "C" {

const char* blp_last_error(void) { return g_last_error.c_str(); }

const char* blp_version(void) { return "libblp 0.1 (gfx950)"; }

int blp_host_alloc(size_t bytes, void** out) {
  BLP_CHECK(out, BLP_E_ARG, "blp_host_alloc: null out");
  *out = host_alloc(bytes);
  BLP_CHECK(*out, BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_host_alloc: out of host memory");
  return BLP_OK;
}

int blp_host_free(void* p, size_t bytes) {
  host_free(p, bytes);
  return BLP_OK;
}

int blp_device_count(int* n) {
  BLP_CHECK(n, BLP_E_ARG, "blp_device_count: null out");
  BLP_HIP(hipGetDeviceCount(n));
  return BLP_OK;
}

int blp_stream_prewarm(int device, int n) {
  BLP_CHECK(n >= 0 && n <= 16, BLP_E_ARG, "blp_stream_prewarm: 0 <= n <= 16");
  BLP_HIP(hipSetDevice(device));
  // first the pinned staging ring of the graph.txt upload: similarity.main's parse, on the other
  // thread, reaches it within milliseconds
  if (preload_staging(device)) return BLP_E_HIP_BASE;
  // Top the pool up to n streams (BLP_PREWARM_ALWAYS=1: always create n, the round-4 behaviour),
  // run one empty kernel on each new one, and hold stream_take until they are in the pool: the
  // caller's first GPU work then neither creates a stream nor overlaps this thread's creation (an
  // overlap that preceded 27-39 ms stalls in similarity.main, profiles/r05_e2e_final_ab_slow_calls.txt).
  size_t have = 0, hi_have = 0;
  {
    std::lock_guard<std::mutex> lk(g_stream_mu);
    if ((size_t)device < g_stream_pool.size()) have = g_stream_pool[device].size();
    if ((size_t)device < g_stream_pool_hi.size()) hi_have = g_stream_pool_hi[device].size();
    if (getenv("BLP_PREWARM_ALWAYS")) have = 0;
    if ((size_t)n > have || (n > 0 && hi_have == 0)) ++g_prewarming;  // stream_take waits until these are in the pool
  }
  const bool latched = (size_t)n > have || (n > 0 && hi_have == 0);
  std::vector<hipStream_t> made;
  hipError_t err = hipSuccess;
  for (int i = (int)std::min<size_t>(have, (size_t)n); i < n && err == hipSuccess; ++i) {
    hipStream_t s = nullptr;
    err = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (err != hipSuccess) break;
    made.push_back(s);
    hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, s);
    err = hipGetLastError();
  }
  // and one highest-priority stream (blp_batch_create_pair's first batch: its own hardware queue)
  hipStream_t made_hi = nullptr;
  if (err == hipSuccess && n > 0 && hi_have == 0) {
    if (!(made_hi = stream_new(true))) {
      err = hipErrorOutOfMemory;
    } else {
      hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, made_hi);
      err = hipGetLastError();
    }
  }
  for (hipStream_t s : made) (void)hipStreamSynchronize(s);
  if (made_hi) (void)hipStreamSynchronize(made_hi);
  std::vector<hipStream_t> extra;  // past the pool's cap (concurrent prewarms): destroyed
  if (latched) {
    std::lock_guard<std::mutex> lk(g_stream_mu);
    if ((size_t)device >= g_stream_pool.size()) g_stream_pool.resize((size_t)device + 1);
    if ((size_t)device >= g_stream_pool_hi.size()) g_stream_pool_hi.resize((size_t)device + 1);
    for (hipStream_t s : made) {
      if (g_stream_pool[device].size() < STREAM_POOL_CAP)
        g_stream_pool[device].push_back(s);
      else
        extra.push_back(s);
    }
    if (made_hi) {
      if (g_stream_pool_hi[device].size() < STREAM_POOL_CAP)
        g_stream_pool_hi[device].push_back(made_hi);
      else
        extra.push_back(made_hi);
    }
    --g_prewarming;
  }
  for (hipStream_t s : extra) (void)hipStreamDestroy(s);
  g_stream_cv.notify_all();
  if (err != hipSuccess) return hip_fail(err, "blp_stream_prewarm", __FILE__, __LINE__);
  // then the code objects of similarity.main's kernels, in the order it first launches them
  // (BLP_NO_PRELOAD=1: A/B knob, each loads on its first launch instead)
  if (!getenv("BLP_NO_PRELOAD"))
    for (int (*f)() : {preload_ingest, preload_csr, preload_graph, preload_hot, preload_node2, preload_wedge,
                       preload_pairs, preload_hop3, preload_repr})
      if (f()) return fail(BLP_E_HIP_BASE, "blp_stream_prewarm: kernel code object load failed");
  return BLP_OK;
}

int blp_device_sync(int device) {
  BLP_HIP(hipSetDevice(device));
  BLP_HIP(hipDeviceSynchronize());
  return BLP_OK;
}

int blp_csr_from_edges(int64_t n, int64_t m, const int32_t* a, const int32_t* b, int64_t* row_ptr,
                       int32_t* col_idx, uint8_t* self_loop, int64_t* nnz_out) {
  BLP_CHECK(n >= 0 && m >= 0 && row_ptr && nnz_out && (m == 0 || (a && b && col_idx)), BLP_E_ARG,
            "blp_csr_from_edges: bad arguments");
  BLP_CHECK(n < (int64_t(1) << 31), BLP_E_ARG, "blp_csr_from_edges: n_nodes must fit int32");
  std::vector<int64_t> cnt(n + 1, 0);
  if (self_loop) std::memset(self_loop, 0, (size_t)n);
  for (int64_t i = 0; i < m; ++i) {
    int32_t u = a[i], v = b[i];
    if (u < 0 || v < 0 || u >= n || v >= n) return fail(BLP_E_ARG, "blp_csr_from_edges: node id out of range");
    if (u == v) {
      if (self_loop) self_loop[u] = 1;
      continue;
    }
    cnt[u + 1]++;
    cnt[v + 1]++;
  }
  for (int64_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
  std::vector<int64_t> cur(cnt.begin(), cnt.end() - 1);
  for (int64_t i = 0; i < m; ++i) {
    int32_t u = a[i], v = b[i];
    if (u == v) continue;
    col_idx[cur[u]++] = v;
    col_idx[cur[v]++] = u;
  }
  // sort each row and drop duplicate edges (SNAP keeps one copy of a multi-edge)
  int64_t w = 0;
  row_ptr[0] = 0;
  for (int64_t r = 0; r < n; ++r) {
    int64_t s = cnt[r], e = cnt[r + 1];
    std::sort(col_idx + s, col_idx + e);
    int64_t start = w;
    for (int64_t i = s; i < e; ++i)
      if (i == s || col_idx[i] != col_idx[i - 1]) col_idx[w++] = col_idx[i];
    (void)start;
    row_ptr[r + 1] = w;
  }
  *nnz_out = w;
  return BLP_OK;
}

int blp_graph_create(const int64_t* row_ptr, const int32_t* col_idx, int64_t n, const double* aaw,
                     int device, blp_graph** out) {
  BLP_CHECK(out && row_ptr && n >= 0, BLP_E_ARG, "blp_graph_create: bad arguments");
  BLP_CHECK(n < (int64_t(1) << 31), BLP_E_ARG, "blp_graph_create: n_nodes must fit int32");
  int64_t nnz = row_ptr[n];
  BLP_CHECK(nnz >= 0 && (nnz == 0 || col_idx), BLP_E_ARG, "blp_graph_create: bad row_ptr/col_idx");
  for (int64_t i = 0; i < n; ++i)
    BLP_CHECK(row_ptr[i] <= row_ptr[i + 1], BLP_E_ARG, "blp_graph_create: row_ptr not monotone");
  for (int64_t i = 0; i < nnz; ++i)
    BLP_CHECK(col_idx[i] >= 0 && col_idx[i] < n, BLP_E_ARG, "blp_graph_create: col_idx out of range");
  int ndev = 0;
  BLP_HIP(hipGetDeviceCount(&ndev));
  BLP_CHECK(device >= 0 && device < ndev, BLP_E_ARG, "blp_graph_create: no such device");
  BLP_HIP(hipSetDevice(device));
  blp_graph* g = new blp_graph();
  g->device = device;
  g->n = n;
  g->nnz = nnz;
  int rc = BLP_OK;
  if ((rc = [&]() -> int {
         BLP_HIP(dev_malloc(&g->d_rp, sizeof(int64_t) * (n + 1)));
         // padded on both sides (CI_PAD ids): the scorers read rows in 16-byte vectors, up to
         // 15 ids past a row end or before a row start
         BLP_HIP(dev_malloc(&g->d_ci, sizeof(int32_t) * (nnz + 2 * CI_PAD)));
         BLP_HIP(hipMemset(g->d_ci, 0, sizeof(int32_t) * (nnz + 2 * CI_PAD)));
         g->d_ci += CI_PAD;
         BLP_HIP(hipMemcpy(g->d_rp, row_ptr, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice));
         if (nnz) BLP_HIP(hipMemcpy(g->d_ci, col_idx, sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
         return BLP_OK;
       }()) != BLP_OK) {
    blp_graph_destroy(g);
    return rc;
  }
  g->h_rp.assign(row_ptr, row_ptr + n + 1);
  g->h_ci.assign(col_idx, col_idx + nnz);
  g->hrp = g->h_rp.data();
  g->hci = g->h_ci.data();
  if ((rc = graph_finish(g, aaw)) != BLP_OK) {
    blp_graph_destroy(g);
    return rc;
  }
  *out = g;
  return BLP_OK;
}

int blp_graph_destroy(blp_graph* g) {
  if (!g) return BLP_OK;
  (void)hipSetDevice(g->device);
  if (g->stream) (void)hipStreamSynchronize(g->stream);
  for (auto& t : g->timers) timer_release(t);
  free_hot_index(g);
  free_wedge_index(g);
  free_node2(g);
  if (g->d_rp) (void)hipFree(g->d_rp);
  if (g->d_ci) (void)hipFree(g->d_ci - CI_PAD);
  if (g->d_aaw_fx) (void)hipFree(g->d_aaw_fx);
  if (g->d_ci_w) (void)hipFree(g->d_ci_w - CI_PAD);
  if (g->d_wtab) (void)hipFree(g->d_wtab);
  stream_give(g->device, g->stream);
  delete g;
  return BLP_OK;
}

int blp_graph_aa_shift(const blp_graph* g, int* shift) {
  BLP_CHECK(g && shift, BLP_E_ARG, "blp_graph_aa_shift: bad arguments");
  *shift = AA_SHIFT;  // fixed: W = w * 2^58 (exact sums, blp_internal.h)
  return BLP_OK;
}

int blp_graph_col_idx(const blp_graph* g, int32_t* out) {
  BLP_CHECK(g && (g->nnz == 0 || out), BLP_E_ARG, "blp_graph_col_idx: bad arguments");
  if (g->nnz == 0) return BLP_OK;
  BLP_HIP(hipSetDevice(g->device));
  prefault_host(out, 4 * (size_t)g->nnz);
  BLP_HIP(hipMemcpy(out, g->d_ci, 4 * (size_t)g->nnz, hipMemcpyDeviceToHost));
  return BLP_OK;
}

int blp_graph_info(const blp_graph* g, int64_t* n, int64_t* nnz, int* device) {
  BLP_CHECK(g, BLP_E_ARG, "blp_graph_info: null graph");
  if (n) *n = g->n;
  if (nnz) *nnz = g->nnz;
  if (device) *device = g->device;
  return BLP_OK;
}

int blp_graph_sync(blp_graph* g) {
  BLP_CHECK(g, BLP_E_ARG, "blp_graph_sync: null graph");
  BLP_HIP(hipSetDevice(g->device));
  BLP_HIP(hipStreamSynchronize(g->stream));
  return BLP_OK;
}

int blp_stats_reset(blp_graph* g) {
  BLP_CHECK(g, BLP_E_ARG, "blp_stats_reset: null graph");
  int rc = timers_collect(g);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g->timer_mu);  // the batches' timers add into the score / group totals
  for (auto& t : g->timers) {
    t.total_ms = 0.0;
    t.launches = 0;
  }
  return BLP_OK;
}

int blp_stats_get(blp_graph* g, int kernel, double* total_ms, int64_t* launches) {
  BLP_CHECK(g && kernel >= 0 && kernel < K_COUNT, BLP_E_ARG, "blp_stats_get: bad arguments");
  int rc = timers_collect(g);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g->timer_mu);
  if (total_ms) *total_ms = g->timers[kernel].total_ms;
  if (launches) *launches = g->timers[kernel].launches;
  return BLP_OK;
}

}  // extern "C"

// Loads this file's GPU code object (blp_stream_prewarm): the HIP runtime loads a translation
// unit's code object on the first launch of any of its kernels, 10-30 ms on the caller's thread.
namespace blp {
int preload_graph() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_code_ids)) == hipSuccess ? 0 : -1;
}
}  // namespace blp
