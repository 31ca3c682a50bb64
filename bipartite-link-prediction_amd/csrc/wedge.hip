// Wedge rows (libblp.so): a second layout of the graph for the short-row scorer.
//
// Building H2(x) (similarity.py:74 GetNodesAtHop(v, 2) on the business side) from CSR takes
// three dependent round trips per source -- N(x), then row_ptr[z] for every z in N(x), then
// the rows N(z) -- and one thread per row, idle beside the longest row of its wave. For a node
// whose neighbours' rows are all short (<= SHORT_ROW_MAX ids: every business of a review
// graph, whose members are users with a few reviews each) the rows N(z), z in N(x), are also
// stored back to back, so the build reads one contiguous range with 16-byte vectors spread
// over the whole workgroup. The volume is sum over eligible x of sum_{z in N(x)} |N(z)| (the
// business side's build elements: 108.8M ids, 435 MB at config 2); it is skipped above
// BLP_WEDGE_MAX_X x nnz ids (default 8) or with BLP_WEDGE=0. Duplicate ids are harmless:
// the build ORs them into a bitmap, so the padding repeats the last id.
#include <algorithm>
#include <cstdlib>
#include <thread>
#include <vector>

#include "blp_internal.h"

namespace {

// One workgroup per node x: the rows N(z), z in N(x), back to back from the device CSR. Each
// round takes 256 of x's neighbours, one per thread: a block scan of their row lengths gives
// every row its offset, then each thread copies its own row (<= SHORT_ROW_MAX ids). The last
// vector is padded with a repeat of the last id. (One wave per node walking N(x) serially took
// 86 ms at config 2: the most reviewed business alone has ~10^5 neighbours.)
constexpr int WF_BLOCK = 256;
__global__ __launch_bounds__(WF_BLOCK) void k_wedge_fill(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                         const int64_t* __restrict__ wp, int64_t n, int32_t* __restrict__ w) {
  __shared__ int red[WF_BLOCK / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t x = blockIdx.x; x < n; x += gridDim.x) {
    int64_t base = 4 * wp[x];
    const int64_t end = 4 * wp[x + 1];
    if (base == end) continue;  // uniform over the block
    const int64_t kb = rp[x], ke = rp[x + 1];
    for (int64_t k0 = kb; k0 < ke; k0 += WF_BLOCK) {
      const int64_t k = k0 + threadIdx.x;
      const bool in = k < ke;
      const int32_t z = in ? ci[k] : 0;
      const int64_t zb = in ? rp[z] : 0;
      const int d = in ? (int)(rp[z + 1] - zb) : 0;
      int inc = d;  // block exclusive scan of d
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      if (lane == 63) red[wid] = inc;
      __syncthreads();
      int before = 0, tot = 0;
#pragma unroll
      for (int q = 0; q < WF_BLOCK / 64; ++q) {
        before += q < wid ? red[q] : 0;
        tot += red[q];
      }
      __syncthreads();  // red is reused by the next round
      const int64_t at = base + before + inc - d;
      for (int j = 0; j < d; ++j) w[at + j] = ci[zb + j];
      base += tot;
    }
    __syncthreads();  // the block's row writes are visible to the block
    if (threadIdx.x < end - base) w[base + threadIdx.x] = w[base - 1];
    __syncthreads();
  }
}

// Large graphs (config 5: 2M businesses, 21G wedge ids): one workgroup per node would leave
// the most reviewed business (11.6M members) on one workgroup for seconds. Items of at most
// WF_ITEM members of one node instead, each reserving its rows' space in the node's range with
// one device atomic (cursor[x]): the rows of a node land in item order, which the bitmap builds
// do not see. k_wedge_pad then repeats the node's first id through its last vector.
constexpr int WF_ITEM = 4096;
struct WedgeItem {
  int64_t k0;   // first CSR entry (member) of the item
  int32_t x;    // node
  int32_t cnt;  // members (<= WF_ITEM)
};

__global__ __launch_bounds__(WF_BLOCK) void k_wedge_fill_items(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                               const int64_t* __restrict__ wp, const WedgeItem* __restrict__ items,
                                                               int64_t n_items, unsigned long long* __restrict__ cursor,
                                                               int32_t* __restrict__ w) {
  __shared__ int red[WF_BLOCK / 64];
  __shared__ long long s_base;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t it = blockIdx.x; it < n_items; it += gridDim.x) {
    const WedgeItem item = items[it];
    for (int m0 = 0; m0 < item.cnt; m0 += WF_BLOCK) {
      const int m = m0 + (int)threadIdx.x;
      const bool in = m < item.cnt;
      const int32_t z = in ? ci[item.k0 + m] : 0;
      const int64_t zb = in ? rp[z] : 0;
      const int d = in ? (int)(rp[z + 1] - zb) : 0;
      int inc = d;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      if (lane == 63) red[wid] = inc;
      __syncthreads();
      int before = 0, tot = 0;
#pragma unroll
      for (int q = 0; q < WF_BLOCK / 64; ++q) {
        before += q < wid ? red[q] : 0;
        tot += red[q];
      }
      if (threadIdx.x == 0) s_base = (long long)atomicAdd(&cursor[item.x], (unsigned long long)tot);
      __syncthreads();
      const int64_t at = 4 * wp[item.x] + s_base + before + inc - d;
      for (int j = 0; j < d; ++j) w[at + j] = ci[zb + j];
      __syncthreads();  // red / s_base are reused by the next round
    }
  }
}

__global__ void k_wedge_pad(const int64_t* __restrict__ wp, const unsigned long long* __restrict__ cursor, int64_t n,
                            int32_t* __restrict__ w) {
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = 4 * wp[x], e = 4 * wp[x + 1];
    for (int64_t q = b + (int64_t)cursor[x]; q < e; ++q) w[q] = w[b];  // a repeat ORs nothing new
  }
}

}  // namespace

namespace blp {

int build_wedge_index(blp_graph* g) {
  if (const char* e = getenv("BLP_WEDGE"))
    if (atoi(e) == 0) return BLP_OK;
  const int64_t n = g->n;
  const int64_t* rp = g->hrp;
  if (n == 0 || g->nnz == 0) return BLP_OK;
  // budget: BLP_WEDGE_MAX_X (16) x nnz ids, and at most 35 % of the free HBM
  double max_x = 16.0;
  if (const char* e = getenv("BLP_WEDGE_MAX_X")) max_x = atof(e);
  size_t free_b = 0, total_b = 0;
  BLP_HIP(hipMemGetInfo(&free_b, &total_b));
  free_b += dev_cache_bytes(g->device);  // cached scratch blocks are free to any allocation (dev_malloc)
  const double budget = std::min(max_x * (double)g->nnz, 0.35 * (double)free_b);
  // members' rows up to BLP_WEDGE_ROW_MAX (64) ids: the short-row scorer's sources (rows <=
  // SHORT_ROW_MAX) always qualify; the chunk-parallel and hash-set scorers use any wedge row
  const int64_t row_max = std::max<int64_t>(SHORT_ROW_MAX, getenv("BLP_WEDGE_ROW_MAX") ? atoll(getenv("BLP_WEDGE_ROW_MAX")) : 64);
  // per-node volume: the two-hop statistics of graph_finish (node2.hip, on the device): x holds a
  // wedge row when every neighbour row is at most row_max ids, of sum |N(z)| ids
  std::vector<int64_t> wp((size_t)n + 1, 0);  // per-node vector counts, then offsets
  for (int64_t x = 0; x < n; ++x)
    wp[x] = (rp[x + 1] > rp[x] && g->h_maxd[x] <= row_max) ? ((int64_t)g->h_w2[x] + 3) / 4 : 0;
  int64_t total = 0;
  for (int64_t x = 0; x < n; ++x) {
    const int64_t c = wp[x];
    wp[x] = total;
    total += c;
  }
  wp[n] = total;
  if (total == 0 || (double)(4 * total) > budget) return BLP_OK;
  // the rows themselves are gathered on the device from the CSR already there (435 MB at
  // config 2: a host fill and upload took ~0.2 s)
  // an index that does not fit is skipped (every scorer also builds from the CSR)
  if (dev_malloc(&g->d_wp, sizeof(int64_t) * (n + 1)) != hipSuccess ||
      dev_malloc(&g->d_wedge, sizeof(int32_t) * 4 * total) != hipSuccess) {
    (void)hipGetLastError();
    if (g->d_wp) (void)hipFree(g->d_wp);
    g->d_wp = nullptr;
    g->d_wedge = nullptr;
    return BLP_OK;
  }
  BLP_HIP(hipMemcpy(g->d_wp, wp.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice));
  int64_t max_deg = 0;
  for (int64_t x = 0; x < n; ++x)
    if (wp[x + 1] > wp[x]) max_deg = std::max<int64_t>(max_deg, rp[x + 1] - rp[x]);
  if (max_deg <= 2 * WF_ITEM && !getenv("BLP_WEDGE_ITEMS")) {  // one workgroup per node
    hipLaunchKernelGGL(k_wedge_fill, dim3((unsigned)std::min<int64_t>(16384, n)), dim3(WF_BLOCK), 0, g->stream,
                       g->d_rp, g->d_ci, g->d_wp, n, g->d_wedge);
  } else {  // items of <= WF_ITEM members (hub nodes)
    std::vector<WedgeItem> items;
    for (int64_t x = 0; x < n; ++x)
      if (wp[x + 1] > wp[x])
        for (int64_t k0 = rp[x]; k0 < rp[x + 1]; k0 += WF_ITEM)
          items.push_back(WedgeItem{k0, (int32_t)x, (int32_t)std::min<int64_t>(WF_ITEM, rp[x + 1] - k0)});
    ScopedBuf d_items, d_cursor;  // freed on every return
    int rc;
    if ((rc = d_items.reserve(sizeof(WedgeItem) * std::max<size_t>(items.size(), 1))) ||
        (rc = d_cursor.reserve(8 * (size_t)n)))
      return rc;
    BLP_HIP(hipMemcpy(d_items.p, items.data(), sizeof(WedgeItem) * items.size(), hipMemcpyHostToDevice));
    BLP_HIP(hipMemsetAsync(d_cursor.p, 0, 8 * (size_t)n, g->stream));
    hipLaunchKernelGGL(k_wedge_fill_items, dim3((unsigned)std::min<size_t>(65536, std::max<size_t>(items.size(), 1))),
                       dim3(WF_BLOCK), 0, g->stream, g->d_rp, g->d_ci, g->d_wp, d_items.as<WedgeItem>(),
                       (int64_t)items.size(), d_cursor.as<unsigned long long>(), g->d_wedge);
    hipLaunchKernelGGL(k_wedge_pad, dim3((unsigned)std::min<int64_t>(8192, (n + 255) / 256)), dim3(256), 0, g->stream,
                       g->d_wp, d_cursor.as<unsigned long long>(), n, g->d_wedge);
    BLP_HIP(hipGetLastError());
    BLP_HIP(hipStreamSynchronize(g->stream));
  }
  BLP_HIP(hipGetLastError());
  BLP_HIP(hipStreamSynchronize(g->stream));
  g->wedge_vecs = total;
  g->h_wp = std::move(wp);
  return BLP_OK;
}

void free_wedge_index(blp_graph* g) {
  if (g->d_wp) (void)hipFree(g->d_wp);
  if (g->d_wedge) (void)hipFree(g->d_wedge);
  g->d_wp = nullptr;
  g->d_wedge = nullptr;
  g->wedge_vecs = 0;
  g->h_wp.clear();
  for (WedgeBitmaps& w : g->wbm) {
    if (w.d_slot) (void)hipFree(w.d_slot);
    if (w.d_pool) (void)hipFree(w.d_pool);
  }
  g->wbm.clear();
  if (g->wset) {  // built from the wedge rows: goes with them
    if (g->wset->d_pool) (void)hipFree(g->wset->d_pool);
    if (g->wset->d_h2) (void)hipFree(g->wset->d_h2);
    delete g->wset;
    g->wset = nullptr;
  }
}

}  // namespace blp

// The wedge-row index of a graph (tests and tools): its vector count (-1: not built), and
// optionally the offsets [n + 1] (in 16-byte vectors) and the ids [4 * n_vecs].
extern "C" int blp_graph_wedge(const blp_graph* g, int64_t* n_vecs, int64_t* wp, int32_t* wedge) {
  BLP_CHECK(g && n_vecs, BLP_E_ARG, "blp_graph_wedge: bad arguments");
  *n_vecs = g->d_wp ? g->wedge_vecs : -1;
  if (!g->d_wp) return BLP_OK;
  BLP_HIP(hipSetDevice(g->device));
  if (wp) BLP_HIP(hipMemcpy(wp, g->d_wp, sizeof(int64_t) * (g->n + 1), hipMemcpyDeviceToHost));
  if (wedge && g->wedge_vecs)
    BLP_HIP(hipMemcpy(wedge, g->d_wedge, sizeof(int32_t) * 4 * g->wedge_vecs, hipMemcpyDeviceToHost));
  return BLP_OK;
}

// Loads this file's GPU code object (blp_stream_prewarm): the HIP runtime loads a translation
// unit's code object on the first launch of any of its kernels, 10-30 ms on the caller's thread.
namespace blp {
int preload_wedge() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_wedge_fill)) == hipSuccess ? 0 : -1;
}
}  // namespace blp
