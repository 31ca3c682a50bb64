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

// One wave per node x: the rows N(z), z in N(x), back to back from the device CSR. The wave
// takes 64 of x's neighbours at a time (their row offsets in one load), then copies their rows
// one after another, one id per lane (rows hold <= SHORT_ROW_MAX < 64 ids), and pads the last
// vector with a repeat of the last id.
__global__ __launch_bounds__(256) void k_wedge_fill(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                    const int64_t* __restrict__ wp, int64_t n, int32_t* __restrict__ w) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t x = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); x < n; x += nwaves) {
    int64_t pos = 4 * wp[x];
    const int64_t end = 4 * wp[x + 1];
    if (pos == end) continue;
    const int64_t kb = rp[x], ke = rp[x + 1];
    int32_t last = 0;
    for (int64_t k0 = kb; k0 < ke; k0 += 64) {
      const bool in = k0 + lane < ke;
      const int32_t z = in ? ci[k0 + lane] : 0;
      const int64_t zb = in ? rp[z] : 0;
      const int d = in ? (int)(rp[z + 1] - zb) : 0;
      const int cnt = (int)min<int64_t>(64, ke - k0);
      for (int j = 0; j < cnt; ++j) {
        const int64_t b = __shfl(zb, j, 64);
        const int dj = __shfl(d, j, 64);
        const int32_t v = lane < dj ? ci[b + lane] : 0;
        if (lane < dj) w[pos + lane] = v;
        if (dj) last = __shfl(v, dj - 1, 64);
        pos += dj;
      }
    }
    if (lane < end - pos) w[pos + lane] = last;
  }
}

}  // namespace

namespace blp {

int build_wedge_index(blp_graph* g) {
  if (const char* e = getenv("BLP_WEDGE"))
    if (atoi(e) == 0) return BLP_OK;
  const int64_t n = g->n;
  const int64_t* rp = g->hrp;
  const int32_t* ci = g->hci;
  if (n == 0 || g->nnz == 0) return BLP_OK;
  double max_x = 8.0;
  if (const char* e = getenv("BLP_WEDGE_MAX_X")) max_x = atof(e);
  const double budget = std::min(max_x * (double)g->nnz, (double)(int64_t(1) << 34));
  // per-node volume: one degree lookup per CSR entry, 16 threads (2B entries at config 5)
  const int nt = (int)std::max<unsigned>(1, std::min<unsigned>(16, std::thread::hardware_concurrency()));
  std::vector<int64_t> wp((size_t)n + 1, 0);  // per-node vector counts, then offsets
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t]() {
        for (int64_t x = t; x < n; x += nt) {
          int64_t len = 0;
          bool ok = true;
          for (int64_t k = rp[x]; k < rp[x + 1]; ++k) {
            const int64_t d = rp[ci[k] + 1] - rp[ci[k]];
            if (d > SHORT_ROW_MAX) {
              ok = false;
              break;
            }
            len += d;
          }
          wp[x] = ok ? (len + 3) / 4 : 0;
        }
      });
    for (auto& t : th) t.join();
  }
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
  BLP_HIP(hipMalloc(&g->d_wp, sizeof(int64_t) * (n + 1)));
  BLP_HIP(hipMalloc(&g->d_wedge, sizeof(int32_t) * 4 * total));
  BLP_HIP(hipMemcpy(g->d_wp, wp.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_wedge_fill, dim3((unsigned)std::min<int64_t>(8192, (n + 3) / 4)), dim3(256), 0, g->stream,
                     g->d_rp, g->d_ci, g->d_wp, n, g->d_wedge);
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
}

}  // namespace blp
