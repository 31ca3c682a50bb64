// Dense-row index (libblp.so): a hybrid CSR + bitmap graph layout for skewed graphs.
//
// A row N(v) that is dense in its own id range (|N(v)| >= HOT_MIN and |N(v)| * DENSITY >=
// range) is also stored as a bitmap over [min N(v), max N(v)] (128-bit aligned) -- at most
// 2x the row's CSR bytes. When H2(x) is built (similarity.py:29 / :74 GetNodesAtHop(x, 2),
// the union of N(z) for z in N(x)), such a row is OR-ed into the LDS bitmap with 16-byte
// vector loads instead of |N(z)| scattered LDS atomics. On the config-2 review graph the
// ~24 most popular businesses carry most of the user-side build work (sum of d_b^2).
#include <algorithm>

#include "blp_internal.h"

namespace {

__global__ void k_hot_fill(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci, const int32_t* __restrict__ rows,
                           const blp::HotRow* __restrict__ tab, uint32_t* __restrict__ pool) {
  const int r = blockIdx.x;
  const int v = rows[r];
  const blp::HotRow h = tab[r];
  uint32_t* dst = pool + 4 * h.vec_off;
  const int64_t base = 128ll * h.vlo;
  for (int64_t e = rp[v] + threadIdx.x; e < rp[v + 1]; e += blockDim.x) {
    const int64_t b = ci[e] - base;
    atomicOr(&dst[b >> 5], 1u << (b & 31));
  }
}

}  // namespace

namespace blp {

int build_hot_index(blp_graph* g) {
  int64_t hot_min = 2048, density = 64;
  if (const char* e = getenv("BLP_HOT_MIN")) hot_min = std::max<int64_t>(1, atoll(e));
  if (const char* e = getenv("BLP_HOT_DENSITY")) density = std::max<int64_t>(1, atoll(e));
  const int64_t* rp = g->hrp;
  const int32_t* ci = g->hci;
  std::vector<int32_t> idx((size_t)g->n, -1), rows;
  std::vector<HotRow> tab;
  int64_t vecs = 0;
  for (int64_t v = 0; v < g->n; ++v) {
    const int64_t d = rp[v + 1] - rp[v];
    if (d < hot_min) continue;
    const int64_t lo = ci[rp[v]], hi = (int64_t)ci[rp[v + 1] - 1] + 1;
    if (d * density < hi - lo) continue;
    const int32_t vlo = (int32_t)(lo >> 7);
    const int32_t nvec = (int32_t)(((hi + 127) >> 7) - vlo);
    idx[v] = (int32_t)rows.size();
    rows.push_back((int32_t)v);
    tab.push_back(HotRow{vecs, vlo, nvec});
    vecs += nvec;
  }
  g->n_hot = (int64_t)rows.size();
  g->hot_pool_words = 4 * vecs;
  if (!g->n_hot) return BLP_OK;
  g->h_hot_idx = idx;
  int32_t* d_rows = nullptr;
  BLP_HIP(hipMalloc(&g->d_hot_idx, 4 * g->n));
  BLP_HIP(hipMalloc(&g->d_hot_tab, sizeof(HotRow) * tab.size()));
  BLP_HIP(hipMalloc(&g->d_hot_pool, 4 * g->hot_pool_words));
  BLP_HIP(hipMalloc(&d_rows, 4 * rows.size()));
  BLP_HIP(hipMemcpy(g->d_hot_idx, idx.data(), 4 * g->n, hipMemcpyHostToDevice));
  BLP_HIP(hipMemcpy(g->d_hot_tab, tab.data(), sizeof(HotRow) * tab.size(), hipMemcpyHostToDevice));
  BLP_HIP(hipMemcpy(d_rows, rows.data(), 4 * rows.size(), hipMemcpyHostToDevice));
  BLP_HIP(hipMemsetAsync(g->d_hot_pool, 0, 4 * g->hot_pool_words, g->stream));
  hipLaunchKernelGGL(k_hot_fill, dim3((unsigned)rows.size()), dim3(1024), 0, g->stream, g->d_rp, g->d_ci, d_rows,
                     (const HotRow*)g->d_hot_tab, g->d_hot_pool);
  BLP_HIP(hipGetLastError());
  BLP_HIP(hipStreamSynchronize(g->stream));
  BLP_HIP(hipFree(d_rows));
  return BLP_OK;
}

void free_hot_index(blp_graph* g) {
  if (g->d_hot_idx) (void)hipFree(g->d_hot_idx);
  if (g->d_hot_tab) (void)hipFree(g->d_hot_tab);
  if (g->d_hot_pool) (void)hipFree(g->d_hot_pool);
  g->d_hot_idx = nullptr;
  g->d_hot_tab = nullptr;
  g->d_hot_pool = nullptr;
}

}  // namespace blp
