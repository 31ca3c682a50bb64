// Per-node two-hop statistics of a graph handle, computed on the device once at graph creation.
//
// For every node x, over its neighbours z in N(x):
//   w2[x]   = sum of |N(z)|                     (the H2 build work of x as a source; its wedge row)
//   lo2[x]  = min over non-empty N(z) of min N(z)  (the id range N(N(x)) spans: the bitmap universe)
//   hi2[x]  = max over non-empty N(z) of max N(z) + 1
//   maxd[x] = max |N(z)|                        (row-per-thread and wedge-row eligibility)
//   flag[x] = bit 0: some z is a dense row (hot.hip)
// These are what blp_batch_create's source loop and build_wedge_index's volume pass gathered on the
// host from the CSR mirror, one random walk over N(x) per source: at config 2 the business batch's
// 100K sources took 60-70 ms of similarity.main's 0.54 s there (profiles/r04_e2e_c2_check2.json,
// BLP_CREATE_PROF). On the device it is one pass over the CSR entries in tiles of N2_T; a tile's
// rows reduce in LDS and a row cut by a tile boundary merges its partials with device atomics.
#include <algorithm>

#include "blp_internal.h"

namespace {

constexpr int N2_BLOCK = 256;
constexpr int N2_T = 2048;                 // CSR entries per tile (so <= N2_T rows per tile)
constexpr int N2_E = N2_T / N2_BLOCK;      // consecutive entries per thread

__global__ __launch_bounds__(N2_BLOCK) void k_node2(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                     const int32_t* __restrict__ hot_idx, int64_t n, int64_t nnz,
                                                     unsigned long long* __restrict__ w2, int32_t* __restrict__ lo2,
                                                     int32_t* __restrict__ hi2, int32_t* __restrict__ maxd,
                                                     uint8_t* __restrict__ flag) {
  __shared__ unsigned long long s_w[N2_T];
  __shared__ int32_t s_lo[N2_T], s_hi[N2_T], s_md[N2_T], s_fl[N2_T];
  __shared__ int64_t s_r0, s_r1;
  for (int64_t tile = blockIdx.x; tile * N2_T < nnz; tile += gridDim.x) {
    const int64_t ts = tile * N2_T, te = min(nnz, ts + N2_T);
    if (threadIdx.x == 0) {  // rows of the first and the last entry: last r with rp[r] <= k
      auto row_of = [&](int64_t k) {
        int64_t l = 0, h = n;  // rp[l] <= k < rp[h]
        while (h - l > 1) {
          const int64_t m = (l + h) >> 1;
          if (rp[m] <= k) l = m; else h = m;
        }
        return l;
      };
      s_r0 = row_of(ts);
      s_r1 = row_of(te - 1);
    }
    __syncthreads();
    const int64_t r0 = s_r0, r1 = s_r1;
    // rows with entries in the tile are <= N2_T, but empty rows between them are not bounded: rows
    // past the LDS table (i >= N2_T) take device atomics directly
    const int nr = (int)min<int64_t>(r1 - r0 + 1, N2_T);
    for (int i = threadIdx.x; i < nr; i += N2_BLOCK) {
      s_w[i] = 0;
      s_lo[i] = INT32_MAX;
      s_hi[i] = 0;
      s_md[i] = 0;
      s_fl[i] = 0;
    }
    __syncthreads();
    // this thread's N2_E consecutive entries: one row search, then a sequential walk
    const int64_t k0 = ts + (int64_t)threadIdx.x * N2_E;
    if (k0 < te) {
      int64_t l = r0, h = r1 + 1;  // rp[l] <= k0 < rp[h]
      while (h - l > 1) {
        const int64_t m = (l + h) >> 1;
        if (rp[m] <= k0) l = m; else h = m;
      }
      int64_t r = l, rend = rp[r + 1];
      const int64_t k1 = min(te, k0 + N2_E);
      for (int64_t k = k0; k < k1; ++k) {
        while (k >= rend) rend = rp[++r + 1];  // empty rows are stepped over
        const int32_t z = ci[k];
        const int64_t zb = rp[z], ze = rp[z + 1];
        const int64_t i = r - r0;
        const bool hot = hot_idx && hot_idx[z] >= 0;
        if (i < N2_T) {
          atomicAdd(&s_w[i], (unsigned long long)(ze - zb));
          atomicMax(&s_md[i], (int32_t)(ze - zb));
          if (ze > zb) {
            atomicMin(&s_lo[i], ci[zb]);
            atomicMax(&s_hi[i], ci[ze - 1] + 1);
          }
          if (hot) atomicOr(&s_fl[i], 1);
        } else {
          atomicAdd(&w2[r], (unsigned long long)(ze - zb));
          atomicMax(&maxd[r], (int32_t)(ze - zb));
          if (ze > zb) {
            atomicMin(&lo2[r], ci[zb]);
            atomicMax(&hi2[r], ci[ze - 1] + 1);
          }
          if (hot) atomicOr(reinterpret_cast<unsigned int*>(flag + (r & ~int64_t(3))), 1u << (8 * (r & 3)));
        }
      }
    }
    __syncthreads();
    // rows wholly inside the tile are its own: plain stores; the (at most two) rows cut by its
    // boundaries merge with the neighbouring tiles' partials through device atomics
    for (int i = threadIdx.x; i < nr; i += N2_BLOCK) {
      const int64_t r = r0 + i;
      const int64_t b = rp[r], e = rp[r + 1];
      if (e == b) continue;  // an empty row between two entries of the tile: untouched
      if (b >= ts && e <= te) {
        w2[r] = s_w[i];
        lo2[r] = s_lo[i];
        hi2[r] = s_hi[i];
        maxd[r] = s_md[i];
        flag[r] = (uint8_t)s_fl[i];
      } else {
        atomicAdd(&w2[r], s_w[i]);
        atomicMin(&lo2[r], s_lo[i]);
        atomicMax(&hi2[r], s_hi[i]);
        atomicMax(&maxd[r], s_md[i]);
        if (s_fl[i]) atomicOr(reinterpret_cast<unsigned int*>(flag + (r & ~int64_t(3))), 1u << (8 * (r & 3)));
      }
    }
    __syncthreads();  // the LDS rows are reused by the next tile
  }
}

}  // namespace

namespace blp {

int build_node2(blp_graph* g) {
  const int64_t n = g->n, nnz = g->nnz;
  g->h_w2.assign((size_t)n, 0);
  g->h_lo2.assign((size_t)n, INT32_MAX);
  g->h_hi2.assign((size_t)n, 0);
  g->h_maxd.assign((size_t)n, 0);
  g->h_flag2.assign((size_t)n, 0);
  free_node2(g);
  if (n == 0 || nnz == 0) return BLP_OK;
  BLP_HIP(dev_malloc(&g->d_w2, 8 * (size_t)n));
  BLP_HIP(dev_malloc(&g->d_lo2, 4 * (size_t)n));
  BLP_HIP(dev_malloc(&g->d_hi2, 4 * (size_t)n));
  BLP_HIP(dev_malloc(&g->d_maxd, 4 * (size_t)n));
  BLP_HIP(dev_malloc(&g->d_flag2, ((size_t)n + 3) / 4 * 4));
  BLP_HIP(hipMemsetAsync(g->d_w2, 0, 8 * (size_t)n, g->stream));
  BLP_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(g->d_lo2), INT32_MAX, (size_t)n, g->stream));
  BLP_HIP(hipMemsetAsync(g->d_hi2, 0, 4 * (size_t)n, g->stream));
  BLP_HIP(hipMemsetAsync(g->d_maxd, 0, 4 * (size_t)n, g->stream));
  BLP_HIP(hipMemsetAsync(g->d_flag2, 0, ((size_t)n + 3) / 4 * 4, g->stream));
  const int64_t tiles = (nnz + N2_T - 1) / N2_T;
  hipLaunchKernelGGL(k_node2, dim3((unsigned)std::min<int64_t>(tiles, (int64_t)g->n_cu * 16)), dim3(N2_BLOCK), 0,
                     g->stream, (const int64_t*)g->d_rp, (const int32_t*)g->d_ci, (const int32_t*)g->d_hot_idx, n, nnz,
                     g->d_w2, g->d_lo2, g->d_hi2, g->d_maxd, g->d_flag2);
  BLP_HIP(hipGetLastError());
  BLP_HIP(hipMemcpyAsync(g->h_w2.data(), g->d_w2, 8 * (size_t)n, hipMemcpyDeviceToHost, g->stream));
  BLP_HIP(hipMemcpyAsync(g->h_lo2.data(), g->d_lo2, 4 * (size_t)n, hipMemcpyDeviceToHost, g->stream));
  BLP_HIP(hipMemcpyAsync(g->h_hi2.data(), g->d_hi2, 4 * (size_t)n, hipMemcpyDeviceToHost, g->stream));
  BLP_HIP(hipMemcpyAsync(g->h_maxd.data(), g->d_maxd, 4 * (size_t)n, hipMemcpyDeviceToHost, g->stream));
  BLP_HIP(hipMemcpyAsync(g->h_flag2.data(), g->d_flag2, (size_t)n, hipMemcpyDeviceToHost, g->stream));
  BLP_HIP(hipStreamSynchronize(g->stream));
  return BLP_OK;
}

void free_node2(blp_graph* g) {
  void* ps[] = {g->d_w2, g->d_lo2, g->d_hi2, g->d_maxd, g->d_flag2};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  g->d_w2 = nullptr;
  g->d_lo2 = g->d_hi2 = g->d_maxd = nullptr;
  g->d_flag2 = nullptr;
}

}  // namespace blp

// Loads this file's GPU code object (blp_stream_prewarm): the HIP runtime loads a translation
// unit's code object on the first launch of any of its kernels, 10-30 ms on the caller's thread.
namespace blp {
int preload_node2() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_node2)) == hipSuccess ? 0 : -1;
}
}  // namespace blp
