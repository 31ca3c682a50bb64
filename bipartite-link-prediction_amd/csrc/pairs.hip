// Pair scoring: common neighbours / Jaccard / Adamic-Adar on candidate pairs (libblp.so).
//
// Replaces the hot loops of similarity.users (similarity.py:20-61) and
// similarity.business (similarity.py:63-106). For a pair (x, y):
//   H2(x) = GetNodesAtHop(G, x, 2)  (similarity.py:29 / :74) -- exact BFS distance 2
//   N(y)  = GetNodesAtHop(G, y, 1)  (similarity.py:41 / :85)
//   cn  = |H2(x) ∩ N(y)|                                       (:113-114)
//   jac = float(cn) / float(|H2(x)| + |N(y)| - cn)              (:108-111)
//   aa  = Σ_{w ∈ H2(x) ∩ N(y)} (log deg w)^-1 [deg > 1]        (:116-126)
//
// One step (blp_batch_score), all on the graph's stream:
//   1. group   counting sort of the raw pair list by source x on the device: run-aggregated
//              counts -> scan -> scatter. The scatter also gathers each pair's N(y) row
//              (start, length) so the scorer never walks the pair -> y -> row_ptr chain.
//   2. heavy   (planned sources only) sources whose H2 build is far above the per-workgroup
//              average are pre-built by several workgroups into HBM bitmaps.
//   3. score   persistent workgroups dequeue sources. Per source: H2(x) as a bitmap in LDS over
//              the batch's node universe [lo, hi) (chunked when larger than LDS), built from
//              the rows of N(x); distance 0/1 removed; |H2| popcounted; then every pair's N(y)
//              is scanned against the bitmap. Both the build and the scan run as merge-path
//              segment loops: the rows of a chunk are concatenated, every thread takes K
//              consecutive elements (K independent loads in flight), one LDS binary search per
//              K elements maps an element to its row. Short and very long rows cost the same.
// Adamic-Adar sums are exact (two-word integer sums of w * 2^58, any order; blp_internal.h).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <numeric>
#include <thread>

#include "blp_internal.h"

#ifndef BLP_RC
#define BLP_RC 1  // row-chunk loops in the large-universe k_score (0: merge-path loops)
#endif
#ifndef BLP_SHORT_MINB
#define BLP_SHORT_MINB 7  // short-row scorer: >= 7 workgroups of 256 per CU (<= 72 VGPRs)
#endif
#ifndef BLP_PF
#define BLP_PF 1  // short-row scorer: first pair segment's metadata loaded before the H2 build
#endif
#ifndef BLP_PFL
#define BLP_PFL 1  // the same for the large-universe row-chunk scorer
#endif
#ifndef BLP_PFN
#define BLP_PFN 1  // ... and every later segment's metadata during the previous segment's scan
#endif
#ifndef BLP_EXP_PHASE
#define BLP_EXP_PHASE 0  // experiment builds only (LDS bank-conflict attribution of the large scorer):
                         // 1 = no pair scan, 2 = no H2 build (dense OR and sparse rows; the scan finds no hits)
#endif
#ifndef BLP_SEGOFF
#define BLP_SEGOFF 0  // large scorer: element and chunk offsets of a segment batch in ONE scan (seg_offsets)
#endif
#ifndef BLP_PP
#define BLP_PP 1  // ping-pong merge-path loops in k_score (0: the single-buffer mp_build / mp_scan)
#endif

namespace {

constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

struct Misc {
  int n_active;
  int queue;
  int zero_div;
  int hq;     // k_score_hash's queue head
  int n_items;  // item grouping: items planned by k_item_plan
  int qh[8];  // k_score_split: one queue head per XCD group (sources s = g mod 8)
  int n_hash_front;  // split batches with hash-routed sources: the active list is partitioned,
  int n_split_back;  // hash sources in [0, n_hash_front), split sources after (k_hash_partition)
  long long dbg[4];  // BLP_DEBUG builds: bound violations, first site, its value, its bound (PS_OK)
};

// BLP_DEBUG builds (make debug -> libblp_debug.so): the scorers' queue claims, queue slots, table
// probes, split-table rows and output indexes are checked against their bounds before the
// access; a violation is counted in the batch's Misc, the first one recorded (site, value,
// bound) and the access skipped, so a check never faults the GPU. blp_batch_fetch then fails
// with the record (BLP_E_STATE). Release builds compile the checks out. Sites:
//   1 claimed source index < n_active        2 source id < n_nodes
//   3 pair range [pbeg, pbeg + pcnt) <= np    4 output index < np
//   5 long-slice queue slot < SPLIT_LQ        6 long-slice queue region < the allocated workgroups
//   7 split-table row < its rows              8 hash-set probes < HT (a full table would spin)
//   9 chunk width <= the bitmap's bits      10 a row read [st, st + len) <= nnz (+ padding)
//  11 wedge-row vectors [wb, we) <= wedge    12 dense row number < n_hot
//  13 dense-row pool vector < pool vectors
#ifdef BLP_DEBUG
__device__ inline bool ps_ok(Misc* m, bool ok, int site, long long v, long long bound) {
  if (!ok && atomicAdd(reinterpret_cast<unsigned long long*>(&m->dbg[0]), 1ull) == 0ull) {
    m->dbg[1] = site;
    m->dbg[2] = v;
    m->dbg[3] = bound;
  }
  return ok;
}
#define PS_OK(m, cond, site, v, bound) ps_ok((m), (cond), (site), (long long)(v), (long long)(bound))
#else
#define PS_OK(m, cond, site, v, bound) ((void)(v), true)
#endif

// ------------------------------------------------------------------ grouping kernels
// Two-pass MSD bucket sort of the pairs by source x, with every atomic in LDS (a device-
// scope atomic executes at the memory side on a multi-XCD part and costs ~50x more):
//   1. k_bucket_hist    per-block histogram of buckets b = x >> shift  (bucket-major table)
//   2. scan_ex          exclusive scan of that table -> bucket/block write offsets
//   3. k_bucket_scatter pair indices into bucket order
//   4. k_bucket_group   one block per bucket: counting sort of its keys in LDS, per-node
//                       off/cnt, grouped pair metadata (caller index, N(y) start and length)
//   5. scan_ex          of the per-bucket active-source counts
//   6. k_active_write   the active-source list in ascending id order
constexpr int HOT_LIST = 64;    // dense rows OR-ed per source (more: all rows go sparse)
constexpr int GP_BLOCK = 1024;  // passes 1 and 3
constexpr int GB_BLOCK = 256;   // passes 4 and 6
constexpr int NB_MAX = 4096;    // buckets

// block-wide exclusive scan of one int per thread; *tot receives the block total
template <int BLOCK>
__device__ inline int block_exscan_i(int v, int* red, int* tot) {
  constexpr int NW = BLOCK / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(inc, d, 64);
    if (lane >= d) inc += t;
  }
  if (lane == 63) red[wid] = inc;
  __syncthreads();
  int base = 0, all = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int t = red[w];
    base += w < wid ? t : 0;
    all += t;
  }
  __syncthreads();
  *tot = all;
  return base + inc - v;
}

// --- generic exclusive scan of an int32 array (3 kernels), total -> *total_out
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_sum(const int32_t* __restrict__ in, int64_t n,
                                                         int32_t* __restrict__ tile_sum) {
  __shared__ int red[SCAN_BLOCK / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int v = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) v += base + k < n ? in[base + k] : 0;
  int tot;
  block_exscan_i<SCAN_BLOCK>(v, red, &tot);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_mid(int32_t* __restrict__ tile_sum, int64_t ntiles,
                                                         int32_t* __restrict__ total_out) {
  __shared__ int red[SCAN_BLOCK / 64];
  int carry = 0;
  for (int64_t b = 0; b < ntiles; b += SCAN_BLOCK) {
    const int64_t i = b + threadIdx.x;
    const int v = i < ntiles ? tile_sum[i] : 0;
    int tot;
    const int e = block_exscan_i<SCAN_BLOCK>(v, red, &tot);
    if (i < ntiles) tile_sum[i] = e + carry;
    carry += tot;
  }
  if (threadIdx.x == 0 && total_out) *total_out = carry;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_out(const int32_t* __restrict__ in, int64_t n,
                                                         const int32_t* __restrict__ tile_sum, int32_t* __restrict__ out) {
  __shared__ int red[SCAN_BLOCK / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int c[SCAN_ITEMS];
  int v = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    c[k] = base + k < n ? in[base + k] : 0;
    v += c[k];
  }
  int tot;
  int o = block_exscan_i<SCAN_BLOCK>(v, red, &tot) + tile_sum[blockIdx.x];
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k)
    if (base + k < n) {
      out[base + k] = o;
      o += c[k];
    }
}

__global__ __launch_bounds__(GP_BLOCK) void k_bucket_hist(const int32_t* __restrict__ x, int64_t np, int32_t xlo,
                                                          int shift, int bmask, int nb, int nblk, int64_t per_blk,
                                                          int32_t* __restrict__ hist) {
  __shared__ int h[NB_MAX];
  for (int i = threadIdx.x; i < nb; i += GP_BLOCK) h[i] = 0;
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * per_blk, b1 = min(np, b0 + per_blk);
#ifndef BLP_HIST_U
#define BLP_HIST_U 8  // (with BLP_ITEMC_U 8 and BLP_SCATTER_U 12: r05_group_rounds)
#endif
  constexpr int U = BLP_HIST_U;
  for (int64_t r = b0; r < b1; r += U * GP_BLOCK) {
    int xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = r + u * GP_BLOCK + threadIdx.x;
      xv[u] = i < b1 ? x[i] : INT32_MIN;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (xv[u] != INT32_MIN) atomicAdd(&h[((xv[u] - xlo) >> shift) & bmask], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += GP_BLOCK) hist[(int64_t)i * nblk + blockIdx.x] = h[i];
}

// The pair itself (caller index, x, y) moves into bucket order, so the group kernel reads
// its bucket contiguously instead of gathering x[i] / y[i] at random caller positions.
// ROWS (round 5): the record carries N(y)'s row instead of y -- (caller index, x, rp[y] as int32,
// |N(y)|) -- gathered HERE, in caller order: similarity.users' order keeps a user's ~750 pairs
// together, so on the business side (y = user) a wave's gathers hit one or two rows and cost
// nothing, where the grouped order of the later write kernel scatters them over the whole
// row_ptr array.
template <bool ROWS = false>
__global__ __launch_bounds__(GP_BLOCK) void k_bucket_scatter(const int32_t* __restrict__ x, const int32_t* __restrict__ y,
                                                             int64_t np, int32_t xlo, int shift, int bmask, int nb, int nblk,
                                                             int64_t per_blk, const int32_t* __restrict__ hoff,
                                                             int4* __restrict__ tmp, const int64_t* __restrict__ rp = nullptr) {
  __shared__ int cur[NB_MAX];
  for (int i = threadIdx.x; i < nb; i += GP_BLOCK) cur[i] = hoff[(int64_t)i * nblk + blockIdx.x];
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * per_blk, b1 = min(np, b0 + per_blk);
#ifndef BLP_SCATTER_U
#define BLP_SCATTER_U 12  // 8: 2.230 / 2.231 / 2.230 against 2.261 / 2.272 / 2.261 ms with 4 (r05_scatter_u); 12: r05_group_rounds
#endif
  constexpr int U = BLP_SCATTER_U;  // U pairs per thread per round: loads and LDS atomics overlap
  for (int64_t r = b0; r < b1; r += U * GP_BLOCK) {
    int xv[U], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = r + u * GP_BLOCK + threadIdx.x;
      xv[u] = i < b1 ? x[i] : INT32_MIN;
      yv[u] = i < b1 ? y[i] : 0;
    }
    int pos[U];
    int sv[U], lv[U];
    if (ROWS) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t b0 = rp[yv[u]], b1 = rp[yv[u] + 1];
        sv[u] = (int)b0;
        lv[u] = (int)(b1 - b0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) pos[u] = xv[u] != INT32_MIN ? atomicAdd(&cur[((xv[u] - xlo) >> shift) & bmask], 1) : -1;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (pos[u] >= 0) {
        const int32_t ci = (int32_t)(r + u * GP_BLOCK + threadIdx.x);
        tmp[pos[u]] = ROWS ? make_int4(ci, xv[u], sv[u], lv[u]) : make_int4(ci, xv[u], yv[u], 0);
      }
  }
}

// One block per bucket of KEYS consecutive node ids.
template <int KEYS>
__global__ __launch_bounds__(GB_BLOCK) void k_bucket_group(const int64_t* __restrict__ rp, const int4* __restrict__ tmp,
                                                           const int32_t* __restrict__ hoff, int nblk, int nb, int shift,
                                                           int32_t xlo, int64_t xspan, int64_t np, int32_t* __restrict__ off,
                                                           int32_t* __restrict__ cnt, int32_t* __restrict__ bucket_active,
                                                           int32_t* __restrict__ g_out, int64_t* __restrict__ g_yb,
                                                           int32_t* __restrict__ g_yl, int32_t* __restrict__ g_y) {
  constexpr int PER = KEYS >= GB_BLOCK ? KEYS / GB_BLOCK : 1;  // KEYS < GB_BLOCK: threads >= KEYS idle
  __shared__ int h[KEYS];
  __shared__ int red[GB_BLOCK / 64];
  const int b = blockIdx.x;
  const int64_t k0 = (int64_t)xlo + ((int64_t)b << shift);
  const int nk = (int)min<int64_t>((int64_t)1 << shift, xspan - ((int64_t)b << shift));
  const int bs = hoff[(int64_t)b * nblk];
  const int be = b + 1 < nb ? hoff[(int64_t)(b + 1) * nblk] : (int)np;
  for (int i = threadIdx.x; i < KEYS; i += GB_BLOCK) h[i] = 0;
  __syncthreads();
  {  // counting pass: UC independent loads in flight per thread, then their LDS atomics (one
     // dependent round trip per UC pairs, not per pair: the bucket's ~5K pairs took 19)
    constexpr int UC = 8;
    for (int kr = bs; kr < be; kr += UC * GB_BLOCK) {
      int xv[UC];
#pragma unroll
      for (int u = 0; u < UC; ++u) {
        const int k = kr + u * GB_BLOCK + threadIdx.x;
        xv[u] = k < be ? tmp[k].y : INT32_MIN;
      }
#pragma unroll
      for (int u = 0; u < UC; ++u)
        if (xv[u] != INT32_MIN) atomicAdd(&h[xv[u] - k0], 1);
    }
  }
  __syncthreads();
  int v = 0, act = 0;
  for (int q = 0; q < PER; ++q) {
    const int j = threadIdx.x * PER + q;
    const int c = j < KEYS ? h[j] : 0;
    v += c;
    act += c > 0;
  }
  int tot;
  int o = block_exscan_i<GB_BLOCK>(v, red, &tot);
  int acts;
  block_exscan_i<GB_BLOCK>(act, red, &acts);
  for (int q = 0; q < PER && threadIdx.x * PER + q < KEYS; ++q) {
    const int j = threadIdx.x * PER + q;
    const int c = h[j];
    if (j < nk) {
      off[k0 + j] = bs + o;
      cnt[k0 + j] = c;
    }
    h[j] = o;  // cursor
    o += c;
  }
  if (threadIdx.x == 0) bucket_active[b] = acts;
  __syncthreads();
  // U pairs per thread per round: their loads, gathers and LDS atomics overlap
#ifndef BLP_GROUP_U
#define BLP_GROUP_U 4
#endif
  constexpr int U = BLP_GROUP_U;
  for (int k0r = bs; k0r < be; k0r += U * GB_BLOCK) {
    int4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0r + u * GB_BLOCK + threadIdx.x;
      t[u] = k < be ? tmp[k] : make_int4(-1, 0, 0, 0);
    }
    int64_t st[U], en[U];
    int pos[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      st[u] = rp[t[u].z];
      en[u] = rp[t[u].z + 1];
      pos[u] = t[u].x >= 0 ? bs + atomicAdd(&h[t[u].y - k0], 1) : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (t[u].x >= 0) {
        g_out[pos[u]] = t[u].x;
        g_yb[pos[u]] = st[u];
        g_yl[pos[u]] = (int32_t)(en[u] - st[u]);
        if (g_y) g_y[pos[u]] = t[u].z;
      }
    }
  }
}

// ---- item grouping (the default for pair lists not grouped by source): skew-proof. Measured
// on config 2's business pass (x = business, Zipf-popular): the bucket of the 64 most popular
// ids holds ~16% of the 7.55M pairs, so k_bucket_group ran one workgroup over 1.2M pairs
// (461 us, the rest of the grid idle) and the hist / scatter LDS counters of that bucket
// serialised. Here buckets INTERLEAVE ids (bucket = v mod nb, key j = v / nb, v = x - xlo) so
// popular ids land in different buckets, and each bucket's pairs are cut into items of at most
// GI_PAIRS, one workgroup each: a source with 1M pairs costs 256 workgroups, not one.
//   k_item_plan   one block: items per bucket, item table (bucket, first, end)
//   k_item_count  per item: LDS histogram of its keys, one device atomic per (item, key) into cnt
//   scans         off = exclusive scan of cnt over the id range; active = ids with cnt > 0
//   k_item_write  per item: the same histogram; per key one device atomic reserves the item's
//                 run inside [off, off + cnt) (fill), then LDS cursors place every pair
// Order within one source's group follows item order (not caller order): every grouped pair
// carries its caller index (g_out), so results do not depend on it.
#ifndef BLP_GI_PAIRS
#define BLP_GI_PAIRS 4096
#endif
constexpr int GI_PAIRS = BLP_GI_PAIRS;

__global__ __launch_bounds__(1024) void k_item_plan(const int32_t* __restrict__ hoff, int nblk, int nb, int64_t np,
                                                    int32_t* __restrict__ item_b, int32_t* __restrict__ item_s,
                                                    int32_t* __restrict__ item_e, int32_t* __restrict__ n_items) {
  __shared__ int red[1024 / 64];
  int carry = 0;
  for (int b0 = 0; b0 < nb; b0 += 1024) {
    const int b = b0 + (int)threadIdx.x;
    const int s = b < nb ? hoff[(int64_t)b * nblk] : 0;
    const int e = b < nb ? (b + 1 < nb ? hoff[(int64_t)(b + 1) * nblk] : (int)np) : 0;
    const int it = (e - s + GI_PAIRS - 1) / GI_PAIRS;
    int tot;
    int o = block_exscan_i<1024>(it, red, &tot) + carry;
    for (int q = 0; q < it; ++q, ++o) {
      item_b[o] = b;
      item_s[o] = s + q * GI_PAIRS;
      item_e[o] = min(e, s + (q + 1) * GI_PAIRS);
    }
    carry += tot;
  }
  if (threadIdx.x == 0) *n_items = carry;
}

template <int KEYS>
__device__ inline void item_hist(const int4* __restrict__ tmp, int s, int e, int32_t xlo, int lognb, int* h) {
  for (int i = threadIdx.x; i < KEYS; i += GB_BLOCK) h[i] = 0;
  __syncthreads();
#ifndef BLP_ITEMC_U
#define BLP_ITEMC_U 8
#endif
  constexpr int UC = BLP_ITEMC_U;  // GI_PAIRS / GB_BLOCK = 16 pairs per thread: UC loads in flight
  for (int kr = s; kr < e; kr += UC * GB_BLOCK) {
    int xv[UC];
#pragma unroll
    for (int u = 0; u < UC; ++u) {
      const int k = kr + u * GB_BLOCK + (int)threadIdx.x;
      xv[u] = k < e ? tmp[k].y : INT32_MIN;
    }
#pragma unroll
    for (int u = 0; u < UC; ++u)
      if (xv[u] != INT32_MIN) atomicAdd(&h[(xv[u] - xlo) >> lognb], 1);
  }
  __syncthreads();
}

template <int KEYS>
__global__ __launch_bounds__(GB_BLOCK) void k_item_count(const int4* __restrict__ tmp, const int32_t* __restrict__ item_b,
                                                         const int32_t* __restrict__ item_s,
                                                         const int32_t* __restrict__ item_e,
                                                         const int32_t* __restrict__ n_items, int32_t xlo, int lognb,
                                                         int32_t* __restrict__ cnt, int32_t* __restrict__ ih) {
  __shared__ int h[KEYS];
  const int i = blockIdx.x;
  if (i >= *n_items) return;  // uniform: the grid is the host's upper bound on items
  const int b = item_b[i];
  item_hist<KEYS>(tmp, item_s[i], item_e[i], xlo, lognb, h);
  for (int j = threadIdx.x; j < KEYS; j += GB_BLOCK) {
    if (h[j]) atomicAdd(&cnt[xlo + b + (j << lognb)], h[j]);
    if (ih) ih[(int64_t)i * KEYS + j] = h[j];  // the item's histogram, for k_item_write_ids
  }
}

template <int KEYS>
__global__ __launch_bounds__(GB_BLOCK) void k_item_write(const int64_t* __restrict__ rp, const int4* __restrict__ tmp,
                                                         const int32_t* __restrict__ item_b,
                                                         const int32_t* __restrict__ item_s,
                                                         const int32_t* __restrict__ item_e,
                                                         const int32_t* __restrict__ n_items, int32_t xlo, int lognb,
                                                         const int32_t* __restrict__ off, int32_t* __restrict__ fill,
                                                         int32_t* __restrict__ g_out, int64_t* __restrict__ g_yb,
                                                         int32_t* __restrict__ g_yl, int32_t* __restrict__ g_y) {
  __shared__ int h[KEYS];
  const int i = blockIdx.x;
  if (i >= *n_items) return;
  const int b = item_b[i], s = item_s[i], e = item_e[i];
  item_hist<KEYS>(tmp, s, e, xlo, lognb, h);
  for (int j = threadIdx.x; j < KEYS; j += GB_BLOCK)
    if (h[j]) {
      const int v = b + (j << lognb);
      h[j] = off[xlo + v] + atomicAdd(&fill[v], h[j]);  // this item's run of source x
    }
  __syncthreads();
  constexpr int U = 4;
  for (int k0r = s; k0r < e; k0r += U * GB_BLOCK) {
    int4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0r + u * GB_BLOCK + (int)threadIdx.x;
      t[u] = k < e ? tmp[k] : make_int4(-1, xlo, 0, 0);
    }
    int64_t st[U], en[U];
    int pos[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      st[u] = rp[t[u].z];
      en[u] = rp[t[u].z + 1];
      pos[u] = t[u].x >= 0 ? atomicAdd(&h[(t[u].y - xlo) >> lognb], 1) : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (t[u].x >= 0) {
        g_out[pos[u]] = t[u].x;
        g_yb[pos[u]] = st[u];
        g_yl[pos[u]] = (int32_t)(en[u] - st[u]);
        if (g_y) g_y[pos[u]] = t[u].z;
      }
    }
  }
}

// The grouping write with the item's pairs first ordered by key in LDS, so each key's run goes
// out as consecutive positions: the grouped metadata leaves in whole runs instead of one scattered
// 4-8 B store per array per pair (k_item_write<64>: 533 us in-step at config 2). The item's
// histogram comes from k_item_count (ih); its records are read ONCE into a 32 KiB LDS stage of
// 8-byte records in key order, and the write loop finds each slot's key by a binary search of the
// key starts. MODE 2: the records already carry N(y)'s row (k_bucket_scatter<true>): (caller
// index, row start) staged, row lengths beside them (48 KiB), no gathers at all. MODE 1: (caller
// index, y) staged, the row gathered from rp here, U slots per thread in flight together.
template <int KEYS, int MODE>  // MODE 1 or 2
__global__ __launch_bounds__(GB_BLOCK) void k_item_write_ids(const int64_t* __restrict__ rp, const int4* __restrict__ tmp,
                                                             const int32_t* __restrict__ item_b,
                                                             const int32_t* __restrict__ item_s,
                                                             const int32_t* __restrict__ item_e,
                                                             const int32_t* __restrict__ n_items, int32_t xlo, int lognb,
                                                             const int32_t* __restrict__ ih,
                                                             const int32_t* __restrict__ off, int32_t* __restrict__ fill,
                                                             int32_t* __restrict__ g_out, int64_t* __restrict__ g_yb,
                                                             int32_t* __restrict__ g_yl, int32_t* __restrict__ g_y) {
  static_assert(KEYS <= 1024, "key tables in LDS");
  constexpr int PER = KEYS >= GB_BLOCK ? KEYS / GB_BLOCK : 1;
  __shared__ int h[KEYS];      // local cursors
  __shared__ int lofs[KEYS];   // the key's first local position
  __shared__ int gbase[KEYS];  // ... and its first global position
  __shared__ int2 stage[GI_PAIRS];
  __shared__ int stage_len[MODE == 2 ? GI_PAIRS : 1];
  __shared__ int red[GB_BLOCK / 64];
  const int i = blockIdx.x;
  if (i >= *n_items) return;
  const int b = item_b[i], s = item_s[i], e = item_e[i];
  int c[PER];
  int v = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int j = (int)threadIdx.x * PER + q;
    c[q] = j < KEYS ? ih[(int64_t)i * KEYS + j] : 0;
    v += c[q];
  }
  int tot;
  int o = block_exscan_i<GB_BLOCK>(v, red, &tot);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int j = (int)threadIdx.x * PER + q;
    if (j < KEYS) {
      const int vv = b + (j << lognb);
      lofs[j] = o;
      gbase[j] = c[q] ? off[xlo + vv] + atomicAdd(&fill[vv], c[q]) : 0;
      h[j] = o;
      o += c[q];
    }
  }
  __syncthreads();
#ifndef BLP_ITEMW_U
#define BLP_ITEMW_U 4
#endif
  constexpr int U = BLP_ITEMW_U;
  for (int kr = s; kr < e; kr += U * GB_BLOCK) {  // the item's records, staged in key order
    int4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = kr + u * GB_BLOCK + (int)threadIdx.x;
      t[u] = k < e ? tmp[k] : make_int4(-1, xlo, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (t[u].x >= 0) {
        const int slot = atomicAdd(&h[(t[u].y - xlo) >> lognb], 1);
        stage[slot] = make_int2(t[u].x, t[u].z);
        if (MODE == 2) stage_len[slot] = t[u].w;
      }
  }
  __syncthreads();
  const int n = e - s;
  for (int pr = 0; pr < n; pr += U * GB_BLOCK) {  // consecutive local slots -> consecutive positions
    int pos[U];
    int2 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = pr + u * GB_BLOCK + (int)threadIdx.x;
      pos[u] = -1;
      if (p < n) {
        // the slot's key: the LAST j with lofs[j] <= p (lofs[0] = 0 <= p). Empty keys share their
        // start with the next key, so the last such j is the non-empty key whose run holds p.
        int lo = 0, hi = KEYS;
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (lofs[mid] <= p)
            lo = mid;
          else
            hi = mid;
        }
        r[u] = stage[p];
        pos[u] = gbase[lo] + (p - lofs[lo]);
      }
    }
    if (MODE == 2) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (pos[u] >= 0) {
          g_out[pos[u]] = r[u].x;
          g_yb[pos[u]] = (int64_t)(uint32_t)r[u].y;
          g_yl[pos[u]] = stage_len[pr + u * GB_BLOCK + (int)threadIdx.x];
        }
    } else {
      int64_t st[U], en[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int yy = pos[u] >= 0 ? r[u].y : 0;
        st[u] = rp[yy];
        en[u] = rp[yy + 1];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (pos[u] >= 0) {
          g_out[pos[u]] = r[u].x;
          g_yb[pos[u]] = st[u];
          g_yl[pos[u]] = (int32_t)(en[u] - st[u]);
          if (g_y) g_y[pos[u]] = r[u].y;
        }
    }
  }
}

// active sources = ids with cnt > 0, ascending (tile counts -> scan -> writes)
__global__ __launch_bounds__(SCAN_BLOCK) void k_nz_count(const int32_t* __restrict__ cnt, int64_t n,
                                                         int32_t* __restrict__ tile_cnt) {
  __shared__ int red[SCAN_BLOCK / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int v = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) v += (base + k < n && cnt[base + k] > 0) ? 1 : 0;
  int tot;
  block_exscan_i<SCAN_BLOCK>(v, red, &tot);
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_nz_write(const int32_t* __restrict__ cnt, int64_t n,
                                                         const int32_t* __restrict__ tile_off, int32_t xlo,
                                                         int32_t* __restrict__ active,
                                                         const int32_t* __restrict__ rank = nullptr,
                                                         int32_t* __restrict__ lpt = nullptr) {
  __shared__ int red[SCAN_BLOCK / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  bool h[SCAN_ITEMS];
  int v = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    h[k] = base + k < n && cnt[base + k] > 0;
    v += h[k] ? 1 : 0;
  }
  int tot;
  int o = block_exscan_i<SCAN_BLOCK>(v, red, &tot) + tile_off[blockIdx.x];
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k)
    if (h[k]) {
      active[o++] = xlo + (int32_t)(base + k);
      if (rank) lpt[rank[base + k]] = xlo + (int32_t)(base + k);  // BLP_LPT: the largest-first queue
    }
}

// ------------------------------------------------------------------ batch planning (device)
// blp_batch_create's statistics of a pair list, in one pass over its pairs on the device (round 5:
// the host walked every pair's row and built a first-appearance source list, 8-30 ms at config
// 2). Per pair: the id bounds, whether x is non-decreasing (source-grouped), |N(y)| (scan work),
// the id range of N(y) (the bitmap universe) and y (rows read). Per distinct source -- the thread
// that sets its bit in `seen` -- the graph's two-hop statistics (node2.hip): its H2 build work,
// the id range of N(N(x)), its longest member row, whether a member row is dense, and N(x)'s own
// id range (rows read); the source is appended to `srcs` (order not meaningful). Per-thread
// partials reduce through the wave, then one atomic per block and field.
struct PlanStats {
  unsigned long long lo, hi;            // universe: min / max + 1 over N(y) rows and N(N(x))
  unsigned long long rows_lo, rows_hi;  // rows read: the y, and the ids of N(x)
  unsigned long long xlo, xhi;          // sources' id range
  unsigned long long scan, max_scan;    // sum / max of |N(y)|
  unsigned long long work, max_build;   // sum of the sources' w2 / max member row
  unsigned long long n_sources;
  unsigned int bad, not_runs, any_hot;
};

constexpr int PLAN_BLOCK = 256;

__device__ inline unsigned long long wave_min_u64(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, (unsigned long long)__shfl_xor(v, o, 64));
  return v;
}
__device__ inline unsigned long long wave_max_u64(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (unsigned long long)__shfl_xor(v, o, 64));
  return v;
}
__device__ inline unsigned long long wave_sum_u64(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(PLAN_BLOCK) void k_plan_pairs(const int32_t* __restrict__ x, const int32_t* __restrict__ y,
                                                           int64_t np, int64_t n, const int64_t* __restrict__ rp,
                                                           const int32_t* __restrict__ ci,
                                                           const unsigned long long* __restrict__ w2,
                                                           const int32_t* __restrict__ lo2, const int32_t* __restrict__ hi2,
                                                           const int32_t* __restrict__ maxd, const uint8_t* __restrict__ flag2,
                                                           uint32_t* __restrict__ seen, int32_t* __restrict__ srcs,
                                                           PlanStats* __restrict__ st) {
  unsigned long long lo = ~0ull, hi = 0, rlo = ~0ull, rhi = 0, xl = ~0ull, xh = 0, scan = 0, mscan = 0, work = 0,
                     mbuild = 0, nsrc = 0;
  unsigned bad = 0, nruns = 0, hot = 0;
  for (int64_t i = (int64_t)blockIdx.x * PLAN_BLOCK + threadIdx.x; i < np; i += (int64_t)gridDim.x * PLAN_BLOCK) {
    const int32_t xi = x[i], yi = y[i];
    const int32_t xp = i > 0 ? x[i - 1] : INT32_MIN;
    if (xi < 0 || xi >= n || yi < 0 || yi >= n) {
      bad = 1;
      continue;
    }
    nruns |= xp > xi ? 1u : 0u;
    const int64_t yb = rp[yi], ye = rp[yi + 1];
    scan += (unsigned long long)(ye - yb);
    mscan = max(mscan, (unsigned long long)(ye - yb));
    if (ye > yb) {
      lo = min(lo, (unsigned long long)ci[yb]);
      hi = max(hi, (unsigned long long)ci[ye - 1] + 1);
    }
    rlo = min(rlo, (unsigned long long)yi);
    rhi = max(rhi, (unsigned long long)yi + 1);
    if (xp == xi) continue;  // a run of one source (similarity.users' order): counted at its head
    const uint32_t bit = 1u << (xi & 31);
    if (seen[xi >> 5] & bit) continue;  // most repeats of a popular source stop at this read
    if (atomicOr(&seen[xi >> 5], bit) & bit) continue;
    srcs[atomicAdd(reinterpret_cast<unsigned long long*>(&st->n_sources), 1ull)] = xi;
    ++nsrc;
    xl = min(xl, (unsigned long long)xi);
    xh = max(xh, (unsigned long long)xi + 1);
    const int64_t xb = rp[xi], xe = rp[xi + 1];
    if (xe > xb) {
      work += w2[xi];
      mbuild = max(mbuild, (unsigned long long)maxd[xi]);
      hot |= flag2[xi] & 1u;
      if (lo2[xi] != INT32_MAX) {
        lo = min(lo, (unsigned long long)lo2[xi]);
        hi = max(hi, (unsigned long long)hi2[xi]);
      }
      rlo = min(rlo, (unsigned long long)ci[xb]);  // rows are sorted: N(x)'s first and last
      rhi = max(rhi, (unsigned long long)ci[xe - 1] + 1);
    }
  }
  (void)nsrc;
  lo = wave_min_u64(lo);
  rlo = wave_min_u64(rlo);
  xl = wave_min_u64(xl);
  hi = wave_max_u64(hi);
  rhi = wave_max_u64(rhi);
  xh = wave_max_u64(xh);
  mscan = wave_max_u64(mscan);
  mbuild = wave_max_u64(mbuild);
  scan = wave_sum_u64(scan);
  work = wave_sum_u64(work);
  const unsigned long long flags = wave_max_u64((unsigned long long)(bad | nruns << 1 | hot << 2));
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&st->lo, lo);
    atomicMax(&st->hi, hi);
    atomicMin(&st->rows_lo, rlo);
    atomicMax(&st->rows_hi, rhi);
    atomicMin(&st->xlo, xl);
    atomicMax(&st->xhi, xh);
    atomicAdd(&st->scan, scan);
    atomicMax(&st->max_scan, mscan);
    atomicAdd(&st->work, work);
    atomicMax(&st->max_build, mbuild);
    if (flags & 1) atomicOr(&st->bad, 1u);
    if (flags & 2) atomicOr(&st->not_runs, 1u);
    if (flags & 4) atomicOr(&st->any_hot, 1u);
  }
}

// Planning outputs that need the whole list's statistics first: the sources above the heavy
// candidate bound (their ids, for the host's heavy-source plan) and, for chunk-parallel batches,
// the hash-set routing flag of every source (flag indexed by node id: hflag[x - base]).
__global__ void k_plan_sources(const int32_t* __restrict__ srcs, int64_t ns, const unsigned long long* __restrict__ w2,
                               const int64_t* __restrict__ rp, unsigned long long heavy_min, int32_t* __restrict__ heavy,
                               unsigned int* __restrict__ n_heavy, unsigned int heavy_cap, uint8_t* __restrict__ hflag,
                               int64_t hbase, unsigned long long hash_cap, unsigned int* __restrict__ n_hash) {
  unsigned nh = 0;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < ns; s += (int64_t)gridDim.x * blockDim.x) {
    const int32_t xs = srcs[s];
    const unsigned long long w = rp[xs + 1] > rp[xs] ? w2[xs] : 0ull;
    if (heavy && w > heavy_min) {
      const unsigned k = atomicAdd(n_heavy, 1u);
      if (k < heavy_cap) heavy[k] = xs;
    }
    if (hflag && w <= hash_cap) {
      hflag[xs - hbase] = 1;
      ++nh;
    }
  }
  if (hflag) {
    for (int o = 32; o > 0; o >>= 1) nh += __shfl_xor(nh, o, 64);
    if ((threadIdx.x & 63) == 0 && nh) atomicAdd(n_hash, nh);
  }
}

// ------------------------------------------------------------------ source records
// Everything the short-row scorer needs about an active source before its first global read of
// row data, gathered once per step after grouping: one 64-byte record per active source (read
// with scalar loads) instead of the dependent chain active[s] -> off / cnt / rp / wp / heavy ->
// ci[rp] (three round trips per source on the latency-bound business side).
struct SrcRec {
  int32_t x, pbeg, pcnt, hslot;
  int64_t xb, xe;  // N(x) = ci[xb, xe)
  int64_t wb, we;  // wedge row of x, in 16-byte vectors (wb == we: none)
  int32_t nx_lo, nx_hi;  // first and last id of N(x) (nx_hi < nx_lo: empty)
  int32_t pad[2];
};
static_assert(sizeof(SrcRec) == 64, "one 64-byte record per source");

// ---- grouping of a pair list that arrives already grouped by source (x non-decreasing, as
// similarity.users walks examples.json: every user's businesses together, similarity.py:
// 30-32): the runs of equal x ARE the groups, so instead of the bucket sort one pass finds
// the run heads (tile counts -> scan -> writes) and the grouped order is the caller's own.
__device__ inline bool run_head(const int32_t* __restrict__ x, int64_t i) { return i == 0 || x[i] != x[i - 1]; }

__global__ __launch_bounds__(SCAN_BLOCK) void k_run_count(const int32_t* __restrict__ x, int64_t np,
                                                          int32_t* __restrict__ tile_cnt, int32_t* __restrict__ zero,
                                                          int zero_words) {
  __shared__ int red[SCAN_BLOCK / 64];
  // block 0 zeroes the batch's counters (Misc up to dbg), which no kernel reads before the next
  // one in stream order: one launch and one dependency fewer than a memset in front
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < zero_words; i += SCAN_BLOCK) zero[i] = 0;
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int v = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) v += (base + k < np && run_head(x, base + k)) ? 1 : 0;
  int tot;
  block_exscan_i<SCAN_BLOCK>(v, red, &tot);
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_run_write(const int32_t* __restrict__ x, const int32_t* __restrict__ y,
                                                          int64_t np, const int64_t* __restrict__ rp,
                                                          const int32_t* __restrict__ tile_off, int32_t* __restrict__ active,
                                                          int32_t* __restrict__ off, int32_t* __restrict__ g_out,
                                                          int64_t* __restrict__ g_yb, int32_t* __restrict__ g_yl,
                                                          int32_t* __restrict__ g_y) {
  __shared__ int red[SCAN_BLOCK / 64];
  const int64_t t0 = (int64_t)blockIdx.x * SCAN_TILE;
  // per-pair metadata, coalesced; the tile's y loads, then its row_ptr gathers, all in flight
  constexpr int PT = SCAN_TILE / SCAN_BLOCK;
  if (g_yb) {  // (null: the scorer reads y and rp itself, pair_row)
    int yv[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const int64_t i = t0 + q * SCAN_BLOCK + threadIdx.x;
      yv[q] = i < np ? y[i] : 0;
    }
    int64_t st[PT], en[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      st[q] = rp[yv[q]];
      en[q] = rp[yv[q] + 1];
    }
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const int64_t i = t0 + q * SCAN_BLOCK + threadIdx.x;
      if (i < np) {
        if (g_out) g_out[i] = (int32_t)i;
        g_yb[i] = st[q];
        g_yl[i] = (int32_t)(en[q] - st[q]);
        if (g_y) g_y[i] = yv[q];
      }
    }
  }
  const int64_t base = t0 + (int64_t)threadIdx.x * SCAN_ITEMS;
  bool h[SCAN_ITEMS];
  int v = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    h[k] = base + k < np && run_head(x, base + k);
    v += h[k] ? 1 : 0;
  }
  int tot;
  int o = block_exscan_i<SCAN_BLOCK>(v, red, &tot) + tile_off[blockIdx.x];
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k)
    if (h[k]) {
      const int xi = x[base + k];
      active[o++] = xi;
      off[xi] = (int32_t)(base + k);
    }
}

// cnt of every run from the next run's head (after k_run_write: off[] of all heads). rank (or
// null): the batch's largest-first order (BLP_LPT, planned at create), the sources copied into
// lpt in that order for the scorer's queue.
__global__ void k_run_cnt(const int32_t* __restrict__ active, const int32_t* __restrict__ n_active, int64_t np,
                          const int32_t* __restrict__ off, int32_t* __restrict__ cnt,
                          const int32_t* __restrict__ rank = nullptr, int32_t xlo = 0, int32_t* __restrict__ lpt = nullptr,
                          SrcRec* __restrict__ rec = nullptr, const int64_t* __restrict__ rp = nullptr,
                          const int32_t* __restrict__ ci = nullptr, const int32_t* __restrict__ heavy_slot = nullptr) {
  const int na = *n_active;
  for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < na; a += gridDim.x * blockDim.x) {
    const int xa = active[a];
    const int pb = off[xa];
    const int nxt = a + 1 < na ? off[active[a + 1]] : (int)np;
    cnt[xa] = nxt - pb;
    const int s = rank ? rank[xa - xlo] : a;  // the source's place in the scorer's queue
    if (rank) lpt[s] = xa;
    if (rec) {  // the large scorer's source record (as k_source_records, without a wedge row)
      SrcRec r;
      r.x = xa;
      r.pbeg = pb;
      r.pcnt = nxt - pb;
      r.hslot = heavy_slot ? heavy_slot[xa] : -1;
      r.xb = rp[xa];
      r.xe = rp[xa + 1];
      r.wb = r.we = 0;
      r.nx_lo = r.xe > r.xb ? ci[r.xb] : 0;
      r.nx_hi = r.xe > r.xb ? ci[r.xe - 1] : -1;
      r.pad[0] = r.pad[1] = 0;
      rec[s] = r;
    }
  }
}

// Run-grouped batches queued largest first (BLP_LPT) whose scorer reads source records: the
// whole grouping in two launches instead of four. Every source is one run (x non-decreasing), so
// the run heads need no prefix order: a head writes off[x] and its queue slot lpt[rank[x]], a run
// tail writes its end into cnt[x]; block 0 zeroes the counters and sets n_active (the number of
// sources). k_run_records then turns the ends into counts and writes the records.
__global__ __launch_bounds__(256) void k_run_heads(const int32_t* __restrict__ x, int64_t np, int32_t xlo,
                                                   const int32_t* __restrict__ rank, int32_t* __restrict__ off,
                                                   int32_t* __restrict__ end, int32_t* __restrict__ lpt,
                                                   int32_t* __restrict__ misc_words, int zero_words, int32_t n_sources) {
  static_assert(offsetof(Misc, n_active) == 0, "n_active is the counters' first word");
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < zero_words; i += blockDim.x) misc_words[i] = i == 0 ? n_sources : 0;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < np; p += (int64_t)gridDim.x * blockDim.x) {
    const int xi = x[p];
    if (p == 0 || x[p - 1] != xi) {
      off[xi] = (int32_t)p;
      lpt[rank[xi - xlo]] = xi;
    }
    if (p == np - 1 || x[p + 1] != xi) end[xi] = (int32_t)(p + 1);
  }
}

__global__ __launch_bounds__(256) void k_run_records(const int32_t* __restrict__ lpt, int32_t n_sources,
                                                     const int32_t* __restrict__ off, int32_t* __restrict__ cnt,
                                                     const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                     const int32_t* __restrict__ heavy_slot, SrcRec* __restrict__ rec) {
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < n_sources; s += gridDim.x * blockDim.x) {
    const int xa = lpt[s];
    const int pb = off[xa], n = cnt[xa] - pb;  // cnt held the run's end
    cnt[xa] = n;
    SrcRec r;
    r.x = xa;
    r.pbeg = pb;
    r.pcnt = n;
    r.hslot = heavy_slot ? heavy_slot[xa] : -1;
    r.xb = rp[xa];
    r.xe = rp[xa + 1];
    r.wb = r.we = 0;
    r.nx_lo = r.xe > r.xb ? ci[r.xb] : 0;
    r.nx_hi = r.xe > r.xb ? ci[r.xe - 1] : -1;
    r.pad[0] = r.pad[1] = 0;
    rec[s] = r;
  }
}

// BLP_LPT planning: each source's scan work, sum of |N(y)| over its pairs (wave-aggregated when
// the wave's pairs share their source, as run-grouped lists do), into est[x - xlo]
__global__ void k_src_scan_work(const int32_t* __restrict__ x, const int32_t* __restrict__ y, int64_t np,
                                const int64_t* __restrict__ rp, int32_t xlo, unsigned long long* __restrict__ est) {
  const int lane = (int)threadIdx.x & 63;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < np; i0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = i0 + threadIdx.x;
    const bool in = i < np;
    const int xi = in ? x[i] : INT32_MIN;
    const unsigned long long w = in ? (unsigned long long)(rp[y[i] + 1] - rp[y[i]]) : 0ull;
    const int x0 = __shfl(xi, 0, 64);
    const bool same = __all(!in || xi == x0);
    if (same) {
      unsigned long long t = w;
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
      if (lane == 0 && x0 != INT32_MIN) atomicAdd(&est[x0 - xlo], t);
    } else if (in) {
      atomicAdd(&est[xi - xlo], w);
    }
  }
}

// est of source i = its scan work + its build work w2[x]
__global__ void k_src_est(const int32_t* __restrict__ srcs, int64_t n, const unsigned long long* __restrict__ est,
                          const unsigned long long* __restrict__ w2, int32_t xlo, unsigned long long* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = est[srcs[i] - xlo] + w2[srcs[i]];
}

// ord[j] = list index of the source placed j-th: rank[srcs[ord[j]] - xlo] = j
__global__ void k_src_rank(const int32_t* __restrict__ srcs, int64_t n, const int32_t* __restrict__ ord, int32_t xlo,
                           int32_t* __restrict__ rank) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
    rank[srcs[ord[j]] - xlo] = (int32_t)j;
}

constexpr int DQ_MAX = 8;  // sources per dequeue (blp_batch::dq)

template <int KEYS>
__global__ __launch_bounds__(GB_BLOCK) void k_active_write(const int32_t* __restrict__ cnt,
                                                           const int32_t* __restrict__ abase, int shift, int32_t xlo,
                                                           int64_t xspan, int32_t* __restrict__ active) {
  constexpr int PER = KEYS >= GB_BLOCK ? KEYS / GB_BLOCK : 1;  // j < nk <= KEYS guards the rest
  __shared__ int red[GB_BLOCK / 64];
  const int b = blockIdx.x;
  const int64_t k0 = (int64_t)xlo + ((int64_t)b << shift);
  const int nk = (int)min<int64_t>((int64_t)1 << shift, xspan - ((int64_t)b << shift));
  int v = 0;
  for (int q = 0; q < PER; ++q) {
    const int j = threadIdx.x * PER + q;
    v += j < nk && cnt[k0 + j] > 0;
  }
  int tot;
  int o = block_exscan_i<GB_BLOCK>(v, red, &tot) + abase[b];
  for (int q = 0; q < PER; ++q) {
    const int j = threadIdx.x * PER + q;
    if (j < nk && cnt[k0 + j] > 0) active[o++] = (int32_t)(k0 + j);
  }
}

// ------------------------------------------------------------------ segment machinery
// Exclusive scan of one int per thread over the block (values of threads >= n are 0). TAIL = false
// drops the closing barrier (it only keeps red from being rewritten while other waves still read
// it): for callers that write their results and reach a barrier before red's next use.
template <int BLOCK, bool TAIL = true>
__device__ inline int block_exscan(int v, int* red, int* total) {
  constexpr int NW = BLOCK / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(inc, d, 64);
    if (lane >= d) inc += t;
  }
  if (lane == 63) red[wid] = inc;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int t = red[w];
    base += w < wid ? t : 0;
    tot += t;
  }
  if (TAIL) __syncthreads();
  *total = tot;
  return base + inc - v;
}

// last s in [lo, hi) with off[s] <= f (requires off[lo] <= f < off[hi])
__device__ __attribute__((always_inline)) inline int seg_search(const int32_t* off, int ns, int f, int lo = 0, int hi = -1) {
  if (hi < 0) hi = ns;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (off[mid] <= f)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// Segment hint table of a batch of segments: hint[j] = segment of element min(j << shift,
// T - 1), for j <= ((T - 1) >> shift) + 1. A merge-path step then binary-searches only
// [hint[f0 >> shift], hint[(f0 >> shift) + 1]] -- one or two LDS round trips on long rows
// instead of log2(ns) dependent ones, which are most of a step's latency. Built once per
// batch (every thread one search at most), ending with a barrier. Returns shift, or -1 (no
// hint) when the batch is a single block step anyway.
template <int BLOCK, int CAP>
__device__ __attribute__((always_inline)) inline int build_hint(const int32_t* s_off, int ns, int step, int32_t* hint) {
  const int T = s_off[ns];
  if (CAP < 4 || T <= step) return -1;
  int shift = 0;
  while (((T - 1) >> shift) + 2 > CAP) ++shift;
  const int nh = ((T - 1) >> shift) + 1;
  for (int j = threadIdx.x; j <= nh; j += BLOCK) hint[j] = seg_search(s_off, ns, min(j << shift, T - 1));
  __syncthreads();
  return shift;
}

// Fetch one merge-path step: the K consecutive elements [f0, f0 + K) of the concatenated
// segments (w = node id or -1, sk = segment or -1). One LDS binary search per K elements
// (narrowed by the hint table when given: shift >= 0).
template <int K>
__device__ __attribute__((always_inline)) inline void mp_fetch(const int32_t* __restrict__ ci, const int64_t* s_start, const int32_t* s_off, int ns,
                                int T, int f0, int* w, int* sk, const int32_t* hint = nullptr, int shift = -1) {
  if (f0 >= T) {
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = sk[k] = -1;
    return;
  }
  int s;
  if (shift >= 0) {
    const int g = f0 >> shift;
    s = seg_search(s_off, ns, f0, hint[g], hint[g + 1] + 1);
  } else {
    s = seg_search(s_off, ns, f0);
  }
  int next = s_off[s + 1];
  int64_t pos = s_start[s] + (f0 - s_off[s]);
  if (f0 + K <= next) {
    // all K elements in one row (the common case on long rows): K/4 16-byte loads, which
    // gfx950 serves at 4-byte alignment, instead of K dword loads
    const blp::U4a* p = reinterpret_cast<const blp::U4a*>(ci + pos);
#pragma unroll
    for (int j = 0; j < K / 4; ++j) {
      const blp::U4a v = p[j];
      w[4 * j] = v.x;
      w[4 * j + 1] = v.y;
      w[4 * j + 2] = v.z;
      w[4 * j + 3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) sk[k] = s;
    return;
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int f = f0 + k;
    w[k] = -1;
    sk[k] = -1;
    if (f < T) {
      while (f >= next) {
        ++s;
        next = s_off[s + 1];
        pos = s_start[s];
      }
      w[k] = ci[pos];
      ++pos;
      sk[k] = s;
    }
  }
}

// Set the bits of every element of the ns segments (rows of ci) inside [c0, c0 + width).
// Software-pipelined: the loads of step i+1 are in flight while step i's atomics issue.
// ci may be the weight-coded copy of the column ids (ScoreArgs::cw): ids are ci & idmask.
// Offset of element value v (an id, possibly weight-coded, or -1 = no element) in the chunk
// [c0, c0 + width): one unsigned compare "< width" then tests both validity and range. keep =
// idmask | sign bit, so -1 maps to >= 2^31 - c0 > width (c0 <= idmask, width < 2^31).
__device__ inline uint32_t in_chunk(int v, uint32_t keep, uint32_t c0u) { return ((uint32_t)v & keep) - c0u; }

// Exact AA terms of the hit ids e[j] (bit j of hm): the code weights from the LDS code table
// (wtab[0] = 0), then the code-0 hits' per-node weights from the global table in a loop of their
// own. (A per-id `code ? wtab[code] : aaw[id]` compiles to one flat load of a selected LDS-or-
// global address, which waits on both memory counters at every hit.)
template <int N>
__device__ __attribute__((always_inline)) inline void aa_terms(const int* e, uint32_t hm, int idbits, uint32_t idmask,
                                                               const long long* wtab, const long long* __restrict__ aaw,
                                                               unsigned long long& acc, uint32_t& acch) {
  uint32_t esc = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const uint32_t code = ((uint32_t)e[j] >> idbits) & 255u;
    const unsigned long long w = ((hm >> j) & 1u) ? (unsigned long long)wtab[code] : 0ull;
    acc += w;
    acch += (uint32_t)(w >> 32);
    esc |= (((hm >> j) & 1u) && code == 0u) ? 1u << j : 0u;
  }
  if (esc) {
#pragma unroll
    for (int j = 0; j < N; ++j)
      if ((esc >> j) & 1u) {
        const unsigned long long w = (unsigned long long)aaw[e[j] & idmask];
        acc += w;
        acch += (uint32_t)(w >> 32);
      }
  }
}

// Exact Adamic-Adar accumulation (blp_internal.h): a term W adds to the wrapping low word and
// its high half to the exact high word. LDS accumulators are interleaved: s_aa[2 t] = lo,
// s_aa[2 t + 1] = hi for segment t.
__device__ inline void aa_push(unsigned long long* s_aa, int t, unsigned long long lo, unsigned long long hi) {
  atomicAdd(&s_aa[2 * t], lo);
  atomicAdd(&s_aa[2 * t + 1], hi);
}

// Packed layout (see rc_scan): the high word in units of 2^PK_HS shares the count's word.
constexpr int PK_CN_BITS = 21;
constexpr int PK_HS = 40;
// One scan run's contribution: count c, low sum lo, high-word sum hh (a run spans <= 32 terms of
// W >> 32 < 2^27, so hh fits 32 bits). Packed: two atomics; else the count and the two words.
template <bool AA, bool PK>
__device__ inline void scan_push(uint32_t* s_cn, unsigned long long* s_aa, int seg, unsigned c, unsigned long long lo,
                                 uint32_t hh) {
  if (PK && AA) {
    atomicAdd(&s_aa[2 * seg], lo);
    atomicAdd(&s_aa[2 * seg + 1], ((unsigned long long)(hh >> (PK_HS - 32)) << PK_CN_BITS) | c);
  } else if (PK) {  // counts only, in the packed word
    atomicAdd(&s_aa[2 * seg + 1], (unsigned long long)c);
  } else {
    atomicAdd(&s_cn[seg], c);
    if (AA) aa_push(s_aa, seg, lo, (unsigned long long)hh);
  }
}

template <int NT, int K, bool GLOBAL = false>
__device__ __attribute__((always_inline)) inline void mp_build(const int32_t* __restrict__ ci, uint32_t idmask, const int64_t* s_start,
                                const int32_t* s_off, int ns, int64_t c0, int64_t width, uint32_t* bm, int tid,
                                const int32_t* hint = nullptr, int shift = -1) {
  const int T = s_off[ns];
  constexpr int STEP = NT * K;
  const uint32_t keep = idmask | 0x80000000u, c0u = (uint32_t)c0, wu = (uint32_t)width;
  int w[K], sk[K];
  mp_fetch<K>(ci, s_start, s_off, ns, T, tid * K, w, sk, hint, shift);
  for (int base = 0; base < T; base += STEP) {
    int wn[K], skn[K];
    mp_fetch<K>(ci, s_start, s_off, ns, T, base + STEP + tid * K, wn, skn, hint, shift);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      // one unsigned compare tests validity and range (see in_chunk)
      const uint32_t r = in_chunk(w[k], keep, c0u);
      if (r < wu) {
        if (GLOBAL)  // the workgroup's private HBM bitmap: the OR is done in the XCD's L2
          __hip_atomic_fetch_or(&bm[r >> 5], 1u << (r & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
          atomicOr(&bm[r >> 5], 1u << (r & 31));
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      w[k] = wn[k];
      sk[k] = skn[k];
    }
  }
}

// Test every element of the ns segments against the bitmap; per-segment hit counts and
// fixed-point Adamic-Adar sums accumulate into s_cn / s_aa (LDS). Pipelined like mp_build;
// the weight gathers of a step are issued BEFORE the next step's loads, so waiting for them
// (vmcnt counts in issue order) does not also wait for the prefetch.
// ci may be the weight-coded copy (ScoreArgs::cw): an element is id | code << idbits; code c
// > 0 has the weight wtab[c], code 0 falls back to the per-node table aaw[id].

template <int NT, int K, bool AA, bool PK = false>
__device__ __attribute__((always_inline)) inline void mp_scan(const int32_t* __restrict__ ci, uint32_t idmask, int idbits,
                               const long long* __restrict__ aaw, const long long* wtab, const int64_t* s_start,
                               const int32_t* s_off, int ns, int64_t c0, int64_t width, const uint32_t* bm,
                               uint32_t* s_cn, unsigned long long* s_aa, int tid, const int32_t* hint = nullptr,
                               int shift = -1) {
  const int T = s_off[ns];
  constexpr int STEP = NT * K;
  const uint32_t keep = idmask | 0x80000000u, c0u = (uint32_t)c0, wu = (uint32_t)width;
  int w[K], sk[K];
  mp_fetch<K>(ci, s_start, s_off, ns, T, tid * K, w, sk, hint, shift);
  for (int base = 0; base < T; base += STEP) {
    // the bitmap words and (AA) the code weights wtab[code] are read together, so one LDS
    // round trip serves both; hits with code 0 then gather aaw, before the next step's loads
    // are issued (rare on a coded id stream)
    bool hit[K];
    long long wt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t r = in_chunk(w[k], keep, c0u);
      const bool in = r < wu;
      const uint32_t word = bm[(in ? r : 0u) >> 5];
      if (AA) wt[k] = wtab[((uint32_t)w[k] >> idbits) & 255u];
      hit[k] = in && ((word >> (r & 31)) & 1u);
    }
    if (AA) {
      bool any_esc = false;
#pragma unroll
      for (int k = 0; k < K; ++k) any_esc |= hit[k] && ((uint32_t)w[k] >> idbits) == 0u;
      if (any_esc) {
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (hit[k] && ((uint32_t)w[k] >> idbits) == 0u) wt[k] = aaw[w[k] & idmask];
      }
#pragma unroll
      for (int k = 0; k < K; ++k) wt[k] = hit[k] ? wt[k] : 0ll;
    }
    int wn[K], skn[K];
    mp_fetch<K>(ci, s_start, s_off, ns, T, base + STEP + tid * K, wn, skn, hint, shift);
    if (sk[0] == sk[K - 1]) {  // the K elements in one segment (or none valid): one run
      unsigned c = 0;
      unsigned long long acc = 0;
      uint32_t acch = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        c += hit[k] ? 1u : 0u;
        if (AA) {
          acc += (unsigned long long)wt[k];
          acch += (uint32_t)((unsigned long long)wt[k] >> 32);
        }
      }
      if (c) scan_push<AA, PK>(s_cn, s_aa, sk[0], c, acc, acch);
    } else {
      int cur = sk[0];
      unsigned c = 0;
      unsigned long long acc = 0;
      uint32_t acch = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (sk[k] != cur) {
          if (c) scan_push<AA, PK>(s_cn, s_aa, cur, c, acc, acch);
          cur = sk[k];
          c = 0;
          acc = 0;
          acch = 0;
        }
        if (hit[k]) {
          ++c;
          if (AA) {
            acc += (unsigned long long)wt[k];
            acch += (uint32_t)((unsigned long long)wt[k] >> 32);
          }
        }
      }
      if (c && cur >= 0) scan_push<AA, PK>(s_cn, s_aa, cur, c, acc, acch);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      w[k] = wn[k];
      sk[k] = skn[k];
    }
  }
}

// ------------------------------------------------------------------ ping-pong merge-path loops
// mp_build / mp_scan keep one step of prefetch in a register copy (w = wn at the loop end).
// The copy needs the prefetched data, and mp_fetch issues 0, K/4 or K loads depending on the
// lane's path, so the compiler's wait before a use is vmcnt(0): each step's global latency is
// exposed and only the 16 waves of the CU hide it. Here two register buffers alternate (the
// loop is unrolled by two, no copies), and every fetch issues exactly 2 * K/4 16-byte loads
// on every path, so the wait before a step's use is vmcnt(2 * K/4): the other buffer's loads
// stay in flight while the step's LDS work runs.
//
// One fetch covers elements [f0, f0 + K): the lane's first row from f0 (vector a), and the
// first non-empty row after it (vector b), read from rem1 ids BEFORE that row's start so that
// element k is a[k] for k < rem1 and b[k] otherwise (ci carries CI_PAD ids of padding on
// both sides). The selection happens at use (PPStep::id), so nothing waits on the loads at
// fetch time. Elements in a third row (only when a row is shorter than K) are handed to
// `rare` at once with plain loads.
// s_waitcnt vmcnt(0) (gfx9 encoding: expcnt and lgkmcnt at their maxima). Each ping-pong loop
// leaves one unused fetch in flight on exit; draining it there keeps the compiler's pending-
// load bookkeeping clean at the next loop's header, where it would otherwise insert waits
// for registers it reuses -- waits that, vmcnt being a counter, stall on the live buffer.
__device__ inline void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

template <int K>
struct PPStep {
  int va[K], vb[K];
  int s1, s2, rem1, limb, lim;  // segments, elements in s1, elements in s1 + s2, valid elements
  __device__ inline int id(int k) const { return k >= lim ? -1 : k < rem1 ? va[k] : k < limb ? vb[k] : -1; }
  // Mark every loaded register as used here, on every path: the compiler then waits for the
  // whole step at once (vmcnt = the other buffer's loads) and knows them complete afterwards;
  // otherwise a register some path never reads stays "pending" into the next iteration,
  // where reusing it costs a wait on the live buffer.
  __device__ inline void land() const {
#pragma unroll
    for (int k = 0; k < K; ++k) asm volatile("" ::"v"(va[k]), "v"(vb[k]));
  }
};

template <int K, typename Rare>
__device__ inline void pp_fetch(const int32_t* __restrict__ ci, const int64_t* s_start, const int32_t* s_off, int ns,
                                int T, int f0, const int32_t* hint, int shift, PPStep<K>& st, Rare rare) {
  int64_t p1 = 0, p2 = 0;
  int n2 = 0;
  st.s1 = -1;
  st.s2 = -1;
  st.rem1 = 0;
  const bool valid = f0 < T;
  if (valid) {
    int s;
    if (shift >= 0) {
      const int g = f0 >> shift;
      s = seg_search(s_off, ns, f0, hint[g], hint[g + 1] + 1);
    } else {
      s = seg_search(s_off, ns, f0);
    }
    const int next = s_off[s + 1];
    st.s1 = s;
    st.rem1 = next - f0;
    p1 = s_start[s] + (f0 - s_off[s]);
    p2 = p1;
    if (st.rem1 < K && next < T) {
      int t = s + 1;
      while (s_off[t + 1] == next) ++t;  // skip empty rows; one with elements exists (next < T)
      st.s2 = t;
      n2 = s_off[t + 1];
      p2 = s_start[t] - st.rem1;
    }
  }
  const blp::U4a* q1 = reinterpret_cast<const blp::U4a*>(ci + p1);
  const blp::U4a* q2 = reinterpret_cast<const blp::U4a*>(ci + p2);
#pragma unroll
  for (int j = 0; j < K / 4; ++j) {
    const blp::U4a v = q1[j];
    st.va[4 * j] = v.x;
    st.va[4 * j + 1] = v.y;
    st.va[4 * j + 2] = v.z;
    st.va[4 * j + 3] = v.w;
  }
#pragma unroll
  for (int j = 0; j < K / 4; ++j) {
    const blp::U4a v = q2[j];
    st.vb[4 * j] = v.x;
    st.vb[4 * j + 1] = v.y;
    st.vb[4 * j + 2] = v.z;
    st.vb[4 * j + 3] = v.w;
  }
  st.limb = st.s2 >= 0 ? n2 - f0 : 0;
  st.lim = valid ? min(T - f0, K) : 0;
  if (st.s2 >= 0 && st.limb < st.lim) {  // a third row: rows shorter than K only
    int t = st.s2;
    for (int f = f0 + st.limb; f < f0 + st.lim; ++f) {
      while (s_off[t + 1] <= f) ++t;
      rare(ci[s_start[t] + (f - s_off[t])], t);
    }
  }
}

// Build: set the bits of every element of the ns segments inside [c0, c0 + width).
template <int NT, int K>
__device__ __attribute__((always_inline)) inline void pp_build(const int32_t* __restrict__ ci, uint32_t idmask, const int64_t* s_start,
                                const int32_t* s_off, int ns, int64_t c0, int64_t width, uint32_t* bm, int tid,
                                const int32_t* hint, int shift) {
  const int T = s_off[ns];
  constexpr int STEP = NT * K;
  const uint32_t keep = idmask | 0x80000000u, c0u = (uint32_t)c0, wu = (uint32_t)width;
  auto mark = [&](int v) {
    const uint32_t r = in_chunk(v, keep, c0u);
    if (r < wu) atomicOr(&bm[r >> 5], 1u << (r & 31));
  };
  auto rare = [&](int v, int) { mark(v); };
  auto proc = [&](const PPStep<K>& st) {
    st.land();
#pragma unroll
    for (int k = 0; k < K; ++k) mark(st.id(k));
  };
  // no exit from the middle of the body: a path leaving with B in flight would merge into the
  // loop header's pending-load state (the waits of the next loop would stall on live loads)
  const int nsteps = (T + STEP - 1) / STEP;
  PPStep<K> A, B;
  vm_drain();  // nothing older than A may look pending at the loop header
  pp_fetch<K>(ci, s_start, s_off, ns, T, tid * K, hint, shift, A, rare);
  for (int i = 0; i + 1 < nsteps; i += 2) {
    pp_fetch<K>(ci, s_start, s_off, ns, T, (i + 1) * STEP + tid * K, hint, shift, B, rare);
    proc(A);
    pp_fetch<K>(ci, s_start, s_off, ns, T, (i + 2) * STEP + tid * K, hint, shift, A, rare);  // may be past T
    proc(B);
  }
  if (nsteps & 1) proc(A);
  vm_drain();
}

// Scan: test every element against the bitmap; hits accumulate per segment into s_cn / s_aa.
// A step's elements lie in at most two segments (s1: k < rem1, s2: the rest), so a step ends
// with at most two pairs of LDS atomics.
template <int NT, int K, bool AA>
__device__ __attribute__((always_inline)) inline void pp_scan(const int32_t* __restrict__ ci, uint32_t idmask, int idbits,
                               const long long* __restrict__ aaw, const long long* wtab, const int64_t* s_start,
                               const int32_t* s_off, int ns, int64_t c0, int64_t width, const uint32_t* bm,
                               uint32_t* s_cn, unsigned long long* s_aa, int tid, const int32_t* hint, int shift) {
  const int T = s_off[ns];
  constexpr int STEP = NT * K;
  const uint32_t keep = idmask | 0x80000000u, c0u = (uint32_t)c0, wu = (uint32_t)width;
  auto rare = [&](int v, int seg) {
    const uint32_t r = in_chunk(v, keep, c0u);
    if (r < wu && ((bm[r >> 5] >> (r & 31)) & 1u)) {
      atomicAdd(&s_cn[seg], 1u);
      if (AA) {
        unsigned long long w = 0;
        uint32_t wh = 0;
        aa_terms<1>(&v, 1u, idbits, idmask, wtab, aaw, w, wh);
        aa_push(s_aa, seg, w, w >> 32);
      }
    }
  };
  auto proc = [&](const PPStep<K>& st) {
    st.land();
    int w[K];
    bool hit[K];
    long long wt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      w[k] = st.id(k);
      const uint32_t r = in_chunk(w[k], keep, c0u);
      const bool in = r < wu;
      const uint32_t word = bm[(in ? r : 0u) >> 5];
      if (AA) wt[k] = wtab[((uint32_t)w[k] >> idbits) & 255u];
      hit[k] = in && ((word >> (r & 31)) & 1u);
    }
    if (AA) {
      bool any_esc = false;
#pragma unroll
      for (int k = 0; k < K; ++k) any_esc |= hit[k] && ((uint32_t)w[k] >> idbits) == 0u;
      if (any_esc) {  // code-0 ids: gather the per-node weight (rare on a coded id stream)
#pragma unroll
        for (int k = 0; k < K; ++k)
          if (hit[k] && ((uint32_t)w[k] >> idbits) == 0u) wt[k] = aaw[w[k] & idmask];
      }
    }
    unsigned c1 = 0, c2 = 0;
    unsigned long long x1 = 0, x2 = 0;
    uint32_t h1 = 0, h2 = 0;  // <= K terms of W >> 32 < 2^27 each
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const unsigned h = hit[k] ? 1u : 0u;
      const unsigned long long v = (AA && hit[k]) ? (unsigned long long)wt[k] : 0ull;
      if (k < st.rem1) {
        c1 += h;
        x1 += v;
        h1 += (uint32_t)(v >> 32);
      } else {
        c2 += h;
        x2 += v;
        h2 += (uint32_t)(v >> 32);
      }
    }
    if (c1) {
      atomicAdd(&s_cn[st.s1], c1);
      if (AA) aa_push(s_aa, st.s1, x1, (unsigned long long)h1);
    }
    if (c2) {
      atomicAdd(&s_cn[st.s2], c2);
      if (AA) aa_push(s_aa, st.s2, x2, (unsigned long long)h2);
    }
  };
  // no exit from the middle of the body: a path leaving with B in flight would merge into the
  // loop header's pending-load state (the waits of the next loop would stall on live loads)
  const int nsteps = (T + STEP - 1) / STEP;
  PPStep<K> A, B;
  vm_drain();  // nothing older than A may look pending at the loop header
  pp_fetch<K>(ci, s_start, s_off, ns, T, tid * K, hint, shift, A, rare);
  for (int i = 0; i + 1 < nsteps; i += 2) {
    pp_fetch<K>(ci, s_start, s_off, ns, T, (i + 1) * STEP + tid * K, hint, shift, B, rare);
    proc(A);
    pp_fetch<K>(ci, s_start, s_off, ns, T, (i + 2) * STEP + tid * K, hint, shift, A, rare);  // may be past T
    proc(B);
  }
  if (nsteps & 1) proc(A);
  vm_drain();
}

// ------------------------------------------------------------------ row-chunk loops
// The merge-path step of pp_* may straddle rows, which costs every element a three-way select
// (own row / next row / past the end) and every step two segment atomics. Measured on the
// config-2 user side, the scorer is VALU-issue bound (25 % of wave cycles issuing with 4 waves
// per SIMD; ~28 VALU instructions per scanned element), so here the unit of work is a row
// CHUNK instead: row s of length L is cut into ceil(L / K) chunks of K ids, the chunks of a
// batch are numbered through (s_coff: exclusive chunk prefix per row), and a lane-step takes
// one chunk. Its K ids come from one row (K/4 16-byte loads; the last chunk of a row reads up
// to K-1 ids past it, masked by the count), so a step has one segment, one pair of atomics,
// and an element costs ~9 VALU (CN) + ~7 (AA). Padding: one short row wastes K - L lanes.
// Same two-buffer pipeline and vmcnt discipline as pp_*.
template <int K>
struct RCStep {
  int v[K];
  int s, cnt;  // row (segment) and valid ids of the chunk (0: none)
  __device__ inline void land() const {
#pragma unroll
    for (int k = 0; k < K; ++k) asm volatile("" ::"v"(v[k]));
  }
};

template <int K>
__device__ __attribute__((always_inline)) inline void rc_fetch(const int32_t* __restrict__ ci, const int64_t* s_start, const int32_t* s_off,
                                const int32_t* s_coff, int ns, int TC, int c, const int32_t* hint, int shift,
                                RCStep<K>& st) {
  int64_t pos = 0;
  st.s = 0;
  st.cnt = 0;
  if (c < TC) {
    int s;
    if (shift >= 0) {
      const int g = c >> shift;
      s = seg_search(s_coff, ns, c, hint[g], hint[g + 1] + 1);
    } else {
      s = seg_search(s_coff, ns, c);
    }
    const int o = (c - s_coff[s]) * K;
    st.s = s;
    st.cnt = min(K, s_off[s + 1] - s_off[s] - o);
    pos = s_start[s] + o;
  }
  const blp::U4a* q = reinterpret_cast<const blp::U4a*>(ci + pos);
#pragma unroll
  for (int j = 0; j < K / 4; ++j) {
    const blp::U4a x = q[j];
    st.v[4 * j] = x.x;
    st.v[4 * j + 1] = x.y;
    st.v[4 * j + 2] = x.z;
    st.v[4 * j + 3] = x.w;
  }
}

// Two-buffer driver: steps of NT chunks; proc(step) after the next step's loads are issued.
// (A third buffer, two steps of loads in flight, measured 2.28 vs 2.26 ms: not kept.)
template <int NT, int K, typename Proc>
__device__ __attribute__((always_inline)) inline void rc_loop(const int32_t* __restrict__ ci, const int64_t* s_start, const int32_t* s_off,
                               const int32_t* s_coff, int ns, int tid, const int32_t* hint, int shift, Proc proc) {
  const int TC = s_coff[ns];
  const int nsteps = (TC + NT - 1) / NT;
  RCStep<K> A, B;
  vm_drain();
  rc_fetch<K>(ci, s_start, s_off, s_coff, ns, TC, tid, hint, shift, A);
  for (int i = 0; i + 1 < nsteps; i += 2) {
    rc_fetch<K>(ci, s_start, s_off, s_coff, ns, TC, (i + 1) * NT + tid, hint, shift, B);
    proc(A);
    rc_fetch<K>(ci, s_start, s_off, s_coff, ns, TC, (i + 2) * NT + tid, hint, shift, A);  // may be past TC
    proc(B);
  }
  if (nsteps & 1) proc(A);
  vm_drain();
}

// LDS bitmap layout for the row-chunk loops: CAP words of bits, then RC_SAFE: one word that
// stays zero (scan lookups of out-of-chunk ids are clamped to it), then 32 per-lane dummy
// words that absorb the build's ORs of out-of-chunk / padding ids without a branch.
constexpr int RC_EXTRA_WORDS = 36;

template <int NT, int K>
__device__ __attribute__((always_inline)) inline void rc_build(const int32_t* __restrict__ ci, uint32_t idmask, const int64_t* s_start,
                                const int32_t* s_off, const int32_t* s_coff, int ns, int64_t c0, int64_t width,
                                uint32_t* bm, int cap_words, int tid, const int32_t* hint, int shift) {
  const uint32_t keep = idmask | 0x80000000u, c0u = (uint32_t)c0, wu = (uint32_t)width;
  const uint32_t dummy = (uint32_t)(cap_words + 1 + (tid & 31)) << 5;
  auto proc = [&](const RCStep<K>& st) {
    st.land();
#pragma unroll
    for (int k = 0; k < K; ++k) {  // branch-free: '&' not '&&' (no exec-mask blocks per id)
      const uint32_t r = ((uint32_t)st.v[k] & keep) - c0u;
      const uint32_t rr = ((k < st.cnt) & (r < wu)) ? r : dummy;
      atomicOr(&bm[rr >> 5], 1u << (rr & 31));
    }
  };
  rc_loop<NT, K>(ci, s_start, s_off, s_coff, ns, tid, hint, shift, proc);
}

// Packed exact-AA layout (packed = true, one LDS chunk): per segment t, s_aa[2 t] = Σ W (wrapping)
// and s_aa[2 t + 1] = (Σ_steps (Σ_step (W >> 32)) >> 8) << PK_CN_BITS | cn -- the high word in
// units of 2^40 shares the count's atomic, so a step issues the same two LDS atomics as a CN +
// 64-bit sum. Valid while cn < 2^PK_CN_BITS (a chunk holds < 2^21 nodes) : each step's high part
// undercounts S by < 2^40 + K * 2^32, so S - hi * 2^40 < cn * 2^41 < 2^64 (blp::aa_exact, hs = 40).

template <int NT, int K, bool AA>
__device__ __attribute__((always_inline)) inline void rc_scan(const int32_t* __restrict__ ci, uint32_t idmask, int idbits,
                               const long long* __restrict__ aaw, const long long* wtab, const int64_t* s_start,
                               const int32_t* s_off, const int32_t* s_coff, int ns, int64_t c0, int64_t width,
                               const uint32_t* bm, int cap_words, uint32_t* s_cn, unsigned long long* s_aa, int tid,
                               const int32_t* hint, int shift, bool packed = false) {
  const uint32_t keep = idmask | 0x80000000u, c0u = (uint32_t)c0, wu = (uint32_t)width;
  const uint32_t safe = (uint32_t)cap_words << 5;
  // Branch-free phases, so the scheduler can issue all K bitmap reads (and weight reads)
  // before the first use: one LDS round trip per step instead of one per id.
  auto proc = [&](const RCStep<K>& st) {
    st.land();
    uint32_t rr[K], wd[K];
    long long wt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t r = ((uint32_t)st.v[k] & keep) - c0u;
      rr[k] = ((k < st.cnt) & (r < wu)) ? r : safe;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) wd[k] = bm[rr[k] >> 5];
    if (AA) {
#pragma unroll
      for (int k = 0; k < K; ++k) wt[k] = wtab[((uint32_t)st.v[k] >> idbits) & 255u];
    }
    uint32_t hm = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) hm |= ((wd[k] >> (rr[k] & 31)) & 1u) << k;
    if (hm) {
      if (AA) {
        // the step's high words fit 32 bits: K <= 16 terms of W >> 32 < 2^27 (W < 2^59)
        unsigned long long acc = 0;
        uint32_t esc = 0, acch = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const bool h = (hm >> k) & 1u;
          const unsigned long long w = h ? (unsigned long long)wt[k] : 0ull;
          acc += w;
          acch += (uint32_t)(w >> 32);
          esc |= (h & ((((uint32_t)st.v[k] >> idbits) & 255u) == 0u)) ? 1u << k : 0u;
        }
        if (esc) {  // code-0 ids: the per-node weight (rare on a coded id stream)
#pragma unroll
          for (int k = 0; k < K; ++k)
            if ((esc >> k) & 1u) {
              const unsigned long long w = (unsigned long long)aaw[st.v[k] & idmask];
              acc += w;
              acch += (uint32_t)(w >> 32);
            }
        }
        if (packed) {
          atomicAdd(&s_aa[2 * st.s], acc);
          atomicAdd(&s_aa[2 * st.s + 1], ((unsigned long long)(acch >> (PK_HS - 32)) << PK_CN_BITS) | (unsigned)__popc(hm));
          return;
        }
        aa_push(s_aa, st.s, acc, acch);
      }
      if (!AA && packed) {  // counts only, in the packed word (the chunk-parallel scorer)
        atomicAdd(&s_aa[2 * st.s + 1], (unsigned long long)__popc(hm));
        return;
      }
      atomicAdd(&s_cn[st.s], (unsigned)__popc(hm));
    }
  };
  rc_loop<NT, K>(ci, s_start, s_off, s_coff, ns, tid, hint, shift, proc);
}

// Chunk prefix of a batch whose element offsets s_off[0..ns] are in LDS: s_coff[t] = sum of
// ceil(len / K) over rows < t; s_coff[ns] = total. Ends with a barrier.
template <int BLOCK, int K>
__device__ __attribute__((always_inline)) inline void rc_chunk_offsets(const int32_t* s_off, int ns, int32_t* s_coff, int* red) {
  const int nc = (int)threadIdx.x < ns ? (s_off[threadIdx.x + 1] - s_off[threadIdx.x] + K - 1) / K : 0;
  int tot;
  const int ex = block_exscan<BLOCK, false>(nc, red, &tot);  // (the barrier below ends red's use)
  if ((int)threadIdx.x < ns) s_coff[threadIdx.x] = ex;
  if (threadIdx.x == 0) s_coff[ns] = tot;
  __syncthreads();
}

// Element AND chunk offsets of a batch of ns segments (thread t < ns holds segment t's length) in
// ONE block scan: the pair (len, ceil(len / K)) packed in 64 bits -- the low half never carries
// into the high one, a batch holds < 2^31 ids -- instead of a scan for s_off followed by
// rc_chunk_offsets' scan for s_coff: three barriers fewer per batch. Ends with a barrier.
template <int BLOCK, int K>
__device__ __attribute__((always_inline)) inline void seg_offsets(int len, int ns, int32_t* s_off, int32_t* s_coff,
                                                                  unsigned long long* red64) {
  constexpr int NW = BLOCK / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long v = ((unsigned long long)(uint32_t)len << 32) | (uint32_t)((len + K - 1) / K);
  unsigned long long inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long t = __shfl_up(inc, d, 64);
    if (lane >= d) inc += t;
  }
  if (lane == 63) red64[wid] = inc;
  __syncthreads();
  unsigned long long base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const unsigned long long t = red64[w];
    base += w < wid ? t : 0ull;
    tot += t;
  }
  const unsigned long long ex = base + inc - v;
  if ((int)threadIdx.x < ns) {
    s_off[threadIdx.x] = (int32_t)(ex >> 32);
    s_coff[threadIdx.x] = (int32_t)(uint32_t)ex;
  }
  if (threadIdx.x == 0) {
    s_off[ns] = (int32_t)(tot >> 32);
    s_coff[ns] = (int32_t)(uint32_t)tot;
  }
  __syncthreads();  // also orders red64's reads before its next use
}

// Short rows (every row of the batch at most SHORT_MAX ids -- the business side, whose rows
// are user rows Γ(w)): one thread per segment reads its whole row with up to SHORT_MAX / 4
// 16-byte loads, all issued before any is used. No merge-path search and no row crossings,
// whose dependent LDS round trips dominate a merge-path step when rows average ~10 ids;
// the cost is idle lanes beside the longest row of the wave. ci is padded past nnz.
constexpr int SHORT_MAX = blp::SHORT_ROW_MAX;
constexpr int SHORT_PART = 16;  // ids held in registers at a time (a row up to SHORT_MAX: two parts)

// Part [h, h + SHORT_PART) of a row of len ids: up to SHORT_PART / 4 16-byte loads, all issued
// before any id is used. Rows of a review graph's users average ~10 ids, so the second part is
// rare; holding one part keeps the scorer inside 64 VGPRs (8 workgroups of 256 per CU).
__device__ inline void row_part(const int32_t* __restrict__ ci, int64_t st, int len, int h, int* e) {
  const blp::U4a* p = reinterpret_cast<const blp::U4a*>(ci + st + h);
#pragma unroll
  for (int q = 0; q < SHORT_PART / 4; ++q) {
    if (h + 4 * q < len) {
      const blp::U4a v = p[q];
      e[4 * q] = v.x;
      e[4 * q + 1] = v.y;
      e[4 * q + 2] = v.z;
      e[4 * q + 3] = v.w;
    }
  }
}

template <int NT>
__device__ __attribute__((always_inline)) inline void row_build(const int32_t* __restrict__ ci, uint32_t idmask, const int64_t* s_start,
                                 const int32_t* s_off, int ns, int64_t c0, int64_t width, uint32_t* bm, int tid) {
  const uint32_t keep = idmask | 0x80000000u, c0u = (uint32_t)c0, wu = (uint32_t)width;
  for (int t = tid; t < ns; t += NT) {
    const int64_t st = s_start[t];
    const int len = s_off[t + 1] - s_off[t];
    for (int h = 0; h < len; h += SHORT_PART) {
      int e[SHORT_PART];
      row_part(ci, st, len, h, e);
#pragma unroll
      for (int k = 0; k < SHORT_PART; ++k) {
        if (h + k < len) {
          const uint32_t r = in_chunk(e[k], keep, c0u);
          if (r < wu) atomicOr(&bm[r >> 5], 1u << (r & 31));
        }
      }
    }
  }
}

template <int NT, bool AA>
__device__ __attribute__((always_inline)) inline void row_scan(const int32_t* __restrict__ ci, uint32_t idmask, int idbits,
                                const long long* __restrict__ aaw, const long long* wtab, const int64_t* s_start,
                                const int32_t* s_off, int ns, int64_t c0, int64_t width, const uint32_t* bm,
                                uint32_t* s_cn, unsigned long long* s_aa, int tid) {
  const uint32_t keep = idmask | 0x80000000u, c0u = (uint32_t)c0, wu = (uint32_t)width;
  for (int t = tid; t < ns; t += NT) {  // the thread owns segment t: plain adds, no atomics
    const int64_t st = s_start[t];
    const int len = s_off[t + 1] - s_off[t];
    unsigned c = 0;
    unsigned long long acc = 0;
    uint32_t acch = 0;  // a row holds <= SHORT_MAX = 32 terms of W >> 32 < 2^27
    for (int h = 0; h < len; h += SHORT_PART) {
      int e[SHORT_PART];
      row_part(ci, st, len, h, e);
#pragma unroll
      for (int k = 0; k < SHORT_PART; ++k) {
        if (h + k < len) {
          const uint32_t r = in_chunk(e[k], keep, c0u);
          const uint32_t word = bm[(r < wu ? r : 0u) >> 5];
          const bool hit = r < wu && ((word >> (r & 31)) & 1u);
          c += hit ? 1u : 0u;
          if (AA && hit) {
            const uint32_t code = ((uint32_t)e[k] >> idbits) & 255u;
            const unsigned long long w = (unsigned long long)(code ? wtab[code] : aaw[e[k] & idmask]);
            acc += w;
            acch += (uint32_t)(w >> 32);
          }
        }
      }
    }
    s_cn[t] += c;
    if (AA) {
      s_aa[2 * t] += acc;
      s_aa[2 * t + 1] += acch;
    }
  }
}

// Load the rows of N(x)[k0, k0 + ns) as segments: start / exclusive offsets (s_off[ns] = total).
template <int BLOCK>
__device__ __attribute__((always_inline)) inline void load_row_segments(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci, int64_t k0,
                                         int ns, int64_t* s_start, int32_t* s_off, int* red,
                                         const int32_t* __restrict__ skip = nullptr) {
  int len = 0;
  if ((int)threadIdx.x < ns) {
    const int z = ci[k0 + threadIdx.x];
    const int64_t st = rp[z];
    s_start[threadIdx.x] = st;
    len = (skip && skip[z] >= 0) ? 0 : (int)(rp[z + 1] - st);  // dense rows were OR-ed in already
  }
  int tot;
  const int ex = block_exscan<BLOCK, false>(len, red, &tot);  // (the barrier below ends red's use)
  if ((int)threadIdx.x < ns) s_off[threadIdx.x] = ex;
  if (threadIdx.x == 0) s_off[ns] = tot;
  __syncthreads();
}

// load_row_segments for the row-chunk loops: element and chunk offsets together (seg_offsets: one
// scan and two barriers, instead of the offset scan and rc_chunk_offsets' second one). Ends with a
// barrier.
template <int BLOCK, int K>
__device__ __attribute__((always_inline)) inline void load_row_segments_rc(const int64_t* __restrict__ rp,
                                                                           const int32_t* __restrict__ ci, int64_t k0,
                                                                           int ns, int64_t* s_start, int32_t* s_off,
                                                                           int32_t* s_coff, unsigned long long* red64,
                                                                           const int32_t* __restrict__ skip) {
  int len = 0;
  if ((int)threadIdx.x < ns) {
    const int z = ci[k0 + threadIdx.x];
    const int64_t st = rp[z];
    s_start[threadIdx.x] = st;
    len = (skip && skip[z] >= 0) ? 0 : (int)(rp[z + 1] - st);  // dense rows were OR-ed in already
  }
  seg_offsets<BLOCK, K>(len, ns, s_off, s_coff, red64);
}

// ------------------------------------------------------------------ heavy-source pre-build
struct HeavyItem {
  int32_t slot;
  int32_t wedge;   // 0: [kb, ke) are CSR positions of N(x); 1: 16-byte vectors of x's wedge row
  int64_t kb, ke;  // rows N(x) = ci[kb, ke) handled by this item
};

struct HeavyArgs {
  const int64_t* rp;
  const int32_t* ci;
  const HeavyItem* items;
  uint32_t* heavy_bm;  // [slots][hb_words]
  int64_t hb_words;
  int64_t lo, width;
  const uint4* wedge;  // wedge rows (wedge.hip), for items with wedge = 1
};

template <int BLOCK, int CAP_WORDS, int SEG>
__global__ __launch_bounds__(BLOCK) void k_heavy(HeavyArgs h) {
  constexpr int K = 8;
  __shared__ uint32_t bm[CAP_WORDS];
  __shared__ int64_t s_start[SEG];
  __shared__ int32_t s_off[SEG + 1];
  __shared__ int red[BLOCK / 64];
  const HeavyItem it = h.items[blockIdx.x];
  const int nw = (int)((h.width + 31) >> 5);
  for (int i = threadIdx.x; i < nw; i += BLOCK) bm[i] = 0;
  __syncthreads();
  if (it.wedge) {  // a slice of x's wedge row: contiguous vectors, two per thread in flight
    const uint32_t c0u = (uint32_t)h.lo, wu = (uint32_t)h.width;
    for (int64_t q = it.kb + threadIdx.x; q < it.ke; q += 2 * BLOCK) {
      const uint4 v0 = h.wedge[q];
      const uint4 v1 = q + BLOCK < it.ke ? h.wedge[q + BLOCK] : v0;
      const uint32_t ids[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t r = in_chunk((int)ids[k], 0x7fffffffu | 0x80000000u, c0u);
        if (r < wu) atomicOr(&bm[r >> 5], 1u << (r & 31));
      }
    }
    __syncthreads();
  } else
  for (int64_t k0 = it.kb; k0 < it.ke; k0 += SEG) {
    const int ns = (int)min<int64_t>(SEG, it.ke - k0);
    load_row_segments<BLOCK>(h.rp, h.ci, k0, ns, s_start, s_off, red);
    mp_build<BLOCK, K>(h.ci, 0x7fffffffu, s_start, s_off, ns, h.lo, h.width, bm, threadIdx.x);
    __syncthreads();
  }
  uint32_t* dst = h.heavy_bm + (int64_t)it.slot * h.hb_words;
  for (int i = threadIdx.x; i < nw; i += BLOCK) {
    const uint32_t v = bm[i];
    if (v) atomicOr(&dst[i], v);
  }
}


__global__ void k_source_records(const int32_t* __restrict__ active, const Misc* __restrict__ misc,
                                 const int32_t* __restrict__ off, const int32_t* __restrict__ cnt,
                                 const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                 const int32_t* __restrict__ heavy_slot, const int64_t* __restrict__ wp,
                                 SrcRec* __restrict__ rec) {
  const int na = misc->n_active;
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < na; s += gridDim.x * blockDim.x) {
    const int x = active[s];
    SrcRec r;
    r.x = x;
    r.pbeg = off[x];
    r.pcnt = cnt[x];
    r.hslot = heavy_slot ? heavy_slot[x] : -1;
    r.xb = rp[x];
    r.xe = rp[x + 1];
    r.wb = wp ? wp[x] : 0;
    r.we = wp ? wp[x + 1] : 0;
    r.nx_lo = r.xe > r.xb ? ci[r.xb] : 0;
    r.nx_hi = r.xe > r.xb ? ci[r.xe - 1] : -1;
    r.pad[0] = r.pad[1] = 0;
    rec[s] = r;
  }
}

// ------------------------------------------------------------------ scorer
struct ScoreArgs {
  const int64_t* rp;
  const int32_t* ci;
  const long long* aaw;    // fixed-point Adamic-Adar weights
  const int32_t* cw;       // column ids streamed by build / scan: id | weight code << idbits
  uint32_t idmask;
  int idbits;
  const long long* wtab;   // [256] fixed-point weight per code (code 0: use aaw)
  const int32_t* off;      // per node: first grouped position of its pairs
  const int32_t* cnt;      // per node: number of pairs with that source
  const int32_t* active;   // active sources
  const int32_t* g_out;    // grouped position -> caller index (null: the identity, run-grouped lists)
  const int64_t* g_yb;     // grouped position -> start of N(y) in ci
  const int32_t* g_yl;     // grouped position -> |N(y)|
  const int32_t* py;       // or (run-grouped large-scorer batches) the caller-order y: N(y) from rp
  const int32_t* hot_idx;     // per node: dense-row number or -1 (null: no dense rows)
  const blp::HotRow* hot_tab;
  const uint4* hot_pool;
  const int32_t* heavy_slot;  // per node: pre-built bitmap slot or -1 (null: none)
  const uint32_t* heavy_bm;
  int64_t hb_words;
  Misc* misc;
  uint32_t* cn;
  double* jac;
  double* aa;
  int64_t lo, hi;    // bitmap universe
  int64_t cap_bits;  // bitmap bits per chunk (<= template capacity; lowered only by tests)
  uint32_t mask;
  int dq;            // sources per dequeue
  int short_rows;    // bit 0: every build row <= SHORT_MAX ids, bit 1: every scan row (row_build / row_scan)
  const int64_t* wp;    // wedge rows (wedge.hip; short-row scorer only, null: build from CSR)
  const uint4* wedge;
  unsigned long long* aa_part;  // [2 n_pairs] exact AA words carried between LDS chunks (k_score, chunks > 1)
  const SrcRec* rec;            // per active source (short-row scorer; null: gather from active[])
  int4* lq;                     // k_score_split: long-slice queues, SPLIT_LQ entries per workgroup
  int64_t np, n_nodes;          // pairs and nodes (BLP_DEBUG bounds)
  int64_t rs_rows;              // rows of the split table (BLP_DEBUG bound)
  int64_t nnz, wedge_vecs;      // CSR entries, wedge-row vectors (BLP_DEBUG bounds)
  int64_t n_hot, hot_vecs;      // dense rows, their pool's vectors (BLP_DEBUG bounds)
  int lq_wgs;                   // workgroups d_lq was sized for (BLP_DEBUG bound)
};

// the caller index of grouped pair gp: g_out, or gp itself when the batch's grouped order is its
// caller order (a list grouped by source: run-head grouping writes no g_out)
__device__ __attribute__((always_inline)) inline int gout(const ScoreArgs& a, int64_t gp) {
  return a.g_out ? a.g_out[gp] : (int)gp;
}

// N(y)'s row [st, st + len) of grouped pair gp, from the grouped metadata g_yb / g_yl.
__device__ __attribute__((always_inline)) inline void pair_row(const ScoreArgs& a, int gp, int64_t& st, int& len) {
  if (a.py) {  // one dependent load more (y, then rp[y]), behind the H2 build like the rest of the header
    const int yv = a.py[gp];
    st = a.rp[yv];
    len = (int)(a.rp[yv + 1] - st);
  } else {
    st = a.g_yb[gp];
    len = a.g_yl[gp];
  }
}

template <int BLOCK, bool TAIL = true>  // TAIL: see block_exscan
__device__ inline unsigned long long block_sum_u64(unsigned long long v, unsigned long long* red) {
  constexpr int NW = BLOCK / 64;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  unsigned long long t = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) t += red[w];
  if (TAIL) __syncthreads();
  return t;
}

#ifdef BLP_PROF
__device__ unsigned long long g_prof[16];
#define PROF_INIT                          \
  unsigned long long prof_t0 = clock64();  \
  unsigned long long prof_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#define PROF(i)                                \
  {                                            \
    const unsigned long long t1_ = clock64();  \
    prof_acc[i] += t1_ - prof_t0;              \
    prof_t0 = t1_;                             \
  }
#define PROF_FLUSH                                                         \
  if (threadIdx.x == 0)                                                    \
    for (int i_ = 0; i_ < 9; ++i_) atomicAdd(&g_prof[i_], prof_acc[i_]);
#else
#define PROF_INIT
#define PROF(i)
#define PROF_FLUSH
#endif

// SHORT: every build and scan row of the batch has at most SHORT_MAX ids (the business side of
// a review graph: user rows), so only the row-per-thread loops are compiled in -- fewer
// registers and no hint table, hence more resident workgroups for these latency-bound sources.
// The SHORT bitmap is dynamic LDS sized to the batch's universe (12.5 KiB for 100K
// businesses), and SAA = false (no Adamic-Adar: the reference's business pass) drops the
// fixed-point sums and the weight table: ~16.5 KiB per workgroup in all, so registers, not
// LDS, bound the residency (BLP_SHORT_MINB workgroups per CU).
extern __shared__ uint4 blp_dyn_lds[];

// PKO: the large scorer for universes of <= 32 * CAP_WORDS < 2^21 nodes in one chunk whose scan
// rows are not all short -- counts always in the packed word, so no per-pair count array, and the
// LDS that frees holds longer scan segments (SEG_PKO pairs: one segment for a typical config-2
// source of ~750 pairs instead of two; each segment costs its offset scans, hint table, barriers
// and a refill of the two-step load pipeline).
template <int BLOCK, int CAP_WORDS, int SEG, int K, bool SHORT = false, bool SAA = true, bool PKO = false>
__global__ __launch_bounds__(BLOCK, SHORT ? BLP_SHORT_MINB : 1) void k_score(ScoreArgs a) {
  static_assert(SEG <= BLOCK, "one pair segment per thread in the output loop");
  constexpr int NW = BLOCK / 64;
  // row-chunk loops (rc_*) for the large-universe variant; the others keep the merge-path loops
  constexpr bool RC = BLP_RC && CAP_WORDS > 16384;  // the large variant
  __shared__ uint32_t bm_st[SHORT ? 4 : CAP_WORDS + (RC ? RC_EXTRA_WORDS : 0)];
  uint32_t* bm = SHORT ? reinterpret_cast<uint32_t*>(blp_dyn_lds) : bm_st;
  __shared__ int32_t s_coff[RC ? SEG + 1 : 1];
  __shared__ int64_t s_start[SEG];
  __shared__ int32_t s_off[SEG + 1];
  __shared__ uint32_t s_cn[PKO ? 1 : SEG];
  __shared__ unsigned long long s_aa[SAA ? 2 * SEG : 1];  // exact AA words, interleaved (aa_push)
  __shared__ unsigned long long red64[NW];
  __shared__ unsigned long long red64s[RC && BLP_SEGOFF ? NW : 1];  // seg_offsets' own (the popcount's red64 is read late)
  __shared__ int red[NW];
  __shared__ int s_src[2];  // the claimed source, alternating slots (no barrier guards its rewrite)
  __shared__ int s_nhot;
  __shared__ blp::HotRow s_hot[SHORT ? 1 : HOT_LIST];
  __shared__ long long s_wtab[SAA ? 256 : 1];
  // hint table where the LDS allows it (the 64 KiB-bitmap variant keeps 2 workgroups per CU)
  constexpr int HC = PKO ? 1024 : SHORT ? 1 : CAP_WORDS > 16384 ? (RC ? 1536 : 2048) : CAP_WORDS >= 16384 ? 1 : 512;
  __shared__ int32_t s_hint[HC];

  if (SAA && a.wtab)  // visible after the first barrier
    for (int i = threadIdx.x; i < 256; i += BLOCK) s_wtab[i] = a.wtab[i];
  if (RC)  // the zero word and the build's dummy words past the bitmap
    for (int i = threadIdx.x; i < RC_EXTRA_WORDS; i += BLOCK) bm[CAP_WORDS + i] = 0;
  const int64_t CAP_BITS = a.cap_bits;
  const int64_t span = a.hi - a.lo;
  const int nchunks = span <= CAP_BITS ? 1 : (int)((span + CAP_BITS - 1) / CAP_BITS);
  const bool want_j = (a.mask & BLP_JACCARD) != 0;
  const bool want_a = SAA && (a.mask & BLP_ADAMIC) != 0;
  // packed count + high word (rc_scan): row-chunk scans of a one-chunk universe (< 2^21 nodes)
  const bool packed = PKO || (RC && want_a && nchunks == 1 && !(a.short_rows & 2) && CAP_BITS < (1 << PK_CN_BITS));
  static_assert(!PKO || (RC && 32ll * CAP_WORDS < (1ll << PK_CN_BITS)), "PKO: one packed chunk");
  uint4* bm4 = reinterpret_cast<uint4*>(bm);
  const int n_active = a.misc->n_active;

  PROF_INIT
  // dequeue one ahead: the next source's atomic is in flight while this one is scored
  int nxt = threadIdx.x == 0 ? atomicAdd(&a.misc->queue, a.dq) : 0;
  if (!SHORT && threadIdx.x == 0) s_nhot = 0;  // (reset again after each use, before a barrier)
  for (int it = 0;; ++it) {
    int s_first;
    // slot it & 1 is rewritten two claims later, after this claim's barriers: one barrier here
    if (threadIdx.x == 0) {
      s_src[it & 1] = nxt;
      if (nxt < n_active) nxt = atomicAdd(&a.misc->queue, a.dq);
    }
    __syncthreads();
    s_first = s_src[it & 1];
    if (s_first >= n_active) break;
    PROF(0)
    const int s_last = min(n_active, s_first + a.dq);
    for (int s = s_first; s < s_last; ++s) {
      int x, pbeg, pcnt, hslot;
      int64_t xb, xe, wb = 0, we = 0, nx_lo, nx_hi;
      if (SHORT || (RC && a.rec)) {  // one record per source (s is uniform): one round trip, not two
        // uniform: kept in scalar registers (the VGPR budget of 7 workgroups per CU is tight)
        const SrcRec& r = a.rec[__builtin_amdgcn_readfirstlane(s)];
        auto u32 = [](int32_t v) { return (int32_t)__builtin_amdgcn_readfirstlane(v); };
        auto u64 = [](int64_t v) {
          return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(v >> 32)) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)v));
        };
        x = u32(r.x);
        pbeg = u32(r.pbeg);
        pcnt = u32(r.pcnt);
        hslot = u32(r.hslot);
        xb = u64(r.xb);
        xe = u64(r.xe);
        wb = u64(r.wb);
        we = u64(r.we);
        nx_lo = u32(r.nx_lo);
        nx_hi = u32(r.nx_hi);
      } else {
        x = a.active[s];
        if (!PS_OK(a.misc, x >= 0 && x < a.n_nodes, 2, x, a.n_nodes)) continue;  // uniform
        pbeg = a.off[x];
        pcnt = a.cnt[x];
        if (!PS_OK(a.misc, pbeg >= 0 && (int64_t)pbeg + pcnt <= a.np, 3, (int64_t)pbeg + pcnt, a.np)) continue;
        xb = a.rp[x];
        xe = a.rp[x + 1];
        hslot = a.heavy_slot ? a.heavy_slot[x] : -1;
        // value range of N(x) (rows are sorted): distance-1 removal is skipped when disjoint
        nx_lo = xe > xb ? a.ci[xb] : 0;
        nx_hi = xe > xb ? a.ci[xe - 1] : -1;
      }
      unsigned long long h2 = 0;
      // short-row scorer (BLP_PF): the first pair segment's metadata is loaded now, so its
      // latency overlaps the H2 build instead of following it
      int64_t pf_start = 0;
      int pf_len = 0, pf_out = 0, pf_y = 0;
      constexpr bool PF = SHORT ? BLP_PF : (RC && BLP_PFL);
      const bool pf_mine = PF && nchunks == 1 && (int)threadIdx.x < min(SEG, pcnt);
      if (pf_mine) {
        const int gp = pbeg + threadIdx.x;
        if (a.py)  // two hops (y, then rp[y]): the second is issued once the bitmap's first phase is out
          pf_y = a.py[gp];
        else
          pair_row(a, gp, pf_start, pf_len);
        pf_out = gout(a, gp);
      }
      auto pf_rows = [&]() {
        if (a.py && pf_mine) {
          pf_start = a.rp[pf_y];
          pf_len = (int)(a.rp[pf_y + 1] - pf_start);
        }
      };
      PROF(1)

      for (int ch = 0; ch < nchunks; ++ch) {
        const int64_t c0 = a.lo + (int64_t)ch * CAP_BITS;
        const int64_t c1 = min(a.hi, c0 + CAP_BITS);
        const int64_t width = max<int64_t>(c1 - c0, 0);
        const int nw4 = (int)((((width + 31) >> 5) + 3) >> 2);
        const bool last = ch == nchunks - 1;
        if (hslot >= 0) {
          // 1'. pre-built by k_heavy (single-chunk universes only)
          const uint4* src4 = reinterpret_cast<const uint4*>(a.heavy_bm + (int64_t)hslot * a.hb_words);
          for (int i = threadIdx.x; i < nw4; i += BLOCK) bm4[i] = src4[i];
          if (ch == 0) pf_rows();
          __syncthreads();
        } else {
          // 1. the dense rows of N(x) initialise the bitmap (their OR, 16-byte vectors), then
          // 2. the sparse rows mark N(N(x)) ∩ [c0, c1) through merge-path row segments
          if constexpr (!SHORT) {  // short rows are never dense: the bitmap is only zeroed
            // (s_nhot is 0 here: set before the loop and after each use below)
            if (a.hot_idx) {
              for (int64_t k = xb + threadIdx.x; k < xe; k += BLOCK) {
                const int hi = a.hot_idx[a.ci[k]];
                if (hi >= 0 && PS_OK(a.misc, hi < a.n_hot, 12, hi, a.n_hot)) {
                  const int slot = atomicAdd(&s_nhot, 1);
                  if (slot < HOT_LIST) s_hot[slot] = a.hot_tab[hi];
                }
              }
            }
            __syncthreads();
          }
          const int nhot = !SHORT && s_nhot <= HOT_LIST ? s_nhot : 0;  // overflow: every row goes sparse
          const int64_t q0 = c0 >> 7;
          if (RC) {
            // every thread owns QPT vectors of the bitmap and ORs each dense row into registers:
            // a row's QPT loads are all in flight at once (one L2 round trip per row, not per
            // vector). Large variant only: the extra registers would cost the small variants a
            // wave per SIMD.
            constexpr int QPT = (CAP_WORDS / 4 + BLOCK - 1) / BLOCK;
            uint4 acc[QPT];
#pragma unroll
            for (int j = 0; j < QPT; ++j) acc[j] = make_uint4(0, 0, 0, 0);
            for (int r = 0; r < (BLP_EXP_PHASE == 2 ? 0 : nhot); ++r) {
              const blp::HotRow h = s_hot[r];
              const uint4* row = a.hot_pool + h.vec_off;
#pragma unroll
              for (int j = 0; j < QPT; ++j) {
                const int q = threadIdx.x + j * BLOCK;
                const int64_t qq = q0 + q - h.vlo;
                if (q < nw4 && qq >= 0 && qq < h.nvec) {
                  const uint4 p = row[qq];
                  acc[j].x |= p.x;
                  acc[j].y |= p.y;
                  acc[j].z |= p.z;
                  acc[j].w |= p.w;
                }
              }
            }
#pragma unroll
            for (int j = 0; j < QPT; ++j) {
              const int q = threadIdx.x + j * BLOCK;
              if (q < nw4) bm4[q] = acc[j];
            }
          } else {
            for (int q = threadIdx.x; q < nw4; q += BLOCK) {
              uint4 v = make_uint4(0, 0, 0, 0);
              for (int r = 0; r < nhot; ++r) {
                const int64_t qq = q0 + q - s_hot[r].vlo;
                if (qq >= 0 && qq < s_hot[r].nvec) {
                  const uint4 p = a.hot_pool[s_hot[r].vec_off + qq];
                  v.x |= p.x;
                  v.y |= p.y;
                  v.z |= p.z;
                  v.w |= p.w;
                }
              }
              bm4[q] = v;
            }
          }
          __syncthreads();
          if (!SHORT && threadIdx.x == 0) s_nhot = 0;  // s_hot / s_nhot are read: ready for the next detection
          if (ch == 0) pf_rows();  // in flight during the sparse build
          PROF(2)
          if (SHORT && a.wp) {
            // N(N(x)) from x's wedge row: one contiguous range, two 16-byte vectors per thread
            // in flight, no row_ptr round trip and no idle lanes beside long rows
            const uint32_t keep = a.idmask | 0x80000000u, c0u = (uint32_t)c0, wu = (uint32_t)width;
            for (int64_t q = wb + threadIdx.x; q < we; q += 2 * BLOCK) {
              const uint4 v0 = a.wedge[q];
              const uint4 v1 = q + BLOCK < we ? a.wedge[q + BLOCK] : v0;  // (a repeat ORs nothing new)
              const uint32_t ids[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
              for (int k = 0; k < 8; ++k) {
                const uint32_t r = in_chunk((int)ids[k], keep, c0u);
                if (r < wu) atomicOr(&bm[r >> 5], 1u << (r & 31));
              }
            }
            __syncthreads();
          } else
          for (int64_t k0 = xb; k0 < xe; k0 += SEG) {
            const int ns = (int)min<int64_t>(SEG, xe - k0);
            // the row-chunk build: its offsets in one scan (BLP_SEGOFF)
            const bool seg1 = RC && BLP_SEGOFF && !(a.short_rows & 1);
            if (seg1)
              load_row_segments_rc<BLOCK, K>(a.rp, a.ci, k0, ns, s_start, s_off, s_coff, red64s, nhot ? a.hot_idx : nullptr);
            else
              load_row_segments<BLOCK>(a.rp, a.ci, k0, ns, s_start, s_off, red, nhot ? a.hot_idx : nullptr);
            if (SHORT || (a.short_rows & 1)) {
              row_build<BLOCK>(a.cw, a.idmask, s_start, s_off, ns, c0, width, bm, threadIdx.x);
            } else if constexpr (!SHORT) {
              if (RC) {
                if (!seg1) rc_chunk_offsets<BLOCK, K>(s_off, ns, s_coff, red);
                const int shift = build_hint<BLOCK, HC>(s_coff, ns, BLOCK, s_hint);
                if (BLP_EXP_PHASE != 2)
                  rc_build<BLOCK, K>(a.cw, a.idmask, s_start, s_off, s_coff, ns, c0, width, bm, CAP_WORDS, threadIdx.x,
                                     s_hint, shift);
              } else {
                const int shift = build_hint<BLOCK, HC>(s_off, ns, BLOCK * K, s_hint);
#if BLP_PP
                pp_build<BLOCK, K>(a.cw, a.idmask, s_start, s_off, ns, c0, width, bm, threadIdx.x, s_hint, shift);
#else
                mp_build<BLOCK, K>(a.cw, a.idmask, s_start, s_off, ns, c0, width, bm, threadIdx.x, s_hint, shift);
#endif
              }
            }
            __syncthreads();
          }
        }
        PROF(3)
        // 3. exact distance 2: drop x (distance 0) and N(x) (distance 1)
        if (nx_hi >= c0 && nx_lo < c1) {
          for (int64_t k = xb + threadIdx.x; k < xe; k += BLOCK) {
            const int64_t r = (int64_t)a.ci[k] - c0;
            if (r >= 0 && r < width) atomicAnd(&bm[r >> 5], ~(1u << (r & 31)));
          }
        }
        if (threadIdx.x == 0 && x >= c0 && x < c1) atomicAnd(&bm[(x - c0) >> 5], ~(1u << ((x - c0) & 31)));
        __syncthreads();
        PROF(4)
        // 4. |H2(x) ∩ chunk|
        if (want_j) {
          unsigned long long pc = 0;
          for (int i = threadIdx.x; i < nw4; i += BLOCK) {
            const uint4 q = bm4[i];
            pc += __popc(q.x) + __popc(q.y) + __popc(q.z) + __popc(q.w);
          }
          h2 += block_sum_u64<BLOCK, false>(pc, red64);  // red64's next use is past the scan's barriers
        }
        PROF(5)
        // 5. scan N(y) of every pair of x, SEG pairs at a time
        bool have_pf = PF && nchunks == 1;  // segment sb's metadata is in pf_* (loaded earlier)
        for (int sb = 0; sb < pcnt; sb += SEG) {
          const int ns = min(SEG, pcnt - sb);
          int len = 0, pout = 0;
          // the next segment's metadata (BLP_PFN), issued during this segment's offsets and scan;
          // with a.py its first hop (y) goes out now, before the offsets' barriers
          const bool nxt = PF && !SHORT && BLP_PFN && nchunks == 1 && sb + SEG < pcnt;
          const bool nxt_mine = nxt && (int)threadIdx.x < min(SEG, pcnt - sb - SEG);
          if (a.py && nxt_mine) pf_y = a.py[pbeg + sb + SEG + threadIdx.x];
          if (have_pf) {
            if ((int)threadIdx.x < ns) {
              s_start[threadIdx.x] = pf_start;
              len = pf_len;
              pout = pf_out;
              if (!PKO) s_cn[threadIdx.x] = 0;
              if (SAA) {
                s_aa[2 * threadIdx.x] = 0;
                s_aa[2 * threadIdx.x + 1] = 0;
              }
            }
          } else if ((int)threadIdx.x < ns) {
            const int gp = pbeg + sb + threadIdx.x;
            int64_t st;
            pair_row(a, gp, st, len);
            s_start[threadIdx.x] = st;
            pout = gout(a, gp);  // used after the scan: its latency hides behind it
            if (!PKO) s_cn[threadIdx.x] = 0;
            if (SAA) {
              s_aa[2 * threadIdx.x] = 0;
              s_aa[2 * threadIdx.x + 1] = 0;
            }
          }
          // the row-chunk scan's element and chunk offsets in one scan (BLP_SEGOFF), else the offsets
          const bool seg2 = RC && BLP_SEGOFF && !SHORT && !(a.short_rows & 2);
          if (seg2) {
            seg_offsets<BLOCK, K>(len, ns, s_off, s_coff, red64s);
          } else {
            int tot;
            const int ex = block_exscan<BLOCK, false>(len, red, &tot);  // (the barrier below ends red's use)
            if ((int)threadIdx.x < ns) s_off[threadIdx.x] = ex;
            if (threadIdx.x == 0) s_off[ns] = tot;
            __syncthreads();
          }
          // the next segment's row bounds, in flight during this segment's scan
          have_pf = nxt;
          if (nxt_mine) {
            const int gp = pbeg + sb + SEG + threadIdx.x;
            if (a.py) {
              pf_start = a.rp[pf_y];
              pf_len = (int)(a.rp[pf_y + 1] - pf_start);
            } else {
              pair_row(a, gp, pf_start, pf_len);
            }
            pf_out = gout(a, gp);
          }
          PROF(6)
          if (SHORT || (a.short_rows & 2)) {
            if (SAA && want_a)
              row_scan<BLOCK, SAA>(a.cw, a.idmask, a.idbits, a.aaw, s_wtab, s_start, s_off, ns, c0, width, bm, s_cn,
                                    s_aa, threadIdx.x);
            else
              row_scan<BLOCK, false>(a.cw, a.idmask, a.idbits, a.aaw, s_wtab, s_start, s_off, ns, c0, width, bm, s_cn,
                                     s_aa, threadIdx.x);
          } else if constexpr (SHORT) {
          } else if (RC) {
            if (!seg2) rc_chunk_offsets<BLOCK, K>(s_off, ns, s_coff, red);
            const int shift = build_hint<BLOCK, HC>(s_coff, ns, BLOCK, s_hint);
            if (BLP_EXP_PHASE == 1) {
            } else if (want_a)
              rc_scan<BLOCK, K, true>(a.cw, a.idmask, a.idbits, a.aaw, s_wtab, s_start, s_off, s_coff, ns, c0, width,
                                      bm, CAP_WORDS, s_cn, s_aa, threadIdx.x, s_hint, shift, packed);
            else
              rc_scan<BLOCK, K, false>(a.cw, a.idmask, a.idbits, a.aaw, s_wtab, s_start, s_off, s_coff, ns, c0, width,
                                       bm, CAP_WORDS, s_cn, s_aa, threadIdx.x, s_hint, shift, packed);
          } else {
            const int shift = build_hint<BLOCK, HC>(s_off, ns, BLOCK * K, s_hint);
#if BLP_PP
            if (want_a)
              pp_scan<BLOCK, K, true>(a.cw, a.idmask, a.idbits, a.aaw, s_wtab, s_start, s_off, ns, c0, width, bm, s_cn,
                                      s_aa, threadIdx.x, s_hint, shift);
            else
              pp_scan<BLOCK, K, false>(a.cw, a.idmask, a.idbits, a.aaw, s_wtab, s_start, s_off, ns, c0, width, bm,
                                       s_cn, s_aa, threadIdx.x, s_hint, shift);
#else
            if (want_a)
              mp_scan<BLOCK, K, true>(a.cw, a.idmask, a.idbits, a.aaw, s_wtab, s_start, s_off, ns, c0, width, bm, s_cn,
                                      s_aa, threadIdx.x, s_hint, shift);
            else
              mp_scan<BLOCK, K, false>(a.cw, a.idmask, a.idbits, a.aaw, s_wtab, s_start, s_off, ns, c0, width, bm,
                                       s_cn, s_aa, threadIdx.x, s_hint, shift);
#endif
          }
          __syncthreads();
          PROF(7)
          for (int t = threadIdx.x; t < ns; t += BLOCK) {  // ns <= SEG <= BLOCK: t == threadIdx.x
            const int p = pout;
            if (!PS_OK(a.misc, p >= 0 && p < a.np, 4, p, a.np)) continue;
            unsigned c = packed ? (unsigned)(s_aa[2 * t + 1] & ((1u << PK_CN_BITS) - 1)) : s_cn[PKO ? 0 : t];
            if (ch > 0) c += a.cn[p];
            a.cn[p] = c;
            if (SAA && want_a && packed) {
              a.aa[p] = blp::aa_value(s_aa[2 * t], s_aa[2 * t + 1] >> PK_CN_BITS, PK_HS);
            } else if (SAA && want_a) {
              unsigned long long lo = s_aa[2 * t], hi = s_aa[2 * t + 1];
              if (ch > 0) {  // the exact words of the earlier chunks
                lo += a.aa_part[2 * (int64_t)p];
                hi += a.aa_part[2 * (int64_t)p + 1];
              }
              if (last) {
                a.aa[p] = blp::aa_value(lo, hi);
              } else {
                a.aa_part[2 * (int64_t)p] = lo;
                a.aa_part[2 * (int64_t)p + 1] = hi;
              }
            }
            if (want_j && last) {
              const long long uni = (long long)h2 + (s_off[t + 1] - s_off[t]) - (long long)c;
              if (uni <= 0) {
                a.jac[p] = __builtin_nan("");
                atomicOr(&a.misc->zero_div, 1);
              } else {
                a.jac[p] = (double)c / (double)uni;  // correctly rounded, as Python's float division
              }
            }
          }
          __syncthreads();
          PROF(8)
        }
      }
    }
  }
  PROF_FLUSH
}

// ------------------------------------------------------------------ short-row scorer, 3 barriers
// The short-row scorer (the business side of a review graph: 100K light sources, ~75 pairs each,
// rows of <= SHORT_MAX ids) restated around its dependent chain (round 5). k_score<..., SHORT>
// passes every pair's row bounds through LDS segments (an offset scan, a segment table, a
// per-segment count array) and popcounts the bitmap: ~9 block barriers per source, each one a
// point where the 4 waves of a workgroup wait for the slowest's round trip. Here:
//   P1  copy the source's pre-built set (wedge-row bitmap / k_heavy slot), counting its bits on
//       the way, or zero the bitmap                                              -- barrier
//   P2  OR in the wedge row, counting the bits an atomicOr newly sets (its return value), so
//       |N(N(x)) ∩ universe| is known without a popcount pass                     -- barrier
//   (general graphs only, N(x) inside the universe: drop distance 1, counting the cleared bits -- barrier)
//   P3  every thread scores its own pairs t, t + 256, ... straight from registers (the first one's
//       metadata was loaded before P1): N(y) tested against the bitmap, x itself skipped (distance
//       0; |H2| = count - x's bit), outputs written                               -- barrier
// Three barriers per source instead of ~9, the same bitmap and the same exact arithmetic.
template <bool SAA>
__global__ __launch_bounds__(256, BLP_SHORT_MINB) void k_score_short(ScoreArgs a) {
  constexpr int BLOCK = 256;
  constexpr int NW = BLOCK / 64;
  uint32_t* bm = reinterpret_cast<uint32_t*>(blp_dyn_lds);
  uint4* bm4 = reinterpret_cast<uint4*>(bm);
  __shared__ long long s_wtab[SAA ? 256 : 1];
  __shared__ int s_src[2];
  __shared__ unsigned s_h2[2];
  (void)NW;
  if (SAA && a.wtab)
    for (int i = threadIdx.x; i < 256; i += BLOCK) s_wtab[i] = a.wtab[i];
  if (threadIdx.x == 0) s_h2[0] = s_h2[1] = 0;
  const int64_t c0 = a.lo, width = max<int64_t>(a.hi - a.lo, 0);
  const int nw4 = (int)((((width + 31) >> 5) + 3) >> 2);
  const uint32_t c0u = (uint32_t)c0, wu = (uint32_t)width, keep = a.idmask | 0x80000000u;
  const bool want_j = (a.mask & BLP_JACCARD) != 0;
  const bool want_a = SAA && (a.mask & BLP_ADAMIC) != 0;
  const int n_active = a.misc->n_active;
  const int lane = threadIdx.x & 63;
  // wave-sum an unsigned count into an LDS counter: one atomic per wave
  auto add_count = [&](unsigned c, unsigned* dst) {
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0 && c) atomicAdd(dst, c);
  };
  // -DBLP_PROF phase clocks: 0 dequeue, 1 header + first pair's metadata issued, 2 P1, 3 P2,
  // 4 distance 1, 5 P3 (scan + outputs + closing barrier)
  PROF_INIT
  // (Staging the next source's record in LDS during this one's P3, with claims dequeued two ahead,
  // cut the scorer 1.60 -> 1.42 ms in-step but slowed the co-scheduled user pass: step 2.135 -> 2.26
  // ms at every CU share tried, r06_ab1-3.)
  int nxt = threadIdx.x == 0 ? atomicAdd(&a.misc->queue, a.dq) : 0;  // dequeue one ahead
  int k = 0;  // sources scored by this workgroup: s_h2 slot k & 1
  for (int it = 0;; ++it) {
    if (threadIdx.x == 0) {
      s_src[it & 1] = nxt;
      if (nxt < n_active) nxt = atomicAdd(&a.misc->queue, a.dq);
    }
    __syncthreads();
    const int s_first = s_src[it & 1];
    PROF(0)
    if (s_first >= n_active) break;
    const int s_last = min(n_active, s_first + a.dq);
    for (int s = s_first; s < s_last; ++s, ++k) {
      const SrcRec& r = a.rec[__builtin_amdgcn_readfirstlane(s)];
      auto u32 = [](int32_t v) { return (int32_t)__builtin_amdgcn_readfirstlane(v); };
      auto u64 = [](int64_t v) {
        return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(v >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)v));
      };
      const int x = u32(r.x), pbeg = u32(r.pbeg), pcnt = u32(r.pcnt), hslot = u32(r.hslot);
      const int64_t xb = u64(r.xb), xe = u64(r.xe), wb = u64(r.wb), we = u64(r.we);
      const int64_t nx_lo = u32(r.nx_lo), nx_hi = u32(r.nx_hi);
      const int slot = k & 1;
      // the first pair's metadata, in flight during P1 / P2
      int64_t pf_start = 0;
      int pf_len = 0, pf_out = 0;
      const bool pairs_ok = PS_OK(a.misc, pbeg >= 0 && (int64_t)pbeg + pcnt <= a.np, 3, (int64_t)pbeg + pcnt, a.np);
      if (pairs_ok && (int)threadIdx.x < pcnt) {
        pair_row(a, pbeg + threadIdx.x, pf_start, pf_len);
        pf_out = gout(a, pbeg + threadIdx.x);
      }
      PROF(1)
      // P1: the pre-built set, counted while copied, or a zeroed bitmap
      unsigned cnt = 0;
      if (hslot >= 0) {
        const uint4* src4 = reinterpret_cast<const uint4*>(a.heavy_bm + (int64_t)hslot * a.hb_words);
        for (int i = threadIdx.x; i < nw4; i += BLOCK) {
          const uint4 q = src4[i];
          bm4[i] = q;
          cnt += __popc(q.x) + __popc(q.y) + __popc(q.z) + __popc(q.w);
        }
      } else {
        for (int i = threadIdx.x; i < nw4; i += BLOCK) bm4[i] = make_uint4(0, 0, 0, 0);
      }
      if (threadIdx.x == 0) s_h2[slot ^ 1] = 0;  // the next source's counter (its last reader is past a barrier)
      add_count(cnt, &s_h2[slot]);
      __syncthreads();
      PROF(2)
      // P2: N(N(x)) from x's wedge row, counting newly set bits
      if (hslot < 0) {
        cnt = 0;
        if (PS_OK(a.misc, wb >= 0 && we <= a.wedge_vecs, 11, we, a.wedge_vecs)) {
          for (int64_t q = wb + threadIdx.x; q < we; q += 2 * BLOCK) {
            const uint4 v0 = a.wedge[q];
            const uint4 v1 = q + BLOCK < we ? a.wedge[q + BLOCK] : v0;  // (a repeat sets nothing new)
            const uint32_t ids[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const uint32_t rr = in_chunk((int)ids[j], keep, c0u);
              if (rr < wu) {
                const uint32_t bit = 1u << (rr & 31);
                cnt += (atomicOr(&bm[rr >> 5], bit) & bit) ? 0u : 1u;
              }
            }
          }
        }
        add_count(cnt, &s_h2[slot]);
        __syncthreads();
      }
      PROF(3)
      // distance 1 (general graphs: N(x) meets the universe): drop it, counting the cleared bits
      if (nx_hi >= c0 && nx_lo < c0 + width) {
        cnt = 0;
        for (int64_t q = xb + threadIdx.x; q < xe; q += BLOCK) {
          const int64_t rr = (int64_t)a.ci[q] - c0;
          if (rr >= 0 && rr < width) {
            const uint32_t bit = 1u << (rr & 31);
            cnt += (atomicAnd(&bm[rr >> 5], ~bit) & bit) ? 1u : 0u;
          }
        }
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
        if (lane == 0 && cnt) atomicSub(&s_h2[slot], cnt);
        __syncthreads();
      }
      PROF(4)
      // P3: |H2(x)| = the count minus x itself (distance 0); each thread scores its own pairs
      const int64_t xr = (int64_t)x - c0;
      const unsigned xbit = (xr >= 0 && xr < width) ? (bm[xr >> 5] >> (xr & 31)) & 1u : 0u;
      const long long h2 = (long long)s_h2[slot] - xbit;
      for (int p = threadIdx.x; pairs_ok && p < pcnt; p += BLOCK) {
        int64_t st = pf_start;
        int len = pf_len, pout = pf_out;
        if (p != (int)threadIdx.x) {
          pair_row(a, pbeg + p, st, len);
          pout = gout(a, pbeg + p);
        }
        if (!PS_OK(a.misc, pout >= 0 && pout < a.np, 4, pout, a.np)) continue;
        if (!PS_OK(a.misc, st >= 0 && st + len <= a.nnz + blp::CI_PAD, 10, st + len, a.nnz)) continue;
        unsigned c = 0;
        unsigned long long acc = 0;
        uint32_t acch = 0;  // <= SHORT_MAX terms of W >> 32 < 2^27
        for (int h = 0; h < len; h += SHORT_PART) {
          int e[SHORT_PART];
          row_part(a.cw, st, len, h, e);
#pragma unroll
          for (int j = 0; j < SHORT_PART; ++j) {
            if (h + j < len) {
              const uint32_t rr = in_chunk(e[j], keep, c0u);
              const uint32_t word = bm[(rr < wu ? rr : 0u) >> 5];
              const bool hit = rr < wu && ((word >> (rr & 31)) & 1u) && (int)((uint32_t)e[j] & a.idmask) != x;
              c += hit ? 1u : 0u;
              if (SAA && want_a && hit) {
                const uint32_t code = ((uint32_t)e[j] >> a.idbits) & 255u;
                const unsigned long long w = (unsigned long long)(code ? s_wtab[code] : a.aaw[e[j] & a.idmask]);
                acc += w;
                acch += (uint32_t)(w >> 32);
              }
            }
          }
        }
        a.cn[pout] = c;
        if (SAA && want_a) a.aa[pout] = blp::aa_value(acc, acch);
        if (want_j) {
          const long long uni = h2 + len - (long long)c;
          if (uni <= 0) {
            a.jac[pout] = __builtin_nan("");
            atomicOr(&a.misc->zero_div, 1);
          } else {
            a.jac[pout] = (double)c / (double)uni;  // correctly rounded, as Python's float division
          }
        }
      }
      __syncthreads();  // the bitmap and this source's counter are free for the next source
      PROF(5)
    }
  }
  PROF_FLUSH
}

// ------------------------------------------------------------------ wedge-set scorer (round 6)
// The business side of a bipartite graph without grouping or per-source builds. For a pair (x, y)
// -- x a business, y a user -- the reference's CN is |H2(x) ∩ N(y)| with H2(x) = N(N(x)) \ {x}
// (similarity.py:63-106). Membership is symmetric: c ∈ N(N(x)) ⟺ x ∈ N(N(c)). So instead of
// building H2(x) in LDS per source (after sorting the pairs by x), each pair tests x's bit in the
// wedge set W(c) of each c ∈ N(y) -- bitmaps the graph keeps in HBM (WedgeSets, hop3.hip; 1.25 GB at
// config 2). One thread per pair, in caller order: a user's pairs are consecutive, so the row N(y)
// and its ~10 sets are shared by a whole run of lanes and stay in L2. |H2(x)| comes from the index
// too. Counts and exact Adamic-Adar words are the short-row scorer's, bit for bit; the outputs are
// written in caller order, coalesced. The grid's blocks are mapped XCD-major: the blocks one XCD
// runs at a time take consecutive pairs, so a run's sets are fetched into one L2, not eight.
struct WsetArgs {
  const int32_t* x;
  const int32_t* y;
  const uint32_t* pool;  // W(c) at pool + (c - lo) * words
  const int32_t* h2;     // |W(c) \ {c}|
  int64_t lo, span, words;
};

template <bool SAA>
// (Two pairs per thread, their chains in flight together: 96 VGPRs, 5 waves per SIMD, and the
// step 1.735-1.741 against 1.716-1.722 ms, r06_check4. Blocks on contiguous pair ranges, each
// thread keeping its user's row in registers across its consecutive pairs: the kernel 0.242 ->
// 0.266 ms, step 1.72 -> 1.73 ms, r06_ab5 -- ~3x more users in flight per XCD, so their sets
// crowd the L2; the grid-stride window keeps one XCD on ~90 consecutive users.)
__global__ __launch_bounds__(256) void k_score_wset(ScoreArgs a, WsetArgs w) {
  __shared__ long long s_wtab[SAA ? 256 : 1];
  if (SAA && a.wtab)
    for (int i = threadIdx.x; i < 256; i += 256) s_wtab[i] = a.wtab[i];
  if (SAA) __syncthreads();
  const bool want_j = (a.mask & BLP_JACCARD) != 0;
  const bool want_a = SAA && (a.mask & BLP_ADAMIC) != 0;
  const uint32_t span = (uint32_t)w.span, lou = (uint32_t)w.lo;
  const int nb = (int)gridDim.x, bid = (int)blockIdx.x;
  const int lb = (nb & 7) == 0 ? (bid & 7) * (nb >> 3) + (bid >> 3) : bid;  // XCD-major (blocks go to XCDs round robin)
  for (int64_t i = (int64_t)lb * 256 + threadIdx.x; i < a.np; i += (int64_t)nb * 256) {
    const int x = w.x[i], y = w.y[i];
    if (!PS_OK(a.misc, x >= 0 && x < a.n_nodes && y >= 0 && y < a.n_nodes, 2, (int64_t)x, a.n_nodes)) continue;
    const uint32_t xr = (uint32_t)x - lou;  // < span (planned: every source lies in the sets' range)
    if (!PS_OK(a.misc, xr < span, 12, (int64_t)xr, w.span)) continue;
    const int64_t st = a.rp[y];
    const int len = (int)(a.rp[y + 1] - st);
    const uint32_t* col = w.pool + (xr >> 5);  // x's word in every set
    const uint32_t xb = xr & 31;
    unsigned c = 0;
    unsigned long long acc = 0;
    uint32_t acch = 0;
    for (int h = 0; h < len; h += SHORT_PART) {
      int e[SHORT_PART];
      row_part(a.cw, st, len, h, e);
      uint32_t wd[SHORT_PART];
#pragma unroll
      for (int j = 0; j < SHORT_PART; ++j) {
        const uint32_t id = (uint32_t)e[j] & a.idmask;
        const uint32_t r = id - lou;
        wd[j] = (h + j < len && r < span && id != (uint32_t)x) ? col[(int64_t)r * w.words] : 0u;
      }
      if constexpr (SAA) {
        uint32_t hm = 0;
#pragma unroll
        for (int j = 0; j < SHORT_PART; ++j) hm |= ((wd[j] >> xb) & 1u) << j;
        c += (unsigned)__popc(hm);
        if (want_a && hm) aa_terms<SHORT_PART>(e, hm, a.idbits, a.idmask, s_wtab, a.aaw, acc, acch);
      } else {
#pragma unroll
        for (int j = 0; j < SHORT_PART; ++j) c += (wd[j] >> xb) & 1u;
      }
    }
    a.cn[i] = c;
    if (SAA && want_a) a.aa[i] = blp::aa_value(acc, acch);
    if (want_j) {
      const long long uni = (long long)w.h2[xr] + len - (long long)c;
      if (uni <= 0) {
        a.jac[i] = __builtin_nan("");
        atomicOr(&a.misc->zero_div, 1);
      } else {
        a.jac[i] = (double)c / (double)uni;  // correctly rounded, as Python's float division
      }
    }
  }
}

// ------------------------------------------------------------------ HBM-bitmap scorer
// Universes wider than one workgroup's LDS (config 5: H2(u) over 50M users = 6.25 MB) would
// need one full H2 rebuild per LDS chunk. Here every workgroup owns a private bitmap slot in
// HBM covering the whole universe: it is built once per source with workgroup-scope atomics
// (performed in the XCD's L2 -- no cross-XCD coherence is needed for private data), then, after
// an agent-scope fence (drains the stores, invalidates the CU's L1), popcounted and scanned with
// plain loads. Same merge-path build / scan loops and pair bookkeeping as k_score.
template <int BLOCK, int SEG, int K>
__global__ __launch_bounds__(BLOCK) void k_score_global(ScoreArgs a, uint32_t* gbm, int64_t gwords) {
  constexpr int NW = BLOCK / 64;
  __shared__ int64_t s_start[SEG];
  __shared__ int32_t s_off[SEG + 1];
  __shared__ uint32_t s_cn[SEG];
  __shared__ unsigned long long s_aa[2 * SEG];
  __shared__ unsigned long long red64[NW];
  __shared__ int red[NW];
  __shared__ int s_src;
  uint32_t* bm = gbm + (int64_t)blockIdx.x * gwords;
  uint4* bm4 = reinterpret_cast<uint4*>(bm);
  const int64_t nw4 = gwords >> 2;
  const int64_t c0 = a.lo, width = a.hi - a.lo;
  const bool want_j = (a.mask & BLP_JACCARD) != 0;
  const bool want_a = (a.mask & BLP_ADAMIC) != 0;
  const int n_active = a.misc->n_active;
  for (;;) {
    if (threadIdx.x == 0) s_src = atomicAdd(&a.misc->queue, a.dq);
    __syncthreads();
    const int s_first = s_src;
    __syncthreads();
    if (s_first >= n_active) break;
    const int s_last = min(n_active, s_first + a.dq);
    for (int s = s_first; s < s_last; ++s) {
      const int x = a.active[s];
      const int pbeg = a.off[x], pcnt = a.cnt[x];
      const int64_t xb = a.rp[x], xe = a.rp[x + 1];
      for (int64_t i = threadIdx.x; i < nw4; i += BLOCK) bm4[i] = make_uint4(0, 0, 0, 0);
      __threadfence();
      __syncthreads();
      for (int64_t k0 = xb; k0 < xe; k0 += SEG) {
        const int ns = (int)min<int64_t>(SEG, xe - k0);
        load_row_segments<BLOCK>(a.rp, a.ci, k0, ns, s_start, s_off, red, nullptr);
        mp_build<BLOCK, K, true>(a.cw, a.idmask, s_start, s_off, ns, c0, width, bm, threadIdx.x);
        __syncthreads();
      }
      for (int64_t k = xb + threadIdx.x; k <= xe; k += BLOCK) {  // drop N(x) and x itself
        const int64_t r = (k == xe ? (int64_t)x : (int64_t)a.ci[k]) - c0;
        if (r >= 0 && r < width)
          __hip_atomic_fetch_and(&bm[r >> 5], ~(1u << (r & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __threadfence();
      __syncthreads();
      unsigned long long h2 = 0;
      if (want_j) {
        unsigned long long pc = 0;
        for (int64_t i = threadIdx.x; i < nw4; i += BLOCK) {
          const uint4 q = bm4[i];
          pc += __popc(q.x) + __popc(q.y) + __popc(q.z) + __popc(q.w);
        }
        h2 = block_sum_u64<BLOCK>(pc, red64);
      }
      for (int sb = 0; sb < pcnt; sb += SEG) {
        const int ns = min(SEG, pcnt - sb);
        int len = 0;
        if ((int)threadIdx.x < ns) {
          const int gp = pbeg + sb + threadIdx.x;
          s_start[threadIdx.x] = a.g_yb[gp];
          len = a.g_yl[gp];
          s_cn[threadIdx.x] = 0;
          s_aa[2 * threadIdx.x] = 0;
          s_aa[2 * threadIdx.x + 1] = 0;
        }
        int tot;
        const int ex = block_exscan<BLOCK>(len, red, &tot);
        if ((int)threadIdx.x < ns) s_off[threadIdx.x] = ex;
        if (threadIdx.x == 0) s_off[ns] = tot;
        __syncthreads();
        if (want_a)
          mp_scan<BLOCK, K, true>(a.cw, a.idmask, a.idbits, a.aaw, a.wtab, s_start, s_off, ns, c0, width, bm, s_cn, s_aa, threadIdx.x);
        else
          mp_scan<BLOCK, K, false>(a.cw, a.idmask, a.idbits, a.aaw, a.wtab, s_start, s_off, ns, c0, width, bm, s_cn, s_aa, threadIdx.x);
        __syncthreads();
        for (int t = threadIdx.x; t < ns; t += BLOCK) {
          const int p = gout(a, pbeg + sb + t);
          const unsigned c = s_cn[t];
          a.cn[p] = c;
          if (want_a) a.aa[p] = blp::aa_value(s_aa[2 * t], s_aa[2 * t + 1]);
          if (want_j) {
            const long long uni = (long long)h2 + (s_off[t + 1] - s_off[t]) - (long long)c;
            if (uni <= 0) {
              a.jac[p] = __builtin_nan("");
              atomicOr(&a.misc->zero_div, 1);
            } else {
              a.jac[p] = (double)c / (double)uni;
            }
          }
        }
        __syncthreads();
      }
    }
  }
}

// ------------------------------------------------------------------ chunk-parallel scorer
// Universes between one and eight 512K-bit chunks (the user side of config 2: 1M users). A
// 125 KB bitmap would hold one workgroup per CU (16 waves) and the scorer is latency-bound, so
// the universe is cut into C chunks of 64 KB bitmaps and every (source, chunk) is an
// independent item: two workgroups per CU (32 waves). Rows are sorted, so a chunk reads only
// its slice of each row N(z) / N(y) -- the slice bounds come from a per-row split table, and
// no element is read twice. Items are source-major (both chunks of a source run at the same
// time on different CUs and share its rows in L2). A (pair, chunk) slice with hits adds its
// count and exact AA words to the pair's accumulators in HBM (device-scope atomics; slices
// without hits add nothing); |H2| partials go to [sources][chunks]; k_split_combine computes
// the final values and Jaccard.
// The split table rsplit[row][c]: int32 offsets into the row. (A 16-bit twin for rows under
// 65535 ids, 196 instead of 392 MB at config 5, measured 514 against 482 ms per step, r05_ab6.)
__global__ void k_row_splits(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci, int64_t v0, int64_t n,
                             int64_t lo, int64_t cap_bits, int C, int32_t* __restrict__ rsplit) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = v0 + i;
    const int64_t b = rp[v], e = rp[v + 1];
    for (int c = 0; c <= C; ++c) {
      const int64_t bound = c == C ? INT64_MAX : lo + c * cap_bits;
      int64_t l = b, h = e;
      while (l < h) {
        const int64_t m = (l + h) >> 1;
        if (ci[m] < bound) l = m + 1; else h = m;
      }
      rsplit[i * (C + 1) + c] = (int32_t)(l - b);
    }
  }
}

// Row offsets [s0, s1) of chunk c of split-table row `row`.
__device__ __attribute__((always_inline)) inline void split_bounds(const int32_t* __restrict__ rsplit, int64_t row,
                                                                   int C, int c, int& s0, int& s1) {
  const int32_t* sp = rsplit + row * (C + 1) + c;
  s0 = sp[0];
  s1 = sp[1];
}

constexpr int SPLIT_CN_BITS = 24;  // k_score_split pk24: count field of the packed per-pair word
constexpr int SPLIT_ROUND = 16;  // k_score_split: 64-pair groups per wave between block syncs (config 5: 4 -> 341, 8 -> 317-324, 16 -> 322 ms)
constexpr int SPLIT_LQ = 16 * SPLIT_ROUND * 64;  // long-slice queue entries per workgroup (16 waves)

template <int BLOCK, int CAP_WORDS, int SEG, int K>
__global__ __launch_bounds__(BLOCK, CAP_WORDS > 16384 ? 4 : 8) void k_score_split(ScoreArgs a, const int32_t* __restrict__ g_y,
                                                       const int32_t* __restrict__ rsplit,
                                                       int64_t rs_lo, int C,
                                                       uint32_t* __restrict__ pcn, unsigned long long* __restrict__ paa,
                                                       uint32_t* __restrict__ ph2, int64_t np, int pk24, int short_max) {
  constexpr int NW = BLOCK / 64;
  static_assert(NW * SPLIT_ROUND * 64 <= SPLIT_LQ, "a round's long slices fit the queue");
  // 128 KiB chunks (one workgroup per CU) use the row-chunk loops of the large scorer
  constexpr bool RCS = BLP_RC && CAP_WORDS > 16384;
  constexpr int HCS = RCS ? 1536 : 1;
  __shared__ uint32_t bm[CAP_WORDS + (RCS ? RC_EXTRA_WORDS : 0)];
  __shared__ int64_t s_start[SEG];
  __shared__ int32_t s_off[SEG + 1];
  __shared__ int32_t s_coff[RCS ? SEG + 1 : 1];
  __shared__ int32_t s_hint[HCS];
  __shared__ unsigned long long s_aa[2 * SEG];  // packed: [2t] Σ W, [2t + 1] high word << 21 | count
  __shared__ unsigned long long red64[NW];
  __shared__ int red[NW];
  __shared__ int64_t s_item[2];  // the claimed item, alternating slots (no barrier guards its rewrite)
  __shared__ int s_nhot;
  __shared__ int s_nl;  // long slices queued in this round
  __shared__ blp::HotRow s_hot[HOT_LIST];
  __shared__ long long s_wtab[RCS ? 256 : 1];  // code weights in LDS (the 64 KiB variant has no room)
  const int64_t CAP_BITS = a.cap_bits;
  const bool want_j = (a.mask & BLP_JACCARD) != 0;
  const bool want_a = (a.mask & BLP_ADAMIC) != 0;
  uint4* bm4 = reinterpret_cast<uint4*>(bm);
  if (RCS && a.wtab)  // visible after the first barrier
    for (int i = threadIdx.x; i < 256; i += BLOCK) s_wtab[i] = a.wtab[i];
  const long long* wtab = RCS ? s_wtab : a.wtab;
  if (RCS)  // the zero word and the build's dummy words past the bitmap
    for (int i = threadIdx.x; i < RC_EXTRA_WORDS; i += BLOCK) bm[CAP_WORDS + i] = 0;
  if (threadIdx.x == 0) s_nl = 0;  // visible after the first barrier
  const int s_base = a.misc->n_hash_front;  // hash-routed sources (partitioned to the front) are not ours
  const int n_src = a.misc->n_active - s_base;
  // Items (source, chunk) are claimed per XCD group: workgroups b and b + 8 share an XCD (and its
  // L2; a placement observation, used for speed only), group g = b mod 8 takes the sources
  // s = g (mod 8), all C chunks of a source in a row, so the C workgroups scanning one source's
  // pair rows chunk by chunk do it on one XCD, close in time, and share those rows in its L2
  // instead of fetching each 128-byte line into several L2s. A group whose sources are done
  // takes items of the next group (queue heads misc->qh[g]). Measured against one global queue
  // in chunk-major order (every source's chunk c before any chunk c + 1): 326 -> 484 ms.
  const int grp = (int)(blockIdx.x & 7);
  constexpr int ngrp = 8;
  int gq = 0;  // thread 0: groups found empty so far
  PROF_INIT  // -DBLP_PROF phase clocks: 0 claim, 1 build, 2 popcount, 3 batch to short scan, 4 long scan, 5 partials
  for (int it = 0;; ++it) {
    if (threadIdx.x == 0) {
      int64_t claimed = -1;
      while (gq < ngrp) {
        const int g = (grp + gq) % ngrp;
        const int64_t n_g = n_src > g ? (n_src - g + ngrp - 1) / ngrp : 0;
        const int k = atomicAdd(&a.misc->qh[g], 1);
        if ((int64_t)k < n_g * C) {
          claimed = (int64_t)(g + (int64_t)ngrp * (k / C)) * C + k % C;
          break;
        }
        ++gq;
      }
      s_item[it & 1] = claimed;  // slot it & 1 is rewritten two claims later, past this one's barriers
    }
    __syncthreads();
    const int64_t item = s_item[it & 1];
    if (item < 0) break;
    PROF(0)
    const int s = s_base + (int)(item / C), c = (int)(item % C);
    if (!PS_OK(a.misc, s < a.misc->n_active, 1, s, a.misc->n_active)) continue;  // uniform
    const int x = a.active[s];
    if (!PS_OK(a.misc, x >= 0 && x < a.n_nodes, 2, x, a.n_nodes)) continue;
    const int pbeg = a.off[x], pcnt = a.cnt[x];
    if (!PS_OK(a.misc, pbeg >= 0 && (int64_t)pbeg + pcnt <= a.np, 3, (int64_t)pbeg + pcnt, a.np)) continue;
    const int64_t xb = a.rp[x], xe = a.rp[x + 1];
    const int hslot = a.heavy_slot ? a.heavy_slot[x] : -1;
    const int64_t c0 = a.lo + (int64_t)c * CAP_BITS;
    const int64_t width = max<int64_t>(min(a.hi, c0 + CAP_BITS) - c0, 0);
    if (!PS_OK(a.misc, width <= 32ll * CAP_WORDS, 9, width, 32ll * CAP_WORDS)) continue;
    const int nw4 = (int)((((width + 31) >> 5) + 3) >> 2);
    int64_t wb = a.wp ? a.wp[x] : 0, we = a.wp ? a.wp[x + 1] : 0;
    if (!PS_OK(a.misc, wb >= 0 && wb <= we && we <= a.wedge_vecs, 11, we, a.wedge_vecs)) wb = we = 0;
    if (hslot >= 0) {
      const uint4* src4 = reinterpret_cast<const uint4*>(a.heavy_bm + (int64_t)hslot * a.hb_words + ((c0 - a.lo) >> 5));
      for (int i = threadIdx.x; i < nw4; i += BLOCK) bm4[i] = src4[i];
      __syncthreads();
    } else if (we > wb) {
      // x's wedge row (wedge.hip: N(N(x)) back to back, a source whose members' rows are short,
      // i.e. the business side): one contiguous stream filtered to this chunk, instead of a
      // row_ptr and two split-table lookups per member for a ~10-id slice
      for (int i = threadIdx.x; i < nw4; i += BLOCK) bm4[i] = make_uint4(0, 0, 0, 0);
      __syncthreads();
      const uint32_t keep = a.idmask | 0x80000000u, c0u = (uint32_t)c0, wu = (uint32_t)width;
      for (int64_t q = wb + threadIdx.x; q < we; q += 2 * BLOCK) {
        const uint4 v0 = a.wedge[q];
        const uint4 v1 = q + BLOCK < we ? a.wedge[q + BLOCK] : v0;  // (a repeat ORs nothing new)
        const uint32_t ids[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t r = in_chunk((int)ids[k], keep, c0u);
          if (r < wu) atomicOr(&bm[r >> 5], 1u << (r & 31));
        }
      }
      __syncthreads();
    } else {
      if (threadIdx.x == 0) s_nhot = 0;
      __syncthreads();
      if (a.hot_idx) {
        for (int64_t k = xb + threadIdx.x; k < xe; k += BLOCK) {
          const int hi = a.hot_idx[a.ci[k]];
          if (hi >= 0 && PS_OK(a.misc, hi < a.n_hot, 12, hi, a.n_hot)) {
            const int slot = atomicAdd(&s_nhot, 1);
            if (slot < HOT_LIST) s_hot[slot] = a.hot_tab[hi];
          }
        }
      }
      __syncthreads();
      const int nhot = s_nhot <= HOT_LIST ? s_nhot : 0;
      const int64_t q0 = c0 >> 7;
      for (int q = threadIdx.x; q < nw4; q += BLOCK) {
        uint4 v = make_uint4(0, 0, 0, 0);
        for (int r = 0; r < nhot; ++r) {
          const int64_t qq = q0 + q - s_hot[r].vlo;
          if (qq >= 0 && qq < s_hot[r].nvec &&
              PS_OK(a.misc, s_hot[r].vec_off + qq < a.hot_vecs, 13, s_hot[r].vec_off + qq, a.hot_vecs)) {
            const uint4 pv = a.hot_pool[s_hot[r].vec_off + qq];
            v.x |= pv.x;
            v.y |= pv.y;
            v.z |= pv.z;
            v.w |= pv.w;
          }
        }
        bm4[q] = v;
      }
      __syncthreads();
      for (int64_t k0 = xb; k0 < xe; k0 += SEG) {
        const int ns = (int)min<int64_t>(SEG, xe - k0);
        int len = 0;
        if ((int)threadIdx.x < ns) {
          const int z = a.ci[k0 + threadIdx.x];
          if (PS_OK(a.misc, (int64_t)z - rs_lo >= 0 && (int64_t)z - rs_lo < a.rs_rows, 7, (int64_t)z - rs_lo, a.rs_rows)) {
            int sp0, sp1;
            split_bounds(rsplit, (int64_t)z - rs_lo, C, c, sp0, sp1);
            s_start[threadIdx.x] = a.rp[z] + sp0;
            len = (nhot && a.hot_idx[z] >= 0) ? 0 : sp1 - sp0;  // dense rows were OR-ed in
            if (!PS_OK(a.misc, sp0 >= 0 && len >= 0 && s_start[threadIdx.x] + len <= a.nnz, 10,
                       s_start[threadIdx.x] + len, a.nnz))
              len = 0;
          } else {
            s_start[threadIdx.x] = 0;
          }
        }
        int tot;
        const int ex = block_exscan<BLOCK>(len, red, &tot);
        if ((int)threadIdx.x < ns) s_off[threadIdx.x] = ex;
        if (threadIdx.x == 0) s_off[ns] = tot;
        __syncthreads();
        if constexpr (RCS) {
          rc_chunk_offsets<BLOCK, K>(s_off, ns, s_coff, red);
          const int shift = build_hint<BLOCK, HCS>(s_coff, ns, BLOCK, s_hint);
          rc_build<BLOCK, K>(a.cw, a.idmask, s_start, s_off, s_coff, ns, c0, width, bm, CAP_WORDS, threadIdx.x, s_hint,
                             shift);
        } else {
          mp_build<BLOCK, K>(a.cw, a.idmask, s_start, s_off, ns, c0, width, bm, threadIdx.x);
        }
        __syncthreads();
      }
    }
    PROF(1)
    // exact distance 2 inside this chunk: drop x and N(x)
    const int64_t nx_lo = xe > xb ? a.ci[xb] : 0, nx_hi = xe > xb ? a.ci[xe - 1] : -1;
    if (nx_hi >= c0 && nx_lo < c0 + width) {
      for (int64_t k = xb + threadIdx.x; k < xe; k += BLOCK) {
        const int64_t r = (int64_t)a.ci[k] - c0;
        if (r >= 0 && r < width) atomicAnd(&bm[r >> 5], ~(1u << (r & 31)));
      }
    }
    if (threadIdx.x == 0 && x >= c0 && x < c0 + width) atomicAnd(&bm[(x - c0) >> 5], ~(1u << ((x - c0) & 31)));
    __syncthreads();
    if (want_j) {
      unsigned long long pc = 0;
      for (int i = threadIdx.x; i < nw4; i += BLOCK) {
        const uint4 q = bm4[i];
        pc += __popc(q.x) + __popc(q.y) + __popc(q.z) + __popc(q.w);
      }
      const unsigned long long h2 = block_sum_u64<BLOCK, false>(pc, red64);  // red64's next use is past a round's barrier
      if (threadIdx.x == 0) ph2[(int64_t)s * C + c] = (uint32_t)h2;
    }
    PROF(2)
    // Pair slices of this chunk, in rounds of NW * SPLIT_ROUND groups of 64 pairs. Within a round
    // every wave runs its own groups with no block barrier: lane = pair, its y / row start
    // (coalesced), its slice bounds from the split table, then -- for a short slice (<=
    // short_max ids; 128 KiB chunks; ~92 % of the slices at config 5) -- one part of up to 16
    // ids in registers tested against the bitmap, and the slice's partial words sent from
    // registers; the 16 waves of the CU hide each other's round trips. A long slice is queued
    // (this workgroup's region of a global queue: row start, length, pair); at the end of the
    // round the block scans the queued slices together with the row-chunk loops, SEG at a time.
    // Partial words: lo = S mod 2^64, hi = (S >> 40) << 21 | count (exact: a slice's terms
    // undercount S by < 2^44).
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t keep = a.idmask | 0x80000000u, c0u = (uint32_t)c0, wu = (uint32_t)width;
    if (!PS_OK(a.misc, (int)blockIdx.x < a.lq_wgs, 6, blockIdx.x, a.lq_wgs)) break;  // uniform
    int4* lq = a.lq + (int64_t)blockIdx.x * SPLIT_LQ;
    // a (pair, chunk) slice's partial words into the pair's accumulators: only slices with a hit
    // add anything, so no [chunks][pairs] partial arrays (config 5: 48 chunks x 199M pairs) and
    // no dense combine reads. With Adamic-Adar and every scanned row shorter than 2^24 (pk24), two
    // atomics: paa[p] += S mod 2^64 and paa[np + p] += (S >> 52) << 24 | count -- exact
    // (blp::aa_exact with hs = 52: the 2^52 remainders of at most C < 2^12 slices sum below 2^64;
    // S >> 52 <= count * 2^7 per slice, so the high field stays below 2^40); otherwise the count,
    // S mod 2^64 and S >> 32 in three. All low words come first, then all high words: a wave's
    // atomics to its 64 consecutive pairs then cover 512 contiguous bytes per word (device-scope
    // atomics execute at the memory side, one request per 64-B segment) instead of 1 KiB with
    // every other word (interleaved [pair][2]: config 5 step 482-489 against 472-477 ms, r06_ab8).
    auto emit = [&](int64_t gp, unsigned long long w0, unsigned long long w1) {
      const unsigned c_t = (unsigned)(w1 & ((1u << PK_CN_BITS) - 1));
      if (!c_t || !PS_OK(a.misc, gp >= 0 && gp < a.np, 4, gp, a.np)) return;
      if (want_a) {
        unsigned long long sh, sl;
        blp::aa_exact(w0, w1 >> PK_CN_BITS, &sh, &sl, PK_HS);
        atomicAdd(&paa[gp], sl);
        if (pk24) {
          atomicAdd(&paa[np + gp], (((sh << 12) | (sl >> 52)) << SPLIT_CN_BITS) | c_t);
        } else {
          atomicAdd(&pcn[gp], c_t);
          atomicAdd(&paa[np + gp], (sh << 32) | (sl >> 32));
        }
      } else {
        atomicAdd(&pcn[gp], c_t);
      }
    };
    const int ngr = (pcnt + 63) >> 6;
    const int rg = NW * SPLIT_ROUND;
    for (int r0 = 0; r0 < ngr; r0 += rg) {
      const int r1 = min(ngr, r0 + rg);
      for (int g = r0 + wv; g < r1; g += NW) {
        const int q = g * 64 + lane;
        int len = 0;
        int64_t st = 0;
        if (q < pcnt) {
          const int gp = pbeg + q;
          const int64_t row = (int64_t)g_y[gp] - rs_lo;
          if (PS_OK(a.misc, row >= 0 && row < a.rs_rows, 7, row, a.rs_rows)) {
            int s0, s1;
            split_bounds(rsplit, row, C, c, s0, s1);
            len = s1 - s0;
            st = a.g_yb[gp] + s0;
            if (!PS_OK(a.misc, s0 >= 0 && len >= 0 && st + len <= a.nnz, 10, st + len, a.nnz)) len = 0;
          }
        }
        if (len > 0 && len <= short_max) {
          int sv[SHORT_PART] = {};  // ids past len stay 0 (masked by len below)
          row_part(a.cw, st, len, 0, sv);
          // branch-free phases (as rc_scan): every bitmap word (and code weight) of the part is read
          // before the first is used -- one LDS round trip per slice, not one per id -- and the
          // weights come from the LDS code table; code-0 hits then gather aaw (rare)
          uint32_t rr[SHORT_PART], wd[SHORT_PART];
#pragma unroll
          for (int k = 0; k < SHORT_PART; ++k) {
            const uint32_t r = in_chunk(sv[k], keep, c0u);
            rr[k] = (k < len && r < wu) ? r : 0u;
          }
#pragma unroll
          for (int k = 0; k < SHORT_PART; ++k) wd[k] = bm[rr[k] >> 5];
          uint32_t hm = 0;
#pragma unroll
          for (int k = 0; k < SHORT_PART; ++k) {
            const uint32_t r = in_chunk(sv[k], keep, c0u);
            hm |= ((k < len && r < wu) ? (wd[k] >> (rr[k] & 31)) & 1u : 0u) << k;
          }
          unsigned long long lo = 0, hi40 = 0;
          if (want_a && hm) {
            long long wt[SHORT_PART];
#pragma unroll
            for (int k = 0; k < SHORT_PART; ++k) wt[k] = wtab[((uint32_t)sv[k] >> a.idbits) & 255u];
            uint32_t esc = 0;
#pragma unroll
            for (int k = 0; k < SHORT_PART; ++k) {
              const bool h = (hm >> k) & 1u;
              const unsigned long long w = h ? (unsigned long long)wt[k] : 0ull;
              lo += w;
              hi40 += w >> PK_HS;
              esc |= (h && ((((uint32_t)sv[k] >> a.idbits) & 255u) == 0u)) ? 1u << k : 0u;
            }
            if (esc) {
#pragma unroll
              for (int k = 0; k < SHORT_PART; ++k)
                if ((esc >> k) & 1u) {
                  const unsigned long long w = (unsigned long long)a.aaw[sv[k] & a.idmask];
                  lo += w;
                  hi40 += w >> PK_HS;
                }
            }
          }
          emit(pbeg + q, lo, (hi40 << PK_CN_BITS) | (uint32_t)__popc(hm));
        } else if (len > short_max) {
          const int slot = atomicAdd(&s_nl, 1);  // < SPLIT_LQ: a round holds NW * SPLIT_ROUND * 64 pairs
          if (PS_OK(a.misc, slot < SPLIT_LQ, 5, slot, SPLIT_LQ))
            lq[slot] = make_int4((int32_t)(uint32_t)st, (int32_t)(st >> 32), len, pbeg + q);
        }
      }
      __syncthreads();
      PROF(3)
      const int nl = min(s_nl, SPLIT_LQ);
      for (int b0 = 0; b0 < nl; b0 += SEG) {  // the round's long slices, block-wide
        const int ns = min(SEG, nl - b0);
        int len = 0, gp = 0;
        if ((int)threadIdx.x < ns) {
          const int4 e = lq[b0 + threadIdx.x];
          s_start[threadIdx.x] = (int64_t)(((uint64_t)(uint32_t)e.y << 32) | (uint32_t)e.x);
          len = e.z;
          gp = e.w;
          s_aa[2 * threadIdx.x] = 0;
          s_aa[2 * threadIdx.x + 1] = 0;
        }
        if constexpr (RCS) {
          seg_offsets<BLOCK, K>(len, ns, s_off, s_coff, red64);
          const int shift = build_hint<BLOCK, HCS>(s_coff, ns, BLOCK, s_hint);
          if (want_a)
            rc_scan<BLOCK, K, true>(a.cw, a.idmask, a.idbits, a.aaw, wtab, s_start, s_off, s_coff, ns, c0, width, bm,
                                    CAP_WORDS, nullptr, s_aa, threadIdx.x, s_hint, shift, true);
          else
            rc_scan<BLOCK, K, false>(a.cw, a.idmask, a.idbits, a.aaw, wtab, s_start, s_off, s_coff, ns, c0, width, bm,
                                     CAP_WORDS, nullptr, s_aa, threadIdx.x, s_hint, shift, true);
        } else {
          int tot;
          const int ex = block_exscan<BLOCK>(len, red, &tot);
          if ((int)threadIdx.x < ns) s_off[threadIdx.x] = ex;
          if (threadIdx.x == 0) s_off[ns] = tot;
          __syncthreads();
          if (want_a)
            mp_scan<BLOCK, K, true, true>(a.cw, a.idmask, a.idbits, a.aaw, a.wtab, s_start, s_off, ns, c0, width, bm,
                                          nullptr, s_aa, threadIdx.x);
          else
            mp_scan<BLOCK, K, false, true>(a.cw, a.idmask, a.idbits, a.aaw, a.wtab, s_start, s_off, ns, c0, width, bm,
                                           nullptr, s_aa, threadIdx.x);
        }
        __syncthreads();
        if ((int)threadIdx.x < ns) emit(gp, s_aa[2 * threadIdx.x], s_aa[2 * threadIdx.x + 1]);
        __syncthreads();
      }
      if (threadIdx.x == 0) s_nl = 0;
      __syncthreads();
      PROF(4)
    }
  }
  PROF_FLUSH
}

// one wave per active source: sum the chunk partials of each of its pairs, then Jaccard
__global__ __launch_bounds__(256) void k_split_combine(ScoreArgs a, int C, const uint32_t* __restrict__ pcn,
                                                      const unsigned long long* __restrict__ paa,
                                                      const uint32_t* __restrict__ ph2, int64_t np, int pk24) {
  const int lane = threadIdx.x & 63;
  const int n_active = a.misc->n_active;
  const bool want_j = (a.mask & BLP_JACCARD) != 0;
  const bool want_a = (a.mask & BLP_ADAMIC) != 0;
  const int s_base = a.misc->n_hash_front;  // sources before it were scored by k_score_hash
  for (int s = s_base + ((blockIdx.x * blockDim.x + threadIdx.x) >> 6); s < n_active; s += (gridDim.x * blockDim.x) >> 6) {
    const int x = a.active[s];
    long long h2 = 0;
    if (want_j)
      for (int c = 0; c < C; ++c) h2 += ph2[(int64_t)s * C + c];
    const int pbeg = a.off[x], pcnt = a.cnt[x];
    for (int t = lane; t < pcnt; t += 64) {
      const int64_t gp = pbeg + t;
      const unsigned long long lo = want_a ? paa[gp] : 0ull, hi = want_a ? paa[np + gp] : 0ull;
      const unsigned cn = pk24 ? (unsigned)(hi & ((1u << SPLIT_CN_BITS) - 1)) : pcn[gp];
      const int p = gout(a, gp);
      if (!PS_OK(a.misc, p >= 0 && p < a.np, 4, p, a.np)) continue;
      a.cn[p] = cn;
      if (want_a) a.aa[p] = pk24 ? blp::aa_value(lo, hi >> SPLIT_CN_BITS, 52) : blp::aa_value(lo, hi);
      if (want_j) {
        const long long uni = h2 + a.g_yl[gp] - (long long)cn;
        if (uni <= 0) {
          a.jac[p] = __builtin_nan("");
          atomicOr(&a.misc->zero_div, 1);
        } else {
          a.jac[p] = (double)cn / (double)uni;
        }
      }
    }
  }
}

// Split batches with hash-routed sources: one pass partitions the active list so that
// k_score_hash claims only its own sources from the front and k_score_split / k_split_combine
// only theirs after them. Each wave moves 64 consecutive entries (ballot, one atomic per list),
// so neighbouring sources stay neighbours inside a wave's run. Without it both persistent
// kernels claimed every source and skipped the other's -- three dependent round trips and two
// block barriers per skipped (source, chunk) item.
__global__ __launch_bounds__(256) void k_hash_partition(const int32_t* __restrict__ active, Misc* __restrict__ misc,
                                                        const uint8_t* __restrict__ hflag, int32_t xlo,
                                                        int32_t* __restrict__ out) {
  const int n = misc->n_active;
  const int lane = threadIdx.x & 63;
  const int nwv = (gridDim.x * blockDim.x) >> 6;
  for (int base = ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64; base < n; base += nwv * 64) {
    const int i = base + lane;
    const int x = i < n ? active[i] : 0;
    const bool h = i < n && hflag[x - xlo];
    const unsigned long long hb = __ballot(h), sb = __ballot(i < n && !h);
    const unsigned long long below = (1ull << lane) - 1;
    int fh = 0, bs = 0;
    if (lane == 0) {
      fh = hb ? atomicAdd(&misc->n_hash_front, __popcll(hb)) : 0;
      bs = sb ? atomicAdd(&misc->n_split_back, __popcll(sb)) : 0;
    }
    fh = __shfl(fh, 0);
    bs = __shfl(bs, 0);
    if (h)
      out[fh + __popcll(hb & below)] = x;
    else if (i < n)
      out[n - bs - __popcll(sb) + __popcll(sb & below)] = x;
  }
}

// ------------------------------------------------------------------ hash-set scorer
// Universes wider than LDS (the chunk-parallel scorer's batches) whose source has a SMALL H2: the
// business side of config 5 (H2(b) = the businesses co-reviewed with b, ~20 |N(b)| ids among 2M)
// pays the chunk-parallel scorer's per-item costs -- a 128 KiB bitmap zeroed and popcounted,
// offsets, barriers -- C times for a few thousand ids. Here H2(x) is an open-addressing hash set
// in LDS (HT slots, linear probing, load <= 1/2: the host routes only sources whose build work,
// the total length of the rows N(z), z in N(x), is at most HT / 2), built with one CAS per new id;
// x and N(x) are then tombstoned (exact distance 2) and every pair's N(y) probes the set. One
// pair per thread, results written directly (cn, Jaccard, exact Adamic-Adar words).
constexpr uint32_t HS_EMPTY = 0xFFFFFFFFu;
constexpr int HS_DQ = 4;  // k_score_hash: sources per claim
template <int HT>
__device__ inline uint32_t hs_slot(uint32_t v) {
  return (v * 2654435761u) >> (32 - __builtin_ctz(HT));
}

template <int BLOCK, int HT>
__global__ __launch_bounds__(BLOCK) void k_score_hash(ScoreArgs a) {
  constexpr int NW = BLOCK / 64;
  static_assert((HT & (HT - 1)) == 0, "HT: a power of two");
  __shared__ uint32_t tab[HT];
  __shared__ unsigned long long red64[NW];
  __shared__ int s_src[2];  // claimed sources, alternating slots
  const int n_hash = a.misc->n_hash_front;  // the partitioned active list's hash sources come first
  const bool want_j = (a.mask & BLP_JACCARD) != 0;
  const bool want_a = (a.mask & BLP_ADAMIC) != 0;
  const uint32_t c0u = (uint32_t)a.lo, wu = (uint32_t)(a.hi - a.lo);
  const uint32_t keep = a.idmask | 0x80000000u;
  auto find = [&](uint32_t v) -> int {  // slot of v (id - lo) or -1
    uint32_t h = hs_slot<HT>(v);
    for (int i = 0; i < HT; ++i) {  // bounded: a full table ends the probe
      const uint32_t t = tab[h];
      if (t == v) return (int)h;
      if (t == HS_EMPTY) return -1;
      h = (h + 1) & (HT - 1);
    }
    return -1;
  };
  // Sources are claimed HS_DQ at a time (one device-scope atomic per HS_DQ sources), and a
  // source's header -- its rows, its pair range and this thread's first pair -- is loaded before
  // the table is cleared, so those round trips overlap the clear instead of following the build.
  int si_next = 0, left = 0, claims = 0;  // uniform over the workgroup
  for (;;) {
    if (left == 0) {
      // slot claims & 1 is rewritten two claims later, past this claim's barriers
      if (threadIdx.x == 0) s_src[claims & 1] = atomicAdd(&a.misc->hq, HS_DQ);
      __syncthreads();
      si_next = s_src[claims & 1];
      ++claims;
      left = HS_DQ;
    }
    const int si = si_next++;
    --left;
    if (si >= n_hash) break;
    const int x = a.active[si];
    if (!PS_OK(a.misc, x >= 0 && x < a.n_nodes, 2, x, a.n_nodes)) continue;  // uniform
    const int64_t xb = a.rp[x], xe = a.rp[x + 1];
    int64_t wb = a.wp ? a.wp[x] : 0, we = a.wp ? a.wp[x + 1] : 0;
    if (!PS_OK(a.misc, wb >= 0 && wb <= we && we <= a.wedge_vecs, 11, we, a.wedge_vecs)) wb = we = 0;
    const int pbeg = a.off[x], pcnt = a.cnt[x];
    if (!PS_OK(a.misc, pbeg >= 0 && (int64_t)pbeg + pcnt <= a.np, 3, (int64_t)pbeg + pcnt, a.np)) continue;
    int64_t st0 = 0;
    int len0 = 0, p0 = 0;
    if ((int)threadIdx.x < pcnt) {
      st0 = a.g_yb[pbeg + threadIdx.x];
      len0 = a.g_yl[pbeg + threadIdx.x];
      p0 = gout(a, pbeg + threadIdx.x);
    }
    for (int i = threadIdx.x; i < HT / 4; i += BLOCK) reinterpret_cast<uint4*>(tab)[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
    __syncthreads();
    // build: one row N(z) per thread, 16 ids at a time (rows padded past nnz), or x's wedge row
    // (N(N(x)) back to back, wedge.hip) 4 ids per 16-byte load, two loads in flight per thread
    unsigned long long added = 0;
    auto insert = [&](uint32_t v) {
      uint32_t h = hs_slot<HT>(v);
      for (int probes = 0;; ++probes) {
        // the host routes only sources of build work <= HT / 2 (load <= 1/2): a full table is a bug
        if (!PS_OK(a.misc, probes < HT, 8, probes, HT)) break;
        const uint32_t t = tab[h];
        if (t == v) break;
        if (t == HS_EMPTY) {
          const uint32_t old = atomicCAS(&tab[h], HS_EMPTY, v);
          if (old == HS_EMPTY) {
            ++added;
            break;
          }
          if (old == v) break;
        }
        h = (h + 1) & (HT - 1);
      }
    };
    if (we > wb) {
      for (int64_t q = wb + threadIdx.x; q < we; q += 2 * BLOCK) {
        const uint4 v0 = a.wedge[q];
        const uint4 v1 = q + BLOCK < we ? a.wedge[q + BLOCK] : v0;  // (a repeat inserts nothing new)
        const uint32_t ids[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t v = in_chunk((int)ids[j], keep, c0u);
          if (v < wu) insert(v);
        }
      }
    } else {
      for (int64_t k = xb + threadIdx.x; k < xe; k += BLOCK) {
        const int z = a.ci[k];
        const int64_t st = a.rp[z];
        int len = (int)(a.rp[z + 1] - st);
        if (!PS_OK(a.misc, st >= 0 && len >= 0 && st + len <= a.nnz, 10, st + len, a.nnz)) len = 0;
        for (int h0 = 0; h0 < len; h0 += SHORT_PART) {
          int e[SHORT_PART];
          row_part(a.cw, st, len, h0, e);
#pragma unroll
          for (int j = 0; j < SHORT_PART; ++j) {
            const uint32_t v = in_chunk(e[j], keep, c0u);
            if (h0 + j < len && v < wu) insert(v);
          }
        }
      }
    }
    __syncthreads();
    // exact distance 2: x and N(x) out (tombstones keep the probe chains intact)
    unsigned long long removed = 0;
    for (int64_t k = xb - 1 + threadIdx.x; k < xe; k += BLOCK) {
      const int w = k < xb ? x : a.ci[k];
      const uint32_t v = (uint32_t)w - c0u;
      if (v < wu) {
        const int h = find(v);
        if (h >= 0) {
          tab[h] = v | 0x80000000u;
          ++removed;
        }
      }
    }
    const unsigned long long h2 = want_j ? block_sum_u64<BLOCK, false>(added - removed, red64) : 0ull;  // (next use: past the source's closing barrier)
    if (!want_j) __syncthreads();  // tombstones written before any probe
    // scan: one pair per thread (the first one's metadata came with the header)
    for (int t = threadIdx.x; t < pcnt; t += BLOCK) {
      const int gp = pbeg + t;
      const bool first = t == (int)threadIdx.x;
      const int64_t st = first ? st0 : a.g_yb[gp];
      int len = first ? len0 : a.g_yl[gp];
      if (!PS_OK(a.misc, st >= 0 && len >= 0 && st + len <= a.nnz, 10, st + len, a.nnz)) len = 0;
      const int p = first ? p0 : gout(a, gp);
      if (!PS_OK(a.misc, p >= 0 && p < a.np, 4, p, a.np)) continue;
      unsigned c = 0;
      unsigned long long acc = 0, acch = 0;
      for (int h0 = 0; h0 < len; h0 += SHORT_PART) {
        int e[SHORT_PART];
        row_part(a.cw, st, len, h0, e);
#pragma unroll
        for (int j = 0; j < SHORT_PART; ++j) {
          const uint32_t v = in_chunk(e[j], keep, c0u);
          if (h0 + j < len && v < wu && find(v) >= 0) {
            ++c;
            if (want_a) {
              const uint32_t code = ((uint32_t)e[j] >> a.idbits) & 255u;
              const unsigned long long w = (unsigned long long)(code ? a.wtab[code] : a.aaw[e[j] & a.idmask]);
              acc += w;
              acch += w >> 32;
            }
          }
        }
      }
      a.cn[p] = c;
      if (want_a) a.aa[p] = blp::aa_value(acc, acch);
      if (want_j) {
        const long long uni = (long long)h2 + len - (long long)c;
        if (uni <= 0) {
          a.jac[p] = __builtin_nan("");
          atomicOr(&a.misc->zero_div, 1);
        } else {
          a.jac[p] = (double)c / (double)uni;  // correctly rounded, as Python's float division
        }
      }
    }
    __syncthreads();  // every probe done before the next source clears the table
  }
}


enum Variant { V_SMALL = 0, V_MED = 1, V_LARGE = 2 };
// LDS bitmap words (16 / 64 / 136 KiB), threads per block, pair/row segments per chunk
constexpr int CAP_SMALL = 4096, CAP_MED = 16384, CAP_LARGE = 33792;  // 1.08M bits: fits 160 KiB with the exact AA words
constexpr int BLOCK_SMALL = 256, BLOCK_MED = 512, BLOCK_LARGE = 1024;
constexpr int HS_BLOCK = 512, HS_HT = 16384;  // hash-set scorer: 64 KiB table, two workgroups per CU
constexpr int HS_BLOCK_BIG = 1024, HS_HT_BIG = 32768;  // ... 128 KiB table, one per CU (BLP_HASH_BIG)
#ifndef BLP_SEG_LARGE
#define BLP_SEG_LARGE 512  // (experiment builds override it: pairs per scan segment of the large scorer)
#endif
constexpr int CAP_PKO = 31744, SEG_PKO = 896;  // k_score PKO: <= 1,015,808-node universes (config 2: 1M users)
constexpr int SEG_SMALL = 256, SEG_MED = 384, SEG_LARGE = BLP_SEG_LARGE;  // MED: two 512-thread workgroups per CU (<= 80 KiB LDS)
constexpr int SEG_MED_NOAA = 512;  // MED without Adamic-Adar (no AA words, no weight table in LDS)
constexpr int G_BLOCK = 1024, G_SEG = 512;  // HBM-bitmap scorer
constexpr int S_BLOCK = 1024, S_CAP = 16384, S_SEG = 512;  // chunk-parallel scorer: 64 KiB chunks, 2 blocks / CU (<= 80 KiB LDS each)
constexpr int S_CAP_BIG = 32768;  // ... or 128 KiB chunks, 1 block / CU: half the (pair, chunk) slices (wide universes)
constexpr int S_MAX_CHUNKS = 128;                          // up to 67M-node universes (config 5: 50M users)

inline int variant_block(int v) { return v == V_SMALL ? BLOCK_SMALL : v == V_MED ? BLOCK_MED : BLOCK_LARGE; }
inline int64_t variant_cap_bits(int v) { return 32ll * (v == V_SMALL ? CAP_SMALL : v == V_MED ? CAP_MED : CAP_LARGE); }

}  // namespace

namespace {
// Environment switches of the pair scorers, read ONCE per batch at blp_batch_create (never while
// scoring): path selectors the tests use to drive every kernel on small graphs, and two tuning
// overrides. Release behaviour is the all-default struct.
struct Knobs {
  bool no_runs = false;          // BLP_NO_RUNS: bucket-sort grouping even for source-grouped lists
  bool no_short = false;         // BLP_NO_SHORT: row-per-thread loops off
  bool no_short_kernel = false;  // BLP_NO_SHORT_KERNEL: the short-row scorer off (block scorer instead)
  int variant = -1;              // BLP_VARIANT: a wider LDS variant than needed
  int64_t chunk_bits = 0;        // BLP_CHUNK_BITS: force multi-chunk universes on small graphs
  int split_big = -1;            // BLP_SPLIT_BIG: 128 KiB (1) or 64 KiB (0) chunk-parallel chunks
  int split = -1;                // BLP_SPLIT: force C chunk-parallel chunks
  bool no_split = false;         // BLP_NO_SPLIT
  bool no_global = false;        // BLP_NO_GLOBAL
  bool force_global = false;     // BLP_FORCE_GLOBAL
  int64_t heavy_work = -1;       // BLP_HEAVY_WORK: heavy-source item size
  bool no_wedge = false;         // BLP_NO_WEDGE: build H2 from the CSR, not the wedge rows
  bool no_wbm_batch = false;     // BLP_NO_WBM_BATCH: no wedge-row bitmaps as pre-built H2 sets
  bool group_buckets = false;    // BLP_GROUP_BUCKETS: one workgroup per contiguous bucket
  bool no_hash = false;          // BLP_NO_HASH: no hash-set scorer in split batches
  bool hash_big = false;         // BLP_HASH_BIG: the 128 KiB-table hash-set scorer (1024 threads, build <= 16K ids)
  int64_t hash_work = -1;        // BLP_HASH_WORK: hash-set routing bound (build ids)
  bool no_wcodes = false;        // BLP_NO_WCODES: plain ids (per-hit weight gathers)
  bool split_nopk = false;       // BLP_SPLIT_NOPK: unpacked split partials
  bool no_ydirect = false;       // BLP_NO_YDIRECT: run-grouped block scorer reads gathered row starts (test knob)
  bool no_run_fast = false;      // BLP_NO_RUN_FAST: run grouping in four launches (scan order; test knob)
  int split_short = -1;          // BLP_SPLIT_SHORT: register-scanned slice bound (0: off)
  int cosched_cus = -1;          // BLP_COSCHED_CUS: tuning override of the co-scheduled CU share
  bool no_pko = false;           // BLP_NO_PKO: the large scorer's general variant instead of PKO
  bool debug_oom = false;        // BLP_DEBUG_OOM (BLP_DEBUG builds): the first create fails out of memory
  int item_nb = 512;             // BLP_ITEM_NB: at most this many interleaved buckets (a power of two; 512:
                                 // 2.271 / 2.261 against 2.317 / 2.315 ms with 2048, r05_group_geometry)
  int group_nblk = -1;           // BLP_GROUP_NBLK: hist / scatter workgroups (default 2 per CU)
  int short_cus = -1;            // BLP_SHORT_CUS: CUs' worth of short-row scorer workgroups (default all)
  int lpt = 1;                   // BLP_LPT: sources queued largest (build + scan work) first -- bit 1: run-grouped
                                 // batches (the default: config-2 step 2.243 / 2.238 / 2.233 -> 2.214 / 2.211 /
                                 // 2.213 ms, r05_pair_hi_second), bit 2: item-grouped batches (no gain); 0: id order
  std::string debug_null;        // BLP_DEBUG_NULL (BLP_DEBUG builds only): null this launch pointer, to
                                 // show the pre-launch pointer check (launch_pointers) refusing it
};

Knobs read_knobs() {
  Knobs k;
  auto on = [](const char* n) { return getenv(n) != nullptr; };
  auto num = [](const char* n, long long dflt) {
    const char* e = getenv(n);
    return e ? atoll(e) : dflt;
  };
  k.no_runs = on("BLP_NO_RUNS");
  k.no_short = on("BLP_NO_SHORT");
  k.no_short_kernel = on("BLP_NO_SHORT_KERNEL");
  k.variant = (int)num("BLP_VARIANT", -1);
  k.chunk_bits = num("BLP_CHUNK_BITS", 0);
  k.split_big = (int)num("BLP_SPLIT_BIG", -1);
  k.split = (int)num("BLP_SPLIT", -1);
  k.no_split = on("BLP_NO_SPLIT");
  k.no_global = on("BLP_NO_GLOBAL");
  k.force_global = on("BLP_FORCE_GLOBAL");
  k.heavy_work = num("BLP_HEAVY_WORK", -1);
  k.no_wedge = on("BLP_NO_WEDGE");
  k.no_wbm_batch = on("BLP_NO_WBM_BATCH");
  k.group_buckets = on("BLP_GROUP_BUCKETS");
  k.no_hash = on("BLP_NO_HASH");
  k.hash_big = on("BLP_HASH_BIG");
  k.hash_work = num("BLP_HASH_WORK", -1);
  k.no_wcodes = on("BLP_NO_WCODES");
  k.split_nopk = on("BLP_SPLIT_NOPK");
  k.no_ydirect = on("BLP_NO_YDIRECT");
  k.no_run_fast = on("BLP_NO_RUN_FAST");
  k.split_short = (int)num("BLP_SPLIT_SHORT", -1);
  k.cosched_cus = (int)num("BLP_COSCHED_CUS", -1);
  k.no_pko = on("BLP_NO_PKO");
  k.item_nb = (int)num("BLP_ITEM_NB", 512);
  k.group_nblk = (int)num("BLP_GROUP_NBLK", -1);
  k.lpt = (int)num("BLP_LPT", 1);
  k.short_cus = (int)num("BLP_SHORT_CUS", -1);
#ifdef BLP_DEBUG
  if (const char* e = getenv("BLP_DEBUG_NULL")) k.debug_null = e;
  k.debug_oom = on("BLP_DEBUG_OOM");
#endif
  return k;
}
}  // namespace

struct blp_batch {
  bool hi_prio = false;  // its stream came from the highest-priority pool (stream_give returns it there)
  blp_graph* g = nullptr;
  int64_t n_pairs = 0;
  int32_t* d_x = nullptr;
  int32_t* d_y = nullptr;
  uint32_t* d_cn = nullptr;
  double* d_jac = nullptr;
  double* d_aa = nullptr;
  int32_t* d_gout = nullptr;
  int64_t* d_gyb = nullptr;
  int32_t* d_gyl = nullptr;
  Misc* d_misc = nullptr;
  // heavy sources (planned at create)
  int32_t* d_heavy_slot = nullptr;
  uint32_t* d_heavy_bm = nullptr;
  const int32_t* wbm_slot = nullptr;  // the graph's wedge-row bitmaps over [lo, hi) (or null):
  const uint32_t* wbm_pool = nullptr; // used as pre-built bitmaps in place of k_heavy's
  HeavyItem* d_heavy_items = nullptr;
  int64_t n_heavy = 0, n_heavy_items = 0, hb_words = 0;
  int64_t lo = 0, hi = 0;
  int variant = V_SMALL;
  int chunks = 1;
  int dq = 1;
  bool use_hot = false;  // some source has a dense row in N(x)
  int short_rows = 0;    // ScoreArgs::short_rows
  bool global = false;   // HBM-bitmap scorer (universe wider than LDS)
  bool pko = false;      // the large scorer's packed-count variant (k_score PKO) takes this batch
  int split = 0;         // chunk-parallel scorer: universe cut into `split` LDS chunks, 2 workgroups / CU
  bool split_big = false;  // ... 128 KiB chunks, one workgroup per CU
  int64_t rs_lo = 0;     // first node of the split table
  int64_t rs_rows = 0;   // its rows
  int32_t* d_gy = nullptr;     // grouped position -> y (split mode)
  int32_t* d_rsplit = nullptr; // [n][split + 1] row offsets where neighbour ids cross chunk boundaries
  int4* d_lq = nullptr;        // k_score_split's long-slice queues (SPLIT_LQ per resident workgroup)
  uint32_t* d_pcn = nullptr;   // [n_pairs] counts, summed over chunks (zeroed per score)
  unsigned long long* d_paa = nullptr;  // [2][n_pairs] exact AA words (low words, then high), summed over chunks
  unsigned long long* d_aa_part = nullptr;  // [n_pairs][2] exact AA words between LDS chunks (chunks > 1)
  uint32_t* d_ph2 = nullptr;   // [n][split] partial |H2|
  uint32_t* d_gbm = nullptr;
  int64_t gwords = 0, gslots = 0;
  int shift = 10, nb = 1, nblk = 1;
  int32_t xlo = 0;
  int64_t xspan = 0;
  int64_t per_blk = 1;
  int64_t cap_bits = 0;
  int64_t n_sources = 0;
  bool runs = false;  // pairs arrive grouped by source (x non-decreasing): run-head grouping
  bool items = false;  // item grouping (interleaved buckets cut into GI_PAIRS items); else k_bucket_group
  blp::KernelTimer t_score, t_group;
  // the batch's own stream and grouping scratch: batches of one graph (the user and the
  // business pass of similarity.main) run concurrently, one filling the other's tail
  hipStream_t stream = nullptr;
  blp::DevBuf cnt, off, active, scratch;
  int cus = 0;  // CUs the persistent block scorer may occupy (0: all; set by blp_batches_score)
  SrcRec* d_rec = nullptr;  // [n_sources] source records of the short-row scorer (or null)
  uint8_t* d_hflag = nullptr;  // [xspan] 1: source scored by k_score_hash (split batches; or null)
  int32_t* d_active2 = nullptr;  // the active list partitioned by k_hash_partition (with d_hflag)
  int32_t* d_rank = nullptr;     // [xspan] BLP_LPT: the source's place in the largest-first order (or null)
  int32_t* d_lpt = nullptr;      // [n_sources] the active list in that order, written by k_run_cnt
  int64_t n_hash = 0;          // such sources
  bool use_short = false;   // the short-row scorer takes this batch (decided once, at create)
  // the graph's dense wedge-set index (k_score_wset; or null): a bipartite business-side batch
  // scored pair by pair in caller order -- no grouping, no per-source bitmap build
  const uint32_t* wset_pool = nullptr;
  const int32_t* wset_h2 = nullptr;
  int64_t wset_lo = 0, wset_span = 0, wset_words = 0;
  bool wedge_user = false;  // its plan reads the graph's wedge index (counted in g->wedge_users)
  int64_t work_elems = 0;  // planned build + scan elements (co-scheduling estimate)
  Knobs kn;               // environment switches, read once at create
};

using namespace blp;

// the short-row scorer (k_score<..., SHORT = true>) takes the batch
static bool short_kernel(const blp_batch* b) {
  return b->variant == V_SMALL && b->short_rows == 3 && !b->global && !b->split && !b->kn.no_short_kernel;
}

template <int BLOCK, int CAP, int SEG>
static int score_occupancy(int* per_cu) {
  BLP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, k_score<BLOCK, CAP, SEG, 8>, BLOCK, 0));
  *per_cu = std::max(*per_cu, 1);
  return BLP_OK;
}

static int variant_occupancy(int v, int* per_cu) {
  if (v == V_SMALL) return score_occupancy<BLOCK_SMALL, CAP_SMALL, SEG_SMALL>(per_cu);
  if (v == V_MED) return score_occupancy<BLOCK_MED, CAP_MED, SEG_MED>(per_cu);
  return score_occupancy<BLOCK_LARGE, CAP_LARGE, SEG_LARGE>(per_cu);
}

template <int BLOCK, int CAP, int SEG, bool SAA = true, bool PKO = false>
static int launch_score(blp_graph* g, hipStream_t st, const ScoreArgs& a, int per_cu, int cus) {
  if (cus <= 0 || cus > g->n_cu) cus = g->n_cu;
  const dim3 grid(cus * per_cu), block(BLOCK);
  hipLaunchKernelGGL((k_score<BLOCK, CAP, SEG, 8, false, SAA, PKO>), grid, block, 0, st, a);
  BLP_HIP(hipGetLastError());
  return BLP_OK;
}

// Short-row scorer (every build and scan row <= SHORT_MAX ids), SAA: Adamic-Adar compiled in.
// Many light sources per workgroup: at least two per dequeue, so the one queue head is not the
// limit (one device-scope atomic word saturates near 90 dequeues per microsecond).
template <bool SAA>
static int launch_short(blp_graph* g, const blp_batch* b, ScoreArgs a, size_t dyn) {
  // the three-barrier scorer takes batches with wedge rows (every review-graph business pass);
  // the segment scorer builds from the CSR otherwise
  const bool three = a.wp != nullptr;
  auto kern = three ? k_score_short<SAA> : k_score<BLOCK_SMALL, CAP_SMALL, SEG_SMALL, 8, true, SAA>;
  int per_cu = 1;
  BLP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, BLOCK_SMALL, dyn));
  const int cus = b->kn.short_cus > 0 ? std::min(b->kn.short_cus, g->n_cu) : g->n_cu;  // tuning knob
  const int64_t n_wg = (int64_t)cus * std::max(per_cu, 1);
  if (b->n_sources >= n_wg * 16) a.dq = std::max(a.dq, 2);
  hipLaunchKernelGGL(kern, dim3((unsigned)n_wg), dim3(BLOCK_SMALL), dyn, b->stream, a);
  BLP_HIP(hipGetLastError());
  return BLP_OK;
}

template <int BLOCK, int CAP, int SEG>
static int launch_heavy(hipStream_t st, const HeavyArgs& h, int64_t n_items) {
  hipLaunchKernelGGL((k_heavy<BLOCK, CAP, SEG>), dim3((unsigned)n_items), dim3(BLOCK), 0, st, h);
  BLP_HIP(hipGetLastError());
  return BLP_OK;
}

// Every device pointer the chosen launch path dereferences, checked on the host before anything is
// enqueued: a null base pointer is not an index, so the kernels' PS_OK bound checks cannot see it,
// and a kernel writing through one faults the GPU (round 4: k_score_split's long-slice queue). The
// scorer arguments are gathered into `a` first, so this sees exactly what the kernels will read.
static int launch_pointers(const blp_graph* g, const blp_batch* b, ScoreArgs& a, uint32_t mask) {
#ifdef BLP_DEBUG
  if (!b->kn.debug_null.empty()) {  // test knob: null one pointer to show the check refusing it
    const std::string& f = b->kn.debug_null;
    if (f == "g_yb") a.g_yb = nullptr;
    if (f == "cn") a.cn = nullptr;
    if (f == "lq") a.lq = nullptr;
    if (f == "wedge") a.wedge = nullptr;
  }
#endif
  const char* missing = nullptr;
  auto need = [&](const void* p, const char* what) {
    if (!p && !missing) missing = what;
  };
  need(a.rp, "row_ptr");
  need(a.ci, "col_idx");
  need(a.cw, "coded col_idx");
  need(a.off, "source offsets");
  need(a.cnt, "source counts");
  need(a.active, "active sources");
  if (!b->runs) need(a.g_out, "grouped caller index");
  if (!a.py) {
    need(a.g_yb, "grouped row starts");
    need(a.g_yl, "grouped row lengths");
  }
  need(a.misc, "batch counters");
  need(a.cn, "cn output");
  need(a.jac, "jaccard output");
  need(a.aa, "adamic output");
  if (mask & BLP_ADAMIC) need(a.aaw, "aa weights");
  if (a.hot_idx) {
    need(a.hot_tab, "dense-row table");
    need(a.hot_pool, "dense-row pool");
  }
  if (a.heavy_slot) need(a.heavy_bm, "pre-built bitmaps");
  if ((a.wp != nullptr) != (a.wedge != nullptr)) missing = missing ? missing : "wedge rows (offsets without ids)";
  if (b->chunks > 1 && (mask & BLP_ADAMIC)) need(a.aa_part, "chunk AA partials");
  if (b->n_heavy) {
    need(b->d_heavy_bm, "heavy bitmaps");
    need(b->d_heavy_items, "heavy items");
  }
  if (b->split) {
    need(a.lq, "long-slice queues");
    need(b->d_gy, "grouped y");
    need(b->d_rsplit, "row split table");
    need(b->d_pcn, "chunk counts");
    need(b->d_ph2, "chunk |H2| partials");
    if (mask & BLP_ADAMIC) need(b->d_paa, "chunk AA words");
    if (b->d_hflag) need(b->d_active2, "partitioned active list");
  }
  if (b->global) need(b->d_gbm, "HBM bitmap slots");
  if ((b->use_short || (b->variant == V_LARGE && !b->split && !b->global)) && b->n_sources) need(b->d_rec, "source records");
  if (!missing) return BLP_OK;
  char msg[160];
  snprintf(msg, sizeof msg, "blp_batch_score: the launch path reads a null device pointer (%s)", missing);
  (void)g;
  return fail(BLP_E_STATE, msg);
}

extern "C" {

}  // extern "C"

// blp_batch_create, and blp_batch_create_pair's second batch: `twin` (or null) is a batch of the
// same pairs with x and y swapped whose device copies are taken (a device-to-device copy after the
// twin's upload, on this batch's stream) instead of a second host-to-device upload.
static int batch_create(blp_graph* g, const int32_t* x, const int32_t* y, int64_t n_pairs, const blp_batch* twin,
                        blp_batch** out, bool retry = false, bool hi_prio = false) {
  BLP_CHECK(g && out && n_pairs >= 0 && (n_pairs == 0 || (x && y)), BLP_E_ARG, "blp_batch_create: bad arguments");
  BLP_CHECK(n_pairs < (int64_t(1) << 31) - 1, BLP_E_ARG, "blp_batch_create: at most 2^31-2 pairs per batch");
  const int64_t n = g->n;
  // BLP_CREATE_PROF=1: the planning stages' wall times on stderr (the e2e score phase)
  const bool cprof = getenv("BLP_CREATE_PROF") != nullptr;
  auto ct0 = std::chrono::steady_clock::now();
  auto stage = [&](const char* what) {
    if (!cprof) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "[blp_batch_create %lld pairs] %-10s %.2f ms\n", (long long)n_pairs, what,
            std::chrono::duration<double, std::milli>(t - ct0).count());
    ct0 = t;
  };
  const Knobs kn = read_knobs();
  blp_batch* b = new blp_batch();
  b->g = g;
  // the batch's timers count into the graph's score / group totals (blp_stats_get)
  b->t_score.mirror = &g->timers[K_SCORE];
  b->t_group.mirror = &g->timers[K_GROUP];
  b->t_score.mirror_mu = b->t_group.mirror_mu = &g->timer_mu;
  {
    std::lock_guard<std::mutex> lk(g->timer_mu);
    g->live_timers.push_back(&b->t_score);
    g->live_timers.push_back(&b->t_group);
  }
  b->n_pairs = n_pairs;
  b->kn = kn;
  auto bail = [&](int rc) {
    blp_batch_destroy(b);
    return rc;
  };
  {  // registered as a reader of the wedge index before planning reads it (d_wp, h_wp, the
     // bitmaps): an out-of-memory retry of a concurrent create cannot free it under this plan
    std::lock_guard<std::mutex> lk(g->wbm_mu);
    if (g->d_wp) {
      ++g->wedge_users;
      b->wedge_user = true;
    }
  }
  int rc = set_device(g);
  if (rc) return bail(rc);
  b->hi_prio = hi_prio;
  if (!(b->stream = stream_take(g->device, hi_prio))) return bail(BLP_E_HIP_BASE);  // pooled (blp_stream_prewarm)
  // ---- the pairs go to HBM first: the device planning pass reads them there
  const size_t np = (size_t)std::max<int64_t>(n_pairs, 1);
  if (dev_malloc(&b->d_x, 4 * np) != hipSuccess || dev_malloc(&b->d_y, 4 * np) != hipSuccess ||
      dev_malloc(&b->d_misc, sizeof(Misc)) != hipSuccess)
    return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create: hipMalloc failed"));
  if (n_pairs && twin) {  // the twin's device copies, swapped, once its upload is done
    hipEvent_t ev;
    BLP_HIP_OR(hipEventCreateWithFlags(&ev, hipEventDisableTiming), bail);
    hipError_t e = hipEventRecord(ev, twin->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(b->stream, ev, 0);
    (void)hipEventDestroy(ev);
    BLP_HIP_OR(e, bail);
    BLP_HIP_OR(hipMemcpyAsync(b->d_x, twin->d_y, 4 * n_pairs, hipMemcpyDeviceToDevice, b->stream), bail);
    BLP_HIP_OR(hipMemcpyAsync(b->d_y, twin->d_x, 4 * n_pairs, hipMemcpyDeviceToDevice, b->stream), bail);
  } else if (n_pairs) {
    if ((rc = copy_sync(b->d_x, x, 4 * n_pairs, hipMemcpyHostToDevice, b->stream)) ||
        (rc = copy_sync(b->d_y, y, 4 * n_pairs, hipMemcpyHostToDevice, b->stream)))
      return bail(rc);
  }
  BLP_HIP_OR(hipMemsetAsync(b->d_misc, 0, sizeof(Misc), b->stream), bail);  // dbg[] is zeroed here, not per score
  {  // the graph's own device work completes before this stream reads the graph (an event, not a
     // host wait), queued after the pair upload: the upload's host syncs then do not wait for the
     // graph build's last kernels
    hipEvent_t ev;
    BLP_HIP_OR(hipEventCreateWithFlags(&ev, hipEventDisableTiming), bail);
    hipError_t e = hipEventRecord(ev, g->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(b->stream, ev, 0);
    (void)hipEventDestroy(ev);
    BLP_HIP_OR(e, bail);
  }
  stage("upload");
  // ---- plan: node universe touched by H2(x) and N(y); per-source build work
  int64_t lo = INT64_MAX, hi = INT64_MIN, scan_work = 0, max_scan_row = 0, max_build_row = 0;
  int64_t rows_lo = INT64_MAX, rows_hi = INT64_MIN, build_work = 0, n_sources = 0;
  int32_t xlo = INT32_MAX, xhi = 0;
  bool bad = false, in_runs = true, any_hot = false;
  std::vector<std::pair<int32_t, int64_t>> heavy_cand;  // sources whose build work may make them heavy
  constexpr int64_t HEAVY_MIN = 2 * 16384;              // 2 * the smallest item_work below
  ScopedBuf d_seen, d_srcs, d_stats, d_heavy;
  // planned on the device from the graph's two-hop statistics (graph_finish always builds them)
  if (n_pairs > 0 && !g->d_w2) return bail(fail(BLP_E_STATE, "blp_batch_create: the graph has no two-hop statistics"));
  const bool dev_plan = n_pairs > 0;
  if (dev_plan) {
    // one pass over the pairs on the device (k_plan_pairs); the host only reads the totals
    const int64_t seen_words = (n + 31) / 32;
    if ((rc = d_seen.reserve(4 * (size_t)seen_words)) || (rc = d_srcs.reserve(4 * (size_t)std::min<int64_t>(n, n_pairs))) ||
        (rc = d_stats.reserve(sizeof(PlanStats) + 64)))
      return bail(rc);
    PlanStats init{};
    init.lo = init.rows_lo = init.xlo = ~0ull;
    BLP_HIP_OR(hipMemsetAsync(d_seen.p, 0, 4 * (size_t)seen_words, b->stream), bail);
    BLP_HIP_OR(hipMemcpyAsync(d_stats.p, &init, sizeof init, hipMemcpyHostToDevice, b->stream), bail);
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>((int64_t)g->n_cu * 8, (n_pairs + PLAN_BLOCK - 1) / PLAN_BLOCK));
    hipLaunchKernelGGL(k_plan_pairs, dim3((unsigned)grid), dim3(PLAN_BLOCK), 0, b->stream, b->d_x, b->d_y, n_pairs, n,
                       g->d_rp, g->d_ci, g->d_w2, g->d_lo2, g->d_hi2, g->d_maxd, g->d_flag2, d_seen.as<uint32_t>(),
                       d_srcs.as<int32_t>(), d_stats.as<PlanStats>());
    BLP_HIP_OR(hipGetLastError(), bail);
    PlanStats ps;
    BLP_HIP_OR(hipMemcpyAsync(&ps, d_stats.p, sizeof ps, hipMemcpyDeviceToHost, b->stream), bail);
    BLP_HIP_OR(hipStreamSynchronize(b->stream), bail);
    bad = ps.bad != 0;
    if (bad) return bail(fail(BLP_E_ARG, "blp_batch_create: node id out of range"));
    in_runs = ps.not_runs == 0;
    any_hot = ps.any_hot != 0;
    scan_work = (int64_t)ps.scan;
    max_scan_row = (int64_t)ps.max_scan;
    max_build_row = (int64_t)ps.max_build;
    build_work = (int64_t)ps.work;
    n_sources = (int64_t)ps.n_sources;
    if (ps.hi > 0) {
      lo = (int64_t)ps.lo;
      hi = (int64_t)ps.hi;
    }
    if (ps.rows_hi > 0) {
      rows_lo = (int64_t)ps.rows_lo;
      rows_hi = (int64_t)ps.rows_hi;
    }
    if (ps.xhi > 0) {
      xlo = (int32_t)ps.xlo;
      xhi = (int32_t)ps.xhi;
    }
  }
  stage("plan");
  if (n_sources == 0) xlo = xhi = 0;
  bool runs = in_runs && !kn.no_runs;  // x non-decreasing: grouped by run heads (BLP_NO_RUNS: bucket sort)
  if (lo > hi) lo = hi = 0;
  const int64_t lo_raw = lo;  // the universe's first id (the wedge-set range starts there, unaligned)
  lo &= ~int64_t(127);  // 128-bit aligned so dense rows map onto whole 16-byte LDS vectors
  b->runs = runs;
  b->lo = lo;
  b->hi = hi;
  b->n_sources = n_sources;
  b->use_hot = any_hot;
  if (!kn.no_short)  // test knob
    b->short_rows = (max_build_row <= SHORT_MAX ? 1 : 0) | (max_scan_row <= SHORT_MAX ? 2 : 0);
  const int64_t span = hi - lo;
  if (span <= variant_cap_bits(V_SMALL))
    b->variant = V_SMALL;
  else if (span <= variant_cap_bits(V_MED))
    b->variant = V_MED;
  else
    b->variant = V_LARGE;
  if (kn.variant > b->variant && kn.variant <= V_LARGE) b->variant = kn.variant;  // test knob: a wider LDS variant
  b->cap_bits = variant_cap_bits(b->variant);
  if (kn.chunk_bits >= 128 && kn.chunk_bits % 128 == 0 && kn.chunk_bits < b->cap_bits)  // test knob: multi-chunk
    b->cap_bits = kn.chunk_bits;
  b->chunks = span <= b->cap_bits ? 1 : (int)((span + b->cap_bits - 1) / b->cap_bits);
  // wider than one LDS bitmap, up to eight 512K-bit chunks: chunk-parallel scorer, (source,
  // chunk) items on 64 KiB bitmaps, two workgroups per CU -- 5.7x the HBM-bitmap scorer on
  // the 2M-user universe of config 4 (BLP_NO_SPLIT: off; BLP_SPLIT=C: force C chunks)
  {
    // 128 KiB chunks, one workgroup per CU, row-chunk loops: a (pair, chunk) slice's fixed cost
    // -- its metadata, row-split lookups and exscan -- dominates the chunk-parallel scorer (5 ids
    // per slice at config 5), and halving the slices beats a second workgroup per CU. Config 5:
    // 1.77 s per step with 64 KiB chunks on both sides, 1.07 s with 128 KiB chunks (both
    // sides). BLP_SPLIT_BIG=0 keeps 64 KiB chunks, two workgroups per CU.
    b->split_big = true;
    if (kn.split_big >= 0) b->split_big = kn.split_big > 0;  // test knob
    const int64_t sbits = 32ll * (b->split_big ? S_CAP_BIG : S_CAP);
    int C = 0;
    if (kn.split >= 0)
      C = std::max(0, std::min(S_MAX_CHUNKS, kn.split));
    else if (span > variant_cap_bits(V_LARGE) && span <= S_MAX_CHUNKS * sbits && !kn.no_split)
      C = (int)((span + sbits - 1) / sbits);
    if (C >= 2 && span > 0) {
      b->split = C;
      b->cap_bits = ((span + C - 1) / C + 127) / 128 * 128;
      b->chunks = 1;
      b->variant = V_LARGE;  // k_heavy's LDS capacity
    }
  }
  // wider than LDS: one HBM bitmap per workgroup instead of an H2 rebuild per LDS chunk
  // (BLP_NO_GLOBAL keeps the chunked path, BLP_FORCE_GLOBAL selects HBM on any universe)
  b->global = !b->split && ((b->chunks > 1 && !kn.no_global) || kn.force_global);
  if (b->global) b->chunks = 1;
  // the large scorer's packed-count variant: one chunk of <= 32 * CAP_PKO nodes, and scan rows not
  // all short (those take row_scan, which counts per pair)
  b->pko = b->variant == V_LARGE && !b->split && !b->global && b->chunks == 1 && span <= 32ll * CAP_PKO &&
           !(b->short_rows & 2) && !kn.no_pko;
  int per_cu = 1;
  if (b->split) {
    BLP_HIP_OR(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_score_split<S_BLOCK, S_CAP, S_SEG, 8>,
                                                            S_BLOCK, 0), bail);
  } else if ((rc = variant_occupancy(b->variant, &per_cu))) {
    return bail(rc);
  }
  const int64_t n_wg = (int64_t)g->n_cu * per_cu;
  // sources per dequeue: the active list is in id order, which need not be balanced; keep it 1
  // unless there are very many light sources per worker
  // (two once a worker has ~64+ sources: the business side of config 2, 1.44 -> 1.30 ms)
  b->dq = b->n_sources >= n_wg * 64 ? (int)std::max<int64_t>(2, std::min<int64_t>(DQ_MAX, b->n_sources / (n_wg * 64))) : 1;
  // ---- hash-set scorer (split batches): sources whose build work fits half the hash table
  // work bounds the distinct ids inserted; at most HT - 1 keeps an empty slot, so every insert
  // and probe chain ends (the knob is clamped: a fuller table is slower, never unbounded)
  const bool want_hash = b->split && n_pairs && !kn.no_hash;
  const int64_t hs_ht = kn.hash_big ? HS_HT_BIG : HS_HT;
  const int64_t hash_want = kn.hash_work >= 0 ? kn.hash_work : hs_ht / 2;
#ifdef BLP_DEBUG
  // debug builds take the knob unclamped, so a test can overfill the table and see the probe
  // bound (PS_OK site 8) report it instead of a spin
  const int64_t hash_cap = kn.hash_work >= 0 ? kn.hash_work : std::min<int64_t>(std::max<int64_t>(1, hash_want), hs_ht - 1);
#else
  const int64_t hash_cap = std::min<int64_t>(std::max<int64_t>(1, hash_want), hs_ht - 1);
#endif
  b->xlo = xlo;
  b->xspan = (int64_t)xhi - xlo;
  if (dev_plan) {
    // the heavy candidates' ids, and (split batches) the hash-set flags, from the device source list
    const int64_t cap_heavy = std::max<int64_t>(1, std::min<int64_t>(n_sources, build_work / HEAVY_MIN + 1));
    if ((rc = d_heavy.reserve(4 * (size_t)cap_heavy + 64))) return bail(rc);
    uint32_t* counts = reinterpret_cast<uint32_t*>(d_heavy.as<int32_t>() + cap_heavy);  // [n_heavy, n_hash]
    BLP_HIP_OR(hipMemsetAsync(counts, 0, 8, b->stream), bail);
    if (want_hash) {
      if (dev_malloc(&b->d_hflag, (size_t)std::max<int64_t>(b->xspan, 1)) != hipSuccess)
        return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create: hash flags"));
      BLP_HIP_OR(hipMemsetAsync(b->d_hflag, 0, (size_t)std::max<int64_t>(b->xspan, 1), b->stream), bail);
    }
    hipLaunchKernelGGL(k_plan_sources, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)g->n_cu * 4, (n_sources + 255) / 256))),
                       dim3(256), 0, b->stream, d_srcs.as<int32_t>(), n_sources, g->d_w2, g->d_rp,
                       (unsigned long long)HEAVY_MIN, d_heavy.as<int32_t>(), counts, (unsigned)cap_heavy, b->d_hflag,
                       (int64_t)xlo, (unsigned long long)hash_cap, counts + 1);
    BLP_HIP_OR(hipGetLastError(), bail);
    uint32_t hc[2];
    BLP_HIP_OR(hipMemcpyAsync(hc, counts, 8, hipMemcpyDeviceToHost, b->stream), bail);
    BLP_HIP_OR(hipStreamSynchronize(b->stream), bail);
    if ((int64_t)hc[0] > cap_heavy) return bail(fail(BLP_E_STATE, "blp_batch_create: heavy candidate list overflow"));
    std::vector<int32_t> hv(hc[0]);
    if (hc[0]) BLP_HIP_OR(hipMemcpy(hv.data(), d_heavy.p, 4 * (size_t)hc[0], hipMemcpyDeviceToHost), bail);
    std::sort(hv.begin(), hv.end());  // id order: the slots do not depend on the atomics' order
    for (int32_t v : hv) heavy_cand.emplace_back(v, (int64_t)g->h_w2[v]);
    b->n_hash = want_hash ? (int64_t)hc[1] : 0;
    if (want_hash && !b->n_hash) {
      (void)hipFree(b->d_hflag);
      b->d_hflag = nullptr;
    }
  }
  if (b->n_hash && dev_malloc(&b->d_active2, 4 * ((size_t)std::max<int64_t>(b->xspan, 1) + 1)) != hipSuccess)
    return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create: hash flags"));
  if (dev_plan && n_sources > 1 && ((runs && (kn.lpt & 1)) || (!runs && !kn.group_buckets && (kn.lpt & 2)))) {
    // BLP_LPT: the sources' queue order, largest estimated work (build w2[x] + scan sum |N(y)|) first
    ScopedBuf d_est, d_out, d_r;
    if ((rc = d_est.reserve(8 * (size_t)std::max<int64_t>(b->xspan, 1))) || (rc = d_out.reserve(8 * (size_t)n_sources)) ||
        (rc = d_r.reserve(4 * (size_t)n_sources)))
      return bail(rc);
    if (dev_malloc(&b->d_rank, 4 * (size_t)std::max<int64_t>(b->xspan, 1)) != hipSuccess ||
        dev_malloc(&b->d_lpt, 4 * (size_t)n_sources + 4) != hipSuccess)
      return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create: source order"));
    BLP_HIP_OR(hipMemsetAsync(d_est.p, 0, 8 * (size_t)std::max<int64_t>(b->xspan, 1), b->stream), bail);
    const unsigned gp = (unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)g->n_cu * 8, (n_pairs + 255) / 256));
    hipLaunchKernelGGL(k_src_scan_work, dim3(gp), dim3(256), 0, b->stream, b->d_x, b->d_y, n_pairs, g->d_rp, (int32_t)xlo,
                       d_est.as<unsigned long long>());
    const unsigned gs = (unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)g->n_cu * 4, (n_sources + 255) / 256));
    hipLaunchKernelGGL(k_src_est, dim3(gs), dim3(256), 0, b->stream, d_srcs.as<int32_t>(), n_sources,
                       d_est.as<unsigned long long>(), reinterpret_cast<const unsigned long long*>(g->d_w2), (int32_t)xlo,
                       d_out.as<unsigned long long>());
    BLP_HIP_OR(hipGetLastError(), bail);
    // the order on the device (a stable radix sort), then rank[x - xlo] = place of x in it
    if ((rc = order_desc_u64(d_out.as<uint64_t>(), n_sources, d_r.as<int32_t>(), b->stream))) return bail(rc);
    hipLaunchKernelGGL(k_src_rank, dim3(gs), dim3(256), 0, b->stream, d_srcs.as<int32_t>(), n_sources, d_r.as<int32_t>(),
                       (int32_t)xlo, b->d_rank);
    BLP_HIP_OR(hipGetLastError(), bail);
    BLP_HIP_OR(hipStreamSynchronize(b->stream), bail);  // the scoped buffers go after this
  }
  stage("sources");
  // ---- heavy sources: build work far above the per-workgroup share goes to k_heavy
  const int64_t total_work = build_work + scan_work;
  b->work_elems = total_work;
  int64_t item_work = std::max<int64_t>(16384, total_work / std::max<int64_t>(4 * n_wg, 1));
  if (kn.heavy_work >= 0) item_work = std::max<int64_t>(1, kn.heavy_work);  // test knob
  if (kn.heavy_work >= 0 && 2 * item_work < HEAVY_MIN) {
    // test knob below the candidate bound: every source is a candidate (host planning's lists)
    heavy_cand.clear();
    if (dev_plan) {
      std::vector<int32_t> all((size_t)n_sources);
      if (n_sources) BLP_HIP_OR(hipMemcpy(all.data(), d_srcs.p, 4 * (size_t)n_sources, hipMemcpyDeviceToHost), bail);
      std::sort(all.begin(), all.end());
      for (int32_t v : all) heavy_cand.emplace_back(v, g->hrp[v + 1] > g->hrp[v] ? (int64_t)g->h_w2[v] : 0);
    }
  }
  std::vector<int32_t> heavy_slot;
  std::vector<int32_t> heavy_src;  // sources given a slot
  std::vector<HeavyItem> items;
  // every source's rows are short and the graph holds wedge rows: heavy sources are split into
  // slices of their wedge rows (the short-row scorer's layout)
  const bool wedge_items = (b->short_rows & 1) && g->d_wp && !kn.no_wedge;
  if (b->chunks == 1 && span > 0 && !b->global && (!b->split || span <= variant_cap_bits(V_LARGE))) {
    const int64_t* rp = g->hrp;
    // CSR items walk N(x) on the host: the column mirror only when some candidate IS heavy (its
    // fetch is ~80 MB at config 2, where the user side's candidates stay below the bound)
    bool csr_items = false;
    for (const auto& hc : heavy_cand) csr_items |= !wedge_items && hc.second > 2 * item_work;
    const int32_t* ci = csr_items ? host_col_idx(g) : g->hci;
    if (csr_items && !ci) return bail(BLP_E_STATE);
    for (const auto& hc : heavy_cand) {
      if (hc.second <= 2 * item_work) continue;
      if (heavy_slot.empty()) heavy_slot.assign((size_t)n, -1);
      const int32_t xs = hc.first;
      const int32_t slot = (int32_t)b->n_heavy++;
      heavy_slot[xs] = slot;
      heavy_src.push_back(xs);
      if (wedge_items) {  // slices of x's wedge row, item_work ids each
        const int64_t wb = g->h_wp[xs], we = g->h_wp[xs + 1], step = std::max<int64_t>(1, item_work / 4);
        for (int64_t q = wb; q < we; q += step) items.push_back(HeavyItem{slot, 1, q, std::min(we, q + step)});
        continue;
      }
      int64_t acc = 0, kb = rp[xs];
      for (int64_t k = rp[xs]; k < rp[xs + 1]; ++k) {
        acc += rp[ci[k] + 1] - rp[ci[k]];
        if (acc >= item_work || k + 1 == rp[xs + 1]) {
          items.push_back(HeavyItem{slot, 0, kb, k + 1});
          kb = k + 1;
          acc = 0;
        }
      }
    }
  }
  b->n_heavy_items = (int64_t)items.size();
  b->hb_words = ((span + 31) / 32 + 3) / 4 * 4;
  stage("heavy");
  // ---- the graph's wedge-row bitmaps (hop3.hip) over this universe: a source whose wedge row is
  // at least as long as its bitmap's words copies the bitmap (its id set, 12.5 KB at config 2)
  // instead of OR-ing the row id by id -- the same slots and copy as k_heavy's pre-built bitmaps,
  // so those sources need no per-step k_heavy either (BLP_NO_WBM_BATCH=1: off)
  if (wedge_items && b->chunks == 1 && span > 0 && !b->global && !b->split && !b->kn.no_wbm_batch) {
    int rcw = BLP_OK;
    const WedgeBitmaps* w = wedge_bitmaps(g, lo, hi, &rcw);
    if (rcw) return bail(rcw);
    if (w && w->slots && w->words == b->hb_words) {
      bool covered = true;  // every planned heavy source has a bitmap (the longest rows do)
      for (size_t i = 0; i < heavy_src.size() && covered; ++i) covered = w->h_slot[heavy_src[i]] >= 0;
      if (covered) {
        b->wbm_slot = w->d_slot;
        b->wbm_pool = w->d_pool;
        b->n_heavy = 0;
        b->n_heavy_items = 0;
        items.clear();
        heavy_slot.clear();
      }
    }
  }
  stage("wbm");
  // ---- grouping geometry: buckets of 2^shift node ids, at most NB_MAX buckets
  {
    // buckets cover the sources' id range [xlo, xhi): ~2K buckets of 2^shift ids each
    b->items = !kn.group_buckets;  // test knob: one workgroup per contiguous bucket
    if (b->items) {
      // nb = 2^shift interleaved buckets, each with ceil(xspan / nb) keys: kn.item_nb of them, or
      // more (<= 2048) when that keeps a bucket's keys <= 1024 (the staged write, k_item_write_ids)
      b->shift = 0;
      int64_t nb_cap = std::max(1, std::min(kn.item_nb, 2048));
      while (nb_cap < 2048 && (b->xspan + nb_cap - 1) / nb_cap > 1024) nb_cap *= 2;
      while ((int64_t(1) << b->shift) < std::min<int64_t>(b->xspan, nb_cap)) ++b->shift;
      b->nb = 1 << b->shift;
      if (((b->xspan + b->nb - 1) >> b->shift) > 32768)
        return bail(fail(BLP_E_UNSUP, "blp_batch_create: source id range too wide"));
    } else {
      b->shift = 0;
      while ((b->xspan >> b->shift) > 2048) ++b->shift;
      b->nb = (int)std::max<int64_t>(1, (b->xspan + (int64_t(1) << b->shift) - 1) >> b->shift);
      if (b->shift > 15 || b->nb > NB_MAX) return bail(fail(BLP_E_UNSUP, "blp_batch_create: source id range too wide"));
    }
    b->nblk = (int)std::max<int64_t>(1, std::min<int64_t>(kn.group_nblk > 0 ? kn.group_nblk : (int64_t)g->n_cu * 2,
                                                          (n_pairs + 4095) / 4096));
    b->per_blk = (n_pairs + b->nblk - 1) / b->nblk;
  }
  // ---- chunk-parallel scorer: per-row chunk offsets and partial-result buffers
  if (b->split && n_pairs) {
    const int C = b->split;
    b->rs_lo = rows_lo;
    const int64_t nrows = std::max<int64_t>(rows_hi - rows_lo, 1);
    b->rs_rows = nrows;
    if (dev_malloc(&b->d_gy, 4 * (size_t)n_pairs) != hipSuccess ||
        dev_malloc(&b->d_rsplit, 4 * (size_t)nrows * (C + 1)) != hipSuccess ||
        dev_malloc(&b->d_pcn, 4 * (size_t)n_pairs) != hipSuccess ||
        dev_malloc(&b->d_paa, 16 * (size_t)n_pairs) != hipSuccess ||
        dev_malloc(&b->d_ph2, 4 * (size_t)std::max<int64_t>(b->n_sources, 1) * C) != hipSuccess ||
        dev_malloc(&b->d_lq, sizeof(int4) * SPLIT_LQ * (size_t)g->n_cu * 2) != hipSuccess)
      return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create: split buffers"));
    // on the batch's stream: ordered before its scoring, no host wait
    hipLaunchKernelGGL(k_row_splits, dim3(2048), dim3(256), 0, b->stream, g->d_rp, g->d_ci, rows_lo, nrows, b->lo,
                       b->cap_bits, C, b->d_rsplit);
    BLP_HIP_OR(hipGetLastError(), bail);
  }
  // ---- HBM bitmap slots: one per resident workgroup of k_score_global
  if (b->global && n_pairs) {
    int per_cu_g = 1;
    BLP_HIP_OR(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_g, k_score_global<G_BLOCK, G_SEG, 8>, G_BLOCK, 0),
               bail);
    b->gslots = (int64_t)g->n_cu * std::max(per_cu_g, 1);
    b->gwords = ((span + 31) / 32 + 3) / 4 * 4;
    if (dev_malloc(&b->d_gbm, 4 * (size_t)b->gwords * b->gslots) != hipSuccess)
      return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create: HBM bitmap slots"));
  }
  stage("split");
  // ---- device buffers
  if (dev_malloc(&b->d_cn, 4 * np) != hipSuccess || dev_malloc(&b->d_jac, 8 * np) != hipSuccess ||
      dev_malloc(&b->d_aa, 8 * np) != hipSuccess || dev_malloc(&b->d_gout, 4 * np) != hipSuccess ||
      dev_malloc(&b->d_gyb, 8 * np) != hipSuccess || dev_malloc(&b->d_gyl, 4 * np) != hipSuccess)
    return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create: hipMalloc failed"));
  if (b->chunks > 1 && dev_malloc(&b->d_aa_part, 16 * np) != hipSuccess)
    return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create: hipMalloc failed"));
  b->use_short = short_kernel(b);  // fixed here: d_rec's allocation and the launch must agree
  // ---- the dense wedge-set path (k_score_wset). In a bipartite graph c ∈ H2(x) ⟺ x ∈ N(N(c)), c ≠ x,
  // so CN(x, y) = #{c ∈ N(y), c ≠ x : bit x of W(c)} with W(c) = N(N(c)) from the graph's wedge-set
  // index, and |H2(x)| = |W(x) \ {x}| from the same index. Taken by short-row batches with wedge
  // rows whose rows read (the y and N(x)) lie outside the sets' range (N(x) is then never at
  // distance 2) -- the business side of a review graph (BLP_NO_WSET=1: the grouped path)
  if (b->use_short && n_pairs > 0 && g->d_wp && !kn.no_wedge && !b->global && !b->split && b->chunks == 1 && span > 0) {
    const int64_t wlo = std::min<int64_t>(lo_raw, xlo), whi = std::max<int64_t>(hi, xhi);
    if (rows_lo >= whi || rows_hi <= wlo) {
      int rcw = BLP_OK;
      const WedgeSets* ws = wedge_sets(g, wlo, whi, &rcw);
      if (rcw) return bail(rcw);
      if (ws) {
        b->wset_pool = ws->d_pool;
        b->wset_h2 = ws->d_h2;
        b->wset_lo = ws->lo;
        b->wset_span = ws->hi - ws->lo;
        b->wset_words = ws->words;
      }
    }
  }
  stage("wset");
  // source records: the short-row scorer, and the large scorer (its header in one round trip)
  const bool want_rec = b->use_short || (b->variant == V_LARGE && !b->split && !b->global);
  if (want_rec &&
      dev_malloc(&b->d_rec, sizeof(SrcRec) * (size_t)std::max<int64_t>(b->n_sources, 1)) != hipSuccess)
    return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create: hipMalloc failed"));
  if (b->n_heavy) {
    if (dev_malloc(&b->d_heavy_slot, 4 * n) != hipSuccess ||
        dev_malloc(&b->d_heavy_bm, 4 * b->hb_words * b->n_heavy) != hipSuccess ||
        dev_malloc(&b->d_heavy_items, sizeof(HeavyItem) * items.size()) != hipSuccess)
      return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create: hipMalloc failed"));
    if (hipMemcpy(b->d_heavy_slot, heavy_slot.data(), 4 * n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(b->d_heavy_items, items.data(), sizeof(HeavyItem) * items.size(), hipMemcpyHostToDevice) !=
            hipSuccess)
      return bail(fail(BLP_E_HIP_BASE, "blp_batch_create: upload failed"));
  }
  stage("buffers");
#ifdef BLP_DEBUG
  if (kn.debug_oom && g->d_wp && !retry)  // test knob: this create runs out of memory once
    return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create [BLP_DEBUG_OOM]: out of memory"));
#endif
  // the plan reads the wedge index (wedge rows, wedge slices of heavy sources, wedge-row bitmaps):
  // the create's registration stays, so an out-of-memory retry releases the index only when no
  // live batch reads it; a plan that does not read it drops the registration
  const bool reads_wedge = b->wedge_user && !kn.no_wedge && (b->use_short || b->split || wedge_items || b->wbm_slot || b->wset_pool);
  if (b->wedge_user && !reads_wedge) {
    std::lock_guard<std::mutex> lk(g->wbm_mu);
    --g->wedge_users;
    b->wedge_user = false;
  }
  *out = b;
  return BLP_OK;
}

extern "C" {

// Out of HBM while creating a batch: the graph's wedge index (up to 35 % of the HBM that was free
// at graph creation, wedge.hip) is an accelerator every scorer can do without, so it is released
// -- when no live batch's plan reads it -- and the batch is planned again without it.
static bool is_oom(int rc) { return rc == BLP_E_HIP_BASE - (int)hipErrorOutOfMemory; }

static int create_or_release(blp_graph* g, const int32_t* x, const int32_t* y, int64_t n, const blp_batch* twin,
                             blp_batch** out, bool hi = false) {
  int rc = batch_create(g, x, y, n, twin, out, false, hi);
  if (is_oom(rc) && g) {  // the device scratch cache first (DevBuf blocks kept for reuse)
    (void)hipGetLastError();
    dev_cache_flush(g->device);
    rc = batch_create(g, x, y, n, twin, out, false, hi);
  }
  if (!is_oom(rc) || !g || !g->d_wp) return rc;
  {
    std::lock_guard<std::mutex> lk(g->wbm_mu);
    if (g->wedge_users > 0) return rc;  // a live batch reads it: the failure stands
    (void)hipGetLastError();
    (void)hipSetDevice(g->device);
    (void)hipStreamSynchronize(g->stream);
    free_wedge_index(g);
  }
  return batch_create(g, x, y, n, twin, out, true, hi);
}

int blp_batch_create(blp_graph* g, const int32_t* x, const int32_t* y, int64_t n_pairs, blp_batch** out) {
  return create_or_release(g, x, y, n_pairs, nullptr, out);
}

int blp_batch_create_pair(blp_graph* g, const int32_t* x, const int32_t* y, int64_t n_pairs, blp_batch** out_xy,
                          blp_batch** out_yx) {
  BLP_CHECK(out_xy && out_yx, BLP_E_ARG, "blp_batch_create_pair: null outputs");
  blp_batch* a = nullptr;
  // the first batch (similarity.main's user pass) on a highest-priority stream: the two passes
  // then run on different hardware queues (BLP_PAIR_SAME_PRIO=1: both from the normal pool;
  // BLP_PAIR_HI_SECOND=1: the second batch takes the highest-priority stream instead)
  const bool same = getenv("BLP_PAIR_SAME_PRIO") != nullptr, second = getenv("BLP_PAIR_HI_SECOND") != nullptr;
  int rc = create_or_release(g, x, y, n_pairs, nullptr, &a, !same && !second);
  if (rc) return rc;
  blp_batch* b = nullptr;
  rc = create_or_release(g, y, x, n_pairs, a, &b, !same && second);
  if (rc) {
    blp_batch_destroy(a);
    return rc;
  }
  *out_xy = a;
  *out_yx = b;
  return BLP_OK;
}

int blp_batch_destroy(blp_batch* b) {
  if (!b) return BLP_OK;
  if (b->g) (void)hipSetDevice(b->g->device);
  if (b->g && b->g->stream) (void)hipStreamSynchronize(b->g->stream);
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  if (b->g) {  // the batch's times join the graph's totals before its events go
    (void)timer_collect(b->t_score);
    (void)timer_collect(b->t_group);
    std::lock_guard<std::mutex> lk(b->g->timer_mu);
    auto& lt = b->g->live_timers;
    lt.erase(std::remove_if(lt.begin(), lt.end(), [&](KernelTimer* t) { return t == &b->t_score || t == &b->t_group; }), lt.end());
  }
  timer_release(b->t_score);
  timer_release(b->t_group);
  b->cnt.release();
  b->off.release();
  b->active.release();
  b->scratch.release();
  if (b->stream) stream_give(b->g ? b->g->device : 0, b->stream, b->hi_prio);  // back to the pool for the next batch
  if (b->wedge_user && b->g) {
    std::lock_guard<std::mutex> lk(b->g->wbm_mu);
    --b->g->wedge_users;
  }
  void* ps[] = {b->d_x,    b->d_y,    b->d_cn,   b->d_jac,  b->d_aa,          b->d_gout,        b->d_gyb,
                b->d_gyl,  b->d_misc, b->d_heavy_slot, b->d_heavy_bm, b->d_heavy_items, b->d_gbm, b->d_gy, b->d_rsplit, b->d_pcn, b->d_paa, b->d_ph2, b->d_aa_part, b->d_rec, b->d_hflag, b->d_lq, b->d_active2, b->d_rank, b->d_lpt};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  delete b;
  return BLP_OK;
}

int blp_batch_plan(const blp_batch* b, int64_t* lo, int64_t* hi, int* chunks, int* block, int* heavy) {
  BLP_CHECK(b, BLP_E_ARG, "blp_batch_plan: null batch");
  if (lo) *lo = b->lo;
  if (hi) *hi = b->hi;
  if (chunks) *chunks = b->global ? 0 : b->split ? -b->split : b->chunks;  // 0: HBM bitmap; -C: chunk-parallel
  if (block) *block = b->global ? G_BLOCK : b->split ? S_BLOCK : variant_block(b->variant);
  if (heavy) *heavy = (int)b->n_heavy;
  return BLP_OK;
}

int blp_batch_kernel(const blp_batch* b, uint32_t mask, char* name, int cap) {
  BLP_CHECK(b && name && cap > 0, BLP_E_ARG, "blp_batch_kernel: bad arguments");
  const bool aa = (mask & BLP_ADAMIC) != 0;
  char buf[96];
  if (b->global)
    snprintf(buf, sizeof buf, "k_score_global<%d, %d, 8>", G_BLOCK, G_SEG);
  else if (b->split)
    snprintf(buf, sizeof buf, "k_score_split<%d, %d, %d, 8>", S_BLOCK, b->split_big ? S_CAP_BIG : S_CAP, S_SEG);
  else if (b->wset_pool)
    snprintf(buf, sizeof buf, "k_score_wset<%s>", aa ? "true" : "false");
  else if (b->use_short && b->g->d_wp && !b->kn.no_wedge)
    snprintf(buf, sizeof buf, "k_score_short<%s>", aa ? "true" : "false");
  else if (b->use_short)
    snprintf(buf, sizeof buf, "k_score<%d, %d, %d, 8, true, %s>", BLOCK_SMALL, CAP_SMALL, SEG_SMALL, aa ? "true" : "false");
  else if (b->variant == V_SMALL)
    snprintf(buf, sizeof buf, "k_score<%d, %d, %d, 8, false, true>", BLOCK_SMALL, CAP_SMALL, SEG_SMALL);
  else if (b->variant == V_MED)
    snprintf(buf, sizeof buf, "k_score<%d, %d, %d, 8, false, %s>", BLOCK_MED, CAP_MED, aa ? SEG_MED : SEG_MED_NOAA,
             aa ? "true" : "false");
  else if (b->pko)
    snprintf(buf, sizeof buf, "k_score<%d, %d, %d, 8, false, true, true>", BLOCK_LARGE, CAP_PKO, SEG_PKO);
  else
    snprintf(buf, sizeof buf, "k_score<%d, %d, %d, 8, false, true>", BLOCK_LARGE, CAP_LARGE, SEG_LARGE);
  snprintf(name, (size_t)cap, "%s", buf);
  return BLP_OK;
}

int blp_batch_routes(const blp_batch* b, int64_t* n_sources, int64_t* n_hash, int* runs, int* wedge_bitmaps) {
  BLP_CHECK(b, BLP_E_ARG, "blp_batch_routes: null batch");
  if (n_sources) *n_sources = b->n_sources;
  if (n_hash) *n_hash = b->n_hash;
  if (runs) *runs = b->runs ? 1 : 0;
  if (wedge_bitmaps) *wedge_bitmaps = b->wbm_slot ? 1 : 0;
  return BLP_OK;
}

#ifdef BLP_PROF
int blp_prof_read(unsigned long long* out) {  // experiment builds only: per-phase clock sums, then reset
  BLP_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * 16));
  unsigned long long z[16] = {0};
  BLP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)));
  return BLP_OK;
}
#endif



// A batch on the wedge-set path (k_score_wset): no grouping; one launch over the pairs
static int score_wset(blp_graph* g, blp_batch* b, uint32_t mask) {
  int rc;
  const int64_t np = b->n_pairs;
  BLP_HIP(hipMemsetAsync(b->d_misc, 0, offsetof(Misc, dbg), b->stream));
  hipEvent_t bt1;
  if ((rc = timer_begin(b->t_score, b->stream, &bt1))) return rc;
  if (np) {
    ScoreArgs a{};
    a.rp = g->d_rp;
    a.ci = g->d_ci;
    a.aaw = g->d_aaw_fx;
    const bool coded = g->d_ci_w && !b->kn.no_wcodes;
    a.cw = coded ? g->d_ci_w : g->d_ci;
    a.idbits = coded ? g->id_bits : 31;
    a.idmask = (uint32_t)((1ull << a.idbits) - 1);
    a.wtab = g->d_wtab;
    a.misc = b->d_misc;
    a.cn = b->d_cn;
    a.jac = b->d_jac;
    a.aa = b->d_aa;
    a.mask = mask | BLP_CN;
    a.np = np;
    a.n_nodes = g->n;
    a.nnz = g->nnz;
    WsetArgs w{b->d_x, b->d_y, b->wset_pool, b->wset_h2, b->wset_lo, b->wset_span, b->wset_words};
#ifdef BLP_DEBUG
    if (b->kn.debug_null == "wset") w.pool = nullptr;  // test knob: the pre-launch check refuses it
#endif
    const char* missing = nullptr;
    auto need = [&](const void* p, const char* what) {
      if (!p && !missing) missing = what;
    };
    need(a.rp, "row offsets");
    need(a.cw, "col_idx");
    need(a.misc, "batch counters");
    need(a.cn, "cn output");
    need(a.jac, "jaccard output");
    need(a.aa, "adamic output");
    need(w.x, "pair x");
    need(w.y, "pair y");
    need(w.pool, "wedge sets");
    need(w.h2, "wedge-set sizes");
    if ((mask & BLP_ADAMIC) && !a.aaw) missing = missing ? missing : "aa weights";
    if (missing) {
      char msg[160];
      snprintf(msg, sizeof msg, "blp_batch_score: the launch path reads a null device pointer (%s)", missing);
      return fail(BLP_E_STATE, msg);
    }
    const int cus = b->cus > 0 ? b->cus : g->n_cu;
    const int64_t want = (np + 255) / 256;
    // 8 blocks per CU, all resident (fewer keep fewer users' sets in an XCD's L2 at once, and lose
    // more in parallelism: 6 / 4 / 3 / 2 per CU gave 1.72-1.74 / 1.74-1.76 / 1.75-1.76 / 1.74-1.75 ms
    // against 1.713-1.716, r06_ab7)
    const int grid = (int)std::max<int64_t>(8, std::min<int64_t>(want, (int64_t)cus * 8) / 8 * 8);
    if (mask & BLP_ADAMIC)
      hipLaunchKernelGGL(k_score_wset<true>, dim3(grid), dim3(256), 0, b->stream, a, w);
    else
      hipLaunchKernelGGL(k_score_wset<false>, dim3(grid), dim3(256), 0, b->stream, a, w);
    BLP_HIP(hipGetLastError());
  }
  if ((rc = timer_end(b->t_score, b->stream, bt1))) return rc;
  return BLP_OK;
}

int blp_batch_score(blp_graph* g, blp_batch* b, uint32_t mask) {
  BLP_CHECK(g && b && b->g == g, BLP_E_ARG, "blp_batch_score: graph/batch mismatch");
  BLP_CHECK((mask & ~7u) == 0, BLP_E_ARG, "blp_batch_score: unknown method bits");
  BLP_CHECK(!(mask & BLP_ADAMIC) || g->d_aaw_fx, BLP_E_STATE,
            "blp_batch_score: adamic_adar requested but the graph has no aa_weight table");
  int rc = set_device(g);
  if (rc) return rc;
  const int64_t n = g->n, np = b->n_pairs;
  const int64_t nh = (int64_t)b->nb * b->nblk;
  const int64_t tiles_h = (nh + SCAN_TILE - 1) / SCAN_TILE, tiles_b = (b->nb + SCAN_TILE - 1) / SCAN_TILE;
  if ((rc = b->cnt.reserve(4 * (n + 1)))) return rc;
  if ((rc = b->off.reserve(4 * (n + 1)))) return rc;
  if ((rc = b->active.reserve(4 * (n + 1)))) return rc;
  // scratch: hist | hoff | tiles | bucket_active | abase | tmp [| fill | item table | id-range tiles]
  const int64_t items_ub = (np + GI_PAIRS - 1) / GI_PAIRS + b->nb;
  const int64_t items_ints = b->items ? b->xspan + 3 * items_ub + 2 * ((b->xspan + SCAN_TILE - 1) / SCAN_TILE + 1) +
                                            1024 * items_ub
                                      : 0;
  const int64_t sc_ints = 2 * nh + std::max(tiles_h, tiles_b) + 1 + 2 * (int64_t)b->nb + 4 * np + items_ints;
  if ((rc = b->scratch.reserve(4 * (sc_ints + 16)))) return rc;
  int32_t* hist = b->scratch.as<int32_t>();
  int32_t* hoff = hist + nh;
  int32_t* tiles = hoff + nh;
  int32_t* bact = tiles + std::max(tiles_h, tiles_b) + 1;
  int32_t* abase = bact + b->nb;
  int4* tmp = reinterpret_cast<int4*>((reinterpret_cast<uintptr_t>(abase + b->nb) + 15) & ~uintptr_t(15));
  if (b->wset_pool) return score_wset(g, b, mask);
  hipEvent_t bt0;
  if ((rc = timer_begin(b->t_group, b->stream, &bt0))) return rc;
  // run-grouped batches: k_run_count zeroes the counters (one launch fewer); the large scorer's
  // source records come from k_run_cnt (one more)
  const bool run_group = np && b->runs;
  const bool rec_in_cnt = run_group && b->d_rec && b->variant == V_LARGE && !b->split && !b->global && !b->use_short;
  // ... and the block scorer of a run-grouped batch finds N(y) from the caller's y itself (grouped
  // order is caller order): no per-pair row starts and lengths are gathered and written per step
  const bool y_direct = run_group && !b->split && !b->global && !b->use_short && !b->kn.no_ydirect;
  // two launches (k_run_heads, k_run_records); no per-pair row metadata is written, so the
  // scorer must find N(y) itself (y_direct)
  const bool run_fast = rec_in_cnt && y_direct && b->d_rank && b->d_lpt && !b->kn.no_run_fast;
  if (!run_group) BLP_HIP(hipMemsetAsync(b->d_misc, 0, offsetof(Misc, dbg), b->stream));  // the debug record persists to fetch
  if (run_fast) {
    const unsigned gh = (unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)g->n_cu * 8, (np + 255) / 256));
    hipLaunchKernelGGL(k_run_heads, dim3(gh), dim3(256), 0, b->stream, b->d_x, np, (int32_t)b->xlo, b->d_rank,
                       b->off.as<int32_t>(), b->cnt.as<int32_t>(), b->d_lpt, reinterpret_cast<int32_t*>(b->d_misc),
                       (int)(offsetof(Misc, dbg) / 4), (int32_t)b->n_sources);
    const unsigned gr = (unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)g->n_cu * 4, (b->n_sources + 255) / 256));
    hipLaunchKernelGGL(k_run_records, dim3(gr), dim3(256), 0, b->stream, b->d_lpt, (int32_t)b->n_sources,
                       b->off.as<int32_t>(), b->cnt.as<int32_t>(), g->d_rp, g->d_ci,
                       (const int32_t*)(b->wbm_slot ? b->wbm_slot : b->d_heavy_slot), b->d_rec);
  } else if (run_group) {
    const int64_t tiles = (np + SCAN_TILE - 1) / SCAN_TILE;
    int32_t* rtile = reinterpret_cast<int32_t*>(tmp);  // the bucket sort's pair buffer is free here
    static_assert(offsetof(Misc, dbg) % 4 == 0, "counters zeroed as words");
    hipLaunchKernelGGL(k_run_count, dim3((unsigned)tiles), dim3(SCAN_BLOCK), 0, b->stream, b->d_x, np, rtile,
                       reinterpret_cast<int32_t*>(b->d_misc), (int)(offsetof(Misc, dbg) / 4));
    hipLaunchKernelGGL(k_scan_mid, dim3(1), dim3(SCAN_BLOCK), 0, b->stream, rtile, tiles, &b->d_misc->n_active);
    hipLaunchKernelGGL(k_run_write, dim3((unsigned)tiles), dim3(SCAN_BLOCK), 0, b->stream, b->d_x, b->d_y, np, g->d_rp,
                       rtile, b->active.as<int32_t>(), b->off.as<int32_t>(), (int32_t*)nullptr,
                       y_direct ? nullptr : b->d_gyb, y_direct ? nullptr : b->d_gyl, y_direct ? nullptr : b->d_gy);
    hipLaunchKernelGGL(k_run_cnt, dim3(1024), dim3(256), 0, b->stream, b->active.as<int32_t>(), &b->d_misc->n_active,
                       np, b->off.as<int32_t>(), b->cnt.as<int32_t>(), b->d_rank, (int32_t)b->xlo, b->d_lpt,
                       rec_in_cnt ? b->d_rec : nullptr, g->d_rp, g->d_ci,
                       (const int32_t*)(b->wbm_slot ? b->wbm_slot : b->d_heavy_slot));
  } else if (np) {
    // items mode: interleaved buckets (v & (nb - 1)); bucket mode: contiguous (v >> shift)
    const int hshift = b->items ? 0 : b->shift, bmask = b->items ? b->nb - 1 : -1;
    hipLaunchKernelGGL(k_bucket_hist, dim3(b->nblk), dim3(GP_BLOCK), 0, b->stream, b->d_x, np, b->xlo, hshift, bmask,
                       b->nb, b->nblk, b->per_blk, hist);
    hipLaunchKernelGGL(k_scan_sum, dim3((unsigned)tiles_h), dim3(SCAN_BLOCK), 0, b->stream, hist, nh, tiles);
    hipLaunchKernelGGL(k_scan_mid, dim3(1), dim3(SCAN_BLOCK), 0, b->stream, tiles, tiles_h, (int32_t*)nullptr);
    hipLaunchKernelGGL(k_scan_out, dim3((unsigned)tiles_h), dim3(SCAN_BLOCK), 0, b->stream, hist, nh, tiles, hoff);
    // item grouping whose write kernel stages runs (<= 1024 keys per bucket) and whose scorer reads
    // grouped row bounds (no g_y): the scatter gathers N(y)'s row in caller order (rec_rows) and
    // writes a compact key array for the item histograms
    const int64_t ub = (np + GI_PAIRS - 1) / GI_PAIRS + b->nb, tx = (b->xspan + SCAN_TILE - 1) / SCAN_TILE;
    const int64_t ikeys = b->items ? (b->xspan + b->nb - 1) >> b->shift : 0;
    const bool rec_rows = b->items && ikeys <= 1024 && !b->d_gy && g->nnz < (int64_t(1) << 31);
    // no key array beside the records: 512 more scattered write streams per block overflowed the
    // XCD's L2 (3x the written bytes, r05_group_pmc); the item counts read the records' x
    // (2.13-2.15 against 2.18-2.20 ms with the array, r05_scatter_nokeys)
    if (rec_rows)
      hipLaunchKernelGGL((k_bucket_scatter<true>), dim3(b->nblk), dim3(GP_BLOCK), 0, b->stream, b->d_x, b->d_y, np,
                         b->xlo, hshift, bmask, b->nb, b->nblk, b->per_blk, hoff, tmp, g->d_rp);
    else
      hipLaunchKernelGGL((k_bucket_scatter<false>), dim3(b->nblk), dim3(GP_BLOCK), 0, b->stream, b->d_x, b->d_y, np,
                         b->xlo, hshift, bmask, b->nb, b->nblk, b->per_blk, hoff, tmp);
    if (b->items) {
      int32_t* fill = reinterpret_cast<int32_t*>(tmp + np);
      int32_t *it_b = fill + b->xspan, *it_s = it_b + ub, *it_e = it_s + ub, *tx1 = it_e + ub, *tx2 = tx1 + tx + 1;
      int32_t *cnt = b->cnt.as<int32_t>(), *off = b->off.as<int32_t>();
      BLP_HIP(hipMemsetAsync(cnt + b->xlo, 0, 4 * (size_t)b->xspan, b->stream));
      BLP_HIP(hipMemsetAsync(fill, 0, 4 * (size_t)b->xspan, b->stream));
      hipLaunchKernelGGL(k_item_plan, dim3(1), dim3(1024), 0, b->stream, hoff, b->nblk, b->nb, np, it_b, it_s, it_e,
                         &b->d_misc->n_items);
      const int64_t keys = ikeys;
      const bool runs_w = keys <= 1024;
      int32_t* ih = tx2 + tx + 1;  // [ub][K] item histograms (runs_w)
#define BLP_ITEM_LAUNCH(K)                                                                                         \
  hipLaunchKernelGGL(k_item_count<K>, dim3((unsigned)ub), dim3(GB_BLOCK), 0, b->stream, tmp, it_b, it_s, it_e,     \
                     &b->d_misc->n_items, b->xlo, b->shift, cnt, runs_w ? ih : nullptr);                           \
  hipLaunchKernelGGL(k_scan_sum, dim3((unsigned)tx), dim3(SCAN_BLOCK), 0, b->stream, cnt + b->xlo, b->xspan, tx1); \
  hipLaunchKernelGGL(k_scan_mid, dim3(1), dim3(SCAN_BLOCK), 0, b->stream, tx1, tx, (int32_t*)nullptr);             \
  hipLaunchKernelGGL(k_scan_out, dim3((unsigned)tx), dim3(SCAN_BLOCK), 0, b->stream, cnt + b->xlo, b->xspan, tx1,  \
                     off + b->xlo);                                                                                 \
  hipLaunchKernelGGL(k_nz_count, dim3((unsigned)tx), dim3(SCAN_BLOCK), 0, b->stream, cnt + b->xlo, b->xspan, tx2); \
  hipLaunchKernelGGL(k_scan_mid, dim3(1), dim3(SCAN_BLOCK), 0, b->stream, tx2, tx, &b->d_misc->n_active);          \
  hipLaunchKernelGGL(k_nz_write, dim3((unsigned)tx), dim3(SCAN_BLOCK), 0, b->stream, cnt + b->xlo, b->xspan, tx2,  \
                     b->xlo, b->active.as<int32_t>(), b->d_rank, b->d_lpt);                                         \
  if (runs_w && rec_rows)                                                                                             \
    hipLaunchKernelGGL((k_item_write_ids<(K <= 1024 ? K : 1024), 2>), dim3((unsigned)ub), dim3(GB_BLOCK), 0,         \
                       b->stream, g->d_rp, tmp, it_b, it_s, it_e, &b->d_misc->n_items, b->xlo, b->shift, ih, off,     \
                       fill, b->d_gout, b->d_gyb, b->d_gyl, b->d_gy);                                                 \
  else if (runs_w)                                                                                                    \
    hipLaunchKernelGGL((k_item_write_ids<(K <= 1024 ? K : 1024), 1>), dim3((unsigned)ub), dim3(GB_BLOCK), 0,         \
                       b->stream, g->d_rp, tmp, it_b, it_s, it_e, &b->d_misc->n_items, b->xlo, b->shift, ih, off,     \
                       fill, b->d_gout, b->d_gyb, b->d_gyl, b->d_gy);                                                 \
  else                                                                                                                \
    hipLaunchKernelGGL(k_item_write<K>, dim3((unsigned)ub), dim3(GB_BLOCK), 0, b->stream, g->d_rp, tmp, it_b, it_s,  \
                       it_e, &b->d_misc->n_items, b->xlo, b->shift, off, fill, b->d_gout, b->d_gyb, b->d_gyl, b->d_gy)
      if (keys <= 64) {  // 272 bytes of LDS: fits beside a 160 KiB large-scorer workgroup
        BLP_ITEM_LAUNCH(64);
      } else if (keys <= 256) {
        BLP_ITEM_LAUNCH(256);
      } else if (keys <= 1024) {
        BLP_ITEM_LAUNCH(1024);
      } else if (keys <= 4096) {
        BLP_ITEM_LAUNCH(4096);
      } else {
        BLP_ITEM_LAUNCH(32768);
      }
#undef BLP_ITEM_LAUNCH
    } else {
      const int keys = 1 << b->shift;
#define BLP_GROUP_LAUNCH(K)                                                                                         \
    hipLaunchKernelGGL(k_bucket_group<K>, dim3(b->nb), dim3(GB_BLOCK), 0, b->stream, g->d_rp, tmp, hoff,               \
                       b->nblk, b->nb, b->shift, b->xlo, b->xspan, np, b->off.as<int32_t>(), b->cnt.as<int32_t>(), bact,  \
                       b->d_gout,                                                                                       \
                       b->d_gyb, b->d_gyl, b->d_gy)
      if (keys <= 64)  // 272 bytes of LDS: fits beside a 160 KiB large-scorer workgroup
        BLP_GROUP_LAUNCH(64);
      else if (keys <= 256)
        BLP_GROUP_LAUNCH(256);
      else if (keys <= 1024)
        BLP_GROUP_LAUNCH(1024);
      else if (keys <= 4096)
        BLP_GROUP_LAUNCH(4096);
      else
        BLP_GROUP_LAUNCH(32768);
#undef BLP_GROUP_LAUNCH
      hipLaunchKernelGGL(k_scan_sum, dim3((unsigned)tiles_b), dim3(SCAN_BLOCK), 0, b->stream, bact, (int64_t)b->nb, tiles);
      hipLaunchKernelGGL(k_scan_mid, dim3(1), dim3(SCAN_BLOCK), 0, b->stream, tiles, tiles_b, &b->d_misc->n_active);
      hipLaunchKernelGGL(k_scan_out, dim3((unsigned)tiles_b), dim3(SCAN_BLOCK), 0, b->stream, bact, (int64_t)b->nb, tiles,
                         abase);
#define BLP_ACTIVE_LAUNCH(K)                                                                                   \
    hipLaunchKernelGGL(k_active_write<K>, dim3(b->nb), dim3(GB_BLOCK), 0, b->stream, b->cnt.as<int32_t>(), abase, b->shift, \
                       b->xlo, b->xspan, b->active.as<int32_t>())
      if (keys <= 64)  // 272 bytes of LDS: fits beside a 160 KiB large-scorer workgroup
        BLP_ACTIVE_LAUNCH(64);
      else if (keys <= 256)
        BLP_ACTIVE_LAUNCH(256);
      else if (keys <= 1024)
        BLP_ACTIVE_LAUNCH(1024);
      else if (keys <= 4096)
        BLP_ACTIVE_LAUNCH(4096);
      else
        BLP_ACTIVE_LAUNCH(32768);
#undef BLP_ACTIVE_LAUNCH
    }
  }
  BLP_HIP(hipGetLastError());
  if ((rc = timer_end(b->t_group, b->stream, bt0))) return rc;

  hipEvent_t bt1;
  if ((rc = timer_begin(b->t_score, b->stream, &bt1))) return rc;
  if (b->n_heavy) {
    BLP_HIP(hipMemsetAsync(b->d_heavy_bm, 0, 4 * b->hb_words * b->n_heavy, b->stream));
    HeavyArgs h{g->d_rp, g->d_ci, b->d_heavy_items, b->d_heavy_bm, b->hb_words, b->lo, b->hi - b->lo,
                reinterpret_cast<const uint4*>(g->d_wedge)};
    if (b->variant == V_SMALL)
      rc = launch_heavy<BLOCK_SMALL, CAP_SMALL, SEG_SMALL>(b->stream, h, b->n_heavy_items);
    else if (b->variant == V_MED)
      rc = launch_heavy<BLOCK_MED, CAP_MED, SEG_MED>(b->stream, h, b->n_heavy_items);
    else
      rc = launch_heavy<BLOCK_LARGE, CAP_LARGE, SEG_LARGE>(b->stream, h, b->n_heavy_items);
    if (rc) return rc;
  }
  ScoreArgs a{};  // value-initialised: a field a path does not set is null / zero, never stale
  a.wp = nullptr;
  a.wedge = nullptr;
  a.rp = g->d_rp;
  a.ci = g->d_ci;
  a.aaw = g->d_aaw_fx;
  a.aa_part = b->d_aa_part;
  a.rec = nullptr;
  const bool coded = g->d_ci_w && !b->kn.no_wcodes;  // test knob
  a.cw = coded ? g->d_ci_w : g->d_ci;
  a.idbits = coded ? g->id_bits : 31;
  a.idmask = (uint32_t)((1ull << a.idbits) - 1);
  a.wtab = g->d_wtab;

  a.off = b->off.as<int32_t>();
  a.cnt = b->cnt.as<int32_t>();
  a.active = b->d_lpt ? b->d_lpt : b->active.as<int32_t>();  // BLP_LPT: the largest-first queue
  a.g_out = b->runs ? nullptr : b->d_gout;  // run-grouped: grouped order is caller order
  a.g_yb = b->d_gyb;
  a.g_yl = b->d_gyl;
  a.py = y_direct ? b->d_y : nullptr;
  a.hot_idx = b->use_hot ? g->d_hot_idx : nullptr;
  a.hot_tab = (const HotRow*)g->d_hot_tab;
  a.hot_pool = (const uint4*)g->d_hot_pool;
  a.heavy_slot = b->wbm_slot ? b->wbm_slot : b->d_heavy_slot;
  a.heavy_bm = b->wbm_slot ? const_cast<uint32_t*>(b->wbm_pool) : b->d_heavy_bm;
  a.hb_words = b->hb_words;
  a.misc = b->d_misc;
  a.cn = b->d_cn;
  a.jac = b->d_jac;
  a.aa = b->d_aa;
  a.lo = b->lo;
  a.hi = b->hi;
  a.cap_bits = b->cap_bits;
  a.mask = mask | BLP_CN;  // counts are always produced (Jaccard needs them)
  a.dq = b->dq;
  a.short_rows = b->short_rows;
  a.np = np;
  a.n_nodes = g->n;
  a.rs_rows = b->rs_rows;
  a.nnz = g->nnz;
  a.wedge_vecs = g->wedge_vecs;
  a.n_hot = g->n_hot;
  a.hot_vecs = g->hot_pool_words / 4;
  a.lq_wgs = b->d_lq ? 2 * g->n_cu : 0;
  if (np && b->split) {
    a.lq = b->d_lq;
    if (g->d_wp && !b->kn.no_wedge) {  // sources with wedge rows build from them (split and hash kernels)
      a.wp = g->d_wp;
      a.wedge = reinterpret_cast<const uint4*>(g->d_wedge);
    }
  } else if (np && b->use_short && g->d_wp && !b->kn.no_wedge) {  // test knob: BLP_NO_WEDGE builds from CSR
    a.wp = g->d_wp;
    a.wedge = reinterpret_cast<const uint4*>(g->d_wedge);
  }
  if (np && (rc = launch_pointers(g, b, a, mask))) return rc;
  if (np && b->split) {
    // AA counts ride in the packed per-pair word while every row (hence every count) < 2^24
    const int pk24 = (mask & BLP_ADAMIC) && g->max_row < (int64_t(1) << SPLIT_CN_BITS) && !b->kn.split_nopk;
    // slices of <= short_max ids scanned by their pair's thread (128 KiB chunks; BLP_SPLIT_SHORT=0: off)
    const int short_max = std::min(SHORT_PART, b->kn.split_short >= 0 ? b->kn.split_short : SHORT_PART);
    // CUs the persistent grids may fill (blp_batches_score), within [1, n_cu]: d_lq holds 2 workgroups per CU
    const int scu = std::max(1, std::min(b->cus > 0 ? b->cus : g->n_cu, g->n_cu));
    if (b->d_hflag) {  // small-H2 sources first, on their own hash-set kernel
      hipLaunchKernelGGL(k_hash_partition, dim3(g->n_cu * 4), dim3(256), 0, b->stream, a.active, b->d_misc, b->d_hflag,
                         (int32_t)b->xlo, b->d_active2);
      BLP_HIP(hipGetLastError());
      a.active = b->d_active2;
      int hcu = 1;
      if (b->kn.hash_big) {
        BLP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&hcu, k_score_hash<HS_BLOCK_BIG, HS_HT_BIG>, HS_BLOCK_BIG, 0));
        hipLaunchKernelGGL((k_score_hash<HS_BLOCK_BIG, HS_HT_BIG>), dim3(scu * std::max(hcu, 1)), dim3(HS_BLOCK_BIG), 0,
                           b->stream, a);
      } else {
        BLP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&hcu, k_score_hash<HS_BLOCK, HS_HT>, HS_BLOCK, 0));
        hipLaunchKernelGGL((k_score_hash<HS_BLOCK, HS_HT>), dim3(scu * std::max(hcu, 1)), dim3(HS_BLOCK), 0, b->stream, a);
      }
      BLP_HIP(hipGetLastError());
    }
    if (!pk24) BLP_HIP(hipMemsetAsync(b->d_pcn, 0, 4 * (size_t)np, b->stream));
    if (mask & BLP_ADAMIC) BLP_HIP(hipMemsetAsync(b->d_paa, 0, 16 * (size_t)np, b->stream));
    int per_cu = 1;
    if (b->split_big) {
      BLP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_score_split<S_BLOCK, S_CAP_BIG, S_SEG, 8>, S_BLOCK, 0));
      hipLaunchKernelGGL((k_score_split<S_BLOCK, S_CAP_BIG, S_SEG, 8>), dim3(scu * std::min(std::max(per_cu, 1), 2)), dim3(S_BLOCK),
                         0, b->stream, a, b->d_gy, b->d_rsplit, b->rs_lo, b->split, b->d_pcn, b->d_paa, b->d_ph2, np, pk24,
                         short_max);
    } else {
      BLP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_score_split<S_BLOCK, S_CAP, S_SEG, 8>, S_BLOCK, 0));
      hipLaunchKernelGGL((k_score_split<S_BLOCK, S_CAP, S_SEG, 8>), dim3(scu * std::min(std::max(per_cu, 1), 2)), dim3(S_BLOCK), 0,
                         b->stream, a, b->d_gy, b->d_rsplit, b->rs_lo, b->split, b->d_pcn, b->d_paa, b->d_ph2, np, pk24,
                         short_max);
    }
    BLP_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_split_combine, dim3(g->n_cu * 8), dim3(256), 0, b->stream, a, b->split, b->d_pcn, b->d_paa,
                       b->d_ph2, np, pk24);
    BLP_HIP(hipGetLastError());
  } else if (np && b->global) {
    a.hot_idx = nullptr;
    hipLaunchKernelGGL((k_score_global<G_BLOCK, G_SEG, 8>), dim3((unsigned)b->gslots), dim3(G_BLOCK), 0, b->stream, a,
                       b->d_gbm, b->gwords);
    BLP_HIP(hipGetLastError());
  } else if (np && b->use_short) {
    // bitmap in dynamic LDS, sized to the universe (whole 16-byte vectors)
    const size_t dyn = 4 * (size_t)std::max<int64_t>(4, ((b->hi - b->lo + 31) / 32 + 3) / 4 * 4);
    if (b->d_rec) {  // one record per active source (after grouping, on the batch stream)
      hipLaunchKernelGGL(k_source_records, dim3((unsigned)std::min<int64_t>((b->n_sources + 255) / 256, 2048)),
                         dim3(256), 0, b->stream, a.active, b->d_misc, a.off, a.cnt, g->d_rp, g->d_ci, a.heavy_slot,
                         a.wp, b->d_rec);
      BLP_HIP(hipGetLastError());
      a.rec = b->d_rec;
    }
    if ((rc = (mask & BLP_ADAMIC) ? launch_short<true>(g, b, a, dyn) : launch_short<false>(g, b, a, dyn))) return rc;
  } else if (np) {
    int per_cu = 1;
    if ((rc = variant_occupancy(b->variant, &per_cu))) return rc;
    if (b->d_rec && b->variant == V_LARGE) {  // the large scorer's source headers (after grouping)
      if (!rec_in_cnt) {  // (run-grouped batches: written by k_run_cnt)
        hipLaunchKernelGGL(k_source_records, dim3((unsigned)std::min<int64_t>((b->n_sources + 255) / 256, 2048)),
                           dim3(256), 0, b->stream, a.active, b->d_misc, a.off, a.cnt, g->d_rp, g->d_ci, a.heavy_slot,
                           nullptr, b->d_rec);
        BLP_HIP(hipGetLastError());
      }
      a.rec = b->d_rec;
    }
    if (b->variant == V_SMALL)
      rc = launch_score<BLOCK_SMALL, CAP_SMALL, SEG_SMALL>(g, b->stream, a, per_cu, b->cus);
    else if (b->variant == V_MED)
      rc = (mask & BLP_ADAMIC) ? launch_score<BLOCK_MED, CAP_MED, SEG_MED>(g, b->stream, a, per_cu, b->cus)
                               : launch_score<BLOCK_MED, CAP_MED, SEG_MED_NOAA, false>(g, b->stream, a, per_cu, b->cus);
    else if (b->pko) {
      a.cap_bits = std::min<int64_t>(a.cap_bits, 32ll * CAP_PKO);
      rc = launch_score<BLOCK_LARGE, CAP_PKO, SEG_PKO, true, true>(g, b->stream, a, per_cu, b->cus);
    } else
      rc = launch_score<BLOCK_LARGE, CAP_LARGE, SEG_LARGE>(g, b->stream, a, per_cu, b->cus);
    if (rc) return rc;
  }
  if ((rc = timer_end(b->t_score, b->stream, bt1))) return rc;
  return BLP_OK;
}

// Several passes of one step enqueued together (similarity.main: the user and the business
// pass), each on its own stream. A large-universe batch (one 160 KiB-LDS workgroup per CU,
// the user side) holds every CU it lands on until it ends, so beside other batches it is given
// a share of the CUs and the short-row scorer and the grouping kernels run on the rest from
// the start, instead of queueing behind it.
//
// Share = n_cu * t_L / (t_L + KAPPA * t_O), clamped to [n_cu / 2, n_cu], from per-batch time
// estimates: planned elements / rate (large-universe scorer ~1.2e9 elements per ms, others
// ~1.8e8) + ~3.9e-8 ms per pair of bucket grouping for the others. KAPPA = 0.38: a
// latency-bound short-row pass does the same work in fewer CU-milliseconds on a few CUs
// than spread over the chip. Calibrated on config 2 (MI355X): the estimate gives 192 of 256
// CUs, the measured optimum (2.73 ms per step; all CUs 2.93, 160: 2.96, 176: 2.79, 208:
// 2.78, 224: 2.87, 240: 3.03). A small second pass leaves the large one (nearly) the whole
// chip. BLP_COSCHED_CUS overrides the share.
int blp_batches_score(blp_graph* g, int n, blp_batch* const* bs, const uint32_t* masks) {
  BLP_CHECK(g && n >= 0 && (n == 0 || (bs && masks)), BLP_E_ARG, "blp_batches_score: bad arguments");
  auto is_large = [](const blp_batch* b) { return b->variant == V_LARGE && !b->split && !b->global; };
  double t_large = 0.0, t_other = 0.0;
  int n_wset = 0;
  for (int i = 0; i < n; ++i) {
    BLP_CHECK(bs[i] && bs[i]->g == g, BLP_E_ARG, "blp_batches_score: graph/batch mismatch");
    if (is_large(bs[i]))
      t_large += (double)bs[i]->work_elems / 1.2e9;
    else if (bs[i]->wset_pool)
      ++n_wset;
    else
      t_other += (double)bs[i]->work_elems / 1.8e8 + 3.9e-8 * (double)bs[i]->n_pairs;
  }
  // wedge-set batches (k_score_wset: no grouping, one light launch) are enqueued beside the large
  // pass, which then holds no CU share: the light launch runs while the large pass groups its
  // pairs, and the large scorer takes the whole chip after it (config 2: 1.715-1.717 ms per step;
  // after the large pass on its stream's completion, BLP_WSET_SERIAL=1: 1.761-1.764 ms; with the
  // large pass held to 240 / 224 / 208 / 192 CUs: 1.80 / 1.85 / 1.96 / 2.05-2.07 ms, r06_check3;
  // gated on the large pass's grouping so its scorer is dispatched first: 1.76-1.77 ms, the light
  // launch's blocks then interleave with the scorer's workgroups, 1.43 -> 1.61 ms, r06_ab6)
  static const bool wset_serial = getenv("BLP_WSET_SERIAL") && atoi(getenv("BLP_WSET_SERIAL")) > 0;
  int share = g->n_cu;
  if (t_large > 0.0 && t_other > 0.0) {
    const double f = t_large / (t_large + 0.38 * t_other);
    share = std::max(g->n_cu / 2, std::min(g->n_cu, (int)std::lround(f * g->n_cu / 8.0) * 8));
  }
  if (n > 0 && bs[0]->kn.cosched_cus > 0) share = bs[0]->kn.cosched_cus;  // tuning knob (read at create)
  // chunk-parallel batches (config 5's two passes) each take the whole chip: holding each
  // persistent grid to a CU share was slower at every share tried (1951 ms per config-5 step in
  // proportion to planned work, 864 / 903 ms at 176 / 128 user CUs, against 743 ms)
  if (n_wset && !wset_serial && n > 0 && bs[0]->kn.cosched_cus > 0 && t_other == 0.0) t_other = 1.0;  // share applies
  int rc = BLP_OK;
  hipEvent_t large_done = nullptr;
  for (int pass = 0; pass < 2 && !rc; ++pass) {  // pass 0: every batch but the serial wedge-set ones
    for (int i = 0; i < n && !rc; ++i) {
      blp_batch* b = bs[i];
      const bool later = wset_serial && b->wset_pool && t_large > 0.0;
      if (later != (pass == 1)) continue;
      if (later && large_done) BLP_HIP(hipStreamWaitEvent(b->stream, large_done, 0));
      b->cus = is_large(b) && t_other > 0.0 ? share : 0;
      rc = blp_batch_score(g, b, masks[i]);
      b->cus = 0;
      if (!rc && is_large(b) && wset_serial && n_wset && !large_done) {
        hipError_t e = hipEventCreateWithFlags(&large_done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventRecord(large_done, b->stream);
        if (e != hipSuccess) rc = hip_fail(e, "blp_batches_score: large-pass event", __FILE__, __LINE__);
      }
    }
  }
  if (large_done) (void)hipEventDestroy(large_done);
  return rc;
}

int blp_batch_stats(blp_batch* b, int which, double* total_ms, int64_t* launches) {
  BLP_CHECK(b && (which == 0 || which == 1), BLP_E_ARG, "blp_batch_stats: bad arguments");
  KernelTimer& t = which == 0 ? b->t_score : b->t_group;
  int rc = set_device(b->g);
  if (rc) return rc;
  if ((rc = timer_collect(t))) return rc;
  std::lock_guard<std::mutex> lk(b->g->timer_mu);
  if (total_ms) *total_ms = t.total_ms;
  if (launches) *launches = t.launches;
  return BLP_OK;
}

int blp_batch_stats_reset(blp_batch* b) {
  BLP_CHECK(b, BLP_E_ARG, "blp_batch_stats_reset: null batch");
  int rc = set_device(b->g);
  if (rc) return rc;
  for (KernelTimer* t : {&b->t_score, &b->t_group}) {
    if ((rc = timer_collect(*t))) return rc;
    std::lock_guard<std::mutex> lk(b->g->timer_mu);  // (a graph stats call may collect this timer)
    t->total_ms = 0;
    t->launches = 0;
  }
  return BLP_OK;
}

int blp_batch_fetch(blp_graph* g, blp_batch* b, uint32_t* cn, double* jac, double* aa) {
  BLP_CHECK(g && b && b->g == g, BLP_E_ARG, "blp_batch_fetch: graph/batch mismatch");
  int rc = set_device(g);
  if (rc) return rc;
  BLP_HIP(hipStreamSynchronize(b->stream));
  const int64_t np = b->n_pairs;
  Misc m;
  BLP_HIP(hipMemcpy(&m, b->d_misc, sizeof(Misc), hipMemcpyDeviceToHost));
  if (np) {
    if (cn) prefault_host(cn, 4 * (size_t)np);
    if (jac) prefault_host(jac, 8 * (size_t)np);
    if (aa) prefault_host(aa, 8 * (size_t)np);
    if (cn && (rc = copy_sync(cn, b->d_cn, 4 * np, hipMemcpyDeviceToHost, b->stream))) return rc;
    if (jac && (rc = copy_sync(jac, b->d_jac, 8 * np, hipMemcpyDeviceToHost, b->stream))) return rc;
    if (aa && (rc = copy_sync(aa, b->d_aa, 8 * np, hipMemcpyDeviceToHost, b->stream))) return rc;
  }
#ifdef BLP_DEBUG
  if (m.dbg[0]) {  // the scorers' bound checks (PS_OK): any violation fails the batch
    const long long z[4] = {0, 0, 0, 0};
    BLP_HIP(hipMemcpy(b->d_misc->dbg, z, sizeof(z), hipMemcpyHostToDevice));
    char msg[160];
    snprintf(msg, sizeof msg, "blp_batch_fetch [BLP_DEBUG]: %lld bound violations; first at site %lld: %lld vs bound %lld",
             m.dbg[0], m.dbg[1], m.dbg[2], m.dbg[3]);
    return fail(BLP_E_STATE, msg);
  }
#endif
  if (m.zero_div && jac) return fail(BLP_E_ZERODIV, "float division by zero (Jaccard union is empty)");
  return BLP_OK;
}

int blp_batch_fetch_repr(blp_graph* g, blp_batch* b, int which, int zero_int, char* out) {
  BLP_CHECK(g && b && b->g == g && (which == BLP_JACCARD || which == BLP_ADAMIC), BLP_E_ARG,
            "blp_batch_fetch_repr: graph/batch mismatch or which is not BLP_JACCARD / BLP_ADAMIC");
  const int64_t np = b->n_pairs;
  BLP_CHECK(np == 0 || out, BLP_E_ARG, "blp_batch_fetch_repr: null output");
  int rc = set_device(g);
  if (rc) return rc;
  BLP_HIP(hipStreamSynchronize(b->stream));
  Misc m;
  BLP_HIP(hipMemcpy(&m, b->d_misc, sizeof(Misc), hipMemcpyDeviceToHost));
#ifdef BLP_DEBUG
  if (m.dbg[0]) {  // the same bound-check report as blp_batch_fetch: no slots from a violating batch
    const long long z[4] = {0, 0, 0, 0};
    BLP_HIP(hipMemcpy(b->d_misc->dbg, z, sizeof(z), hipMemcpyHostToDevice));
    char msg[160];
    snprintf(msg, sizeof msg,
             "blp_batch_fetch_repr [BLP_DEBUG]: %lld bound violations; first at site %lld: %lld vs bound %lld",
             m.dbg[0], m.dbg[1], m.dbg[2], m.dbg[3]);
    return fail(BLP_E_STATE, msg);
  }
#endif
  if (which == BLP_JACCARD && m.zero_div) return fail(BLP_E_ZERODIV, "float division by zero (Jaccard union is empty)");
  if (np == 0) return BLP_OK;
  ScopedBuf slots;
  if ((rc = slots.reserve((size_t)blp::REPR_SLOT_BYTES * np))) return rc;
  rc = repr_launch(which == BLP_JACCARD ? b->d_jac : b->d_aa, np, zero_int != 0, slots.as<char>(), g->n_cu, b->stream);
  if (rc) return rc;
  prefault_host(out, (size_t)blp::REPR_SLOT_BYTES * np);  // while the formatter runs
  return copy_sync(out, slots.p, (size_t)blp::REPR_SLOT_BYTES * np, hipMemcpyDeviceToHost, b->stream);
}

int blp_score_pairs(blp_graph* g, int side, uint32_t mask, const int32_t* pu, const int32_t* pb, int64_t n_pairs,
                    uint32_t* cn, double* jac, double* aa) {
  BLP_CHECK(g && (side == 0 || side == 1), BLP_E_ARG, "blp_score_pairs: bad graph or side");
  BLP_CHECK(!(mask & BLP_CN) || cn, BLP_E_ARG, "blp_score_pairs: cn output missing");
  BLP_CHECK(!(mask & BLP_JACCARD) || jac, BLP_E_ARG, "blp_score_pairs: jaccard output missing");
  BLP_CHECK(!(mask & BLP_ADAMIC) || aa, BLP_E_ARG, "blp_score_pairs: adamic output missing");
  blp_batch* b = nullptr;
  int rc = side == 0 ? blp_batch_create(g, pu, pb, n_pairs, &b) : blp_batch_create(g, pb, pu, n_pairs, &b);
  if (rc) return rc;
  rc = blp_batch_score(g, b, mask);
  if (!rc)
    rc = blp_batch_fetch(g, b, (mask & BLP_CN) ? cn : nullptr, (mask & BLP_JACCARD) ? jac : nullptr,
                         (mask & BLP_ADAMIC) ? aa : nullptr);
  blp_batch_destroy(b);
  return rc;
}

}  // extern "C"

// Loads this file's GPU code object (blp_stream_prewarm): the HIP runtime loads a translation
// unit's code object on the first launch of any of its kernels, 10-30 ms on the caller's thread.
namespace blp {
int preload_pairs() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_scan_sum)) == hipSuccess ? 0 : -1;
}
}  // namespace blp
