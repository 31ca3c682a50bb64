// Pair scoring: common neighbours / Jaccard / Adamic-Adar on candidate pairs (libblp.so).
//
// Replaces the hot loops of similarity.users (similarity.py:20-61) and
// similarity.business (similarity.py:63-106). For a pair (x, y):
//   H2(x) = GetNodesAtHop(G, x, 2)  (similarity.py:29 / :74) -- exact BFS distance 2
//   N(y)  = GetNodesAtHop(G, y, 1)  (similarity.py:41 / :85)
//   cn  = |H2(x) ∩ N(y)|                                       (:113-114)
//   jac = float(cn) / float(|H2(x)| + |N(y)| - cn)              (:108-111)
//   aa  = Σ_{w ∈ H2(x) ∩ N(y)} aaw[w],  aaw = (log deg)^-1 | 0  (:116-126)
//
// One step (blp_batch_score), all on the graph's stream:
//   1. group:  counting sort of the pairs by source x on the device (count -> scan ->
//              scatter) + compaction of the active sources.
//   2. score:  persistent workgroups dequeue one source at a time. The workgroup builds
//              H2(x) as a bitmap in LDS over the batch's node universe [lo, hi) (chunked
//              when it exceeds LDS), removes distance 0/1 (x and N(x)), popcounts |H2(x)|,
//              then scans N(y) of every pair of x, testing bits. Lanes are split into
//              groups of G (8..64) so short rows do not idle a whole wave.
// The graph, the pairs and the outputs stay in HBM; the host only plans the launch.
#include <algorithm>
#include <cmath>

#include "blp_internal.h"

namespace {

constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

struct Misc {
  int n_active;
  int queue;
  int zero_div;
  int pad;
};

// ------------------------------------------------------------------ grouping kernels
__global__ void k_count(const int32_t* __restrict__ x, int64_t n_pairs, int32_t* __restrict__ cnt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_pairs; i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[x[i]], 1);
}

// block-wide exclusive scan of (count, flag) pairs; returns the block total in *tot
__device__ inline int2 block_exscan2(int2 v, int2* lds, int2* tot) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int NW = SCAN_BLOCK / 64;
  int2 inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int tx = __shfl_up(inc.x, d, 64);
    int ty = __shfl_up(inc.y, d, 64);
    if (lane >= d) {
      inc.x += tx;
      inc.y += ty;
    }
  }
  if (lane == 63) lds[wid] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int2 run = make_int2(0, 0);
    for (int w = 0; w < NW; ++w) {
      int2 t = lds[w];
      lds[w] = run;
      run.x += t.x;
      run.y += t.y;
    }
    lds[NW] = run;
  }
  __syncthreads();
  int2 base = lds[wid];
  *tot = lds[NW];
  __syncthreads();
  return make_int2(base.x + inc.x - v.x, base.y + inc.y - v.y);
}

// pass 1: per-tile totals of (cnt, cnt > 0)
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_tiles(const int32_t* __restrict__ cnt, int64_t n,
                                                           int2* __restrict__ tile_sum) {
  __shared__ int2 lds[SCAN_BLOCK / 64 + 1];
  int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int2 v = make_int2(0, 0);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    int64_t i = base + k;
    int c = i < n ? cnt[i] : 0;
    v.x += c;
    v.y += c > 0;
  }
  int2 tot;
  block_exscan2(v, lds, &tot);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}

// pass 2: exclusive scan of the tile totals (one block); writes n_active
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_tilesums(int2* __restrict__ tile_sum, int64_t ntiles,
                                                              Misc* __restrict__ misc) {
  __shared__ int2 lds[SCAN_BLOCK / 64 + 1];
  int2 carry = make_int2(0, 0);
  for (int64_t b = 0; b < ntiles; b += SCAN_BLOCK) {
    int64_t i = b + threadIdx.x;
    int2 v = i < ntiles ? tile_sum[i] : make_int2(0, 0);
    int2 tot;
    int2 e = block_exscan2(v, lds, &tot);
    if (i < ntiles) tile_sum[i] = make_int2(e.x + carry.x, e.y + carry.y);
    carry.x += tot.x;
    carry.y += tot.y;
  }
  if (threadIdx.x == 0) misc->n_active = carry.y;
}

// pass 3: offsets, scatter cursors, active-source list
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_apply(const int32_t* __restrict__ cnt, int64_t n,
                                                           const int2* __restrict__ tile_sum,
                                                           int32_t* __restrict__ off, int32_t* __restrict__ cursor,
                                                           int32_t* __restrict__ active) {
  __shared__ int2 lds[SCAN_BLOCK / 64 + 1];
  int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
  int c[SCAN_ITEMS];
  int2 v = make_int2(0, 0);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    int64_t i = base + k;
    c[k] = i < n ? cnt[i] : 0;
    v.x += c[k];
    v.y += c[k] > 0;
  }
  int2 tot;
  int2 e = block_exscan2(v, lds, &tot);
  int2 t = tile_sum[blockIdx.x];
  int o = e.x + t.x, a = e.y + t.y;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    int64_t i = base + k;
    if (i < n) {
      off[i] = o;
      cursor[i] = o;
      if (c[k] > 0) active[a++] = (int32_t)i;
      o += c[k];
    }
  }
}

__global__ void k_scatter(const int32_t* __restrict__ x, int64_t n_pairs, int32_t* __restrict__ cursor,
                          int32_t* __restrict__ perm) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_pairs; i += (int64_t)gridDim.x * blockDim.x) {
    int pos = atomicAdd(&cursor[x[i]], 1);
    perm[pos] = (int32_t)i;
  }
}

// ------------------------------------------------------------------ scorer
struct ScoreArgs {
  const int64_t* rp;
  const int32_t* ci;
  const double* aaw;
  const int32_t* y;       // pair targets, caller order
  const int32_t* perm;    // grouped position -> caller index
  const int32_t* off;     // per node: first grouped position of its pairs
  const int32_t* cnt;     // per node: number of pairs with that source
  const int32_t* active;  // active sources
  Misc* misc;
  uint32_t* cn;
  double* jac;
  double* aa;
  int64_t lo, hi;  // bitmap universe
  uint32_t mask;
  int group;         // lanes per pair group
  int64_t cap_bits;  // bitmap bits per chunk (<= template capacity; lowered only by tests)
  int64_t long_row;  // rows longer than this go to the block-cooperative loops
};

template <typename T>
__device__ inline T group_sum(T v, int G) {
  for (int o = G >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int BLOCK>
__device__ inline unsigned long long block_sum_u64(unsigned long long v, unsigned long long* red) {
  constexpr int NW = BLOCK / 64;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  unsigned long long t = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) t += red[w];
  __syncthreads();
  return t;
}

// Rows longer than LONG_ROW(BLOCK) entries are deferred from the lane-group loops to a
// block-cooperative loop, so one very popular node (d up to ~2e5 at config 2) cannot
// leave one wave working while the rest of the workgroup waits at the next barrier.
constexpr int LONG_LIST = 256;

template <int BLOCK, int CAP_WORDS>
__global__ __launch_bounds__(BLOCK) void k_score(ScoreArgs a) {
  constexpr int NW = BLOCK / 64;
  const int64_t CAP_BITS = a.cap_bits;
  const int64_t LONG_ROW = a.long_row;
  __shared__ uint32_t bm[CAP_WORDS];
  __shared__ unsigned long long red[NW];
  __shared__ double redd[NW];
  __shared__ int s_src;
  __shared__ int s_nlong;
  __shared__ int s_long[LONG_LIST];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int G = a.group;
  const int gpw = 64 / G;
  const int gid = lane / G, gl = lane - gid * G;
  const int n_groups = NW * gpw;
  const int my_group = wid * gpw + gid;
  const int64_t span = a.hi - a.lo;
  const int nchunks = span <= CAP_BITS ? 1 : (int)((span + CAP_BITS - 1) / CAP_BITS);
  const bool want_j = (a.mask & BLP_JACCARD) != 0;
  const bool want_a = (a.mask & BLP_ADAMIC) != 0;
  uint4* bm4 = reinterpret_cast<uint4*>(bm);

  for (;;) {
    if (threadIdx.x == 0) {
      s_src = atomicAdd(&a.misc->queue, 1);
      s_nlong = 0;
    }
    __syncthreads();
    const int s = s_src;
    if (s >= a.misc->n_active) break;
    const int x = a.active[s];
    const int pbeg = a.off[x], pcnt = a.cnt[x];
    const int64_t xb = a.rp[x], xe = a.rp[x + 1];
    unsigned long long h2 = 0;

    for (int ch = 0; ch < nchunks; ++ch) {
      const int64_t c0 = a.lo + (int64_t)ch * CAP_BITS;
      const int64_t c1 = min(a.hi, c0 + CAP_BITS);
      const int64_t width = max<int64_t>(c1 - c0, 0);
      const int nw4 = (int)((((width + 31) >> 5) + 3) >> 2);
      const bool last = ch == nchunks - 1;
      // 1. clear the chunk's words
      for (int i = threadIdx.x; i < nw4; i += BLOCK) bm4[i] = make_uint4(0, 0, 0, 0);
      __syncthreads();
      // 2. mark N(N(x)) within [c0, c1): short rows by lane groups, long rows deferred
      for (int64_t k = xb + my_group; k < xe; k += n_groups) {
        const int z = a.ci[k];
        const int64_t zb = a.rp[z], ze = a.rp[z + 1];
        if (ze - zb > LONG_ROW && gl == 0) {
          const int slot = atomicAdd(&s_nlong, 1);
          if (slot < LONG_LIST) s_long[slot] = z;
        }
        if (ze - zb > LONG_ROW) continue;  // deferred: block loop below (list or rescan)
        for (int64_t e = zb + gl; e < ze; e += G) {
          const int64_t r = (int64_t)a.ci[e] - c0;
          if (r >= 0 && r < width) atomicOr(&bm[r >> 5], 1u << (r & 31));
        }
      }
      __syncthreads();
      {
        const int nl = s_nlong;
        // overflowed long rows (more than LONG_LIST of them) are found again by a block scan
        if (nl > LONG_LIST) {
          for (int64_t k = xb; k < xe; ++k) {
            const int z = a.ci[k];
            const int64_t zb = a.rp[z], ze = a.rp[z + 1];
            if (ze - zb <= LONG_ROW) continue;
            for (int64_t e = zb + threadIdx.x; e < ze; e += BLOCK) {
              const int64_t r = (int64_t)a.ci[e] - c0;
              if (r >= 0 && r < width) atomicOr(&bm[r >> 5], 1u << (r & 31));
            }
          }
        } else {
          for (int l = 0; l < nl; ++l) {
            const int z = s_long[l];
            const int64_t zb = a.rp[z], ze = a.rp[z + 1];
            for (int64_t e = zb + threadIdx.x; e < ze; e += BLOCK) {
              const int64_t r = (int64_t)a.ci[e] - c0;
              if (r >= 0 && r < width) atomicOr(&bm[r >> 5], 1u << (r & 31));
            }
          }
        }
      }
      __syncthreads();
      if (threadIdx.x == 0) s_nlong = 0;
      // 3. exact distance 2: drop x (distance 0) and N(x) (distance 1)
      for (int64_t k = xb + threadIdx.x; k <= xe; k += BLOCK) {
        const int64_t r = (k == xe ? (int64_t)x : (int64_t)a.ci[k]) - c0;
        if (r >= 0 && r < width) atomicAnd(&bm[r >> 5], ~(1u << (r & 31)));
      }
      __syncthreads();
      // 4. |H2(x) ∩ chunk|
      if (want_j) {
        unsigned long long pc = 0;
        for (int i = threadIdx.x; i < nw4; i += BLOCK) {
          uint4 q = bm4[i];
          pc += __popc(q.x) + __popc(q.y) + __popc(q.z) + __popc(q.w);
        }
        h2 += block_sum_u64<BLOCK>(pc, red);
      }
      // 5. scan N(y) for every pair of x (long rows deferred to the block loop below)
      for (int j = my_group; j < pcnt; j += n_groups) {
        const int p = a.perm[pbeg + j];
        const int y = a.y[p];
        const int64_t yb = a.rp[y], ye = a.rp[y + 1];
        if (ye - yb > LONG_ROW) {
          if (gl == 0) {
            const int slot = atomicAdd(&s_nlong, 1);
            if (slot < LONG_LIST) s_long[slot] = j;
          }
          continue;
        }
        unsigned c = 0;
        double sw = 0.0;
        for (int64_t e = yb + gl; e < ye; e += G) {
          const int w = a.ci[e];
          const int64_t r = (int64_t)w - c0;
          if (r >= 0 && r < width && ((bm[r >> 5] >> (r & 31)) & 1u)) {
            ++c;
            if (want_a) sw += a.aaw[w];
          }
        }
        c = group_sum(c, G);
        if (want_a) sw = group_sum(sw, G);
        if (gl == 0) {
          if (ch > 0) {
            c += a.cn[p];
            if (want_a) sw += a.aa[p];
          }
          a.cn[p] = c;
          if (want_a) a.aa[p] = sw;
          if (want_j && last) {
            const long long uni = (long long)h2 + (ye - yb) - (long long)c;
            if (uni <= 0) {
              a.jac[p] = __builtin_nan("");
              atomicOr(&a.misc->zero_div, 1);
            } else {
              a.jac[p] = (double)c / (double)uni;
            }
          }
        }
      }
      __syncthreads();
      {
        const int nl = s_nlong;
        const int count = nl > LONG_LIST ? pcnt : nl;
        for (int l = 0; l < count; ++l) {
          const int j = nl > LONG_LIST ? l : s_long[l];
          const int p = a.perm[pbeg + j];
          const int y = a.y[p];
          const int64_t yb = a.rp[y], ye = a.rp[y + 1];
          if (ye - yb <= LONG_ROW) continue;  // only in the overflow rescan
          unsigned long long c = 0;
          double sw = 0.0;
          for (int64_t e = yb + threadIdx.x; e < ye; e += BLOCK) {
            const int w = a.ci[e];
            const int64_t r = (int64_t)w - c0;
            if (r >= 0 && r < width && ((bm[r >> 5] >> (r & 31)) & 1u)) {
              ++c;
              if (want_a) sw += a.aaw[w];
            }
          }
          c = block_sum_u64<BLOCK>(c, red);
          if (want_a) {
            for (int o = 32; o > 0; o >>= 1) sw += __shfl_xor(sw, o, 64);
            if (lane == 0) redd[wid] = sw;
            __syncthreads();
            sw = 0.0;
            for (int w2 = 0; w2 < NW; ++w2) sw += redd[w2];
            __syncthreads();
          }
          if (threadIdx.x == 0) {
            unsigned cc = (unsigned)c;
            if (ch > 0) {
              cc += a.cn[p];
              if (want_a) sw += a.aa[p];
            }
            a.cn[p] = cc;
            if (want_a) a.aa[p] = sw;
            if (want_j && last) {
              const long long uni = (long long)h2 + (ye - yb) - (long long)cc;
              if (uni <= 0) {
                a.jac[p] = __builtin_nan("");
                atomicOr(&a.misc->zero_div, 1);
              } else {
                a.jac[p] = (double)cc / (double)uni;
              }
            }
          }
        }
      }
      __syncthreads();
      if (threadIdx.x == 0) s_nlong = 0;
      __syncthreads();
    }
  }
}

enum Variant { V_SMALL = 0, V_MED = 1, V_LARGE = 2 };
constexpr int CAP_SMALL = 4096, CAP_MED = 16384, CAP_LARGE = 36864;  // words: 16 / 64 / 144 KiB
constexpr int BLOCK_SMALL = 256, BLOCK_MED = 512, BLOCK_LARGE = 1024;

}  // namespace

struct blp_batch {
  blp_graph* g = nullptr;
  int64_t n_pairs = 0;
  int32_t* d_x = nullptr;
  int32_t* d_y = nullptr;
  uint32_t* d_cn = nullptr;
  double* d_jac = nullptr;
  double* d_aa = nullptr;
  int32_t* d_perm = nullptr;
  Misc* d_misc = nullptr;
  int64_t lo = 0, hi = 0;
  int variant = V_SMALL;
  int group = 64;
  int chunks = 1;
  int64_t n_sources = 0;
  blp::KernelTimer t_score, t_group;
};

using namespace blp;

template <int BLOCK, int CAP>
static int launch_score(blp_graph* g, const ScoreArgs& a) {
  int per_cu = 0;
  BLP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_score<BLOCK, CAP>, BLOCK, 0));
  per_cu = std::max(per_cu, 1);
  const int grid = g->n_cu * per_cu;
  hipLaunchKernelGGL((k_score<BLOCK, CAP>), dim3(grid), dim3(BLOCK), 0, g->stream, a);
  BLP_HIP(hipGetLastError());
  return BLP_OK;
}

extern "C" {

int blp_batch_create(blp_graph* g, const int32_t* x, const int32_t* y, int64_t n_pairs, blp_batch** out) {
  BLP_CHECK(g && out && n_pairs >= 0 && (n_pairs == 0 || (x && y)), BLP_E_ARG, "blp_batch_create: bad arguments");
  BLP_CHECK(n_pairs < (int64_t(1) << 31) - 1, BLP_E_ARG, "blp_batch_create: at most 2^31-2 pairs per batch");
  const int64_t n = g->n;
  const int64_t* rp = g->h_rp.data();
  const int32_t* ci = g->h_ci.data();
  // ---- plan: node universe touched by H2(x) and N(y), lane group size
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  std::vector<uint8_t> seen((size_t)n, 0);
  double ysum = 0.0;
  int64_t n_src = 0;
  for (int64_t i = 0; i < n_pairs; ++i) {
    const int32_t xi = x[i], yi = y[i];
    if (xi < 0 || xi >= n || yi < 0 || yi >= n) return fail(BLP_E_ARG, "blp_batch_create: node id out of range");
    if (rp[yi + 1] > rp[yi]) {
      lo = std::min<int64_t>(lo, ci[rp[yi]]);
      hi = std::max<int64_t>(hi, (int64_t)ci[rp[yi + 1] - 1] + 1);
    }
    ysum += (double)(rp[yi + 1] - rp[yi]);
    if (!seen[xi]) {
      seen[xi] = 1;
      ++n_src;
      for (int64_t k = rp[xi]; k < rp[xi + 1]; ++k) {
        const int32_t z = ci[k];
        if (rp[z + 1] > rp[z]) {
          lo = std::min<int64_t>(lo, ci[rp[z]]);
          hi = std::max<int64_t>(hi, (int64_t)ci[rp[z + 1] - 1] + 1);
        }
      }
    }
  }
  if (lo > hi) lo = hi = 0;
  blp_batch* b = new blp_batch();
  b->g = g;
  b->n_pairs = n_pairs;
  b->lo = lo;
  b->hi = hi;
  b->n_sources = n_src;
  const int64_t span = hi - lo;
  if (span <= (int64_t)CAP_SMALL * 32)
    b->variant = V_SMALL;
  else if (span <= (int64_t)CAP_MED * 32)
    b->variant = V_MED;
  else
    b->variant = V_LARGE;
  int64_t cap_bits = 32ll * (b->variant == V_SMALL ? CAP_SMALL : b->variant == V_MED ? CAP_MED : CAP_LARGE);
  if (const char* e = getenv("BLP_CHUNK_BITS")) {
    int64_t v = atoll(e);
    if (v >= 128 && v % 128 == 0 && v < cap_bits) cap_bits = v;
  }
  b->chunks = span <= cap_bits ? 1 : (int)((span + cap_bits - 1) / cap_bits);
  const double ymean = n_pairs ? ysum / (double)n_pairs : 64.0;
  b->group = ymean >= 48 ? 64 : ymean >= 24 ? 32 : ymean >= 12 ? 16 : 8;
  if (const char* e = getenv("BLP_GROUP")) {
    int gsz = atoi(e);
    if (gsz == 8 || gsz == 16 || gsz == 32 || gsz == 64) b->group = gsz;
  }
  // ---- device buffers
  auto bail = [&](int rc) {
    blp_batch_destroy(b);
    return rc;
  };
  int rc = set_device(g);
  if (rc) return bail(rc);
  const size_t np = (size_t)std::max<int64_t>(n_pairs, 1);
  if (hipMalloc(&b->d_x, 4 * np) != hipSuccess || hipMalloc(&b->d_y, 4 * np) != hipSuccess ||
      hipMalloc(&b->d_cn, 4 * np) != hipSuccess || hipMalloc(&b->d_jac, 8 * np) != hipSuccess ||
      hipMalloc(&b->d_aa, 8 * np) != hipSuccess || hipMalloc(&b->d_perm, 4 * np) != hipSuccess ||
      hipMalloc(&b->d_misc, sizeof(Misc)) != hipSuccess)
    return bail(fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_batch_create: hipMalloc failed"));
  if (n_pairs) {
    if (hipMemcpy(b->d_x, x, 4 * n_pairs, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(b->d_y, y, 4 * n_pairs, hipMemcpyHostToDevice) != hipSuccess)
      return bail(fail(BLP_E_HIP_BASE, "blp_batch_create: upload failed"));
  }
  *out = b;
  return BLP_OK;
}

int blp_batch_destroy(blp_batch* b) {
  if (!b) return BLP_OK;
  if (b->g) (void)hipSetDevice(b->g->device);
  if (b->g && b->g->stream) (void)hipStreamSynchronize(b->g->stream);
  timer_release(b->t_score);
  timer_release(b->t_group);
  void* ps[] = {b->d_x, b->d_y, b->d_cn, b->d_jac, b->d_aa, b->d_perm, b->d_misc};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  delete b;
  return BLP_OK;
}

int blp_batch_plan(const blp_batch* b, int64_t* lo, int64_t* hi, int* chunks, int* block, int* group) {
  BLP_CHECK(b, BLP_E_ARG, "blp_batch_plan: null batch");
  if (lo) *lo = b->lo;
  if (hi) *hi = b->hi;
  if (chunks) *chunks = b->chunks;
  if (block) *block = b->variant == V_SMALL ? BLOCK_SMALL : b->variant == V_MED ? BLOCK_MED : BLOCK_LARGE;
  if (group) *group = b->group;
  return BLP_OK;
}

int blp_batch_score(blp_graph* g, blp_batch* b, uint32_t mask) {
  BLP_CHECK(g && b && b->g == g, BLP_E_ARG, "blp_batch_score: graph/batch mismatch");
  BLP_CHECK((mask & ~7u) == 0, BLP_E_ARG, "blp_batch_score: unknown method bits");
  BLP_CHECK(!(mask & BLP_ADAMIC) || g->d_aaw, BLP_E_STATE,
            "blp_batch_score: adamic_adar requested but the graph has no aa_weight table");
  int rc = set_device(g);
  if (rc) return rc;
  const int64_t n = g->n, np = b->n_pairs;
  const int64_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  if ((rc = g->cnt.reserve(4 * (n + 1)))) return rc;
  if ((rc = g->off.reserve(4 * (n + 1)))) return rc;
  if ((rc = g->cursor.reserve(4 * (n + 1)))) return rc;
  if ((rc = g->active.reserve(4 * (n + 1)))) return rc;
  if ((rc = g->scratch.reserve(sizeof(int2) * (ntiles + 1)))) return rc;
  hipEvent_t t0, bt0;
  if ((rc = timer_begin(g, K_GROUP, &t0))) return rc;
  if ((rc = timer_begin(b->t_group, g->stream, &bt0))) return rc;
  BLP_HIP(hipMemsetAsync(g->cnt.p, 0, 4 * (n + 1), g->stream));
  BLP_HIP(hipMemsetAsync(b->d_misc, 0, sizeof(Misc), g->stream));
  const int ew_grid = (int)std::min<int64_t>(std::max<int64_t>((np + 255) / 256, 1), (int64_t)g->n_cu * 16);
  if (np) hipLaunchKernelGGL(k_count, dim3(ew_grid), dim3(256), 0, g->stream, b->d_x, np, g->cnt.as<int32_t>());
  if (ntiles) {
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)ntiles), dim3(SCAN_BLOCK), 0, g->stream, g->cnt.as<int32_t>(), n,
                       g->scratch.as<int2>());
    hipLaunchKernelGGL(k_scan_tilesums, dim3(1), dim3(SCAN_BLOCK), 0, g->stream, g->scratch.as<int2>(), ntiles,
                       b->d_misc);
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)ntiles), dim3(SCAN_BLOCK), 0, g->stream, g->cnt.as<int32_t>(), n,
                       g->scratch.as<int2>(), g->off.as<int32_t>(), g->cursor.as<int32_t>(), g->active.as<int32_t>());
  }
  if (np) hipLaunchKernelGGL(k_scatter, dim3(ew_grid), dim3(256), 0, g->stream, b->d_x, np, g->cursor.as<int32_t>(), b->d_perm);
  BLP_HIP(hipGetLastError());
  if ((rc = timer_end(b->t_group, g->stream, bt0))) return rc;
  if ((rc = timer_end(g, K_GROUP, t0))) return rc;

  ScoreArgs a;
  a.rp = g->d_rp;
  a.ci = g->d_ci;
  a.aaw = g->d_aaw;
  a.y = b->d_y;
  a.perm = b->d_perm;
  a.off = g->off.as<int32_t>();
  a.cnt = g->cnt.as<int32_t>();
  a.active = g->active.as<int32_t>();
  a.misc = b->d_misc;
  a.cn = b->d_cn;
  a.jac = b->d_jac;
  a.aa = b->d_aa;
  a.lo = b->lo;
  a.hi = b->hi;
  a.mask = mask | BLP_CN;  // counts are always produced (Jaccard needs them)
  a.group = b->group;
  const int block = b->variant == V_SMALL ? BLOCK_SMALL : b->variant == V_MED ? BLOCK_MED : BLOCK_LARGE;
  a.cap_bits = 32ll * (b->variant == V_SMALL ? CAP_SMALL : b->variant == V_MED ? CAP_MED : CAP_LARGE);
  a.long_row = block;
  if (const char* e = getenv("BLP_CHUNK_BITS")) {  // test knob: force multi-chunk on small graphs
    int64_t v = atoll(e);
    if (v >= 128 && v % 128 == 0 && v < a.cap_bits) a.cap_bits = v;
  }
  if (const char* e = getenv("BLP_LONG_ROW")) {  // test knob: exercise the deferred-row loops
    int64_t v = atoll(e);
    if (v >= 1) a.long_row = v;
  }
  hipEvent_t t1, bt1;
  if ((rc = timer_begin(g, K_SCORE, &t1))) return rc;
  if ((rc = timer_begin(b->t_score, g->stream, &bt1))) return rc;
  if (np) {
    if (b->variant == V_SMALL)
      rc = launch_score<BLOCK_SMALL, CAP_SMALL>(g, a);
    else if (b->variant == V_MED)
      rc = launch_score<BLOCK_MED, CAP_MED>(g, a);
    else
      rc = launch_score<BLOCK_LARGE, CAP_LARGE>(g, a);
    if (rc) return rc;
  }
  if ((rc = timer_end(b->t_score, g->stream, bt1))) return rc;
  return timer_end(g, K_SCORE, t1);
}

int blp_batch_stats(blp_batch* b, int which, double* total_ms, int64_t* launches) {
  BLP_CHECK(b && (which == 0 || which == 1), BLP_E_ARG, "blp_batch_stats: bad arguments");
  KernelTimer& t = which == 0 ? b->t_score : b->t_group;
  int rc = set_device(b->g);
  if (rc) return rc;
  if ((rc = timer_collect(t))) return rc;
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
    t->total_ms = 0;
    t->launches = 0;
  }
  return BLP_OK;
}

int blp_batch_fetch(blp_graph* g, blp_batch* b, uint32_t* cn, double* jac, double* aa) {
  BLP_CHECK(g && b && b->g == g, BLP_E_ARG, "blp_batch_fetch: graph/batch mismatch");
  int rc = set_device(g);
  if (rc) return rc;
  BLP_HIP(hipStreamSynchronize(g->stream));
  const int64_t np = b->n_pairs;
  Misc m;
  BLP_HIP(hipMemcpy(&m, b->d_misc, sizeof(Misc), hipMemcpyDeviceToHost));
  if (np) {
    if (cn) BLP_HIP(hipMemcpy(cn, b->d_cn, 4 * np, hipMemcpyDeviceToHost));
    if (jac) BLP_HIP(hipMemcpy(jac, b->d_jac, 8 * np, hipMemcpyDeviceToHost));
    if (aa) BLP_HIP(hipMemcpy(aa, b->d_aa, 8 * np, hipMemcpyDeviceToHost));
  }
  if (m.zero_div && jac) return fail(BLP_E_ZERODIV, "float division by zero (Jaccard union is empty)");
  return BLP_OK;
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
