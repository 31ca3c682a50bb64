// Hop-3 candidate generation (dataset_maker.make_examples, dataset_maker.py:137-144).
//
// For each sampled source u:  H3(u) = GetNodesAtHop(G, u, 3) (nodes at EXACT distance 3,
// :139). A candidate b is labelled 1 if (u, b) is a held-out new edge (:141-142), else kept
// as a negative with probability `rate` (:143-144). The reference draws Python's
// random.random() in SNAP's BFS order; here the draw is a counter-based hash of
// (seed, u, b), so the kept set is reproducible and order-independent (the sample itself is
// statistical parity only; the candidate SET is exact -- tested with rate = 1).
//
// One workgroup per source (dequeued), two LDS bitmaps: H2(u) over [lo2, hi2) and the
// distance-3 marks over [lo3, hi3). Positives are emitted first (in the caller's order),
// then the sampled negatives in ascending dense id.
#include <algorithm>
#include <cstdlib>

#include "blp_internal.h"

#ifndef BLP_HOP3_TEST
#define BLP_HOP3_TEST 1  // k_hop3_wedge: read a word before OR-ing into it (0: OR every id)
#endif

namespace {

constexpr int H_BLOCK = 1024;
constexpr int H_WORDS = 39936;  // 156 KiB of LDS shared by the two bitmaps

struct Hop3Args {
  const int64_t* rp;
  const int32_t* ci;
  const int32_t* src;      // sources (dense ids)
  const int32_t* pos_off;  // [n_src+1] positives per source
  const int32_t* pos_y;    // positive targets
  int n_src;
  int64_t lo2, hi2, lo3, hi3;
  int w2;  // words of the H2 bitmap (the H3 bitmap follows)
  double rate;
  uint64_t seed;
  int32_t* out_x;
  int32_t* out_y;
  uint8_t* out_label;
  int64_t cap;
  unsigned long long* counters;  // [0] queue, [1] emitted
  const int32_t* wbm_slot;       // wedge-row bitmaps (k_hop3_wedge): slot of b or -1; null: none
  const uint4* wbm_pool;         // [slots][wbm_vecs]
  int wbm_vecs;
};

__device__ inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ inline bool keep_negative(uint64_t seed, int u, int b, double rate) {
  const uint64_t h = mix64(seed ^ mix64(((uint64_t)(uint32_t)u << 32) | (uint32_t)b));
  return (double)(h >> 11) * 0x1.0p-53 < rate;
}

__device__ inline bool bit_test(const uint32_t* bm, int64_t r) { return (bm[r >> 5] >> (r & 31)) & 1u; }

// The two bitmaps live in LDS, or -- universes wider than LDS (configs 4/5) -- in a private
// HBM slot per workgroup: workgroup-scope atomics (done in the XCD's L2) and agent-scope fences
// between phases (drain the stores, invalidate the CU's L1), as k_score_global (pairs.hip).
template <bool G>
__device__ inline void bit_or(uint32_t* p, uint32_t v) {
  if (G)
    __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else
    atomicOr(p, v);
}

template <bool G>
__device__ inline void bit_and(uint32_t* p, uint32_t v) {
  if (G)
    __hip_atomic_fetch_and(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else
    atomicAnd(p, v);
}

template <bool G>
__device__ inline void phase_sync() {
  if (G) __threadfence();
  __syncthreads();
}

// Emission of one source's candidates (after the exact distance-3 marks are final in bm3):
// positives first, in the caller's order, cleared from the marks; then the sampled negatives,
// each thread a contiguous word range so the ids come out ascending.
template <bool G, int NT>
__device__ inline void emit(const Hop3Args& a, int it, int x, uint32_t* bm3, int w3, int64_t span3, unsigned* s_warp,
                            unsigned long long* s_base_p) {
  unsigned long long& s_base = *s_base_p;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // positives first (caller order), cleared from the candidate marks
  const int pb = a.pos_off[it], pe = a.pos_off[it + 1];
  if (threadIdx.x == 0) {
    for (int k = pb; k < pe; ++k) {
      const int64_t r = (int64_t)a.pos_y[k] - a.lo3;
      if (r >= 0 && r < span3 && bit_test(bm3, r)) {
        bm3[r >> 5] &= ~(1u << (r & 31));
        const unsigned long long o = atomicAdd(&a.counters[1], 1ull);
        if ((int64_t)o < a.cap) {
          a.out_x[o] = x;
          a.out_y[o] = a.pos_y[k];
          a.out_label[o] = 1;
        }
      }
    }
  }
  phase_sync<G>();
  // sampled negatives: per-thread contiguous word ranges keep ascending id order
  const int per = (w3 + NT - 1) / NT;
  const int w_beg = min(w3, (int)threadIdx.x * per), w_end = min(w3, w_beg + per);
  unsigned mine = 0;
  for (int wi = w_beg; wi < w_end; ++wi) {
    uint32_t bits = bm3[wi];
    while (bits) {
      const int t = __ffs(bits) - 1;
      bits &= bits - 1;
      if (keep_negative(a.seed, x, (int)(a.lo3 + (int64_t)wi * 32 + t), a.rate)) ++mine;
    }
  }
  // block exclusive scan of the per-thread counts
  unsigned inc = mine;
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned t = __shfl_up(inc, d, 64);
    if (lane >= d) inc += t;
  }
  if (lane == 63) s_warp[wid] = inc;
  phase_sync<G>();
  if (threadIdx.x == 0) {
    unsigned run = 0;
    for (int w = 0; w < NT / 64; ++w) {
      const unsigned t = s_warp[w];
      s_warp[w] = run;
      run += t;
    }
    s_base = atomicAdd(&a.counters[1], (unsigned long long)run);
  }
  phase_sync<G>();
  unsigned long long o = s_base + s_warp[wid] + inc - mine;
  for (int wi = w_beg; wi < w_end; ++wi) {
    uint32_t bits = bm3[wi];
    while (bits) {
      const int t = __ffs(bits) - 1;
      bits &= bits - 1;
      const int b = (int)(a.lo3 + (int64_t)wi * 32 + t);
      if (keep_negative(a.seed, x, b, a.rate)) {
        if ((int64_t)o < a.cap) {
          a.out_x[o] = x;
          a.out_y[o] = b;
          a.out_label[o] = 0;
        }
        ++o;
      }
    }
  }
}

template <bool G>
__global__ __launch_bounds__(H_BLOCK) void k_hop3(Hop3Args a, uint32_t* gbm, int64_t gwords) {
  uint32_t* lds;
  if constexpr (G) {
    lds = gbm + (int64_t)blockIdx.x * gwords;
  } else {
    __shared__ uint32_t lds_bm[H_WORDS];
    lds = lds_bm;
  }
  __shared__ int s_item;
  __shared__ unsigned s_warp[H_BLOCK / 64];
  __shared__ unsigned long long s_base;
  uint32_t* bm2 = lds;
  uint32_t* bm3 = lds + a.w2;
  const int64_t span2 = a.hi2 - a.lo2, span3 = a.hi3 - a.lo3;
  const int w3 = (int)((span3 + 31) >> 5);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (;;) {
    if (threadIdx.x == 0) s_item = (int)atomicAdd(&a.counters[0], 1ull);
    phase_sync<G>();
    const int it = s_item;
    if (it >= a.n_src) break;
    const int x = a.src[it];
    for (int i = threadIdx.x; i < a.w2 + w3; i += H_BLOCK) lds[i] = 0;
    phase_sync<G>();
    const int64_t xb = a.rp[x], xe = a.rp[x + 1];
    // H2 marks: N(N(x)); one wave per z, lanes stride the row
    for (int64_t k = xb + wid; k < xe; k += H_BLOCK / 64) {
      const int z = a.ci[k];
      for (int64_t e = a.rp[z] + lane; e < a.rp[z + 1]; e += 64) {
        const int64_t r = (int64_t)a.ci[e] - a.lo2;
        if (r >= 0 && r < span2) bit_or<G>(&bm2[r >> 5], 1u << (r & 31));
      }
    }
    phase_sync<G>();
    for (int64_t k = xb + threadIdx.x; k <= xe; k += H_BLOCK) {
      const int64_t r = (k == xe ? (int64_t)x : (int64_t)a.ci[k]) - a.lo2;
      if (r >= 0 && r < span2) bit_and<G>(&bm2[r >> 5], ~(1u << (r & 31)));
    }
    phase_sync<G>();
    // distance-3 marks: N(H2(x)); each thread walks the set bits of its H2 words
    for (int wi = threadIdx.x; wi < a.w2; wi += H_BLOCK) {
      uint32_t bits = bm2[wi];
      while (bits) {
        const int t = __ffs(bits) - 1;
        bits &= bits - 1;
        const int w = (int)(a.lo2 + (int64_t)wi * 32 + t);
        for (int64_t e = a.rp[w]; e < a.rp[w + 1]; ++e) {
          const int64_t r = (int64_t)a.ci[e] - a.lo3;
          if (r >= 0 && r < span3) bit_or<G>(&bm3[r >> 5], 1u << (r & 31));
        }
      }
    }
    phase_sync<G>();
    // exact distance: drop x, N(x) and H2(x) from the distance-3 marks
    for (int64_t k = xb + threadIdx.x; k <= xe; k += H_BLOCK) {
      const int64_t r = (k == xe ? (int64_t)x : (int64_t)a.ci[k]) - a.lo3;
      if (r >= 0 && r < span3) bit_and<G>(&bm3[r >> 5], ~(1u << (r & 31)));
    }
    // H2 ∩ [lo3, hi3) (general graphs only: the ranges are disjoint for bipartite files)
    {
      const int64_t olo = max(a.lo2, a.lo3), ohi = min(a.hi2, a.hi3);
      for (int64_t v = olo + threadIdx.x; v < ohi; v += H_BLOCK)
        if (bit_test(bm2, v - a.lo2)) bit_and<G>(&bm3[(v - a.lo3) >> 5], ~(1u << ((v - a.lo3) & 31)));
    }
    phase_sync<G>();
    emit<G, H_BLOCK>(a, it, x, bm3, w3, span3, s_warp, &s_base);
    phase_sync<G>();
  }
}

// Wedge-row variant (bipartite review graphs; the graph's wedge index, wedge.hip): for a user
// x, N(N(N(x))) = the union over b in N(x) of b's wedge row (the rows N(z), z in N(b), stored
// back to back), so the distance-3 marks come from contiguous 16-byte vectors -- no H2 bitmap,
// no per-member row_ptr gathers and no one-id-per-load row walks (the row walk of k_hop3 moved
// 2-4x its algorithmic bytes). Exact distance 3 = marks minus N(x): x and every distance-2 node
// lie in N(N(x)), whose id range the host checked to be disjoint from the marks' range.
// Work items are chunks of HW_CH vectors of one wedge row, one wave each, four vectors per lane
// in flight; the mark bitmap is dynamic LDS sized to the target range.
constexpr int HW_BLOCK = 1024;
constexpr int HW_SEG = 1024;  // N(x) entries per batch
constexpr int HW_CH = 1024;   // wedge vectors per work item
extern __shared__ uint32_t hw_dyn[];

__device__ inline int hw_exscan(int v, int* red, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = v;
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(inc, d, 64);
    if (lane >= d) inc += t;
  }
  if (lane == 63) red[wid] = inc;
  __syncthreads();
  int base = 0, tot = 0;
  for (int w = 0; w < HW_BLOCK / 64; ++w) {
    base += w < wid ? red[w] : 0;
    tot += red[w];
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

__global__ __launch_bounds__(HW_BLOCK) void k_hop3_wedge(Hop3Args a, const int64_t* __restrict__ wp,
                                                         const uint4* __restrict__ wedge) {
  __shared__ int64_t s_ws[HW_SEG];
  __shared__ int32_t s_wl[HW_SEG];
  __shared__ int32_t s_co[HW_SEG + 1];
  __shared__ int red[HW_BLOCK / 64];
  __shared__ int s_item;
  __shared__ unsigned s_warp[HW_BLOCK / 64];
  __shared__ unsigned long long s_base;
  uint32_t* bm3 = hw_dyn;
  const int64_t span3 = a.hi3 - a.lo3;
  const int w3 = (int)((span3 + 31) >> 5);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t c0u = (uint32_t)a.lo3, wu = (uint32_t)span3;
  for (;;) {
    if (threadIdx.x == 0) s_item = (int)atomicAdd(&a.counters[0], 1ull);
    __syncthreads();
    const int it = s_item;
    if (it >= a.n_src) break;
    const int x = a.src[it];
    for (int i = threadIdx.x; i < w3; i += HW_BLOCK) bm3[i] = 0;
    const int64_t xb = a.rp[x], xe = a.rp[x + 1];
    __syncthreads();
    for (int64_t k0 = xb; k0 < xe; k0 += HW_SEG) {
      const int ns = (int)min<int64_t>(HW_SEG, xe - k0);
      int nch = 0;
      if ((int)threadIdx.x < ns) {
        const int b = a.ci[k0 + threadIdx.x];
        const int slot = a.wbm_slot ? a.wbm_slot[b] : -1;
        if (slot >= 0) {  // the row's id set as a bitmap: its words, negative length marks it
          s_ws[threadIdx.x] = (int64_t)slot * a.wbm_vecs;
          s_wl[threadIdx.x] = -a.wbm_vecs;
          nch = (a.wbm_vecs + HW_CH - 1) / HW_CH;
        } else {
          const int64_t ws = wp[b], we = wp[b + 1];
          s_ws[threadIdx.x] = ws;
          s_wl[threadIdx.x] = (int)(we - ws);
          nch = (int)((we - ws + HW_CH - 1) / HW_CH);
        }
      }
      int tot;
      const int ex = hw_exscan(nch, red, &tot);
      if ((int)threadIdx.x < ns) s_co[threadIdx.x] = ex;
      if (threadIdx.x == 0) s_co[ns] = tot;
      __syncthreads();
      for (int item = wid; item < tot; item += HW_BLOCK / 64) {
        int lo = 0, hi = ns;  // the row of this item: last lo with s_co[lo] <= item
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (s_co[mid] <= item) lo = mid; else hi = mid;
        }
        if (s_wl[lo] < 0) {  // a wedge-row bitmap: OR its nonzero words (consecutive: no bank conflicts)
          const int64_t b0 = s_ws[lo], vb = (int64_t)(item - s_co[lo]) * HW_CH;
          const int64_t ve = min<int64_t>(vb + HW_CH, -s_wl[lo]);
          for (int64_t q = vb + lane; q < ve; q += 64) {
            const uint4 v = a.wbm_pool[b0 + q];
            uint32_t* d = bm3 + 4 * q;
            if (v.x) atomicOr(d, v.x);
            if (v.y) atomicOr(d + 1, v.y);
            if (v.z) atomicOr(d + 2, v.z);
            if (v.w) atomicOr(d + 3, v.w);
          }
          continue;
        }
        const int64_t row_end = s_ws[lo] + s_wl[lo];
        const int64_t base = s_ws[lo] + (int64_t)(item - s_co[lo]) * HW_CH;
        const int64_t end = min(base + HW_CH, row_end);
        for (int64_t q = base + lane; q < end; q += 4 * 64) {
          uint4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = wedge[q + 64 * u < end ? q + 64 * u : q];  // a repeat ORs nothing new
#if BLP_HOP3_TEST
          // Read before OR: the wedge rows repeat the popular targets in nearly every row, so
          // their words are set early and most ORs would be redundant -- and the 64 lanes of an
          // OR to one hot word serialise on its bank. Reads of one address broadcast, so the
          // words are read first (all 16 in one LDS round trip) and only lanes whose bit is
          // still clear OR it in (a stale read only costs a redundant, harmless OR).
          uint32_t rr[16], wd[16];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            rr[4 * u] = v[u].x - c0u;
            rr[4 * u + 1] = v[u].y - c0u;
            rr[4 * u + 2] = v[u].z - c0u;
            rr[4 * u + 3] = v[u].w - c0u;
          }
#pragma unroll
          for (int c = 0; c < 16; ++c) wd[c] = bm3[(rr[c] < wu ? rr[c] : 0u) >> 5];
#pragma unroll
          for (int c = 0; c < 16; ++c)
            if (rr[c] < wu && !((wd[c] >> (rr[c] & 31)) & 1u)) atomicOr(&bm3[rr[c] >> 5], 1u << (rr[c] & 31));
#else
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t ids[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const uint32_t r = ids[c] - c0u;
              if (r < wu) atomicOr(&bm3[r >> 5], 1u << (r & 31));
            }
          }
#endif
        }
      }
      __syncthreads();
    }
    // exact distance 3: drop N(x) (distance 1); x and H2(x) lie outside [lo3, hi3)
    for (int64_t k = xb + threadIdx.x; k < xe; k += HW_BLOCK) {
      const uint32_t r = (uint32_t)a.ci[k] - c0u;
      if (r < wu) atomicAnd(&bm3[r >> 5], ~(1u << (r & 31)));
    }
    __syncthreads();
    emit<false, HW_BLOCK>(a, it, x, bm3, w3, span3, s_warp, &s_base);
    __syncthreads();
  }
}

// Wedge-row bitmaps. A popular business b's wedge row holds |N(z)| ids for each of its
// members z -- millions at config 2 -- yet only its SET W(b) = N(N(b)) matters for the marks, and
// that set lives in a range of w3 words (12.5 KB at config 2). Every source reviewing b streamed
// the whole row (k_hop3_wedge read ~37 GB per call for 0.44 GB of wedge rows). Rows longer than
// their bitmap are OR-ed once into one bitmap each (this kernel, one workgroup per row); the
// hop-3 kernel then ORs those words instead. Same set, so the same marks.
__global__ __launch_bounds__(HW_BLOCK) void k_wbm_fill(const int64_t* __restrict__ wp, const uint4* __restrict__ wedge,
                                                       const int32_t* __restrict__ rows, int64_t lo3, int64_t span3,
                                                       int words, uint32_t* __restrict__ pool) {
  uint32_t* bm = hw_dyn;
  const int b = rows[blockIdx.x];
  for (int i = threadIdx.x; i < words; i += HW_BLOCK) bm[i] = 0;
  __syncthreads();
  const uint32_t c0u = (uint32_t)lo3, wu = (uint32_t)span3;
  const int64_t s = wp[b], e = wp[b + 1];
  for (int64_t q = s + threadIdx.x; q < e; q += 4 * HW_BLOCK) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = wedge[q + HW_BLOCK * u < e ? q + HW_BLOCK * u : q];  // a repeat ORs nothing new
    uint32_t rr[16], wd[16];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      rr[4 * u] = v[u].x - c0u;
      rr[4 * u + 1] = v[u].y - c0u;
      rr[4 * u + 2] = v[u].z - c0u;
      rr[4 * u + 3] = v[u].w - c0u;
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) wd[c] = bm[(rr[c] < wu ? rr[c] : 0u) >> 5];
#pragma unroll
    for (int c = 0; c < 16; ++c)
      if (rr[c] < wu && !((wd[c] >> (rr[c] & 31)) & 1u)) atomicOr(&bm[rr[c] >> 5], 1u << (rr[c] & 31));
  }
  __syncthreads();
  uint32_t* dst = pool + (int64_t)blockIdx.x * words;
  for (int i = threadIdx.x; i < words; i += HW_BLOCK) dst[i] = bm[i];
}

// The dense wedge-set index (blp_internal.h WedgeSets): one workgroup per node c of [lo, lo + n):
// W(c) = the set of ids of c's wedge row inside [lo, hi), OR-ed in LDS (a word is read before its
// bit is OR-ed: a wedge row repeats the popular ids of its member rows), then written out whole,
// with |W(c) \ {c}| counted on the way.
__global__ __launch_bounds__(HW_BLOCK) void k_wset_fill(const int64_t* __restrict__ wp, const uint4* __restrict__ wedge,
                                                        int64_t lo, int64_t span, int words, uint32_t* __restrict__ pool,
                                                        int32_t* __restrict__ h2) {
  uint32_t* bm = hw_dyn;
  __shared__ unsigned red[HW_BLOCK / 64];
  const int64_t c = lo + blockIdx.x;
  for (int i = threadIdx.x; i < words; i += HW_BLOCK) bm[i] = 0;
  __syncthreads();
  const uint32_t c0u = (uint32_t)lo, wu = (uint32_t)span;
  const int64_t s = wp[c], e = wp[c + 1];
  for (int64_t q = s + threadIdx.x; q < e; q += 4 * HW_BLOCK) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = wedge[q + HW_BLOCK * u < e ? q + HW_BLOCK * u : q];  // a repeat ORs nothing new
    uint32_t rr[16], wd[16];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      rr[4 * u] = v[u].x - c0u;
      rr[4 * u + 1] = v[u].y - c0u;
      rr[4 * u + 2] = v[u].z - c0u;
      rr[4 * u + 3] = v[u].w - c0u;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) wd[k] = bm[(rr[k] < wu ? rr[k] : 0u) >> 5];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (rr[k] < wu && !((wd[k] >> (rr[k] & 31)) & 1u)) atomicOr(&bm[rr[k] >> 5], 1u << (rr[k] & 31));
  }
  __syncthreads();
  uint32_t* dst = pool + (int64_t)blockIdx.x * words;
  unsigned cnt = 0;
  for (int i = threadIdx.x; i < words; i += HW_BLOCK) {
    const uint32_t w = bm[i];
    dst[i] = w;
    cnt += __popc(w);
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = 0;
    for (int w = 0; w < HW_BLOCK / 64; ++w) t += red[w];
    const uint32_t own = (bm[blockIdx.x >> 5] >> (blockIdx.x & 31)) & 1u;  // c itself (distance 0)
    h2[blockIdx.x] = (int32_t)(t - own);
  }
}

}  // namespace

using namespace blp;

// The graph's wedge-row bitmaps over [lo, hi) (blp_internal.h), built on first use: rows of at
// least BLP_WBM_MIN_X (default 1) times their bitmap's words, longest first, within BLP_WBM_MB of
// HBM (default 2048) per range; at most 4 ranges are kept per graph.
namespace blp {
const WedgeBitmaps* wedge_bitmaps(blp_graph* g, int64_t lo, int64_t hi, int* rc) {
  *rc = BLP_OK;
  if (!g->d_wp || hi <= lo) return nullptr;
  // two batches of one graph may be created on two host threads at once (similarity.py's user and
  // business passes): the whole lookup-or-build is one critical section
  std::lock_guard<std::mutex> lock(g->wbm_mu);
  for (const WedgeBitmaps& w : g->wbm)
    if (w.lo == lo && w.hi == hi) return &w;
  if (g->wbm.size() >= 4) return nullptr;
  g->wbm.reserve(4);  // entries never move: batches keep their device pointers
  const int64_t words = (((hi - lo) + 31) / 32 + 3) / 4 * 4;
  const double min_x = getenv("BLP_WBM_MIN_X") ? atof(getenv("BLP_WBM_MIN_X")) : 1.0;
  const int64_t budget = (getenv("BLP_WBM_MB") ? atoll(getenv("BLP_WBM_MB")) : 2048) << 20;
  std::vector<std::pair<int64_t, int32_t>> rows;  // (-ids, x)
  for (int64_t x = 0; x < g->n; ++x) {
    const int64_t ids = 4 * (g->h_wp[x + 1] - g->h_wp[x]);
    if (ids > 0 && (double)ids >= min_x * (double)words) rows.push_back({-ids, (int32_t)x});
  }
  std::sort(rows.begin(), rows.end());
  rows.resize((size_t)std::min<int64_t>((int64_t)rows.size(), budget / (4 * words)));
  // built into a local entry; it joins the cache only once complete, so a failure leaves no
  // half-built entry behind and frees what it allocated
  WedgeBitmaps w;
  w.lo = lo;
  w.hi = hi;
  w.words = words;
  if (!rows.empty()) {
    w.h_slot.assign((size_t)g->n, -1);
    std::vector<int32_t> order(rows.size());
    for (size_t i = 0; i < rows.size(); ++i) {
      w.h_slot[rows[i].second] = (int32_t)i;
      order[i] = rows[i].second;
    }
    ScopedBuf d_rows;
    auto hip = [&](hipError_t e, const char* what) {
      if (e != hipSuccess) *rc = hip_fail(e, what, __FILE__, __LINE__);
      return e == hipSuccess;
    };
    bool ok = hip(dev_malloc(&w.d_slot, 4 * (size_t)g->n), "hipMalloc") &&
              hip(dev_malloc(&w.d_pool, 4 * (size_t)words * rows.size()), "hipMalloc (wedge bitmaps)");
    if (ok && (*rc = d_rows.reserve(4 * rows.size())) != BLP_OK) ok = false;
    ok = ok && hip(hipMemcpy(w.d_slot, w.h_slot.data(), 4 * (size_t)g->n, hipMemcpyHostToDevice), "hipMemcpy") &&
         hip(hipMemcpy(d_rows.p, order.data(), 4 * order.size(), hipMemcpyHostToDevice), "hipMemcpy");
    if (ok) {
      hipLaunchKernelGGL(k_wbm_fill, dim3((unsigned)rows.size()), dim3(HW_BLOCK), 4 * (size_t)words, g->stream,
                         (const int64_t*)g->d_wp, (const uint4*)g->d_wedge, d_rows.as<int32_t>(), lo, hi - lo,
                         (int)words, w.d_pool);
      ok = hip(hipGetLastError(), "k_wbm_fill launch") && hip(hipStreamSynchronize(g->stream), "hipStreamSynchronize");
    }
    d_rows.release();
    if (!ok) {
      if (w.d_slot) (void)hipFree(w.d_slot);
      if (w.d_pool) (void)hipFree(w.d_pool);
      return nullptr;
    }
    w.slots = (int64_t)rows.size();
  }
  g->wbm.push_back(std::move(w));
  return &g->wbm.back();
}
const WedgeSets* wedge_sets(blp_graph* g, int64_t lo, int64_t hi, int* rc) {
  *rc = BLP_OK;
  if (!g->d_wp || hi <= lo || getenv("BLP_NO_WSET")) return nullptr;
  std::lock_guard<std::mutex> lock(g->wbm_mu);
  if (g->wset) return g->wset->lo == lo && g->wset->hi == hi ? g->wset : nullptr;
  const int64_t span = hi - lo, words = (span + 31) / 32;
  if (span >= (int64_t(1) << 31) || words > 16 * 1024) return nullptr;  // one LDS bitmap per node (<= 64 KiB)
  // every node of the range with neighbours needs its wedge row (the set is built from it)
  for (int64_t c = lo; c < hi; ++c)
    if (g->hrp[c + 1] > g->hrp[c] && g->h_wp[c + 1] == g->h_wp[c]) return nullptr;
  const double bytes = 4.0 * (double)words * (double)span + 4.0 * (double)span;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  free_b += dev_cache_bytes(g->device);
  const double budget = std::min((double)((getenv("BLP_WSET_MB") ? atoll(getenv("BLP_WSET_MB")) : 4096) << 20),
                                 0.25 * (double)free_b);
  if (bytes > budget) return nullptr;
  auto* w = new WedgeSets();
  w->lo = lo;
  w->hi = hi;
  w->words = words;
  auto hip = [&](hipError_t e, const char* what) {
    if (e != hipSuccess) *rc = hip_fail(e, what, __FILE__, __LINE__);
    return e == hipSuccess;
  };
  bool ok = hip(dev_malloc(&w->d_pool, 4 * (size_t)words * (size_t)span), "hipMalloc (wedge sets)") &&
            hip(dev_malloc(&w->d_h2, 4 * (size_t)span), "hipMalloc (wedge-set sizes)");
  if (ok) {
    hipLaunchKernelGGL(k_wset_fill, dim3((unsigned)span), dim3(HW_BLOCK), 4 * (size_t)words, g->stream,
                       (const int64_t*)g->d_wp, (const uint4*)g->d_wedge, lo, span, (int)words, w->d_pool, w->d_h2);
    ok = hip(hipGetLastError(), "k_wset_fill launch") && hip(hipStreamSynchronize(g->stream), "hipStreamSynchronize");
  }
  if (!ok) {
    if (w->d_pool) (void)hipFree(w->d_pool);
    if (w->d_h2) (void)hipFree(w->d_h2);
    delete w;
    if (*rc == BLP_E_HIP_BASE - (int)hipErrorOutOfMemory) {  // no room: the batch takes the grouped path
      (void)hipGetLastError();
      *rc = BLP_OK;
    }
    return nullptr;
  }
  g->wset = w;
  return w;
}

}  // namespace blp

extern "C" int blp_hop3_sample(blp_graph* g, const int32_t* src, int64_t n_src, const int32_t* pos_off,
                               const int32_t* pos_y, double rate, uint64_t seed, int32_t* out_x, int32_t* out_y,
                               uint8_t* out_label, int64_t cap, int64_t* n_out) {
  BLP_CHECK(g && n_out && n_src >= 0 && (n_src == 0 || (src && pos_off)), BLP_E_ARG, "blp_hop3_sample: bad arguments");
  BLP_CHECK(n_src < (int64_t(1) << 31), BLP_E_ARG, "blp_hop3_sample: too many sources");
  BLP_CHECK(cap == 0 || (out_x && out_y && out_label), BLP_E_ARG, "blp_hop3_sample: null outputs");
  const int64_t* rp = g->hrp;
  const int32_t* ci = host_col_idx(g);
  if (!ci) return BLP_E_STATE;
  const int64_t n = g->n;
  // plan the two universes: H2 ⊂ N(N(x)), distance-3 marks ⊂ N(H2) ⊂ the rows' neighbour ranges
  int64_t lo2 = INT64_MAX, hi2 = INT64_MIN;
  for (int64_t i = 0; i < n_src; ++i) {
    const int32_t x = src[i];
    if (x < 0 || x >= n) return fail(BLP_E_ARG, "blp_hop3_sample: source id out of range");
    for (int64_t k = rp[x]; k < rp[x + 1]; ++k) {
      const int32_t z = ci[k];
      if (rp[z + 1] > rp[z]) {
        lo2 = std::min<int64_t>(lo2, ci[rp[z]]);
        hi2 = std::max<int64_t>(hi2, (int64_t)ci[rp[z + 1] - 1] + 1);
      }
    }
  }
  if (lo2 > hi2) lo2 = hi2 = 0;
  int64_t lo3 = INT64_MAX, hi3 = INT64_MIN;
  for (int64_t v = lo2; v < hi2; ++v)
    if (rp[v + 1] > rp[v]) {
      lo3 = std::min<int64_t>(lo3, ci[rp[v]]);
      hi3 = std::max<int64_t>(hi3, (int64_t)ci[rp[v + 1] - 1] + 1);
    }
  if (lo3 > hi3) lo3 = hi3 = 0;
  const int64_t w2 = (((hi2 - lo2) + 31) / 32 + 3) / 4 * 4, w3 = ((hi3 - lo3) + 31) / 32;
  const bool global = w2 + w3 > H_WORDS || getenv("BLP_HOP3_FORCE_GLOBAL");
  // wedge-row path: every target range disjoint from N(N(x))'s, every b in N(x) holding a
  // wedge row (or no members), and the mark bitmap within LDS (BLP_HOP3_NO_WEDGE: off)
  const int64_t w3v = (w3 + 3) / 4;  // the mark bitmap in 16-byte vectors (wedge-row bitmaps OR whole vectors)
  bool wedge = g->d_wp && !getenv("BLP_HOP3_NO_WEDGE") && (hi2 <= lo3 || hi3 <= lo2) &&
               (size_t)16 * w3v + 20480 <= 160 * 1024;
  for (int64_t i = 0; wedge && i < n_src; ++i)
    for (int64_t k = rp[src[i]]; k < rp[src[i] + 1] && wedge; ++k) {
      const int32_t b = ci[k];
      wedge = g->h_wp[b + 1] > g->h_wp[b] || rp[b + 1] == rp[b];
    }
  const int64_t gwords = (w2 + w3 + 3) / 4 * 4;
  for (int64_t i = 0; i < (n_src ? pos_off[n_src] : 0); ++i)
    BLP_CHECK(pos_y[i] >= 0 && pos_y[i] < n, BLP_E_ARG, "blp_hop3_sample: positive id out of range");
  int rc = set_device(g);
  if (rc) return rc;
  Hop3Args a{};
  void *d_src = nullptr, *d_off = nullptr, *d_pos = nullptr, *d_cnt = nullptr, *d_x = nullptr, *d_y = nullptr,
       *d_l = nullptr, *d_gbm = nullptr;
  const int64_t npos = n_src ? pos_off[n_src] : 0;
  auto cleanup = [&]() {
    for (void* p : {d_src, d_off, d_pos, d_cnt, d_x, d_y, d_l, d_gbm})
      if (p) (void)hipFree(p);
  };
  auto hip = [&](hipError_t e, const char* what) {
    if (e != hipSuccess) {
      cleanup();
      return hip_fail(e, what, __FILE__, __LINE__);
    }
    return 0;
  };
  if ((rc = hip(dev_malloc(&d_src, 4 * std::max<int64_t>(n_src, 1)), "hipMalloc"))) return rc;
  if ((rc = hip(dev_malloc(&d_off, 4 * (n_src + 1)), "hipMalloc"))) return rc;
  if ((rc = hip(dev_malloc(&d_pos, 4 * std::max<int64_t>(npos, 1)), "hipMalloc"))) return rc;
  if ((rc = hip(dev_malloc(&d_cnt, 16), "hipMalloc"))) return rc;
  const int64_t dcap = std::max<int64_t>(cap, 1);
  if ((rc = hip(dev_malloc(&d_x, 4 * dcap), "hipMalloc"))) return rc;
  if ((rc = hip(dev_malloc(&d_y, 4 * dcap), "hipMalloc"))) return rc;
  if ((rc = hip(dev_malloc(&d_l, dcap), "hipMalloc"))) return rc;
  if (global && !wedge && (rc = hip(dev_malloc(&d_gbm, 4 * (size_t)gwords * g->n_cu), "hipMalloc (HBM bitmaps)")))
    return rc;
  if (n_src) {
    if ((rc = hip(hipMemcpy(d_src, src, 4 * n_src, hipMemcpyHostToDevice), "hipMemcpy"))) return rc;
    if ((rc = hip(hipMemcpy(d_off, pos_off, 4 * (n_src + 1), hipMemcpyHostToDevice), "hipMemcpy"))) return rc;
  }
  if (npos && (rc = hip(hipMemcpy(d_pos, pos_y, 4 * npos, hipMemcpyHostToDevice), "hipMemcpy"))) return rc;
  if ((rc = hip(hipMemsetAsync(d_cnt, 0, 16, g->stream), "hipMemsetAsync"))) return rc;
  a.rp = g->d_rp;
  a.ci = g->d_ci;
  a.src = (const int32_t*)d_src;
  a.pos_off = (const int32_t*)d_off;
  a.pos_y = (const int32_t*)d_pos;
  a.n_src = (int)n_src;
  a.lo2 = lo2;
  a.hi2 = hi2;
  a.lo3 = lo3;
  a.hi3 = hi3;
  a.w2 = (int)w2;
  a.rate = rate;
  a.seed = seed;
  a.out_x = (int32_t*)d_x;
  a.out_y = (int32_t*)d_y;
  a.out_label = (uint8_t*)d_l;
  a.cap = cap;
  a.counters = (unsigned long long*)d_cnt;
  hipEvent_t t0;
  if ((rc = timer_begin(g, K_HOP3, &t0))) return cleanup(), rc;
  if (n_src && wedge) {
    if (!getenv("BLP_HOP3_NO_WBM")) {
      const WedgeBitmaps* w = wedge_bitmaps(g, lo3, hi3, &rc);
      if (rc) return cleanup(), rc;
      if (w && w->slots) {
        a.wbm_slot = w->d_slot;
        a.wbm_pool = (const uint4*)w->d_pool;
        a.wbm_vecs = (int)(w->words / 4);
      }
    }
    const size_t dyn = 16 * (size_t)std::max<int64_t>(w3v, 1);
    int per_cu = 1;
    if ((rc = hip(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_hop3_wedge, HW_BLOCK, dyn), "occupancy")))
      return rc;
    hipLaunchKernelGGL(k_hop3_wedge, dim3(g->n_cu * std::max(per_cu, 1)), dim3(HW_BLOCK), dyn, g->stream, a,
                       (const int64_t*)g->d_wp, (const uint4*)g->d_wedge);
    if ((rc = hip(hipGetLastError(), "k_hop3_wedge launch"))) return rc;
  } else if (n_src) {
    if (global)
      hipLaunchKernelGGL(k_hop3<true>, dim3(g->n_cu), dim3(H_BLOCK), 0, g->stream, a, (uint32_t*)d_gbm, gwords);
    else
      hipLaunchKernelGGL(k_hop3<false>, dim3(g->n_cu), dim3(H_BLOCK), 0, g->stream, a, (uint32_t*)nullptr, gwords);
    if ((rc = hip(hipGetLastError(), "k_hop3 launch"))) return rc;
  }
  if ((rc = timer_end(g, K_HOP3, t0))) return cleanup(), rc;
  if ((rc = hip(hipStreamSynchronize(g->stream), "hipStreamSynchronize"))) return rc;
  unsigned long long cnt[2];
  if ((rc = hip(hipMemcpy(cnt, d_cnt, 16, hipMemcpyDeviceToHost), "hipMemcpy"))) return rc;
  const int64_t got = (int64_t)cnt[1];
  const int64_t ncopy = std::min(got, cap);
  if (ncopy > 0) {
    if ((rc = hip(hipMemcpy(out_x, d_x, 4 * ncopy, hipMemcpyDeviceToHost), "hipMemcpy"))) return rc;
    if ((rc = hip(hipMemcpy(out_y, d_y, 4 * ncopy, hipMemcpyDeviceToHost), "hipMemcpy"))) return rc;
    if ((rc = hip(hipMemcpy(out_label, d_l, ncopy, hipMemcpyDeviceToHost), "hipMemcpy"))) return rc;
  }
  cleanup();
  *n_out = got;
  return BLP_OK;
}

// Loads this file's GPU code object (blp_stream_prewarm): the HIP runtime loads a translation
// unit's code object on the first launch of any of its kernels, 10-30 ms on the caller's thread.
namespace blp {
int preload_hop3() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_hop3<true>)) == hipSuccess ? 0 : -1;
}
}  // namespace blp
