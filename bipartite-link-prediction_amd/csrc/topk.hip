// Full-candidate top-k (BASELINE.json configs[2], "config 3"; SURVEY.md §8(b) blp_topk,
// §8(d) "Full-candidate top-k").
//
// For every source x (a user on the user side) ALL targets b at exact distance 3 are scored
// with the reference's measures -- common_neighbors / jaccard / adamic_adar of
// (H2(x), N(b)), similarity.py:108-126 -- and the k best are kept per method (score
// descending, then dense target id ascending; the reference has no top-k).
// In a bipartite graph the distance-3 targets are exactly the targets with CN(x,b) > 0
// outside N(x), so the whole candidate set is one push over the A^T A projection:
//
//     CN(x, b) = #{ w in H2(x) : b in N(w) }.
//
// One workgroup per source (dequeued). H2(x) is never materialised: the pairs (b', w) with
// b' in N(x), w in N(b') are walked, and w is pushed only from b' = min(N(w) ∩ N(x))
// ("ownership"), so each w in H2(x) is pushed exactly once (duplicates cost one scan of the
// short row N(w)). The targets are renumbered by degree (descending) so the per-target
// counters can be tiered in LDS: CN <= deg(b), hence a target of degree <= 255 gets a u8
// counter, <= 65535 a u16, else a u32 (config 3: 100K businesses -> 114 KB, one pass).
//
// Adamic-Adar: every w that reaches a distance-3 target has degree >= 2, so
// CN * wmin <= AA <= CN * wmax with the extreme weights of such w. From the CN counts the
// candidates that can still reach the k-th AA lower bound are collected (usually a few
// hundred), and one more push accumulates their exact sums (the pair kernel's two-word integer
// arithmetic, blp_internal.h, so the values are bit-identical to blp_score_pairs). When the
// candidates do not fit, the source falls back to chunked direct accumulation. AA selection
// keys are the bits of the correctly rounded double (monotone for non-negative doubles).
//
// Dense wedge counts (hot targets). On a Zipf review graph the members of the most popular
// targets carry most of the push volume (config 3: the ~100 most reviewed businesses, ~85 % of
// 10.3G pushes per run). For each such target b (a prefix of the degree order) the counts of ALL
// its members, C_b[t] = |N(b) ∩ N(t)|, and their fused AA words are built once at create
// (k_tk_dense_fill), with N(b) as a bitmap over the sources. A source x whose N'(x) starts with
// hot targets b_0 < b_1 < ... (address order) adds C_{b_i} word by word instead of walking N(b_i):
// first the members of b_i already counted through an earlier b_j are subtracted (N(b_i) ∩
// ∪_{j<i} N(b_j), from the bitmaps), then C_{b_i} is added, then x's own row is subtracted. Every
// intermediate count is a count of distinct users reviewing t, so the tiered counters never
// overflow, and the result is the ownership walk's exactly: a member of a hot b_i is owned by the
// first hot target that holds it, and the walk of the other targets skips it as before.
#include <algorithm>
#include <cmath>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "blp_internal.h"

namespace {

#ifndef BLP_TK_NT
#define BLP_TK_NT 1024  // workgroup size (512: no VGPR spills, but 25.2 against 17.0 ms at config 3, r05_tk_ab)
#endif
constexpr int TK_NT = BLP_TK_NT;
constexpr int TK_SEL = 2048;          // selection buffer entries (also the AA hash table)
constexpr int TK_AH = TK_SEL / 2;     // AA hash slots: two u64 words each in s.key (exact sums)
constexpr int TK_HCAP = TK_AH / 2;    // AA candidates handled by the hash (load <= 1/2)
constexpr int TK_SEG = 256;           // N(x) entries staged per batch
constexpr int TK_FILT = 128;          // words of the N'(x) membership filter (4096 bits)
constexpr int TK_ACC_WORDS = 32768;   // counter space: 128 KiB
constexpr int TK_KMAX = 256;
constexpr int TK_WB = TK_SEL / (TK_NT / 64);  // sel_counts_wave: selection entries per wave (128)
constexpr int TK_WK = 64;                     // ... for lists of at most 64 (one per lane after a sort)
#ifndef BLP_TK_RB
#define BLP_TK_RB 8
#endif
#ifndef BLP_TK_FLAT
#define BLP_TK_FLAT 1  // count passes: the wave's owned rows pushed as one flat run (0: a row per lane)
#endif
#ifndef BLP_TK_TAIL16
#define BLP_TK_TAIL16 1  // row entries past the first TK_RB read as 16-byte vectors (4 per load); 0: one by one
#endif
constexpr int TK_RB = BLP_TK_RB;   // row entries loaded up front per element (16-byte vectors)
constexpr uint32_t TK_EMPTY = 0xFFFFFFFFu;

// Counter layout: permuted target p has a byte address -- 4p for the u32 tier (p < n32),
// A16 + 2(p - n32) for the u16 tier (p < n16), A8 + (p - n16) for the u8 tier -- increasing in
// p, so the rows store addresses (order and ownership tests are unchanged) and a push is one
// shift-add with no tier branch. A chunk is the permuted range [c0, c1) = addresses [a0, a1),
// a0 4-aligned, counted in LDS words from a0.
struct TkChunk {
  int64_t c0, c1, a0, a1;
};

struct TkArgs {
  const int64_t* rp;
  const int32_t* ci;
  const int32_t* pci;  // source-side rows with permuted target ids, sorted; row w at pci + rp[w] - pbase
  int64_t pbase;
  const int32_t* paddr; // [T] target (dense id - tlo) -> counter byte address of its permuted id
  int64_t n32, n16, A16, A8;  // counter tiers (see TkChunk)
  const int32_t* inv;   // [T] permuted id -> dense target id
  const int32_t* tdeg;  // [T] |N(b)| by permuted id
  const int32_t* ge;    // [ge_n] ge[d] = number of targets of degree >= d (a prefix of the permuted order)
  int64_t ge_n;
  const long long* wtab;  // Adamic-Adar weight (fixed point) of a source by its degree
  const int64_t* x2_off;  // [target-side CSR entries + 1] start of each wedge row in x2 (or null)
  const int32_t* x2;      // wedge rows: for each target b' and member w of N(b'), N'(w)
  int64_t kbase;          // rp[tlo]
  const int32_t* src;
  const int32_t* order;  // [n_src] dequeue order: list index of the q-th source claimed (or null: q itself)
  int n_src;
  int64_t tlo, T;
  const TkChunk* chunks;
  int n_chunks;
  int64_t aa_chunk;  // targets per direct-AA chunk (two u64 words each)
  int64_t H, AH;     // fused AA: the H most popular targets (addresses < AH) get exact sums in the count pass
  int64_t h_word;    // ... stored at LDS word h_word (8-byte aligned, after the chunk's counters)
  int k;
  uint32_t mask;
  double ratio;  // wmin / wmax over sources of degree >= 2 (fixed point)
  int hcap;      // AA candidates allowed on the hash path (<= TK_HCAP)
  unsigned long long* keys;  // [3][n_src][k]
  int32_t* cols;             // [3][n_src][k]
  int64_t* ncand;            // [n_src]
  unsigned long long* counters;  // [0] queue, [1] AA hash path, [2] AA direct path, [3] sum |H2|, [4] sum of |N(w)| over H2, [5] AA fused path
  int64_t acc_words;  // counter words in use (<= TK_ACC_WORDS; test knob BLP_TOPK_ACC_WORDS)
  int64_t pci_len, x2_len;  // entries of pci / x2 including their padding (BLP_DEBUG bounds)
  // dense wedge counts of the hot targets p < dw_n (single counter chunk; see the header)
  const uint32_t* dw_cv;            // [dw_n][dw_words] packed counts of all members of N(b)
  const unsigned long long* dw_ca;  // [dw_n][2 H] their fused AA words (or null)
  uint32_t* dw_bm;                  // [dw_n][dw_bmw] N(b) over the sources (bit w - slo)
  long long* dw_info;               // [dw_n][2] |N(b)|, sum of |N(w)| over w in N(b)
  unsigned long long* dw_caf;       // [dw_n][2 T] the members' exact AA words for EVERY target (the
                                    // hash / direct AA passes; or null: those passes walk every target)
  int dw_n, dw_max;                 // hot targets; at most dw_max of them per source
  int64_t dw_words, dw_bmw, slo;
  int wavesel;  // CN / Jaccard selection per wave (sel_counts_wave; k <= TK_WK; default), else block rounds (BLP_TK_WAVESEL=0)
};

// BLP_DEBUG builds (make debug -> libblp_debug.so): every LDS index and every row read of the
// walk is checked against its bound before the access; a violation is counted, the first one
// recorded (site, value, bound) and the access skipped, so the check never faults the GPU.
// blp_topk_run then fails with the record (BLP_E_STATE). Release builds compile the checks out.
#ifdef BLP_DEBUG
__device__ long long g_tk_dbg[4];  // violations, first site, its value, its bound
__device__ inline bool tk_ok(bool ok, int site, long long v, long long bound) {
  if (!ok && atomicAdd((unsigned long long*)&g_tk_dbg[0], 1ull) == 0ull) {
    g_tk_dbg[1] = site;
    g_tk_dbg[2] = v;
    g_tk_dbg[3] = bound;
  }
  return ok;
}
#define TK_OK(cond, site, v, bound) tk_ok((cond), (site), (long long)(v), (long long)(bound))
#else
#define TK_OK(cond, site, v, bound) ((void)(v), true)
#endif
// sites: 1 acc_add, 2 acc_get, 3 acc_clear, 4 fused AA word, 5 hash AA word, 6 direct AA word,
// 7 segment index, 8 16-byte row read, 9 row entry read, 10 selection slot, 11 hash probe length,
// 12 dense: hot target index, 13 dense: member bitmap word, 14 dense: member row read

struct TkShared {
  uint32_t acc[TK_ACC_WORDS];
  unsigned long long key[TK_SEL];
  int32_t col[TK_SEL];
  int64_t seg_rs[TK_SEG];
  int64_t seg_kx[TK_SEG];
  int64_t seg_off[TK_SEG + 1];
  int32_t seg_p[TK_SEG];
  uint32_t filt[TK_FILT];
  long long red[TK_NT / 64];
  unsigned long long thr_key;
  int thr_col, have_thr, n, item;
  int need[2];  // a selection round (by parity) left the buffer past TK_SEL - TK_NT: compact (sel_round_end)
  int nv[3];
  int nd;  // hot targets of this source handled by dense_pass
  unsigned long long sthr;  // sel_counts_wave: the best of the waves' k-th keys (a shared pruning bound)
  int wcnt[TK_NT / 64];     // sel_counts_wave: entries each wave hands to the final merge
};

__device__ inline uint32_t filt_bit(int32_t e) { return ((uint32_t)e * 2654435761u) >> 20; }

__device__ inline bool better(unsigned long long ka, int ca, unsigned long long kb, int cb) {
  return ka > kb || (ka == kb && ca < cb);
}

__device__ inline int64_t addr_of(const TkArgs& a, int64_t p) {
  return p < a.n32 ? 4 * p : p < a.n16 ? a.A16 + 2 * (p - a.n32) : a.A8 + (p - a.n16);
}

__device__ inline int64_t p_of(const TkArgs& a, int64_t e) {
  return e < a.A16 ? e >> 2 : e < a.A8 ? a.n32 + ((e - a.A16) >> 1) : a.n16 + (e - a.A8);
}

__device__ inline uint32_t width_mask(const TkArgs& a, int64_t e) {
  return e < a.A16 ? 0xFFFFFFFFu : e < a.A8 ? 0xFFFFu : 0xFFu;
}

__device__ inline void acc_add(const TkArgs& a, uint32_t* acc, const TkChunk& c, int64_t e) {
  const int64_t off = e - c.a0;
  if (TK_OK(off >= 0 && (off >> 2) < a.acc_words, 1, off, a.acc_words)) atomicAdd(&acc[off >> 2], 1u << ((off & 3) << 3));
}

__device__ inline uint32_t acc_get(const TkArgs& a, const uint32_t* acc, const TkChunk& c, int64_t e) {
  const int64_t off = e - c.a0;
  if (!TK_OK(off >= 0 && (off >> 2) < a.acc_words, 2, off, a.acc_words)) return 0;
  return (acc[off >> 2] >> ((off & 3) << 3)) & width_mask(a, e);
}

__device__ inline void acc_clear(const TkArgs& a, uint32_t* acc, const TkChunk& c, int64_t e) {
  const int64_t off = e - c.a0;
  if (TK_OK(off >= 0 && (off >> 2) < a.acc_words, 3, off, a.acc_words))
    atomicAnd(&acc[off >> 2], ~(width_mask(a, e) << ((off & 3) << 3)));
}

constexpr int TK_HBITS = 10;  // log2(TK_AH)
__device__ inline int hash_slot(int32_t e) { return (int)(((uint32_t)e * 2654435761u) >> (32 - TK_HBITS)); }

// one term W into target t's exact AA words (lo wrapping, hi = sum of W >> 32)
__device__ inline void aa_push2(unsigned long long* w2, int64_t t, unsigned long long W) {
  atomicAdd(&w2[2 * t], W);
  atomicAdd(&w2[2 * t + 1], W >> 32);
}

// removal of one count / one AA term (the inverse of acc_add / aa_push2: wrapping adds of the
// negation; the removed contribution is always present, so no tier field borrows)
__device__ inline void acc_sub(const TkArgs& a, uint32_t* acc, int64_t e) {
  if (TK_OK(e >= 0 && (e >> 2) < a.acc_words, 1, e, a.acc_words)) atomicAdd(&acc[e >> 2], 0u - (1u << ((e & 3) << 3)));
}

__device__ inline void aa_sub2(unsigned long long* w2, int64_t t, unsigned long long W) {
  atomicAdd(&w2[2 * t], 0ull - W);
  atomicAdd(&w2[2 * t + 1], 0ull - (W >> 32));
}

// selection key of an exact AA word pair: the bits of the correctly rounded double
__device__ inline unsigned long long aa_key(const unsigned long long* w2, int64_t t) {
  return (unsigned long long)__double_as_longlong(blp::aa_value(w2[2 * t], w2[2 * t + 1]));
}

__device__ __attribute__((always_inline)) long long block_sum(TkShared& s, long long v) {
  for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s.red[threadIdx.x >> 6] = v;
  __syncthreads();
  long long t = 0;
  for (int w = 0; w < TK_NT / 64; ++w) t += s.red[w];
  return t;
}

// is permuted target e in N'(x)?  filter bit, then binary search of x's sorted permuted row
__device__ inline bool in_row_x(const TkShared& s, const int32_t* rowx, int du, int32_t e) {
  const uint32_t b = filt_bit(e);
  if (!((s.filt[b >> 5] >> (b & 31)) & 1u)) return false;
  int lo = 0, hi = du;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (rowx[mid] < e) lo = mid + 1; else hi = mid;
  }
  return lo < du && rowx[lo] == e;
}

// Every helper that takes TkShared& is forced inline: an out-of-line copy (the compiler made one
// of push_pass<2> when the kernel grew) reaches LDS through generic pointers with flat
// instructions and a call stack in scratch, and that build faulted.
// MODE 0: CN counts into the tiered counters of chunk c (and |H2(x)| when count_h2)
// MODE 3: MODE 0 plus the exact AA words of the H most popular targets (fused AA)
// MODE 1: exact AA of the hashed candidates (counter >= thr) into s.key[2 slot], s.key[2 slot + 1]
// MODE 2: direct exact AA words of targets [c0, c1) into the u64 view of s.acc
// (two words per target: the wrapping sum of W and the sum of W >> 32, blp_internal.h)
template <int MODE>
__device__ __attribute__((always_inline)) long long push_pass(const TkArgs& a, TkShared& s, int x, int64_t xb, int du, const int32_t* rowx,
                               const TkChunk& c, uint32_t thr, int64_t d0, int64_t d1, bool count_h2,
                               long long* pushed = nullptr, int32_t a_dense = 0) {
  long long h2 = 0, npush = 0;
  unsigned long long* acc64 = reinterpret_cast<unsigned long long*>(s.acc);
  const int tid = threadIdx.x;
  for (int s0 = 0; s0 < du; s0 += TK_SEG) {
    const int ns = min(TK_SEG, du - s0);
    __syncthreads();  // the previous batch's readers are done with the segment table
    long long len = 0;
    if (tid < ns) {
      const int b = a.ci[xb + s0 + tid];
      const int64_t rs = a.rp[b];
      len = a.rp[b + 1] - rs;
      s.seg_rs[tid] = rs;
      s.seg_p[tid] = a.paddr[b - a.tlo];
      if (s.seg_p[tid] < a_dense) len = 0;  // a hot target already counted by dense_pass
      if (a.x2) {  // position of x in N(b') (sorted): its own wedge is skipped
        int64_t lo = rs, hi = rs + len;
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if (a.ci[mid] < x) lo = mid + 1; else hi = mid;
        }
        s.seg_kx[tid] = lo;
      }
    }
    // exclusive scan of the segment lengths (ns <= TK_SEG <= TK_NT)
    {
      long long inc = len;
      const int lane = tid & 63, wid = tid >> 6;
      for (int d = 1; d < 64; d <<= 1) {
        const long long t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
      }
      if (lane == 63) s.red[wid] = inc;
      __syncthreads();
      long long base = 0;
      for (int w = 0; w < wid; ++w) base += s.red[w];
      if (tid < ns) s.seg_off[tid] = base + inc - len;
      if (tid == TK_NT - 1) s.seg_off[ns] = base + inc;  // total (threads >= ns carry len 0)
      __syncthreads();
    }
    const int64_t E = s.seg_off[ns];
    // Software-pipelined walk. Element idx of the batch is (segment b', i-th member w of
    // N(b')); its row N'(w) is located either through the expanded wedge array (x2: the rows
    // of N(b')'s members stored back to back, read sequentially) or through rp[w]. The next
    // element's row bounds are fetched while the current row is processed, and the first
    // TK_RB entries of a row are loaded as independent predicated loads (rows are short).
    const int32_t* base = a.x2 ? a.x2 : a.pci;
    const int64_t base_len = a.x2 ? a.x2_len : a.pci_len;  // entries incl. padding (BLP_DEBUG bound)
    (void)base_len;
    int sg = 0;
    auto fetch = [&](int64_t id, int64_t& r0, int64_t& r1, int32_t& pp) -> bool {
      while (s.seg_off[sg + 1] <= id) ++sg;
      if (!TK_OK(sg < ns, 7, sg, ns)) return true;
      const int64_t k = s.seg_rs[sg] + (id - s.seg_off[sg]);
      pp = s.seg_p[sg];
      if (a.x2) {
        if (k == s.seg_kx[sg]) return true;  // x itself
        r0 = a.x2_off[k - a.kbase];
        r1 = a.x2_off[k - a.kbase + 1];
        return false;
      }
      const int w = a.ci[k];
      if (w == x) return true;
      r0 = a.rp[w] - a.pbase;
      r1 = a.rp[w + 1] - a.pbase;
      return false;
    };
    int64_t idx = tid, r0n = 0, r1n = 0;
    int32_t ppn = 0;
    bool skipn = true;
    if (idx < E) skipn = fetch(idx, r0n, r1n, ppn);
    if constexpr ((MODE == 0 || MODE == 3) && BLP_TK_FLAT) {
      // Wave-flattened push. A lane still owns one element (b', w) per round and decides its
      // ownership, but the owned rows of the wave's 64 lanes are then pushed as ONE run: lane l
      // takes entries [l q, (l + 1) q) of their concatenation (q = ceil(total / 64)). Rows hold
      // 1..28 ids (~11), so a row per lane left most lanes idle beside the wave's longest row,
      // and the 64 lanes all pushed their rows' FIRST entries -- the most popular targets, whose
      // counters share a few LDS words -- in the same instruction. Every count is the same sum.
      // The wave's row table (start, exclusive prefix, weight) lives in s.key / s.col, which the
      // count pass does not otherwise use (the selection reloads them afterwards).
      const int lane = tid & 63, wv = tid >> 6;
      int64_t* rt_base = reinterpret_cast<int64_t*>(s.key) + wv * 64;
      unsigned long long* rt_w = s.key + TK_SEL / 2 + wv * 64;
      int32_t* rt_excl = s.col + wv * 65;
      unsigned long long* aah = acc64 + (a.h_word >> 1);
      for (int64_t wb = tid - lane; wb < E; wb += TK_NT) {  // wave-uniform rounds
        const bool skip = idx >= E || skipn;
        const int64_t r0 = r0n;
        const int len_w = skip ? 0 : (int)(r1n - r0n);
        const int32_t pp = ppn;
        const int32_t* roww = base + r0;
        int32_t e[TK_RB];
        const blp::U4a* rv = reinterpret_cast<const blp::U4a*>(roww);
#pragma unroll
        for (int q = 0; q < TK_RB / 4; ++q) {
          blp::U4a v = {0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF};
          if (4 * q < len_w && TK_OK(r0 >= 0 && r0 + 4 * q + 4 <= base_len, 8, r0 + 4 * q + 4, base_len)) v = rv[q];
          e[4 * q] = 4 * q < len_w ? v.x : 0x7FFFFFFF;
          e[4 * q + 1] = 4 * q + 1 < len_w ? v.y : 0x7FFFFFFF;
          e[4 * q + 2] = 4 * q + 2 < len_w ? v.z : 0x7FFFFFFF;
          e[4 * q + 3] = 4 * q + 3 < len_w ? v.w : 0x7FFFFFFF;
        }
        idx += TK_NT;
        if (idx < E) skipn = fetch(idx, r0n, r1n, ppn);
        // ownership: no entry of N'(w) below b' is in N'(x)
        bool owned = !skip;
#pragma unroll
        for (int j = 0; j < TK_RB; ++j)
          if (owned && e[j] < pp && in_row_x(s, rowx, du, e[j])) owned = false;
        for (int j = TK_RB; j < len_w && owned; j += 4) {
          blp::U4a v = {0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF};
          if (TK_OK(r0 + j + 4 <= base_len, 8, r0 + j + 4, base_len)) v = *reinterpret_cast<const blp::U4a*>(roww + j);
          const int32_t t[4] = {v.x, j + 1 < len_w ? v.y : 0x7FFFFFFF, j + 2 < len_w ? v.z : 0x7FFFFFFF,
                                j + 3 < len_w ? v.w : 0x7FFFFFFF};
          if (t[0] >= pp) break;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (t[q] < pp && in_row_x(s, rowx, du, t[q])) owned = false;
          if (t[3] >= pp) break;
        }
        const int mylen = owned ? len_w : 0;
        if (count_h2 && owned) {
          ++h2;
          npush += len_w;
        }
        int incl = mylen;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int t = __shfl_up(incl, d, 64);
          if (lane >= d) incl += t;
        }
        const int T = __shfl(incl, 63, 64);
        if (T == 0) continue;  // uniform
        rt_base[lane] = r0;
        rt_excl[lane] = incl - mylen;
        if (lane == 63) rt_excl[64] = T;
        if (MODE == 3) rt_w[lane] = (unsigned long long)a.wtab[len_w];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int qn = (T + 63) >> 6;
        const int f0 = lane * qn, f1 = min(T, f0 + qn);
        if (f0 < f1) {
          int r = 0, hi = 64;  // the row holding entry f0: last r with excl[r] <= f0
          while (hi - r > 1) {
            const int mid = (r + hi) >> 1;
            if (rt_excl[mid] <= f0) r = mid; else hi = mid;
          }
          int rs = rt_excl[r], re = rt_excl[r + 1];
          int64_t rb = rt_base[r];
          unsigned long long wr = MODE == 3 ? rt_w[r] : 0ull;
          for (int f = f0; f < f1; f += 4) {  // four entries' loads in flight per group
            int64_t ad[4];
            unsigned long long wu[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int fu = min(f + u, f1 - 1);  // past the end: a repeat of the last, not pushed
              while (fu >= re) {
                ++r;
                rs = re;
                re = rt_excl[r + 1];
                rb = rt_base[r];
                if (MODE == 3) wr = rt_w[r];
              }
              ad[u] = rb + (fu - rs);
              wu[u] = wr;
            }
            int32_t ev[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
              ev[u] = TK_OK(ad[u] >= 0 && ad[u] < base_len, 9, ad[u], base_len) ? base[ad[u]] : 0x7FFFFFFF;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              if (f + u >= f1) break;
              const int32_t ej = ev[u];
              if (ej >= c.a0 && ej < c.a1) acc_add(a, s.acc, c, ej);
              if (MODE == 3 && ej < a.AH) {
                const int64_t t = p_of(a, ej);
                if (TK_OK(t >= 0 && (a.h_word >> 1) + 2 * t + 1 < a.acc_words / 2, 4, t, a.acc_words))
                  aa_push2(aah, t, wu[u]);
              }
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the table is rewritten next round
      }
      continue;  // the next batch of N(x) (its first barrier orders this batch's pushes)
    }
    while (idx < E) {
      const bool skip = skipn;
      const int64_t r0 = r0n;
      const int len_w = (int)(r1n - r0n);
      const int32_t pp = ppn;
      const int32_t* roww = base + r0;
      // the first TK_RB entries as 16-byte vectors (rows are padded past their ends)
      int32_t e[TK_RB];
      const blp::U4a* rv = reinterpret_cast<const blp::U4a*>(roww);
#pragma unroll
      for (int q = 0; q < TK_RB / 4; ++q) {
        blp::U4a v = {0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF};
        if (!skip && 4 * q < len_w && TK_OK(r0 >= 0 && r0 + 4 * q + 4 <= base_len, 8, r0 + 4 * q + 4, base_len)) v = rv[q];
        e[4 * q] = 4 * q < len_w ? v.x : 0x7FFFFFFF;
        e[4 * q + 1] = 4 * q + 1 < len_w ? v.y : 0x7FFFFFFF;
        e[4 * q + 2] = 4 * q + 2 < len_w ? v.z : 0x7FFFFFFF;
        e[4 * q + 3] = 4 * q + 3 < len_w ? v.w : 0x7FFFFFFF;
      }
      idx += TK_NT;
      if (idx < E) skipn = fetch(idx, r0n, r1n, ppn);
      if (skip) continue;
      // row entry j >= TK_RB (bounds-checked in BLP_DEBUG builds)
      auto entry = [&](int j) -> int32_t {
        return TK_OK(r0 + j < base_len, 9, r0 + j, base_len) ? roww[j] : 0x7FFFFFFF;
      };
      // the entries past the first TK_RB, four at a time as 16-byte vectors (BLP_TK_TAIL16): the
      // last vector reads up to 3 entries past the row, inside the next row or the array padding
      auto tail4 = [&](int j, int32_t* t) {
        blp::U4a v = {0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF};
        if (TK_OK(r0 + j + 4 <= base_len, 8, r0 + j + 4, base_len)) v = *reinterpret_cast<const blp::U4a*>(roww + j);
        t[0] = v.x;
        t[1] = j + 1 < len_w ? v.y : 0x7FFFFFFF;
        t[2] = j + 2 < len_w ? v.z : 0x7FFFFFFF;
        t[3] = j + 3 < len_w ? v.w : 0x7FFFFFFF;
      };
      (void)tail4;
      bool owned = true;
#pragma unroll
      for (int j = 0; j < TK_RB; ++j)
        if (e[j] < pp && in_row_x(s, rowx, du, e[j])) owned = false;
#if BLP_TK_TAIL16
      for (int j = TK_RB; j < len_w && owned; j += 4) {
        int32_t t[4];
        tail4(j, t);
        if (t[0] >= pp) break;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (t[q] < pp && in_row_x(s, rowx, du, t[q])) owned = false;
        if (t[3] >= pp) break;
      }
#else
      for (int j = TK_RB; j < len_w && owned; ++j) {
        const int32_t ej = entry(j);
        if (ej >= pp) break;
        if (in_row_x(s, rowx, du, ej)) owned = false;
      }
#endif
      if (!owned) continue;
      if (MODE == 3) {
        unsigned long long* aah = acc64 + (a.h_word >> 1);
        const unsigned long long wfx = (unsigned long long)a.wtab[len_w];
        auto push3 = [&](int32_t ej) {
          const int64_t t = p_of(a, ej);
          if (ej < a.AH && TK_OK(t >= 0 && (a.h_word >> 1) + 2 * t + 1 < a.acc_words / 2, 4, t, a.acc_words))
            aa_push2(aah, t, wfx);
        };
        for (int j = 0; j < TK_RB; ++j)
          if (j < len_w) push3(e[j]);
        for (int j = TK_RB; j < len_w; ++j) push3(entry(j));
      }
      if (MODE == 0 || MODE == 3) {
        if (count_h2) {
          ++h2;
          npush += len_w;
        }
#pragma unroll
        for (int j = 0; j < TK_RB; ++j)
          if (j < len_w && e[j] >= c.a0 && e[j] < c.a1) acc_add(a, s.acc, c, e[j]);
#if BLP_TK_TAIL16
        for (int j = TK_RB; j < len_w; j += 4) {
          int32_t t[4];
          tail4(j, t);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (t[q] >= c.a0 && t[q] < c.a1) acc_add(a, s.acc, c, t[q]);
        }
#else
        for (int j = TK_RB; j < len_w; ++j) {
          const int32_t ej = entry(j);
          if (ej >= c.a0 && ej < c.a1) acc_add(a, s.acc, c, ej);
        }
#endif
      } else if (MODE == 1) {
        const unsigned long long wfx = (unsigned long long)a.wtab[len_w];
        auto push1 = [&](int32_t ej) {
          if (acc_get(a, s.acc, c, ej) >= thr) {
            int h = hash_slot(ej), probes = 0;
            while (s.col[h] != ej) {
              ++probes;
              if (!TK_OK(probes < TK_AH, 11, probes, TK_AH)) break;
              h = (h + 1) & (TK_AH - 1);
            }
            if (s.col[h] == ej && TK_OK(2 * h + 1 < TK_SEL, 5, h, TK_SEL)) aa_push2(s.key, h, wfx);
          }
        };
#pragma unroll
        for (int j = 0; j < TK_RB; ++j)
          if (j < len_w) push1(e[j]);
        for (int j = TK_RB; j < len_w; ++j) push1(entry(j));
      } else {
        const unsigned long long wfx = (unsigned long long)a.wtab[len_w];
        auto push2 = [&](int64_t p) {
          if (p >= d0 && p < d1 && TK_OK(2 * (p - d0) + 1 < a.acc_words / 2, 6, p - d0, a.acc_words / 4))
            aa_push2(acc64, p - d0, wfx);
        };
#pragma unroll
        for (int j = 0; j < TK_RB; ++j)
          if (j < len_w) push2(p_of(a, e[j]));
        for (int j = TK_RB; j < len_w; ++j) push2(p_of(a, entry(j)));
      }
    }
  }
  __syncthreads();
  if (pushed) *pushed = npush;
  return h2;
}

#ifdef BLP_PROF  // experiment builds only: per-phase clock sums of thread 0 (blp_topk_prof_read)
__device__ unsigned long long g_tkprof[16];
#define TKP_INIT                          \
  unsigned long long tkp_t0 = clock64();  \
  unsigned long long tkp_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#define TKP(i)                                 \
  {                                            \
    const unsigned long long t1_ = clock64();  \
    tkp_acc[i] += t1_ - tkp_t0;                \
    tkp_t0 = t1_;                              \
  }
#define TKP_FLUSH \
  if (tid == 0)   \
    for (int i_ = 0; i_ < 10; ++i_) atomicAdd(&g_tkprof[i_], tkp_acc[i_]);
// selection rounds walked per method (g_tkprof[10 + METHOD]) and compactions ([12])
#define TKP_ROUND(m) \
  if (threadIdx.x == 0) atomicAdd(&g_tkprof[10 + (m)], 1ull);
#define TKP_COMPACT \
  if (threadIdx.x == 0) atomicAdd(&g_tkprof[12], 1ull);
// sel_counts_wave: 64-target blocks walked, per method, over all waves ([13 + METHOD])
#define TKP_WROUND(m) \
  if ((threadIdx.x & 63) == 0) atomicAdd(&g_tkprof[13 + (m)], 1ull);
#else
#define TKP_ROUND(m)
#define TKP_COMPACT
#define TKP_WROUND(m)
#define TKP_INIT
#define TKP(i)
#define TKP_FLUSH
#endif

// Sort s.key/s.col[0, TK_SEL) best-first (bitonic), keep min(n, k); update the threshold.
__device__ __attribute__((always_inline)) void compact(const TkArgs& a, TkShared& s, int n) {
  const int tid = threadIdx.x;
  TKP_COMPACT
  for (int i = n + tid; i < TK_SEL; i += TK_NT) {
    s.key[i] = 0;
    s.col[i] = 0x7FFFFFFF;
  }
  __syncthreads();
  int size_lim = 2;
  while (size_lim < n) size_lim <<= 1;  // entries past n are padding; sort the smallest power of two
  for (int size = 2; size <= size_lim; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < size_lim / 2; t += TK_NT) {
        const int i = 2 * t - (t & (stride - 1));
        const int j = i + stride;
        const bool desc = ((i & size) == 0) || size == size_lim;
        const unsigned long long ki = s.key[i], kj = s.key[j];
        const int ci = s.col[i], cj = s.col[j];
        const bool sw = desc ? better(kj, cj, ki, ci) : better(ki, ci, kj, cj);
        if (sw) {
          s.key[i] = kj;
          s.key[j] = ki;
          s.col[i] = cj;
          s.col[j] = ci;
        }
      }
      __syncthreads();
    }
  }
  if (tid == 0) {
    const int keep = min(n, a.k);
    s.n = keep;
    s.need[0] = s.need[1] = 0;
    if (keep == a.k) {
      s.thr_key = s.key[keep - 1];
      s.thr_col = s.col[keep - 1];
      s.have_thr = 1;
    }
  }
  __syncthreads();
}

__device__ __attribute__((always_inline)) void sel_begin(const TkArgs& a, TkShared& s, int m, int it) {
  const int nv = s.nv[m];
  const size_t base = ((size_t)m * a.n_src + it) * a.k;
  for (int i = threadIdx.x; i < nv; i += TK_NT) {
    s.key[i] = a.keys[base + i];
    s.col[i] = a.cols[base + i];
  }
  if (threadIdx.x == 0) {
    s.n = nv;
    s.need[0] = s.need[1] = 0;
    s.have_thr = nv == a.k;
    if (nv == a.k) {
      s.thr_key = a.keys[base + nv - 1];
      s.thr_col = a.cols[base + nv - 1];
    }
  }
  __syncthreads();
}

__device__ __attribute__((always_inline)) void sel_end(const TkArgs& a, TkShared& s, int m, int it) {
  compact(a, s, s.n);
  const int nv = s.n;
  const size_t base = ((size_t)m * a.n_src + it) * a.k;
  for (int i = threadIdx.x; i < nv; i += TK_NT) {
    a.keys[base + i] = s.key[i];
    a.cols[base + i] = s.col[i];
  }
  if (threadIdx.x == 0) s.nv[m] = nv;
  __syncthreads();
}

// A round of offers, then ONE barrier (round 5, BLP_TK_ONEBAR=1; measured no faster, so the default
// keeps two). The buffer passes TK_SEL - TK_NT in a
// round exactly when one offer of that round takes slot TK_SEL - TK_NT (slots are consecutive), and
// that offer raises the round's flag need[parity]. After the barrier every thread reads the flag of
// ITS round: the next round's offers raise the other parity's flag, so a thread that runs ahead
// into round r + 1 cannot change what a slow one reads for round r (reading s.n instead would need
// a second barrier to stop exactly that). compact() clears both flags.
__device__ inline void sel_offer(TkShared& s, bool ok, unsigned long long key, int col, int par) {
  if (ok && (!s.have_thr || better(key, col, s.thr_key, s.thr_col))) {
    const int slot = atomicAdd(&s.n, 1);
    if (TK_OK(slot < TK_SEL, 10, slot, TK_SEL)) {
      s.key[slot] = key;
      s.col[slot] = col;
    }
    if (slot == TK_SEL - TK_NT) s.need[par] = 1;
  }
}

#ifndef BLP_TK_ONEBAR
#define BLP_TK_ONEBAR 0  // 1: one barrier per round (parity flags); measured 17.09 / 17.10 against 16.99 / 17.02 ms
#endif
__device__ inline void sel_round_end(const TkArgs& a, TkShared& s, int par) {
  __syncthreads();
  if (!BLP_TK_ONEBAR) {
    const int n = s.n;
    __syncthreads();
    if (n > TK_SEL - TK_NT) compact(a, s, n);
    return;
  }
  if (s.need[par]) compact(a, s, s.n);  // uniform: no offer runs until compact's own barriers are passed
}

// METHOD 0: CN key; 1: Jaccard key (fp64 bits); the counters of chunk c
template <int METHOD>
__device__ __attribute__((always_inline)) long long sel_counts(const TkArgs& a, TkShared& s, int it, const TkChunk& c, long long h2, bool count) {
  sel_begin(a, s, METHOD, it);
  long long nc = 0;
  if (count)  // targets with a count (the chunk's share of |H3(x)|): all of them, before the pruned walk
    for (int64_t q = c.c0 + threadIdx.x; q < c.c1; q += TK_NT) nc += acc_get(a, s.acc, c, addr_of(a, q)) > 0;
  // the next round's target ids (and degrees) are loaded while this round is offered: each
  // round ends in barriers, so a load issued in the round that uses it costs a full L2 round
  // trip per round (~100 rounds per method at config 3)
  int64_t p = c.c0 + threadIdx.x;
  int inv_c = p < c.c1 ? a.inv[p] : 0;
  int deg_c = METHOD == 1 && p < c.c1 ? a.tdeg[p] : 0;
  for (int64_t base = c.c0; base < c.c1; base += TK_NT, p += TK_NT) {
    const int64_t pn = p + TK_NT;
    const int inv_n = pn < c.c1 ? a.inv[pn] : 0;
    const int deg_n = METHOD == 1 && pn < c.c1 ? a.tdeg[pn] : 0;
    bool ok = false;
    unsigned long long key = 0;
    int col = 0;
    if (p < c.c1) {
      const uint32_t cnt = acc_get(a, s.acc, c, addr_of(a, p));
      ok = cnt > 0;
      if (ok) {
        if (METHOD == 0) {
          key = cnt;
        } else {
          const double jac = (double)cnt / (double)(h2 + (long long)deg_c - (long long)cnt);
          key = (unsigned long long)__double_as_longlong(jac);
        }
        col = inv_c;
      }
    }
    const int par = (int)(((base - c.c0) / TK_NT) & 1);
    TKP_ROUND(METHOD)
    sel_offer(s, ok, key, col, par);
    sel_round_end(a, s, par);
    inv_c = inv_n;
    deg_c = deg_n;
    // Pruning: targets are in degree order (descending), and a target of degree d scores at
    // most CN = d, Jaccard = d / |H2| (once d <= |H2|; c / (|H2| + d - c) grows with c <= d,
    // and the rounded quotients keep that order). Once that bound is below the current k-th
    // key -- strictly, so no tie can still win on the id -- no later target can enter the list.
    // The decision is uniform: shared threshold, the same degree load in every thread.
    const int64_t pn0 = base + TK_NT;
    if (pn0 < c.c1 && s.have_thr) {
      const long long d = a.tdeg[pn0];
      const bool stop = METHOD == 0 ? (unsigned long long)d < s.thr_key
                                    : h2 > 0 && d <= h2 &&
                                          (unsigned long long)__double_as_longlong((double)d / (double)h2) < s.thr_key;
      if (stop) break;
    }
  }
  sel_end(a, s, METHOD, it);
  return nc;
}

// ---- per-wave selection (round 5, the default; BLP_TK_WAVESEL=0 for block rounds): each wave walks its own blocks of 64 targets
// (wave w takes blocks w, w + 16, ... of the degree order) with NO block barrier: offers are
// appended to the wave's 128-entry region of s.key / s.col by ballot, and when it passes 64 the
// wave sorts its region in registers (two entries per lane, bitonic over lane shuffles) and keeps
// the best k. A wave stops when the degree bound of its next block falls below max(its own k-th
// key, s.sthr), s.sthr being the best of every wave's k-th key (each wave's k-th best is a lower
// bound of the list's: the list's k-th is the best k-th over any k candidates). At the end the
// waves' lists (<= k each) are packed and sel_end merges them.
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// sort the wave's region [0, n) (n <= TK_WB) best-first; lane i ends holding entry i in (ka, ca)
// (entries past n are padding: key 0, col INT_MAX)
__device__ __attribute__((always_inline)) void wave_sort(const unsigned long long* wk, const int32_t* wc, int n,
                                                         unsigned long long& ka, int& ca) {
  const int lane = threadIdx.x & 63;
  ka = lane < n ? wk[lane] : 0ull;
  ca = lane < n ? wc[lane] : 0x7FFFFFFF;
  unsigned long long kb = lane + 64 < n ? wk[lane + 64] : 0ull;
  int cb = lane + 64 < n ? wc[lane + 64] : 0x7FFFFFFF;
#pragma unroll
  for (int size = 2; size <= TK_WB; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride == 64) {  // the two entries of this lane: indexes lane (lower) and lane + 64
        const bool desc = true;  // size == TK_WB
        const bool sw = desc ? better(kb, cb, ka, ca) : better(ka, ca, kb, cb);
        if (sw) {
          const unsigned long long tk = ka;
          const int tc = ca;
          ka = kb, ca = cb, kb = tk, cb = tc;
        }
        continue;
      }
      const unsigned long long oka = __shfl_xor(ka, stride, 64), okb = __shfl_xor(kb, stride, 64);
      const int oca = __shfl_xor(ca, stride, 64), ocb = __shfl_xor(cb, stride, 64);
      const bool lower = (lane & stride) == 0;
      // entry A has index lane, entry B index lane + 64; the pair's lower index decides the direction
      const bool desc_a = ((((lane & ~stride)) & size) == 0) || size == TK_WB;
      const bool desc_b = ((((lane + 64) & ~stride) & size) == 0) || size == TK_WB;
      // the lower entry of a descending pair keeps the better one
      const bool keep_better_a = lower == desc_a, keep_better_b = lower == desc_b;
      const bool a_better = better(ka, ca, oka, oca), b_better = better(kb, cb, okb, ocb);
      if (keep_better_a != a_better) ka = oka, ca = oca;
      if (keep_better_b != b_better) kb = okb, cb = ocb;
    }
  }
}

// METHOD 0: CN key; 1: Jaccard key; the same list as sel_counts for k <= TK_WK
template <int METHOD>
__device__ __attribute__((always_inline)) long long sel_counts_wave(const TkArgs& a, TkShared& s, int it, const TkChunk& c,
                                                                    long long h2, bool count) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int NWV = TK_NT / 64;
  unsigned long long* wk = s.key + w * TK_WB;
  int32_t* wc = s.col + w * TK_WB;
  const int k = a.k;
  const int nv = s.nv[METHOD];
  const size_t gbase = ((size_t)METHOD * a.n_src + it) * a.k;
  if (tid == 0) s.sthr = 0;
  // wave 0 starts from the list of the earlier chunks (best-first, nv <= k <= 64 entries)
  int n = w == 0 ? nv : 0;
  if (w == 0 && lane < nv) {
    wk[lane] = a.keys[gbase + lane];
    wc[lane] = a.cols[gbase + lane];
  }
  bool have = w == 0 && nv == k;
  unsigned long long tkey = have ? a.keys[gbase + k - 1] : 0ull;
  int tcol = have ? a.cols[gbase + k - 1] : 0;
  __syncthreads();  // s.sthr reset, the old list in place, s.nv read by all
  if (have) atomicMax(&s.sthr, tkey);
  long long nc = 0;
  if (count)
    for (int64_t q = c.c0 + tid; q < c.c1; q += TK_NT) nc += acc_get(a, s.acc, c, addr_of(a, q)) > 0;
  for (int64_t base = c.c0 + (int64_t)w * 64; base < c.c1; base += (int64_t)NWV * 64) {
    // prune: the block's first target has its largest degree
    const unsigned long long sthr = s.sthr;
    const unsigned long long thr = have && tkey > sthr ? tkey : sthr;
    if (thr > 0) {
      const long long d = a.tdeg[base];
      const bool stop = METHOD == 0 ? (unsigned long long)d < thr
                                    : h2 > 0 && d <= h2 && (unsigned long long)__double_as_longlong((double)d / (double)h2) < thr;
      if (stop) break;  // uniform in the wave
    }
    TKP_WROUND(METHOD)
    const int64_t p = base + lane;
    bool ok = false;
    unsigned long long key = 0;
    int col = 0;
    if (p < c.c1) {
      const uint32_t cnt = acc_get(a, s.acc, c, addr_of(a, p));
      if (cnt > 0) {
        if (METHOD == 0) {
          key = cnt;
        } else {
          const double jac = (double)cnt / (double)(h2 + (long long)a.tdeg[p] - (long long)cnt);
          key = (unsigned long long)__double_as_longlong(jac);
        }
        col = a.inv[p];
        ok = key >= sthr && (!have || better(key, col, tkey, tcol));
      }
    }
    if (n > TK_WB - 64) {  // room for a full block of offers: keep the best k first
      wave_sync();
      unsigned long long ka;
      int ca;
      wave_sort(wk, wc, n, ka, ca);
      n = min(n, k);
      wave_sync();
      if (lane < n) {
        wk[lane] = ka;
        wc[lane] = ca;
      }
      if (n == k) {
        tkey = __shfl(ka, k - 1, 64);
        tcol = __shfl(ca, k - 1, 64);
        have = true;
        if (lane == 0) atomicMax(&s.sthr, tkey);
        ok = ok && better(key, col, tkey, tcol);
      }
    }
    const unsigned long long bal = __ballot(ok);
    if (ok) {
      const int slot = n + (int)__popcll(bal & ((1ull << lane) - 1ull));
      if (TK_OK(slot < TK_WB, 10, slot, TK_WB)) {
        wk[slot] = key;
        wc[slot] = col;
      }
    }
    n += (int)__popcll(bal);
  }
  // each wave's best k, packed in wave order, then one merge (sel_end)
  wave_sync();
  unsigned long long ka;
  int ca;
  wave_sort(wk, wc, n, ka, ca);
  const int m = min(n, k);
  if (lane == 0) s.wcnt[w] = m;
  __syncthreads();  // every wave holds its entries in registers before any region is overwritten
  int off = 0;
  for (int v = 0; v < w; ++v) off += s.wcnt[v];
  if (lane < m && TK_OK(off + lane < TK_SEL, 10, off + lane, TK_SEL)) {
    s.key[off + lane] = ka;
    s.col[off + lane] = ca;
  }
  if (tid == 0) {
    int tot = 0;
    for (int v = 0; v < NWV; ++v) tot += s.wcnt[v];
    s.n = tot;
  }
  __syncthreads();
  sel_end(a, s, METHOD, it);
  return nc;
}



// Dense counts of the hot prefix of N'(x) (single counter chunk, a0 = 0; header comment). h2 /
// np / fix receive this thread's share of |H2(x)|, of sum_{w in H2(x)} |N(w)| and of the rows
// pushed as corrections. Returns the address bound below which the walk skips targets.
// The members of hot target b_i (i >= 1) already counted through b_0 .. b_{i-1} -- the bits of
// N(b_i) AND (N(b_0) OR ... OR N(b_{i-1})), x's bit cleared -- each handed to fn(w, r0, len) by the
// thread owning its bitmap word (r0: w's row in pci, len = |N(w)|).
template <class Fn>
__device__ __attribute__((always_inline)) void dense_overlap(const TkArgs& a, const int32_t* rowx, int i, int x, Fn fn) {
  const int64_t pi = p_of(a, rowx[i]);
  const int64_t xo = (int64_t)x - a.slo;
  const uint32_t* bi = a.dw_bm + pi * a.dw_bmw;
  for (int64_t k = threadIdx.x; k < a.dw_bmw; k += TK_NT) {
    uint32_t o = 0;
    for (int j = 0; j < i; ++j) o |= a.dw_bm[p_of(a, rowx[j]) * a.dw_bmw + k];
    uint32_t m = bi[k] & o;
    if (k == (xo >> 5)) m &= ~(1u << (xo & 31));  // x: handled by the caller
    while (m) {
      const int bit = __ffs(m) - 1;
      m &= m - 1;
      const int64_t w = a.slo + 32 * k + bit;
      const int64_t r0 = a.rp[w] - a.pbase;
      fn(w, r0, (int)(a.rp[w + 1] - a.rp[w]));
    }
  }
}

template <bool FUSED>
__device__ __attribute__((always_inline)) int32_t dense_pass(const TkArgs& a, TkShared& s, int x, int du,
                                                             const int32_t* rowx, long long& h2, long long& np,
                                                             long long& fix) {
  const int tid = threadIdx.x;
  unsigned long long* aah = reinterpret_cast<unsigned long long*>(s.acc) + (a.h_word >> 1);
  if (tid == 0) {
    const int32_t abound = (int32_t)addr_of(a, a.dw_n);
    int nd = 0;
    while (nd < du && nd < a.dw_max && rowx[nd] < abound) ++nd;
    s.nd = nd;
  }
  __syncthreads();
  const int nd = s.nd;
  if (nd == 0) return 0;
  const unsigned long long wx = FUSED ? (unsigned long long)a.wtab[du] : 0ull;
  for (int i = 0; i < nd; ++i) {
    const int64_t pi = p_of(a, rowx[i]);
    if (!TK_OK(pi >= 0 && pi < a.dw_n, 12, pi, a.dw_n)) continue;  // uniform
    if (i > 0) {  // members of b_i counted before through b_0 .. b_{i-1}: remove them once
      dense_overlap(a, rowx, i, x, [&](int64_t, int64_t r0, int len) {
        const unsigned long long ww = FUSED ? (unsigned long long)a.wtab[len] : 0ull;
        for (int q = 0; q < len; ++q) {
          const int32_t e = TK_OK(r0 + q >= 0 && r0 + q < a.pci_len, 14, r0 + q, a.pci_len) ? a.pci[r0 + q] : 0;
          acc_sub(a, s.acc, e);
          if (FUSED && e < a.AH) aa_sub2(aah, p_of(a, e), ww);
        }
        h2 -= 1;
        np -= len;
        fix += len;
      });
      __syncthreads();
    }
    // every member's counts (and fused AA words), one word per thread
    const uint32_t* cv = a.dw_cv + pi * a.dw_words;
    for (int64_t k = tid; k < a.dw_words; k += TK_NT) s.acc[k] += cv[k];
    if (FUSED) {
      const unsigned long long* ca = a.dw_ca + pi * 2 * a.H;
      for (int64_t k = tid; k < 2 * a.H; k += TK_NT) aah[k] += ca[k];
    }
    __syncthreads();
    // x is a member of every b_i but not in H2(x)
    for (int j = tid; j < du; j += TK_NT) {
      const int32_t e = rowx[j];
      acc_sub(a, s.acc, e);
      if (FUSED && e < a.AH) aa_sub2(aah, p_of(a, e), wx);
    }
    __syncthreads();
    if (tid == 0) {
      h2 += a.dw_info[2 * pi] - 1;
      np += a.dw_info[2 * pi + 1] - du;
      fix += du;
    }
  }
  return rowx[nd - 1] + 1;
}

// The hash AA pass (MODE 1) with the same nd hot targets as the count pass: each hashed
// candidate t gets sum_i CAF_{b_i}[t] (the exact words of ALL members of b_i), then the members of
// b_i already counted through an earlier b_j give their term back. x's own term never reaches a
// candidate (candidates lie outside N'(x)). Returns the walk's skip bound (0: no dense targets).
__device__ __attribute__((always_inline)) int32_t dense_aa_hash(const TkArgs& a, TkShared& s, int x, const int32_t* rowx) {
  const int nd = s.nd;
  if (nd == 0 || !a.dw_caf) return 0;
  for (int h = threadIdx.x; h < TK_AH; h += TK_NT) {
    const int32_t e = s.col[h];
    if (e == (int32_t)TK_EMPTY) continue;
    const int64_t t = p_of(a, e);
    unsigned long long lo = 0, hi = 0;
    for (int i = 0; i < nd; ++i) {
      const unsigned long long* caf = a.dw_caf + 2 * (p_of(a, rowx[i]) * a.T + t);
      lo += caf[0];
      hi += caf[1];
    }
    s.key[2 * h] += lo;
    s.key[2 * h + 1] += hi;
  }
  __syncthreads();
  for (int i = 1; i < nd; ++i)
    dense_overlap(a, rowx, i, x, [&](int64_t, int64_t r0, int len) {
      const unsigned long long ww = (unsigned long long)a.wtab[len];
      for (int q = 0; q < len; ++q) {
        const int32_t e = a.pci[r0 + q];
        int h = hash_slot(e);
        for (int pr = 0; pr < TK_AH; ++pr) {
          const int32_t c = s.col[h];
          if (c == e) {
            aa_sub2(s.key, h, ww);
            break;
          }
          if (c == (int32_t)TK_EMPTY) break;
          h = (h + 1) & (TK_AH - 1);
        }
      }
    });
  __syncthreads();
  return rowx[nd - 1] + 1;
}

// The direct AA pass (MODE 2), targets [d0, d1) as word pairs in acc64: the same dense
// contributions for the slice (x's own entries are cleared after the pass anyway).
__device__ __attribute__((always_inline)) int32_t dense_aa_direct(const TkArgs& a, TkShared& s, int x, const int32_t* rowx,
                                                                  int64_t d0, int64_t d1) {
  const int nd = s.nd;
  if (nd == 0 || !a.dw_caf) return 0;
  unsigned long long* acc64 = reinterpret_cast<unsigned long long*>(s.acc);
  for (int64_t q = threadIdx.x; q < 2 * (d1 - d0); q += TK_NT) {
    unsigned long long v = 0;
    for (int i = 0; i < nd; ++i) v += a.dw_caf[2 * (p_of(a, rowx[i]) * a.T + d0) + q];
    acc64[q] += v;
  }
  __syncthreads();
  for (int i = 1; i < nd; ++i)
    dense_overlap(a, rowx, i, x, [&](int64_t, int64_t r0, int len) {
      const unsigned long long ww = (unsigned long long)a.wtab[len];
      for (int q = 0; q < len; ++q) {
        const int64_t p = p_of(a, a.pci[r0 + q]);
        if (p >= d0 && p < d1) aa_sub2(acc64, p - d0, ww);
      }
    });
  __syncthreads();
  return rowx[nd - 1] + 1;
}

// Dense counts of one hot target p (one workgroup): every member w of N(b) pushes N'(w) into LDS
// counters (and the fused AA words of the H most popular targets), w's bit is set in the member
// bitmap, and the words go out to dw_cv / dw_ca. dw_bm and dw_info are zeroed before.
__global__ __launch_bounds__(TK_NT) void k_tk_dense_fill(TkArgs a) {
  __shared__ uint32_t acc[TK_ACC_WORDS];
  __shared__ long long red[TK_NT / 64];
  const int tid = threadIdx.x;
  const int p = blockIdx.x;
  for (int64_t i = tid; i < a.acc_words; i += TK_NT) acc[i] = 0;
  __syncthreads();
  unsigned long long* aah = reinterpret_cast<unsigned long long*>(acc) + (a.h_word >> 1);
  const int b = a.inv[p];
  const int64_t rs = a.rp[b], re = a.rp[b + 1];
  long long sum = 0;
  for (int64_t k = rs + tid; k < re; k += TK_NT) {
    const int w = a.ci[k];
    const int64_t wo = (int64_t)w - a.slo;
    atomicOr(&a.dw_bm[(int64_t)p * a.dw_bmw + (wo >> 5)], 1u << (wo & 31));
    const int64_t r0 = a.rp[w] - a.pbase;
    const int len = (int)(a.rp[w + 1] - a.rp[w]);
    unsigned long long* caf = a.dw_caf ? a.dw_caf + 2 * (int64_t)p * a.T : nullptr;
    const unsigned long long ww = a.H > 0 || caf ? (unsigned long long)a.wtab[len] : 0ull;
    for (int q = 0; q < len; ++q) {
      const int32_t e = a.pci[r0 + q];
      atomicAdd(&acc[e >> 2], 1u << ((e & 3) << 3));
      if (a.H > 0 && e < a.AH)
        aa_push2(aah, p_of(a, e), ww);
      else if (caf)
        aa_push2(caf, p_of(a, e), ww);  // device-scope: the targets outside the fused region
    }
    sum += len;
  }
  for (int d = 32; d > 0; d >>= 1) sum += __shfl_down(sum, d, 64);
  if ((tid & 63) == 0) red[tid >> 6] = sum;
  __syncthreads();
  if (tid == 0) {
    long long t = 0;
    for (int w = 0; w < TK_NT / 64; ++w) t += red[w];
    a.dw_info[2 * p] = re - rs;
    a.dw_info[2 * p + 1] = t;
  }
  for (int64_t k = tid; k < a.dw_words; k += TK_NT) const_cast<uint32_t*>(a.dw_cv)[(int64_t)p * a.dw_words + k] = acc[k];
  if (a.H > 0 && a.dw_ca)
    for (int64_t k = tid; k < 2 * a.H; k += TK_NT) {
      const_cast<unsigned long long*>(a.dw_ca)[(int64_t)p * 2 * a.H + k] = aah[k];
      if (a.dw_caf) a.dw_caf[2 * (int64_t)p * a.T + k] = aah[k];  // the fused targets' words, in CAF too
    }
}

// The arguments stay a by-value struct: through a pointer (round 6) the kernel spilled fewer
// registers (SGPR spills 315 -> 52, VGPR spills 126 -> 65, scratch 396 -> 248 bytes per lane) and
// was slower: 15.47 / 15.48 against 15.33 / 15.30 ms alternating on one box (r06_ab1).
__global__ __launch_bounds__(TK_NT) void k_topk(TkArgs a) {
  __shared__ TkShared s;
  const int tid = threadIdx.x;
  unsigned long long* acc64 = reinterpret_cast<unsigned long long*>(s.acc);
  TKP_INIT
  for (;;) {
    __syncthreads();
    if (tid == 0) s.item = (int)atomicAdd(&a.counters[0], 1ull);
    __syncthreads();
    if (s.item >= a.n_src) break;
    const int it = a.order ? a.order[s.item] : s.item;
    TKP(0)
    const int x = a.src[it];
    const int64_t xb = a.rp[x];
    const int du = (int)(a.rp[x + 1] - xb);
    const int32_t* rowx = a.pci + (xb - a.pbase);
    for (int i = tid; i < TK_FILT; i += TK_NT) s.filt[i] = 0;
    if (tid < 3) s.nv[tid] = 0;
    if (tid == 0) s.nd = 0;
    __syncthreads();
    for (int j = tid; j < du; j += TK_NT) {
      const uint32_t b = filt_bit(rowx[j]);
      atomicOr(&s.filt[b >> 5], 1u << (b & 31));
    }
    __syncthreads();
    const bool want_cn = a.mask & (BLP_CN | BLP_ADAMIC), want_j = a.mask & BLP_JACCARD,
               want_aa = a.mask & BLP_ADAMIC;
    long long h2 = 0, ncand = 0;
    for (int ci = 0; ci < a.n_chunks; ++ci) {
      const TkChunk c = a.chunks[ci];
      const bool fused = want_aa && a.H > 0 && a.n_chunks == 1;
      const int words = fused ? (int)(a.h_word + 4 * a.H) : (int)((c.a1 - c.a0 + 3) >> 2);
      for (int i = tid; i < words; i += TK_NT) s.acc[i] = 0;
      __syncthreads();
      TKP(1)
      long long np = 0, dh = 0, dnp = 0, dfix = 0;
      int32_t a_dense = 0;  // hot targets below this address were counted densely
      if (a.dw_n > 0 && a.n_chunks == 1)
        a_dense = fused ? dense_pass<true>(a, s, x, du, rowx, dh, dnp, dfix)
                        : dense_pass<false>(a, s, x, du, rowx, dh, dnp, dfix);
      const long long h = fused ? push_pass<3>(a, s, x, xb, du, rowx, c, 0, 0, 0, ci == 0, &np, a_dense)
                                : push_pass<0>(a, s, x, xb, du, rowx, c, 0, 0, 0, ci == 0, &np, a_dense);
      TKP(2)
      if (ci == 0) {
        h2 = block_sum(s, h + dh);
        const long long walked = block_sum(s, np);
        np = block_sum(s, np + dnp);
        dfix = block_sum(s, dfix);
        if (tid == 0) {
          atomicAdd(&a.counters[3], (unsigned long long)h2);
          atomicAdd(&a.counters[4], (unsigned long long)np);
          atomicAdd(&a.counters[6], (unsigned long long)(walked + dfix));
          atomicAdd(&a.counters[7], (unsigned long long)s.nd);
        }
      }
      for (int j = tid; j < du; j += TK_NT) {
        const int32_t e = rowx[j];
        if (e >= c.a0 && e < c.a1) acc_clear(a, s.acc, c, e);
      }
      __syncthreads();
      const bool wsel = TK_WB == 128 && a.wavesel && a.k <= TK_WK;  // wave_sort: two entries per lane
      if (want_cn) ncand += wsel ? sel_counts_wave<0>(a, s, it, c, h2, true) : sel_counts<0>(a, s, it, c, h2, true);
      TKP(3)
      if (want_j)
        ncand += wsel ? sel_counts_wave<1>(a, s, it, c, h2, !want_cn) : sel_counts<1>(a, s, it, c, h2, !want_cn);
      TKP(8)
    }
    ncand = block_sum(s, ncand);
    if (want_aa && ncand > 0) {
      bool done = false;
      if (a.n_chunks == 1) {
        const TkChunk c = a.chunks[0];
        uint32_t thr = 1;
        if (s.nv[0] == a.k) {
          const unsigned long long cnt_k = a.keys[((size_t)0 * a.n_src + it) * a.k + a.k - 1];
          thr = (uint32_t)max(1.0, floor((double)cnt_k * a.ratio * (1.0 - 1e-9)));
        }
        long long nc = 0, nc_out = 0;
        // a count >= thr needs degree >= thr: only the prefix of the degree order can qualify
        const int64_t pcut = min(c.c1, thr < a.ge_n ? (int64_t)a.ge[thr] : (int64_t)0);
        for (int64_t p = c.c0 + tid; p < pcut; p += TK_NT) {
          const bool hit = acc_get(a, s.acc, c, addr_of(a, p)) >= thr;
          nc += hit;
          nc_out += hit && p >= a.H;
        }
        nc = block_sum(s, nc);
        nc_out = block_sum(s, nc_out);
        if (a.H > 0 && nc_out == 0) {
          // every target that can reach the top k is one of the H fused ones: their exact
          // sums are already in LDS (the candidates are the targets with a count)
          const unsigned long long* aah = acc64 + (a.h_word >> 1);
          sel_begin(a, s, 2, it);
          for (int64_t base = 0; base < a.H; base += TK_NT) {
            const int64_t p = base + tid;
            const bool ok = p < a.H && acc_get(a, s.acc, c, addr_of(a, p)) > 0;
            const int par = (int)((base / TK_NT) & 1);
            sel_offer(s, ok, ok ? aa_key(aah, p) : 0ull, ok ? a.inv[p] : 0, par);
            sel_round_end(a, s, par);
          }
          sel_end(a, s, 2, it);
          if (tid == 0) atomicAdd(&a.counters[5], 1ull);
          done = true;
          TKP(4)
        } else if (nc <= a.hcap) {
          for (int i = tid; i < TK_SEL; i += TK_NT) {
            s.col[i] = (int32_t)TK_EMPTY;
            s.key[i] = 0;
          }
          __syncthreads();
          for (int64_t p = c.c0 + tid; p < pcut; p += TK_NT) {
            const int32_t e = (int32_t)addr_of(a, p);
            if (acc_get(a, s.acc, c, e) >= thr) {
              int h = hash_slot(e), probes = 0;
              while (atomicCAS(&s.col[h], (int32_t)TK_EMPTY, e) != (int32_t)TK_EMPTY) {
                ++probes;
                if (!TK_OK(probes < TK_AH, 11, probes, TK_AH)) break;
                h = (h + 1) & (TK_AH - 1);
              }
            }
          }
          __syncthreads();
          const int32_t a_dense1 = dense_aa_hash(a, s, x, rowx);
          push_pass<1>(a, s, x, xb, du, rowx, c, thr, 0, 0, false, nullptr, a_dense1);
          // hash slots -> selection entries (key = bits of the exact AA double, col = dense target id)
          unsigned long long kv[TK_SEL / TK_NT];
          int cv[TK_SEL / TK_NT];
          for (int r = 0; r < TK_SEL / TK_NT; ++r) {
            const int i = tid + r * TK_NT;
            const int32_t e = i < TK_AH ? s.col[i] : (int32_t)TK_EMPTY;
            kv[r] = e == (int32_t)TK_EMPTY ? 0ull : aa_key(s.key, i);
            cv[r] = e == (int32_t)TK_EMPTY ? 0x7FFFFFFF : a.inv[p_of(a, e)];
          }
          __syncthreads();
          for (int r = 0; r < TK_SEL / TK_NT; ++r) {
            s.key[tid + r * TK_NT] = kv[r];
            s.col[tid + r * TK_NT] = cv[r];
          }
          if (tid == 0) {
            s.have_thr = 0;
            s.n = TK_SEL;
          }
          __syncthreads();
          compact(a, s, TK_SEL);
          {
            // entries with key 0 are empty slots sorted last; at most nc are real
            const int nv = min((int)nc, a.k);
            const size_t base = ((size_t)2 * a.n_src + it) * a.k;
            for (int i = tid; i < nv; i += TK_NT) {
              a.keys[base + i] = s.key[i];
              a.cols[base + i] = s.col[i];
            }
            if (tid == 0) s.nv[2] = nv;
            __syncthreads();
          }
          if (tid == 0) atomicAdd(&a.counters[1], 1ull);
          done = true;
          TKP(5)
        }
      }
      if (!done) {
        for (int64_t d0 = 0; d0 < a.T; d0 += a.aa_chunk) {
          const int64_t d1 = min(a.T, d0 + a.aa_chunk);
          for (int64_t i = tid; i < 2 * (d1 - d0); i += TK_NT) acc64[i] = 0;
          __syncthreads();
          const int32_t a_dense2 = dense_aa_direct(a, s, x, rowx, d0, d1);
          push_pass<2>(a, s, x, xb, du, rowx, a.chunks[0], 0, d0, d1, false, nullptr, a_dense2);
          for (int j = tid; j < du; j += TK_NT) {
            const int64_t p = p_of(a, rowx[j]);
            if (p >= d0 && p < d1 && TK_OK(2 * (p - d0) + 1 < a.acc_words / 2, 6, p - d0, a.acc_words / 4))
              acc64[2 * (p - d0)] = acc64[2 * (p - d0) + 1] = 0;
          }
          __syncthreads();
          sel_begin(a, s, 2, it);
          for (int64_t base = d0; base < d1; base += TK_NT) {
            const int64_t p = base + tid;
            const unsigned long long v = p < d1 ? aa_key(acc64, p - d0) : 0ull;
            const int par = (int)(((base - d0) / TK_NT) & 1);
            sel_offer(s, v > 0, v, v > 0 ? a.inv[p] : 0, par);
            sel_round_end(a, s, par);
          }
          sel_end(a, s, 2, it);
        }
        if (tid == 0) atomicAdd(&a.counters[2], 1ull);
        TKP(6)
      }
    }
    // pad the unused tail of each list
    for (int m = 0; m < 3; ++m) {
      const size_t base = ((size_t)m * a.n_src + it) * a.k;
      for (int i = s.nv[m] + tid; i < a.k; i += TK_NT) {
        a.keys[base + i] = 0;
        a.cols[base + i] = -1;
      }
    }
    if (tid == 0) a.ncand[it] = ncand;
    TKP(7)
  }
  TKP_FLUSH
}

}  // namespace

using namespace blp;

#ifdef BLP_PROF
extern "C" int blp_topk_prof_read(unsigned long long* out) {  // experiment builds only; then reset
  BLP_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tkprof), sizeof(unsigned long long) * 16));
  unsigned long long z[16] = {0};
  BLP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_tkprof), z, sizeof(z)));
  return BLP_OK;
}
#endif

struct blp_topk {
  blp_graph* g = nullptr;
  int64_t slo = 0, shi = 0, tlo = 0, thi = 0, T = 0;
  int64_t pbase = 0;
  int64_t n32 = 0, n16 = 0;  // tier boundaries in permuted order
  int64_t A16 = 0, A8 = 0;   // byte addresses where the u16 / u8 tiers start
  int64_t H = 0, AH = 0, h_word = 0;  // fused AA targets
  int64_t ge_n = 0;                   // entries of ge (degree -> prefix length)
  int64_t acc_words = TK_ACC_WORDS;
  double ratio = 0.0;
  bool have_aa = false;
  std::vector<TkChunk> chunks;
  int64_t aa_chunk = 0;
  DevBuf perm, inv, tdeg, ge, pci, d_chunks, src, order, keys, cols, ncand, counters, wtab, x2_off, x2;
  bool ordered = false;  // t->order holds a largest-first dequeue order of the sources
  std::vector<int32_t> h_perm;  // target offset -> permuted id (the hot targets are p < dw_n)
  DevBuf dw_cv, dw_ca, dw_bm, dw_info, dw_caf;  // dense counts of the hot targets (see the header comment)
  int64_t dw_n = 0, dw_words = 0, dw_bmw = 0;
  int64_t kbase = 0, x2_entries = -1;
  int64_t pci_n = 0, x2_n = 0;  // entries uploaded to pci / x2, padding included
  int64_t n_src = 0;
  int k = 0;
  uint32_t mask = 0;
  bool ran = false;
  KernelTimer timer;
};

namespace {

int64_t env_i64(const char* name, int64_t dflt) {
  const char* v = getenv(name);
  return (v && *v) ? atoll(v) : dflt;
}

int64_t host_addr(const blp_topk* t, int64_t p) {
  return p < t->n32 ? 4 * p : p < t->n16 ? t->A16 + 2 * (p - t->n32) : t->A8 + (p - t->n16);
}

int64_t chunk_words(const blp_topk* t, int64_t c0, int64_t c1) { return (host_addr(t, c1) - host_addr(t, c0) + 3) / 4; }

void plan_chunks(blp_topk* t) {
  t->chunks.clear();
  int64_t c0 = 0;
  do {
    int64_t lo = c0 + 1, hi = t->T;  // largest c1 in [c0+1, T] that fits
    if (hi <= c0) hi = c0 + 1;
    while (lo < hi) {
      const int64_t mid = lo + (hi - lo + 1) / 2;
      if (chunk_words(t, c0, mid) <= t->acc_words) lo = mid; else hi = mid - 1;
    }
    int64_t c1 = std::min<int64_t>(lo, std::max<int64_t>(t->T, c0 + 1));
    while (c1 < t->T && c1 > c0 + 1 && host_addr(t, c1) % 4) --c1;  // next chunk starts on a word
    TkChunk c{};
    c.c0 = c0;
    c.c1 = c1;
    c.a0 = host_addr(t, c0);
    c.a1 = host_addr(t, c1);
    t->chunks.push_back(c);
    c0 = c1;
  } while (c0 < t->T);
  t->aa_chunk = t->acc_words / 4;
  // fused AA (single counter chunk): the most popular targets get exact word pairs in the spare words
  t->H = 0;
  if (t->chunks.size() == 1 && !env_i64("BLP_TOPK_NO_FUSE", 0)) {
    t->h_word = (chunk_words(t, 0, t->T) + 1) / 2 * 2;
    t->H = std::max<int64_t>(0, std::min<int64_t>(t->T, (t->acc_words - t->h_word) / 4));
    t->H = std::min<int64_t>(t->H, env_i64("BLP_TOPK_FUSE_H", t->H));  // test knob: fewer fused targets
  }
  t->AH = t->H > 0 ? host_addr(t, t->H) : 0;
}

}  // namespace

// the kernel arguments of a run (k, mask) of handle t
static TkArgs topk_args(blp_topk* t, int k, uint32_t mask) {
  TkArgs a{};
  a.rp = t->g->d_rp;
  a.ci = t->g->d_ci;
  a.pci = t->pci.as<int32_t>();
  a.pbase = t->pbase;
  a.paddr = t->perm.as<int32_t>();
  a.H = (mask & BLP_ADAMIC) ? t->H : 0;
  a.AH = t->AH;
  a.h_word = t->h_word;
  a.n32 = t->n32;
  a.n16 = t->n16;
  a.A16 = t->A16;
  a.A8 = t->A8;
  a.inv = t->inv.as<int32_t>();
  a.tdeg = t->tdeg.as<int32_t>();
  a.ge = t->ge.as<int32_t>();
  a.ge_n = t->ge_n;
  a.wtab = t->wtab.as<long long>();
  a.x2_off = t->x2_entries >= 0 ? t->x2_off.as<int64_t>() : nullptr;
  a.x2 = t->x2_entries >= 0 ? t->x2.as<int32_t>() : nullptr;
  a.kbase = t->kbase;
  a.src = t->src.as<int32_t>();
  a.order = t->ordered ? t->order.as<int32_t>() : nullptr;
  a.n_src = (int)t->n_src;
  a.tlo = t->tlo;
  a.T = t->T;
  a.chunks = t->d_chunks.as<TkChunk>();
  a.n_chunks = (int)t->chunks.size();
  a.aa_chunk = t->aa_chunk;
  a.k = k;
  a.mask = mask;
  a.ratio = t->ratio;
  a.hcap = (int)std::max<int64_t>(0, std::min<int64_t>(TK_HCAP, env_i64("BLP_TOPK_HCAP", TK_HCAP)));
  a.keys = t->keys.as<unsigned long long>();
  a.cols = t->cols.as<int32_t>();
  a.ncand = t->ncand.as<int64_t>();
  a.counters = t->counters.as<unsigned long long>();
  a.acc_words = t->acc_words;
  a.pci_len = t->pci_n;
  a.x2_len = t->x2_n;
  a.dw_cv = t->dw_n ? t->dw_cv.as<uint32_t>() : nullptr;
  a.dw_ca = t->dw_n && a.H > 0 ? t->dw_ca.as<unsigned long long>() : nullptr;
  a.dw_bm = t->dw_n ? t->dw_bm.as<uint32_t>() : nullptr;
  a.dw_info = t->dw_n ? t->dw_info.as<long long>() : nullptr;
  a.dw_caf = t->dw_n && (mask & BLP_ADAMIC) && t->dw_caf.p ? t->dw_caf.as<unsigned long long>() : nullptr;
  a.dw_n = (int)t->dw_n;
  a.dw_max = (int)std::max<int64_t>(1, env_i64("BLP_TOPK_DENSE_MAX", 4));
  if (a.H > 0 && !a.dw_ca) a.dw_n = 0;  // counts without their AA words: walk every target
  a.dw_words = t->dw_words;
  a.dw_bmw = t->dw_bmw;
  a.slo = t->slo;
  a.wavesel = (int)env_i64("BLP_TK_WAVESEL", 1);  // r05_tk: 16.99 / 17.05 -> 16.53 / 16.48 ms at config 3
  return a;
}

extern "C" int blp_topk_create(blp_graph* g, int64_t src_lo, int64_t src_hi, int64_t tgt_lo, int64_t tgt_hi,
                               blp_topk** out) {
  BLP_CHECK(g && out, BLP_E_ARG, "blp_topk_create: bad arguments");
  BLP_CHECK(0 <= src_lo && src_lo <= src_hi && src_hi <= g->n && 0 <= tgt_lo && tgt_lo < tgt_hi && tgt_hi <= g->n,
            BLP_E_ARG, "blp_topk_create: bad id ranges");
  BLP_CHECK(src_hi <= tgt_lo || tgt_hi <= src_lo, BLP_E_ARG, "blp_topk_create: source and target ranges overlap");
  const int64_t* rp = g->hrp;
  const int32_t* ci = host_col_idx(g);
  if (!ci) return BLP_E_STATE;
  // bipartite check: every source row points into the targets and every target row into the sources
  for (int64_t v = src_lo; v < src_hi; ++v)
    for (int64_t e = rp[v]; e < rp[v + 1]; ++e)
      if (ci[e] < tgt_lo || ci[e] >= tgt_hi)
        return fail(BLP_E_UNSUP, "blp_topk_create: graph is not bipartite between the given ranges");
  for (int64_t v = tgt_lo; v < tgt_hi; ++v)
    for (int64_t e = rp[v]; e < rp[v + 1]; ++e)
      if (ci[e] < src_lo || ci[e] >= src_hi)
        return fail(BLP_E_UNSUP, "blp_topk_create: graph is not bipartite between the given ranges");
  int rc = set_device(g);
  if (rc) return rc;
  auto* t = new blp_topk();
  t->g = g;
  t->slo = src_lo;
  t->shi = src_hi;
  t->tlo = tgt_lo;
  t->thi = tgt_hi;
  t->T = tgt_hi - tgt_lo;
  t->pbase = rp[src_lo];
  const int64_t T = t->T;
  std::vector<int32_t> order(T), perm(T), inv(T), tdeg(T);
  for (int64_t i = 0; i < T; ++i) order[i] = (int32_t)i;
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
    return rp[tgt_lo + a + 1] - rp[tgt_lo + a] > rp[tgt_lo + b + 1] - rp[tgt_lo + b];
  });
  for (int64_t j = 0; j < T; ++j) {
    perm[order[j]] = (int32_t)j;
    inv[j] = (int32_t)(tgt_lo + order[j]);
    tdeg[j] = (int32_t)(rp[tgt_lo + order[j] + 1] - rp[tgt_lo + order[j]]);
  }
  t->h_perm = perm;
  // counter tiers: CN(x, b) <= |N(b)|, so |N(b)| <= 255 fits a u8 and <= 65535 a u16.
  // BLP_TOPK_T8 / BLP_TOPK_T16 lower the limits and BLP_TOPK_ACC_WORDS the counter space
  // (test knobs for the u32 tier and the multi-chunk path).
  const int64_t t8 = std::min<int64_t>(255, env_i64("BLP_TOPK_T8", 255));
  const int64_t t16 = std::min<int64_t>(65535, env_i64("BLP_TOPK_T16", 65535));
  t->acc_words = std::max<int64_t>(64, std::min<int64_t>(TK_ACC_WORDS, env_i64("BLP_TOPK_ACC_WORDS", TK_ACC_WORDS)));
  t->n32 = 0;
  while (t->n32 < T && tdeg[t->n32] > t16) ++t->n32;
  t->n16 = t->n32;
  while (t->n16 < T && tdeg[t->n16] > t8) ++t->n16;
  t->A16 = 4 * t->n32;
  t->A8 = (t->A16 + 2 * (t->n16 - t->n32) + 3) / 4 * 4;
  if (host_addr(t, T) >= (int64_t(1) << 31)) {
    delete t;
    return fail(BLP_E_UNSUP, "blp_topk_create: too many targets");
  }
  std::vector<int32_t> paddr(T);
  for (int64_t i = 0; i < T; ++i) paddr[i] = (int32_t)host_addr(t, perm[i]);
  // source rows with permuted target ids, each sorted (multi-threaded)
  const int64_t m = rp[src_hi] - t->pbase;
  std::vector<int32_t> pci(m + TK_RB, 0x7FFFFFFF);  // padded: rows are read in 16-byte vectors
  {
    const int nth = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    const int64_t nrows = src_hi - src_lo;
    for (int q = 0; q < nth; ++q) {
      th.emplace_back([&, q]() {
        const int64_t r0 = src_lo + nrows * q / nth, r1 = src_lo + nrows * (q + 1) / nth;
        for (int64_t v = r0; v < r1; ++v) {
          int32_t* row = pci.data() + (rp[v] - t->pbase);
          const int64_t len = rp[v + 1] - rp[v];
          for (int64_t e = 0; e < len; ++e) row[e] = paddr[ci[rp[v] + e] - tgt_lo];
          std::sort(row, row + len);
        }
      });
    }
    for (auto& h : th) h.join();
  }
  // Adamic-Adar: a source's weight depends on its degree only (bipartite: no self-loops), so
  // the kernel reads it from a per-degree table; the bounds use the sources of degree >= 2
  // (the only ones that reach a distance-3 target).
  int64_t maxdeg = 0;
  for (int64_t v = src_lo; v < src_hi; ++v) maxdeg = std::max<int64_t>(maxdeg, rp[v + 1] - rp[v]);
  std::vector<long long> wtab(maxdeg + 1, 0);
  if (g->d_aaw_fx && src_hi > src_lo) {
    std::vector<long long> w(src_hi - src_lo);
    BLP_HIP_OR(hipMemcpy(w.data(), g->d_aaw_fx + src_lo, 8 * w.size(), hipMemcpyDeviceToHost),
               [&](int r) { delete t; return r; });
    long long wmin = LLONG_MAX, wmax = 0;
    for (int64_t v = src_lo; v < src_hi; ++v) {
      const int64_t d = rp[v + 1] - rp[v];
      wtab[d] = w[v - src_lo];
      if (d >= 2) {
        wmin = std::min(wmin, w[v - src_lo]);
        wmax = std::max(wmax, w[v - src_lo]);
      }
    }
    t->have_aa = true;
    t->ratio = wmax > 0 ? (double)wmin / (double)wmax : 1.0;
  }
  // Expanded wedge rows: for every target b' (CSR order) and member w of N(b'), N'(w) stored
  // back to back (sum over sources of deg^2 entries). A source's walk then reads each N(b')'s
  // wedges sequentially instead of chasing rp[w] -> N(w) per member. Skipped above a memory
  // budget (BLP_TOPK_EXPAND_MB, default 16 GiB) or with BLP_TOPK_EXPAND=0.
  const int64_t kbase = rp[tgt_lo], mt = rp[tgt_hi] - kbase;
  std::vector<int64_t> x2_off;
  std::vector<int32_t> x2;
  {
    int64_t total = 0;
    for (int64_t v = src_lo; v < src_hi; ++v) total += (rp[v + 1] - rp[v]) * (rp[v + 1] - rp[v]);
    const int64_t budget = env_i64("BLP_TOPK_EXPAND_MB", 16384) << 20;
    if (env_i64("BLP_TOPK_EXPAND", 1) != 0 && 4 * total <= budget) {
      x2_off.resize(mt + 1);
      x2_off[0] = 0;
      for (int64_t i = 0; i < mt; ++i) {
        const int32_t w = ci[kbase + i];
        x2_off[i + 1] = x2_off[i] + (rp[w + 1] - rp[w]);
      }
      x2.resize(x2_off[mt] + TK_RB, 0x7FFFFFFF);  // padded like pci
      const int nth = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
      std::vector<std::thread> th;
      for (int q = 0; q < nth; ++q) {
        th.emplace_back([&, q]() {
          for (int64_t i = mt * q / nth; i < mt * (q + 1) / nth; ++i) {
            const int32_t w = ci[kbase + i];
            const int32_t* row = pci.data() + (rp[w] - t->pbase);
            std::copy(row, row + (rp[w + 1] - rp[w]), x2.data() + x2_off[i]);
          }
        });
      }
      for (auto& h : th) h.join();
    }
  }
  t->kbase = kbase;
  t->x2_entries = x2.empty() ? -1 : x2_off[mt];
  t->pci_n = (int64_t)pci.size();
  t->x2_n = (int64_t)x2.size();
  // ge[d] = targets of degree >= d, d in [0, max degree + 1] (degrees are non-increasing in p)
  std::vector<int32_t> ge((size_t)(T ? tdeg[0] : 0) + 2, 0);
  for (int64_t d = 0, j = T; d < (int64_t)ge.size(); ++d) {
    while (j > 0 && tdeg[j - 1] < d) --j;
    ge[d] = (int32_t)j;
  }
  t->ge_n = (int64_t)ge.size();
  plan_chunks(t);
  auto up = [&](DevBuf& b, const void* h, size_t bytes) -> int {
    int r = b.reserve(bytes);
    if (r) return r;
    BLP_HIP(hipMemcpy(b.p, h, bytes, hipMemcpyHostToDevice));
    return BLP_OK;
  };
  if ((rc = up(t->perm, paddr.data(), 4 * T)) || (rc = up(t->inv, inv.data(), 4 * T)) ||
      (rc = up(t->tdeg, tdeg.data(), 4 * T)) || (rc = up(t->ge, ge.data(), 4 * ge.size())) || (rc = up(t->pci, pci.data(), 4 * pci.size())) ||
      (rc = up(t->d_chunks, t->chunks.data(), sizeof(TkChunk) * t->chunks.size())) ||
      (rc = up(t->wtab, wtab.data(), 8 * wtab.size())) ||
      (!x2.empty() && ((rc = up(t->x2_off, x2_off.data(), 8 * x2_off.size())) ||
                       (rc = up(t->x2, x2.data(), 4 * x2.size())))) ||
      (rc = t->counters.reserve(64))) {
    blp_topk_destroy(t);
    return rc;
  }
  // dense counts of the hot targets (header comment): the prefix of the degree order whose
  // members' rows hold at least BLP_TOPK_DENSE_F (8) times the counter words, within
  // BLP_TOPK_DENSE_MB (1024) of HBM and 256 targets; one counter chunk only (BLP_TOPK_NO_DENSE=1: off)
  if (t->chunks.size() == 1 && T > 0 && !env_i64("BLP_TOPK_NO_DENSE", 0)) {
    const int64_t words = chunk_words(t, 0, T);
    const double f = getenv("BLP_TOPK_DENSE_F") ? atof(getenv("BLP_TOPK_DENSE_F")) : 8.0;
    const int64_t bmw = ((src_hi - src_lo + 31) / 32 + 3) / 4 * 4;
    const int64_t hw = t->have_aa ? 2 * t->H : 0;  // u64 AA words per target
    const int64_t per = 4 * words + 8 * hw + 4 * bmw;
    const int64_t cap = std::min<int64_t>(256, (env_i64("BLP_TOPK_DENSE_MB", 1024) << 20) / std::max<int64_t>(per, 1));
    int64_t n = 0;
    while (n < std::min<int64_t>(T, cap)) {
      const int b = inv[n];
      int64_t sum = 0;
      for (int64_t e = rp[b]; e < rp[b + 1]; ++e) sum += rp[ci[e] + 1] - rp[ci[e]];
      if ((double)sum < f * (double)words) break;
      ++n;
    }
    if (n > 0) {
      auto fail_out = [&](int r) {
        blp_topk_destroy(t);
        return r;
      };
      if ((rc = t->dw_cv.reserve(4 * words * n)) || (rc = t->dw_bm.reserve(4 * bmw * n)) ||
          (rc = t->dw_info.reserve(16 * n)) || (hw && (rc = t->dw_ca.reserve(8 * hw * n))))
        return fail_out(rc);
      // every target's exact AA words of the members (the hash / direct AA passes), within
      // BLP_TOPK_DENSE_AA_MB (2048) of HBM; without them those passes walk every target
      const int64_t caf_bytes = 16 * T * n;
      if (t->have_aa && caf_bytes <= (env_i64("BLP_TOPK_DENSE_AA_MB", 2048) << 20)) {
        if ((rc = t->dw_caf.reserve(caf_bytes))) return fail_out(rc);
        BLP_HIP_OR(hipMemsetAsync(t->dw_caf.p, 0, caf_bytes, g->stream), fail_out);
      }
      BLP_HIP_OR(hipMemsetAsync(t->dw_bm.p, 0, 4 * bmw * n, g->stream), fail_out);  // ordered before the fill
      t->dw_n = n;
      t->dw_words = words;
      t->dw_bmw = bmw;
      const TkArgs a = topk_args(t, 1, t->have_aa ? 7u : 3u);
      hipLaunchKernelGGL(k_tk_dense_fill, dim3((unsigned)n), dim3(TK_NT), 0, g->stream, a);
      BLP_HIP_OR(hipGetLastError(), fail_out);
      BLP_HIP_OR(hipStreamSynchronize(g->stream), fail_out);
    }
  }
  *out = t;
  return BLP_OK;
}

extern "C" int blp_topk_destroy(blp_topk* t) {
  if (!t) return BLP_OK;
  (void)set_device(t->g);
  for (DevBuf* b : {&t->perm, &t->inv, &t->tdeg, &t->ge, &t->pci, &t->d_chunks, &t->src, &t->order, &t->keys, &t->cols, &t->ncand,
                    &t->counters, &t->wtab, &t->x2_off, &t->x2, &t->dw_cv, &t->dw_ca, &t->dw_bm, &t->dw_info,
                    &t->dw_caf})
    b->release();
  timer_release(t->timer);
  delete t;
  return BLP_OK;
}

extern "C" int blp_topk_info(const blp_topk* t, int64_t* n_chunks, int64_t* tier32, int64_t* tier16,
                             int64_t* wedge_entries) {
  BLP_CHECK(t, BLP_E_ARG, "blp_topk_info: null handle");
  if (wedge_entries) *wedge_entries = t->x2_entries;
  if (n_chunks) *n_chunks = (int64_t)t->chunks.size();
  if (tier32) *tier32 = t->n32;
  if (tier16) *tier16 = t->n16 - t->n32;
  return BLP_OK;
}

extern "C" int blp_topk_set_sources(blp_topk* t, const int32_t* src, int64_t n_src) {
  BLP_CHECK(t && n_src >= 0 && (n_src == 0 || src), BLP_E_ARG, "blp_topk_set_sources: bad arguments");
  BLP_CHECK(n_src < (int64_t(1) << 31), BLP_E_ARG, "blp_topk_set_sources: too many sources");
  for (int64_t i = 0; i < n_src; ++i)
    BLP_CHECK(src[i] >= t->slo && src[i] < t->shi, BLP_E_ARG, "blp_topk_set_sources: source id outside the source range");
  int rc = set_device(t->g);
  if (rc) return rc;
  if ((rc = t->src.reserve(4 * std::max<int64_t>(n_src, 1)))) return rc;
  if (n_src) BLP_HIP(hipMemcpy(t->src.p, src, 4 * n_src, hipMemcpyHostToDevice));
  t->n_src = n_src;
  // Largest first: the one-workgroup-per-source kernel claims sources in descending order of their
  // two-hop walk, sum over b in N(x) of |N(b)|, so the long sources start early instead of
  // finishing last on a few CUs (BLP_TK_ORDER=0: list order). Results land by list index.
  t->ordered = false;
  const int64_t how = env_i64("BLP_TK_ORDER", 1);
  const int32_t* ci = n_src > 1 && how != 0 ? host_col_idx(t->g) : nullptr;
  if (n_src > 1 && how != 0 && !ci) return BLP_E_STATE;  // the column mirror fetch failed (its error is set)
  if (n_src > 1 && ci && how != 0) {
    const int64_t* rp = t->g->hrp;
    // 1: the walk's wedges, sum |N(b)|; 2 (measurement): its pushes, sum w2[b] over the walked
    // targets plus the counter words of each dense (hot) target's add
    const bool pushes = how == 2 && (int64_t)t->g->h_w2.size() > t->thi - 1 && (int64_t)t->h_perm.size() == t->T;
    std::vector<int64_t> est((size_t)n_src);
    for (int64_t i = 0; i < n_src; ++i) {
      int64_t w = 0;
      for (int64_t e = rp[src[i]]; e < rp[src[i] + 1]; ++e) {
        if (!pushes)
          w += rp[ci[e] + 1] - rp[ci[e]];
        else if (t->h_perm[ci[e] - t->tlo] < t->dw_n)
          w += t->dw_words;
        else
          w += (int64_t)t->g->h_w2[ci[e]];
      }
      est[i] = w;
    }
    std::vector<int32_t> ord((size_t)n_src);
    for (int64_t i = 0; i < n_src; ++i) ord[i] = (int32_t)i;
    std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return est[a] > est[b]; });
    if ((rc = t->order.reserve(4 * n_src))) return rc;
    BLP_HIP(hipMemcpy(t->order.p, ord.data(), 4 * n_src, hipMemcpyHostToDevice));
    t->ordered = true;
  }
  t->ran = false;
  return BLP_OK;
}

extern "C" int blp_topk_run(blp_topk* t, int k, uint32_t mask) {
  BLP_CHECK(t && k >= 1 && k <= TK_KMAX, BLP_E_ARG, "blp_topk_run: k must be in [1, 256]");
  BLP_CHECK(mask && !(mask & ~7u), BLP_E_ARG, "blp_topk_run: bad method mask");
  BLP_CHECK(!(mask & BLP_ADAMIC) || t->have_aa, BLP_E_STATE, "blp_topk_run: graph has no Adamic-Adar weights");
  int rc = set_device(t->g);
  if (rc) return rc;
  const size_t nk = (size_t)std::max<int64_t>(t->n_src, 1) * k;
  if ((rc = t->keys.reserve(3 * nk * 8)) || (rc = t->cols.reserve(3 * nk * 4)) ||
      (rc = t->ncand.reserve(8 * std::max<int64_t>(t->n_src, 1))))
    return rc;
  hipStream_t st = t->g->stream;
  BLP_HIP(hipMemsetAsync(t->counters.p, 0, 64, st));
  TkArgs a = topk_args(t, k, mask);
  hipEvent_t t0;
  if ((rc = timer_begin(t->timer, st, &t0))) return rc;
  if (t->n_src) {
    const int grid = (int)std::min<int64_t>(t->g->n_cu, t->n_src);
    hipLaunchKernelGGL(k_topk, dim3(grid), dim3(TK_NT), 0, st, a);
    BLP_HIP(hipGetLastError());
  }
  if ((rc = timer_end(t->timer, st, t0))) return rc;
#ifdef BLP_DEBUG
  {  // the walk's bound checks (see TK_OK): any violation fails the run
    long long dbg[4];
    BLP_HIP(hipStreamSynchronize(st));
    BLP_HIP(hipMemcpyFromSymbol(dbg, HIP_SYMBOL(g_tk_dbg), sizeof(dbg)));
    if (dbg[0]) {
      const long long z[4] = {0, 0, 0, 0};
      BLP_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_tk_dbg), z, sizeof(z)));
      char msg[160];
      snprintf(msg, sizeof msg, "blp_topk_run [BLP_DEBUG]: %lld bound violations; first at site %lld: %lld vs bound %lld",
               dbg[0], dbg[1], dbg[2], dbg[3]);
      return fail(BLP_E_STATE, msg);
    }
  }
#endif
  t->k = k;
  t->mask = mask;
  t->ran = true;
  return BLP_OK;
}

extern "C" int blp_topk_fetch(blp_topk* t, uint32_t method, int32_t* cols, double* scores, int64_t* n_cand) {
  BLP_CHECK(t && t->ran, BLP_E_STATE, "blp_topk_fetch: no completed run");
  BLP_CHECK(method == BLP_CN || method == BLP_JACCARD || method == BLP_ADAMIC, BLP_E_ARG,
            "blp_topk_fetch: method must be one of BLP_CN, BLP_JACCARD, BLP_ADAMIC");
  BLP_CHECK(t->mask & method, BLP_E_STATE, "blp_topk_fetch: method was not requested in the run");
  int rc = set_device(t->g);
  if (rc) return rc;
  BLP_HIP(hipStreamSynchronize(t->g->stream));
  const int m = method == BLP_CN ? 0 : method == BLP_JACCARD ? 1 : 2;
  const size_t nk = (size_t)t->n_src * t->k;
  if (nk && (cols || scores)) {
    std::vector<unsigned long long> keys(nk);
    std::vector<int32_t> c(nk);
    BLP_HIP(hipMemcpy(keys.data(), t->keys.as<unsigned long long>() + m * nk, 8 * nk, hipMemcpyDeviceToHost));
    BLP_HIP(hipMemcpy(c.data(), t->cols.as<int32_t>() + m * nk, 4 * nk, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nk; ++i) {
      if (cols) cols[i] = c[i];
      if (scores) {
        double v = 0.0;
        if (c[i] >= 0) {
          if (m == 0) v = (double)keys[i];
          else if (m == 1) { memcpy(&v, &keys[i], 8); }
          else memcpy(&v, &keys[i], 8);  // AA: the exact sum's double (blp_internal.h)
        }
        scores[i] = v;
      }
    }
  }
  if (n_cand && t->n_src) BLP_HIP(hipMemcpy(n_cand, t->ncand.p, 8 * t->n_src, hipMemcpyDeviceToHost));
  return BLP_OK;
}

extern "C" int blp_topk_stats(blp_topk* t, int which, double* total_ms, int64_t* launches) {
  BLP_CHECK(t && which >= 0 && which <= 8, BLP_E_ARG, "blp_topk_stats: bad arguments");
  int rc = set_device(t->g);
  if (rc) return rc;
  if (which == 8) {  // bytes one dense hot-target add reads: its packed counts and fused AA words
    if (total_ms) *total_ms = 0.0;
    if (launches) *launches = t->dw_n ? 4 * t->dw_words + (t->have_aa ? 16 * t->H : 0) : 0;
    return BLP_OK;
  }
  if (which == 0) {
    if ((rc = timer_collect(t->timer))) return rc;
    if (total_ms) *total_ms = t->timer.total_ms;
    if (launches) *launches = t->timer.launches;
    return BLP_OK;
  }
  // 1 / 2: sources whose AA went through the candidate hash / direct accumulation;
  // 3: sum of |H2(x)|; 4: sum over x and w in H2(x) of |N(w)| (the push volume of one pass);
  // 5: sources whose AA top-k came straight from the fused sums; 6: row entries actually pushed by
  // the count pass (walk + dense corrections); 7: dense target counts added; 8 (above): bytes read
  // per dense add
  BLP_HIP(hipStreamSynchronize(t->g->stream));  // blp_topk_run is asynchronous on g->stream
  unsigned long long c[8];
  BLP_HIP(hipMemcpy(c, t->counters.p, 64, hipMemcpyDeviceToHost));
  if (total_ms) *total_ms = 0.0;
  if (launches) *launches = (int64_t)c[which];
  return BLP_OK;
}

extern "C" int blp_topk_stats_reset(blp_topk* t) {
  BLP_CHECK(t, BLP_E_ARG, "blp_topk_stats_reset: null handle");
  int rc = set_device(t->g);
  if (rc) return rc;
  if ((rc = timer_collect(t->timer))) return rc;
  t->timer.total_ms = 0.0;
  t->timer.launches = 0;
  return BLP_OK;
}
