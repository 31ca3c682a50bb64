// Truncated-SVD scorer (svd.py:7-31), reconstruction on MI355X.
//
// The reference factors the binary user x business matrix with ARPACK (svd.py:24,
// sparse.linalg.svds) and scores a pair as np.dot(us[row], vt[:, col]) with us = u * s
// (svd.py:25-30). The factorisation stays on the host (the reference's own numeric,
// SURVEY.md §8(a) a9); the factors live in HBM in fp64 and the reconstruction runs here:
//   * k_svd_pairs  -- candidate pairs: 8 lanes per pair, 16-byte loads, xor-shuffle reduce.
//   * k_svd_topk   -- every business for a block of users: fp64 MFMA tiles
//                     (v_mfma_f64_16x16x4f64, D[user][business] = US[user] . Vt[:, business])
//                     with a fused running top-k per user (threshold + LDS candidate buffer),
//                     one partial list per (user, business chunk).
//   * k_svd_merge  -- merges the per-chunk lists: score descending, then column ascending.
//   * norm-pruned top-k (default; blp_svd_set_prune): a score is us[u] . v[b], so
//     |score| <= ||us[u]|| ||v[b]||. The businesses are numbered by ||v[b]|| descending (a
//     permuted copy of Vt, built once per handle), a first pass scores the first TK_SEED_COLS
//     of that order for every user, and the rest of the columns go to chunks that take tiles
//     round-robin (each chunk sees the norms descending) starting from the first pass's k-th
//     score: a wave stops when the bound of the next tile, ||us[u]|| ||v[c]|| (1 + 1e-9), is
//     strictly below every one of its 16 users' thresholds, since no later column can enter
//     a list. Same MFMA dot products, same lists as the dense pass (bit-exact).
// Factor layout: US [n_rows][kpad] and V [n_cols][kpad] row-major, Vt [kpad][ncol_pad];
// kpad = k rounded up to 16 (zero padding adds exact zeros to every dot product).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <vector>

#include "blp_internal.h"

struct blp_svd {
  int device = 0;
  int n_cu = 256;
  hipStream_t stream = nullptr;
  int64_t n_rows = 0, n_cols = 0, ncol_pad = 0;
  int k = 0, kpad = 0;
  double* d_us = nullptr;  // [n_rows][kpad]
  double* d_v = nullptr;   // [n_cols][kpad]
  double* d_vt = nullptr;  // [kpad][ncol_pad]
  blp::KernelTimer t_pairs, t_topk;
  hipEvent_t join_ev = nullptr;  // blp_svd_stream_join
  double* d_ps = nullptr;  // top-k scratch: per (user, chunk) partial lists, part_cap entries
  int32_t* d_pc = nullptr;
  int64_t part_cap = 0;
  // norm-pruned top-k (built on first use): Vt with columns by ||v|| descending, the sorted
  // norms (zeros past n_cols), the order (sorted position -> column; INT32_MAX past n_cols)
  int prune = 1;
  double* d_vtp = nullptr;
  double* d_vnp = nullptr;
  int32_t* d_perm = nullptr;
  unsigned long long* d_tiles = nullptr;  // MFMA tiles scored since the last blp_svd_tiles
  int64_t tiles_total = 0;                // tiles of the dense pass over the same calls
  int64_t tiles_dense = 0;                // tiles scored by dense-pass calls
};

namespace {

typedef double double4_t __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- pairs
__global__ __launch_bounds__(256) void k_svd_pairs(const double* __restrict__ us, const double* __restrict__ v, int kpad,
                                                   const int32_t* __restrict__ rows, const int32_t* __restrict__ cols,
                                                   int64_t n, double* __restrict__ out) {
  const int lane8 = threadIdx.x & 7;
  const int64_t groups = (int64_t)gridDim.x * (blockDim.x >> 3);
  for (int64_t p = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 3; p < n; p += groups) {
    const double2* a = reinterpret_cast<const double2*>(us + (int64_t)rows[p] * kpad);
    const double2* b = reinterpret_cast<const double2*>(v + (int64_t)cols[p] * kpad);
    double acc = 0.0;
    for (int j = lane8; j < kpad / 2; j += 8) {
      const double2 x = a[j], y = b[j];
      acc = fma(x.x, y.x, acc);
      acc = fma(x.y, y.y, acc);
    }
    acc += __shfl_xor(acc, 4, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 1, 64);
    if (lane8 == 0) out[p] = acc;
  }
}

// ---------------------------------------------------------------- dense top-k
constexpr int TK_WAVES = 4;        // waves per block; each owns 16 users
constexpr int TK_MAX = 32;         // largest top-k
constexpr int TK_BUF = 16;         // compaction once a user's buffer holds more (+16 per tile at most:
                                   // TK_MAX + TK_BUF + 16 <= 64 entries, one per lane)
constexpr int TK_GROUP = 16;       // tiles per LDS exclusion-mask refill

struct TopkArgs {
  const double* us;        // [n_rows][kpad]
  const double* vt;        // [kpad][ncol_pad]
  const int32_t* users;    // selected rows, n_users
  const int64_t* ex_off;   // exclusion CSR over selected users (or null)
  const int32_t* ex_col;
  int64_t n_users, n_cols, ncol_pad;
  int kpad, topk;
  int64_t chunk;           // businesses per chunk (multiple of 16)
  int n_chunks;
  double* part_score;      // [n_users][n_chunks][topk]
  int32_t* part_col;
  int64_t n_rows;          // rows of us: a selected row outside [0, n_rows) reads no memory
  // norm-pruned pass (PR = 1): vt is the norm-sorted copy, perm maps a sorted position to its
  // column, vnorm the sorted norms; chunk j of the grid takes the tiles col_base + 16 (j + i S),
  // S = gridDim.y, below n_cols; its list is chunk chunk_base + j of part_*; seeded: start
  // every user's threshold at the k-th entry of its chunk-0 list (the first pass)
  const int32_t* perm;
  const double* vnorm;
  int64_t col_base;
  int chunk_base, seeded;  // seeded: lists 0 .. seeded-1 hold the first pass
  unsigned long long* tiles;  // tiles scored (or null)
};

// better = higher score, then lower column
__device__ inline bool better(double s, int c, double t, int tc) { return s > t || (s == t && c < tc); }

// Keep the best `topk` of top[0..topk) + buf[0..nb) in top: one entry per lane (topk + nb <=
// 64), a 64-lane bitonic sort through cross-lane shuffles (21 compare-exchange stages, no
// LDS traffic beyond the loads and the stores), better-first; the k-th entry becomes the
// row's threshold.
__device__ inline void tk_compact(double* top_s, int* top_c, const double* buf_s, const int* buf_c, int nb, int topk,
                                  int lane, double* th_s, int* th_c) {
  double v = -DBL_MAX;
  int c = INT32_MAX;
  if (lane < topk) {
    v = top_s[lane];
    c = top_c[lane];
  } else if (lane < topk + nb) {
    v = buf_s[lane - topk];
    c = buf_c[lane - topk];
  }
#pragma unroll
  for (int k2 = 2; k2 <= 64; k2 <<= 1)
#pragma unroll
    for (int j = k2 >> 1; j > 0; j >>= 1) {
      const double pv = __shfl_xor(v, j, 64);
      const int pc = __shfl_xor(c, j, 64);
      const bool first = ((lane & j) == 0) == ((lane & k2) == 0);  // this lane keeps the better one
      if (first == better(pv, pc, v, c)) {
        v = pv;
        c = pc;
      }
    }
  const double tv = __shfl(v, topk - 1, 64);
  const int tc = __shfl(c, topk - 1, 64);
  if (lane < topk) {
    top_s[lane] = v;
    top_c[lane] = c;
  }
  if (lane == 0) {
    *th_s = tv;
    *th_c = tc;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// RT row tiles per wave (16 RT users): every B fragment fetched feeds RT MFMA chains, so the
// Vt stream per score is 8 KiB / (256 RT) -- RT = 2 halves the L2/MALL traffic of RT = 1.
// EXP = 1 (timing experiment only; no launch site instantiates it): the MFMA chains and fragment loads without
// the top-k epilogue (results are NOT valid)
template <int KPAD, int RT, int WAVES, int EXP = 0, int PR = 0>
__global__ __launch_bounds__(WAVES * 64) void k_svd_topk(TopkArgs a) {
  constexpr int R = 16 * RT;  // users per wave
  __shared__ double s_top[WAVES][R][TK_MAX];
  __shared__ int s_topc[WAVES][R][TK_MAX];
  __shared__ double s_buf[WAVES][R][TK_BUF + 16];
  __shared__ int s_bufc[WAVES][R][TK_BUF + 16];
  __shared__ int s_nb[WAVES][R];
  __shared__ double s_th[WAVES][R];
  __shared__ int s_thc[WAVES][R];
  __shared__ unsigned short s_exm[WAVES][R][TK_GROUP];
  constexpr int KS = KPAD / 4;  // MFMA k-steps
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t u0 = ((int64_t)blockIdx.x * WAVES + w) * R;
  if (u0 >= a.n_users) return;  // whole wave idle (no block barriers below)
  const int chunk = blockIdx.y;
  const int64_t cb = PR ? a.col_base + 16 * (int64_t)chunk : (int64_t)chunk * a.chunk;
  const int64_t ce = PR ? a.n_cols : min(a.n_cols, cb + a.chunk);
  const int64_t TS = PR ? 16 * (int64_t)gridDim.y : 16;  // column step between this chunk's tiles
  const int topk = a.topk;
  for (int i = lane; i < R * TK_MAX; i += 64) {
    s_top[w][i / TK_MAX][i % TK_MAX] = -DBL_MAX;
    s_topc[w][i / TK_MAX][i % TK_MAX] = INT32_MAX;
  }
  if (lane < R) {
    s_nb[w][lane] = 0;
    s_th[w][lane] = -DBL_MAX;
    s_thc[w][lane] = INT32_MAX;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // A fragments of tile t: A[i = lane & 15][k = 4 s + (lane >> 4)] = US[users[u0 + 16 t + i]][k]
  double af[RT][KS];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int64_t ui = u0 + 16 * t + (lane & 15);
    int64_t row = ui < a.n_users ? a.users[ui] : -1;
    if (row >= a.n_rows) row = -1;  // device-side guard (blp_svd_topk_device does not range-check)
#pragma unroll
    for (int s = 0; s < KS; ++s) af[t][s] = row >= 0 ? a.us[row * KPAD + 4 * s + (lane >> 4)] : 0.0;
  }
  const int my_row = lane >> 4;  // the C/D rows of this lane in tile t are 16 t + my_row + 4 r
  // Exclusions (the user's own reviews, sorted): every TK_GROUP tiles, lane r < R writes row
  // r's excluded columns of the next TK_GROUP * 16 columns into an LDS mask (one 16-bit word
  // per tile), reading its sorted list 4 entries at a time; each tile then takes its mask with
  // one LDS read. The global loads (and their vmcnt wait, which also waits for the B fragments
  // in flight: vmcnt counts in issue order) happen once per group, not inside the tile loop.
  int64_t ex_p = 0, ex_e = 0;
  if (!PR && a.ex_off && lane < R && u0 + lane < a.n_users) {
    ex_p = a.ex_off[u0 + lane];
    ex_e = a.ex_off[u0 + lane + 1];
    while (ex_p < ex_e && a.ex_col[ex_p] < cb) ++ex_p;
  }
  auto ex_group = [&](int64_t g0) __attribute__((always_inline)) {
    if (lane < R) {
#pragma unroll
      for (int q = 0; q < TK_GROUP; ++q) s_exm[w][lane][q] = 0;
      const int64_t g1 = g0 + 16 * TK_GROUP;
      while (ex_p < ex_e) {
        int v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ex_p + q < ex_e ? a.ex_col[ex_p + q] : INT32_MAX;
        int used = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (v[q] < g1) {  // sorted: a prefix of the four
            ++used;
            if (v[q] >= g0) s_exm[w][lane][(v[q] - g0) >> 4] |= (unsigned short)(1u << ((v[q] - g0) & 15));
          }
        ex_p += used;
        if (used < 4) break;
      }
    }
  };
  // B[k = 4 s + (lane >> 4)][j = lane & 15] = Vt[k][c0 + j]  (padded columns are zero).
  // Two fragment sets alternate (tiles c0 and c0 + 16): the loads of one tile are issued a
  // whole tile (16 dependent MFMAs) before its chain needs them, and no register copy sits
  // between a load and its use (a copy made the compiler wait on the just-issued loads at
  // the end of every tile: vmcnt(0), i.e. no prefetch at all).
  const double* vt_lane = a.vt + (int64_t)(lane >> 4) * a.ncol_pad + (lane & 15);
  double th[RT][4];  // thresholds of this lane's C/D rows (mirrors s_th / s_thc)
  int thc[RT][4];
  bool rowok[RT][4];  // the row is a real user (the last wave may be partial)
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) rowok[t][r] = u0 + 16 * t + my_row + 4 * r < a.n_users;
  double sd[RT][4];  // PR: the first pass's k-th entry of each row (the floor of its threshold)
  int sdc[RT][4];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sd[t][r] = -DBL_MAX;
      sdc[t][r] = INT32_MAX;
      const int64_t u = u0 + 16 * t + my_row + 4 * r;
      // the best k-th entry of the first pass's lists: the union of those lists holds topk
      // entries at least that good, so the final k-th score is never below it
      for (int j = 0; PR && j < a.seeded && u < a.n_users; ++j) {
        const int64_t o = (u * a.n_chunks + j) * topk + topk - 1;
        const double v = a.part_score[o];
        const int vc = a.part_col[o];
        if (better(v, vc, sd[t][r], sdc[t][r])) {
          sd[t][r] = v;
          sdc[t][r] = vc;
        }
      }
      th[t][r] = sd[t][r];
      thc[t][r] = sdc[t][r];
    }
  // PR: ||us[u]|| of this lane's rows (lanes 0-15 hold row lane & 15's sum of squares after the
  // cross-group reduction) and the rows' exclusion ranges (checked per candidate by search)
  double un[RT][4];
  int64_t exb[RT][4], exe[RT][4];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    double q = 0.0;
    if (PR) {
#pragma unroll
      for (int s = 0; s < KS; ++s) q = fma(af[t][s], af[t][s], q);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * t + my_row + 4 * r;
      un[t][r] = PR ? sqrt(__shfl(q, row & 15, 64)) : 0.0;
      exb[t][r] = exe[t][r] = 0;
      if (PR && a.ex_off && u0 + row < a.n_users) {
        exb[t][r] = a.ex_off[u0 + row];
        exe[t][r] = a.ex_off[u0 + row + 1];
      }
    }
  }
  int pcol0 = 0, pcol1 = 0;  // PR: the columns of the two fragment sets' tiles
  auto load_b = [&](double* bf, int& pcol, int64_t c) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < KS; ++s) bf[s] = vt_lane[(int64_t)(4 * s) * a.ncol_pad + c];
    if (PR) pcol = a.perm[c + (lane & 15)];
    // keep the scheduler from sinking these loads into the previous tile's MFMA chain (it
    // does so to shorten live ranges, which brings the wait back)
    __builtin_amdgcn_sched_barrier(0);
  };
  auto tile = [&](int64_t c0, const double* bf, int pcol) __attribute__((always_inline)) {
    double4_t d[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) d[t] = double4_t{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int t = 0; t < RT; ++t) d[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[t][s], bf[s], d[t], 0, 0, 0);
    const int cidx = (int)(c0 + (lane & 15));
    const int col = PR ? pcol : cidx;  // the business id (lists and ties use it)
    if (EXP == 1) {
#pragma unroll
      for (int t = 0; t < RT; ++t) th[t][0] += d[t][0] + d[t][1] + d[t][2] + d[t][3];
      return;
    }
    // lane r < R: excluded columns of row r in this tile
    const unsigned exm = !PR && a.ex_off && lane < R ? s_exm[w][lane][((c0 - cb) >> 4) % TK_GROUP] : 0u;
    // Thresholds live in registers (they change only when a row is compacted), so a tile
    // whose scores all fall below them costs a few VALU compares and one ballot: no LDS
    // round trip, no cross-lane shuffle unless the tile holds an excluded column.
    const bool anyex = __ballot(exm != 0) != 0;  // wave-uniform
    const bool colok = cidx < ce;
    bool pass[RT][4];
    bool anyp = false;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * t + my_row + 4 * r;
        // non-short-circuit: compares and mask ANDs, no branches
        const double sc = d[t][r];
        bool ok = colok & rowok[t][r] & ((sc > th[t][r]) | ((sc == th[t][r]) & (col < thc[t][r])));
        if (anyex) {
          const unsigned rm = (unsigned)__shfl((int)exm, row, 64);
          ok = ok && !((rm >> (lane & 15)) & 1u);
        }
        if (PR && ok && exe[t][r] > exb[t][r]) {  // a rare candidate: search the sorted exclusions
          int64_t lo = exb[t][r], hi = exe[t][r];
          while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (a.ex_col[mid] < col) lo = mid + 1; else hi = mid;
          }
          ok = !(lo < exe[t][r] && a.ex_col[lo] == col);
        }
        pass[t][r] = ok;
        anyp |= ok;
      }
    const bool last = c0 + TS >= ce;
    if (__ballot(anyp) == 0 && !last) return;  // wave-uniform: nothing enters any list
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (pass[t][r]) {
          const int row = 16 * t + my_row + 4 * r;
          const int slot = atomicAdd(&s_nb[w][row], 1);
          s_buf[w][row][slot] = d[t][r];
          s_bufc[w][row][slot] = col;
        }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // compact rows whose buffer could overflow on the next tile (one LDS read and a ballot
    // find them; the loop visits only those rows)
    const int my_nb = lane < R ? s_nb[w][lane] : 0;
    unsigned long long due = __ballot(lane < R && (my_nb > TK_BUF || (last && my_nb > 0)));
    if (!due) return;
    while (due) {
      const int row = __builtin_ctzll(due);
      due &= due - 1;
      const int nb = s_nb[w][row];
      tk_compact(s_top[w][row], s_topc[w][row], s_buf[w][row], s_bufc[w][row], nb, topk, lane, &s_th[w][row],
                 &s_thc[w][row]);
      if (lane == 0) s_nb[w][row] = 0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        th[t][r] = s_th[w][16 * t + my_row + 4 * r];
        thc[t][r] = s_thc[w][16 * t + my_row + 4 * r];
        if (PR && better(sd[t][r], sdc[t][r], th[t][r], thc[t][r])) {  // never below the first pass's
          th[t][r] = sd[t][r];
          thc[t][r] = sdc[t][r];
        }
      }
  };
  // PR: true when no column from c on can enter any of the wave's lists (wave-uniform)
  auto pruned = [&](int64_t c) __attribute__((always_inline)) {
    const double bn = a.vnorm[c] * (1.0 + 1e-9);
    bool keep = false;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) keep |= rowok[t][r] && !(un[t][r] * bn < th[t][r]);
    return __ballot(keep) == 0;
  };
  double b0[KS], b1[KS];
  unsigned long long n_tiles = 0;
  if (cb < ce) load_b(b0, pcol0, cb);
  for (int64_t c0 = cb; c0 < ce; c0 += 2 * TS) {
    if (!PR && a.ex_off && ((c0 - cb) >> 4) % TK_GROUP == 0) ex_group(c0);  // (TK_GROUP is even)
    const int64_t c1 = c0 + TS;
    load_b(b1, pcol1, c1 < ce ? c1 : c0);  // (past the chunk: a harmless re-read)
    if (PR && pruned(c0)) break;
    tile(c0, b0, pcol0);
    ++n_tiles;
    if (c1 >= ce) break;
    load_b(b0, pcol0, c1 + TS < ce ? c1 + TS : c1);
    if (PR && pruned(c1)) break;
    tile(c1, b1, pcol1);
    ++n_tiles;
  }
  if (PR) {
    // a pruned stop leaves buffered candidates: fold them into the lists
    unsigned long long due = __ballot(lane < R && s_nb[w][lane] > 0);
    while (due) {
      const int row = __builtin_ctzll(due);
      due &= due - 1;
      tk_compact(s_top[w][row], s_topc[w][row], s_buf[w][row], s_bufc[w][row], s_nb[w][row], topk, lane,
                 &s_th[w][row], &s_thc[w][row]);
      if (lane == 0) s_nb[w][row] = 0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    if (a.tiles && lane == 0) atomicAdd(a.tiles, n_tiles);
  }
  if (EXP == 1 && th[0][0] == 1.2345e300) a.part_score[0] = th[0][0];  // keeps the chains live
  for (int i = lane; i < R * topk; i += 64) {
    const int row = i / topk, q = i % topk;
    const int64_t u = u0 + row;
    if (u < a.n_users) {
      const int64_t o = (u * a.n_chunks + (PR ? a.chunk_base + chunk : chunk)) * topk + q;
      a.part_score[o] = s_top[w][row][q];
      a.part_col[o] = s_topc[w][row][q];
    }
  }
}

// One wave per user: best topk of n_chunks * topk partial entries. The filled entries (empty
// slots carry column INT32_MAX; a pruned chunk's list is all empty) are gathered into LDS
// first and ranked among themselves (columns are distinct across lists: no exact ties);
// slots past the filled count get (0.0, -1). More than TK_MERGE_CAP filled: rank in place.
constexpr int TK_MERGE_CAP = 1024;
__global__ __launch_bounds__(64) void k_svd_merge(const double* __restrict__ ps, const int32_t* __restrict__ pc,
                                                  int64_t n_users, int n_chunks, int topk, double* __restrict__ out_s,
                                                  int32_t* __restrict__ out_c) {
  __shared__ double m_s[TK_MERGE_CAP];
  __shared__ int m_c[TK_MERGE_CAP];
  __shared__ int m_n;
  const int64_t u = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = n_chunks * topk;
  const double* s = ps + u * n;
  const int32_t* c = pc + u * n;
  if (lane == 0) m_n = 0;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  for (int i = lane; i < n; i += 64) {
    const int vc = c[i];
    if (vc != INT32_MAX) {
      const int slot = atomicAdd(&m_n, 1);
      if (slot < TK_MERGE_CAP) {
        m_s[slot] = s[i];
        m_c[slot] = vc;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const int m = m_n;
  if (m <= TK_MERGE_CAP) {
    for (int i = lane; i < m; i += 64) {
      const double v = m_s[i];
      const int vc = m_c[i];
      int r = 0;
      for (int j = 0; j < m; ++j) r += better(m_s[j], m_c[j], v, vc);
      if (r < topk) {
        out_s[u * topk + r] = v;
        out_c[u * topk + r] = vc;
      }
    }
    for (int q = m + lane; q < topk; q += 64) {
      out_s[u * topk + q] = 0.0;
      out_c[u * topk + q] = -1;
    }
    return;
  }
  for (int i = lane; i < n; i += 64) {
    const double v = s[i];
    const int vc = c[i];
    int r = 0;
    for (int j = 0; j < n; ++j) r += better(s[j], c[j], v, vc) || (s[j] == v && c[j] == vc && j < i);
    if (r < topk) {
      out_s[u * topk + r] = vc == INT32_MAX ? 0.0 : v;
      out_c[u * topk + r] = vc == INT32_MAX ? -1 : vc;
    }
  }
}

// ---------------------------------------------------------------- norm order (pruned top-k)
constexpr int TK_SEED_COLS = 2048;  // the first pass: this many columns of largest ||v|| per user
constexpr int TK_PR_CHUNKS = 16;    // chunks of the pruned pass (tiles dealt round-robin)
constexpr int TK_SEED_CHUNKS = 4;   // chunks of the first pass (its tiles dealt round-robin too)

// key = the bits of ||v[c]|| (non-negative doubles order as their bit patterns), value = c
__global__ void k_vnorm(const double* __restrict__ v, int64_t n_cols, int kpad, unsigned long long* __restrict__ key,
                        int32_t* __restrict__ idx) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n_cols; c += (int64_t)gridDim.x * blockDim.x) {
    double q = 0.0;
    for (int j = 0; j < kpad; ++j) q = fma(v[c * kpad + j], v[c * kpad + j], q);
    key[c] = (unsigned long long)__double_as_longlong(sqrt(q));
    idx[c] = (int32_t)c;
  }
}

// sorted position j: the column, its norm and its Vt column (padding past n_cols: zeros)
__global__ void k_vt_perm(const double* __restrict__ vt, int64_t ncol_pad, int64_t n_cols, int kpad,
                          const unsigned long long* __restrict__ skey, const int32_t* __restrict__ sidx,
                          double* __restrict__ vtp, double* __restrict__ vnp, int32_t* __restrict__ perm) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < ncol_pad; j += (int64_t)gridDim.x * blockDim.x) {
    const bool in = j < n_cols;
    const int32_t c = in ? sidx[j] : INT32_MAX;
    perm[j] = c;
    vnp[j] = in ? __longlong_as_double((long long)skey[j]) : 0.0;
    for (int k = 0; k < kpad; ++k) vtp[k * ncol_pad + j] = in ? vt[k * ncol_pad + c] : 0.0;
  }
}

}  // namespace

using namespace blp;

// The norm-ordered copy of the factors (first pruned top-k): a stable descending sort of
// ||v[c]||, so equal norms keep column order.
static int svd_prune_prepare(blp_svd* h) {
  if (h->d_vtp) return BLP_OK;
  const int64_t n = h->n_cols, np = h->ncol_pad;
  DevBuf key, idx, skey, sidx, temp;
  int rc;
  if ((rc = key.reserve(8 * n)) || (rc = idx.reserve(4 * n)) || (rc = skey.reserve(8 * n)) || (rc = sidx.reserve(4 * n)))
    return rc;
  auto done = [&](int r) {
    (void)hipStreamSynchronize(h->stream);
    for (DevBuf* b : {&key, &idx, &skey, &sidx, &temp}) b->release();
    return r;
  };
  hipLaunchKernelGGL(k_vnorm, dim3(1024), dim3(256), 0, h->stream, h->d_v, n, h->kpad, key.as<unsigned long long>(),
                     idx.as<int32_t>());
  size_t tb = 0;
  BLP_HIP_OR(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tb, key.as<unsigned long long>(),
                                                          skey.as<unsigned long long>(), idx.as<int32_t>(),
                                                          sidx.as<int32_t>(), (int)n, 0, 64, h->stream), done);
  if ((rc = temp.reserve(tb))) return done(rc);
  BLP_HIP_OR(hipcub::DeviceRadixSort::SortPairsDescending(temp.p, tb, key.as<unsigned long long>(),
                                                          skey.as<unsigned long long>(), idx.as<int32_t>(),
                                                          sidx.as<int32_t>(), (int)n, 0, 64, h->stream), done);
  BLP_HIP_OR(dev_malloc(&h->d_vtp, 8 * (size_t)h->kpad * np), done);
  BLP_HIP_OR(dev_malloc(&h->d_vnp, 8 * (size_t)np), done);
  BLP_HIP_OR(dev_malloc(&h->d_perm, 4 * (size_t)np), done);
  BLP_HIP_OR(dev_malloc(&h->d_tiles, 8), done);
  BLP_HIP_OR(hipMemsetAsync(h->d_tiles, 0, 8, h->stream), done);
  hipLaunchKernelGGL(k_vt_perm, dim3(1024), dim3(256), 0, h->stream, h->d_vt, np, n, h->kpad,
                     skey.as<unsigned long long>(), sidx.as<int32_t>(), h->d_vtp, h->d_vnp, h->d_perm);
  BLP_HIP_OR(hipGetLastError(), done);
  return done(BLP_OK);
}

// the two pruned passes: n1 first-pass chunks over the seed columns, n2 chunks over the rest
template <int KP>
static void svd_pr_launch(blp_svd* h, const TopkArgs& a, int64_t ublocks, int n1, int n2, int64_t seed_cols) {
  const dim3 block(TK_WAVES * 64);
  hipLaunchKernelGGL((k_svd_topk<KP, 1, TK_WAVES, 0, 1>), dim3((unsigned)ublocks, (unsigned)n1), block, 0, h->stream, a);
  if (!n2) return;
  TopkArgs b = a;
  b.n_cols = h->n_cols;
  b.col_base = seed_cols;
  b.chunk_base = n1;
  b.seeded = n1;
  hipLaunchKernelGGL((k_svd_topk<KP, 1, TK_WAVES, 0, 1>), dim3((unsigned)ublocks, (unsigned)n2), block, 0, h->stream, b);
}

extern "C" {

int blp_svd_create(const double* us, int64_t n_rows, const double* v, int64_t n_cols, int k, int device, blp_svd** out) {
  BLP_CHECK(out && us && v && n_rows > 0 && n_cols > 0 && k > 0 && k <= 256, BLP_E_ARG, "blp_svd_create: bad arguments");
  BLP_CHECK(n_rows < (int64_t(1) << 31) && n_cols < (int64_t(1) << 31), BLP_E_ARG, "blp_svd_create: too many rows");
  BLP_HIP(hipSetDevice(device));
  blp_svd* h = new blp_svd();
  h->device = device;
  h->n_rows = n_rows;
  h->n_cols = n_cols;
  h->k = k;
  h->kpad = (k + 15) / 16 * 16;
  h->ncol_pad = (n_cols + 15) / 16 * 16;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) h->n_cu = prop.multiProcessorCount;
  auto fail_hip = [&](hipError_t e, const char* what) {
    blp_svd_destroy(h);
    return hip_fail(e, what, __FILE__, __LINE__);
  };
  hipError_t e;
  if ((e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking)) != hipSuccess) return fail_hip(e, "stream");
  const int kp = h->kpad;
  std::vector<double> buf((size_t)std::max(n_rows, n_cols) * kp, 0.0);
  for (int64_t r = 0; r < n_rows; ++r) std::copy(us + r * k, us + r * k + k, buf.begin() + r * kp);
  if ((e = dev_malloc(&h->d_us, 8 * n_rows * kp)) != hipSuccess) return fail_hip(e, "hipMalloc");
  if ((e = hipMemcpy(h->d_us, buf.data(), 8 * n_rows * kp, hipMemcpyHostToDevice)) != hipSuccess) return fail_hip(e, "copy");
  std::fill(buf.begin(), buf.end(), 0.0);
  for (int64_t c = 0; c < n_cols; ++c) std::copy(v + c * k, v + c * k + k, buf.begin() + c * kp);
  if ((e = dev_malloc(&h->d_v, 8 * n_cols * kp)) != hipSuccess) return fail_hip(e, "hipMalloc");
  if ((e = hipMemcpy(h->d_v, buf.data(), 8 * n_cols * kp, hipMemcpyHostToDevice)) != hipSuccess) return fail_hip(e, "copy");
  std::vector<double> vt((size_t)kp * h->ncol_pad, 0.0);
  for (int64_t c = 0; c < n_cols; ++c)
    for (int j = 0; j < k; ++j) vt[(size_t)j * h->ncol_pad + c] = v[c * k + j];
  if ((e = dev_malloc(&h->d_vt, 8 * vt.size())) != hipSuccess) return fail_hip(e, "hipMalloc");
  if ((e = hipMemcpy(h->d_vt, vt.data(), 8 * vt.size(), hipMemcpyHostToDevice)) != hipSuccess) return fail_hip(e, "copy");
  *out = h;
  return BLP_OK;
}

int blp_svd_destroy(blp_svd* h) {
  if (!h) return BLP_OK;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  timer_release(h->t_pairs);
  timer_release(h->t_topk);
  if (h->join_ev) (void)hipEventDestroy(h->join_ev);
  for (void* p : {(void*)h->d_us, (void*)h->d_v, (void*)h->d_vt, (void*)h->d_ps, (void*)h->d_pc, (void*)h->d_vtp,
                  (void*)h->d_vnp, (void*)h->d_perm, (void*)h->d_tiles})
    if (p) (void)hipFree(p);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return BLP_OK;
}

// Device pairs (rows/cols/out are device pointers): enqueue on the handle's stream.
int blp_svd_score_pairs_device(blp_svd* h, const int32_t* d_rows, const int32_t* d_cols, int64_t n, double* d_out) {
  BLP_CHECK(h && n >= 0, BLP_E_ARG, "blp_svd_score_pairs_device: bad arguments");
  BLP_HIP(hipSetDevice(h->device));
  hipEvent_t t0;
  int rc = timer_begin(h->t_pairs, h->stream, &t0);
  if (rc) return rc;
  if (n) {
    const int64_t blocks = std::min<int64_t>((n * 8 + 255) / 256, (int64_t)h->n_cu * 32);
    hipLaunchKernelGGL(k_svd_pairs, dim3((unsigned)blocks), dim3(256), 0, h->stream, h->d_us, h->d_v, h->kpad, d_rows,
                       d_cols, n, d_out);
    BLP_HIP(hipGetLastError());
  }
  return timer_end(h->t_pairs, h->stream, t0);
}

int blp_svd_score_pairs(blp_svd* h, const int32_t* rows, const int32_t* cols, int64_t n, double* out) {
  BLP_CHECK(h && n >= 0 && (n == 0 || (rows && cols && out)), BLP_E_ARG, "blp_svd_score_pairs: bad arguments");
  for (int64_t i = 0; i < n; ++i)
    BLP_CHECK(rows[i] >= 0 && rows[i] < h->n_rows && cols[i] >= 0 && cols[i] < h->n_cols, BLP_E_ARG,
              "blp_svd_score_pairs: row/column out of range");
  if (!n) return BLP_OK;
  BLP_HIP(hipSetDevice(h->device));
  int32_t *dr = nullptr, *dc = nullptr;
  double* dout = nullptr;
  int rc = BLP_OK;
  if (dev_malloc(&dr, 4 * n) != hipSuccess || dev_malloc(&dc, 4 * n) != hipSuccess || dev_malloc(&dout, 8 * n) != hipSuccess) {
    rc = fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_svd_score_pairs: hipMalloc failed");
  } else if (hipMemcpy(dr, rows, 4 * n, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(dc, cols, 4 * n, hipMemcpyHostToDevice) != hipSuccess) {
    rc = fail(BLP_E_HIP_BASE, "blp_svd_score_pairs: upload failed");
  } else if (!(rc = blp_svd_score_pairs_device(h, dr, dc, n, dout))) {
    if (hipStreamSynchronize(h->stream) != hipSuccess || hipMemcpy(out, dout, 8 * n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(BLP_E_HIP_BASE, "blp_svd_score_pairs: download failed");
  }
  for (void* p : {(void*)dr, (void*)dc, (void*)dout})
    if (p) (void)hipFree(p);
  return rc;
}

static int part_reserve(blp_svd* h, int64_t np) {
  if (np <= h->part_cap) return BLP_OK;
  if (h->d_ps) (void)hipFree(h->d_ps);
  if (h->d_pc) (void)hipFree(h->d_pc);
  h->d_ps = nullptr;
  h->d_pc = nullptr;
  h->part_cap = 0;
  if (dev_malloc(&h->d_ps, 8 * np) != hipSuccess || dev_malloc(&h->d_pc, 4 * np) != hipSuccess)
    return fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_svd_topk: partial buffers");
  h->part_cap = np;
  return BLP_OK;
}

// The norm-pruned top-k: pass 1 scores the TK_SEED_COLS columns of largest ||v|| for every user
// (lists 0 .. n1-1, its tiles dealt round-robin over n1 chunks), pass 2 deals the remaining tiles
// round-robin over TK_PR_CHUNKS chunks (lists n1 ..), each starting from the best k-th entry of
// the first pass's lists and stopping at the norm bound; then the merge.
static int svd_topk_pruned(blp_svd* h, const int32_t* d_users, int64_t n_users, const int64_t* d_exo,
                           const int32_t* d_exc, int topk, int32_t* d_oc, double* d_os) {
  const int64_t ublocks = (n_users + 16 * TK_WAVES - 1) / (16 * TK_WAVES);
  const int64_t seed_cols = std::min<int64_t>(h->ncol_pad, TK_SEED_COLS);
  const int64_t rest_tiles = (h->ncol_pad - seed_cols) / 16;
  const int n2 = (int)std::min<int64_t>(TK_PR_CHUNKS, rest_tiles);
  const int n1 = (int)std::max<int64_t>(1, std::min<int64_t>(TK_SEED_CHUNKS, seed_cols / 16));
  const int n_chunks = n1 + n2;
  int rc = part_reserve(h, n_users * n_chunks * topk);
  if (rc) return rc;
  TopkArgs a{h->d_us, h->d_vtp, d_users, d_exo, d_exc, n_users, std::min<int64_t>(h->n_cols, seed_cols), h->ncol_pad,
             h->kpad, topk, 0, n_chunks, h->d_ps, h->d_pc, h->n_rows, h->d_perm, h->d_vnp, 0, 0, 0, h->d_tiles};
  hipEvent_t t0;
  if ((rc = timer_begin(h->t_topk, h->stream, &t0))) return rc;
  switch (h->kpad) {
    case 16: svd_pr_launch<16>(h, a, ublocks, n1, n2, seed_cols); break;
    case 32: svd_pr_launch<32>(h, a, ublocks, n1, n2, seed_cols); break;
    case 48: svd_pr_launch<48>(h, a, ublocks, n1, n2, seed_cols); break;
    case 64: svd_pr_launch<64>(h, a, ublocks, n1, n2, seed_cols); break;
    default: svd_pr_launch<128>(h, a, ublocks, n1, n2, seed_cols); break;
  }
  hipLaunchKernelGGL(k_svd_merge, dim3((unsigned)n_users), dim3(64), 0, h->stream, h->d_ps, h->d_pc, n_users,
                     n_chunks, topk, d_os, d_oc);
  if (hipGetLastError() != hipSuccess) return fail(BLP_E_HIP_BASE, "blp_svd_topk: launch failed");
  h->tiles_total += ((n_users + 15) / 16) * (h->ncol_pad / 16);
  return timer_end(h->t_topk, h->stream, t0);
}

// Enqueue the top-k of device-resident inputs on the handle's stream; the per-chunk partial
// lists live in handle-owned scratch (grown on demand, freed with the handle).
static int svd_topk_enqueue(blp_svd* h, const int32_t* d_users, int64_t n_users, const int64_t* d_exo,
                            const int32_t* d_exc, int topk, int32_t* d_oc, double* d_os) {
  BLP_HIP(hipSetDevice(h->device));
  // chunks: enough blocks to fill the chip, >= 16 tiles each
  // one 16-user tile per wave, 4 waves per block. Measured alternatives (config 4): two tiles
  // per wave (2 waves per block, same LDS: 1 wave per SIMD) 15.4 ms against 10.0 ms; two
  // accumulation chains per tile (halving the dependent MFMA chain) 10.2 ms
  const int waves = TK_WAVES;
  const int64_t upb = 16 * waves;  // users per block
  const int64_t ublocks = (n_users + upb - 1) / upb;
  // Column chunks: just enough (user block, chunk) blocks to occupy every block slot of the
  // chip ONCE. Each chunk restarts its users' top-k lists from an empty threshold, and the
  // insertions a list takes grow as C k (1 + ln(N / (C k))) over C chunks (config 4: 14
  // chunks 10.0 ms, 3 chunks 7.2 ms), so more chunks than slots only cost.
  const void* kfn = nullptr;
#define BLP_SVD_FN(KP) kfn = (const void*)&k_svd_topk<KP, 1, TK_WAVES>;
  switch (h->kpad) {
    case 16: BLP_SVD_FN(16); break;
    case 32: BLP_SVD_FN(32); break;
    case 48: BLP_SVD_FN(48); break;
    case 64: BLP_SVD_FN(64); break;
    default: BLP_SVD_FN(128); break;
  }
#undef BLP_SVD_FN
  if (h->prune) {
    int rc0 = svd_prune_prepare(h);
    if (rc0) return rc0;
    return svd_topk_pruned(h, d_users, n_users, d_exo, d_exc, topk, d_oc, d_os);
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, waves * 64, 0) != hipSuccess || per_cu < 1) per_cu = 1;
  // (capped so the merge ranks at most TK_MERGE_CAP partial entries per user in LDS: a 64-user
  // call would otherwise cut 200K columns into ~780 chunks and the merge rank 15.6K entries per
  // user in place, O(n^2): 100 ms for a 4 us top-k)
  int n_chunks = (int)std::max<int64_t>(
      1, std::min<int64_t>({(int64_t)h->n_cu * per_cu / ublocks, h->ncol_pad / 256, (int64_t)(TK_MERGE_CAP / topk)}));
  const int64_t chunk = ((h->n_cols + n_chunks - 1) / n_chunks + 15) / 16 * 16;
  n_chunks = (int)((h->n_cols + chunk - 1) / chunk);
  {
    int rc0 = part_reserve(h, n_users * n_chunks * topk);
    if (rc0) return rc0;
  }
  TopkArgs a{h->d_us, h->d_vt, d_users, d_exo, d_exc, n_users, h->n_cols, h->ncol_pad, h->kpad, topk, chunk, n_chunks,
             h->d_ps, h->d_pc, h->n_rows, nullptr, nullptr, 0, 0, 0, nullptr};
  h->tiles_total += ((n_users + 15) / 16) * (h->ncol_pad / 16);
  h->tiles_dense += ((n_users + 15) / 16) * (h->ncol_pad / 16);
  hipEvent_t t0;
  int rc = timer_begin(h->t_topk, h->stream, &t0);
  if (rc) return rc;
  const dim3 grid((unsigned)ublocks, (unsigned)n_chunks), block(waves * 64);
#define BLP_SVD_TOPK(KP) hipLaunchKernelGGL((k_svd_topk<KP, 1, TK_WAVES>), grid, block, 0, h->stream, a);
  switch (h->kpad) {
    case 16: BLP_SVD_TOPK(16); break;
    case 32: BLP_SVD_TOPK(32); break;
    case 48: BLP_SVD_TOPK(48); break;
    case 64: BLP_SVD_TOPK(64); break;
    default: BLP_SVD_TOPK(128); break;
  }
#undef BLP_SVD_TOPK
  hipLaunchKernelGGL(k_svd_merge, dim3((unsigned)n_users), dim3(64), 0, h->stream, h->d_ps, h->d_pc, n_users,
                     n_chunks, topk, d_os, d_oc);
  if (hipGetLastError() != hipSuccess) return fail(BLP_E_HIP_BASE, "blp_svd_topk: launch failed");
  return timer_end(h->t_topk, h->stream, t0);
}

int blp_svd_topk_device(blp_svd* h, const int32_t* d_users, int64_t n_users, const int64_t* d_ex_off,
                        const int32_t* d_ex_col, int topk, int32_t* d_out_cols, double* d_out_scores) {
  BLP_CHECK(h && d_users && n_users > 0 && topk > 0 && topk <= TK_MAX && d_out_cols && d_out_scores &&
                (!d_ex_off == !d_ex_col),
            BLP_E_ARG, "blp_svd_topk_device: bad arguments");
  BLP_CHECK(h->kpad == 16 || h->kpad == 32 || h->kpad == 48 || h->kpad == 64 || h->kpad == 128, BLP_E_UNSUP,
            "blp_svd_topk_device: k must pad to 16/32/48/64/128");
  return svd_topk_enqueue(h, d_users, n_users, d_ex_off, d_ex_col, topk, d_out_cols, d_out_scores);
}

int blp_svd_topk(blp_svd* h, const int32_t* users, int64_t n_users, const int64_t* ex_off, const int32_t* ex_col,
                 int topk, int32_t* out_cols, double* out_scores) {
  BLP_CHECK(h && users && n_users > 0 && topk > 0 && topk <= TK_MAX && out_cols && out_scores, BLP_E_ARG,
            "blp_svd_topk: bad arguments");
  BLP_CHECK(h->kpad == 16 || h->kpad == 32 || h->kpad == 48 || h->kpad == 64 || h->kpad == 128, BLP_E_UNSUP,
            "blp_svd_topk: k must pad to 16/32/48/64/128");
  for (int64_t i = 0; i < n_users; ++i)
    BLP_CHECK(users[i] >= 0 && users[i] < h->n_rows, BLP_E_ARG, "blp_svd_topk: user row out of range");
  BLP_HIP(hipSetDevice(h->device));
  const int64_t nex = ex_off ? ex_off[n_users] : 0;
  void *d_users = nullptr, *d_exo = nullptr, *d_exc = nullptr, *d_os = nullptr, *d_oc = nullptr;
  auto cleanup = [&]() {
    for (void* p : {d_users, d_exo, d_exc, d_os, d_oc})
      if (p) (void)hipFree(p);
  };
  if (dev_malloc(&d_users, 4 * n_users) != hipSuccess || dev_malloc(&d_os, 8 * n_users * topk) != hipSuccess ||
      dev_malloc(&d_oc, 4 * n_users * topk) != hipSuccess ||
      (ex_off && (dev_malloc(&d_exo, 8 * (n_users + 1)) != hipSuccess || dev_malloc(&d_exc, 4 * std::max<int64_t>(nex, 1)) != hipSuccess))) {
    cleanup();
    return fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_svd_topk: hipMalloc failed");
  }
  (void)hipMemcpy(d_users, users, 4 * n_users, hipMemcpyHostToDevice);
  if (ex_off) {
    (void)hipMemcpy(d_exo, ex_off, 8 * (n_users + 1), hipMemcpyHostToDevice);
    if (nex) (void)hipMemcpy(d_exc, ex_col, 4 * nex, hipMemcpyHostToDevice);
  }
  int rc = svd_topk_enqueue(h, (const int32_t*)d_users, n_users, (const int64_t*)d_exo, (const int32_t*)d_exc, topk,
                            (int32_t*)d_oc, (double*)d_os);
  if (rc) return cleanup(), rc;
  if (hipStreamSynchronize(h->stream) != hipSuccess ||
      hipMemcpy(out_scores, d_os, 8 * n_users * topk, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(out_cols, d_oc, 4 * n_users * topk, hipMemcpyDeviceToHost) != hipSuccess) {
    cleanup();
    return fail(BLP_E_HIP_BASE, "blp_svd_topk: execution failed");
  }
  cleanup();
  return BLP_OK;
}

int blp_svd_set_prune(blp_svd* h, int on) {
  BLP_CHECK(h, BLP_E_ARG, "blp_svd_set_prune: null handle");
  h->prune = on ? 1 : 0;
  return BLP_OK;
}

int blp_svd_tiles(blp_svd* h, int64_t* scored, int64_t* dense) {
  BLP_CHECK(h, BLP_E_ARG, "blp_svd_tiles: null handle");
  BLP_HIP(hipSetDevice(h->device));
  BLP_HIP(hipStreamSynchronize(h->stream));
  unsigned long long v = 0;
  if (h->d_tiles) {
    BLP_HIP(hipMemcpy(&v, h->d_tiles, 8, hipMemcpyDeviceToHost));
    BLP_HIP(hipMemset(h->d_tiles, 0, 8));
  }
  if (scored) *scored = (int64_t)v + h->tiles_dense;
  if (dense) *dense = h->tiles_total;
  h->tiles_total = 0;
  h->tiles_dense = 0;
  return BLP_OK;
}

int blp_svd_stats(blp_svd* h, int which, double* total_ms, int64_t* launches) {
  BLP_CHECK(h && (which == 0 || which == 1), BLP_E_ARG, "blp_svd_stats: bad arguments");
  KernelTimer& t = which == 0 ? h->t_pairs : h->t_topk;
  BLP_HIP(hipSetDevice(h->device));
  int rc = timer_collect(t);
  if (rc) return rc;
  if (total_ms) *total_ms = t.total_ms;
  if (launches) *launches = t.launches;
  return BLP_OK;
}

int blp_svd_stream_join(blp_svd* h, void* stream, int handle_waits) {
  BLP_CHECK(h, BLP_E_ARG, "blp_svd_stream_join: null handle");
  BLP_HIP(hipSetDevice(h->device));
  if (!h->join_ev) BLP_HIP(hipEventCreateWithFlags(&h->join_ev, hipEventDisableTiming));
  hipStream_t other = (hipStream_t)stream;
  if (handle_waits) {
    BLP_HIP(hipEventRecord(h->join_ev, other));
    BLP_HIP(hipStreamWaitEvent(h->stream, h->join_ev, 0));
  } else {
    BLP_HIP(hipEventRecord(h->join_ev, h->stream));
    BLP_HIP(hipStreamWaitEvent(other, h->join_ev, 0));
  }
  return BLP_OK;
}

int blp_svd_sync(blp_svd* h) {
  BLP_CHECK(h, BLP_E_ARG, "blp_svd_sync: null handle");
  BLP_HIP(hipSetDevice(h->device));
  BLP_HIP(hipStreamSynchronize(h->stream));
  return BLP_OK;
}

}  // extern "C"
