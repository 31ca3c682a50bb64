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
// Factor layout: US [n_rows][kpad] and V [n_cols][kpad] row-major, Vt [kpad][ncol_pad];
// kpad = k rounded up to 16 (zero padding adds exact zeros to every dot product).
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
constexpr int TK_BUF = 48;         // candidate buffer per user (+16 per tile at most)

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
};

// better = higher score, then lower column
__device__ inline bool better(double s, int c, double t, int tc) { return s > t || (s == t && c < tc); }

// Keep the best `topk` of top[0..topk) + buf[0..nb) in top (wave-cooperative rank select).
__device__ inline void tk_compact(double* top_s, int* top_c, double* buf_s, int* buf_c, int nb, int topk, int lane,
                                  double* th_s, int* th_c) {
  const int n = topk + nb;
  double vs[2];
  int vc[2], rk[2];
  for (int q = 0; q < 2; ++q) {
    const int i = lane + 64 * q;
    vs[q] = -DBL_MAX;
    vc[q] = INT32_MAX;
    rk[q] = INT32_MAX;
    if (i < n) {
      vs[q] = i < topk ? top_s[i] : buf_s[i - topk];
      vc[q] = i < topk ? top_c[i] : buf_c[i - topk];
      int r = 0;
      for (int j = 0; j < n; ++j) {
        const double s = j < topk ? top_s[j] : buf_s[j - topk];
        const int c = j < topk ? top_c[j] : buf_c[j - topk];
        r += better(s, c, vs[q], vc[q]) || (s == vs[q] && c == vc[q] && j < i);
      }
      rk[q] = r;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  for (int q = 0; q < 2; ++q)
    if (rk[q] < topk) {
      top_s[rk[q]] = vs[q];
      top_c[rk[q]] = vc[q];
    }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    *th_s = top_s[topk - 1];
    *th_c = top_c[topk - 1];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <int KPAD>
__global__ __launch_bounds__(TK_WAVES * 64) void k_svd_topk(TopkArgs a) {
  __shared__ double s_top[TK_WAVES][16][TK_MAX];
  __shared__ int s_topc[TK_WAVES][16][TK_MAX];
  __shared__ double s_buf[TK_WAVES][16][TK_BUF + 16];
  __shared__ int s_bufc[TK_WAVES][16][TK_BUF + 16];
  __shared__ int s_nb[TK_WAVES][16];
  __shared__ double s_th[TK_WAVES][16];
  __shared__ int s_thc[TK_WAVES][16];
  constexpr int KS = KPAD / 4;  // MFMA k-steps
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t u0 = ((int64_t)blockIdx.x * TK_WAVES + w) * 16;
  if (u0 >= a.n_users) return;  // whole wave idle (no block barriers below)
  const int chunk = blockIdx.y;
  const int64_t cb = (int64_t)chunk * a.chunk, ce = min(a.n_cols, cb + a.chunk);
  const int topk = a.topk;
  for (int i = lane; i < 16 * TK_MAX; i += 64) {
    s_top[w][i / TK_MAX][i % TK_MAX] = -DBL_MAX;
    s_topc[w][i / TK_MAX][i % TK_MAX] = INT32_MAX;
  }
  if (lane < 16) {
    s_nb[w][lane] = 0;
    s_th[w][lane] = -DBL_MAX;
    s_thc[w][lane] = INT32_MAX;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // A fragments: A[i = lane & 15][k = 4 s + (lane >> 4)] = US[users[u0 + i]][k]
  double af[KS];
  {
    const int64_t ui = u0 + (lane & 15);
    const int64_t row = ui < a.n_users ? a.users[ui] : -1;
#pragma unroll
    for (int s = 0; s < KS; ++s) af[s] = row >= 0 ? a.us[row * KPAD + 4 * s + (lane >> 4)] : 0.0;
  }
  const int my_row = lane >> 4;  // the C/D rows of this lane are my_row + 4 r
  // Exclusions (the user's own reviews, sorted): lane r < 16 walks row r's list alongside the
  // tiles (ex_p = position, ex_n = next excluded column) and publishes a 16-bit mask of the
  // tile's excluded columns; a global load happens only when a tile holds one (~deg times per
  // row), instead of a binary search per threshold-passing score.
  int64_t ex_p = 0, ex_e = 0;
  int ex_n = INT32_MAX;
  if (a.ex_off && lane < 16 && u0 + lane < a.n_users) {
    ex_p = a.ex_off[u0 + lane];
    ex_e = a.ex_off[u0 + lane + 1];
    while (ex_p < ex_e && a.ex_col[ex_p] < cb) ++ex_p;
    ex_n = ex_p < ex_e ? a.ex_col[ex_p] : INT32_MAX;
  }
  // B[k = 4 s + (lane >> 4)][j = lane & 15] = Vt[k][c0 + j]  (padded columns are zero);
  // the next tile's fragments are in flight while this tile's MFMA chain runs
  const double* vt_lane = a.vt + (int64_t)(lane >> 4) * a.ncol_pad + (lane & 15);
  double bf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) bf[s] = vt_lane[(int64_t)(4 * s) * a.ncol_pad + cb];
  for (int64_t c0 = cb; c0 < ce; c0 += 16) {
    double4_t d = {0.0, 0.0, 0.0, 0.0};
    const int col = (int)(c0 + (lane & 15));
    const int64_t cn = c0 + 16 < ce ? c0 + 16 : c0;
    double nb[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) nb[s] = vt_lane[(int64_t)(4 * s) * a.ncol_pad + cn];
#pragma unroll
    for (int s = 0; s < KS; ++s) d = __builtin_amdgcn_mfma_f64_16x16x4f64(af[s], bf[s], d, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s) bf[s] = nb[s];
    unsigned exm = 0;  // lane r < 16: excluded columns of row r in this tile
    while (ex_n < c0 + 16) {
      if (ex_n >= c0) exm |= 1u << (ex_n - c0);  // (a duplicate or out-of-order id is skipped)
      ex_n = ++ex_p < ex_e ? a.ex_col[ex_p] : INT32_MAX;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = my_row + 4 * r;
      const double sc = d[r];
      const unsigned rm = (unsigned)__shfl((int)exm, row, 64);
      if (col < ce && u0 + row < a.n_users && !((rm >> (lane & 15)) & 1u) &&
          better(sc, col, s_th[w][row], s_thc[w][row])) {
        const int slot = atomicAdd(&s_nb[w][row], 1);
        s_buf[w][row][slot] = sc;
        s_bufc[w][row][slot] = col;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // compact rows whose buffer could overflow on the next tile (one LDS read and a ballot
    // find them; the loop visits only those rows)
    const int my_nb = lane < 16 ? s_nb[w][lane] : 0;
    unsigned long long due = __ballot(lane < 16 && (my_nb > TK_BUF - 16 || (c0 + 16 >= ce && my_nb > 0)));
    while (due) {
      const int row = __builtin_ctzll(due);
      due &= due - 1;
      const int nb = s_nb[w][row];
      {
        tk_compact(s_top[w][row], s_topc[w][row], s_buf[w][row], s_bufc[w][row], nb, topk, lane, &s_th[w][row],
                   &s_thc[w][row]);
        if (lane == 0) s_nb[w][row] = 0;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
  for (int i = lane; i < 16 * topk; i += 64) {
    const int row = i / topk, q = i % topk;
    const int64_t u = u0 + row;
    if (u < a.n_users) {
      const int64_t o = (u * a.n_chunks + chunk) * topk + q;
      a.part_score[o] = s_top[w][row][q];
      a.part_col[o] = s_topc[w][row][q];
    }
  }
}

// One wave per user: best topk of n_chunks * topk partial entries.
__global__ __launch_bounds__(64) void k_svd_merge(const double* __restrict__ ps, const int32_t* __restrict__ pc,
                                                  int64_t n_users, int n_chunks, int topk, double* __restrict__ out_s,
                                                  int32_t* __restrict__ out_c) {
  const int64_t u = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = n_chunks * topk;
  const double* s = ps + u * n;
  const int32_t* c = pc + u * n;
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

}  // namespace

using namespace blp;

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
  if ((e = hipMalloc(&h->d_us, 8 * n_rows * kp)) != hipSuccess) return fail_hip(e, "hipMalloc");
  if ((e = hipMemcpy(h->d_us, buf.data(), 8 * n_rows * kp, hipMemcpyHostToDevice)) != hipSuccess) return fail_hip(e, "copy");
  std::fill(buf.begin(), buf.end(), 0.0);
  for (int64_t c = 0; c < n_cols; ++c) std::copy(v + c * k, v + c * k + k, buf.begin() + c * kp);
  if ((e = hipMalloc(&h->d_v, 8 * n_cols * kp)) != hipSuccess) return fail_hip(e, "hipMalloc");
  if ((e = hipMemcpy(h->d_v, buf.data(), 8 * n_cols * kp, hipMemcpyHostToDevice)) != hipSuccess) return fail_hip(e, "copy");
  std::vector<double> vt((size_t)kp * h->ncol_pad, 0.0);
  for (int64_t c = 0; c < n_cols; ++c)
    for (int j = 0; j < k; ++j) vt[(size_t)j * h->ncol_pad + c] = v[c * k + j];
  if ((e = hipMalloc(&h->d_vt, 8 * vt.size())) != hipSuccess) return fail_hip(e, "hipMalloc");
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
  for (void* p : {(void*)h->d_us, (void*)h->d_v, (void*)h->d_vt})
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
  if (hipMalloc(&dr, 4 * n) != hipSuccess || hipMalloc(&dc, 4 * n) != hipSuccess || hipMalloc(&dout, 8 * n) != hipSuccess) {
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

int blp_svd_topk(blp_svd* h, const int32_t* users, int64_t n_users, const int64_t* ex_off, const int32_t* ex_col,
                 int topk, int32_t* out_cols, double* out_scores) {
  BLP_CHECK(h && users && n_users > 0 && topk > 0 && topk <= TK_MAX && out_cols && out_scores, BLP_E_ARG,
            "blp_svd_topk: bad arguments");
  BLP_CHECK(h->kpad == 16 || h->kpad == 32 || h->kpad == 48 || h->kpad == 64 || h->kpad == 128, BLP_E_UNSUP,
            "blp_svd_topk: k must pad to 16/32/48/64/128");
  for (int64_t i = 0; i < n_users; ++i)
    BLP_CHECK(users[i] >= 0 && users[i] < h->n_rows, BLP_E_ARG, "blp_svd_topk: user row out of range");
  BLP_HIP(hipSetDevice(h->device));
  // chunks: enough blocks to fill the chip, >= 16 tiles each
  const int64_t ublocks = (n_users + 16 * TK_WAVES - 1) / (16 * TK_WAVES);
  int n_chunks = (int)std::max<int64_t>(1, std::min<int64_t>((h->n_cu * 8 + ublocks - 1) / ublocks, h->ncol_pad / 256));
  const int64_t chunk = ((h->n_cols + n_chunks - 1) / n_chunks + 15) / 16 * 16;
  n_chunks = (int)((h->n_cols + chunk - 1) / chunk);
  const int64_t nex = ex_off ? ex_off[n_users] : 0;
  void *d_users = nullptr, *d_exo = nullptr, *d_exc = nullptr, *d_ps = nullptr, *d_pc = nullptr, *d_os = nullptr,
       *d_oc = nullptr;
  auto cleanup = [&]() {
    for (void* p : {d_users, d_exo, d_exc, d_ps, d_pc, d_os, d_oc})
      if (p) (void)hipFree(p);
  };
  const int64_t np = n_users * n_chunks * topk;
  if (hipMalloc(&d_users, 4 * n_users) != hipSuccess || hipMalloc(&d_ps, 8 * np) != hipSuccess ||
      hipMalloc(&d_pc, 4 * np) != hipSuccess || hipMalloc(&d_os, 8 * n_users * topk) != hipSuccess ||
      hipMalloc(&d_oc, 4 * n_users * topk) != hipSuccess ||
      (ex_off && (hipMalloc(&d_exo, 8 * (n_users + 1)) != hipSuccess || hipMalloc(&d_exc, 4 * std::max<int64_t>(nex, 1)) != hipSuccess))) {
    cleanup();
    return fail(BLP_E_HIP_BASE - (int)hipErrorOutOfMemory, "blp_svd_topk: hipMalloc failed");
  }
  (void)hipMemcpy(d_users, users, 4 * n_users, hipMemcpyHostToDevice);
  if (ex_off) {
    (void)hipMemcpy(d_exo, ex_off, 8 * (n_users + 1), hipMemcpyHostToDevice);
    if (nex) (void)hipMemcpy(d_exc, ex_col, 4 * nex, hipMemcpyHostToDevice);
  }
  TopkArgs a{h->d_us, h->d_vt, (const int32_t*)d_users, (const int64_t*)d_exo, (const int32_t*)d_exc, n_users,
             h->n_cols, h->ncol_pad, h->kpad, topk, chunk, n_chunks, (double*)d_ps, (int32_t*)d_pc};
  hipEvent_t t0;
  int rc = timer_begin(h->t_topk, h->stream, &t0);
  if (rc) return cleanup(), rc;
  const dim3 grid((unsigned)ublocks, (unsigned)n_chunks), block(TK_WAVES * 64);
  switch (h->kpad) {
    case 16: hipLaunchKernelGGL(k_svd_topk<16>, grid, block, 0, h->stream, a); break;
    case 32: hipLaunchKernelGGL(k_svd_topk<32>, grid, block, 0, h->stream, a); break;
    case 48: hipLaunchKernelGGL(k_svd_topk<48>, grid, block, 0, h->stream, a); break;
    case 64: hipLaunchKernelGGL(k_svd_topk<64>, grid, block, 0, h->stream, a); break;
    default: hipLaunchKernelGGL(k_svd_topk<128>, grid, block, 0, h->stream, a); break;
  }
  hipLaunchKernelGGL(k_svd_merge, dim3((unsigned)n_users), dim3(64), 0, h->stream, (const double*)d_ps,
                     (const int32_t*)d_pc, n_users, n_chunks, topk, (double*)d_os, (int32_t*)d_oc);
  if (hipGetLastError() != hipSuccess) {
    cleanup();
    return fail(BLP_E_HIP_BASE, "blp_svd_topk: launch failed");
  }
  if ((rc = timer_end(h->t_topk, h->stream, t0))) return cleanup(), rc;
  if (hipStreamSynchronize(h->stream) != hipSuccess ||
      hipMemcpy(out_scores, d_os, 8 * n_users * topk, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(out_cols, d_oc, 4 * n_users * topk, hipMemcpyDeviceToHost) != hipSuccess) {
    cleanup();
    return fail(BLP_E_HIP_BASE, "blp_svd_topk: execution failed");
  }
  cleanup();
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

int blp_svd_sync(blp_svd* h) {
  BLP_CHECK(h, BLP_E_ARG, "blp_svd_sync: null handle");
  BLP_HIP(hipSetDevice(h->device));
  BLP_HIP(hipStreamSynchronize(h->stream));
  return BLP_OK;
}

}  // extern "C"
