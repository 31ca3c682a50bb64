// Truncated SVD on the GPU: block subspace iteration with Rayleigh-Ritz,
// the device half of blp.factor.svds, which replaces scipy.sparse.linalg.svds (svd.py:24).
//
// The binary matrix M (n_rows x n_cols, CSR) and its transpose live in HBM. One iteration on a
// block Q (n_cols x P, fp64, orthonormal columns):
//     Z = M Q            k_spmm over M's rows      (each row: sum of its columns' Q rows)
//     W = M^T Z          k_spmm over M^T's rows
//     S = Q^T W          k_gram (fp64 MFMA) + k_gram_reduce  -> Ritz values on the host
//     Q = orth(W)        CholeskyQR2: k_gram of W, host Cholesky of the P x P Gram, k_apply
// and at the end us = Z V_k, v = Q V_k from the P x P eigenvectors V (blp.factor.svds).
// P = 128 (2x oversampling of k = 64): the top-64 subspace converges to machine precision in
// ~50 iterations on the review graphs (tests/test_gpu_factor.py checks it against ARPACK).
//
// Layouts: blocks are row-major [rows][P]. k_spmm: one wave per (row, <= SPMM_CH columns)
// item, lane l holds columns 2l, 2l+1 (16-byte loads: a Q row is one coalesced 1 KiB read);
// rows longer than SPMM_CH are split, their partials summed in a fixed order (deterministic).
#include <algorithm>
#include <vector>

#include "blp_internal.h"

namespace {

constexpr int P = 128;
constexpr int SPMM_CH = 2048;
typedef double double4_t __attribute__((ext_vector_type(4)));

struct SpItem {
  int32_t row;
  int32_t slot;  // -1: whole row, store directly; else partial slot
  int64_t kb, ke;
};

__global__ __launch_bounds__(256) void k_spmm(const int32_t* __restrict__ col, const SpItem* __restrict__ items,
                                             int64_t n_items, const double* __restrict__ X, double* __restrict__ Y,
                                             double* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t it = wave; it < n_items; it += nwaves) {
    const SpItem t = items[it];
    double2 acc = make_double2(0.0, 0.0);
    int64_t k = t.kb;
    for (; k + 4 <= t.ke; k += 4) {
      const int c0 = col[k], c1 = col[k + 1], c2 = col[k + 2], c3 = col[k + 3];
      const double2 v0 = reinterpret_cast<const double2*>(X + (int64_t)c0 * P)[lane];
      const double2 v1 = reinterpret_cast<const double2*>(X + (int64_t)c1 * P)[lane];
      const double2 v2 = reinterpret_cast<const double2*>(X + (int64_t)c2 * P)[lane];
      const double2 v3 = reinterpret_cast<const double2*>(X + (int64_t)c3 * P)[lane];
      acc.x += v0.x;
      acc.y += v0.y;
      acc.x += v1.x;
      acc.y += v1.y;
      acc.x += v2.x;
      acc.y += v2.y;
      acc.x += v3.x;
      acc.y += v3.y;
    }
    for (; k < t.ke; ++k) {
      const double2 v = reinterpret_cast<const double2*>(X + (int64_t)col[k] * P)[lane];
      acc.x += v.x;
      acc.y += v.y;
    }
    double2* dst = reinterpret_cast<double2*>(t.slot < 0 ? Y + (int64_t)t.row * P : part + (int64_t)t.slot * P);
    dst[lane] = acc;
  }
}

// split rows: Y[row] = sum of its partial slots, in slot order
__global__ void k_spmm_reduce(const int32_t* __restrict__ srow, const int32_t* __restrict__ soff, int n_split,
                              const double* __restrict__ part, double* __restrict__ Y) {
  for (int i = blockIdx.x; i < n_split; i += gridDim.x) {
    for (int c = threadIdx.x; c < P; c += blockDim.x) {
      double s = 0.0;
      for (int q = soff[i]; q < soff[i + 1]; ++q) s += part[(int64_t)q * P + c];
      Y[(int64_t)srow[i] * P + c] = s;
    }
  }
}

// Partial cross-Gram of a row range: G_b = X[r0:r1]^T Y[r0:r1] (P x P), fp64 MFMA 16x16x4.
// 4 waves per block, wave w owns the 4 x 4 output tiles of quadrant (w >> 1, w & 1).
// Fragments (v_mfma_f64_16x16x4f64): lane l gives A[i = l & 15][k = l >> 4] = X[r + (l >> 4)][16 ti + (l & 15)]
// and B[k = l >> 4][j = l & 15] = Y[r + (l >> 4)][16 tj + (l & 15)]; D[(l >> 4) + 4 q][l & 15].
__global__ __launch_bounds__(256) void k_gram(const double* __restrict__ X, const double* __restrict__ Y,
                                             int64_t n, int64_t rows_per_block, double* __restrict__ partial) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qi = w >> 1, qj = w & 1;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block, r1 = min(n, r0 + rows_per_block);
  double4_t acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = {0.0, 0.0, 0.0, 0.0};
  const int li = lane & 15, lk = lane >> 4;
  for (int64_t r = r0; r < r1; r += 4) {
    const int64_t rr = r + lk;
    const bool ok = rr < r1;
    double av[4], bv[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) av[a] = ok ? X[rr * P + (qi * 4 + a) * 16 + li] : 0.0;
#pragma unroll
    for (int b = 0; b < 4; ++b) bv[b] = ok ? Y[rr * P + (qj * 4 + b) * 16 + li] : 0.0;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
  }
  double* G = partial + (int64_t)blockIdx.x * P * P;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = (qi * 4 + a) * 16 + lk + 4 * q;
        const int j = (qj * 4 + b) * 16 + li;
        G[i * P + j] = acc[a][b][q];
      }
}

__global__ void k_gram_reduce(const double* __restrict__ partial, int nb, double* __restrict__ G) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P * P) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += partial[(int64_t)b * P * P + e];
  G[e] = s;
}

// Y = X R (n x P times P x P, row-major), R staged in LDS; each wave: 16 rows x P columns.
// A[i = l & 15][k = l >> 4] = X[row0 + i][4 s + k]; B[k = l >> 4][j = l & 15] = R[4 s + k][16 tj + j].
__global__ __launch_bounds__(256) void k_apply(const double* __restrict__ X, const double* __restrict__ R, int64_t n,
                                              double* __restrict__ Yout) {
  __shared__ double sR[P * P];
  for (int e = threadIdx.x; e < P * P; e += blockDim.x) sR[e] = R[e];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  for (int64_t row0 = ((int64_t)blockIdx.x * 4 + w) * 16; row0 < n; row0 += (int64_t)gridDim.x * 64) {
    double4_t acc[P / 16];
#pragma unroll
    for (int t = 0; t < P / 16; ++t) acc[t] = {0.0, 0.0, 0.0, 0.0};
    const int64_t xr = row0 + li;
#pragma unroll 2
    for (int s = 0; s < P / 4; ++s) {
      const double a = xr < n ? X[xr * P + 4 * s + lk] : 0.0;
#pragma unroll
      for (int t = 0; t < P / 16; ++t)
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, sR[(4 * s + lk) * P + 16 * t + li], acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < P / 16; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t r = row0 + lk + 4 * q;
        if (r < n) Yout[r * P + 16 * t + li] = acc[t][q];
      }
  }
}

}  // namespace

using namespace blp;

struct blp_fact {
  int device = 0;
  int n_cu = 256;
  hipStream_t stream = nullptr;
  int64_t n_rows = 0, n_cols = 0, nnz = 0;
  DevBuf rcol, ccol;              // column ids of M's rows / M^T's rows
  DevBuf ritems, citems;          // SpItem lists
  DevBuf rsrow, rsoff, csrow, csoff;
  int64_t n_ritems = 0, n_citems = 0;
  int n_rsplit = 0, n_csplit = 0, n_rslots = 0, n_cslots = 0;
  DevBuf Q, W, Z, part, gpart, G, R;
  int gram_blocks = 0;
  KernelTimer t_spmm, t_dense;
};

namespace {

int plan_items(const std::vector<int64_t>& rp, int64_t n, std::vector<SpItem>& items, std::vector<int32_t>& srow,
               std::vector<int32_t>& soff, int* n_slots) {
  items.clear();
  srow.clear();
  soff.assign(1, 0);
  int slots = 0;
  for (int64_t r = 0; r < n; ++r) {
    const int64_t b = rp[r], e = rp[r + 1];
    if (e - b <= SPMM_CH) {
      items.push_back(SpItem{(int32_t)r, -1, b, e});
      continue;
    }
    srow.push_back((int32_t)r);
    for (int64_t k = b; k < e; k += SPMM_CH) items.push_back(SpItem{(int32_t)r, slots++, k, std::min(e, k + SPMM_CH)});
    soff.push_back(slots);
  }
  *n_slots = slots;
  return BLP_OK;
}

int upload(DevBuf& b, const void* h, size_t bytes) {
  int rc = b.reserve(std::max<size_t>(bytes, 8));
  if (rc) return rc;
  if (bytes) BLP_HIP(hipMemcpy(b.p, h, bytes, hipMemcpyHostToDevice));
  return BLP_OK;
}

int spmm(blp_fact* f, bool transpose, const double* X, double* Y) {
  const SpItem* items = (transpose ? f->citems : f->ritems).as<SpItem>();
  const int64_t n_items = transpose ? f->n_citems : f->n_ritems;
  const int32_t* col = (transpose ? f->ccol : f->rcol).as<int32_t>();
  const int n_split = transpose ? f->n_csplit : f->n_rsplit;
  if (n_items) {
    const int64_t blocks = std::min<int64_t>((n_items + 3) / 4, (int64_t)f->n_cu * 32);
    hipLaunchKernelGGL(k_spmm, dim3((unsigned)blocks), dim3(256), 0, f->stream, col, items, n_items, X, Y,
                       f->part.as<double>());
    BLP_HIP(hipGetLastError());
  }
  if (n_split) {
    hipLaunchKernelGGL(k_spmm_reduce, dim3((unsigned)std::min(n_split, 4096)), dim3(P), 0, f->stream,
                       (transpose ? f->csrow : f->rsrow).as<int32_t>(), (transpose ? f->csoff : f->rsoff).as<int32_t>(),
                       n_split, f->part.as<double>(), Y);
    BLP_HIP(hipGetLastError());
  }
  return BLP_OK;
}

// host G = X^T Y over n rows
int gram(blp_fact* f, const double* X, const double* Y, int64_t n, double* Ghost) {
  const int nb = f->gram_blocks;
  const int64_t per = ((n + nb - 1) / nb + 3) / 4 * 4;
  hipLaunchKernelGGL(k_gram, dim3(nb), dim3(256), 0, f->stream, X, Y, n, std::max<int64_t>(per, 4),
                     f->gpart.as<double>());
  BLP_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_gram_reduce, dim3((P * P + 255) / 256), dim3(256), 0, f->stream, f->gpart.as<double>(), nb,
                     f->G.as<double>());
  BLP_HIP(hipGetLastError());
  BLP_HIP(hipMemcpyAsync(Ghost, f->G.p, 8 * P * P, hipMemcpyDeviceToHost, f->stream));
  BLP_HIP(hipStreamSynchronize(f->stream));
  return BLP_OK;
}

int apply(blp_fact* f, const double* X, int64_t n, const double* Rhost, double* Y) {
  BLP_HIP(hipMemcpyAsync(f->R.p, Rhost, 8 * P * P, hipMemcpyHostToDevice, f->stream));
  const int64_t blocks = std::min<int64_t>((n + 63) / 64, (int64_t)f->n_cu * 4);
  if (blocks > 0) {
    hipLaunchKernelGGL(k_apply, dim3((unsigned)blocks), dim3(256), 0, f->stream, X, f->R.as<double>(), n, Y);
    BLP_HIP(hipGetLastError());
  }
  return BLP_OK;
}

}  // namespace

extern "C" {

int blp_fact_create(const int64_t* row_ptr, const int32_t* col_idx, int64_t n_rows, int64_t n_cols, int device,
                    blp_fact** out) {
  BLP_CHECK(out && row_ptr && n_rows > 0 && n_cols > 0, BLP_E_ARG, "blp_fact_create: bad arguments");
  BLP_CHECK(n_rows < (int64_t(1) << 31) && n_cols < (int64_t(1) << 31), BLP_E_ARG, "blp_fact_create: too large");
  const int64_t nnz = row_ptr[n_rows];
  BLP_CHECK(nnz >= 0 && (nnz == 0 || col_idx), BLP_E_ARG, "blp_fact_create: bad CSR");
  for (int64_t r = 0; r < n_rows; ++r)
    BLP_CHECK(row_ptr[r] <= row_ptr[r + 1], BLP_E_ARG, "blp_fact_create: row_ptr not monotone");
  for (int64_t e = 0; e < nnz; ++e)
    BLP_CHECK(col_idx[e] >= 0 && col_idx[e] < n_cols, BLP_E_ARG, "blp_fact_create: column out of range");
  BLP_HIP(hipSetDevice(device));
  auto* f = new blp_fact();
  f->device = device;
  f->n_rows = n_rows;
  f->n_cols = n_cols;
  f->nnz = nnz;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) f->n_cu = prop.multiProcessorCount;
  auto bail = [&](int rc) {
    blp_fact_destroy(f);
    return rc;
  };
  BLP_HIP_OR(hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking), bail);
  // M^T by counting sort of the columns
  std::vector<int64_t> rp(row_ptr, row_ptr + n_rows + 1), cp(n_cols + 1, 0);
  for (int64_t e = 0; e < nnz; ++e) cp[col_idx[e] + 1]++;
  for (int64_t c = 0; c < n_cols; ++c) cp[c + 1] += cp[c];
  std::vector<int32_t> tcol(std::max<int64_t>(nnz, 1));
  {
    std::vector<int64_t> cur(cp.begin(), cp.end() - 1);
    for (int64_t r = 0; r < n_rows; ++r)
      for (int64_t e = rp[r]; e < rp[r + 1]; ++e) tcol[cur[col_idx[e]]++] = (int32_t)r;
  }
  std::vector<SpItem> ri, ci;
  std::vector<int32_t> rsr, rso, csr_, cso;
  plan_items(rp, n_rows, ri, rsr, rso, &f->n_rslots);
  plan_items(cp, n_cols, ci, csr_, cso, &f->n_cslots);
  f->n_ritems = (int64_t)ri.size();
  f->n_citems = (int64_t)ci.size();
  f->n_rsplit = (int)rsr.size();
  f->n_csplit = (int)csr_.size();
  f->gram_blocks = f->n_cu * 2;
  int rc;
  if ((rc = upload(f->rcol, col_idx, 4 * nnz)) || (rc = upload(f->ccol, tcol.data(), 4 * nnz)) ||
      (rc = upload(f->ritems, ri.data(), sizeof(SpItem) * ri.size())) ||
      (rc = upload(f->citems, ci.data(), sizeof(SpItem) * ci.size())) ||
      (rc = upload(f->rsrow, rsr.data(), 4 * rsr.size())) || (rc = upload(f->rsoff, rso.data(), 4 * rso.size())) ||
      (rc = upload(f->csrow, csr_.data(), 4 * csr_.size())) || (rc = upload(f->csoff, cso.data(), 4 * cso.size())) ||
      (rc = f->Q.reserve(8 * n_cols * P)) || (rc = f->W.reserve(8 * n_cols * P)) ||
      (rc = f->Z.reserve(8 * n_rows * P)) ||
      (rc = f->part.reserve(8 * (size_t)std::max(std::max(f->n_rslots, f->n_cslots), 1) * P)) ||
      (rc = f->gpart.reserve(8 * (size_t)f->gram_blocks * P * P)) || (rc = f->G.reserve(8 * P * P)) ||
      (rc = f->R.reserve(8 * P * P)))
    return bail(rc);
  *out = f;
  return BLP_OK;
}

int blp_fact_destroy(blp_fact* f) {
  if (!f) return BLP_OK;
  (void)hipSetDevice(f->device);
  if (f->stream) (void)hipStreamSynchronize(f->stream);
  for (DevBuf* b : {&f->rcol, &f->ccol, &f->ritems, &f->citems, &f->rsrow, &f->rsoff, &f->csrow, &f->csoff, &f->Q,
                    &f->W, &f->Z, &f->part, &f->gpart, &f->G, &f->R})
    b->release();
  timer_release(f->t_spmm);
  timer_release(f->t_dense);
  if (f->stream) (void)hipStreamDestroy(f->stream);
  delete f;
  return BLP_OK;
}

int blp_fact_block_width(void) { return P; }

int blp_fact_set_q(blp_fact* f, const double* q) {
  BLP_CHECK(f && q, BLP_E_ARG, "blp_fact_set_q: bad arguments");
  BLP_HIP(hipSetDevice(f->device));
  BLP_HIP(hipMemcpy(f->Q.p, q, 8 * f->n_cols * P, hipMemcpyHostToDevice));
  return BLP_OK;
}

// Z = M Q; W = M^T Z; S = Q^T W (host, P x P row-major)
int blp_fact_step(blp_fact* f, double* S) {
  BLP_CHECK(f && S, BLP_E_ARG, "blp_fact_step: bad arguments");
  BLP_HIP(hipSetDevice(f->device));
  int rc;
  hipEvent_t t0;
  if ((rc = timer_begin(f->t_spmm, f->stream, &t0))) return rc;
  if ((rc = spmm(f, false, f->Q.as<double>(), f->Z.as<double>()))) return rc;
  if ((rc = spmm(f, true, f->Z.as<double>(), f->W.as<double>()))) return rc;
  if ((rc = timer_end(f->t_spmm, f->stream, t0))) return rc;
  if ((rc = timer_begin(f->t_dense, f->stream, &t0))) return rc;
  if ((rc = gram(f, f->Q.as<double>(), f->W.as<double>(), f->n_cols, S))) return rc;
  return timer_end(f->t_dense, f->stream, t0);
}

// G = W^T W (host)
int blp_fact_gram_w(blp_fact* f, double* G) {
  BLP_CHECK(f && G, BLP_E_ARG, "blp_fact_gram_w: bad arguments");
  BLP_HIP(hipSetDevice(f->device));
  return gram(f, f->W.as<double>(), f->W.as<double>(), f->n_cols, G);
}

// W <- W R (R host, P x P row-major); the result lands in Q (the next iterate) when to_q
int blp_fact_apply_w(blp_fact* f, const double* R, int to_q) {
  BLP_CHECK(f && R, BLP_E_ARG, "blp_fact_apply_w: bad arguments");
  BLP_HIP(hipSetDevice(f->device));
  int rc;
  hipEvent_t t0;
  if ((rc = timer_begin(f->t_dense, f->stream, &t0))) return rc;
  // out-of-place: W R -> Q, then (when !to_q) Q -> W
  if ((rc = apply(f, f->W.as<double>(), f->n_cols, R, f->Q.as<double>()))) return rc;
  if (!to_q) BLP_HIP(hipMemcpyAsync(f->W.p, f->Q.p, 8 * f->n_cols * P, hipMemcpyDeviceToDevice, f->stream));
  return timer_end(f->t_dense, f->stream, t0);
}

// us = Z V[:, :k], v = Q V[:, :k] (V host P x P row-major; outputs host [n][k] row-major)
int blp_fact_extract(blp_fact* f, const double* V, int k, double* us, double* v) {
  BLP_CHECK(f && V && k >= 1 && k <= P && us && v, BLP_E_ARG, "blp_fact_extract: bad arguments");
  BLP_HIP(hipSetDevice(f->device));
  int rc;
  // reuse W as the output buffer of Q V, part of Z's buffer trick: compute Z V into a fresh buffer
  DevBuf zv;
  if ((rc = zv.reserve(8 * f->n_rows * P))) return rc;
  if ((rc = apply(f, f->Z.as<double>(), f->n_rows, V, zv.as<double>()))) return zv.release(), rc;
  if ((rc = apply(f, f->Q.as<double>(), f->n_cols, V, f->W.as<double>()))) return zv.release(), rc;
  BLP_HIP_OR(hipStreamSynchronize(f->stream), [&](int r) { zv.release(); return r; });
  BLP_HIP_OR(hipMemcpy2D(us, 8 * k, zv.p, 8 * P, 8 * k, f->n_rows, hipMemcpyDeviceToHost),
             [&](int r) { zv.release(); return r; });
  BLP_HIP_OR(hipMemcpy2D(v, 8 * k, f->W.p, 8 * P, 8 * k, f->n_cols, hipMemcpyDeviceToHost),
             [&](int r) { zv.release(); return r; });
  zv.release();
  return BLP_OK;
}

// which 0: SpMM pair (Z = M Q, W = M^T Z) ms/launches; 1: dense (Gram / apply)
int blp_fact_stats(blp_fact* f, int which, double* total_ms, int64_t* launches) {
  BLP_CHECK(f && (which == 0 || which == 1), BLP_E_ARG, "blp_fact_stats: bad arguments");
  BLP_HIP(hipSetDevice(f->device));
  KernelTimer& t = which == 0 ? f->t_spmm : f->t_dense;
  int rc = timer_collect(t);
  if (rc) return rc;
  if (total_ms) *total_ms = t.total_ms;
  if (launches) *launches = t.launches;
  return BLP_OK;
}

}  // extern "C"
