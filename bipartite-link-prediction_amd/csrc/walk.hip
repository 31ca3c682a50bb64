// Damped random walks (random_walks.py:9-53) on MI355X.
//
// The reference walks p <- (1 - jump_p) * (p . T) for `iterations` steps from e_u, with
// T = D^-1 A (random_walks.py:26-29,43-53), one scipy sparse row-vector product per step
// and per example user. Here a batch of WB start nodes walks together as a dense fp64 block
// P[n][WB] (node-major: the WB values of one node are one 256-byte row), and each step is a
// pull SpMM over W = T^T in CSR:  P'[j][:] = scale * sum_e W[j, e] * P[col e][:].
// Rows are cut into work items of at most WALK_CH stored entries so that a node with 2e5
// neighbours does not serialise a step; a row cut into several items is accumulated with
// fp64 atomics (only those rows; everything else is a plain store).
#include <algorithm>
#include <vector>

#include "blp_internal.h"

namespace {

constexpr int WB = 32;        // starts per batch (P row = 256 B)
constexpr int WALK_CH = 256;  // stored entries per work item

struct WalkItem {
  int32_t row;
  int32_t split;  // 1: row is shared by several items (atomic accumulate)
  int64_t eb, ee;
};

__global__ __launch_bounds__(256) void k_walk_zero_split(const int32_t* __restrict__ rows, int64_t n_rows,
                                                         double* __restrict__ pn) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_rows * WB; i += (int64_t)gridDim.x * blockDim.x)
    pn[(int64_t)rows[i / WB] * WB + (i % WB)] = 0.0;
}

// One 32-lane group per work item (two items per wave).
__global__ __launch_bounds__(256) void k_walk_step(const WalkItem* __restrict__ items, int64_t n_items,
                                                   const int32_t* __restrict__ col, const double* __restrict__ val,
                                                   const double* __restrict__ p, double* __restrict__ pn, double scale) {
  const int b = threadIdx.x & (WB - 1);
  const int64_t groups = (int64_t)gridDim.x * (blockDim.x / WB);
  for (int64_t it = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / WB; it < n_items; it += groups) {
    const WalkItem w = items[it];
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
    int64_t e = w.eb;
    for (; e + 4 <= w.ee; e += 4) {
      const int c0 = col[e], c1 = col[e + 1], c2 = col[e + 2], c3 = col[e + 3];
      acc0 = fma(val[e], p[(int64_t)c0 * WB + b], acc0);
      acc1 = fma(val[e + 1], p[(int64_t)c1 * WB + b], acc1);
      acc2 = fma(val[e + 2], p[(int64_t)c2 * WB + b], acc2);
      acc3 = fma(val[e + 3], p[(int64_t)c3 * WB + b], acc3);
    }
    for (; e < w.ee; ++e) acc0 = fma(val[e], p[(int64_t)col[e] * WB + b], acc0);
    const double v = scale * ((acc0 + acc1) + (acc2 + acc3));
    double* dst = pn + (int64_t)w.row * WB + b;
    if (w.split)
      atomicAdd(dst, v);
    else
      *dst = v;
  }
}

__global__ void k_walk_init(const int32_t* __restrict__ starts, int nb, double* __restrict__ p) {
  const int b = threadIdx.x;
  if (b < nb) p[(int64_t)starts[b] * WB + b] = 1.0;
}

__global__ void k_walk_gather(const double* __restrict__ p, const int32_t* __restrict__ qb,
                              const int32_t* __restrict__ qn, int64_t nq, double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nq; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = p[(int64_t)qn[i] * WB + qb[i]];
}

}  // namespace

struct blp_walk {
  int device = 0;
  int n_cu = 256;
  hipStream_t stream = nullptr;
  int64_t n = 0, nnz = 0, n_items = 0, n_split_rows = 0;
  int32_t* d_col = nullptr;
  double* d_val = nullptr;
  WalkItem* d_items = nullptr;
  int32_t* d_split_rows = nullptr;
  double *d_p = nullptr, *d_pn = nullptr;
  blp::KernelTimer timer;
};

using namespace blp;

extern "C" {

int blp_walk_create(const int64_t* row_ptr, const int32_t* col, const double* val, int64_t n, int device,
                    blp_walk** out) {
  BLP_CHECK(out && row_ptr && n > 0 && n < (int64_t(1) << 31), BLP_E_ARG, "blp_walk_create: bad arguments");
  const int64_t nnz = row_ptr[n];
  BLP_CHECK(nnz >= 0 && (nnz == 0 || (col && val)), BLP_E_ARG, "blp_walk_create: bad matrix");
  for (int64_t i = 0; i < nnz; ++i) BLP_CHECK(col[i] >= 0 && col[i] < n, BLP_E_ARG, "blp_walk_create: column out of range");
  BLP_HIP(hipSetDevice(device));
  std::vector<WalkItem> items;
  std::vector<int32_t> split_rows;
  for (int64_t r = 0; r < n; ++r) {
    const int64_t b = row_ptr[r], e = row_ptr[r + 1];
    if (e - b <= WALK_CH) {
      items.push_back(WalkItem{(int32_t)r, 0, b, e});
    } else {
      split_rows.push_back((int32_t)r);
      for (int64_t s = b; s < e; s += WALK_CH) items.push_back(WalkItem{(int32_t)r, 1, s, std::min(e, s + WALK_CH)});
    }
  }
  blp_walk* w = new blp_walk();
  w->device = device;
  w->n = n;
  w->nnz = nnz;
  w->n_items = (int64_t)items.size();
  w->n_split_rows = (int64_t)split_rows.size();
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) w->n_cu = prop.multiProcessorCount;
  auto bad = [&](hipError_t e) {
    blp_walk_destroy(w);
    return hip_fail(e, "blp_walk_create", __FILE__, __LINE__);
  };
  hipError_t e;
  if ((e = hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking)) != hipSuccess) return bad(e);
  if ((e = dev_malloc(&w->d_col, 4 * std::max<int64_t>(nnz, 1))) != hipSuccess) return bad(e);
  if ((e = dev_malloc(&w->d_val, 8 * std::max<int64_t>(nnz, 1))) != hipSuccess) return bad(e);
  if ((e = dev_malloc(&w->d_items, sizeof(WalkItem) * std::max<size_t>(items.size(), 1))) != hipSuccess) return bad(e);
  if ((e = dev_malloc(&w->d_split_rows, 4 * std::max<size_t>(split_rows.size(), 1))) != hipSuccess) return bad(e);
  if ((e = dev_malloc(&w->d_p, 8 * n * WB)) != hipSuccess) return bad(e);
  if ((e = dev_malloc(&w->d_pn, 8 * n * WB)) != hipSuccess) return bad(e);
  if (nnz && ((e = hipMemcpy(w->d_col, col, 4 * nnz, hipMemcpyHostToDevice)) != hipSuccess ||
              (e = hipMemcpy(w->d_val, val, 8 * nnz, hipMemcpyHostToDevice)) != hipSuccess))
    return bad(e);
  if (!items.empty() &&
      (e = hipMemcpy(w->d_items, items.data(), sizeof(WalkItem) * items.size(), hipMemcpyHostToDevice)) != hipSuccess)
    return bad(e);
  if (!split_rows.empty() &&
      (e = hipMemcpy(w->d_split_rows, split_rows.data(), 4 * split_rows.size(), hipMemcpyHostToDevice)) != hipSuccess)
    return bad(e);
  *out = w;
  return BLP_OK;
}

int blp_walk_destroy(blp_walk* w) {
  if (!w) return BLP_OK;
  (void)hipSetDevice(w->device);
  if (w->stream) (void)hipStreamSynchronize(w->stream);
  timer_release(w->timer);
  for (void* p : {(void*)w->d_col, (void*)w->d_val, (void*)w->d_items, (void*)w->d_split_rows, (void*)w->d_p,
                  (void*)w->d_pn})
    if (p) (void)hipFree(p);
  if (w->stream) (void)hipStreamDestroy(w->stream);
  delete w;
  return BLP_OK;
}

// Walk from every start (WB at a time) and read q_out[k] = p_{q_start[k]}[q_node[k]]
// after `iterations` steps; queries must be grouped by start (q_start ascending).
int blp_walk_run(blp_walk* w, const int32_t* starts, int64_t n_starts, int iterations, double scale,
                 const int32_t* q_start, const int32_t* q_node, int64_t n_q, double* q_out) {
  BLP_CHECK(w && n_starts >= 0 && iterations >= 0 && (n_starts == 0 || starts) && (n_q == 0 || (q_start && q_node && q_out)),
            BLP_E_ARG, "blp_walk_run: bad arguments");
  for (int64_t i = 0; i < n_starts; ++i)
    BLP_CHECK(starts[i] >= 0 && starts[i] < w->n, BLP_E_ARG, "blp_walk_run: start out of range");
  for (int64_t k = 0; k < n_q; ++k) {
    BLP_CHECK(q_start[k] >= 0 && q_start[k] < n_starts && q_node[k] >= 0 && q_node[k] < w->n, BLP_E_ARG,
              "blp_walk_run: query out of range");
    BLP_CHECK(k == 0 || q_start[k] >= q_start[k - 1], BLP_E_ARG, "blp_walk_run: queries must be grouped by start");
  }
  BLP_HIP(hipSetDevice(w->device));
  int32_t *d_starts = nullptr, *d_qb = nullptr, *d_qn = nullptr;
  double* d_out = nullptr;
  const int64_t qcap = std::max<int64_t>(n_q, 1);
  BLP_HIP(dev_malloc(&d_starts, 4 * std::max<int64_t>(n_starts, 1)));
  BLP_HIP(dev_malloc(&d_qb, 4 * qcap));
  BLP_HIP(dev_malloc(&d_qn, 4 * qcap));
  BLP_HIP(dev_malloc(&d_out, 8 * qcap));
  if (n_starts) BLP_HIP(hipMemcpy(d_starts, starts, 4 * n_starts, hipMemcpyHostToDevice));
  std::vector<int32_t> qb(qcap);
  for (int64_t k = 0; k < n_q; ++k) qb[k] = q_start[k] % WB;
  if (n_q) {
    BLP_HIP(hipMemcpy(d_qb, qb.data(), 4 * n_q, hipMemcpyHostToDevice));
    BLP_HIP(hipMemcpy(d_qn, q_node, 4 * n_q, hipMemcpyHostToDevice));
  }
  const int step_grid = (int)std::min<int64_t>((w->n_items * WB + 255) / 256, (int64_t)w->n_cu * 32);
  hipEvent_t t0;
  int rc = timer_begin(w->timer, w->stream, &t0);
  if (rc) return rc;
  int64_t qk = 0;
  for (int64_t b0 = 0; b0 < n_starts; b0 += WB) {
    const int nb = (int)std::min<int64_t>(WB, n_starts - b0);
    BLP_HIP(hipMemsetAsync(w->d_p, 0, 8 * w->n * WB, w->stream));
    hipLaunchKernelGGL(k_walk_init, dim3(1), dim3(WB), 0, w->stream, d_starts + b0, nb, w->d_p);
    for (int it = 0; it < iterations; ++it) {
      if (w->n_split_rows)
        hipLaunchKernelGGL(k_walk_zero_split, dim3((unsigned)std::min<int64_t>((w->n_split_rows * WB + 255) / 256, 4096)),
                           dim3(256), 0, w->stream, w->d_split_rows, w->n_split_rows, w->d_pn);
      hipLaunchKernelGGL(k_walk_step, dim3(step_grid), dim3(256), 0, w->stream, w->d_items, w->n_items, w->d_col,
                         w->d_val, w->d_p, w->d_pn, scale);
      std::swap(w->d_p, w->d_pn);
    }
    int64_t qe = qk;
    while (qe < n_q && q_start[qe] < b0 + nb) ++qe;
    if (qe > qk)
      hipLaunchKernelGGL(k_walk_gather, dim3((unsigned)std::min<int64_t>((qe - qk + 255) / 256, 4096)), dim3(256), 0,
                         w->stream, w->d_p, d_qb + qk, d_qn + qk, qe - qk, d_out + qk);
    qk = qe;
  }
  BLP_HIP(hipGetLastError());
  if ((rc = timer_end(w->timer, w->stream, t0))) return rc;
  BLP_HIP(hipStreamSynchronize(w->stream));
  if (n_q) BLP_HIP(hipMemcpy(q_out, d_out, 8 * n_q, hipMemcpyDeviceToHost));
  for (void* p : {(void*)d_starts, (void*)d_qb, (void*)d_qn, (void*)d_out}) (void)hipFree(p);
  return BLP_OK;
}

// Single start, full probability vector (random_walks.run_random_walk, :43-53).
int blp_walk_run_dense(blp_walk* w, int32_t start, int iterations, double scale, double* p_out) {
  BLP_CHECK(w && p_out && start >= 0 && start < w->n && iterations >= 0, BLP_E_ARG, "blp_walk_run_dense: bad arguments");
  BLP_HIP(hipSetDevice(w->device));
  std::vector<int32_t> qs(w->n, 0), qn(w->n);
  for (int64_t i = 0; i < w->n; ++i) qn[i] = (int32_t)i;
  return blp_walk_run(w, &start, 1, iterations, scale, qs.data(), qn.data(), w->n, p_out);
}

int blp_walk_stats(blp_walk* w, double* total_ms, int64_t* launches) {
  BLP_CHECK(w, BLP_E_ARG, "blp_walk_stats: null handle");
  BLP_HIP(hipSetDevice(w->device));
  int rc = timer_collect(w->timer);
  if (rc) return rc;
  if (total_ms) *total_ms = w->timer.total_ms;
  if (launches) *launches = w->timer.launches;
  return BLP_OK;
}

}  // extern "C"
