// Device CSR builder: the multi-GPU ingest path.
//
// After the RCCL all-gather of the per-rank edge partials, every rank holds the complete edge
// list in HBM (int32 endpoints, dense ids). This builds the same undirected simple-graph CSR
// as blp_csr_from_edges (graph.hip; SNAP LoadEdgeList semantics, similarity.py:16): both
// directions, duplicates merged, rows sorted, self-loops flagged but not stored. One 64-bit
// key (row << 32 | col) per directed entry, a device radix sort over the bits that carry ids,
// a unique pass, and the row offsets by binary search of the sorted keys. 1B edges: 2B keys,
// 32 GB of keys + sort scratch on a 288 GB part.
#include <hipcub/hipcub.hpp>

#include "blp_internal.h"

namespace {

constexpr uint64_t KEY_NONE = ~0ull;  // self-loop placeholders sort last and are dropped

__global__ void k_edge_keys(const int32_t* a, const int32_t* b, int64_t m, int64_t n, uint64_t* keys,
                            uint8_t* self_loop, int* bad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t u = a[i], v = b[i];
    if (u < 0 || v < 0 || u >= n || v >= n) {
      *bad = 1;
      keys[2 * i] = keys[2 * i + 1] = KEY_NONE;
      continue;
    }
    if (u == v) {
      self_loop[u] = 1;
      keys[2 * i] = keys[2 * i + 1] = KEY_NONE;
      continue;
    }
    keys[2 * i] = ((uint64_t)(uint32_t)u << 32) | (uint32_t)v;
    keys[2 * i + 1] = ((uint64_t)(uint32_t)v << 32) | (uint32_t)u;
  }
}

// row_ptr[r] = first sorted key with row >= r (r in [0, n]); col_idx = low halves
__global__ void k_row_ptr(const uint64_t* keys, int64_t nnz, int64_t n, int64_t* rp) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r <= n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t want = (uint64_t)r << 32;
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < want) lo = mid + 1; else hi = mid;
    }
    rp[r] = lo;
  }
}

__global__ void k_low_halves(const uint64_t* keys, int64_t nnz, int32_t* ci) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x)
    ci[i] = (int32_t)(uint32_t)keys[i];
}

__global__ void k_iota(int32_t* v, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] = (int32_t)i;
}

}  // namespace

using namespace blp;

// A CSR built on the device and kept there (blp_csr_build_device): the row offsets, the
// padded column ids (CI_PAD ids of zeros on each side, the layout blp_graph uses) and the
// self-loop flags. blp_graph_create_from_csr adopts the buffers; no host round trip.
struct blp_csr {
  int device = 0;
  int64_t n = 0, nnz = 0;
  int64_t* d_rp = nullptr;   // [n + 1]
  int32_t* d_ci = nullptr;   // [nnz], CI_PAD ids readable on each side (allocation starts at d_ci - CI_PAD)
  uint8_t* d_self = nullptr; // [max(n, 1)]
};

extern "C" int blp_csr_destroy(blp_csr* c) {
  if (!c) return BLP_OK;
  (void)hipSetDevice(c->device);
  if (c->d_rp) (void)hipFree(c->d_rp);
  if (c->d_ci) (void)hipFree(c->d_ci - CI_PAD);
  if (c->d_self) (void)hipFree(c->d_self);
  delete c;
  return BLP_OK;
}

// sync_device: the endpoints come from another stream (the RCCL all-gather, a torch copy), so
// wait for everything queued on the device first (a one-off ingest step). blp_csr_build_host's
// uploads are synchronous already and skip it, so a graph load never waits for other graphs'
// batches still running on the device.
int blp::csr_build(int device, const int32_t* d_a, const int32_t* d_b, int64_t m, int64_t n, blp_csr** out,
                   bool sync_device) {
  BLP_CHECK(out && n >= 0 && m >= 0 && (m == 0 || (d_a && d_b)), BLP_E_ARG, "blp_csr_build_device: bad arguments");
  BLP_CHECK(n < (int64_t(1) << 31), BLP_E_ARG, "blp_csr_build_device: n_nodes must fit int32");
  int ndev = 0;
  BLP_HIP(hipGetDeviceCount(&ndev));
  BLP_CHECK(device >= 0 && device < ndev, BLP_E_ARG, "blp_csr_build_device: no such device");
  BLP_HIP(hipSetDevice(device));
  if (sync_device) BLP_HIP(hipDeviceSynchronize());
  hipStream_t st = stream_take(device);  // pooled (blp_stream_prewarm)
  if (!st) return BLP_E_HIP_BASE;
  blp_csr* c = new blp_csr();
  c->device = device;
  c->n = n;
  DevBuf keys, sorted, temp, flag, nsel;
  auto done = [&](int rc) {
    for (DevBuf* b : {&keys, &sorted, &temp, &flag, &nsel}) b->release();
    stream_give(device, st);  // synchronized first
    if (rc != BLP_OK) blp_csr_destroy(c);
    return rc;
  };
  int rc;
  const int64_t mk = 2 * m;
  BLP_HIP_OR(dev_malloc(&c->d_rp, 8 * (n + 1)), done);
  BLP_HIP_OR(dev_malloc(&c->d_self, std::max<int64_t>(n, 1)), done);
  if ((rc = flag.reserve(4)) || (rc = nsel.reserve(8))) return done(rc);
  BLP_HIP_OR(hipMemsetAsync(c->d_self, 0, std::max<int64_t>(n, 1), st), done);
  BLP_HIP_OR(hipMemsetAsync(flag.p, 0, 4, st), done);
  BLP_HIP_OR(hipMemsetAsync(c->d_rp, 0, 8 * (n + 1), st), done);
  int64_t nnz = 0;
  const uint64_t* uq = nullptr;  // the unique sorted keys (in keys or sorted)
  if (m) {
    if ((rc = keys.reserve(8 * mk)) || (rc = sorted.reserve(8 * mk))) return done(rc);
    hipLaunchKernelGGL(k_edge_keys, dim3(4096), dim3(256), 0, st, d_a, d_b, m, n, keys.as<uint64_t>(), c->d_self,
                       flag.as<int>());
    BLP_HIP_OR(hipGetLastError(), done);
    // sort only the bits that carry ids: 32 + ceil(log2 n) (KEY_NONE has them all set)
    int idbits = 1;
    while ((int64_t(1) << idbits) < n) ++idbits;
    const int end_bit = std::min(64, 32 + idbits + 1);
    size_t tb = 0, tb2 = 0;
    // the sort ping-pongs between the two key buffers (no third one of the same size inside the
    // temporary storage), then the unique keys go to whichever buffer the sorted ones are not in
    hipcub::DoubleBuffer<uint64_t> kb(keys.as<uint64_t>(), sorted.as<uint64_t>());
    BLP_HIP_OR(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, kb, mk, 0, end_bit, st), done);
    BLP_HIP_OR(hipcub::DeviceSelect::Unique(nullptr, tb2, kb.Current(), kb.Alternate(), nsel.as<int64_t>(), mk, st),
               done);
    if ((rc = temp.reserve(std::max(tb, tb2)))) return done(rc);
    tb = temp.bytes;
    BLP_HIP_OR(hipcub::DeviceRadixSort::SortKeys(temp.p, tb, kb, mk, 0, end_bit, st), done);
    tb2 = temp.bytes;
    BLP_HIP_OR(hipcub::DeviceSelect::Unique(temp.p, tb2, kb.Current(), kb.Alternate(), nsel.as<int64_t>(), mk, st),
               done);
    uq = kb.Alternate();
    int64_t nu = 0;
    int bad = 0;
    BLP_HIP_OR(hipMemcpyAsync(&nu, nsel.p, 8, hipMemcpyDeviceToHost, st), done);
    BLP_HIP_OR(hipMemcpyAsync(&bad, flag.p, 4, hipMemcpyDeviceToHost, st), done);
    BLP_HIP_OR(hipStreamSynchronize(st), done);
    if (bad) return done(fail(BLP_E_ARG, "blp_csr_build_device: node id out of range"));
    nnz = nu;
    if (nnz > 0) {  // a trailing KEY_NONE (self-loops present) is not an entry
      uint64_t last = 0;
      BLP_HIP_OR(hipMemcpyAsync(&last, uq + nnz - 1, 8, hipMemcpyDeviceToHost, st), done);
      BLP_HIP_OR(hipStreamSynchronize(st), done);
      if (last == KEY_NONE) --nnz;
    }
    (uq == keys.as<uint64_t>() ? sorted : keys).release();  // the buffer not holding the unique keys
    temp.release();
    hipLaunchKernelGGL(k_row_ptr, dim3(2048), dim3(256), 0, st, uq, nnz, n, c->d_rp);
    BLP_HIP_OR(hipGetLastError(), done);
  }
  BLP_HIP_OR(dev_malloc(&c->d_ci, sizeof(int32_t) * (nnz + 2 * CI_PAD)), done);
  c->d_ci += CI_PAD;
  BLP_HIP_OR(hipMemsetAsync(c->d_ci - CI_PAD, 0, sizeof(int32_t) * (nnz + 2 * CI_PAD), st), done);
  if (nnz) {
    hipLaunchKernelGGL(k_low_halves, dim3(4096), dim3(256), 0, st, uq, nnz, c->d_ci);
    BLP_HIP_OR(hipGetLastError(), done);
  }
  BLP_HIP_OR(hipStreamSynchronize(st), done);
  c->nnz = nnz;
  *out = c;
  return done(BLP_OK);
}

extern "C" int blp_csr_build_device(int device, const int32_t* d_a, const int32_t* d_b, int64_t m, int64_t n,
                                    blp_csr** out) {
  return csr_build(device, d_a, d_b, m, n, out, true);
}

// Host-resident endpoints (similarity.main's graph.txt load): upload, then the device build.
extern "C" int blp_csr_build_host(int device, const int32_t* a, const int32_t* b, int64_t m, int64_t n, blp_csr** out) {
  BLP_CHECK(out && m >= 0 && (m == 0 || (a && b)), BLP_E_ARG, "blp_csr_build_host: bad arguments");
  int ndev = 0;
  BLP_HIP(hipGetDeviceCount(&ndev));
  BLP_CHECK(device >= 0 && device < ndev, BLP_E_ARG, "blp_csr_build_host: no such device");
  BLP_HIP(hipSetDevice(device));
  DevBuf da, db;
  int rc;
  if ((rc = da.reserve(4 * std::max<int64_t>(m, 1))) || (rc = db.reserve(4 * std::max<int64_t>(m, 1)))) return rc;
  if (m) {
    hipError_t e = hipMemcpy(da.p, a, 4 * m, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(db.p, b, 4 * m, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      da.release();
      db.release();
      return hip_fail(e, "hipMemcpy (edge upload)", __FILE__, __LINE__);
    }
  }
  rc = csr_build(device, da.as<int32_t>(), db.as<int32_t>(), m, n, out, false);  // uploads were synchronous
  da.release();
  db.release();
  return rc;
}

extern "C" int blp_csr_info(const blp_csr* c, int64_t* n_nodes, int64_t* nnz) {
  BLP_CHECK(c, BLP_E_ARG, "blp_csr_info: null csr");
  if (n_nodes) *n_nodes = c->n;
  if (nnz) *nnz = c->nnz;
  return BLP_OK;
}

extern "C" int blp_csr_fetch(const blp_csr* c, int64_t* row_ptr, int32_t* col_idx, uint8_t* self_loop) {
  BLP_CHECK(c, BLP_E_ARG, "blp_csr_fetch: null csr");
  BLP_HIP(hipSetDevice(c->device));
  prefault_host(row_ptr, 8 * (size_t)(c->n + 1));
  if (c->nnz && col_idx) prefault_host(col_idx, 4 * (size_t)c->nnz);
  hipStream_t st = stream_take(c->device);
  if (!st) return BLP_E_HIP_BASE;
  int rc = BLP_OK;
  if (row_ptr) rc = copy_sync(row_ptr, c->d_rp, 8 * (c->n + 1), hipMemcpyDeviceToHost, st);
  if (!rc && col_idx && c->nnz) rc = copy_sync(col_idx, c->d_ci, 4 * c->nnz, hipMemcpyDeviceToHost, st);
  if (!rc && self_loop && c->n) rc = copy_sync(self_loop, c->d_self, c->n, hipMemcpyDeviceToHost, st);
  stream_give(c->device, st);
  if (rc) return rc;
  return BLP_OK;
}

extern "C" int blp_graph_create_from_csr(blp_csr* c, const int64_t* row_ptr, const int32_t* col_idx,
                                         const double* aaw, blp_graph** out) {
  BLP_CHECK(c && out && row_ptr, BLP_E_ARG, "blp_graph_create_from_csr: bad arguments");  // col_idx may be NULL (fetched on demand)
  BLP_CHECK(row_ptr[c->n] == c->nnz, BLP_E_ARG, "blp_graph_create_from_csr: host mirror does not match the csr");
  BLP_HIP(hipSetDevice(c->device));
  blp_graph* g = new blp_graph();
  g->device = c->device;
  g->n = c->n;
  g->nnz = c->nnz;
  g->hrp = row_ptr;  // borrowed: the caller keeps them alive and unchanged for the graph's lifetime
  g->hci = col_idx;
  g->d_rp = c->d_rp;  // the device CSR, adopted once everything derived from it is built
  g->d_ci = c->d_ci;
  int rc = graph_finish(g, aaw);
  if (rc != BLP_OK) {
    g->d_rp = nullptr;  // c still owns its buffers: the caller may retry or destroy it
    g->d_ci = nullptr;
    blp_graph_destroy(g);
    return rc;
  }
  c->d_rp = nullptr;  // c is consumed
  c->d_ci = nullptr;
  blp_csr_destroy(c);
  *out = g;
  return BLP_OK;
}

extern "C" int blp_csr_from_edges_device(int device, const int32_t* d_a, const int32_t* d_b, int64_t m, int64_t n,
                                         int64_t* row_ptr, int32_t* col_idx, uint8_t* self_loop, int64_t* nnz_out) {
  BLP_CHECK(n >= 0 && m >= 0 && row_ptr && nnz_out && (m == 0 || (d_a && d_b && col_idx)), BLP_E_ARG,
            "blp_csr_from_edges_device: bad arguments");
  blp_csr* c = nullptr;
  int rc = blp_csr_build_device(device, d_a, d_b, m, n, &c);
  if (rc) return rc;
  rc = blp_csr_fetch(c, row_ptr, col_idx, self_loop);
  if (!rc) *nnz_out = c->nnz;
  blp_csr_destroy(c);
  return rc;
}

// Loads this file's GPU code object (blp_stream_prewarm): the HIP runtime loads a translation
// unit's code object on the first launch of any of its kernels, 10-30 ms on the caller's thread.
namespace blp {
int preload_csr() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_edge_keys)) == hipSuccess ? 0 : -1;
}
}  // namespace blp

// Indices 0..n-1 ordered by key descending, ties by index (a stable radix sort of (key, index)
// pairs): blp_batch_create's largest-first source order (BLP_LPT), on the batch's stream.
int blp::order_desc_u64(const uint64_t* d_keys, int64_t n, int32_t* d_idx, hipStream_t st) {
  if (n <= 0) return BLP_OK;
  DevBuf kout, iin, temp;
  auto done = [&](int rc) {
    const hipError_t se = hipStreamSynchronize(st);  // the scratch goes back after the sort ran
    for (DevBuf* b : {&kout, &iin, &temp}) {
      const int r = b->release();
      if (!rc) rc = r;
    }
    if (se != hipSuccess && !rc) rc = hip_fail(se, "hipStreamSynchronize (order_desc_u64)", __FILE__, __LINE__);
    return rc;
  };
  int rc;
  if ((rc = kout.reserve(8 * n)) || (rc = iin.reserve(4 * n))) return done(rc);
  hipLaunchKernelGGL(k_iota, dim3((unsigned)std::min<int64_t>(1024, (n + 255) / 256)), dim3(256), 0, st, iin.as<int32_t>(), n);
  BLP_HIP_OR(hipGetLastError(), done);
  size_t tb = 0;
  BLP_HIP_OR(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tb, d_keys, kout.as<uint64_t>(), iin.as<int32_t>(), d_idx,
                                                          (int)n, 0, 64, st), done);
  if ((rc = temp.reserve(std::max<size_t>(tb, 16)))) return done(rc);
  tb = temp.bytes;
  BLP_HIP_OR(hipcub::DeviceRadixSort::SortPairsDescending(temp.p, tb, d_keys, kout.as<uint64_t>(), iin.as<int32_t>(), d_idx,
                                                          (int)n, 0, 64, st), done);
  return done(BLP_OK);
}
