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

}  // namespace

using namespace blp;

extern "C" int blp_csr_from_edges_device(int device, const int32_t* d_a, const int32_t* d_b, int64_t m, int64_t n,
                                         int64_t* row_ptr, int32_t* col_idx, uint8_t* self_loop, int64_t* nnz_out) {
  BLP_CHECK(n >= 0 && m >= 0 && row_ptr && nnz_out && (m == 0 || (d_a && d_b && col_idx)), BLP_E_ARG,
            "blp_csr_from_edges_device: bad arguments");
  BLP_CHECK(n < (int64_t(1) << 31), BLP_E_ARG, "blp_csr_from_edges_device: n_nodes must fit int32");
  BLP_HIP(hipSetDevice(device));
  hipStream_t st = nullptr;
  BLP_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  DevBuf keys, sorted, temp, rp, selfb, flag, nsel;
  auto done = [&](int rc) {
    for (DevBuf* b : {&keys, &sorted, &temp, &rp, &selfb, &flag, &nsel}) b->release();
    (void)hipStreamDestroy(st);
    return rc;
  };
  int rc;
  const int64_t mk = 2 * m;
  if ((rc = keys.reserve(8 * std::max<int64_t>(mk, 1))) || (rc = sorted.reserve(8 * std::max<int64_t>(mk, 1))) ||
      (rc = rp.reserve(8 * (n + 1))) || (rc = selfb.reserve(std::max<int64_t>(n, 1))) || (rc = flag.reserve(4)) ||
      (rc = nsel.reserve(8)))
    return done(rc);
  BLP_HIP_OR(hipMemsetAsync(selfb.p, 0, std::max<int64_t>(n, 1), st), done);
  BLP_HIP_OR(hipMemsetAsync(flag.p, 0, 4, st), done);
  int64_t nnz = 0;
  if (m) {
    hipLaunchKernelGGL(k_edge_keys, dim3(4096), dim3(256), 0, st, d_a, d_b, m, n, keys.as<uint64_t>(),
                       selfb.as<uint8_t>(), flag.as<int>());
    BLP_HIP_OR(hipGetLastError(), done);
    // sort only the bits that carry ids: 32 + ceil(log2 n) (KEY_NONE has them all set)
    int idbits = 1;
    while ((int64_t(1) << idbits) < n) ++idbits;
    const int end_bit = std::min(64, 32 + idbits + 1);
    size_t tb = 0, tb2 = 0;
    BLP_HIP_OR(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, keys.as<uint64_t>(), sorted.as<uint64_t>(), mk, 0,
                                                 end_bit, st), done);
    BLP_HIP_OR(hipcub::DeviceSelect::Unique(nullptr, tb2, sorted.as<uint64_t>(), keys.as<uint64_t>(),
                                            nsel.as<int64_t>(), mk, st), done);
    if ((rc = temp.reserve(std::max(tb, tb2)))) return done(rc);
    tb = temp.bytes;
    BLP_HIP_OR(hipcub::DeviceRadixSort::SortKeys(temp.p, tb, keys.as<uint64_t>(), sorted.as<uint64_t>(), mk, 0,
                                                 end_bit, st), done);
    tb2 = temp.bytes;
    BLP_HIP_OR(hipcub::DeviceSelect::Unique(temp.p, tb2, sorted.as<uint64_t>(), keys.as<uint64_t>(),
                                            nsel.as<int64_t>(), mk, st), done);
    int64_t nu = 0;
    int bad = 0;
    BLP_HIP_OR(hipMemcpyAsync(&nu, nsel.p, 8, hipMemcpyDeviceToHost, st), done);
    BLP_HIP_OR(hipMemcpyAsync(&bad, flag.p, 4, hipMemcpyDeviceToHost, st), done);
    BLP_HIP_OR(hipStreamSynchronize(st), done);
    if (bad) return done(fail(BLP_E_ARG, "blp_csr_from_edges_device: node id out of range"));
    nnz = nu;
    if (nnz > 0) {  // a trailing KEY_NONE (self-loops present) is not an entry
      uint64_t last = 0;
      BLP_HIP_OR(hipMemcpy(&last, keys.as<uint64_t>() + nnz - 1, 8, hipMemcpyDeviceToHost), done);
      if (last == KEY_NONE) --nnz;
    }
    hipLaunchKernelGGL(k_row_ptr, dim3(2048), dim3(256), 0, st, keys.as<uint64_t>(), nnz, n, rp.as<int64_t>());
    BLP_HIP_OR(hipGetLastError(), done);
    // the low halves go into the (now free) sort buffer, then to the host
    hipLaunchKernelGGL(k_low_halves, dim3(4096), dim3(256), 0, st, keys.as<uint64_t>(), nnz, sorted.as<int32_t>());
    BLP_HIP_OR(hipGetLastError(), done);
    BLP_HIP_OR(hipMemcpyAsync(row_ptr, rp.p, 8 * (n + 1), hipMemcpyDeviceToHost, st), done);
    if (nnz) BLP_HIP_OR(hipMemcpyAsync(col_idx, sorted.p, 4 * nnz, hipMemcpyDeviceToHost, st), done);
  } else {
    for (int64_t i = 0; i <= n; ++i) row_ptr[i] = 0;
  }
  if (self_loop && n) BLP_HIP_OR(hipMemcpyAsync(self_loop, selfb.p, n, hipMemcpyDeviceToHost, st), done);
  BLP_HIP_OR(hipStreamSynchronize(st), done);
  *nnz_out = nnz;
  return done(BLP_OK);
}
