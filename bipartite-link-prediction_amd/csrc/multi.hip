// The engine's own communicator for the row-block sharded ingest (config 5):
// the exchange step of blp/dist.py (torch.distributed over RCCL) as C-ABI entry points, so a
// non-Python host drives the multi-GPU path with the same calls it uses for scoring.
//
// One process per GPU. The exchange is ONE RCCL all-gather of every rank's int32 edge partial:
// the per-rank counts go first (an all-gather of one int64 per rank), then the partials, padded
// to the largest count because RCCL has no all-gather-v, in one call whose send buffer holds
// the rank's `a` ids followed by its `b` ids. The padding is dropped on the device (one copy per
// rank's valid prefix) and the union's CSR is built and kept in HBM (csr.hip). Every rank ends
// with the same graph; all scoring after it is rank-local. Per rank the all-gather receives
// 8 * m_max * (world - 1) bytes: ~7 GB at 1B edges and 8 ranks, over xGMI's point-to-point links.
//
// RCCL is loaded at run time (dlopen of librccl.so.1 from the ROCm install), so libblp.so keeps
// depending only on the HIP runtime; without RCCL these entry points return BLP_E_UNSUP.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <mutex>

#include "blp_internal.h"

using namespace blp;

namespace {

struct Rccl {
  void* h = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

// the resolved library, or null (with the reason in the error string)
const Rccl* rccl() {
  static std::once_flag once;
  static Rccl r;
  static bool ok = false;
  std::call_once(once, [] {
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      r.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (r.h) break;
    }
    if (!r.h) return;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(r.h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(r.h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(r.h, "ncclCommDestroy"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(r.h, "ncclAllGather"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(r.h, "ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(r.h, "ncclGetErrorString"));
    ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.all_reduce && r.error_string;
  });
  return ok ? &r : nullptr;
}

int comm_fail(const Rccl* r, ncclResult_t e, const char* what) {
  return fail(BLP_E_COMM, std::string(what) + ": " + (r ? r->error_string(e) : "RCCL unavailable"));
}

#define BLP_NCCL_OR(call, handler)                                  \
  do {                                                              \
    ncclResult_t _e = (call);                                       \
    if (_e != ncclSuccess) return handler(comm_fail(R, _e, #call)); \
  } while (0)

int no_rccl() { return fail(BLP_E_UNSUP, "RCCL (librccl.so.1) could not be loaded"); }

// true if p is device memory of the current device (hipMalloc / torch CUDA tensors)
bool on_device(const void* p) {
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // an unregistered host pointer: clear the sticky error
    return false;
  }
  return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

}  // namespace

struct blp_multi {
  int world = 0, rank = 0, device = 0;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  DevBuf scratch;  // counts / reductions (16 B per rank)
};

extern "C" int blp_multi_unique_id(uint8_t* id) {
  BLP_CHECK(id, BLP_E_ARG, "blp_multi_unique_id: null id");
  const Rccl* R = rccl();
  if (!R) return no_rccl();
  ncclUniqueId u;
  const ncclResult_t e = R->get_unique_id(&u);
  if (e != ncclSuccess) return comm_fail(R, e, "ncclGetUniqueId");
  static_assert(sizeof(u.internal) == BLP_MULTI_ID_BYTES, "RCCL id size");
  std::copy(u.internal, u.internal + BLP_MULTI_ID_BYTES, reinterpret_cast<char*>(id));
  return BLP_OK;
}

extern "C" int blp_multi_destroy(blp_multi* m) {
  if (!m) return BLP_OK;
  (void)hipSetDevice(m->device);
  if (m->stream) (void)hipStreamSynchronize(m->stream);
  const Rccl* R = rccl();
  if (m->comm && R) R->comm_destroy(m->comm);
  m->scratch.release();
  if (m->stream) (void)hipStreamDestroy(m->stream);
  delete m;
  return BLP_OK;
}

extern "C" int blp_multi_init(const uint8_t* id, int world, int rank, int device, blp_multi** out) {
  BLP_CHECK(id && out && world >= 1 && rank >= 0 && rank < world, BLP_E_ARG, "blp_multi_init: bad arguments");
  const Rccl* R = rccl();
  if (!R) return no_rccl();
  int ndev = 0;
  BLP_HIP(hipGetDeviceCount(&ndev));
  BLP_CHECK(device >= 0 && device < ndev, BLP_E_ARG, "blp_multi_init: no such device");
  BLP_HIP(hipSetDevice(device));
  blp_multi* m = new blp_multi();
  m->world = world;
  m->rank = rank;
  m->device = device;
  auto done = [&](int rc) {
    if (rc != BLP_OK) blp_multi_destroy(m);
    return rc;
  };
  BLP_HIP_OR(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking), done);
  int rc = m->scratch.reserve(16 * (size_t)world + 16);
  if (rc) return done(rc);
  ncclUniqueId u;
  std::copy(reinterpret_cast<const char*>(id), reinterpret_cast<const char*>(id) + BLP_MULTI_ID_BYTES, u.internal);
  BLP_NCCL_OR(R->comm_init_rank(&m->comm, world, u, rank), done);
  *out = m;
  return BLP_OK;
}

extern "C" int blp_multi_info(const blp_multi* m, int* world, int* rank, int* device) {
  BLP_CHECK(m, BLP_E_ARG, "blp_multi_info: null handle");
  if (world) *world = m->world;
  if (rank) *rank = m->rank;
  if (device) *device = m->device;
  return BLP_OK;
}

extern "C" int blp_multi_allreduce(blp_multi* m, double* v, int op) {
  BLP_CHECK(m && v && (op == BLP_MULTI_SUM || op == BLP_MULTI_MAX), BLP_E_ARG, "blp_multi_allreduce: bad arguments");
  const Rccl* R = rccl();
  BLP_HIP(hipSetDevice(m->device));
  double* d = m->scratch.as<double>();
  BLP_HIP(hipMemcpyAsync(d, v, 8, hipMemcpyHostToDevice, m->stream));
  auto ret = [](int rc) { return rc; };
  BLP_NCCL_OR(R->all_reduce(d, d + 1, 1, ncclFloat64, op == BLP_MULTI_MAX ? ncclMax : ncclSum, m->comm, m->stream),
              ret);
  BLP_HIP(hipMemcpyAsync(v, d + 1, 8, hipMemcpyDeviceToHost, m->stream));
  BLP_HIP(hipStreamSynchronize(m->stream));
  return BLP_OK;
}

namespace {

// The post-gather half of the exchange: recv holds `world` slots of [a | b], each half padded to
// m_max = max(counts) (slot r: rank r's a ids in [0, m_max), its b ids in [m_max, 2 m_max)); the
// valid prefixes are copied back to back on `st` (device or host recv) and the union's CSR is
// built in HBM. The padding is never read.
int compact_csr(int device, hipStream_t st, const int32_t* recv, const int64_t* cnt, int W, int64_t n_nodes,
                blp_csr** out, int64_t* bytes_in) {
  int64_t m_max = 0, m_tot = 0;
  for (int r = 0; r < W; ++r) {
    BLP_CHECK(cnt[r] >= 0, BLP_E_ARG, "blp_multi_compact_csr: negative count");
    m_max = std::max(m_max, cnt[r]);
    m_tot += cnt[r];
  }
  BLP_CHECK(m_max == 0 || recv, BLP_E_ARG, "blp_multi_compact_csr: null receive buffer");
  ScopedBuf ua, ub;
  int rc;
  if ((rc = ua.reserve(4 * (size_t)std::max<int64_t>(m_tot, 1))) ||
      (rc = ub.reserve(4 * (size_t)std::max<int64_t>(m_tot, 1))))
    return rc;
  if (m_max > 0) {
    const hipMemcpyKind k = on_device(recv) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    int64_t off = 0;
    for (int r = 0; r < W; ++r) {
      if (!cnt[r]) continue;
      const int32_t* src = recv + (size_t)r * 2 * m_max;
      BLP_HIP(hipMemcpyAsync(ua.as<int32_t>() + off, src, 4 * (size_t)cnt[r], k, st));
      BLP_HIP(hipMemcpyAsync(ub.as<int32_t>() + off, src + m_max, 4 * (size_t)cnt[r], k, st));
      off += cnt[r];
    }
    BLP_HIP(hipStreamSynchronize(st));
  }
  rc = blp_csr_build_device(device, ua.as<int32_t>(), ub.as<int32_t>(), m_tot, n_nodes, out);
  if (rc == BLP_OK && bytes_in) *bytes_in = 8 * m_max * (int64_t)(W - 1);
  return rc;
}

}  // namespace

extern "C" int blp_multi_compact_csr(int device, const int32_t* recv, const int64_t* counts, int world, int64_t n_nodes,
                                     blp_csr** out, int64_t* bytes_in) {
  BLP_CHECK(counts && out && world >= 1 && n_nodes >= 0, BLP_E_ARG, "blp_multi_compact_csr: bad arguments");
  int ndev = 0;
  BLP_HIP(hipGetDeviceCount(&ndev));
  BLP_CHECK(device >= 0 && device < ndev, BLP_E_ARG, "blp_multi_compact_csr: no such device");
  BLP_HIP(hipSetDevice(device));
  hipStream_t st = nullptr;
  BLP_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int rc = compact_csr(device, st, recv, counts, world, n_nodes, out, bytes_in);
  (void)hipStreamSynchronize(st);
  (void)hipStreamDestroy(st);
  return rc;
}

extern "C" int blp_multi_gather_csr(blp_multi* m, const int32_t* a, const int32_t* b, int64_t m_r, int64_t n_nodes,
                                    blp_csr** out, int64_t* bytes_in) {
  BLP_CHECK(m && out && m_r >= 0 && n_nodes >= 0 && (m_r == 0 || (a && b)), BLP_E_ARG,
            "blp_multi_gather_csr: bad arguments");
  const Rccl* R = rccl();
  BLP_HIP(hipSetDevice(m->device));
  const int W = m->world;
  ScopedBuf send, recv;
  auto done = [&](int rc) {
    (void)hipStreamSynchronize(m->stream);
    return rc;
  };
  // 1. counts: one int64 per rank
  int64_t* d_cnt = m->scratch.as<int64_t>();
  std::vector<int64_t> cnt(W);
  BLP_HIP_OR(hipMemcpyAsync(d_cnt, &m_r, 8, hipMemcpyHostToDevice, m->stream), done);
  BLP_NCCL_OR(R->all_gather(d_cnt, d_cnt + 1, 1, ncclInt64, m->comm, m->stream), done);
  BLP_HIP_OR(hipMemcpyAsync(cnt.data(), d_cnt + 1, 8 * (size_t)W, hipMemcpyDeviceToHost, m->stream), done);
  BLP_HIP_OR(hipStreamSynchronize(m->stream), done);
  const int64_t m_max = *std::max_element(cnt.begin(), cnt.end());
  BLP_CHECK(cnt[m->rank] == m_r, BLP_E_COMM, "blp_multi_gather_csr: count exchange mismatch");
  int rc;
  if (m_max > 0) {
    // 2. the partials: [a | b] per rank, each half padded to m_max (padding never read)
    if ((rc = send.reserve(8 * (size_t)m_max)) || (rc = recv.reserve(8 * (size_t)m_max * W))) return done(rc);
    int32_t* s = send.as<int32_t>();
    if (m_r) {
      const hipMemcpyKind ka = on_device(a) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
      const hipMemcpyKind kb = on_device(b) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
      BLP_HIP_OR(hipMemcpyAsync(s, a, 4 * (size_t)m_r, ka, m->stream), done);
      BLP_HIP_OR(hipMemcpyAsync(s + m_max, b, 4 * (size_t)m_r, kb, m->stream), done);
    }
    BLP_NCCL_OR(R->all_gather(s, recv.p, 2 * (size_t)m_max, ncclInt32, m->comm, m->stream), done);
    send.release();
  }
  // 3. drop the padding and build the union's CSR, kept in HBM
  return done(compact_csr(m->device, m->stream, recv.as<int32_t>(), cnt.data(), W, n_nodes, out, bytes_in));
}
