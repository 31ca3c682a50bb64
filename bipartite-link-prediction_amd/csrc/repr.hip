// Score-file doubles formatted on the device: repr(v) of every value into a 24-byte slot
// (repr.h), so similarity.main's host writer only copies bytes. At config 2 the three
// double-valued files hold 22.6M values; CPython-exact shortest formatting costs ~70 ns per
// value on a host core (std::to_chars), 1.6 s of CPU per main() spread over 16 threads,
// about two thirds of the file phase. One thread per value here, the slot stored as three
// 8-byte words.
#include "blp_internal.h"
#include "repr.h"

namespace {

__device__ const uint64_t g_repr_p5[2 * BLP_REPR_N_P5] = BLP_REPR_P5_INIT;
__device__ const uint64_t g_repr_inv[2 * BLP_REPR_N_INV] = BLP_REPR_INV_INIT;
const uint64_t h_repr_p5[2 * BLP_REPR_N_P5] = BLP_REPR_P5_INIT;
const uint64_t h_repr_inv[2 * BLP_REPR_N_INV] = BLP_REPR_INV_INIT;

constexpr int REPR_BLOCK = 256;

__global__ __launch_bounds__(REPR_BLOCK) void k_repr(const double* __restrict__ v, int64_t n, int zero_int,
                                                     uint64_t* __restrict__ out) {
  const blp::ReprTables t{g_repr_p5, g_repr_inv};
  for (int64_t i = blockIdx.x * (int64_t)REPR_BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * REPR_BLOCK) {
    blp::Repr24 r;
    blp::repr_double(v[i], zero_int != 0, t, r);
    out[3 * i] = r.w0;
    out[3 * i + 1] = r.w1;
    out[3 * i + 2] = r.w2;
  }
}

}  // namespace

namespace blp {

int repr_launch(const double* d_v, int64_t n, bool zero_int, char* d_out, int n_cu, hipStream_t s) {
  if (n <= 0) return BLP_OK;
  const int64_t blocks = std::min<int64_t>((n + REPR_BLOCK - 1) / REPR_BLOCK, (int64_t)n_cu * 32);
  hipLaunchKernelGGL(k_repr, dim3((unsigned)blocks), dim3(REPR_BLOCK), 0, s, d_v, n, zero_int ? 1 : 0,
                     reinterpret_cast<uint64_t*>(d_out));
  BLP_HIP(hipGetLastError());
  return BLP_OK;
}

}  // namespace blp

extern "C" {

int blp_repr_format(const double* values, int64_t n, int zero_int, char* out) {
  BLP_CHECK(n >= 0 && (n == 0 || (values && out)), BLP_E_ARG, "blp_repr_format: bad arguments");
  const blp::ReprTables t{h_repr_p5, h_repr_inv};
  for (int64_t i = 0; i < n; ++i) {
    blp::Repr24 r;
    blp::repr_double(values[i], zero_int != 0, t, r);
    std::memcpy(out + blp::REPR_SLOT * i, &r.w0, 8);
    std::memcpy(out + blp::REPR_SLOT * i + 8, &r.w1, 8);
    std::memcpy(out + blp::REPR_SLOT * i + 16, &r.w2, 8);
  }
  return BLP_OK;
}

int blp_repr_format_device(int device, const double* d_values, int64_t n, int zero_int, char* d_out) {
  BLP_CHECK(n >= 0 && (n == 0 || (d_values && d_out)), BLP_E_ARG, "blp_repr_format_device: bad arguments");
  if (n == 0) return BLP_OK;
  BLP_HIP(hipSetDevice(device));
  int n_cu = 0;
  BLP_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device));
  int rc = blp::repr_launch(d_values, n, zero_int != 0, d_out, n_cu, nullptr);
  if (rc) return rc;
  BLP_HIP(hipDeviceSynchronize());
  return BLP_OK;
}

}  // extern "C"

// Loads this file's GPU code object (blp_stream_prewarm): the HIP runtime loads a translation
// unit's code object on the first launch of any of its kernels, 10-30 ms on the caller's thread.
namespace blp {
int preload_repr() {
  hipFuncAttributes fa;
  return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_repr)) == hipSuccess ? 0 : -1;
}
}  // namespace blp
