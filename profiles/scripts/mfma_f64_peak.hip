// Microbenchmark: sustained v_mfma_f64_16x16x4f64 rate on one MI355X (the guides list no FP64
// MFMA figure). Two shapes of chain per wave:
//   indep: NC independent accumulators, issued round-robin (the pipe never waits on a result)
//   dep:   one accumulator, every MFMA depends on the previous one (k_svd_topk's K-chain)
// build: hipcc -O3 --offload-arch=gfx950 -o profiles/scripts/mfma_f64_peak profiles/scripts/mfma_f64_peak.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double double4_t __attribute__((ext_vector_type(4)));

template <int NC>
__global__ __launch_bounds__(256) void k_chain(int iters, double* out) {
  double a = 1.0 + 1e-9 * threadIdx.x, b = 1.0 - 1e-9 * threadIdx.x;
  double4_t d[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) d[c] = double4_t{0.0, 0.0, 0.0, 0.0};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int s = 0; s < 16; ++s)
#pragma unroll
      for (int c = 0; c < NC; ++c) d[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d[c], 0, 0, 0);
  }
  double acc = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) acc += d[c][0] + d[c][1] + d[c][2] + d[c][3];
  if (acc == 12345.0) out[threadIdx.x] = acc;  // keeps the chains live
}

template <int NC>
static void run(const char* name, int blocks, int iters, double* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k_chain<NC>, dim3(blocks), dim3(256), 0, 0, 10, out);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_chain<NC>, dim3(blocks), dim3(256), 0, 0, iters, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 16 * 16 * 4 * 16.0 * NC * iters * (double)blocks * 4;  // 4 waves per block
  printf("{\"chain\": \"%s\", \"accumulators\": %d, \"blocks\": %d, \"ms\": %.3f, \"tflops\": %.2f}\n", name, NC,
         blocks, ms, flops / ms / 1e9);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  double* out;
  hipMalloc(&out, 256 * sizeof(double));
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 2000;
  for (int per_cu : {1, 2, 4}) {
    run<1>("dep", cus * per_cu, iters, out);
    run<2>("indep", cus * per_cu, iters, out);
    run<4>("indep", cus * per_cu, iters, out);
  }
  hipFree(out);
  return 0;
}
