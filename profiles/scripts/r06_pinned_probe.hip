// Round 6 probe (not product code): what a pinned staging ring costs on the box.
// hipHostMalloc of 16 / 64 MiB; hipMemcpyAsync of 2 MiB chunks from pinned memory: the time the
// call takes to return and the time until the stream has drained; one 128 MiB pinned copy.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
int main() {
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (size_t mb : {16, 64, 64, 128}) {
    void* h = nullptr;
    double t0 = now_ms();
    CK(hipHostMalloc(&h, mb << 20, hipHostMallocDefault));
    double t1 = now_ms();
    void* d = nullptr;
    CK(hipMalloc(&d, mb << 20));
    memset(h, 1, mb << 20);
    // one whole copy
    double t2 = now_ms();
    CK(hipMemcpyAsync(d, h, mb << 20, hipMemcpyHostToDevice, st));
    double t3 = now_ms();
    CK(hipStreamSynchronize(st));
    double t4 = now_ms();
    // chunks of 2 MiB and 512 KiB
    for (size_t ck : {size_t(2) << 20, size_t(512) << 10}) {
      double call = 0, tw0 = now_ms();
      for (size_t o = 0; o < (mb << 20); o += ck) {
        double a = now_ms();
        CK(hipMemcpyAsync((char*)d + o, (char*)h + o, ck, hipMemcpyHostToDevice, st));
        call += now_ms() - a;
      }
      double tw1 = now_ms();
      CK(hipStreamSynchronize(st));
      double tw2 = now_ms();
      printf("%3zu MiB: chunks of %zu KiB: calls sum %.3f ms, issue wall %.3f ms, drained at %.3f ms (%.1f GB/s)\n", mb,
             ck >> 10, call, tw1 - tw0, tw2 - tw0, (mb << 20) / ((tw2 - tw0) * 1e6));
    }
    printf("%3zu MiB: hipHostMalloc %.3f ms; one copy: call %.3f ms, done %.3f ms (%.1f GB/s)\n", mb, t1 - t0, t3 - t2,
           t4 - t2, (mb << 20) / ((t4 - t2) * 1e6));
    CK(hipFree(d));
    double t5 = now_ms();
    CK(hipHostFree(h));
    printf("%3zu MiB: hipHostFree %.3f ms\n", mb, now_ms() - t5);
  }
  return 0;
}
