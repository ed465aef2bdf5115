// PCIe bandwidth of the ways the host pipeline moves bytes (one MI355X, pinned host memory):
//   H2D DMA, D2H DMA (hipMemcpyAsync, one stream / two streams), and kernel stores into
//   host-mapped pinned memory (the tape job's way of writing host tapes), 64 MB each.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_store(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t B = 64ull << 20;
  void *h, *h2, *d, *d2, *hd;
  (void)hipHostMalloc(&h, B, hipHostMallocDefault);
  (void)hipHostMalloc(&h2, B, hipHostMallocDefault);
  (void)hipMalloc(&d, B);
  (void)hipMalloc(&d2, B);
  (void)hipHostGetDevicePointer(&hd, h, 0);
  hipStream_t s1, s2;
  (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  (void)hipMemset(d, 1, B);
  for (int rep = 0; rep < 2; ++rep) {
    double t = now();
    for (int i = 0; i < 8; ++i) (void)hipMemcpyAsync(d, h, B, hipMemcpyHostToDevice, s1);
    (void)hipStreamSynchronize(s1);
    const double h2d = 8.0 * B / (now() - t) / 1e9;
    t = now();
    for (int i = 0; i < 8; ++i) (void)hipMemcpyAsync(h, d, B, hipMemcpyDeviceToHost, s1);
    (void)hipStreamSynchronize(s1);
    const double d2h = 8.0 * B / (now() - t) / 1e9;
    t = now();
    for (int i = 0; i < 8; ++i) {
      (void)hipMemcpyAsync(h, d, B / 2, hipMemcpyDeviceToHost, s1);
      (void)hipMemcpyAsync((char*)h2 + B / 2, (char*)d + B / 2, B / 2, hipMemcpyDeviceToHost, s2);
    }
    (void)hipStreamSynchronize(s1);
    (void)hipStreamSynchronize(s2);
    const double d2h2 = 8.0 * B / (now() - t) / 1e9;
    t = now();
    for (int i = 0; i < 8; ++i) {
      (void)hipMemcpyAsync(d2, h2, B, hipMemcpyHostToDevice, s2);
      (void)hipMemcpyAsync(h, d, B, hipMemcpyDeviceToHost, s1);
    }
    (void)hipStreamSynchronize(s1);
    (void)hipStreamSynchronize(s2);
    const double both = 16.0 * B / (now() - t) / 1e9;
    t = now();
    for (int i = 0; i < 8; ++i)
      hipLaunchKernelGGL(k_store, dim3(1024), dim3(256), 0, s1, (uint4*)hd, (const uint4*)d, B / 16);
    (void)hipStreamSynchronize(s1);
    const double kst = 8.0 * B / (now() - t) / 1e9;
    printf("H2D %.1f GB/s | D2H %.1f GB/s | D2H on 2 streams %.1f GB/s | H2D+D2H together %.1f GB/s | "
           "kernel stores to pinned %.1f GB/s\n", h2d, d2h, d2h2, both, kst);
  }
  return 0;
}
