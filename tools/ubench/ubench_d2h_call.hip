// Host time per hipMemcpyAsync device-to-host call and the copy rate, for the host pipeline's per-slot output
// copies: 3-MB copies (one config-2 batch's results and tape) from HBM into hipHostMalloc'd memory, with and
// without a compute kernel writing HBM beside them on another stream.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_busy(uint4* __restrict__ p, size_t n, int reps) {
  for (int r = 0; r < reps; ++r)
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
      p[i] = make_uint4(p[i].x + 1, p[i].y, p[i].z, r);
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t B = 3u << 20, N = 64;
  void *h, *d, *w;
  (void)hipHostMalloc(&h, B * N, hipHostMallocDefault);
  (void)hipMalloc(&d, B * N);
  (void)hipMalloc(&w, 256u << 20);
  hipStream_t s1, s2;
  (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  (void)hipMemset(d, 1, B * N);
  for (int busy = 0; busy < 2; ++busy) {
    for (int rep = 0; rep < 2; ++rep) {
      if (busy) hipLaunchKernelGGL(k_busy, dim3(1024), dim3(256), 0, s2, (uint4*)w, (256u << 20) / 16, 40);
      const double t = now();
      double host = 0;
      for (size_t i = 0; i < N; ++i) {
        const double a = now();
        (void)hipMemcpyAsync((char*)h + i * B, (char*)d + i * B, B, hipMemcpyDeviceToHost, s1);
        host += now() - a;
      }
      (void)hipStreamSynchronize(s1);
      const double dt = now() - t;
      (void)hipStreamSynchronize(s2);
      printf("busy %d: %zu copies of 3 MB: host %.1f us per call, %.1f GB/s\n", busy, N, host / N * 1e6,
             (double)B * N / dt / 1e9);
    }
  }
  return 0;
}
