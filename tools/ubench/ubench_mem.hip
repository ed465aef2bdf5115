// Single-wave global-memory latencies on gfx950: does a store issued before a load lengthen the
// wait for that load (loads and stores share vmcnt on this family)?
//   chase        x = p[x]                        (L2-resident pointer chase)
//   store+chase  q[i] = x; x = p[x]              (one store ahead of every dependent load)
//   chase+store  y = p[x]; q[i] = x; x = y       (the store issued after the load)
//   4st+chase    four stores ahead of every load
// cycles per iteration from s_memtime, one wave, 4096 iterations after a warm pass.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 1 << 14;  // 64 KB chain
constexpr int IT = 4096;

template <int MODE>
__global__ void k_mem(const int* __restrict__ p, int* __restrict__ q, unsigned long long* out) {
  int x = threadIdx.x;
  for (int i = 0; i < IT; ++i) x = p[x];  // warm
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < IT; ++i) {
    if (MODE == 0) {
      x = p[x];
    } else if (MODE == 1) {
      q[(i * 64 + threadIdx.x) & (N - 1)] = x;
      x = p[x];
    } else if (MODE == 2) {
      const int y = p[x];
      q[(i * 64 + threadIdx.x) & (N - 1)] = x;
      x = y;
    } else {
      for (int k = 0; k < 4; ++k) q[((i * 4 + k) * 64 + threadIdx.x) & (N - 1)] = x + k;
      x = p[x];
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = (unsigned long long)x;
  }
}

int main() {
  int *p, *q;
  unsigned long long* o;
  (void)hipMalloc(&p, N * sizeof(int));
  (void)hipMalloc(&q, N * sizeof(int));
  (void)hipMalloc(&o, 64);
  int* h = new int[N];
  for (int i = 0; i < N; ++i) h[i] = (i + 97 * 32) % N;  // stride of 97 lines
  (void)hipMemcpy(p, h, N * sizeof(int), hipMemcpyHostToDevice);
  const char* names[] = {"chase", "store+chase", "chase+store", "4st+chase"};
  void (*ks[])(const int*, int*, unsigned long long*) = {k_mem<0>, k_mem<1>, k_mem<2>, k_mem<3>};
  for (int m = 0; m < 4; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(ks[m], dim3(1), dim3(64), 0, 0, p, q, o);
      (void)hipDeviceSynchronize();
    }
    unsigned long long r[2];
    (void)hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
    printf("%-12s %8.1f cycles/iter\n", names[m], (double)r[0] / IT);
  }
  return 0;
}
