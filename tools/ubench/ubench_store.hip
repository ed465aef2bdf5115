// Single-wave store throughput on gfx950: how many cycles does a chain of fire-and-forget global
// stores cost when nothing waits for them (the hot-symbol path's write-through pattern)?
//   MODE 0  ALU only (the loop's own cost)
//   MODE 1  one 4-B store per iteration, lane 0, a new line each time
//   MODE 2  four 4-B stores per iteration, lane 0, new lines
//   MODE 3  the hot-path record mix: 2 x 16-B stores over 16 lanes (fills), a 4-B store over 16 lanes,
//           16-B + 1-B + 8-B + 4-B stores from lane 0, all to new lines
//   MODE 4  MODE 3 aimed at the same few lines every iteration (a hot level)
// cycles per iteration from s_memtime, one wave, IT iterations after a warm pass.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int IT = 8192;
constexpr size_t LINES = 1 << 20;  // 128 MB of 128-B lines

template <int MODE>
__global__ void k_store(unsigned char* __restrict__ q, unsigned long long* out) {
  const int lane = threadIdx.x;
  unsigned long long acc = lane;
  auto line = [&](int i, int k) -> unsigned char* {
    const size_t l = MODE == 4 ? (size_t)(k * 7) : ((size_t)i * 8 + k) * 97 % LINES;
    return q + l * 128;
  };
  unsigned long long t0 = 0;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < IT; ++i) {
      acc = acc * 6364136223846793005ull + 1442695040888963407ull;
      if (MODE == 1) {
        if (lane == 0) *(unsigned*)line(i, 0) = (unsigned)acc;
      } else if (MODE == 2) {
        if (lane == 0)
          for (int k = 0; k < 4; ++k) *(unsigned*)line(i, k) = (unsigned)acc + k;
      } else if (MODE >= 3) {
        if (lane < 16) {
          uint4* f = (uint4*)line(i, 0) + lane * 2;
          f[0] = make_uint4((unsigned)acc, 1, 2, 3);
          f[1] = make_uint4(4, 5, 6, (unsigned)acc);
          ((unsigned*)line(i, 1))[lane] = (unsigned)acc;
        }
        if (lane == 0) {
          *(uint4*)line(i, 2) = make_uint4((unsigned)acc, 0, 0, 1);
          *line(i, 3) = (unsigned char)acc;
          *(unsigned long long*)line(i, 4) = acc;
          *(unsigned*)line(i, 5) = (unsigned)acc;
        }
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_waitcnt(0);
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = acc;
  }
}

template <int MODE>
static void run(unsigned char* q, unsigned long long* o, const char* name, int waves) {
  hipLaunchKernelGGL(k_store<MODE>, dim3(waves), dim3(64), 0, 0, q, o);
  (void)hipDeviceSynchronize();
  unsigned long long h[2];
  (void)hipMemcpy(h, o, 16, hipMemcpyDeviceToHost);
  printf("%-28s waves=%3d  %8.1f cycles/iteration\n", name, waves, (double)h[0] / IT);
}

int main() {
  unsigned char* q;
  unsigned long long* o;
  (void)hipMalloc(&q, LINES * 128);
  (void)hipMalloc(&o, 64);
  (void)hipMemset(q, 0, LINES * 128);
  for (int w : {1, 16}) {
    run<0>(q, o, "alu only", w);
    run<1>(q, o, "1 store, new line", w);
    run<2>(q, o, "4 stores, new lines", w);
    run<3>(q, o, "record mix, new lines", w);
    run<4>(q, o, "record mix, same lines", w);
  }
  return 0;
}
