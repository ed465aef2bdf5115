// Single-wave instruction latency microbenchmarks on gfx950 (one wave per SIMD, like k_match_reg):
// s_memtime cycles per iteration of small dependent chains. Every loop lives inside one asm block
// (its own counter and branch), so the compiler's code never sees the clobbered SCC / exec.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 1024
#define LOOP_BEGIN "s_movk_i32 %[cnt], " "1024" "\n 9:\n"
#define LOOP_END "s_sub_u32 %[cnt], %[cnt], 1\n s_cmp_lg_u32 %[cnt], 0\n s_cbranch_scc1 9b\n"

#define KERNEL(name, body, ...)                                       \
  __global__ void name(unsigned long long* out, int n) {                          \
    int v = threadIdx.x + n, t = 0, s = 3, cnt;                                    \
    __shared__ int buf[256];                                                       \
    buf[threadIdx.x] = 0;                                                          \
    __syncthreads();                                                               \
    int a = threadIdx.x * 4;                                                       \
    unsigned long long t0 = __builtin_amdgcn_s_memtime();                          \
    asm volatile(LOOP_BEGIN body LOOP_END __VA_ARGS__);                \
    unsigned long long t1 = __builtin_amdgcn_s_memtime();                          \
    if (threadIdx.x == 0) {                                                        \
      out[blockIdx.x * 4 + 0] = t1 - t0;                                           \
      out[blockIdx.x * 4 + 1] = v + t + s + a;                                     \
    }                                                                              \
  }

KERNEL(k_empty, "", : [cnt] "=&s"(cnt) : : "scc")
KERNEL(k_salu, "s_add_u32 %[s], %[s], 1\n s_add_u32 %[s], %[s], 1\n s_add_u32 %[s], %[s], 1\n s_add_u32 %[s], %[s], 1\n",
       : [cnt] "=&s"(cnt), [s] "+s"(s) : : "scc")
KERNEL(k_valu, "v_add_u32 %[v], %[v], 1\n v_add_u32 %[v], %[v], 1\n v_add_u32 %[v], %[v], 1\n v_add_u32 %[v], %[v], 1\n",
       : [cnt] "=&s"(cnt), [v] "+v"(v) : : "scc")
KERNEL(k_pingpong, "v_readfirstlane_b32 %[s], %[v]\n s_add_u32 %[s], %[s], 1\n v_add_u32 %[v], %[s], %[v]\n",
       : [cnt] "=&s"(cnt), [v] "+v"(v), [s] "+s"(s) : : "scc")
KERNEL(k_exec, "v_cmp_gt_u32 vcc, 16, %[v]\n s_and_saveexec_b64 s[20:21], vcc\n v_add_u32 %[v], 1, %[v]\n s_or_b64 exec, exec, s[20:21]\n",
       : [cnt] "=&s"(cnt), [v] "+v"(v) : : "scc", "vcc", "s20", "s21")
KERNEL(k_lds, "ds_read_b32 %[a], %[a]\n s_waitcnt lgkmcnt(0)\n v_add_u32 %[a], %[a], %[a]\n",
       : [cnt] "=&s"(cnt), [a] "+v"(a) : : "scc", "memory")
KERNEL(k_branch, "s_add_u32 %[s], %[s], 1\n s_branch 1f\n s_nop 0\n s_nop 0\n 1:\n s_add_u32 %[s], %[s], 1\n s_branch 2f\n s_nop 0\n 2:\n",
       : [cnt] "=&s"(cnt), [s] "+s"(s) : : "scc")
KERNEL(k_nbranch, "s_cmp_eq_u32 %[s], 12345\n s_cbranch_scc1 1f\n s_add_u32 %[s], %[s], 1\n s_cmp_eq_u32 %[s], 12345\n s_cbranch_scc1 1f\n s_add_u32 %[s], %[s], 1\n 1:\n",
       : [cnt] "=&s"(cnt), [s] "+s"(s) : : "scc")
KERNEL(k_readlane, "v_readlane_b32 %[s], %[v], %[s]\n s_and_b32 %[s], %[s], 63\n",
       : [cnt] "=&s"(cnt), [v] "+v"(v), [s] "+s"(s) : : "scc")
KERNEL(k_dpp, "s_nop 1\n v_mov_b32_dpp %[t], %[v] row_shr:1 bound_ctrl:0\n v_add_u32 %[v], %[v], %[t]\n",
       : [cnt] "=&s"(cnt), [v] "+v"(v), [t] "+v"(t) : : "scc")
KERNEL(k_nop, "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n", : [cnt] "=&s"(cnt) : : "scc")
KERNEL(k_vcmp_sgpr, "v_cmp_gt_u32 s[20:21], %[v], 5\n s_bcnt1_i32_b64 %[s], s[20:21]\n v_add_u32 %[v], %[s], %[v]\n",
       : [cnt] "=&s"(cnt), [v] "+v"(v), [s] "+s"(s) : : "scc", "s20", "s21")

int main() {
  unsigned long long* d;
  (void)hipMalloc(&d, 4096 * 32);
  unsigned long long h[4096 * 4];
  struct K { const char* name; void (*f)(unsigned long long*, int); };
  K ks[] = {{"empty loop", k_empty}, {"4 dep salu", k_salu}, {"4 dep valu", k_valu},
            {"readfirstlane->salu->valu", k_pingpong}, {"vcmp+saveexec+valu+restore", k_exec},
            {"lds dep read+wait+valu", k_lds}, {"2 taken branches + 2 salu", k_branch},
            {"2 not-taken cbr + 4 salu", k_nbranch}, {"readlane(sidx)->salu", k_readlane},
            {"nop+dpp mov+add", k_dpp}, {"4 s_nop 0", k_nop}, {"vcmp->sgpr->bcnt->valu", k_vcmp_sgpr}};
  for (auto& k : ks) {
    printf("%-30s", k.name);
    fflush(stdout);
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(k.f, dim3(256), dim3(64), 0, 0, d, 1);
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, d, 256 * 4 * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int b = 0; b < 256; ++b) s += h[b * 4];
    printf(" %8.2f cycles per iteration\n", s / 256 / REP);
    fflush(stdout);
  }
  return 0;
}
