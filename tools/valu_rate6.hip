// valu_rate6.hip — issue cost of VCC-reading e32 v_cndmask runs (one compare, several selects) against
// the e64 form, and of a VALU op under a half-wave exec mask (diagnostic only; 8 waves per SIMD):
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate6.hip -o build/valu_rate6 && build/valu_rate6
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int ITERS = 256;
#define BODY8(ins) ins "\n" ins "\n" ins "\n" ins "\n" ins "\n" ins "\n" ins "\n" ins
#define KERNEL(name, init, ins, clob...)                                                   \
  __global__ void __launch_bounds__(256) name(float* out) {                              \
    asm volatile(init ::: clob);                                                         \
    for (int i = 0; i < ITERS; ++i) asm volatile(BODY8(ins) ::: clob);                   \
    asm volatile("s_mov_b64 exec, -1" ::: "exec");                                       \
  }
#define INIT "v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v10, 3.0\n v_cmp_lt_f32 vcc, v8, v9\n v_cmp_lt_f32 s[20:21], v8, v9"
#define CL "v8", "v9", "v10", "v14", "v15", "v16", "vcc", "s20", "s21", "exec", "memory"
KERNEL(k_add, INIT, "v_add_f32 v14, v8, v9", CL)
KERNEL(k_cmp3cnd, INIT, "v_cmp_lt_f32 vcc, v8, v9\n s_nop 1\n v_cndmask_b32 v14, v8, v9, vcc\n v_cndmask_b32 v15, v8, v10, vcc\n v_cndmask_b32 v16, v9, v10, vcc", CL)
KERNEL(k_cmp3cnd64, INIT, "v_cmp_lt_f32_e64 s[20:21], v8, v9\n s_nop 1\n v_cndmask_b32_e64 v14, v8, v9, s[20:21]\n v_cndmask_b32_e64 v15, v8, v10, s[20:21]\n v_cndmask_b32_e64 v16, v9, v10, s[20:21]", CL)
KERNEL(k_cmpnop1cnd, INIT, "v_cmp_lt_f32 vcc, v8, v9\n s_nop 1\n v_cndmask_b32 v14, v8, v9, vcc", CL)
KERNEL(k_cnd_then_add, INIT, "v_cndmask_b32 v14, v8, v9, vcc\n v_add_f32 v15, v8, v9", CL)
KERNEL(k_add_half, INIT "\n s_mov_b32 exec_hi, 0", "v_add_f32 v14, v8, v9", CL)
KERNEL(k_add_lo0, INIT "\n s_mov_b32 exec_lo, 0", "v_add_f32 v14, v8, v9", CL)
KERNEL(k_madu64_half, INIT "\n s_mov_b32 exec_hi, 0", "v_mad_u64_u32 v[14:15], s[20:21], v8, v9, 0", CL)
KERNEL(k_madu64, INIT, "v_mad_u64_u32 v[14:15], s[20:21], v8, v9, 0", CL)

int main() {
  float* out;
  (void)hipMalloc(&out, 4);
  struct K { const char* n; void (*f)(float*); } ks[] = {
      {"v_add_f32", k_add},
      {"v_cmp vcc + s_nop 1 + 3 x v_cndmask vcc (group)", k_cmp3cnd},
      {"v_cmp s[] + s_nop 1 + 3 x v_cndmask_e64 s[] (group)", k_cmp3cnd64},
      {"v_cmp vcc + s_nop 1 + v_cndmask vcc (group)", k_cmpnop1cnd},
      {"v_cndmask vcc + v_add_f32 (group)", k_cnd_then_add},
      {"v_add_f32, exec_hi = 0", k_add_half},
      {"v_add_f32, exec_lo = 0", k_add_lo0},
      {"v_mad_u64_u32", k_madu64},
      {"v_mad_u64_u32, exec_hi = 0", k_madu64_half}};
  const int blocks = 256 * 8;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (auto& k : ks) {
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out);
    (void)hipEventRecord(a);
    for (int rep = 0; rep < 10; ++rep) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double per_simd = 10.0 * blocks * 4 * ITERS * 8 / 1024.0;
    const double ns = ms * 1e6 / per_simd;
    printf("%-52s %.3f ns per (group of) instruction(s) per SIMD (%.1f cyc @2.4GHz)\n", k.n, ns, ns * 2.4);
    fflush(stdout);
  }
  return 0;
}
