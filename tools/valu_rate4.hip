// valu_rate4.hip — issue cost per SIMD of the encodings the step kernels lean on, at full
// occupancy (8 waves per SIMD), relative to v_add_f32 (diagnostic only):
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate4.hip -o build/valu_rate4 && build/valu_rate4
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int ITERS = 256;
#define BODY8(ins) ins "\n" ins "\n" ins "\n" ins "\n" ins "\n" ins "\n" ins "\n" ins
#define KERNEL(name, init, ins, clob...)                                                   \
  __global__ void __launch_bounds__(256) name(float* out) {                              \
    asm volatile(init ::: clob);                                                         \
    for (int i = 0; i < ITERS; ++i) asm volatile(BODY8(ins) ::: clob);                   \
  }
#define INIT "v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v10, 3.0\n v_mov_b32 v11, 1.5\n v_mov_b32 v12, 7\n v_mov_b32 v13, 9"
#define CL "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "vcc", "s20", "s21"
KERNEL(k_add, INIT, "v_add_f32 v14, v8, v9", CL)
KERNEL(k_sqrt, INIT, "v_sqrt_f32 v14, v8", CL)
KERNEL(k_rcp, INIT, "v_rcp_f32 v14, v8", CL)
KERNEL(k_mad64, INIT, "v_mad_u64_u32 v[14:15], s[20:21], v12, v13, 0", CL)
KERNEL(k_mulhi, INIT, "v_mul_hi_u32 v14, v12, v13", CL)
KERNEL(k_mullo, INIT, "v_mul_lo_u32 v14, v12, v13", CL)
KERNEL(k_mul24, INIT, "v_mul_u32_u24 v14, v12, v13", CL)
KERNEL(k_addf64, INIT, "v_add_f64 v[14:15], v[8:9], v[10:11]", CL)
KERNEL(k_fmaf64, INIT, "v_fma_f64 v[14:15], v[8:9], v[10:11], v[8:9]", CL)
KERNEL(k_cvtf64, INIT, "v_cvt_f64_f32 v[14:15], v8", CL)
KERNEL(k_cvtf32, INIT, "v_cvt_f32_f64 v14, v[8:9]", CL)
KERNEL(k_med3u, INIT, "v_med3_u32 v14, v12, v13, v8", CL)
KERNEL(k_pkadd, INIT, "v_pk_add_f32 v[14:15], v[8:9], v[10:11]", CL)
KERNEL(k_pkfma, INIT, "v_pk_fma_f32 v[14:15], v[8:9], v[10:11], v[8:9]", CL)
KERNEL(k_dpp, INIT, "v_add_f32_dpp v14, v8, v9 wave_ror:1 row_mask:0xf bank_mask:0xf", CL)
KERNEL(k_cndmask, INIT, "v_cndmask_b32 v14, v8, v9, vcc", CL)
KERNEL(k_sqrtf64, INIT, "v_sqrt_f64 v[14:15], v[8:9]", CL)

int main() {
  float* out;
  hipMalloc(&out, 4);
  struct K { const char* n; void (*f)(float*); } ks[] = {
      {"v_add_f32", k_add}, {"v_sqrt_f32", k_sqrt}, {"v_rcp_f32", k_rcp}, {"v_mad_u64_u32", k_mad64},
      {"v_mul_hi_u32", k_mulhi}, {"v_mul_lo_u32", k_mullo}, {"v_mul_u32_u24", k_mul24},
      {"v_add_f64", k_addf64}, {"v_fma_f64", k_fmaf64}, {"v_cvt_f64_f32", k_cvtf64}, {"v_cvt_f32_f64", k_cvtf32},
      {"v_med3_u32", k_med3u}, {"v_pk_add_f32", k_pkadd}, {"v_pk_fma_f32", k_pkfma}, {"v_add_f32_dpp", k_dpp},
      {"v_cndmask_b32", k_cndmask}, {"v_sqrt_f64", k_sqrtf64}};
  const int blocks = 256 * 8;  // 8 waves per SIMD at 4 waves per workgroup
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  double base = 0;
  for (auto& k : ks) {
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out);
    hipEventRecord(a);
    for (int rep = 0; rep < 10; ++rep) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    // wave-instructions per SIMD: blocks*4 waves * ITERS*8 / 1024 SIMDs, 10 launches
    const double per_simd = 10.0 * blocks * 4 * ITERS * 8 / 1024.0;
    const double ns = ms * 1e6 / per_simd;
    if (base == 0) base = ns;
    printf("%-16s %.3f ns per wave-instruction per SIMD  (%.2fx v_add_f32; %.1f cyc @2.4GHz)\n", k.n, ns, ns / base,
           ns * 2.4);
  }
  return 0;
}
