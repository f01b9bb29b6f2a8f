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
KERNEL(k_minf, INIT, "v_min_f32 v14, v8, v9", CL)
KERNEL(k_maxf, INIT, "v_max_f32 v14, v8, v9", CL)
KERNEL(k_med3f, INIT, "v_med3_f32 v14, v8, v9, v10", CL)
KERNEL(k_min3f, INIT, "v_min3_f32 v14, v8, v9, v10", CL)
KERNEL(k_minu, INIT, "v_min_u32 v14, v12, v13", CL)
KERNEL(k_fmaf, INIT, "v_fma_f32 v14, v8, v9, v10", CL)
KERNEL(k_mulf, INIT, "v_mul_f32 v14, v8, v9", CL)
KERNEL(k_subf, INIT, "v_sub_f32 v14, v8, v9", CL)
KERNEL(k_addabs, INIT, "v_add_f32_e64 v14, |v8|, v9", CL)
KERNEL(k_andor, INIT, "v_and_or_b32 v14, v12, v13, v8", CL)
KERNEL(k_and, INIT, "v_and_b32 v14, v12, v13", CL)
KERNEL(k_or, INIT, "v_or_b32 v14, v12, v13", CL)
KERNEL(k_bfi, INIT, "v_bfi_b32 v14, v12, v13, v8", CL)
KERNEL(k_addu, INIT, "v_add_u32 v14, v12, v13", CL)
KERNEL(k_xor, INIT, "v_xor_b32 v14, v12, v13", CL)
KERNEL(k_mov, INIT, "v_mov_b32 v14, v12", CL)
KERNEL(k_cmpf, INIT, "v_cmp_lt_f32 vcc, v8, v9", CL)
KERNEL(k_cnd64, INIT, "v_cndmask_b32_e64 v14, v8, v9, s[20:21]", CL)
KERNEL(k_cvtfi, INIT, "v_cvt_f32_u32 v14, v12", CL)
KERNEL(k_pkmul, INIT, "v_pk_mul_f32 v[14:15], v[8:9], v[10:11]", CL)
KERNEL(k_fmac, INIT, "v_fmac_f32 v14, v8, v9", CL)
KERNEL(k_ldexp, INIT, "v_ldexp_f32 v14, v8, v12", CL)
KERNEL(k_mulhif, INIT, "v_mul_hi_u32_u24 v14, v12, v13", CL)
KERNEL(k_lshl, INIT, "v_lshlrev_b32 v14, 2, v12", CL)
KERNEL(k_addf_dep, INIT, "v_add_f32 v14, v14, v9", CL)
KERNEL(k_med3u_dep, INIT, "v_med3_u32 v14, v14, v13, v8", CL)
KERNEL(k_med3f_dep, INIT, "v_med3_f32 v14, v14, v9, v10", CL)

int main() {
  float* out;
  hipMalloc(&out, 4);
  struct K { const char* n; void (*f)(float*); } ks[] = {
      {"v_add_f32", k_add}, {"v_sqrt_f32", k_sqrt}, {"v_rcp_f32", k_rcp}, {"v_mad_u64_u32", k_mad64},
      {"v_mul_hi_u32", k_mulhi}, {"v_mul_lo_u32", k_mullo}, {"v_mul_u32_u24", k_mul24},
      {"v_add_f64", k_addf64}, {"v_fma_f64", k_fmaf64}, {"v_cvt_f64_f32", k_cvtf64}, {"v_cvt_f32_f64", k_cvtf32},
      {"v_med3_u32", k_med3u}, {"v_pk_add_f32", k_pkadd}, {"v_pk_fma_f32", k_pkfma}, {"v_add_f32_dpp", k_dpp},
      {"v_cndmask_b32", k_cndmask}, {"v_sqrt_f64", k_sqrtf64},
      {"v_min_f32", k_minf}, {"v_max_f32", k_maxf}, {"v_med3_f32", k_med3f}, {"v_min3_f32", k_min3f},
      {"v_min_u32", k_minu}, {"v_fma_f32", k_fmaf}, {"v_mul_f32", k_mulf}, {"v_sub_f32", k_subf},
      {"v_add_f32 |a|", k_addabs}, {"v_and_or_b32", k_andor}, {"v_and_b32", k_and}, {"v_or_b32", k_or},
      {"v_bfi_b32", k_bfi}, {"v_add_u32", k_addu}, {"v_xor_b32", k_xor}, {"v_mov_b32", k_mov},
      {"v_cmp_lt_f32", k_cmpf}, {"v_cndmask_e64 s", k_cnd64}, {"v_cvt_f32_u32", k_cvtfi}, {"v_pk_mul_f32", k_pkmul},
      {"v_fmac_f32", k_fmac}, {"v_ldexp_f32", k_ldexp}, {"v_mul_hi_u32_u24", k_mulhif}, {"v_lshlrev_b32", k_lshl},
      {"v_add_f32 dep", k_addf_dep}, {"v_med3_u32 dep", k_med3u_dep}, {"v_med3_f32 dep", k_med3f_dep}};
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
