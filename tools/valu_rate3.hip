// valu_rate3.hip — issue cost per SIMD of more VALU encodings (diagnostic only)
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int ITERS = 2048;
__global__ void __launch_bounds__(64) k0(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_min_f32_e32 v10, v10, v8\nv_min_f32_e32 v11, v11, v8\nv_min_f32_e32 v12, v12, v8\nv_min_f32_e32 v13, v13, v8\nv_min_f32_e32 v14, v14, v8\nv_min_f32_e32 v15, v15, v8\nv_min_f32_e32 v16, v16, v8\nv_min_f32_e32 v17, v17, v8" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k1(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_max_f32_e32 v10, v10, v8\nv_max_f32_e32 v11, v11, v8\nv_max_f32_e32 v12, v12, v8\nv_max_f32_e32 v13, v13, v8\nv_max_f32_e32 v14, v14, v8\nv_max_f32_e32 v15, v15, v8\nv_max_f32_e32 v16, v16, v8\nv_max_f32_e32 v17, v17, v8" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k2(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_med3_f32 v10, v10, v8, v9\nv_med3_f32 v11, v11, v8, v9\nv_med3_f32 v12, v12, v8, v9\nv_med3_f32 v13, v13, v8, v9\nv_med3_f32 v14, v14, v8, v9\nv_med3_f32 v15, v15, v8, v9\nv_med3_f32 v16, v16, v8, v9\nv_med3_f32 v17, v17, v8, v9" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k3(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_mul_f32_e32 v10, v10, v8\nv_mul_f32_e32 v11, v11, v8\nv_mul_f32_e32 v12, v12, v8\nv_mul_f32_e32 v13, v13, v8\nv_mul_f32_e32 v14, v14, v8\nv_mul_f32_e32 v15, v15, v8\nv_mul_f32_e32 v16, v16, v8\nv_mul_f32_e32 v17, v17, v8" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k4(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_and_b32_e32 v10, v10, v8\nv_and_b32_e32 v11, v11, v8\nv_and_b32_e32 v12, v12, v8\nv_and_b32_e32 v13, v13, v8\nv_and_b32_e32 v14, v14, v8\nv_and_b32_e32 v15, v15, v8\nv_and_b32_e32 v16, v16, v8\nv_and_b32_e32 v17, v17, v8" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k5(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_lshlrev_b32_e32 v10, 2, v10\nv_lshlrev_b32_e32 v11, 2, v11\nv_lshlrev_b32_e32 v12, 2, v12\nv_lshlrev_b32_e32 v13, 2, v13\nv_lshlrev_b32_e32 v14, 2, v14\nv_lshlrev_b32_e32 v15, 2, v15\nv_lshlrev_b32_e32 v16, 2, v16\nv_lshlrev_b32_e32 v17, 2, v17" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k6(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_add_u32_e32 v10, v10, v8\nv_add_u32_e32 v11, v11, v8\nv_add_u32_e32 v12, v12, v8\nv_add_u32_e32 v13, v13, v8\nv_add_u32_e32 v14, v14, v8\nv_add_u32_e32 v15, v15, v8\nv_add_u32_e32 v16, v16, v8\nv_add_u32_e32 v17, v17, v8" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k7(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_max_u32_e32 v10, v10, v8\nv_max_u32_e32 v11, v11, v8\nv_max_u32_e32 v12, v12, v8\nv_max_u32_e32 v13, v13, v8\nv_max_u32_e32 v14, v14, v8\nv_max_u32_e32 v15, v15, v8\nv_max_u32_e32 v16, v16, v8\nv_max_u32_e32 v17, v17, v8" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k8(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_min_i32_e32 v10, v10, v8\nv_min_i32_e32 v11, v11, v8\nv_min_i32_e32 v12, v12, v8\nv_min_i32_e32 v13, v13, v8\nv_min_i32_e32 v14, v14, v8\nv_min_i32_e32 v15, v15, v8\nv_min_i32_e32 v16, v16, v8\nv_min_i32_e32 v17, v17, v8" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k9(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_sub_f32_e32 v10, v10, v8\nv_sub_f32_e32 v11, v11, v8\nv_sub_f32_e32 v12, v12, v8\nv_sub_f32_e32 v13, v13, v8\nv_sub_f32_e32 v14, v14, v8\nv_sub_f32_e32 v15, v15, v8\nv_sub_f32_e32 v16, v16, v8\nv_sub_f32_e32 v17, v17, v8" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k10(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_cvt_f32_f64_e32 v10, v[4:5]\nv_cvt_f32_f64_e32 v11, v[4:5]\nv_cvt_f32_f64_e32 v12, v[4:5]\nv_cvt_f32_f64_e32 v13, v[4:5]\nv_cvt_f32_f64_e32 v14, v[4:5]\nv_cvt_f32_f64_e32 v15, v[4:5]\nv_cvt_f32_f64_e32 v16, v[4:5]\nv_cvt_f32_f64_e32 v17, v[4:5]" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k11(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_mul_f64 v[20:21], v[20:21], v[4:5]\nv_mul_f64 v[22:23], v[22:23], v[4:5]\nv_mul_f64 v[24:25], v[24:25], v[4:5]\nv_mul_f64 v[26:27], v[26:27], v[4:5]\nv_mul_f64 v[20:21], v[20:21], v[4:5]\nv_mul_f64 v[22:23], v[22:23], v[4:5]\nv_mul_f64 v[24:25], v[24:25], v[4:5]\nv_mul_f64 v[26:27], v[26:27], v[4:5]" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k12(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_fma_f64 v[20:21], v[20:21], v[4:5], v[4:5]\nv_fma_f64 v[22:23], v[22:23], v[4:5], v[4:5]\nv_fma_f64 v[24:25], v[24:25], v[4:5], v[4:5]\nv_fma_f64 v[26:27], v[26:27], v[4:5], v[4:5]\nv_fma_f64 v[20:21], v[20:21], v[4:5], v[4:5]\nv_fma_f64 v[22:23], v[22:23], v[4:5], v[4:5]\nv_fma_f64 v[24:25], v[24:25], v[4:5], v[4:5]\nv_fma_f64 v[26:27], v[26:27], v[4:5], v[4:5]" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k13(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_rsq_f32 v10, v10\nv_rsq_f32 v11, v11\nv_rsq_f32 v12, v12\nv_rsq_f32 v13, v13\nv_rsq_f32 v14, v14\nv_rsq_f32 v15, v15\nv_rsq_f32 v16, v16\nv_rsq_f32 v17, v17" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k14(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_cmp_lt_f32_e32 vcc, v10, v8\n v_cndmask_b32_e32 v10, v10, v8, vcc\nv_cmp_lt_f32_e32 vcc, v11, v8\n v_cndmask_b32_e32 v11, v11, v8, vcc\nv_cmp_lt_f32_e32 vcc, v12, v8\n v_cndmask_b32_e32 v12, v12, v8, vcc\nv_cmp_lt_f32_e32 vcc, v13, v8\n v_cndmask_b32_e32 v13, v13, v8, vcc\nv_cmp_lt_f32_e32 vcc, v14, v8\n v_cndmask_b32_e32 v14, v14, v8, vcc\nv_cmp_lt_f32_e32 vcc, v15, v8\n v_cndmask_b32_e32 v15, v15, v8, vcc\nv_cmp_lt_f32_e32 vcc, v16, v8\n v_cndmask_b32_e32 v16, v16, v8, vcc\nv_cmp_lt_f32_e32 vcc, v17, v8\n v_cndmask_b32_e32 v17, v17, v8, vcc" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k15(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_pk_min_u16 v10, v10, v8\nv_pk_min_u16 v11, v11, v8\nv_pk_min_u16 v12, v12, v8\nv_pk_min_u16 v13, v13, v8\nv_pk_min_u16 v14, v14, v8\nv_pk_min_u16 v15, v15, v8\nv_pk_min_u16 v16, v16, v8\nv_pk_min_u16 v17, v17, v8" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
__global__ void __launch_bounds__(64) k16(float* out) {
  asm volatile("v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n s_mov_b64 vcc, -1\n s_mov_b64 s[20:21], -1" ::: "v4","v5","v8","v9","vcc","s20","s21");
  for (int i = 0; i < ITERS; ++i) asm volatile("v_max3_f32 v10, v10, v8, v9\nv_max3_f32 v11, v11, v8, v9\nv_max3_f32 v12, v12, v8, v9\nv_max3_f32 v13, v13, v8, v9\nv_max3_f32 v14, v14, v8, v9\nv_max3_f32 v15, v15, v8, v9\nv_max3_f32 v16, v16, v8, v9\nv_max3_f32 v17, v17, v8, v9" ::: "v4","v5","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v20","v21","v22","v23","v24","v25","v26","v27","vcc","s22");
}
template <typename F> void run(const char* name, F f, float* out, int cus) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  printf("%-10s", name);
  for (int w = 1; w <= 8; w *= 2) {
    hipLaunchKernelGGL(f, dim3(cus*4*w), dim3(64), 0, 0, out);
    (void)hipEventRecord(a); hipLaunchKernelGGL(f, dim3(cus*4*w), dim3(64), 0, 0, out); (void)hipEventRecord(b);
    (void)hipEventSynchronize(b); float ms; (void)hipEventElapsedTime(&ms, a, b);
    printf("  w%d %6.3f", w, ms * 1e6 / ((double)w * ITERS * 8));
  }
  printf("  ns/instr/SIMD\n");
}

int main() { hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, 0); float* out; (void)hipMalloc(&out, 4096);
  run("min_f32", k0, out, p.multiProcessorCount);
  run("max_f32", k1, out, p.multiProcessorCount);
  run("med3_f32", k2, out, p.multiProcessorCount);
  run("mul_f32", k3, out, p.multiProcessorCount);
  run("and_b32", k4, out, p.multiProcessorCount);
  run("lshlrev", k5, out, p.multiProcessorCount);
  run("add_u32", k6, out, p.multiProcessorCount);
  run("max_u32", k7, out, p.multiProcessorCount);
  run("min_i32", k8, out, p.multiProcessorCount);
  run("sub_f32", k9, out, p.multiProcessorCount);
  run("cvt_f32_f64", k10, out, p.multiProcessorCount);
  run("mul_f64", k11, out, p.multiProcessorCount);
  run("fma_f64", k12, out, p.multiProcessorCount);
  run("rsq", k13, out, p.multiProcessorCount);
  run("cmp_cnd", k14, out, p.multiProcessorCount);
  run("min_u16pk", k15, out, p.multiProcessorCount);
  run("max3_f32", k16, out, p.multiProcessorCount);
  return 0; }
