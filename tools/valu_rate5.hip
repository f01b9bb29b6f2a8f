// valu_rate5.hip — issue cost of the v_cndmask / v_cmp forms hipcc emits, and of the LDS
// exchange instructions of the pair pass, at 8 waves per SIMD (diagnostic only):
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate5.hip -o build/valu_rate5 && build/valu_rate5
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int ITERS = 256;
#define BODY8(ins) ins "\n" ins "\n" ins "\n" ins "\n" ins "\n" ins "\n" ins "\n" ins
#define KERNEL(name, init, ins, clob...)                                                   \
  __global__ void __launch_bounds__(256) name(float* out) {                              \
    __shared__ float lds[256 * 4];                                                       \
    lds[threadIdx.x] = 1.0f;                                                             \
    __syncthreads();                                                                     \
    asm volatile(init ::: clob);                                                         \
    for (int i = 0; i < ITERS; ++i) asm volatile(BODY8(ins) ::: clob);                   \
  }
#define INIT "v_mov_b32 v8, 1.0\n v_mov_b32 v9, 2.0\n v_mov_b32 v10, 3.0\n v_mov_b32 v11, 1.5\n v_mov_b32 v12, 7\n v_mov_b32 v13, 9\n v_cmp_lt_f32 vcc, v8, v9\n v_cmp_lt_f32 s[20:21], v8, v9\n v_lshlrev_b32 v16, 2, v0"
#define CL "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "vcc", "s20", "s21", "memory"
KERNEL(k_add, INIT, "v_add_f32 v14, v8, v9", CL)
KERNEL(k_cnd_vcc, INIT, "v_cndmask_b32 v14, v8, v9, vcc", CL)
KERNEL(k_cnd_vcc64, INIT, "v_cndmask_b32_e64 v14, v8, v9, vcc", CL)
KERNEL(k_cnd_s, INIT, "v_cndmask_b32_e64 v14, v8, v9, s[20:21]", CL)
KERNEL(k_cmp_cnd, INIT, "v_cmp_lt_f32 vcc, v8, v9\n v_cndmask_b32 v14, v8, v9, vcc", CL)
KERNEL(k_cmp_cnd64, INIT, "v_cmp_lt_f32_e64 s[20:21], v8, v9\n v_cndmask_b32_e64 v14, v8, v9, s[20:21]", CL)
KERNEL(k_cmpvcc, INIT, "v_cmp_lt_f32 vcc, v8, v9", CL)
KERNEL(k_cmps, INIT, "v_cmp_lt_f32_e64 s[20:21], v8, v9", CL)
KERNEL(k_addc, INIT, "v_add_co_u32 v14, vcc, v12, v13", CL)
KERNEL(k_bperm, INIT, "ds_bpermute_b32 v14, v16, v12", CL)
KERNEL(k_read2, INIT, "ds_read2_b32 v[14:15], v16 offset1:1", CL)
KERNEL(k_readb128, INIT, "ds_read_b128 v[16:19], v14", CL)
KERNEL(k_snop, INIT, "s_nop 0", CL)

int main() {
  float* out;
  (void)hipMalloc(&out, 4);
  struct K { const char* n; void (*f)(float*); } ks[] = {
      {"v_add_f32", k_add}, {"v_cndmask vcc (e32)", k_cnd_vcc}, {"v_cndmask_e64 vcc", k_cnd_vcc64},
      {"v_cndmask_e64 s[]", k_cnd_s}, {"v_cmp vcc + v_cndmask vcc (pair)", k_cmp_cnd},
      {"v_cmp s[] + v_cndmask s[] (pair)", k_cmp_cnd64}, {"v_cmp -> vcc", k_cmpvcc}, {"v_cmp -> s[]", k_cmps},
      {"v_add_co_u32 (vcc carry)", k_addc}, {"ds_bpermute_b32", k_bperm}, {"ds_read2_b32", k_read2},
      {"ds_read_b128", k_readb128}, {"s_nop 0", k_snop}};
  const int blocks = 256 * 8;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  double base = 0;
  for (auto& k : ks) {
    printf("%s ...\n", k.n);
    fflush(stdout);
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out);
    (void)hipEventRecord(a);
    for (int rep = 0; rep < 10; ++rep) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double per_simd = 10.0 * blocks * 4 * ITERS * 8 / 1024.0;
    const double ns = ms * 1e6 / per_simd;
    if (base == 0) base = ns;
    printf("%-36s %.3f ns per (group of) instruction(s) per SIMD (%.1f cyc @2.4GHz)\n", k.n, ns, ns * 2.4);
    fflush(stdout);
  }
  return 0;
}
