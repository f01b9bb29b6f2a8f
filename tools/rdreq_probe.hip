// rdreq_probe.hip — memory-side read requests (TCC_EA0_RDREQ) per known byte count for the access
// shapes of the step kernels' loads (diagnostic; run under rocprofv3 --pmc, one launch per shape on a
// buffer region no earlier launch touched):
//   hipcc --offload-arch=gfx950 -O3 tools/rdreq_probe.hip -o build/rdreq_probe
//   rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum -- build/rdreq_probe
// Shapes (one wave per "env", E = 8192 envs):
//   row192_dword : 48 lanes x 4 B = one 192-B row per env at env * 192 (step16q's 16-drone rows)
//   row256_dword : 64 lanes x 4 B = one 256-B row per env at env * 256 (two whole 128-B lines)
//   row768_x3    : 64 lanes x 12 B = one 768-B row per env at env * 768 (step64's pos / vel rows)
//   row16_byte   : 16 lanes x 1 B per env at env * 16 (step16q's active bytes)
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr int E = 8192;
__global__ void __launch_bounds__(64) row192_dword(const float* __restrict__ src, float* out) {
  const int t = threadIdx.x, e = blockIdx.x;
  float v = 0.f;
  if (t < 48) v = src[(size_t)e * 48 + t];
  if (v == 12345.f) out[e] = v;  // keeps the load
}
__global__ void __launch_bounds__(64) row256_dword(const float* __restrict__ src, float* out) {
  const int t = threadIdx.x, e = blockIdx.x;
  const float v = src[(size_t)e * 64 + t];
  if (v == 12345.f) out[e] = v;
}
__global__ void __launch_bounds__(64) row768_x3(const float* __restrict__ src, float* out) {
  const int t = threadIdx.x, e = blockIdx.x;
  const float* r = src + (size_t)e * 192 + 3 * t;
  const float v = r[0] + r[1] + r[2];
  if (v == 12345.f) out[e] = v;
}
__global__ void __launch_bounds__(64) row16_byte(const unsigned char* __restrict__ src, float* out) {
  const int t = threadIdx.x, e = blockIdx.x;
  unsigned char v = 0;
  if (t < 16) v = src[(size_t)e * 16 + t];
  if (v == 77) out[e] = 1.f;
}
int main() {
  const size_t region = (size_t)E * 768;  // bytes per shape (the largest shape's footprint)
  char* buf;
  float* out;
  if (hipMalloc(&buf, 8 * region) != hipSuccess || hipMalloc(&out, E * 4) != hipSuccess) return 1;
  // no initialisation: a memset would leave the regions in the caches (the values are never used)
  // each shape reads its own region (never touched by a kernel before): memory-side requests only
  hipLaunchKernelGGL(row192_dword, dim3(E), dim3(64), 0, 0, (const float*)(buf + 0 * region), out);
  hipLaunchKernelGGL(row256_dword, dim3(E), dim3(64), 0, 0, (const float*)(buf + 2 * region), out);
  hipLaunchKernelGGL(row768_x3, dim3(E), dim3(64), 0, 0, (const float*)(buf + 4 * region), out);
  hipLaunchKernelGGL(row16_byte, dim3(E), dim3(64), 0, 0, (const unsigned char*)(buf + 6 * region), out);
  (void)hipDeviceSynchronize();
  printf("bytes per launch: row192_dword %d, row256_dword %d, row768_x3 %d, row16_byte %d\n", E * 192, E * 256,
         E * 768, E * 16);
  printf("128-B lines touched: row192_dword %d, row256_dword %d, row768_x3 %d, row16_byte %d\n",
         (E * 192 + 127) / 128, E * 2, E * 6, (E * 16 + 127) / 128);
  return 0;
}
