// Exhaustive check (diagnostic): is (float)v_sqrt_f64((double)x) the correctly rounded sqrtf(x)
// for every non-negative finite float x?  Per-block mismatch counts, plain vector stores.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

__device__ __forceinline__ double raw_sqrt_f64(double d) {
  double r;
  asm volatile("v_sqrt_f64 %0, %1" : "=v"(r) : "v"(d));
  return r;
}

__global__ void __launch_bounds__(256) check(unsigned base, unsigned* out_count, unsigned* out_first) {
  __shared__ unsigned cnt[256];
  __shared__ unsigned first[256];
  const unsigned i = base + blockIdx.x * 256u * 64u + threadIdx.x;
  unsigned c = 0, f = 0xffffffffu;
  for (int k = 0; k < 64; ++k) {
    const unsigned bits = i + 256u * (unsigned)k;
    if (bits >= 0x7f800000u) break;
    const float x = __uint_as_float(bits);
    const float a = __builtin_sqrtf(x);  // llvm.sqrt.f32: IEEE correctly rounded sequence
    const float b = (float)raw_sqrt_f64((double)x);
    if (__float_as_uint(a) != __float_as_uint(b)) { ++c; if (f == 0xffffffffu) f = bits; }
  }
  cnt[threadIdx.x] = c;
  first[threadIdx.x] = f;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned s = 0, mf = 0xffffffffu;
    for (int t = 0; t < 256; ++t) { s += cnt[t]; mf = first[t] < mf ? first[t] : mf; }
    out_count[blockIdx.x] = s;
    out_first[blockIdx.x] = mf;
  }
}

int main() {
  const unsigned per_block = 256u * 64u;
  const unsigned total = 0x7f800000u;
  const unsigned blocks = (total + per_block - 1) / per_block;
  unsigned *dc, *df;
  hipMalloc(&dc, blocks * 4);
  hipMalloc(&df, blocks * 4);
  hipLaunchKernelGGL(check, dim3(blocks), dim3(256), 0, 0, 0u, dc, df);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
  unsigned* hc = (unsigned*)malloc(blocks * 4);
  unsigned* hf = (unsigned*)malloc(blocks * 4);
  hipMemcpy(hc, dc, blocks * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hf, df, blocks * 4, hipMemcpyDeviceToHost);
  unsigned long long s = 0;
  unsigned mf = 0xffffffffu;
  for (unsigned b = 0; b < blocks; ++b) { s += hc[b]; if (hf[b] < mf) mf = hf[b]; }
  printf("checked %u floats [0, 0x7f800000): mismatches %llu, first 0x%08x\n", total, s, mf);
  return 0;
}
