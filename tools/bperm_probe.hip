// Probe: do ds_bpermute_b32 lane rotations (step64's mirror exchange) count as LDS bank
// conflicts on gfx950?  Kernel `rot`: 32 ds_bpermute rotations (r = 1..32) per wave, the pattern
// of pair_group_s64's mirror keys; kernel `ident`: the same count of identity bpermutes; kernel
// `rd`: 32 ds_read_b32 of consecutive words (conflict-free reference).  Run under
//   rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES -- build/bperm_probe
//   hipcc --offload-arch=gfx950 -O2 tools/bperm_probe.hip -o build/bperm_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void __launch_bounds__(256) rot(unsigned* out, int reps) {
  const unsigned t = threadIdx.x & 63;
  unsigned v = t * 2654435761u, acc = 0;
  for (int k = 0; k < reps; ++k) {
#pragma unroll
    for (int r = 1; r <= 32; ++r)
      acc += (unsigned)__builtin_amdgcn_ds_bpermute((int)(((t + 64 - r) & 63) << 2), (int)(v + r));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void __launch_bounds__(256) ident(unsigned* out, int reps) {
  const unsigned t = threadIdx.x & 63;
  unsigned v = t * 2654435761u, acc = 0;
  for (int k = 0; k < reps; ++k) {
#pragma unroll
    for (int r = 1; r <= 32; ++r) acc += (unsigned)__builtin_amdgcn_ds_bpermute((int)(t << 2), (int)(v + r));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void __launch_bounds__(256) rd(unsigned* out, int reps) {
  __shared__ unsigned s[256 + 64];
  const unsigned t = threadIdx.x;
  s[t] = t * 3u;
  if (t < 64) s[256 + t] = t;
  __syncthreads();
  unsigned acc = 0;
  for (int k = 0; k < reps; ++k) {
    const unsigned* p = s + (t & ~63u) + (t & 63);
    asm volatile("" : "+v"(p));
#pragma unroll
    for (int r = 1; r <= 32; ++r) acc += p[r];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  unsigned* o;
  if (hipMalloc(&o, 1024 * 256 * sizeof(unsigned)) != hipSuccess) return 1;
  hipLaunchKernelGGL(rot, dim3(1024), dim3(256), 0, 0, o, 16);
  hipLaunchKernelGGL(ident, dim3(1024), dim3(256), 0, 0, o, 16);
  hipLaunchKernelGGL(rd, dim3(1024), dim3(256), 0, 0, o, 16);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("ok\n");
  return 0;
}
