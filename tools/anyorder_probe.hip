// Probe: does hipExtAnyOrderLaunch let a kernel start before the previous kernel on the SAME
// stream has finished (AQL barrier bit clear) on gfx950?  And are the workgroups of launch k all
// dispatched before any workgroup of launch k+1 (the in-order dispatch a cross-launch flag wait
// would rely on)?
//   hipcc --offload-arch=gfx950 -O2 tools/anyorder_probe.hip -o build/anyorder_probe
// Kernel A: `blocks` workgroups, each spins ~spin_us (s_memrealtime, 100 MHz) and records start /
// end.  Kernel B (launched after A, any-order or not): records the start of each workgroup.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void spin_kernel(unsigned long long* ts, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < ticks) {
    __builtin_amdgcn_s_sleep(2);
    t = __builtin_amdgcn_s_memrealtime();
  }
  if (threadIdx.x == 0) { ts[2 * blockIdx.x] = t0; ts[2 * blockIdx.x + 1] = t; }
}

__global__ void mark_kernel(unsigned long long* ts) {
  if (threadIdx.x == 0) ts[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 1;
  const int spin_us = argc > 2 ? atoi(argv[2]) : 200;
  const int mblocks = argc > 3 ? atoi(argv[3]) : 8;
  unsigned long long *a, *b;
  CHECK(hipMalloc(&a, 2 * blocks * sizeof(unsigned long long)));
  CHECK(hipMalloc(&b, mblocks * sizeof(unsigned long long)));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int flags = 0; flags <= 1; ++flags) {
    for (int rep = 0; rep < 3; ++rep) {
      CHECK(hipMemset(a, 0, 2 * blocks * sizeof(unsigned long long)));
      CHECK(hipMemset(b, 0, mblocks * sizeof(unsigned long long)));
      CHECK(hipDeviceSynchronize());
      hipExtLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s, nullptr, nullptr, 0, a,
                            (unsigned long long)spin_us * 100ull);
      hipExtLaunchKernelGGL(mark_kernel, dim3(mblocks), dim3(64), 0, s, nullptr, nullptr, (uint32_t)flags, b);
      CHECK(hipGetLastError());
      CHECK(hipStreamSynchronize(s));
      unsigned long long ha[4096], hb[1024];
      CHECK(hipMemcpy(ha, a, 2 * blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(hb, b, mblocks * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      unsigned long long a0 = ~0ull, a1 = 0, b0 = ~0ull, b1 = 0;
      for (int i = 0; i < blocks; ++i) { if (ha[2 * i] < a0) a0 = ha[2 * i]; if (ha[2 * i + 1] > a1) a1 = ha[2 * i + 1]; }
      for (int i = 0; i < mblocks; ++i) { if (hb[i] < b0) b0 = hb[i]; if (hb[i] > b1) b1 = hb[i]; }
      printf("flags=%d rep=%d  A: start 0 end %.1f us | B: first start %+.1f us last start %+.1f us -> %s\n", flags, rep,
             (a1 - a0) / 100.0, ((double)b0 - (double)a0) / 100.0, ((double)b1 - (double)a0) / 100.0,
             b0 < a1 ? "OVERLAP (B started before A ended)" : "serialised");
    }
  }
  return 0;
}
