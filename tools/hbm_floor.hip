// hbm_floor.hip — the bytes-only floor of the headline step's memory pattern (diagnostic):
// per env (N = 64 drones) read pos / vel / actions (36 B per drone) + active (1 B), write pos / vel
// (24 B per drone) + the 37-float obs rows (148 B per drone) + reward (4 B) + 3 flag bytes, i.e.
// the 216 B per agent of the step's algorithmic traffic, with no compute.  One wave per env as in
// swarm_step64_once (4 envs per 256-thread workgroup), obs as coalesced 16-B stores (sc1 or plain).
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_floor.hip -o build/hbm_floor && build/hbm_floor [E]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int N = 64, D = 37;
typedef int v4i __attribute__((ext_vector_type(4)));

template <int AUX, bool READS>
__global__ void __launch_bounds__(256) floor_kernel(const float* __restrict__ pos_in, float* __restrict__ pos,
                                                    float* __restrict__ vel, const float* __restrict__ act,
                                                    uint8_t* __restrict__ active, float* __restrict__ obs,
                                                    float* __restrict__ rew, uint8_t* __restrict__ flags, int E) {
  const int t = threadIdx.x & 63;
  const int env = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (env >= E) return;
  const size_t a = (size_t)env * N + t;
  float s = (float)t;
  if (READS) {
    s += pos_in[a * 3] + pos_in[a * 3 + 1] + pos_in[a * 3 + 2];
    s += vel[a * 3] + vel[a * 3 + 1] + vel[a * 3 + 2];
    s += act[a * 3] + act[a * 3 + 1] + act[a * 3 + 2] + (float)active[a];
  }
  pos[a * 3] = s; pos[a * 3 + 1] = s; pos[a * 3 + 2] = s;
  vel[a * 3] = s; vel[a * 3 + 1] = s; vel[a * 3 + 2] = s;
  rew[a] = s;
  flags[(size_t)env * N * 3 + t] = (uint8_t)s;
  flags[(size_t)env * N * 3 + 64 + t] = (uint8_t)s;
  flags[(size_t)env * N * 3 + 128 + t] = (uint8_t)s;
  // obs: the env's 64 x 37 floats = 592 float4 as coalesced 16-B stores
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(obs + (size_t)env * N * D, 0, N * D * 4, 0x00020000);
  const v4i v = {__float_as_int(s), __float_as_int(s), __float_as_int(s), __float_as_int(s)};
  for (int i = t; i < N * D / 4; i += 64) __builtin_amdgcn_raw_buffer_store_b128(v, r, 16 * i, 0, AUX);
}

template <int AUX, bool READS>
static float run(int E, int G, float* pos_in, float* pos, float* vel, float* act, uint8_t* active, float* obs,
                 float* rew, uint8_t* flags, hipStream_t* st) {
  const int eg = E / G;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&](int g) {
    const size_t o = (size_t)g * eg * N;
    hipLaunchKernelGGL((floor_kernel<AUX, READS>), dim3((eg + 3) / 4), dim3(256), 0, st[g], pos_in + o * 3,
                       pos + o * 3, vel + o * 3, act + o * 3, active + o, obs + o * D, rew + o, flags + o * 3, eg);
  };
  for (int k = 0; k < 200; ++k)
    for (int g = 0; g < G; ++g) launch(g);
  (void)hipDeviceSynchronize();
  const int K = 400;
  (void)hipEventRecord(a, 0);
  (void)hipDeviceSynchronize();
  for (int k = 0; k < K; ++k)
    for (int g = 0; g < G; ++g) launch(g);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / K;
}

int main(int argc, char** argv) {
  const int E = argc > 1 ? atoi(argv[1]) : 8192;
  const size_t A = (size_t)E * N;
  float *pos_in, *pos, *vel, *act, *obs, *rew;
  uint8_t *active, *flags;
  (void)hipMalloc(&pos_in, A * 12);
  (void)hipMalloc(&pos, A * 12);
  (void)hipMalloc(&vel, A * 12);
  (void)hipMalloc(&act, A * 12);
  (void)hipMalloc(&obs, A * D * 4);
  (void)hipMalloc(&rew, A * 4);
  (void)hipMalloc(&active, A);
  (void)hipMalloc(&flags, A * 3);
  (void)hipMemset(pos_in, 0, A * 12);
  (void)hipMemset(vel, 0, A * 12);
  (void)hipMemset(act, 0, A * 12);
  (void)hipMemset(active, 1, A);
  hipStream_t st[4];
  for (auto& s : st) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const double bytes = 216.0 * A;  // the step's algorithmic bytes per launch (117 B per env omitted)
  for (int G : {1, 2, 3, 4}) {
    const float sc1 = run<16, true>(E, G, pos_in, pos, vel, act, active, obs, rew, flags, st);
    const float plain = run<0, true>(E, G, pos_in, pos, vel, act, active, obs, rew, flags, st);
    const float wo = run<16, false>(E, G, pos_in, pos, vel, act, active, obs, rew, flags, st);
    printf("E=%d groups=%d: reads+writes sc1 %.2f us (%.2f TB/s)  plain %.2f us (%.2f TB/s)  writes-only sc1 %.2f us\n",
           E, G, sc1, bytes / sc1 * 1e-6, plain, bytes / plain * 1e-6, wo);
    fflush(stdout);
  }
  return 0;
}
