// swarm_kernel.hip — fused swarm step / reset / observe kernel for gfx950 (MI355X, CDNA4),
// plus the C-ABI entry points declared in include/swarm_mi355x.h.
//
// One launch processes E envs.  A "team" of L = next_pow2(N) lanes owns one env (one lane per
// drone); a 256-thread workgroup holds G = 256/L teams (N <= 256) or one team of L lanes.
// Per launch and env:
//   HBM -> regs/LDS : own pos/vel/action (12 B each per lane, coalesced), goal, obstacles
//   integrate       : kinematic Euler (drone_swarm_env.py:103-117) or the point-mass
//                     restatement of the PyBullet substep loop (drone_physics_env.py:323-360)
//   pair pass       : every lane scans all N drones from LDS (broadcast reads): exact float
//                     squared distance, top-(K+1) (s, j) keys, collision, formation sum
//   obstacle pass   : exact axis-path distances, top-Ms keys, obstacle collision
//   reductions      : team LDS counters (any_collision, continuing count)
//   auto-reset      : Philox4x32-10 draws + a second kNN pass for envs whose episode ended
//   obs             : rows staged in LDS [team][N][D] then stored as 16-B coalesced writes
//
// Bit-exactness (SURVEY.md §8a parity spec): no FP contraction (-ffp-contract=off + explicit
// __f*_rn / __d*_rn), correctly rounded sqrt/div where the reference's value is observable.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "swarm_mi355x.h"

namespace {

constexpr uint64_t KEY_EMPTY = ~0ull;
constexpr int MODE_STEP = 0;
constexpr int MODE_RESET = 1;
constexpr int MODE_OBSERVE = 2;
constexpr int DYN_KIN = SWARM_DYN_KINEMATIC;
constexpr int DYN_PHYS = SWARM_DYN_POINTMASS_PHYSICS;
constexpr int MAX_N = 1024;
constexpr int MAX_K = 16;
constexpr int MAX_MS = 16;
constexpr int STAGE_LDS_BUDGET = 64 * 1024;  // stage obs through LDS below this footprint
constexpr int LDS_LIMIT = 160 * 1024;

// Derived, launch-ready parameters (host computes once per call).
struct KParams {
  int E, N, M, K, Ms, D, max_steps, reward_mode, auto_reset, substeps, damping_law;
  int lanes, log2_lanes, envs_per_block, stage_obs, obs_vec4;
  int pos_stride, obst_stride;  // float4 per team in LDS (padded by one to spread banks)
  int off_obst, off_team, off_block, off_stage;
  long long env_offset;
  unsigned seed_lo, seed_hi;
  float half_w, neg_half_w, width_w;
  float dt, vmax, amax, eps_speed;
  float s_pair, s_obst;             // kinematic collision thresholds in squared-distance space
  float s_phys_pair, s_phys_obst, ground_z;
  float h, g, gcomp;
  double goal_radius, desired_spacing, kp, r_goal, r_col, kf, vmax_d;
};

// ------------------------------------------------------------------ exact numerics
// No FP contraction anywhere in this file (the reference's NumPy ops round every product).
#pragma clang fp contract(off)
// Correctly rounded square roots.  NB: HIP's __fsqrt_rn is v_sqrt_f32 (1 ulp) unless
// OCML_BASIC_ROUNDED_OPERATIONS is defined; llvm.sqrt lowers to the IEEE-exact sequence.
__device__ __forceinline__ float sqrt_rn(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ double dsqrt_rn(double x) { return __builtin_sqrt(x); }
// np.linalg.norm(v) of a float32 3-vector: OpenBLAS sdot = double accumulation of float
// products, rounded to float; sqrt in float.  Returns the float sum s (d = sqrtf(s)).
__device__ __forceinline__ float sqsum_1d(float x, float y, float z) {
  const float xx = __fmul_rn(x, x), yy = __fmul_rn(y, y), zz = __fmul_rn(z, z);
  return __double2float_rn(__dadd_rn(__dadd_rn((double)xx, (double)yy), (double)zz));
}
// np.linalg.norm(A, axis=1): float32 ((x*x)+(y*y))+(z*z).
__device__ __forceinline__ float sqsum_axis(float x, float y, float z) {
  return __fadd_rn(__fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y)), __fmul_rn(z, z));
}
__device__ __forceinline__ uint64_t make_key(float v, int idx) {
  return ((uint64_t)__float_as_uint(v) << 32) | (uint32_t)idx;
}
__device__ __forceinline__ float key_val(uint64_t k) { return __uint_as_float((uint32_t)(k >> 32)); }
__device__ __forceinline__ int key_idx(uint64_t k) { return (int)(uint32_t)(k & 0xffffffffu); }

// Insert `key` into the ascending list k[0..S-1], dropping the largest.
template <int S>
__device__ __forceinline__ void topk_insert(uint64_t (&k)[S], uint64_t key) {
#pragma unroll
  for (int s = S - 1; s > 0; --s) {
    const uint64_t lo = k[s - 1];
    const uint64_t cur = k[s];
    k[s] = (key < lo) ? lo : ((key < cur) ? key : cur);
  }
  k[0] = (key < k[0]) ? key : k[0];
}

// ------------------------------------------------------------------ Philox4x32-10 (device reset)
__device__ __forceinline__ void philox4x32_10(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = (uint32_t)p1;
    c[2] = n2;
    c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
__device__ __forceinline__ float uni(uint32_t x, float lo, float width) {
  const float u = __fmul_rn((float)(x >> 8), 0x1p-24f);
  return __fadd_rn(lo, __fmul_rn(u, width));
}
__device__ __forceinline__ void draw_block(const KParams& P, long long genv, uint32_t episode,
                                           uint32_t block, uint32_t (&w)[4]) {
  w[0] = block;
  w[1] = episode;
  w[2] = (uint32_t)((unsigned long long)genv & 0xffffffffull);
  w[3] = (uint32_t)((unsigned long long)genv >> 32);
  philox4x32_10(w, P.seed_lo, P.seed_hi);
}

// ------------------------------------------------------------------ passes
// PASS 0: kNN keys only.  PASS 1: kinematic step (+ collision among active drones, formation).
// PASS 2: physics step (+ collision among all drones).
template <int KS, int PASS>
__device__ __forceinline__ void neighbor_pass(const float4* __restrict__ pos4, int N, int t,
                                              float px, float py, float pz, bool act_i,
                                              float s_thr, double ds, uint64_t (&nk)[KS > 0 ? KS : 1],
                                              bool& coll, double& fsum) {
  for (int j = 0; j < N; ++j) {
    const float4 q = pos4[j];
    const float s = sqsum_1d(__fsub_rn(q.x, px), __fsub_rn(q.y, py), __fsub_rn(q.z, pz));
    if constexpr (KS > 0) {
      const uint64_t key = (j == t) ? KEY_EMPTY : make_key(s, j);
      topk_insert<KS>(nk, key);
    }
    if constexpr (PASS == 1) {
      const bool pair = act_i && (q.w != 0.0f) && (j != t);
      coll = coll || (pair && (s <= s_thr));
      // formation uses d_ij widened to double; v_sqrt_f32 (<=1 ulp) keeps the reward within
      // ~1e-7 of the reference's mean, well inside the 1e-5 contract.
      const float d = __builtin_amdgcn_sqrtf(s);
      const double e = fabs(__dsub_rn((double)d, ds));
      fsum = __dadd_rn(fsum, pair ? e : 0.0);
    } else if constexpr (PASS == 2) {
      coll = coll || ((j != t) && (s <= s_thr));
    }
  }
}

template <int MSL, bool COLL>
__device__ __forceinline__ void obstacle_pass(const float4* __restrict__ obst4, int M, float px,
                                              float py, float pz, bool chk, float s_thr,
                                              uint64_t (&ok)[MSL > 0 ? MSL : 1], bool& coll) {
  for (int m = 0; m < M; ++m) {
    const float4 q = obst4[m];
    const float s = sqsum_axis(__fsub_rn(q.x, px), __fsub_rn(q.y, py), __fsub_rn(q.z, pz));
    if constexpr (MSL > 0) topk_insert<MSL>(ok, make_key(sqrt_rn(s), m));
    if constexpr (COLL) coll = coll || (chk && (s <= s_thr));
  }
}

// ------------------------------------------------------------------ the kernel
template <int DYN, int KS, int MSL>
__global__ void __launch_bounds__(1024)
swarm_kernel(const KParams P, const swarm_state_t S, const float* __restrict__ actions,
             const uint8_t* __restrict__ amask, const swarm_out_t O,
             const uint8_t* __restrict__ env_mask, int mode) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int L = P.lanes;
  const int team = tid >> P.log2_lanes;
  const int t = tid & (L - 1);
  const int G = P.envs_per_block;
  const int N = P.N, M = P.M, D = P.D;
  const long long env0 = (long long)blockIdx.x * G;
  const long long env = env0 + team;
  const bool env_ok = env < P.E;
  const bool is_agent = env_ok && t < N;
  float4* pos4 = reinterpret_cast<float4*>(smem) + team * P.pos_stride;
  float4* obst4 = reinterpret_cast<float4*>(smem + P.off_obst) + team * P.obst_stride;
  int* tint = reinterpret_cast<int*>(smem + P.off_team) + team * 4;
  int* bflag = reinterpret_cast<int*>(smem + P.off_block);
  float* stage = reinterpret_cast<float*>(smem + P.off_stage);

  // envs this call writes: every env (step) or the masked ones (reset / observe)
  bool sel = env_ok;
  if (mode != MODE_STEP && env_mask != nullptr && env_ok) sel = env_mask[env] != 0;

  // ---- load
  if (t == 0) { tint[0] = 0; tint[1] = 0; tint[2] = 0; tint[3] = 0; }
  if (tid == 0) bflag[0] = 0;
  int stepc = 0;
  float gx = 0.f, gy = 0.f, gz = 0.f;
  if (env_ok) {
    for (int m = t; m < M; m += L) {
      const float* o = S.obstacles + (env * M + m) * 3;
      obst4[m] = make_float4(o[0], o[1], o[2], 0.f);
    }
    gx = S.goal[env * 3 + 0];
    gy = S.goal[env * 3 + 1];
    gz = S.goal[env * 3 + 2];
    stepc = S.step_count[env];
  }
  float px = 0.f, py = 0.f, pz = 0.f, vx = 0.f, vy = 0.f, vz = 0.f, damp = 0.f;
  bool act = false;
  const long long ag = env * N + t;
  if (is_agent) {
    px = S.pos[ag * 3 + 0]; py = S.pos[ag * 3 + 1]; pz = S.pos[ag * 3 + 2];
    vx = S.vel[ag * 3 + 0]; vy = S.vel[ag * 3 + 1]; vz = S.vel[ag * 3 + 2];
    act = S.active[ag] != 0;
    if constexpr (DYN == DYN_PHYS) damp = S.damping[ag];
  }
  __syncthreads();
  if (is_agent && act) atomicAdd(&tint[0], 1);
  __syncthreads();
  const int n_active = tint[0];

  // ---- integrate (step) or draw (explicit reset)
  float prev_d = 0.f;
  uint32_t episode_new = 0;
  const long long genv = P.env_offset + env;
  if (mode == MODE_STEP && is_agent) {
    float ax = actions[ag * 3 + 0], ay = actions[ag * 3 + 1], az = actions[ag * 3 + 2];
    const bool has = (amask == nullptr) || (amask[ag] != 0);
    if constexpr (DYN == DYN_KIN) {
      if (act) {  // drone_swarm_env.py:98-111
        prev_d = sqrt_rn(sqsum_1d(__fsub_rn(gx, px), __fsub_rn(gy, py), __fsub_rn(gz, pz)));
        if (!has) { ax = 0.f; ay = 0.f; az = 0.f; }
        ax = __fmul_rn(fminf(fmaxf(ax, -1.f), 1.f), P.amax);
        ay = __fmul_rn(fminf(fmaxf(ay, -1.f), 1.f), P.amax);
        az = __fmul_rn(fminf(fmaxf(az, -1.f), 1.f), P.amax);
        vx = __fadd_rn(vx, __fmul_rn(ax, P.dt));
        vy = __fadd_rn(vy, __fmul_rn(ay, P.dt));
        vz = __fadd_rn(vz, __fmul_rn(az, P.dt));
        const float sp = sqrt_rn(sqsum_1d(vx, vy, vz));  // _clip_speed :179-183
        if (!(sp <= P.vmax || sp < P.eps_speed)) {
          vx = __fmul_rn(__fdiv_rn(vx, sp), P.vmax);
          vy = __fmul_rn(__fdiv_rn(vy, sp), P.vmax);
          vz = __fmul_rn(__fdiv_rn(vz, sp), P.vmax);
        }
        px = __fadd_rn(px, __fmul_rn(vx, P.dt));
        py = __fadd_rn(py, __fmul_rn(vy, P.dt));
        pz = __fadd_rn(pz, __fmul_rn(vz, P.dt));
      }
      if (n_active > 0) {  // world clip of ALL drones, :113-117
        px = fminf(fmaxf(px, P.neg_half_w), P.half_w);
        py = fminf(fmaxf(py, P.neg_half_w), P.half_w);
        pz = fminf(fmaxf(pz, P.neg_half_w), P.half_w);
      }
    } else {
      // point-mass restatement of drone_physics_env.py:323-360
      const float h = P.h;
      const float cx = has ? __fmul_rn(ax, P.amax) : 0.f;
      const float cy = has ? __fmul_rn(ay, P.amax) : 0.f;
      float cz = has ? __fadd_rn(__fmul_rn(az, P.amax), P.gcomp) : 0.f;
      cz = __fadd_rn(cz, P.g);
      float fac = 1.f;
      if (P.damping_law == 1) fac = __double2float_rn(pow((double)__fsub_rn(1.f, damp), (double)h));
      for (int s = 0; s < P.substeps; ++s) {
        const float sp = sqrt_rn(sqsum_1d(vx, vy, vz));
        if (has && sp > P.vmax) {
          vx = __fmul_rn(__fdiv_rn(vx, sp), P.vmax);
          vy = __fmul_rn(__fdiv_rn(vy, sp), P.vmax);
          vz = __fmul_rn(__fdiv_rn(vz, sp), P.vmax);
        }
        if (P.damping_law == 0) {
          const float sp2 = sqrt_rn(sqsum_1d(vx, vy, vz));
          const float c = __fmul_rn(damp, __fadd_rn(1.f, sp2));
          vx = __fadd_rn(vx, __fmul_rn(h, __fsub_rn(cx, __fmul_rn(c, vx))));
          vy = __fadd_rn(vy, __fmul_rn(h, __fsub_rn(cy, __fmul_rn(c, vy))));
          vz = __fadd_rn(vz, __fmul_rn(h, __fsub_rn(cz, __fmul_rn(c, vz))));
        } else {
          vx = __fmul_rn(__fadd_rn(vx, __fmul_rn(h, cx)), fac);
          vy = __fmul_rn(__fadd_rn(vy, __fmul_rn(h, cy)), fac);
          vz = __fmul_rn(__fadd_rn(vz, __fmul_rn(h, cz)), fac);
        }
        px = __fadd_rn(px, __fmul_rn(h, vx));
        py = __fadd_rn(py, __fmul_rn(h, vy));
        pz = __fadd_rn(pz, __fmul_rn(h, vz));
      }
    }
  }

  // explicit device reset: draw the new episode before the observation pass
  if (mode == MODE_RESET && sel) {
    episode_new = S.episode[env] + 1u;
    uint32_t w[4];
    if (t < N) {
      draw_block(P, genv, episode_new, (uint32_t)t, w);
      px = uni(w[0], P.neg_half_w, P.width_w);
      py = uni(w[1], P.neg_half_w, P.width_w);
      pz = uni(w[2], P.neg_half_w, P.width_w);
      vx = vy = vz = 0.f;
      act = true;
      if constexpr (DYN == DYN_PHYS) {
        pz = fmaxf(pz, 1.0f);
        damp = __fmul_rn(0.5f, uni(w[3], 0.8f, 0.4f));
      }
    }
    for (int m = t; m < M; m += L) {
      draw_block(P, genv, episode_new, (uint32_t)(N + m), w);
      float oz = uni(w[2], P.neg_half_w, P.width_w);
      if constexpr (DYN == DYN_PHYS) oz = fmaxf(oz, 0.5f);
      obst4[m] = make_float4(uni(w[0], P.neg_half_w, P.width_w), uni(w[1], P.neg_half_w, P.width_w), oz, 0.f);
    }
    draw_block(P, genv, episode_new, (uint32_t)(N + M), w);
    gx = uni(w[0], P.neg_half_w, P.width_w);
    gy = uni(w[1], P.neg_half_w, P.width_w);
    gz = uni(w[2], P.neg_half_w, P.width_w);
    if constexpr (DYN == DYN_PHYS) gz = uni(w[3], 0.5f, 1.5f);
    stepc = 0;
  }

  if (is_agent) {
    const float wflag = (DYN == DYN_KIN) ? (act ? 1.f : 0.f) : 1.f;
    pos4[t] = make_float4(px, py, pz, wflag);
  }
  __syncthreads();

  // ---- pair + obstacle passes
  uint64_t nk[KS > 0 ? KS : 1];
  uint64_t ok[MSL > 0 ? MSL : 1];
#pragma unroll
  for (int s = 0; s < (KS > 0 ? KS : 1); ++s) nk[s] = KEY_EMPTY;
#pragma unroll
  for (int s = 0; s < (MSL > 0 ? MSL : 1); ++s) ok[s] = KEY_EMPTY;
  bool coll = false;
  double fsum = 0.0;
  const bool do_pass = is_agent && (mode == MODE_STEP || sel);
  if (do_pass) {
    if (mode == MODE_STEP) {
      if constexpr (DYN == DYN_KIN) {
        neighbor_pass<KS, 1>(pos4, N, t, px, py, pz, act, P.s_pair, P.desired_spacing, nk, coll, fsum);
        obstacle_pass<MSL, true>(obst4, M, px, py, pz, act, P.s_obst, ok, coll);
      } else {
        neighbor_pass<KS, 2>(pos4, N, t, px, py, pz, act, P.s_phys_pair, 0.0, nk, coll, fsum);
        obstacle_pass<MSL, true>(obst4, M, px, py, pz, true, P.s_phys_obst, ok, coll);
      }
    } else {
      neighbor_pass<KS, 0>(pos4, N, t, px, py, pz, act, 0.f, 0.0, nk, coll, fsum);
      obstacle_pass<MSL, false>(obst4, M, px, py, pz, false, 0.f, ok, coll);
    }
  }

  // ---- rewards / terminations (step)
  float rew = 0.f, dist_out = 0.f;
  bool term = false, trunc = false, cont = false, reached = false, collided = false;
  bool term_all = false, trunc_all = false, do_reset = false;
  int new_step = stepc;
  double dist_phys = 0.0;
  if (mode == MODE_STEP) {
    if (is_agent) {
      if constexpr (DYN == DYN_KIN) {
        const float curr = sqrt_rn(sqsum_1d(__fsub_rn(gx, px), __fsub_rn(gy, py), __fsub_rn(gz, pz)));
        dist_out = curr;
        if (act) {
          reached = (double)curr <= P.goal_radius;  // fp64 compare, :124-127
          collided = coll;
          if (collided) atomicOr(&tint[1], 1);
          if (!reached && !collided) atomicAdd(&tint[2], 1);
          double r = __dmul_rn(__dsub_rn((double)prev_d, (double)curr), P.kp);
          if (n_active > 1) r = __dadd_rn(r, __dmul_rn(-P.kf, __ddiv_rn(fsum, (double)(n_active - 1))));
          if (reached) r = __dadd_rn(r, P.r_goal);
          if (collided) r = __dadd_rn(r, P.r_col);
          rew = __double2float_rn(r);
        }
      } else {
        const double dx = __dsub_rn((double)px, (double)gx);
        const double dy = __dsub_rn((double)py, (double)gy);
        const double dz = __dsub_rn((double)pz, (double)gz);
        dist_phys = dsqrt_rn(__dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz)));
        dist_out = __double2float_rn(dist_phys);
        collided = coll || (pz <= P.ground_z);
        reached = dist_phys < P.goal_radius;
        if (act) {
          if (collided) atomicOr(&tint[1], 1);
          if (!collided && !reached) atomicOr(&tint[3], 1);
          double r = __dmul_rn(-dist_phys, 0.1);
          if (collided) r = __dsub_rn(r, 10.0);
          else if (reached) r = __dadd_rn(r, 50.0);
          rew = __double2float_rn(r);
        }
      }
    }
    __syncthreads();
    const bool any_c = tint[1] != 0;
    if constexpr (DYN == DYN_KIN) {
      if (n_active == 0) {  // drone_swarm_env.py:93-95
        term_all = true;
      } else {
        new_step = stepc + 1;
        const bool tl = new_step >= P.max_steps;
        const bool all_reached = (tint[2] == 0) && !any_c && !tl;
        term_all = all_reached || any_c;
        trunc_all = tl && !term_all;
        if (act) {
          const bool done_i = reached || collided;
          term = done_i;
          trunc = tl && !done_i;
          cont = !done_i && !tl && !any_c;
        }
      }
    } else {
      new_step = stepc + 1;
      const bool tl = new_step >= P.max_steps;
      const bool all_goals = tint[3] == 0;
      const bool done = any_c || all_goals || tl;
      trunc_all = done && tl && !any_c && !all_goals;
      term_all = done && !trunc_all;
      term = term_all;
      trunc = trunc_all;
      cont = true;
    }
    do_reset = P.auto_reset && env_ok && (term_all || trunc_all);
    if (t == 0 && do_reset) atomicOr(bflag, 1);
    __syncthreads();
    if (bflag[0]) {  // block-uniform: some team re-draws its env in-kernel
      if (do_reset) {
        episode_new = S.episode[env] + 1u;
        uint32_t w[4];
        if (t < N) {
          draw_block(P, genv, episode_new, (uint32_t)t, w);
          float nx = uni(w[0], P.neg_half_w, P.width_w);
          float ny = uni(w[1], P.neg_half_w, P.width_w);
          float nz = uni(w[2], P.neg_half_w, P.width_w);
          if constexpr (DYN == DYN_PHYS) {
            nz = fmaxf(nz, 1.0f);
            damp = __fmul_rn(0.5f, uni(w[3], 0.8f, 0.4f));
          }
          px = nx; py = ny; pz = nz;
          vx = vy = vz = 0.f;
          pos4[t] = make_float4(px, py, pz, 1.f);
        }
        for (int m = t; m < M; m += L) {
          draw_block(P, genv, episode_new, (uint32_t)(N + m), w);
          float oz = uni(w[2], P.neg_half_w, P.width_w);
          if constexpr (DYN == DYN_PHYS) oz = fmaxf(oz, 0.5f);
          obst4[m] = make_float4(uni(w[0], P.neg_half_w, P.width_w), uni(w[1], P.neg_half_w, P.width_w), oz, 0.f);
        }
        draw_block(P, genv, episode_new, (uint32_t)(N + M), w);
        gx = uni(w[0], P.neg_half_w, P.width_w);
        gy = uni(w[1], P.neg_half_w, P.width_w);
        gz = uni(w[2], P.neg_half_w, P.width_w);
        if constexpr (DYN == DYN_PHYS) gz = uni(w[3], 0.5f, 1.5f);
      }
      __syncthreads();
      if (do_reset && is_agent) {
#pragma unroll
        for (int s = 0; s < (KS > 0 ? KS : 1); ++s) nk[s] = KEY_EMPTY;
#pragma unroll
        for (int s = 0; s < (MSL > 0 ? MSL : 1); ++s) ok[s] = KEY_EMPTY;
        bool c2 = false;
        double f2 = 0.0;
        neighbor_pass<KS, 0>(pos4, N, t, px, py, pz, true, 0.f, 0.0, nk, c2, f2);
        obstacle_pass<MSL, false>(obst4, M, px, py, pz, false, 0.f, ok, c2);
      }
    }
  } else if (sel && is_agent) {
    dist_out = sqrt_rn(sqsum_1d(__fsub_rn(gx, px), __fsub_rn(gy, py), __fsub_rn(gz, pz)));
  }

  // ---- observation row: [p | v | g-p | K x (p_j-p_i, d) | Ms x (o_m-p_i, d)]
  const bool write_env = (mode == MODE_STEP) ? env_ok : sel;
  if (is_agent && write_env) {
    float* row = P.stage_obs ? stage + (size_t)(team * N + t) * D : O.obs + (size_t)ag * D;
    row[0] = px; row[1] = py; row[2] = pz;
    if constexpr (DYN == DYN_PHYS) {  // velocity clamped in the obs only (drone_physics_env.py:438-442)
      const double dvx = (double)vx, dvy = (double)vy, dvz = (double)vz;
      const double nv = dsqrt_rn(__dadd_rn(__dadd_rn(__dmul_rn(dvx, dvx), __dmul_rn(dvy, dvy)), __dmul_rn(dvz, dvz)));
      if (nv > P.vmax_d) {
        row[3] = __double2float_rn(__dmul_rn(__ddiv_rn(dvx, nv), P.vmax_d));
        row[4] = __double2float_rn(__dmul_rn(__ddiv_rn(dvy, nv), P.vmax_d));
        row[5] = __double2float_rn(__dmul_rn(__ddiv_rn(dvz, nv), P.vmax_d));
      } else {
        row[3] = vx; row[4] = vy; row[5] = vz;
      }
    } else {
      row[3] = vx; row[4] = vy; row[5] = vz;
    }
    row[6] = __fsub_rn(gx, px); row[7] = __fsub_rn(gy, py); row[8] = __fsub_rn(gz, pz);
    int col = 9;
    if constexpr (KS > 0) {
      // keys were ranked by the exact float squared sum; re-rank the K+1 survivors by the exact
      // distance so (d, j) order matches the reference's argsort on d
      uint64_t k2[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s)
        k2[s] = (nk[s] == KEY_EMPTY) ? KEY_EMPTY : make_key(sqrt_rn(key_val(nk[s])), key_idx(nk[s]));
#pragma unroll
      for (int s = 1; s < KS; ++s) {
#pragma unroll
        for (int r = s; r > 0; --r) {
          const uint64_t a = k2[r - 1], b = k2[r];
          const bool sw = b < a;
          k2[r - 1] = sw ? b : a;
          k2[r] = sw ? a : b;
        }
      }
#pragma unroll
      for (int s = 0; s < KS - 1; ++s) {
        if (s < P.K) {
          float f0 = 0.f, f1 = 0.f, f2 = 0.f, f3 = 0.f;
          if (k2[s] != KEY_EMPTY) {
            const float4 q = pos4[key_idx(k2[s])];
            f0 = __fsub_rn(q.x, px); f1 = __fsub_rn(q.y, py); f2 = __fsub_rn(q.z, pz);
            f3 = key_val(k2[s]);
          }
          row[col + 4 * s + 0] = f0; row[col + 4 * s + 1] = f1;
          row[col + 4 * s + 2] = f2; row[col + 4 * s + 3] = f3;
        }
      }
    }
    col += 4 * P.K;  // neighbor_slots() guarantees KS >= K + 1
    if (P.Ms > 0) {
#pragma unroll
      for (int s = 0; s < (MSL > 0 ? MSL : 1); ++s) {
        if (s < P.Ms) {
          float f0 = 0.f, f1 = 0.f, f2 = 0.f, f3 = 0.f;
          if (MSL > 0 && ok[s] != KEY_EMPTY) {
            const float4 q = obst4[key_idx(ok[s])];
            f0 = __fsub_rn(q.x, px); f1 = __fsub_rn(q.y, py); f2 = __fsub_rn(q.z, pz);
            f3 = key_val(ok[s]);
          }
          row[col + 4 * s + 0] = f0; row[col + 4 * s + 1] = f1;
          row[col + 4 * s + 2] = f2; row[col + 4 * s + 3] = f3;
        }
      }
      for (int s = (MSL > 0 ? MSL : 1); s < P.Ms; ++s) {  // Ms > slots only when Ms > M: padding
        row[col + 4 * s + 0] = 0.f; row[col + 4 * s + 1] = 0.f;
        row[col + 4 * s + 2] = 0.f; row[col + 4 * s + 3] = 0.f;
      }
    }
  }
  if (P.stage_obs) {
    __syncthreads();
    const int teamf = N * D;
    if (mode == MODE_STEP || env_mask == nullptr) {
      // whole block region [env0, env0+nvalid) is one contiguous run of floats
      long long nvalid = P.E - env0;
      if (nvalid > G) nvalid = G;
      const long long total = nvalid * teamf;
      float* dst = O.obs + env0 * teamf;
      if (P.obs_vec4) {
        const long long n4 = total >> 2;
        const float4* s4 = reinterpret_cast<const float4*>(stage);
        float4* d4 = reinterpret_cast<float4*>(dst);
        for (long long i = tid; i < n4; i += blockDim.x) d4[i] = s4[i];
        for (long long i = (n4 << 2) + tid; i < total; i += blockDim.x) dst[i] = stage[i];
      } else {
        for (long long i = tid; i < total; i += blockDim.x) dst[i] = stage[i];
      }
    } else if (sel) {
      const float* src = stage + (size_t)team * teamf;
      float* dst = O.obs + env * teamf;
      for (int i = t; i < teamf; i += L) dst[i] = src[i];
    }
  }

  // ---- per-agent outputs and state write-back
  if (is_agent) {
    if (mode == MODE_STEP) {
      O.reward[ag] = rew;
      O.terminated[ag] = term ? 1 : 0;
      O.truncated[ag] = trunc ? 1 : 0;
      if (O.dist_goal) O.dist_goal[ag] = dist_out;
      if (O.info_flags)
        O.info_flags[ag] = (uint8_t)((act ? SWARM_AGENT_STEPPED : 0u) | (act && reached ? SWARM_AGENT_REACHED : 0u) |
                                     (act && collided ? SWARM_AGENT_COLLISION : 0u) | (cont ? SWARM_AGENT_HAS_OBS : 0u));
      bool new_act;
      if constexpr (DYN == DYN_KIN) new_act = cont;
      else new_act = act && !(term_all || trunc_all);
      if (do_reset) new_act = true;
      S.pos[ag * 3 + 0] = px; S.pos[ag * 3 + 1] = py; S.pos[ag * 3 + 2] = pz;
      S.vel[ag * 3 + 0] = vx; S.vel[ag * 3 + 1] = vy; S.vel[ag * 3 + 2] = vz;
      S.active[ag] = new_act ? 1 : 0;
      if (DYN == DYN_PHYS && do_reset) S.damping[ag] = damp;
    } else if (sel) {
      if (O.dist_goal) O.dist_goal[ag] = dist_out;
      if (mode == MODE_RESET) {
        S.pos[ag * 3 + 0] = px; S.pos[ag * 3 + 1] = py; S.pos[ag * 3 + 2] = pz;
        S.vel[ag * 3 + 0] = 0.f; S.vel[ag * 3 + 1] = 0.f; S.vel[ag * 3 + 2] = 0.f;
        S.active[ag] = 1;
        if constexpr (DYN == DYN_PHYS) S.damping[ag] = damp;
      }
    }
    if (O.global_state && write_env) {
      float* gs = O.global_state + env * (6LL * N + 3);
      gs[3 * t + 0] = px; gs[3 * t + 1] = py; gs[3 * t + 2] = pz;
      gs[3 * N + 3 * t + 0] = vx; gs[3 * N + 3 * t + 1] = vy; gs[3 * N + 3 * t + 2] = vz;
      if (t == 0) { gs[6 * N + 0] = gx; gs[6 * N + 1] = gy; gs[6 * N + 2] = gz; }
    }
  }
  const bool new_episode = (mode == MODE_STEP) ? do_reset : (mode == MODE_RESET && sel);
  if (env_ok && t == 0) {
    if (mode == MODE_STEP) {
      O.env_done[env] = (uint8_t)((term_all ? SWARM_ENV_TERMINATED : 0u) | (trunc_all ? SWARM_ENV_TRUNCATED : 0u) |
                                  (do_reset ? SWARM_ENV_RESET : 0u));
      S.step_count[env] = do_reset ? 0 : new_step;
    } else if (mode == MODE_RESET && sel) {
      S.step_count[env] = 0;
    }
    if (new_episode) {
      S.episode[env] = episode_new;
      S.goal[env * 3 + 0] = gx; S.goal[env * 3 + 1] = gy; S.goal[env * 3 + 2] = gz;
    }
  }
  if (env_ok && new_episode) {
    for (int m = t; m < M; m += L) {
      float* o = S.obstacles + (env * M + m) * 3;
      const float4 q = obst4[m];
      o[0] = q.x; o[1] = q.y; o[2] = q.z;
    }
  }
}

// ------------------------------------------------------------------ host side
thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// Largest float s >= 0 with sqrtf(s) <= T: lets the pair loop compare the exact float squared
// sum instead of taking a correctly rounded sqrt per pair, with identical outcomes.
float s_threshold(float T) {
  if (!(T >= 0.0f)) return -1.0f;
  if (isinf(T)) return INFINITY;
  float s = T * T;
  while (s > 0.0f && sqrtf(s) > T) s = nextafterf(s, -INFINITY);
  for (;;) {
    const float nx = nextafterf(s, INFINITY);
    if (isinf(nx) || sqrtf(nx) > T) break;
    s = nx;
  }
  return s;
}

int next_pow2(int n) {
  int l = 1;
  while (l < n) l <<= 1;
  return l;
}
int ilog2(int v) {
  int r = 0;
  while ((1 << r) < v) ++r;
  return r;
}
int neighbor_slots(int K) {
  if (K <= 0) return 0;
  if (K <= 3) return 4;
  if (K == 4) return 5;
  if (K <= 8) return 9;
  return 17;
}
int obstacle_slots(int Ms, int M) {
  const int need = Ms < M ? Ms : M;
  if (need <= 0) return 0;
  if (need <= 4) return 4;
  if (need <= 8) return 8;
  return 16;
}

int obs_dim_of(const swarm_params_t* p) {
  return 9 + 4 * (p->neighbor_k > 0 ? p->neighbor_k : 0) + 4 * (p->sensed_obstacles > 0 ? p->sensed_obstacles : 0);
}

int build_kparams(const swarm_params_t* p, KParams* kp, swarm_launch_info_t* info) {
  if (!p) return fail(SWARM_ENULL, "params is NULL");
  if (p->abi_version != SWARM_ABI_VERSION)
    return fail(SWARM_EINVAL, "abi_version %d != library %d", p->abi_version, SWARM_ABI_VERSION);
  if (p->num_envs < 0) return fail(SWARM_EINVAL, "num_envs must be >= 0 (got %d)", p->num_envs);
  if (p->num_drones < 1 || p->num_drones > MAX_N)
    return fail(SWARM_ELIMIT, "num_drones must be in [1, %d] (got %d)", MAX_N, p->num_drones);
  if (p->num_obstacles < 0) return fail(SWARM_EINVAL, "num_obstacles must be >= 0");
  if (p->neighbor_k > MAX_K) return fail(SWARM_ELIMIT, "neighbor_k > %d unsupported (got %d)", MAX_K, p->neighbor_k);
  const int msn = p->sensed_obstacles < p->num_obstacles ? p->sensed_obstacles : p->num_obstacles;
  if (msn > MAX_MS) return fail(SWARM_ELIMIT, "sensed_obstacles > %d unsupported (got %d)", MAX_MS, p->sensed_obstacles);
  if (p->dynamics != DYN_KIN && p->dynamics != DYN_PHYS) return fail(SWARM_EINVAL, "unknown dynamics %d", p->dynamics);
  if (p->reward_mode != SWARM_REW_SWARM && p->reward_mode != SWARM_REW_PHYSICS)
    return fail(SWARM_EINVAL, "unknown reward_mode %d", p->reward_mode);
  if ((p->dynamics == DYN_KIN) != (p->reward_mode == SWARM_REW_SWARM))
    return fail(SWARM_EINVAL, "dynamics/reward_mode pairing must be kinematic+swarm or physics+physics");
  if (p->dynamics == DYN_PHYS && p->physics_substeps < 0) return fail(SWARM_EINVAL, "physics_substeps < 0");
  if (p->damping_law != 0 && p->damping_law != 1) return fail(SWARM_EINVAL, "damping_law must be 0 or 1");

  KParams k;
  memset(&k, 0, sizeof(k));
  k.E = p->num_envs;
  k.N = p->num_drones;
  k.M = p->num_obstacles;
  k.K = p->neighbor_k > 0 ? p->neighbor_k : 0;
  k.Ms = p->sensed_obstacles > 0 ? p->sensed_obstacles : 0;
  k.D = obs_dim_of(p);
  k.max_steps = p->max_steps;
  k.reward_mode = p->reward_mode;
  k.auto_reset = p->auto_reset ? 1 : 0;
  k.substeps = p->physics_substeps;
  k.damping_law = p->damping_law;
  k.lanes = next_pow2(k.N);
  k.log2_lanes = ilog2(k.lanes);
  const int threads = k.lanes >= 256 ? k.lanes : 256;
  k.envs_per_block = threads / k.lanes;
  const int G = k.envs_per_block;
  k.pos_stride = k.N + 1;
  k.obst_stride = k.M + 1;
  const int pos_bytes = G * k.pos_stride * 16;
  k.off_obst = pos_bytes;
  k.off_team = k.off_obst + G * k.obst_stride * 16;
  k.off_block = k.off_team + G * 16;
  k.off_stage = k.off_block + 16;
  const long long stage_bytes = (long long)G * k.N * k.D * 4;
  long long lds = k.off_stage;
  k.stage_obs = (lds + stage_bytes) <= STAGE_LDS_BUDGET ? 1 : 0;
  if (k.stage_obs) lds += stage_bytes;
  if (lds > LDS_LIMIT) return fail(SWARM_ELIMIT, "LDS footprint %lld B exceeds %d B (N=%d, M=%d)", lds, LDS_LIMIT, k.N, k.M);
  k.obs_vec4 = (((long long)G * k.N * k.D) % 4 == 0) ? 1 : 0;
  k.env_offset = p->env_offset;
  k.seed_lo = (unsigned)(p->seed & 0xffffffffull);
  k.seed_hi = (unsigned)(p->seed >> 32);
  k.half_w = (float)(p->world_size / 2.0);
  k.neg_half_w = (float)(-p->world_size / 2.0);
  k.width_w = (float)p->world_size;
  k.dt = (float)p->dt;
  k.vmax = (float)p->max_speed;
  k.amax = (float)p->max_accel;
  k.eps_speed = (float)1e-8;
  k.s_pair = s_threshold((float)(2.0 * p->collision_radius));
  k.s_obst = s_threshold((float)(p->collision_radius + p->obstacle_radius));
  k.s_phys_pair = s_threshold((float)(2.0 * p->drone_contact_radius));
  k.s_phys_obst = s_threshold((float)(p->obstacle_radius + p->drone_contact_radius));
  k.ground_z = (float)p->ground_contact_height;
  k.h = (float)p->substep_dt;
  k.g = (float)p->gravity;
  k.gcomp = (float)p->gravity_comp;
  k.goal_radius = p->goal_radius;
  k.desired_spacing = p->desired_spacing;
  k.kp = p->reward_progress_scale;
  k.r_goal = p->reward_goal;
  k.r_col = p->reward_collision;
  k.kf = p->reward_formation_scale;
  k.vmax_d = p->max_speed;
  *kp = k;
  if (info) {
    info->threads_per_block = threads;
    info->envs_per_block = G;
    info->lanes_per_env = k.lanes;
    info->blocks = (int)((k.E + G - 1) / G);
    info->lds_bytes = (int)lds;
    info->neighbor_slots = neighbor_slots(k.K);
    info->obstacle_slots = obstacle_slots(k.Ms, k.M);
    info->obs_dim = k.D;
    info->staged_obs = k.stage_obs;
  }
  return SWARM_OK;
}

typedef void (*kernel_fn)(const KParams, const swarm_state_t, const float*, const uint8_t*, const swarm_out_t,
                          const uint8_t*, int);

template <int DYN, int KS>
kernel_fn pick_ms(int msl) {
  switch (msl) {
    case 0: return swarm_kernel<DYN, KS, 0>;
    case 4: return swarm_kernel<DYN, KS, 4>;
    case 8: return swarm_kernel<DYN, KS, 8>;
    default: return swarm_kernel<DYN, KS, 16>;
  }
}
template <int DYN>
kernel_fn pick_ks(int ks, int msl) {
  switch (ks) {
    case 0: return pick_ms<DYN, 0>(msl);
    case 4: return pick_ms<DYN, 4>(msl);
    case 5: return pick_ms<DYN, 5>(msl);
    case 9: return pick_ms<DYN, 9>(msl);
    default: return pick_ms<DYN, 17>(msl);
  }
}

int launch(int mode, const swarm_params_t* p, const swarm_state_t* s, const float* actions, const uint8_t* amask,
           const uint8_t* env_mask, const swarm_out_t* o, void* stream) {
  KParams kp;
  swarm_launch_info_t info;
  int rc = build_kparams(p, &kp, &info);
  if (rc) return rc;
  if (!s || !o) return fail(SWARM_ENULL, "state/out is NULL");
  if (kp.E == 0) return SWARM_OK;
  if (!s->pos || !s->vel || !s->goal || !s->active || !s->step_count || !s->episode)
    return fail(SWARM_ENULL, "state buffer is NULL (pos/vel/goal/active/step_count/episode required)");
  if (kp.M > 0 && !s->obstacles) return fail(SWARM_ENULL, "state.obstacles is NULL with num_obstacles > 0");
  if (p->dynamics == DYN_PHYS && !s->damping) return fail(SWARM_ENULL, "state.damping is NULL in physics mode");
  if (!o->obs) return fail(SWARM_ENULL, "out.obs is NULL");
  if (mode == MODE_STEP) {
    if (!actions) return fail(SWARM_ENULL, "actions is NULL");
    if (!o->reward || !o->terminated || !o->truncated || !o->env_done)
      return fail(SWARM_ENULL, "out.reward/terminated/truncated/env_done required by swarm_step");
  }
  if (((uintptr_t)o->obs) % 16 != 0) kp.obs_vec4 = 0;
  kernel_fn fn = (p->dynamics == DYN_KIN) ? pick_ks<DYN_KIN>(info.neighbor_slots, info.obstacle_slots)
                                          : pick_ks<DYN_PHYS>(info.neighbor_slots, info.obstacle_slots);
  if (info.lds_bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       info.lds_bytes);
    if (e != hipSuccess) return fail(SWARM_EHIP, "hipFuncSetAttribute: %s", hipGetErrorString(e));
  }
  hipLaunchKernelGGL(fn, dim3(info.blocks), dim3(info.threads_per_block), info.lds_bytes, (hipStream_t)stream, kp,
                     *s, actions, amask, *o, env_mask, mode);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(SWARM_EHIP, "kernel launch: %s", hipGetErrorString(e));
  return SWARM_OK;
}

}  // namespace

extern "C" {

int swarm_abi_version(void) { return SWARM_ABI_VERSION; }

const char* swarm_last_error(void) { return g_err; }

void swarm_params_default(swarm_params_t* p) {
  if (!p) return;
  memset(p, 0, sizeof(*p));
  p->abi_version = SWARM_ABI_VERSION;
  p->num_envs = 1;
  p->num_drones = 3;
  p->num_obstacles = 8;
  p->sensed_obstacles = 4;
  p->neighbor_k = 3;
  p->max_steps = 400;
  p->dynamics = SWARM_DYN_KINEMATIC;
  p->reward_mode = SWARM_REW_SWARM;
  p->auto_reset = 0;
  p->physics_substeps = 24;
  p->damping_law = 0;
  p->env_offset = 0;
  p->seed = 0;
  p->world_size = 20.0;
  p->dt = 0.1;
  p->max_speed = 4.0;
  p->max_accel = 2.0;
  p->collision_radius = 0.5;
  p->goal_radius = 0.8;
  p->obstacle_radius = 0.8;
  p->desired_spacing = 2.5;
  p->reward_progress_scale = 2.0;
  p->reward_goal = 25.0;
  p->reward_collision = -25.0;
  p->reward_formation_scale = 0.15;
  p->gravity = -9.81;
  p->gravity_comp = 9.5;
  p->substep_dt = 1.0 / 240.0;
  p->drone_contact_radius = 0.15;
  p->ground_contact_height = 0.025;
}

int swarm_obs_dim(const swarm_params_t* p) {
  if (!p) return fail(SWARM_ENULL, "params is NULL");
  return obs_dim_of(p);
}

int swarm_query_launch(const swarm_params_t* p, swarm_launch_info_t* info) {
  KParams kp;
  if (!info) return fail(SWARM_ENULL, "info is NULL");
  return build_kparams(p, &kp, info);
}

int swarm_step(const swarm_params_t* p, const swarm_state_t* s, const float* actions, const uint8_t* action_mask,
               const swarm_out_t* o, void* hip_stream) {
  return launch(MODE_STEP, p, s, actions, action_mask, nullptr, o, hip_stream);
}

int swarm_reset(const swarm_params_t* p, const swarm_state_t* s, const uint8_t* env_mask, const swarm_out_t* o,
                void* hip_stream) {
  return launch(MODE_RESET, p, s, nullptr, nullptr, env_mask, o, hip_stream);
}

int swarm_observe(const swarm_params_t* p, const swarm_state_t* s, const uint8_t* env_mask, const swarm_out_t* o,
                  void* hip_stream) {
  return launch(MODE_OBSERVE, p, s, nullptr, nullptr, env_mask, o, hip_stream);
}

}  // extern "C"
