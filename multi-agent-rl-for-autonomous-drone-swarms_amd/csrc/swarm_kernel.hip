// swarm_kernel.hip — fused swarm step / reset / observe kernels for gfx950 (MI355X, CDNA4),
// plus the C-ABI entry points declared in include/swarm_mi355x.h.
//
// A "team" of L = next_pow2(N) lanes owns one env (one lane per drone).
//   WAVE kernel  (L <= 64): 64-thread workgroups = one wave holding G = 64/L teams.  The N x N
//                pair pass is symmetric: at rotation r lane t evaluates drone t+r and receives,
//                by ds_bpermute, the value lane t-r evaluated for the pair (t-r, t).  Team
//                reductions are wave ballots.
//   BLOCK kernel (L > 64): one env per workgroup of L threads; ascending broadcast pair loop.
// Step and reset/observe are separate instantiations (KIND) so the step kernel carries no
// dead paths (SGPR pressure).
//
// Ranking vs exactness.  The reference's neighbour distance is
//   d = sqrtf((float)(((double)(x*x) + (double)(y*y)) + (double)(z*z)))   (OpenBLAS sdot)
// The pair loop ranks with the cheaper all-float sum s' = ((x*x)+(y*y))+(z*z), which is within
// 2^-21 relative of the exact s (or with d~ = v_sqrt_f32(s') in the kinematic step, whose
// formation term needs it anyway).  Neighbours are kept as packed 32-bit keys (float bits of the
// ranking value with the low bits replaced by the neighbour index / rotation offset; one
// v_med3_u32 per slot and insert).  The
// K+1 survivors are re-ranked with the exact d; a lower bound on every non-survivor proves the
// top-K exact, else an exact selection runs (rare).  Pair collisions compare the exact nearest
// distance (all-eligible fast path) or an error-banded running minimum with exact re-check.
//
// Bit-exactness: no FP contraction, IEEE sqrt/div where the reference's value is
// observable, the sdot double-accumulated norm for 1-D norms and the float axis norm for obstacles.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <type_traits>

#include "swarm_mi355x.h"

#pragma clang fp contract(off)

// Build partitioning: the kernel instantiations are compiled as parallel translation units.
// SWARM_PART k in 0..3 holds the kernels of (KIND, DYN) = (k >> 1, k & 1); SWARM_PART 4 holds
// the host side and the C-ABI; SWARM_PART 5 the headline specialisation swarm_step64; SWARM_PART 6
// the config-2 specialisation swarm_step16q; SWARM_PART 7 the config-5 specialisation swarm_step256;
// SWARM_PART -1 (default) is everything in one unit (tools/).
#ifndef SWARM_PART
#define SWARM_PART -1
#endif
#define SWARM_HAS_PART(k) (SWARM_PART == -1 || SWARM_PART == (k))
#define SWARM_HAS_HOST (SWARM_PART == -1 || SWARM_PART == 4)
// the generic kernel's instantiations (parts 0-3)
#define SWARM_PARTS_GENERIC (SWARM_HAS_PART(0) || SWARM_HAS_PART(1) || SWARM_HAS_PART(2) || SWARM_HAS_PART(3))

// Diagnostic phase timestamps (tools/stamps.py; never set in the product build)
#include "swarm_stamps.h"  // diagnostic phase stamps (empty unless -DSWARM_STAMPS)

// Tuning constants (each measured against its alternatives)
constexpr int FB_BATCH = 8;            // exact scans: LDS reads in flight per batch
constexpr int S64_PAIR_BATCH = 4;      // step64 pair pass: rotations per scheduling group
#ifndef SWARM_S64_F32SUM
#define SWARM_S64_F32SUM 1  // step64 formation sum: one f32 chain per pass, widened once
#endif
#ifndef SWARM_OBST_OMIN
#define SWARM_OBST_OMIN 1  // obstacle passes: collisions from the running minimum (no exec-mask chain)
#endif
#ifndef SWARM_S64_BIGSQRT
#define SWARM_S64_BIGSQRT 1  // step64 finish: square roots without the tiny-input branch when the keys prove it
#endif
constexpr int S64_CH_ROWS = 32;        // step64 obs rows per LDS staging chunk
constexpr int S64_WG_ENVS_C = 4;       // step64: one-env waves per workgroup
constexpr int S64_EVAL_WAVES = 8;      // step64 with the fused eval: waves per EU
[[maybe_unused]] constexpr int Q16_WAVES_PER_EU = 4;    // step16q register budget (71 VGPRs, no spills)
constexpr int H_BATCH_C = 8;           // step256 passes: rotations per scheduling batch
constexpr bool WT_STORES = true;       // obs rows as write-through (sc1) buffer stores
constexpr int OBS_STORE_AUX = 16;      // their cache-policy bits (16 = sc1)

// Device helpers (structs, constants, inline functions) live in namespace swarm_dev: inline functions
// with external linkage, so a helper that one translation unit (SWARM_PART) does not use is neither
// emitted nor warned about.  The kernels are in anonymous namespaces (each translation unit's own).
namespace swarm_dev {}
using namespace swarm_dev;
namespace swarm_dev {

constexpr uint32_t KEY_EMPTY = 0xffffffffu;
constexpr int MODE_STEP = 0;
constexpr int MODE_RESET = 1;
constexpr int MODE_OBSERVE = 2;
constexpr int KIND_STEP = 0;
[[maybe_unused]] constexpr int KIND_AUX = 1;  // reset / observe
constexpr int DYN_KIN = SWARM_DYN_KINEMATIC;
constexpr int DYN_PHYS = SWARM_DYN_POINTMASS_PHYSICS;
[[maybe_unused]] constexpr int MAX_N = 1024;
[[maybe_unused]] constexpr int MAX_K = 16;
[[maybe_unused]] constexpr int MAX_MS = 16;
[[maybe_unused]] constexpr int STAGE_BUDGET = 8 * 1024;  // bytes of LDS for one obs staging chunk
[[maybe_unused]] constexpr int LDS_LIMIT = 160 * 1024;
constexpr float PAD_POS = 1e18f;        // position of padding lanes (t >= N): never a neighbour
constexpr float FAST_LO = 1.0f - 0x1p-18f;  // |s' - s| <= 2^-21 s; bands use an 8x margin
constexpr float FAST_HI = 1.0f + 0x1p-18f;

// Derived, launch-ready parameters (host computes once per call).
struct KParams {
  int E, N, M, K, Ms, D, max_steps, auto_reset, substeps, damping_law;
  int log2_lanes, envs_per_block, chunk_rows, obs_vec4, pack_bytes;
  int off_obst, off_stage, obst_stride, ring;   // ring: pos4 slots per team (2L wave, L block)
  int off_pair;   // block teams with N a power of two: pair-entry ring (BLK_PAIR_STRIDE floats x 2N)
  int obs_direct;  // multi-team wave kernels: obs rows stored from registers (no LDS staging)
  uint32_t nb_keep, ob_keep;        // key masks: high bits kept from the distance, low bits = index
  long long env_offset;
  unsigned seed_lo, seed_hi;
  float half_w, neg_half_w, width_w;
  float dt, vmax, amax, ds_f, s_vmax;  // s_vmax: largest s with sqrt_rn(s) <= vmax
  float thr_pair, s_pair, s_obst;   // kinematic: distance threshold, squared-space thresholds
  float thr_ppair, s_phys_pair, s_phys_obst, ground_z;
  float h, g, gcomp;
  float s_goal;  // largest s with (double)sqrt_rn(s) <= goal_radius (step16q's reached test)
  double goal_radius, kp, r_goal, r_col, kf, vmax_d;
};

// The launch-uniform parameters as a per-env record (swarm_env_cfg_t: what swarm_env_cfg_set
// derives from the same values, field for field).
__device__ __forceinline__ swarm_env_cfg_t uniform_env_cfg(const KParams& P) {
  swarm_env_cfg_t c;
  c.half_w = P.half_w;
  c.neg_half_w = P.neg_half_w;
  c.width_w = P.width_w;
  c.dt = P.dt;
  c.max_speed = P.vmax;
  c.max_accel = P.amax;
  c.s_vmax = P.s_vmax;
  c.s_obst = P.s_obst;
  c.s_phys_obst = P.s_phys_obst;
  c.max_steps = P.max_steps;
  c.num_obstacles = P.M;
  c.reserved = 0;
  c.max_speed_d = P.vmax_d;
  c.world_size = 0.0;
  return c;
}
__device__ __forceinline__ int clamp_obstacles(int m, int M) { return m < 0 ? 0 : (m > M ? M : m); }

// ------------------------------------------------------------------ exact numerics
// Correctly rounded square roots.  NB: HIP's __fsqrt_rn is v_sqrt_f32 (1 ulp) unless
// OCML_BASIC_ROUNDED_OPERATIONS is defined; llvm.sqrt lowers to the IEEE-exact sequence.
// The fast path is OCML's own correction step without its input scaling (needed only below
// 2^-96) and special-value fixup (inf/NaN/negative never occur here): bit-identical results.
__device__ __forceinline__ float sqrt_rn(float x) {
  if (__builtin_expect(__ballot(!(x >= 0x1p-96f || x == 0.0f)) != 0, 0)) return __builtin_sqrtf(x);
  float r = __builtin_amdgcn_sqrtf(x);  // v_sqrt_f32, within 1 ulp
  const float rm = __uint_as_float(__float_as_uint(r) - 1u), rp = __uint_as_float(__float_as_uint(r) + 1u);
  const float em = __builtin_fmaf(-rm, r, x), ep = __builtin_fmaf(-rp, r, x);
  r = (em <= 0.0f) ? rm : r;
  r = (ep > 0.0f) ? rp : r;
  return r;
}

// sqrt_rn's fast path alone, for branch-free loops: `tiny` records an input below 2^-96 (the
// caller redoes the loop with sqrt_rn when any lane saw one; the value returned then is unused)
__device__ __forceinline__ float sqrt_rn_nb(float x, bool& tiny) {
  tiny = tiny | !(x >= 0x1p-96f || x == 0.0f);
  float r = __builtin_amdgcn_sqrtf(x);
  const float rm = __uint_as_float(__float_as_uint(r) - 1u), rp = __uint_as_float(__float_as_uint(r) + 1u);
  const float em = __builtin_fmaf(-rm, r, x), ep = __builtin_fmaf(-rp, r, x);
  r = (em <= 0.0f) ? rm : r;
  r = (ep > 0.0f) ? rp : r;
  return r;
}
// sqrt_rn for an input the caller proved is 0 or >= 2^-96 (no slow-path test, no branch)
__device__ __forceinline__ float sqrt_rn_big(float x) {
  bool unused = false;
  return sqrt_rn_nb(x, unused);
}
__device__ __forceinline__ double dsqrt_rn(double x) { return __builtin_sqrt(x); }
// np.linalg.norm(v) of a float32 3-vector: OpenBLAS sdot = double accumulation of float
// products, rounded to float.  Returns the float sum s; the norm is sqrt_rn(s).
__device__ __forceinline__ float sqsum_1d(float x, float y, float z) {
  const float xx = x * x, yy = y * y, zz = z * z;
  return (float)(((double)xx + (double)yy) + (double)zz);
}
// np.linalg.norm(A, axis=1): float32 ((x*x)+(y*y))+(z*z).
__device__ __forceinline__ float sqsum_f(float x, float y, float z) { return ((x * x) + (y * y)) + (z * z); }
// The 64-lane pair passes' ranking value s': FMA-contracted (3 VALU instead of 5), within two
// roundings of the exact sum.  Every use is banded (2^-18 >> 2^-21) or re-checked with the exact
// norms (keys -> finish_keys, running minimum -> exact_pair_collision, formation -> 1e-5 reward
// contract), so it need not reproduce the reference's bits.
__device__ __forceinline__ float sqsum_rank(float x, float y, float z) {
  return __builtin_fmaf(z, z, __builtin_fmaf(y, y, x * x));
}
// A float4 gathered from LDS whose .w the caller ignores: the compiler would read the 12 used bytes
// with ds_read_b96, banked (a/4) mod 32 in 8-lane groups, so two 16-B entries 128 B apart collide
// (obstacle j and j + 8).  Keeping .w alive makes it one ds_read_b128, banked (a/4) mod 64 in
// 16-lane groups: the 16-entry obstacle table is one bank row, conflict-free.
__device__ __forceinline__ float4 lds_f4(const float4* __restrict__ p) {
  const float4 q = *p;
  asm volatile("" ::"v"(q.w));
  return q;
}
// Whole-wave rotate by one lane (DPP wave_ror:1, gfx9): lane i receives lane i-1's value.
__device__ __forceinline__ float wave_ror1(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x13C, 0xF, 0xF, false));
}

// A missing agent's action is zero (drone_swarm_env.py:104): the three components ANDed with a lane
// mask (one select + three full-rate v_and_b32).  `if (!has) a = 0` compiled to three e32 v_cndmask
// reading VCC, and runs of those issue ~7 ns apart per SIMD against ~2 for the e64 form
// (tools/valu_rate6.hip, profiles/r06d_valu_rate6.txt); the mask is opaque so the AND is not folded
// back into the selects.  Bitwise the same values (+0 for a missing agent).  Off by default: three
// same-box pairs each (profiles/r06k_act_mask_ab.jsonl) put the headline default command 0.1 us slower
// with the mask and configs 2 / driver within noise; the run of three cndmasks sits once per wave
// where the scheduler hides it.
#ifndef SWARM_ACT_MASK
#define SWARM_ACT_MASK 0
#endif
__device__ __forceinline__ void zero_unless(bool has, float& ax, float& ay, float& az) {
  if constexpr (SWARM_ACT_MASK) {
    uint32_t m = has ? 0xffffffffu : 0u;
    asm volatile("" : "+v"(m));
    ax = __uint_as_float(__float_as_uint(ax) & m);
    ay = __uint_as_float(__float_as_uint(ay) & m);
    az = __uint_as_float(__float_as_uint(az) & m);
  } else if (!has) {
    ax = 0.f; ay = 0.f; az = 0.f;
  }
}
// np.clip of a float32 in [lo, hi] (lo <= hi): one v_med3_f32
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// 1/n for the formation mean (np.mean over the n_active - 1 partner terms): v_rcp_f32 (1 ulp)
// instead of an f64 division; the mean is then within ~1e-7 relative, inside the 1e-5 reward
// contract (the terms themselves carry d~ = v_sqrt_f32 distances).
__device__ __forceinline__ double inv_count(int n) { return (double)__builtin_amdgcn_rcpf((float)n); }
// Insert key into the ascending list k[0..S-1] (drops the largest): one med3 per slot.
template <int S>
__device__ __forceinline__ void kins(uint32_t (&k)[S], uint32_t key) {
#pragma unroll
  for (int s = S - 1; s > 0; --s) k[s] = med3u(k[s - 1], key, k[s]);
  k[0] = min(k[0], key);
}

// kins into a list whose slots `filled` .. S-1 still hold KEY_EMPTY (`filled` must fold to a
// constant): those slots stay empty, slot `filled` takes max(k[filled-1], key) — the med3 / min
// against KEY_EMPTY that kins would issue are skipped (same list, fewer instructions).
template <int S>
__device__ __forceinline__ void kins_n(uint32_t (&k)[S], uint32_t key, int filled) {
  if (filled >= S) {
    kins<S>(k, key);
    return;
  }
  if (filled == 0) {
    k[0] = key;
    return;
  }
#pragma unroll
  for (int s = S - 1; s > 0; --s) {
    if (s == filled) k[s] = max(k[s - 1], key);
    else if (s < filled) k[s] = med3u(k[s - 1], key, k[s]);
  }
  k[0] = min(k[0], key);
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
  const float u = (float)(x >> 8) * 0x1p-24f;
  return lo + u * width;
}
__device__ __forceinline__ void draw_block_k(uint32_t k0, uint32_t k1, long long genv, uint32_t episode,
                                             uint32_t block, uint32_t (&w)[4]) {
  w[0] = block;
  w[1] = episode;
  w[2] = (uint32_t)((unsigned long long)genv & 0xffffffffull);
  w[3] = (uint32_t)((unsigned long long)genv >> 32);
  philox4x32_10(w, k0, k1);
}
__device__ __forceinline__ void draw_block(const KParams& P, long long genv, uint32_t episode,
                                           uint32_t block, uint32_t (&w)[4]) {
  w[0] = block;
  w[1] = episode;
  w[2] = (uint32_t)((unsigned long long)genv & 0xffffffffull);
  w[3] = (uint32_t)((unsigned long long)genv >> 32);
  philox4x32_10(w, P.seed_lo, P.seed_hi);
}

// ------------------------------------------------------------------ pair passes
// PASS 0: kNN keys only.  PASS 1: kinematic (+ formation sum, + running min of d~ over
// active pairs unless FAST).  PASS 2: physics (+ running min over real drones unless FAST).
// FAST: every drone of the wave's teams is eligible (all active / all real, N == L): no masks,
// pair collisions are decided from the exact nearest neighbour after the pass.
// `self` = this drone's eligibility; ring[j].w carries drone j's.
//
// Wave teams: at rotation r lane t evaluates the pair (t, t+r) once for both drones.  Keys carry
// the rotation offset (r for the own side, L-r for the mirror), a lane-independent constant; the
// neighbour is drone (t + offset) mod L.  The mirror receives the pair value by ds_bpermute (sign
// bit = sender eligibility).
// Pair value space: PASS 1 (kinematic step) ranks and exchanges d~ = v_sqrt_f32(s'), monotone in
// s' and within 2^-21 relative of the reference distance, because the formation term needs d
// for both drones of the pair; PASS 0/2 rank by s' (no sqrt at all).  finish_keys and the banded
// collision test take the space into account.
template <int PASS>
__device__ __forceinline__ float pair_value(float s) {
  if constexpr (PASS == 1) return __builtin_amdgcn_sqrtf(s);
  else return s;
}
template <int KS, int PASS, bool FAST>
__device__ __forceinline__ uint32_t own_pair(uint32_t (&nk)[KS > 0 ? KS : 1], float s, uint32_t low, bool pr,
                                             uint32_t keep, float ds, float& smin, float& esum, float& term) {
  const float v = pair_value<PASS>(s);
  if constexpr (KS > 0) kins<KS>(nk, (__float_as_uint(v) & keep) | low);
  if constexpr (PASS != 0 && (!FAST || KS == 0)) smin = fminf(smin, (FAST || pr) ? v : __builtin_inff());
  if constexpr (PASS == 1) {
    // formation uses d_ij widened to double in the reference; d~ keeps the mean within ~1e-6
    // relative, far inside the 1e-5 reward contract.
    float e = fabsf(v - ds);
    if constexpr (!FAST) e = pr ? e : 0.f;
    esum += e;
    term = e;
  }
  return __float_as_uint(v);
}
template <int KS, int PASS, bool FAST>
__device__ __forceinline__ uint32_t own_pair(uint32_t (&nk)[KS > 0 ? KS : 1], float s, uint32_t low, bool pr,
                                             uint32_t keep, float ds, float& smin, float& esum) {
  float term;
  return own_pair<KS, PASS, FAST>(nk, s, low, pr, keep, ds, smin, esum, term);
}
template <int KS, int PASS, bool FAST, bool FORM = true>
__device__ __forceinline__ void mirror_pair(uint32_t (&nk)[KS > 0 ? KS : 1], uint32_t rcv, uint32_t low, bool self,
                                            uint32_t keep_m, float ds, float& smin, float& esum) {
  const float v = __uint_as_float(rcv & 0x7fffffffu);
  const bool pr = FAST || (self && !(rcv >> 31));
  if constexpr (KS > 0) kins<KS>(nk, (rcv & keep_m) | low);
  if constexpr (PASS != 0 && (!FAST || KS == 0)) smin = fminf(smin, pr ? v : __builtin_inff());
  if constexpr (PASS == 1 && FORM) {
    float e = fabsf(v - ds);
    if constexpr (!FAST) e = pr ? e : 0.f;
    esum += e;
  }
}

// General wave team (L = 2..64, G = 64/L teams per wave).
template <int KS, int PASS, bool FAST>
__device__ __forceinline__ void pair_pass_wave(const float4* __restrict__ ring, int L, int t, int tid, float px,
                                               float py, float pz, bool self, uint32_t keep, float ds,
                                               uint32_t (&nk)[KS > 0 ? KS : 1], float& smin, double& fsum) {
  const int half = L >> 1;
  if (half == 0) return;
  const uint32_t sflag = (FAST || self) ? 0u : 0x80000000u;
  const uint32_t keep_m = keep & 0x7fffffffu;
  const uint32_t lm4 = (uint32_t)(L - 1) << 2;
  const uint32_t tid4 = (uint32_t)tid << 2;
  const uint32_t hi4 = tid4 & ~lm4;
  const uint32_t Lu = (uint32_t)L;
  const float4* q0 = ring + t;  // ring holds drone j at j and j + L
  // Rotations 1 .. half-1 carry a mirror, processed two at a time so that two independent
  // distance chains and two ds_bpermutes are in flight together.
  int r = 1;
  for (; r + 1 < half; r += 2) {
    const float4 qa = q0[r];
    const float4 qb = q0[r + 1];
    const float sa = sqsum_f(qa.x - px, qa.y - py, qa.z - pz);
    const float sb = sqsum_f(qb.x - px, qb.y - py, qb.z - pz);
    const uint32_t srca = ((tid4 - ((uint32_t)r << 2)) & lm4) | hi4;  // lane (t - r) mod L
    const uint32_t srcb = ((tid4 - ((uint32_t)(r + 1) << 2)) & lm4) | hi4;
    float esum = 0.f;
    const uint32_t va = own_pair<KS, PASS, FAST>(nk, sa, (uint32_t)r, self && (qa.w != 0.f), keep, ds, smin, esum);
    const uint32_t vb = own_pair<KS, PASS, FAST>(nk, sb, (uint32_t)(r + 1), self && (qb.w != 0.f), keep, ds, smin, esum);
    const uint32_t ra = (uint32_t)__builtin_amdgcn_ds_bpermute((int)srca, (int)(va | sflag));
    const uint32_t rb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)srcb, (int)(vb | sflag));
    mirror_pair<KS, PASS, FAST>(nk, ra, Lu - (uint32_t)r, self, keep_m, ds, smin, esum);
    mirror_pair<KS, PASS, FAST>(nk, rb, Lu - (uint32_t)(r + 1), self, keep_m, ds, smin, esum);
    if constexpr (PASS == 1) fsum += (double)esum;
  }
  float esum = 0.f;
  if (r < half) {  // odd leftover rotation with a mirror
    const float4 qa = q0[r];
    const float sa = sqsum_f(qa.x - px, qa.y - py, qa.z - pz);
    const uint32_t srca = ((tid4 - ((uint32_t)r << 2)) & lm4) | hi4;
    const uint32_t va = own_pair<KS, PASS, FAST>(nk, sa, (uint32_t)r, self && (qa.w != 0.f), keep, ds, smin, esum);
    const uint32_t ra = (uint32_t)__builtin_amdgcn_ds_bpermute((int)srca, (int)(va | sflag));
    mirror_pair<KS, PASS, FAST>(nk, ra, Lu - (uint32_t)r, self, keep_m, ds, smin, esum);
  }
  // r = L/2 pairs t with t+L/2 from both sides: own evaluation only
  const float4 qh = q0[half];
  const float sh = sqsum_f(qh.x - px, qh.y - py, qh.z - pz);
  own_pair<KS, PASS, FAST>(nk, sh, (uint32_t)half, self && (qh.w != 0.f), keep, ds, smin, esum);
  if constexpr (PASS == 1) fsum += (double)esum;
}

// One team per wave (L = 64): fully unrolled, every LDS / ds_bpermute address is the lane's
// base plus an immediate offset (ds_bpermute takes the source lane modulo 64).  Rotations
// 31 .. 1 (the ones with a mirror) run in descending groups of NB: ring reads, distances and
// ds_bpermutes of a group are in flight together.  The mirror keys travel by ds_bpermute; the
// mirror formation terms do not: the pair term is symmetric (masked by both drones'
// eligibility, which the sender knows from the ring), so it rides a traveling f32 sum `macc`
// that rotates one lane per rotation (DPP wave_ror:1, macc = ror(macc) + T_r for r = 31 .. 1,
// then one more ror): the term of pair (t, t+r) lands on lane t+r.  1 VALU per pair instead of 2
// on the receiving side.  Own terms are summed in f32 per group, then added in f64.
template <int KS, int PASS, bool FAST, int RT, int NB, bool MIRROR>
__device__ __forceinline__ void pair_group_w64(const float4* __restrict__ q0, uint32_t t4, float px, float py, float pz,
                                               bool self, uint32_t sflag, uint32_t keep, uint32_t keep_m, float ds,
                                               uint32_t (&nk)[KS > 0 ? KS : 1], float& smin, double& fsum,
                                               float& macc) {
  float4 q[NB];
  float sq[NB], term[NB];
  uint32_t v[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) q[i] = q0[RT - i];
#pragma unroll
  for (int i = 0; i < NB; ++i) sq[i] = sqsum_rank(q[i].x - px, q[i].y - py, q[i].z - pz);
  float esum = 0.f;
#pragma unroll
  for (int i = 0; i < NB; ++i)
    v[i] = own_pair<KS, PASS, FAST>(nk, sq[i], (uint32_t)(RT - i), self & (q[i].w != 0.f), keep, ds, smin, esum,
                                    term[i]);
  if constexpr (MIRROR) {
    uint32_t rc[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i)
      rc[i] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(t4 + (uint32_t)(256 - 4 * (RT - i))), (int)(v[i] | sflag));
#pragma unroll
    for (int i = 0; i < NB; ++i)
      mirror_pair<KS, PASS, FAST, false>(nk, rc[i], (uint32_t)(64 - RT + i), self, keep_m, ds, smin, esum);
    if constexpr (PASS == 1) {
#pragma unroll
      for (int i = 0; i < NB; ++i) macc = wave_ror1(macc) + term[i];
    }
  }
  if constexpr (PASS == 1) fsum += (double)esum;
}
template <int KS, int PASS, bool FAST, int RT, int B>
__device__ __forceinline__ void pair_groups_w64(const float4* __restrict__ q0, uint32_t t4, float px, float py, float pz,
                                                bool self, uint32_t sflag, uint32_t keep, uint32_t keep_m, float ds,
                                                uint32_t (&nk)[KS > 0 ? KS : 1], float& smin, double& fsum,
                                                float& macc) {
  if constexpr (RT >= 1) {
    constexpr int NB = RT < B ? RT : B;
    pair_group_w64<KS, PASS, FAST, RT, NB, true>(q0, t4, px, py, pz, self, sflag, keep, keep_m, ds, nk, smin, fsum,
                                                 macc);
    pair_groups_w64<KS, PASS, FAST, RT - NB, B>(q0, t4, px, py, pz, self, sflag, keep, keep_m, ds, nk, smin, fsum,
                                                macc);
  }
}
template <int KS, int PASS, bool FAST>
__device__ __forceinline__ void pair_pass_w64(const float4* __restrict__ ring, int t, float px, float py, float pz,
                                              bool self, uint32_t keep, float ds, uint32_t (&nk)[KS > 0 ? KS : 1],
                                              float& smin, double& fsum) {
  const uint32_t sflag = (FAST || self) ? 0u : 0x80000000u;
  const uint32_t keep_m = keep & 0x7fffffffu;
  const uint32_t t4 = (uint32_t)t << 2;
  float macc = 0.f;
  pair_groups_w64<KS, PASS, FAST, 31, S64_PAIR_BATCH>(ring + t, t4, px, py, pz, self, sflag, keep, keep_m, ds, nk,
                                                        smin, fsum, macc);
  if constexpr (PASS == 1) fsum += (double)wave_ror1(macc);
  // rotation 32 pairs t with t+32 from both sides: own evaluation only
  pair_group_w64<KS, PASS, FAST, 32, 1, false>(ring + t, t4, px, py, pz, self, sflag, keep, keep_m, ds, nk, smin, fsum,
                                               macc);
}

template <int KS, int PASS>
__device__ __forceinline__ void pair_pass_block(const float4* __restrict__ pos4, int N, int t, float px, float py,
                                                float pz, bool self, uint32_t keep, float ds,
                                                uint32_t (&nk)[KS > 0 ? KS : 1], float& smin, double& fsum) {
  // runtime N: unrolled by 4 unless the body holds key inserts (their v_med3_u32 inline asm is
  // convergent, which rules out the unroller's remainder loop)
  constexpr int UNROLL = KS > 0 ? 1 : 4;
#pragma unroll UNROLL
  for (int j = 0; j < N; ++j) {
    const float4 q = pos4[j];
    const float v = pair_value<PASS>(sqsum_f(q.x - px, q.y - py, q.z - pz));
    const bool other = j != t;
    if constexpr (KS > 0) kins<KS>(nk, other ? ((__float_as_uint(v) & keep) | (uint32_t)j) : KEY_EMPTY);
    const bool pr = self && (q.w != 0.f) && other;
    if constexpr (PASS != 0) smin = fminf(smin, pr ? v : __builtin_inff());
    if constexpr (PASS == 1) {
      const float e = fabsf(v - ds);
      fsum += (double)(pr ? e : 0.f);
    }
  }
}

// Block teams (one env per workgroup, N a power of two > 64), every drone eligible: rotation pass
// j = t + r (r = 1 .. N-1) over a ring of pair entries — entry j holds drones j and j+1 (mod N)
// as (x_j, x_j+1, y_j, y_j+1, z_j, z_j+1, pad): one ds_read2_b32 per coordinate feeds the
// packed-f32 distances of rotations r and r+1 (7-float stride: conflict-free lanes).  Keys carry
// the rotation offset (decoded as (t + r) & (N-1), like the wave teams), so no self-pair select;
// formation terms are summed in f32 per 8 pairs then in f64.  Same values as pair_pass_block.
constexpr int BLK_PAIR_STRIDE = 7;
typedef float blk_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void blk_put_pair(float* __restrict__ pr, int N, int t, float px, float py, float pz) {
  // drone t is the first half of entries t, t+N and the second half of entries t-1, t-1+N
  const int a = t, b = (t + N - 1) & (N - 1);
  float* e0 = pr + a * BLK_PAIR_STRIDE;
  float* e1 = pr + (a + N) * BLK_PAIR_STRIDE;
  float* e2 = pr + b * BLK_PAIR_STRIDE + 1;
  float* e3 = pr + (b + N) * BLK_PAIR_STRIDE + 1;
  e0[0] = px; e0[2] = py; e0[4] = pz;
  e1[0] = px; e1[2] = py; e1[4] = pz;
  e2[0] = px; e2[2] = py; e2[4] = pz;
  e3[0] = px; e3[2] = py; e3[4] = pz;
}
// KEYS = false (the step's first pass of a block team): formation terms and the running minimum
// of d~ only — the keys follow in a PASS 0 pass once the env is known not to reset (at N >= 128
// almost every env resets every step, and a reset env's keys come from its new positions).
template <int KS, int PASS, bool KEYS = true>
__device__ __forceinline__ void pair_pass_block_fast(const float* __restrict__ pr, int N, int t, float px, float py,
                                                     float pz, uint32_t keep, float ds,
                                                     uint32_t (&nk)[KS > 0 ? KS : 1], double& fsum,
                                                     float& vmin) {
  const float* q = pr + t * BLK_PAIR_STRIDE;
  float esum = 0.f;
  int r = 1;
  // runtime N: unrolled by 4 unless the body holds key inserts (convergent inline asm, above)
  constexpr int UNROLL = KS > 0 && KEYS ? 1 : 4;
#pragma unroll UNROLL
  for (; r + 1 < N; r += 2) {
    const float* e = q + r * BLK_PAIR_STRIDE;
    const blk_f2 X = {e[0], e[1]}, Y = {e[2], e[3]}, Z = {e[4], e[5]};
    const blk_f2 dx = X - px, dy = Y - py, dz = Z - pz;
    blk_f2 sq = dx * dx;
    sq = __builtin_elementwise_fma(dy, dy, sq);
    sq = __builtin_elementwise_fma(dz, dz, sq);
    const float va = pair_value<PASS>(sq.x), vb = pair_value<PASS>(sq.y);
    if constexpr (KS > 0 && KEYS) {
      kins<KS>(nk, (__float_as_uint(va) & keep) | (uint32_t)r);
      kins<KS>(nk, (__float_as_uint(vb) & keep) | (uint32_t)(r + 1));
    }
    if constexpr (!KEYS) vmin = fminf(vmin, fminf(va, vb));
    if constexpr (PASS == 1) {
      const blk_f2 V = {va, vb};
      const blk_f2 Ed = V - ds;
      esum += fabsf(Ed.x);
      esum += fabsf(Ed.y);
      if ((r & 7) == 7) {
        fsum += (double)esum;
        esum = 0.f;
      }
    }
  }
  if (r < N) {  // N - 1 is odd: the last rotation alone
    const float* e = q + r * BLK_PAIR_STRIDE;
    const float v = pair_value<PASS>(sqsum_rank(e[0] - px, e[2] - py, e[4] - pz));
    if constexpr (KS > 0 && KEYS) kins<KS>(nk, (__float_as_uint(v) & keep) | (uint32_t)r);
    if constexpr (!KEYS) vmin = fminf(vmin, v);
    if constexpr (PASS == 1) esum += fabsf(v - ds);
  }
  if constexpr (PASS == 1) fsum += (double)esum;
}

template <int MSL, bool COLL>
__device__ __forceinline__ void obstacle_pass(const float4* __restrict__ obst4, int M, float px, float py, float pz,
                                              bool chk, float s_thr, uint32_t keep,
                                              uint32_t (&ok)[MSL > 0 ? MSL : 1], bool& coll) {
  for (int m = 0; m < M; ++m) {
    const float4 q = lds_f4(obst4 + m);
    const float s = sqsum_f(q.x - px, q.y - py, q.z - pz);  // exact axis-path value
    if constexpr (MSL > 0) kins<MSL>(ok, (__float_as_uint(s) & keep) | (uint32_t)m);
    if constexpr (COLL) coll = coll || (chk && (s <= s_thr));
  }
}

// Re-rank the S surviving keys by exact distance (the reference sorts by the float distance;
// ties by index).  Returns false when an entry outside the survivors could still precede the
// K-th winner — the caller then runs exact_select.  APPROX: keys hold s' or d~ (pairs; `dkey`
// selects d~) rather than the exact squared value (obstacles), so the non-survivor bound is
// widened by FAST_LO.
template <int S, bool AXIS, bool APPROX>
__device__ __forceinline__ bool finish_keys(const uint32_t (&k)[S], const float4* __restrict__ pts, int count,
                                            int ibase, int imod, int K, uint32_t keep, bool dkey, float px, float py,
                                            float pz, float (&wd)[S], int (&wj)[S]) {
  const uint32_t imask = ~keep;
  // The keys are already ordered by the (truncated) ranking value; the exact order can differ
  // only where two survivors lie within the truncation/error band of each other (near-tie,
  // band 2^-18 relative >> the 1-ulp collapse of sqrt).  Without one, the first K keys are the
  // answer in order and only their exact distances are needed.
  bool near = false;
#pragma unroll
  for (int s = 0; s + 1 < S; ++s)
    near = near | ((k[s + 1] != KEY_EMPTY) &
                   (__uint_as_float(k[s + 1] & keep) <= __uint_as_float((k[s] & keep) | imask) * FAST_HI));
  const int need = near ? S : K;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const uint32_t key = k[s];
    const int j = ((int)(key & imask) + ibase) & imod;
    const bool valid = (key != KEY_EMPTY) & (j < count) & (s < need);
    float d = __builtin_inff();
    if (valid) {
      const float4 q = pts[j];
      d = AXIS ? sqrt_rn(sqsum_f(q.x - px, q.y - py, q.z - pz)) : sqrt_rn(sqsum_1d(q.x - px, q.y - py, q.z - pz));
    }
    wd[s] = d;
    wj[s] = valid ? j : 0x7fffffff;
  }
  if (near) {
#pragma unroll
    for (int s = 1; s < S; ++s) {
#pragma unroll
      for (int r = s; r > 0; --r) {
        const float a = wd[r - 1], b = wd[r];
        const int ja = wj[r - 1], jb = wj[r];
        const bool sw = (b < a) || (b == a && jb < ja);
        wd[r - 1] = sw ? b : a; wd[r] = sw ? a : b;
        wj[r - 1] = sw ? jb : ja; wj[r] = sw ? ja : jb;
      }
    }
  }
  const uint32_t last = k[S - 1];
  if (last == KEY_EMPTY || ((((int)(last & imask) + ibase) & imod) >= count)) return true;
  if (K <= 0) return true;
  const float base = __uint_as_float(last & keep);
  const float w = wd[K - 1];
  if (APPROX && dkey) return base * FAST_LO > w;
  // squared space (no sqrt): base(1 - 2^-18) > w^2 (1 + 2^-18) in f32 implies every
  // non-survivor's exact distance exceeds w strictly (keys are within 2^-21 of exact s; key
  // truncation only lowers base); a near-equality falls to exact_select, which is exact anyway
  return (APPROX ? base * FAST_LO : base) > (w * w) * FAST_HI;
}

// Largest of the first K entries of a register array (= entry K-1 of a sorted list), as a
// reduction: a select chain on the index gets folded back into a dynamic alloca index, which
// moves the whole array to scratch.
template <int S>
__device__ __forceinline__ float max_first(const float (&arr)[S], int K) {
  float v = 0.f;
#pragma unroll
  for (int u = 0; u < S; ++u) v = (u < K) ? fmaxf(v, arr[u]) : v;
  return v;
}

// Exact (distance, index) selection of the K nearest of `count` points (rare fallback, taken when
// finish_keys cannot prove its top-K).  `dmax` bounds the K-th exact distance from above (the
// K-th of the re-ranked survivors), so only points whose f32 squared sum lies within dmax^2 (plus
// the f32 error band) can belong to the answer: a cheap scan filters, and the exact distance is
// evaluated only for those few.
template <int S, bool AXIS>
__device__ __forceinline__ void exact_select(const float4* __restrict__ pts, int count, int self, int K, float dmax,
                                             float px, float py, float pz, float (&wd)[S], int (&wj)[S]) {
#pragma unroll
  for (int u = 0; u < S; ++u) { wd[u] = __builtin_inff(); wj[u] = 0x7fffffff; }
  const float s_cut = (dmax * dmax) * FAST_HI;
  // batches of 8 points: the batch's LDS reads are issued together and its filter sums computed
  // before the first (divergent) exact evaluation, instead of one exposed LDS round trip per
  // point — a wave in this fallback is the last of its launch more often than not
  constexpr int B = FB_BATCH;
#pragma unroll 1
  for (int j0 = 0; j0 < count; j0 += B) {
    float4 q[B];
    float sq[B];
#pragma unroll
    for (int u = 0; u < B; ++u) q[u] = pts[j0 + u < count ? j0 + u : j0];
#pragma unroll
    for (int u = 0; u < B; ++u) sq[u] = sqsum_f(q[u].x - px, q[u].y - py, q[u].z - pz);
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int j = j0 + u;
      if (j < count && j != self && sq[u] <= s_cut) {
        float cd = AXIS ? sqrt_rn(sq[u]) : sqrt_rn(sqsum_1d(q[u].x - px, q[u].y - py, q[u].z - pz));
        int cj = j;
#pragma unroll
        for (int v = 0; v < S; ++v) {  // insertion by exchange: the largest falls off slot K-1
          if (v < K) {
            const bool lt = (cd < wd[v]) || (cd == wd[v] && cj < wj[v]);
            const float td = wd[v];
            const int tj = wj[v];
            wd[v] = lt ? cd : td; wj[v] = lt ? cj : tj;
            cd = lt ? td : cd; cj = lt ? tj : cj;
          }
        }
      }
    }
  }
}

// A nearest key whose value bits are 0 decides the band without the exact scan (coincident
// drones, e.g. stacked in a world-clip corner).  d~ keys (DKEY): v_sqrt_f32 of a nonzero s'
// (denormals are kept in this code) is >= 2^-75, so value bits 0 mean s' = 0, i.e. every f32
// square rounds to 0, i.e. the sdot sum is 0: within any threshold >= 0.  s' keys: value bits 0
// mean s' < 2^-143, and the exact sum is then below FLT_MIN: within any threshold >= FLT_MIN.
template <bool DKEY>
__device__ __forceinline__ bool key_zero_hit(uint32_t key, uint32_t keep, float s_thr) {
  return (key & keep) == 0u && s_thr >= (DKEY ? 0.f : 0x1p-126f);
}

// exact "any eligible pair within s_thr" (fallback of the banded running minimum); the f32 sum
// filters, the sdot-exact sum decides
__device__ __forceinline__ bool exact_pair_collision(const float4* __restrict__ pts, int count, int self,
                                                     float px, float py, float pz, float s_thr) {
  bool c = false;
  const float s_cut = s_thr * FAST_HI;
  constexpr int B = FB_BATCH;  // batched LDS reads, as exact_select
#pragma unroll 1
  for (int j0 = 0; j0 < count; j0 += B) {
    float4 q[B];
#pragma unroll
    for (int u = 0; u < B; ++u) q[u] = pts[j0 + u < count ? j0 + u : j0];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int j = j0 + u;
      if (j < count && j != self && q[u].w != 0.f && sqsum_f(q[u].x - px, q[u].y - py, q[u].z - pz) <= s_cut)
        c = c || (sqsum_1d(q[u].x - px, q[u].y - py, q[u].z - pz) <= s_thr);
    }
  }
  return c;
}

// step64 observation rows leave through write-through (sc1) buffer stores when WT_STORES:
// the lines are dropped from the XCD's L2 instead of staying dirty for the end-of-kernel
// write-back (MI355X_MICROARCH.md, store flavours; a kernel boundary pays for the dirty bytes it
// leaves): -5 % kernel time.  A compiler-visible buffer store (not inline asm) so the hazard and
// waitcnt passes see it.  `base` must be wave-uniform (it becomes the buffer descriptor).
constexpr int BUF_DWORD3 = 0x00020000;  // gfx9 raw buffer descriptor word 3
__device__ __forceinline__ void store_obs(float* base, uint32_t nbytes, uint32_t byte_off, float4 v) {
  if constexpr (WT_STORES) {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const v4i d = {__float_as_int(v.x), __float_as_int(v.y), __float_as_int(v.z), __float_as_int(v.w)};
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)nbytes, BUF_DWORD3);
    __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)byte_off, 0, OBS_STORE_AUX);
  } else {
    *reinterpret_cast<float4*>(reinterpret_cast<char*>(base) + byte_off) = v;
  }
}

// ------------------------------------------------------------------ the kernel
// LM (lane mode): 0 = BLOCK (L > 64), 1 = WAVE with 64/L teams, 2 = WAVE with one team (L == 64)
}  // namespace swarm_dev
namespace {  // kernels: internal to this translation unit
template <int KIND, int DYN, int KS, int MSL, int LM>
__global__ void __launch_bounds__(LM != 0 ? 64 : 1024)
swarm_kernel(const KParams P, const swarm_state_t S, const float* __restrict__ actions,
             const uint8_t* __restrict__ amask, const swarm_out_t O,
             const uint8_t* __restrict__ env_mask, int mode_arg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // compile-time mode in the step kernel; reset/observe share the aux kernel
  const int mode = (KIND == KIND_STEP) ? MODE_STEP : (mode_arg == MODE_RESET ? MODE_RESET : MODE_OBSERVE);
  STAMP(0);
  STAMP_BEGIN(blockIdx.x, threadIdx.x == 0);
  constexpr bool WAVE = LM != 0;
  constexpr bool W64 = LM == 2;
  const int tid = threadIdx.x;
  const int L = W64 ? 64 : 1 << P.log2_lanes;
  const int team = W64 ? 0 : tid >> P.log2_lanes;
  const int t = W64 ? tid : tid & (L - 1);
  const int G = W64 ? 1 : P.envs_per_block;
  const int N = P.N, M = P.M, D = P.D, K = P.K, Ms = P.Ms;
  const long long env0 = (long long)blockIdx.x * G;
  const long long env = env0 + team;
  const bool env_ok = env < P.E;
  // this env's parameters: its swarm_env_cfg_t record (per-env curriculum / randomisation) or
  // the launch-uniform values
  swarm_env_cfg_t C;
  if (S.env_cfg != nullptr && env_ok) C = S.env_cfg[env];
  else C = uniform_env_cfg(P);
  int Me = clamp_obstacles(C.num_obstacles, M);  // active obstacles (slots >= Me are ignored)
  const bool is_agent = env_ok && t < N;
  float4* ring = reinterpret_cast<float4*>(smem) + team * P.ring;
  float4* obst4 = reinterpret_cast<float4*>(smem + P.off_obst) + team * P.obst_stride;
  float* stage = reinterpret_cast<float*>(smem + P.off_stage);
  float* pair_ring = reinterpret_cast<float*>(smem + P.off_pair);  // block teams, P.off_pair > 0
  uint64_t team_bits = 0;
  // one env of exactly 64 agents per wave: the per-agent byte outputs (terminated, truncated,
  // active) leave as three 64-B dword stores built from wave ballots instead of 3 x 64 byte stores
  const bool packed_bytes = W64 && KIND == KIND_STEP && P.pack_bytes;
  bool new_act_out = false;
  if constexpr (WAVE) team_bits = (W64 || L == 64) ? ~0ull : (((1ull << L) - 1ull) << (team * L));

  // envs this call writes: every env (step) or the masked ones (reset / observe)
  bool sel = env_ok;
  if (mode != MODE_STEP && env_mask != nullptr && env_ok) sel = env_mask[env] != 0;

  // ---- load
  int stepc = 0;
  float gx = 0.f, gy = 0.f, gz = 0.f;
  if (env_ok) {
    for (int m = t; m < Me; m += L) {
      const float* o = S.obstacles + (env * M + m) * 3;
      obst4[m] = make_float4(o[0], o[1], o[2], 0.f);
    }
    gx = S.goal[env * 3 + 0];
    gy = S.goal[env * 3 + 1];
    gz = S.goal[env * 3 + 2];
    if (mode == MODE_STEP) stepc = S.step_count[env];
  }
  float px = PAD_POS, py = PAD_POS, pz = PAD_POS, vx = 0.f, vy = 0.f, vz = 0.f, damp = 0.f;
  bool act = false;
  const long long ag = env * N + t;
  float ax = 0.f, ay = 0.f, az = 0.f;
  bool has = true;
  if (is_agent) {
    if (mode == MODE_STEP) {
      ax = actions[ag * 3 + 0]; ay = actions[ag * 3 + 1]; az = actions[ag * 3 + 2];
      has = (amask == nullptr) || (amask[ag] != 0);
    }
    px = S.pos[ag * 3 + 0]; py = S.pos[ag * 3 + 1]; pz = S.pos[ag * 3 + 2];
    vx = S.vel[ag * 3 + 0]; vy = S.vel[ag * 3 + 1]; vz = S.vel[ag * 3 + 2];
    act = S.active[ag] != 0;
    if constexpr (DYN == DYN_PHYS) {
      if (mode == MODE_STEP) damp = S.damping[ag];
    }
  }
  int n_active = 0;
  if (mode == MODE_STEP) {
    if constexpr (WAVE) n_active = __popcll(__ballot(is_agent && act) & team_bits);
    else n_active = __syncthreads_count(is_agent && act);
  }

  // ---- integrate (step) or draw (explicit reset)
  STAMP(1);
  float prev_d = 0.f;
  uint32_t episode_new = 0;
  const long long genv = P.env_offset + env;
  if (mode == MODE_STEP && is_agent) {
    if constexpr (DYN == DYN_KIN) {
      if (act) {  // drone_swarm_env.py:98-111
        prev_d = sqrt_rn(sqsum_1d(gx - px, gy - py, gz - pz));
        if (!has) { ax = 0.f; ay = 0.f; az = 0.f; }
        ax = clampf(ax, -1.f, 1.f) * C.max_accel;
        ay = clampf(ay, -1.f, 1.f) * C.max_accel;
        az = clampf(az, -1.f, 1.f) * C.max_accel;
        vx = vx + ax * C.dt;
        vy = vy + ay * C.dt;
        vz = vz + az * C.dt;
        const float s_sp = sqsum_1d(vx, vy, vz);  // _clip_speed :179-183
        if (!(s_sp <= C.s_vmax)) {
          const float sp = sqrt_rn(s_sp);
          if (!(sp <= C.max_speed || sp < (float)1e-8)) {
            vx = (vx / sp) * C.max_speed;
            vy = (vy / sp) * C.max_speed;
            vz = (vz / sp) * C.max_speed;
          }
        }
        px = px + vx * C.dt;
        py = py + vy * C.dt;
        pz = pz + vz * C.dt;
      }
      if (n_active > 0) {  // world clip of ALL drones, :113-117
        px = clampf(px, C.neg_half_w, C.half_w);
        py = clampf(py, C.neg_half_w, C.half_w);
        pz = clampf(pz, C.neg_half_w, C.half_w);
      }
    } else {
      // point-mass restatement of drone_physics_env.py:323-360
      const float h = P.h;
      const float cx = has ? ax * C.max_accel : 0.f;
      const float cy = has ? ay * C.max_accel : 0.f;
      float cz = has ? az * C.max_accel + P.gcomp : 0.f;
      cz = cz + P.g;
      float fac = 1.f;
      if (P.damping_law == 1) fac = (float)pow((double)(1.f - damp), (double)h);
      // One correctly rounded norm per substep in the common case: the clamp test runs in
      // squared space (s_vmax: sqrt_rn(s) > vmax exactly when s > s_vmax), and an unclamped
      // velocity's norm after the clamp is the norm before it, so the damping law reuses it.
      const bool law0 = P.damping_law == 0;
      for (int s = 0; s < P.substeps; ++s) {
        const float s_sp = sqsum_1d(vx, vy, vz);
        float sp2 = 0.f;
        if (has && s_sp > C.s_vmax) {
          const float sp = sqrt_rn(s_sp);
          vx = (vx / sp) * C.max_speed;
          vy = (vy / sp) * C.max_speed;
          vz = (vz / sp) * C.max_speed;
          if (law0) sp2 = sqrt_rn(sqsum_1d(vx, vy, vz));
        } else if (law0) {
          sp2 = sqrt_rn(s_sp);
        }
        if (law0) {
          const float c = damp * (1.f + sp2);
          vx = vx + h * (cx - c * vx);
          vy = vy + h * (cy - c * vy);
          vz = vz + h * (cz - c * vz);
        } else {
          vx = (vx + h * cx) * fac;
          vy = (vy + h * cy) * fac;
          vz = (vz + h * cz) * fac;
        }
        px = px + h * vx;
        py = py + h * vy;
        pz = pz + h * vz;
      }
    }
  }

  auto draw_env = [&]() {  // new episode for this team (drone_swarm_env.py:72-80 ranges)
    if (S.env_cfg_next != nullptr) {  // the next episode's parameters take over
      C = S.env_cfg_next[env];
      Me = clamp_obstacles(C.num_obstacles, M);
    }
    uint32_t w[4];
    if (t < N) {
      draw_block(P, genv, episode_new, (uint32_t)t, w);
      px = uni(w[0], C.neg_half_w, C.width_w);
      py = uni(w[1], C.neg_half_w, C.width_w);
      pz = uni(w[2], C.neg_half_w, C.width_w);
      vx = vy = vz = 0.f;
      act = true;
      if constexpr (DYN == DYN_PHYS) {
        pz = fmaxf(pz, 1.0f);
        damp = 0.5f * uni(w[3], 0.8f, 0.4f);
      }
    }
    for (int m = t; m < M; m += L) {
      if (m >= Me) {  // inactive slot of a per-env obstacle count: stored as zeros
        obst4[m] = make_float4(0.f, 0.f, 0.f, 0.f);
        continue;
      }
      draw_block(P, genv, episode_new, (uint32_t)(N + m), w);
      float oz = uni(w[2], C.neg_half_w, C.width_w);
      if constexpr (DYN == DYN_PHYS) oz = fmaxf(oz, 0.5f);
      obst4[m] = make_float4(uni(w[0], C.neg_half_w, C.width_w), uni(w[1], C.neg_half_w, C.width_w), oz, 0.f);
    }
    draw_block(P, genv, episode_new, (uint32_t)(N + Me), w);
    gx = uni(w[0], C.neg_half_w, C.width_w);
    gy = uni(w[1], C.neg_half_w, C.width_w);
    gz = uni(w[2], C.neg_half_w, C.width_w);
    if constexpr (DYN == DYN_PHYS) gz = uni(w[3], 0.5f, 1.5f);
  };
  auto put_ring = [&](float w) {
    ring[t] = make_float4(px, py, pz, w);
    if constexpr (WAVE) ring[t + L] = make_float4(px, py, pz, w);
    if constexpr (!WAVE) {
      if (P.off_pair > 0 && t < N) blk_put_pair(pair_ring, N, t, px, py, pz);
    }
  };

  if (mode == MODE_RESET && sel) {  // explicit device reset: draw before the observation pass
    episode_new = S.episode[env] + 1u;
    draw_env();
    stepc = 0;
  }

  STAMP(2);
  // LDS slot: (p, eligibility); padding lanes sit far away with flag 0
  const bool elig = (DYN == DYN_KIN) ? act : is_agent;
  put_ring(elig ? 1.f : 0.f);
  __syncthreads();

  // ---- pair + obstacle passes
  constexpr int NW = KS > 0 ? KS : 1;
  constexpr int OW = MSL > 0 ? MSL : 1;
  uint32_t nk[NW];
  uint32_t ok[OW];
#pragma unroll
  for (int s = 0; s < NW; ++s) nk[s] = KEY_EMPTY;
#pragma unroll
  for (int s = 0; s < OW; ++s) ok[s] = KEY_EMPTY;
  bool ocoll = false;
  float smin = __builtin_inff();  // running min of the pair value over eligible pairs (banded)
  double fsum = 0.0;
  const bool pass_env = (mode == MODE_STEP) ? env_ok : sel;
  // all-eligible fast path: wave-uniform, needs the nearest neighbour (KS > 0) and no padding
  bool fast = false;
  if constexpr (WAVE) fast = (KS > 0) && (N == L) && __all(elig);
  // block teams: the rotation pass over the pair-entry ring (N a power of two, kinematic)
  if constexpr (!WAVE && KS > 0 && DYN == DYN_KIN) fast = P.off_pair > 0 && __syncthreads_and(!is_agent || elig) != 0;
  const bool blk_rot = !WAVE && P.off_pair > 0;  // aux / reset passes of block teams rotate too
  if (pass_env) {
    if (mode == MODE_STEP) {
      constexpr int PASS = (DYN == DYN_KIN) ? 1 : 2;
      if constexpr (WAVE) {
        if constexpr (W64) {
          if (fast) pair_pass_w64<KS, PASS, true>(ring, t, px, py, pz, elig, P.nb_keep, P.ds_f, nk, smin, fsum);
          else pair_pass_w64<KS, PASS, false>(ring, t, px, py, pz, elig, P.nb_keep, P.ds_f, nk, smin, fsum);
        } else {
          if (fast)
            pair_pass_wave<KS, PASS, true>(ring, L, t, tid, px, py, pz, elig, P.nb_keep, P.ds_f, nk, smin, fsum);
          else
            pair_pass_wave<KS, PASS, false>(ring, L, t, tid, px, py, pz, elig, P.nb_keep, P.ds_f, nk, smin, fsum);
        }
      } else {
        if constexpr (DYN == DYN_KIN) {
          if (fast) pair_pass_block_fast<KS, PASS, false>(pair_ring, N, t, px, py, pz, P.nb_keep, P.ds_f, nk, fsum, smin);
          else pair_pass_block<KS, PASS>(ring, N, t, px, py, pz, elig, P.nb_keep, P.ds_f, nk, smin, fsum);
        } else {
          pair_pass_block<KS, PASS>(ring, N, t, px, py, pz, elig, P.nb_keep, P.ds_f, nk, smin, fsum);
        }
      }
      if constexpr (DYN == DYN_KIN) obstacle_pass<MSL, true>(obst4, Me, px, py, pz, act, C.s_obst, P.ob_keep, ok, ocoll);
      else obstacle_pass<MSL, true>(obst4, Me, px, py, pz, true, C.s_phys_obst, P.ob_keep, ok, ocoll);
    } else {
      if constexpr (WAVE) {
        if constexpr (W64) pair_pass_w64<KS, 0, true>(ring, t, px, py, pz, true, P.nb_keep, 0.f, nk, smin, fsum);
        else pair_pass_wave<KS, 0, true>(ring, L, t, tid, px, py, pz, true, P.nb_keep, 0.f, nk, smin, fsum);
      } else {
        if (blk_rot) pair_pass_block_fast<KS, 0>(pair_ring, N, t, px, py, pz, P.nb_keep, 0.f, nk, fsum, smin);
        else pair_pass_block<KS, 0>(ring, N, t, px, py, pz, true, P.nb_keep, 0.f, nk, smin, fsum);
      }
      obstacle_pass<MSL, false>(obst4, Me, px, py, pz, false, 0.f, P.ob_keep, ok, ocoll);
    }
  }

  STAMP(3);
  // ---- exact top-K for the current (post-step) state
  float wd[NW], od[OW];
  int wj[NW], oj[OW];
#pragma unroll
  for (int s = 0; s < NW; ++s) { wd[s] = 0.f; wj[s] = 0x7fffffff; }
#pragma unroll
  for (int s = 0; s < OW; ++s) { od[s] = 0.f; oj[s] = 0x7fffffff; }
  // neighbour keys carry the rotation offset (wave teams, block rotation passes: `rot`) or the
  // drone index (block pair_pass_block)
  const int Kq = K;
  auto select_topk = [&](bool run, bool dkey, bool rot) {
    const int Mse = Ms < Me ? Ms : Me;
    bool slow_nb = false, slow_ob = false;
    if (run) {
      const int imod = rot ? (L - 1) : 0x7fffffff;
      if constexpr (KS > 0) slow_nb = !finish_keys<KS, false, true>(nk, ring, N, rot ? t : 0, imod, Kq, P.nb_keep, dkey, px, py, pz, wd, wj);
      if constexpr (MSL > 0) slow_ob = !finish_keys<MSL, true, false>(ok, obst4, Me, 0, 0x7fffffff, Mse, P.ob_keep, false, px, py, pz, od, oj);
    }
    if constexpr (KS > 0) {
      if (slow_nb) exact_select<NW, false>(ring, N, t, Kq, max_first(wd, Kq), px, py, pz, wd, wj);
    }
    if constexpr (MSL > 0) {
      if (slow_ob) exact_select<OW, true>(obst4, Me, -1, Mse, max_first(od, Mse), px, py, pz, od, oj);
    }
  };
  // the step's kinematic pass ranks by d~, every other pass by s'.  A step runs the finish only
  // for the observation it emits (after the reset decision: a resetting env finishes once, for
  // its new episode); reset / observe run it now.
  if (mode != MODE_STEP) select_topk(is_agent && pass_env, false, WAVE || blk_rot);
  STAMP(4);

  // ---- rewards / terminations (step)
  float rew = 0.f, dist_out = 0.f;
  bool term = false, trunc = false, cont = false, reached = false, collided = false;
  bool term_all = false, trunc_all = false, do_reset = false;
  int new_step = stepc;
  if (mode == MODE_STEP) {
    bool p_coll = false, p_cand = false, p_notall = false;
    if (is_agent) {
      // pair collision: exact nearest (fast) or banded running minimum with exact re-check
      const float s_exact_thr = (DYN == DYN_KIN) ? P.s_pair : P.s_phys_pair;
      const float d_thr = (DYN == DYN_KIN) ? P.thr_pair : P.thr_ppair;
      bool pcoll;
      if (fast && WAVE) {
        // the nearest key bounds the exact nearest distance (d~ keys: kinematic; s' keys:
        // physics): [key & keep, key | ~keep] x [FAST_LO, FAST_HI]; exact scan inside the band
        const float thr = (DYN == DYN_KIN) ? d_thr : s_exact_thr;
        pcoll = __uint_as_float(nk[0] | ~P.nb_keep) * FAST_HI <= thr;
        if (!pcoll && __uint_as_float(nk[0] & P.nb_keep) * FAST_LO <= thr)
          pcoll = key_zero_hit<DYN == DYN_KIN>(nk[0], P.nb_keep, s_exact_thr) ||
                  exact_pair_collision(ring, N, t, px, py, pz, s_exact_thr);
      } else {
        // smin holds d~ (kinematic) or s' (physics): certain below the band, exact inside it
        const float band_thr = (DYN == DYN_KIN) ? d_thr : s_exact_thr;
        pcoll = smin <= band_thr * FAST_LO;
        if (!pcoll && smin <= band_thr * FAST_HI && elig)
          pcoll = exact_pair_collision(ring, N, t, px, py, pz, s_exact_thr);
      }
      if constexpr (DYN == DYN_KIN) {
        const float curr = sqrt_rn(sqsum_1d(gx - px, gy - py, gz - pz));
        dist_out = curr;
        if (act) {
          reached = (double)curr <= P.goal_radius;  // fp64 compare, :124-127
          collided = ocoll || pcoll;
          p_coll = collided;
          p_cand = !reached && !collided;
          double r = ((double)prev_d - (double)curr) * P.kp;
          if (n_active > 1) r = r + (-P.kf) * (fsum * inv_count(n_active - 1));
          if (reached) r = r + P.r_goal;
          if (collided) r = r + P.r_col;
          rew = (float)r;
        }
      } else {
        const double dx = (double)px - (double)gx;
        const double dy = (double)py - (double)gy;
        const double dz = (double)pz - (double)gz;
        const double dist_phys = dsqrt_rn(((dx * dx) + (dy * dy)) + (dz * dz));
        dist_out = (float)dist_phys;
        collided = ocoll || pcoll || (pz <= P.ground_z);
        reached = dist_phys < P.goal_radius;
        if (act) {
          p_coll = collided;
          p_notall = !collided && !reached;
          double r = (-dist_phys) * 0.1;
          if (collided) r = r - 10.0;
          else if (reached) r = r + 50.0;
          rew = (float)r;
        }
      }
    }
    bool any_c, any_cand, any_notall;
    if constexpr (WAVE) {
      any_c = (__ballot(p_coll) & team_bits) != 0;
      any_cand = (__ballot(p_cand) & team_bits) != 0;
      any_notall = (__ballot(p_notall) & team_bits) != 0;
    } else {
      any_c = __syncthreads_or(p_coll) != 0;
      any_cand = __syncthreads_or(p_cand) != 0;
      any_notall = __syncthreads_or(p_notall) != 0;
    }
    if constexpr (DYN == DYN_KIN) {
      if (n_active == 0) {  // drone_swarm_env.py:93-95
        term_all = true;
      } else {
        new_step = stepc + 1;
        const bool tl = new_step >= C.max_steps;
        const bool all_reached = !any_cand && !any_c && !tl;
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
      const bool tl = new_step >= C.max_steps;
      const bool all_goals = !any_notall;
      const bool done = any_c || all_goals || tl;
      trunc_all = done && tl && !any_c && !all_goals;
      term_all = done && !trunc_all;
      term = term_all;
      trunc = trunc_all;
      cont = true;
    }
    do_reset = P.auto_reset && env_ok && (term_all || trunc_all);
    bool dkey_step = DYN == DYN_KIN;
    if constexpr (!WAVE && DYN == DYN_KIN) {
      if (fast && !do_reset) {  // block uniform: the keys of the emitted observation
        float s3 = 0.f;
        double f3 = 0.0;
        pair_pass_block_fast<KS, 0>(pair_ring, N, t, px, py, pz, P.nb_keep, 0.f, nk, f3, s3);
        dkey_step = false;  // PASS 0 keys rank by s'
      }
    }
    select_topk(is_agent && !do_reset, dkey_step, WAVE || fast);

    // per-agent step outputs (the episode that just ended, for reset envs)
    if (is_agent) {
      O.reward[ag] = rew;
      if (!packed_bytes) {
        O.terminated[ag] = term ? 1 : 0;
        O.truncated[ag] = trunc ? 1 : 0;
      }
      if (O.dist_goal) O.dist_goal[ag] = dist_out;
      if (O.info_flags)
        O.info_flags[ag] = (uint8_t)((act ? SWARM_AGENT_STEPPED : 0u) | (act && reached ? SWARM_AGENT_REACHED : 0u) |
                                     (act && collided ? SWARM_AGENT_COLLISION : 0u) | (cont ? SWARM_AGENT_HAS_OBS : 0u));
    }
    if (env_ok && t == 0)
      O.env_done[env] = (uint8_t)((term_all ? SWARM_ENV_TERMINATED : 0u) | (trunc_all ? SWARM_ENV_TRUNCATED : 0u) |
                                  (do_reset ? SWARM_ENV_RESET : 0u));

    STAMP(5);
    bool any_reset;
    if constexpr (WAVE) any_reset = __ballot(do_reset) != 0;
    else any_reset = __syncthreads_or(do_reset) != 0;
    if (any_reset) {  // block-uniform: some team re-draws its env in-kernel
      __syncthreads();  // pass-1 reads of ring/obst4 are done
      if (do_reset) {
        episode_new = S.episode[env] + 1u;
        draw_env();
        put_ring(1.f);
      }
      __syncthreads();
      if (do_reset) {
#pragma unroll
        for (int s = 0; s < NW; ++s) nk[s] = KEY_EMPTY;
#pragma unroll
        for (int s = 0; s < OW; ++s) ok[s] = KEY_EMPTY;
        bool c2 = false;
        float s2 = 0.f;
        double f2 = 0.0;
        if constexpr (WAVE) {
          if constexpr (W64) pair_pass_w64<KS, 0, true>(ring, t, px, py, pz, true, P.nb_keep, 0.f, nk, s2, f2);
          else pair_pass_wave<KS, 0, true>(ring, L, t, tid, px, py, pz, true, P.nb_keep, 0.f, nk, s2, f2);
        } else if (blk_rot) {
          pair_pass_block_fast<KS, 0>(pair_ring, N, t, px, py, pz, P.nb_keep, 0.f, nk, f2, s2);
        } else {
          pair_pass_block<KS, 0>(ring, N, t, px, py, pz, true, P.nb_keep, 0.f, nk, s2, f2);
        }
        obstacle_pass<MSL, false>(obst4, Me, px, py, pz, false, 0.f, P.ob_keep, ok, c2);
      }
      select_topk(do_reset && is_agent, false, WAVE || blk_rot);
    }
  } else if (sel && is_agent) {
    dist_out = sqrt_rn(sqsum_1d(gx - px, gy - py, gz - pz));
  }

  STAMP(6);
  // ---- state write-back
  const bool write_env = (mode == MODE_STEP) ? env_ok : sel;
  if (is_agent) {
    if (mode == MODE_STEP) {
      bool new_act;
      if constexpr (DYN == DYN_KIN) new_act = cont;
      else new_act = act && !(term_all || trunc_all);
      if (do_reset) new_act = true;
      S.pos[ag * 3 + 0] = px; S.pos[ag * 3 + 1] = py; S.pos[ag * 3 + 2] = pz;
      S.vel[ag * 3 + 0] = vx; S.vel[ag * 3 + 1] = vy; S.vel[ag * 3 + 2] = vz;
      if (!packed_bytes) S.active[ag] = new_act ? 1 : 0;
      new_act_out = new_act;
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
  if (packed_bytes && env_ok) {  // wave-uniform (W64: the block is one env)
    const uint64_t mt = __ballot(term), mr = __ballot(trunc), ma = __ballot(new_act_out);
    const int grp = t >> 4;
    if (grp < 3) {
      const uint64_t m = grp == 0 ? mt : (grp == 1 ? mr : ma);
      const uint32_t nib = (uint32_t)(m >> (4 * (t & 15))) & 0xFu;
      const uint32_t word = (nib & 1u) | ((nib & 2u) << 7) | ((nib & 4u) << 14) | ((nib & 8u) << 21);
      uint8_t* base = grp == 0 ? O.terminated : (grp == 1 ? O.truncated : S.active);
      *reinterpret_cast<uint32_t*>(base + env * 64 + 4 * (t & 15)) = word;
    }
  }
  const bool new_episode = (mode == MODE_STEP) ? do_reset : (mode == MODE_RESET && sel);
  if (env_ok && t == 0) {
    if (mode == MODE_STEP) S.step_count[env] = do_reset ? 0 : new_step;
    else if (mode == MODE_RESET && sel) S.step_count[env] = 0;
    if (new_episode) {
      if (S.env_cfg_next != nullptr) S.env_cfg[env] = C;
      S.episode[env] = episode_new;
      S.goal[env * 3 + 0] = gx; S.goal[env * 3 + 1] = gy; S.goal[env * 3 + 2] = gz;
    }
  }
  if (env_ok && new_episode) {
    for (int m = t; m < M; m += L) {
      float* o = S.obstacles + (env * M + m) * 3;
      const float4 q = lds_f4(obst4 + m);
      o[0] = q.x; o[1] = q.y; o[2] = q.z;
    }
  }

  STAMP(7);
  // observation velocity (physics clamps it in the obs only, drone_physics_env.py:438-442)
  float ovx = vx, ovy = vy, ovz = vz;
  if constexpr (DYN == DYN_PHYS) {
    const double dvx = (double)vx, dvy = (double)vy, dvz = (double)vz;
    const double nv = dsqrt_rn(((dvx * dvx) + (dvy * dvy)) + (dvz * dvz));
    if (nv > C.max_speed_d) {
      ovx = (float)((dvx / nv) * C.max_speed_d);
      ovy = (float)((dvy / nv) * C.max_speed_d);
      ovz = (float)((dvz / nv) * C.max_speed_d);
    }
  }

  // ---- observation rows: [p | v | g-p | K x (p_j-p_i, d) | Ms x (o_m-p_i, d)]
  auto write_row = [&](float* row) {
    row[0] = px; row[1] = py; row[2] = pz;
    row[3] = ovx; row[4] = ovy; row[5] = ovz;
    row[6] = gx - px; row[7] = gy - py; row[8] = gz - pz;
    int col = 9;
    if constexpr (KS > 0) {
#pragma unroll
      for (int s = 0; s < KS - 1; ++s) {
        if (s < K) {
          float f0 = 0.f, f1 = 0.f, f2 = 0.f, f3 = 0.f;
          if (wj[s] < N) {
            const float4 q = lds_f4(ring + wj[s]);
            f0 = q.x - px; f1 = q.y - py; f2 = q.z - pz; f3 = wd[s];
          }
          row[col + 4 * s + 0] = f0; row[col + 4 * s + 1] = f1;
          row[col + 4 * s + 2] = f2; row[col + 4 * s + 3] = f3;
        }
      }
    }
    col += 4 * K;
    for (int s = 0; s < Ms; ++s) {
      float f0 = 0.f, f1 = 0.f, f2 = 0.f, f3 = 0.f;
      int m = 0x7fffffff;
      float d = 0.f;
      if constexpr (MSL > 0) {
#pragma unroll
        for (int u = 0; u < MSL - 1; ++u)
          if (u == s) { m = oj[u]; d = od[u]; }
      }
      if (m < Me) {
        const float4 q = lds_f4(obst4 + m);
        f0 = q.x - px; f1 = q.y - py; f2 = q.z - pz; f3 = d;
      }
      row[col + 4 * s + 0] = f0; row[col + 4 * s + 1] = f1;
      row[col + 4 * s + 2] = f2; row[col + 4 * s + 3] = f3;
    }
  };

  if ((mode != MODE_STEP && env_mask != nullptr) || (LM != 2 && P.obs_direct)) {
    // masked reset/observe (off the hot path), and small multi-team launches (latency-bound: the
    // LDS round trip and barriers of the staging lengthen every wave): rows straight to memory
    if (is_agent && sel) write_row(O.obs + (size_t)ag * D);
  } else {
    // chunks of CH rows staged in LDS, then 16-B coalesced stores of the contiguous block region
    long long nvalid = P.E - env0;
    if (nvalid > G) nvalid = G;
    const int rows = (int)nvalid * N;
    const int row_id = team * N + t;
    const int CH = P.chunk_rows;
    const int nthr = blockDim.x;
    float* dst0 = O.obs + env0 * N * D;
    for (int c = 0; c < G * N; c += CH) {  // block-uniform trip count
      if (is_agent && row_id >= c && row_id < c + CH) write_row(stage + (size_t)(row_id - c) * D);
      __syncthreads();
      const int nrow = rows - c < CH ? rows - c : CH;
      if (nrow > 0) {
        const int total = nrow * D;
        float* dst = dst0 + (long long)c * D;
        if (P.obs_vec4) {
          const int n4 = total >> 2;
          const float4* s4 = reinterpret_cast<const float4*>(stage);
          float4* d4 = reinterpret_cast<float4*>(dst);
          int i = tid;
          for (; i + 3 * nthr < n4; i += 4 * nthr) {
            const float4 a0 = s4[i], a1 = s4[i + nthr], a2 = s4[i + 2 * nthr], a3 = s4[i + 3 * nthr];
            d4[i] = a0; d4[i + nthr] = a1; d4[i + 2 * nthr] = a2; d4[i + 3 * nthr] = a3;
          }
          for (; i < n4; i += nthr) d4[i] = s4[i];
          for (int i = (n4 << 2) + tid; i < total; i += nthr) dst[i] = stage[i];
        } else {
          for (int i = tid; i < total; i += nthr) dst[i] = stage[i];
        }
      }
      __syncthreads();
    }
  }
  STAMP(8);
  STAMP_END(blockIdx.x, threadIdx.x == 0);
}
}  // namespace
namespace swarm_dev {

// ------------------------------------------------------------------ step64: the headline kernel
// Specialisation of the step for one env of exactly 64 drones per 64-lane wave, kinematic
// dynamics + swarm reward, K = 3 neighbours, Ms = 4 sensed obstacles, 4 <= M <= 16 obstacles
// (DroneEnvConfig defaults at N = 64: SURVEY.md §8d config 3).  Same phases, numerics and helper
// functions as swarm_kernel<0, 0, 4, 5, 2>; outputs are bit-identical to it
// (tests/test_gpu_step64.py).  Laid out for 8 waves per SIMD (<= 64 VGPRs, < 5 KB LDS per wave)
// so that every wave of the 8192-env headline launch is resident at once:
//  * env-uniform data (goal, step counter, episode, base addresses) lives in SGPRs and per-lane
//    addresses are 32-bit offsets from them (no per-lane 64-bit address arithmetic);
//  * a 96-entry structure-of-arrays position ring (drone j at j, and at j + 64 for j < 32):
//    rotation r reads soa[t + r] as base + immediate, two rotations per ds_read2_b32;
//  * the observation row is built in registers once, staged in LDS CH rows at a time and stored
//    with coalesced 16-B global stores.
constexpr int S64_N = 64;
constexpr int S64_K = 3;
constexpr int S64_MS = 4;
constexpr int S64_D = 9 + 4 * S64_K + 4 * S64_MS;  // 37
constexpr int S64_MMAX = 16;
constexpr int S64_RING = 96;
// obs rows per LDS staging chunk (multiple of 4: 16-B aligned chunks).  The staging buffer
// aliases the wave's ring and obstacles (dead once the rows are built in registers), so 32-row
// chunks (4.6 KB per wave, 148 KB for 32 waves per CU) fit: half the chunk passes and LDS row
// writes of 16-row chunks.
[[maybe_unused]] constexpr int S64_CH = S64_CH_ROWS;
constexpr int S64_HEADS = 8;  // env-queue heads, one per XCD (blockIdx mod 8)
constexpr int S64_HEAD_STRIDE = SWARM_WORK_WORDS / S64_HEADS;  // one 128-B line per head
[[maybe_unused]] constexpr int S64_WPS_DEFAULT = 0;  // persistent grid only on request (waves_per_simd > 0): slower here
constexpr int S64_MIN_WAVES = 6;    // register budget of swarm_step64 (<= 80 VGPRs)

// LDS ordering inside one wave: every LDS region of the step64 body belongs to one wave, whose
// LDS instructions execute in issue order, so a compiler fence is all that is needed (several
// envs share a workgroup without coupling their waves through s_barrier).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// XCD-aware workgroup order: the dispatcher places workgroup b on XCD b mod 8 (round robin), and
// each XCD's L2 fetches a line that two envs share (rows that are not 128-B multiples: step16q's
// 192-B position rows, every kernel's active bytes, goals, obstacles) once for each XCD that
// touches it.  The bijection below hands XCD x a contiguous block of workgroup slots, so
// neighbouring envs share an XCD and their shared lines are fetched once (r06e: TCC_EA0_RDREQ
// counts one 128-B request per line and XCD, tools/rdreq_probe.hip).  Envs are independent: the
// order never changes a result.
// Measured (r06f, three alternating pairs each): config 2 (step16q) 5.42-5.45 vs 5.74-5.75 us and reads
// 1.60 -> 1.05 MB; config 5 (step256w) 35.98-36.17 vs 36.16-36.50 us; the headline (step64_once,
// whose rows are whole lines: only active bytes, goals and obstacles are shared) within the spread
// (driver command 24.0-25.0 vs 23.8-24.4 us), so step64 keeps the dispatch order (SWARM_S64_XCD_MAP).
#ifndef SWARM_XCD_MAP
#define SWARM_XCD_MAP 1
#endif
#ifndef SWARM_S64_XCD_MAP
#define SWARM_S64_XCD_MAP 0
#endif
template <bool ON = SWARM_XCD_MAP != 0>
__device__ __forceinline__ int xcd_slot(int b, int nb) {
  if (!ON) return b;
  const int q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
  return x * q + (x < r ? x : r) + k;
}

// A wave's LDS: positions + obstacles during the step, the obs staging chunk afterwards.
// Positions are held twice: `ring` (float4 per drone, for the exact finish and the obs row) and
// the pair-pass ring as structure-of-arrays `soa` (x, y, z, eligibility planes of S64_SOA
// floats; drone j at j and at j + 64 for j < 32), so that rotations r and r-1 of one coordinate
// are one ds_read2_b32 into a register pair, the operand of the packed-f32 distance math.
constexpr int S64_SOA = S64_RING;
template <int CH>
union S64Lds {
  struct {
    float4 ring[S64_N];
    float soa[4 * S64_SOA];
    float4 obst[S64_MMAX];
    float osoa[3 * S64_MMAX];  // obstacle x, y, z planes (packed-f32 obstacle pass)
  } w;
  float4 stage[CH * S64_D / 4];
};

// step64's pair pass: pair_pass_w64's rotation scheme (same keys, formation terms, mirror
// exchange and results, bit for bit) with the squared distances of two rotations per packed
// f32 operation: 3 v_pk_add + v_pk_mul + 2 v_pk_fma per two pairs instead of 12 VALU.  The
// arithmetic per element is sqsum_rank's (fma(z,z, fma(y,y, x*x)) of the same differences).
typedef float s64_f2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(3))) float s64_lds_cf;
typedef __attribute__((address_space(1))) uint8_t s64_gu8;
// F0: key slots filled before this group (the list starts empty at the pass's first group)
template <int KS, int PASS, bool FAST, int RT, int NB, bool MIRROR, int F0 = (KS > 0 ? KS : 1), class FS = double>
__device__ __forceinline__ void pair_group_s64(s64_lds_cf* __restrict__ s0, uint32_t t4, float px, float py, float pz,
                                               bool self, uint32_t sflag, uint32_t keep, uint32_t keep_m, float ds,
                                               uint32_t (&nk)[KS > 0 ? KS : 1], float& smin, FS& fsum,
                                               float& macc) {
  float sq[NB], term[NB];
  bool el[NB];
  uint32_t v[NB];
  // FAST passes with keys send the own key to the mirror (no eligibility flags, no running
  // minimum, formation travels by DPP): the mirror needs only the key
  constexpr bool XKEY = FAST && KS > 0;
#pragma unroll
  for (int i = 0; i + 1 < NB; i += 2) {
    const s64_f2 X = {s0[RT - i], s0[RT - i - 1]};
    const s64_f2 Y = {s0[S64_SOA + RT - i], s0[S64_SOA + RT - i - 1]};
    const s64_f2 Z = {s0[2 * S64_SOA + RT - i], s0[2 * S64_SOA + RT - i - 1]};
    const s64_f2 dx = X - px, dy = Y - py, dz = Z - pz;
    s64_f2 s = dx * dx;
    s = __builtin_elementwise_fma(dy, dy, s);
    s = __builtin_elementwise_fma(dz, dz, s);
    sq[i] = s.x;
    sq[i + 1] = s.y;
  }
  if constexpr (NB % 2) {
    constexpr int i = NB - 1;
    sq[i] = sqsum_rank(s0[RT - i] - px, s0[S64_SOA + RT - i] - py, s0[2 * S64_SOA + RT - i] - pz);
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) el[i] = FAST ? true : (self & (s0[3 * S64_SOA + RT - i] != 0.f));
  float esum = 0.f;
  if constexpr (PASS == 1 && FAST) {
    // own_pair's FAST kinematic body with the formation differences d~ - d* of two rotations
    // in one v_pk_add_f32 (same values, same summation order)
    float dv[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) dv[i] = pair_value<PASS>(sq[i]);
#pragma unroll
    for (int i = 0; i + 1 < NB; i += 2) {
      const s64_f2 V = {dv[i], dv[i + 1]};
      const s64_f2 Ed = V - ds;
      term[i] = fabsf(Ed.x);
      term[i + 1] = fabsf(Ed.y);
    }
    if constexpr (NB % 2) term[NB - 1] = fabsf(dv[NB - 1] - ds);
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (KS > 0) {
        v[i] = (__float_as_uint(dv[i]) & keep) | (uint32_t)(RT - i);
        kins_n<KS>(nk, v[i], F0 + i);
      } else {
        v[i] = __float_as_uint(dv[i]);
        smin = fminf(smin, dv[i]);  // no keys: the running minimum decides pair collisions
      }
      esum += term[i];
    }
  } else if constexpr (XKEY) {
    // FAST keys-only passes (PASS 0 / 2): the own key, sent as is to the mirror (below)
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      v[i] = (__float_as_uint(pair_value<PASS>(sq[i])) & keep) | (uint32_t)(RT - i);
      kins_n<KS>(nk, v[i], F0 + i);
    }
  } else {
#pragma unroll
    for (int i = 0; i < NB; ++i)
      v[i] = own_pair<KS, PASS, FAST>(nk, sq[i], (uint32_t)(RT - i), el[i], keep, ds, smin, esum, term[i]);
  }
  if constexpr (MIRROR) {
    uint32_t rc[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i)
      rc[i] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(t4 + (uint32_t)(256 - 4 * (RT - i))), (int)(v[i] | sflag));
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (XKEY) {
        // the sender's key with its offset code RT - i swapped for the mirror's 64 - RT + i: one
        // v_xor_b32 (full rate) instead of v_and_or_b32 on the raw value (same key: the value
        // is >= 0, so keep and keep_m agree on it)
        kins_n<KS>(nk, rc[i] ^ ((uint32_t)(RT - i) ^ (uint32_t)(64 - RT + i)), F0 + NB + i);
      } else {
        mirror_pair<KS, PASS, FAST, false>(nk, rc[i], (uint32_t)(64 - RT + i), self, keep_m, ds, smin, esum);
      }
    }
    if constexpr (PASS == 1) {
#pragma unroll
      for (int i = 0; i < NB; ++i) macc = wave_ror1(macc) + term[i];
    }
  }
  if constexpr (PASS == 1) fsum += (FS)esum;
}
template <int KS, int PASS, bool FAST, int RT, int B, int F0 = (KS > 0 ? KS : 1), class FS = double>
__device__ __forceinline__ void pair_groups_s64(s64_lds_cf* __restrict__ s0, uint32_t t4, float px, float py, float pz,
                                                bool self, uint32_t sflag, uint32_t keep, uint32_t keep_m, float ds,
                                                uint32_t (&nk)[KS > 0 ? KS : 1], float& smin, FS& fsum,
                                                float& macc) {
  if constexpr (RT >= 1) {
    constexpr int NB = RT < B ? RT : B;
    constexpr int F1 = F0 + 2 * NB < KS ? F0 + 2 * NB : (KS > 0 ? KS : 1);
    pair_group_s64<KS, PASS, FAST, RT, NB, true, F0, FS>(s0, t4, px, py, pz, self, sflag, keep, keep_m, ds, nk, smin,
                                                         fsum, macc);
    pair_groups_s64<KS, PASS, FAST, RT - NB, B, F1, FS>(s0, t4, px, py, pz, self, sflag, keep, keep_m, ds, nk, smin,
                                                        fsum, macc);
  }
}
// `soa` = the wave's pair-pass ring (S64Lds::soa); lane t reads from soa + t.
template <int KS, int PASS, bool FAST>
__device__ __forceinline__ void pair_pass_s64(const float* __restrict__ soa, int t, float px, float py, float pz,
                                              bool self, uint32_t keep, float ds, uint32_t (&nk)[KS > 0 ? KS : 1],
                                              float& smin, double& fsum) {
  const uint32_t sflag = (FAST || self) ? 0u : 0x80000000u;
  const uint32_t keep_m = keep & 0x7fffffffu;
  const uint32_t t4 = (uint32_t)t << 2;
  // lane base &soa[t] as an opaque LDS address: every plane/rotation is then an immediate
  // offset of ds_read2_b32 (x, y, z planes within its 1020-B reach); derived from the wave's LDS
  // base, the compiler folds the plane offsets into one v_add per read instead
  s64_lds_cf* s0 = (s64_lds_cf*)(soa + t);
  asm volatile("" : "+v"(s0));
  float macc = 0.f;
  // the formation sum: one f32 chain over the pass (own terms group by group, the travelled mirror
  // sum, rotation 32), widened once — the f64 add per 4-rotation group cost a conversion and an
  // f64 add (both half rate) each; the sum's rounding stays ~1e-6 of the reward (1e-5 contract,
  // the mirror sum was already one f32 chain)
  using FS = typename std::conditional<SWARM_S64_F32SUM != 0, float, double>::type;
  FS fs = 0;
  // every caller starts the pass with an empty key list (F0 = 0)
  pair_groups_s64<KS, PASS, FAST, 31, S64_PAIR_BATCH, 0, FS>(s0, t4, px, py, pz, self, sflag, keep, keep_m, ds, nk,
                                                               smin, fs, macc);
  if constexpr (PASS == 1) fs += (FS)wave_ror1(macc);
  // rotation 32 pairs t with t+32 from both sides: own evaluation only
  pair_group_s64<KS, PASS, FAST, 32, 1, false, (KS > 0 ? KS : 1), FS>(s0, t4, px, py, pz, self, sflag, keep, keep_m,
                                                                      ds, nk, smin, fs, macc);
  if constexpr (PASS == 1) fsum += (double)fs;
}
// step64's obstacle pass: obstacle_pass's exact axis-path squared sums ((x*x + y*y) + z*z, no
// FMA) and keys for two obstacles per packed-f32 operation, from the obstacle planes `os`
// (x at os[m], y at os[16 + m], z at os[32 + m]; all lanes read the same word: LDS broadcast).
template <int MSL, bool COLL>
__device__ __forceinline__ void obstacle_pass_s64(const float* __restrict__ os, int M, float px, float py, float pz,
                                                  bool chk, float s_thr, uint32_t keep,
                                                  uint32_t (&ok)[MSL > 0 ? MSL : 1], bool& coll) {
  int m = 0;
  // software pipelined: pair m+2's planes are read while pair m is ranked (index clamped into
  // the 16-entry planes; the stale values of a pair past M are never used)
  s64_f2 X = {os[0], os[1]};
  s64_f2 Y = {os[S64_MMAX], os[S64_MMAX + 1]};
  s64_f2 Z = {os[2 * S64_MMAX], os[2 * S64_MMAX + 1]};
  // collisions: the running minimum of s over the obstacles (one v_min3_f32 per two) against
  // the threshold once at the end — the same boolean as a per-obstacle compare, without the
  // short-circuit exec-mask branches a `coll || ...` chain compiles to
  float omin = __builtin_inff();
  // `filled`: key slots filled before pair m (the list starts empty; the first two pairs are
  // peeled, M >= 4 for every caller: Ms = 4 <= M)
  auto pair = [&](int filled) {
    const int n = m + 2 < S64_MMAX - 1 ? m + 2 : S64_MMAX - 2;
    const s64_f2 Xn = {os[n], os[n + 1]};
    const s64_f2 Yn = {os[S64_MMAX + n], os[S64_MMAX + n + 1]};
    const s64_f2 Zn = {os[2 * S64_MMAX + n], os[2 * S64_MMAX + n + 1]};
    const s64_f2 dx = X - px, dy = Y - py, dz = Z - pz;
    X = Xn;
    Y = Yn;
    Z = Zn;
    const s64_f2 sq = (dx * dx + dy * dy) + dz * dz;
    if constexpr (MSL > 0) {
      kins_n<MSL>(ok, (__float_as_uint(sq.x) & keep) | (uint32_t)m, filled);
      kins_n<MSL>(ok, (__float_as_uint(sq.y) & keep) | (uint32_t)(m + 1), filled + 1);
    }
    if constexpr (COLL) {
      if constexpr (SWARM_OBST_OMIN) omin = fminf(omin, fminf(sq.x, sq.y));
      else coll = coll || (chk && ((sq.x <= s_thr) || (sq.y <= s_thr)));
    }
  };
  pair(0);
  m = 2;
  pair(2);
  for (m = 4; m + 1 < M; m += 2) pair(MSL > 0 ? MSL : 1);
  if (m < M) {
    const float sq = sqsum_f(os[m] - px, os[S64_MMAX + m] - py, os[2 * S64_MMAX + m] - pz);
    if constexpr (MSL > 0) kins<MSL>(ok, (__float_as_uint(sq) & keep) | (uint32_t)m);
    if constexpr (COLL) {
      if constexpr (SWARM_OBST_OMIN) omin = fminf(omin, sq);
      else coll = coll || (chk && (sq <= s_thr));
    }
  }
  if constexpr (COLL && SWARM_OBST_OMIN) coll = coll || (chk && omin <= s_thr);
}
__device__ __forceinline__ void s64_put_obst(float4* __restrict__ obst, float* __restrict__ os, int t, float ox,
                                             float oy, float oz) {
  obst[t] = make_float4(ox, oy, oz, 0.f);
  os[t] = ox; os[S64_MMAX + t] = oy; os[2 * S64_MMAX + t] = oz;
}

// Drone j's position from the float4 ring (one ds_read_b128; reading it across lanes with
// ds_bpermute instead conflicts as much and costs more LDS issue cycles)
__device__ __forceinline__ float4 s64_ring_gather(const float4* __restrict__ ring, int j, float, float, float) {
  return lds_f4(ring + j);
}

// Drone t's entry of both rings (float4 ring for the finish / obs row, SoA pair-pass ring).
__device__ __forceinline__ void s64_put(float4* __restrict__ ring, float* __restrict__ soa, int t, float px, float py,
                                        float pz, float w) {
  ring[t] = make_float4(px, py, pz, w);
  soa[t] = px; soa[S64_SOA + t] = py; soa[2 * S64_SOA + t] = pz; soa[3 * S64_SOA + t] = w;
  if (t < S64_SOA - S64_N) {
    soa[t + S64_N] = px; soa[S64_SOA + t + S64_N] = py; soa[2 * S64_SOA + t + S64_N] = pz;
    soa[3 * S64_SOA + t + S64_N] = w;
  }
}

// step64's finish in the common case, straight-line: N = 64 > K and M >= Ms fill every survivor
// slot, so finish_keys' per-slot validity branches (which serialise the nine exact-distance
// chains into separate basic blocks) are not needed.  The first K neighbour and Ms obstacle
// survivors get their exact distances as independent chains; the answer is finish_keys' own
// whenever no two survivors are a near-tie and the survivor bound holds.  Returns false for a
// lane that needs the general finish (finish_keys + exact_select); the caller runs that for the
// whole wave when any lane does (its answer for the other lanes is the same).
// Flags of s64_finish_fast (per lane): a near-tie among the neighbour / obstacle survivors, and
// the survivor bound failing on either side.
constexpr uint32_t S64F_NEAR_NB = 1u, S64F_NEAR_OB = 2u, S64F_BOUND_NB = 4u, S64F_BOUND_OB = 8u;
// BIG: the caller proved every survivor's squared distance is 0 or >= 2^-96 (sqrt_rn_big: the
// exact square roots without sqrt_rn's per-call wave test and branch, one basic block)
template <int KS, int MSL, bool BIG = false>
__device__ __forceinline__ uint32_t s64_finish_fast(const uint32_t (&nk)[KS], const uint32_t (&ok)[MSL],
                                                    const float4* __restrict__ ring, const float4* __restrict__ obst,
                                                    int t, int M, uint32_t nb_keep, uint32_t ob_keep, bool dkey,
                                                    float px, float py, float pz, float (&wd)[KS], int (&wj)[KS],
                                                    float (&od)[MSL], int (&oj)[MSL], float (&nd)[3 * (KS - 1)]) {
  constexpr int K = KS - 1, MS = MSL - 1;
  const uint32_t nim = ~nb_keep, oim = ~ob_keep;
  bool near_nb = false, near_ob = false;
#pragma unroll
  for (int s = 0; s + 1 < KS; ++s)
    near_nb = near_nb | (__uint_as_float(nk[s + 1] & nb_keep) <= __uint_as_float((nk[s] & nb_keep) | nim) * FAST_HI);
#pragma unroll
  for (int s = 0; s + 1 < MSL; ++s)
    near_ob = near_ob | ((ok[s + 1] != KEY_EMPTY) &
                         (__uint_as_float(ok[s + 1] & ob_keep) <= __uint_as_float((ok[s] & ob_keep) | oim) * FAST_HI));
#pragma unroll
  for (int s = 0; s < K; ++s) {
    const int j = (t + (int)(nk[s] & nim)) & (S64_N - 1);
    const float4 q = s64_ring_gather(ring, j, px, py, pz);
    const float dx = q.x - px, dy = q.y - py, dz = q.z - pz;
    wd[s] = BIG ? sqrt_rn_big(sqsum_1d(dx, dy, dz)) : sqrt_rn(sqsum_1d(dx, dy, dz));
    wj[s] = j;
    nd[3 * s] = dx; nd[3 * s + 1] = dy; nd[3 * s + 2] = dz;  // the obs row's neighbour columns
  }
  wd[K] = __builtin_inff();
  wj[K] = 0x7fffffff;
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    const int j = (int)(ok[s] & oim);
    const float4 q = lds_f4(obst + (j & (S64_MMAX - 1)));
    const float so = sqsum_f(q.x - px, q.y - py, q.z - pz);
    od[s] = BIG ? sqrt_rn_big(so) : sqrt_rn(so);
    oj[s] = j;
  }
  od[MS] = __builtin_inff();
  oj[MS] = 0x7fffffff;
  // survivor bounds (finish_keys' tails: APPROX neighbour keys, exact obstacle keys)
  const float nb_base = __uint_as_float(nk[K] & nb_keep) * FAST_LO;
  const float w = wd[K - 1];
  const bool ok_nb = dkey ? nb_base > w : nb_base > (w * w) * FAST_HI;
  const uint32_t last = ok[MS];
  const float wo = od[MS - 1];
  const bool ok_ob = last == KEY_EMPTY || (int)(last & oim) >= M ||
                     __uint_as_float(last & ob_keep) > (wo * wo) * FAST_HI;
  return (near_nb ? S64F_NEAR_NB : 0u) | (near_ob ? S64F_NEAR_OB : 0u) | (ok_nb ? 0u : S64F_BOUND_NB) |
         (ok_ob ? 0u : S64F_BOUND_OB);
}

// The rest of finish_keys for the lanes s64_finish_fast flagged, straight-line (finish_keys'
// per-slot validity branches serialise its exact-distance chains, and a wave in this path tends
// to be its launch's last): the exact distances of slots 0 .. K-1 / 0 .. MS-1 are s64_finish_fast's
// (the same formulas); a near-tie adds the last slot's and re-sorts all slots by (distance,
// index); then finish_keys' survivor bound on the sorted list.  Returns the lanes' (slow_nb,
// slow_ob): their answer needs exact_select.  Same results as finish_keys, slot for slot.
// NR drones in `ring`; ROT: neighbour keys carry an offset from drone t (step64), else the drone
// index (step256); MMAX obstacle slots in `obst`.
template <int KS, int MSL, int NR = S64_N, bool ROT = true, int MMAX = S64_MMAX>
__device__ __forceinline__ void s64_finish_general(uint32_t flags, const uint32_t (&nk)[KS], const uint32_t (&ok)[MSL],
                                                   const float4* __restrict__ ring, const float4* __restrict__ obst,
                                                   int t, int M, uint32_t nb_keep, uint32_t ob_keep, bool dkey,
                                                   float px, float py, float pz, float (&wd)[KS], int (&wj)[KS],
                                                   float (&od)[MSL], int (&oj)[MSL], bool& slow_nb, bool& slow_ob) {
  constexpr int K = KS - 1, MS = MSL - 1;
  const uint32_t nim = ~nb_keep, oim = ~ob_keep;
  const bool near_nb = (flags & S64F_NEAR_NB) != 0, near_ob = (flags & S64F_NEAR_OB) != 0;
  if (__ballot(near_nb) != 0) {
    // N > KS: slot K is always a drone
    const int j = ((ROT ? t : 0) + (int)(nk[K] & nim)) & (NR - 1);
    const float4 q = lds_f4(ring + j);
    const float d = sqrt_rn(sqsum_1d(q.x - px, q.y - py, q.z - pz));
    if (near_nb) {
      wd[K] = d;
      wj[K] = j;
#pragma unroll
      for (int a = 1; a < KS; ++a)
#pragma unroll
        for (int r = a; r > 0; --r) {
          const float x = wd[r - 1], y = wd[r];
          const int jx = wj[r - 1], jy = wj[r];
          const bool sw = (y < x) || (y == x && jy < jx);
          wd[r - 1] = sw ? y : x; wd[r] = sw ? x : y;
          wj[r - 1] = sw ? jy : jx; wj[r] = sw ? jx : jy;
        }
    }
  }
  if (__ballot(near_ob) != 0) {
    const uint32_t key = ok[MS];
    const int j = (int)(key & oim);
    const bool valid = key != KEY_EMPTY && j < M;
    const float4 q = lds_f4(obst + (j & (MMAX - 1)));
    const float d = sqrt_rn(sqsum_f(q.x - px, q.y - py, q.z - pz));
    if (near_ob) {
      od[MS] = valid ? d : __builtin_inff();
      oj[MS] = valid ? j : 0x7fffffff;
#pragma unroll
      for (int a = 1; a < MSL; ++a)
#pragma unroll
        for (int r = a; r > 0; --r) {
          const float x = od[r - 1], y = od[r];
          const int jx = oj[r - 1], jy = oj[r];
          const bool sw = (y < x) || (y == x && jy < jx);
          od[r - 1] = sw ? y : x; od[r] = sw ? x : y;
          oj[r - 1] = sw ? jy : jx; oj[r] = sw ? jx : jy;
        }
    }
  }
  // finish_keys' bound: the last key bounds every non-survivor (N = 64 > KS: it is a drone)
  const float nb_base = __uint_as_float(nk[K] & nb_keep);
  const float w = wd[K - 1];
  slow_nb = !(dkey ? nb_base * FAST_LO > w : nb_base * FAST_LO > (w * w) * FAST_HI);
  const uint32_t last = ok[MS];
  const float wo = od[MS - 1];
  slow_ob = !(last == KEY_EMPTY || (int)(last & oim) >= M || __uint_as_float(last & ob_keep) > (wo * wo) * FAST_HI);
}

// One env's inputs, loaded one env ahead of its compute (software pipeline): raw loaded values
// only — any arithmetic on them here would make the wave wait for the loads right away.
struct S64In {
  float px, py, pz, vx, vy, vz, ax, ay, az;  // lane t = drone t
  float ox, oy, oz;                          // lanes t < M: obstacle t
  uint32_t act, has;                         // raw bytes of active / action_mask
  float damp;                                // physics: drone t's linear damping
  uint32_t gse;  // lanes 0-2: goal x, y, z bits
  uint32_t se;   // lane 0: step count; lane 1: episode counter
};

// The kernel's only argument.  The body re-reads the fields it needs from the kernarg segment
// phase by phase (s64_args: an opaque copy of the kernarg pointer, so the compiler cannot keep
// the ~40 loop-invariant parameters and pointers live in SGPRs across the persistent loop and
// spill them; scalar-cache hits cost a few cycles).
// The eval tracker's per-step accumulators (swarm_out_t.eval, SWARM_EVAL_STEP_FUSED): device
// pointers of this launch's env rows, NULL status = off.
// A wave-uniform double (after a full butterfly) into SGPRs
__device__ __forceinline__ double s64_uniform(double v) {
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
struct S64Eval {
  double* ep_reward;
  int32_t* ep_steps;
  int32_t* reached_step;
  uint8_t* status;
  double* traveled;
  double* fe_sum;
  float* start;        // [E,N,3] episode start positions
  float* goal;         // [E,N,3] the protocol's goal estimate, start + obs[6:9]
  double* records;     // swarm_eval_t.records / count / capacity / update_index / seg_base / segments
  uint32_t* count;
  int32_t capacity, update_index, seg_base, segments;
  double spacing;      // DroneEnvConfig.desired_spacing (the formation error's d*)
};
struct S64Args {
  KParams P;
  swarm_state_t S;
  const float* actions;
  const uint8_t* amask;
  swarm_out_t O;
  S64Eval EV;
};
#define KARG __attribute__((address_space(4)))
typedef const KARG S64Args* S64ArgPtr;
// OFF: the S64Args block's byte offset in the kernarg segment (0, or behind a kernel's leading
// preloaded arguments: S64_HOT_BYTES)
template <uint32_t OFF = 0>
__device__ __forceinline__ S64ArgPtr s64_args() {
  uint64_t v = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr()) + OFF;
  asm volatile("" : "+s"(v));
  return reinterpret_cast<S64ArgPtr>(v);
}

// The one-wave-per-env step kernels' leading kernel arguments: the addresses of the loads the
// integrate waits for, plus E and M, which the gfx950 kernarg preload puts in SGPRs at wave start
// (this translation unit is built with -amdgpu-kernarg-preload-count=16; 14 user SGPRs are left
// for it): the env bound test and those global loads need no scalar load of the kernarg segment
// first.  The S64Args block follows them at byte offset S64_HOT_BYTES.
struct S64Hot {
  const float* pos;
  const float* vel;
  const float* actions;
  const uint8_t* active;
  const uint32_t* goal;
  const uint8_t* amask;  // NULL: every agent has an action
  int E, M;
};
constexpr uint32_t S64_HOT_BYTES = 56;
static_assert(alignof(S64Args) <= 8, "S64Args at kernarg offset 56");

template <int DYN = DYN_KIN>
__device__ __forceinline__ void s64_load(S64ArgPtr A, const S64Hot& H, int env, int t, S64In& c) {
  // 32-bit element offsets (E <= SPEC_MAX_E = 2^22, step64_applies: E x 64 x 3 < 2^32)
  const uint32_t ea = (uint32_t)env * S64_N;
  const uint32_t t3 = 3u * (uint32_t)t;
  const float* __restrict__ pe = H.pos + 3u * ea;
  const float* __restrict__ ve = H.vel + 3u * ea;
  const float* __restrict__ ae = H.actions + 3u * ea;
  c.gse = 0u;
  if (t < 3) c.gse = H.goal[3u * (uint32_t)env + (uint32_t)t];
  c.ax = ae[t3]; c.ay = ae[t3 + 1]; c.az = ae[t3 + 2];
  c.px = pe[t3]; c.py = pe[t3 + 1]; c.pz = pe[t3 + 2];
  c.vx = ve[t3]; c.vy = ve[t3 + 1]; c.vz = ve[t3 + 2];
  // unconditional loads (no phi with a default value: that would need the data at once)
  c.act = (H.active + ea)[t];
  c.has = (H.amask != nullptr ? H.amask : H.active)[ea + t];  // without a mask: ignored by the body
  // every load above is addressed from the leading (preloaded) arguments: all of them issue before
  // the first wait for a kernarg-segment scalar load (the addresses below)
  __builtin_amdgcn_sched_barrier(0);
  {  // env-uniform words, one per lane (a uniform load would be waited for at once); the two bases
    // pinned to SGPRs first (a lane-selected kernarg field became a per-lane load of the pointer)
    // (global-typed: made opaque, a plain pointer loses its address space and the load becomes a
    // flat load, which every later scalar-load wait would also wait for)
    typedef const __attribute__((address_space(1))) uint32_t gcu32;
    const gcu32* sp = (const gcu32*)A->S.step_count;
    const gcu32* ep = (const gcu32*)A->S.episode;
    asm volatile("" : "+s"(sp), "+s"(ep));
    c.se = (t == 0 ? sp : ep)[env];  // every lane (branch-free): lanes > 1 re-read the episode word
  }
  c.damp = 0.f;
  if constexpr (DYN == DYN_PHYS) c.damp = (A->S.damping + ea)[t];
  const int m = t < H.M ? t : H.M - 1;  // lanes >= M re-load the last obstacle (unused)
  const float* __restrict__ o = A->S.obstacles + 3u * ((uint32_t)env * (uint32_t)H.M + (uint32_t)m);
  c.ox = o[0]; c.oy = o[1]; c.oz = o[2];
  __builtin_amdgcn_sched_barrier(0);
}
// The leading arguments' values read from the S64Args block (kernels without preloaded arguments)
__device__ __forceinline__ S64Hot s64_hot(S64ArgPtr A) {
  return S64Hot{A->S.pos, A->S.vel, A->actions, A->S.active, reinterpret_cast<const uint32_t*>(A->S.goal), A->amask,
                (int)A->P.E, A->P.M};
}

// One env of the step (all phases) from its prefetched inputs.
// `prefetch` runs once every input has been consumed (after the integrate phase): it may
// overwrite `c` with the next env's inputs, whose loads then overlap the rest of this env.
// LANDED: wait for them (and the queue ticket) after the pair pass, before this env issues any
// store — vmcnt counts loads and stores in order, so a wait left to the next env's first use would
// also wait for this env's stores.
template <int CH, bool LANDED, class Prefetch, int DYN = DYN_KIN, bool EVAL = false, uint32_t AOFF = 0>
__device__ __forceinline__ void s64_env(const int env, const int M, const S64In& c, float4* __restrict__ ring,
                                        float4* __restrict__ obst, float* __restrict__ stage, const int lane,
                                        Prefetch&& prefetch) {
  constexpr int KS = S64_K + 1, MSL = S64_MS + 1, D = S64_D;
  static_assert(CH % 4 == 0 && S64_N % CH == 0, "chunk rows");
  // opaque copy of the lane index: keeps the ~40 lane-derived addresses and constants of the
  // body (ds_bpermute sources, Philox products) from being hoisted out of the persistent loop,
  // where they would be live across the whole body and spill
  int t = lane;
  asm volatile("" : "+v"(t));
  const unsigned t3 = 3u * (unsigned)t;
  const size_t ea = (size_t)env * S64_N;  // first agent of the env (uniform)
  float* __restrict__ const soa = reinterpret_cast<float*>(ring + S64_N);  // S64Lds::w.soa
  S64ArgPtr A = s64_args<AOFF>();  // re-fetched at every phase boundary
  STAMP_VAR(const int srec = env + (int)A->P.env_offset);  // stamp record: the global env (env groups)
  STAMP_AT(srec, 0);
  STAMP_BEGIN(srec, (threadIdx.x & 63) == 0);

  // ---- inputs (prefetched): env-uniform scalars, per-lane rows, obstacles to LDS
  float gx = __uint_as_float(__builtin_amdgcn_readlane(c.gse, 0));
  float gy = __uint_as_float(__builtin_amdgcn_readlane(c.gse, 1));
  float gz = __uint_as_float(__builtin_amdgcn_readlane(c.gse, 2));
  float ax = c.ax, ay = c.ay, az = c.az;
  uint32_t hraw = c.has;
  // pinned here: left to the compiler, the action / mask loads sank into the `act` branch of the
  // integrate and issued only after every earlier load had returned (a second round trip)
  asm volatile("" : "+v"(ax), "+v"(ay), "+v"(az), "+v"(hraw));
  const bool has = s64_args<AOFF>()->amask == nullptr || hraw != 0;
  float px = c.px, py = c.py, pz = c.pz;
  float vx = c.vx, vy = c.vy, vz = c.vz;
  bool act = c.act != 0;
  float* __restrict__ const osoa = reinterpret_cast<float*>(obst + S64_MMAX);  // S64Lds::w.osoa
  const int n_active = __popcll(__ballot(act));
  STAMP_AT(srec, 1);

  // ---- integrate: drone_swarm_env.py:98-117 (identical to swarm_kernel, DYN_KIN) or the
  // point-mass physics substeps (identical to swarm_kernel, DYN_PHYS)
  float prev_d = 0.f;
  float damp = c.damp;
  if constexpr (DYN == DYN_PHYS) {
    const float h = A->P.h;
    const float amax = A->P.amax, vmax = A->P.vmax, s_vmax = A->P.s_vmax;
    const float cx = has ? ax * amax : 0.f;
    const float cy = has ? ay * amax : 0.f;
    float cz = has ? az * amax + A->P.gcomp : 0.f;
    cz = cz + A->P.g;
    const bool law0 = A->P.damping_law == 0;
    float fac = 1.f;
    if (!law0) fac = (float)pow((double)(1.f - damp), (double)h);
    const int substeps = A->P.substeps;
    for (int s = 0; s < substeps; ++s) {
      const float s_sp = sqsum_1d(vx, vy, vz);
      float sp2 = 0.f;
      if (has && s_sp > s_vmax) {
        const float sp = sqrt_rn(s_sp);
        vx = (vx / sp) * vmax;
        vy = (vy / sp) * vmax;
        vz = (vz / sp) * vmax;
        if (law0) sp2 = sqrt_rn(sqsum_1d(vx, vy, vz));
      } else if (law0) {
        sp2 = sqrt_rn(s_sp);
      }
      if (law0) {
        const float cc = damp * (1.f + sp2);
        vx = vx + h * (cx - cc * vx);
        vy = vy + h * (cy - cc * vy);
        vz = vz + h * (cz - cc * vz);
      } else {
        vx = (vx + h * cx) * fac;
        vy = (vy + h * cy) * fac;
        vz = (vz + h * cz) * fac;
      }
      px = px + h * vx;
      py = py + h * vy;
      pz = pz + h * vz;
    }
  } else if (act) {
    prev_d = sqrt_rn(sqsum_1d(gx - px, gy - py, gz - pz));
    zero_unless(has, ax, ay, az);
    ax = clampf(ax, -1.f, 1.f) * A->P.amax;
    ay = clampf(ay, -1.f, 1.f) * A->P.amax;
    az = clampf(az, -1.f, 1.f) * A->P.amax;
    vx = vx + ax * A->P.dt;
    vy = vy + ay * A->P.dt;
    vz = vz + az * A->P.dt;
    const float s_sp = sqsum_1d(vx, vy, vz);
    if (!(s_sp <= A->P.s_vmax)) {  // sqrt_rn(s_sp) <= vmax otherwise: the speed is needed only here
      const float sp = sqrt_rn(s_sp);
      if (!(sp <= A->P.vmax || sp < (float)1e-8)) {
        vx = (vx / sp) * A->P.vmax;
        vy = (vy / sp) * A->P.vmax;
        vz = (vz / sp) * A->P.vmax;
      }
    }
    px = px + vx * A->P.dt;
    py = py + vy * A->P.dt;
    pz = pz + vz * A->P.dt;
  }
  if (DYN == DYN_KIN && n_active > 0) {
    px = clampf(px, A->P.neg_half_w, A->P.half_w);
    py = clampf(py, A->P.neg_half_w, A->P.half_w);
    pz = clampf(pz, A->P.neg_half_w, A->P.half_w);
  }
  // obstacles to LDS and the step / episode words here, after the integrate: their loads
  // (addressed from the kernarg segment, issued last) land while it runs
  if (t < M) s64_put_obst(obst, osoa, t, c.ox, c.oy, c.oz);
  const int stepc = (int)__builtin_amdgcn_readlane(c.se, 0);
  const uint32_t episode0 = (uint32_t)__builtin_amdgcn_readlane(c.se, 1);
  // eligibility: active drones (kinematic), every drone (physics contacts)
  s64_put(ring, soa, t, px, py, pz, (DYN == DYN_PHYS || act) ? 1.f : 0.f);
  wave_sync();
  prefetch();  // `c` is dead from here on
  STAMP_AT(srec, 2);
  A = s64_args<AOFF>();

  // ---- pair + obstacle passes
  uint32_t nk[KS], ok[MSL];
#pragma unroll
  for (int s = 0; s < KS; ++s) nk[s] = KEY_EMPTY;
#pragma unroll
  for (int s = 0; s < MSL; ++s) ok[s] = KEY_EMPTY;
  bool ocoll = false;
  float smin = __builtin_inff();
  double fsum = 0.0;
  const bool fast = DYN == DYN_PHYS || __all(act);
  bool early = false;  // kinematic: the episode ends whatever the pair pass finds (no keys needed)
  if constexpr (DYN == DYN_PHYS) {  // s' keys, no formation; every drone is a contact candidate
    pair_pass_s64<KS, 2, true>(soa, t, px, py, pz, true, A->P.nb_keep, 0.f, nk, smin, fsum);
    obstacle_pass_s64<MSL, true>(osoa, M, px, py, pz, true, A->P.s_phys_obst, A->P.ob_keep, ok, ocoll);
  } else {
    // obstacle pass first: an obstacle collision (or the time limit) ends the episode whatever
    // the pair pass finds, so such an env — ~half of the resetting ones — runs the pair pass
    // without neighbour keys (they would rank the positions the reset replaces): formation terms
    // and the running minimum only, the same sums bit for bit
    obstacle_pass_s64<MSL, true>(osoa, M, px, py, pz, act, A->P.s_obst, A->P.ob_keep, ok, ocoll);
    A = s64_args<AOFF>();
    early = fast && A->P.auto_reset &&
            (__ballot(act && ocoll) != 0 || stepc + 1 >= A->P.max_steps);
    if (early) {
      uint32_t nk0[1] = {KEY_EMPTY};
      pair_pass_s64<0, 1, true>(soa, t, px, py, pz, true, A->P.nb_keep, A->P.ds_f, nk0, smin, fsum);
    } else if (fast) {
      pair_pass_s64<KS, 1, true>(soa, t, px, py, pz, true, A->P.nb_keep, A->P.ds_f, nk, smin, fsum);
    } else pair_pass_s64<KS, 1, false>(soa, t, px, py, pz, act, A->P.nb_keep, A->P.ds_f, nk, smin, fsum);
  }
  if constexpr (LANDED) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the next env's inputs are in
  STAMP_AT(srec, 3);
  A = s64_args<AOFF>();

  // ---- exact top-K (finish_keys, rare exact_select)
  float wd[KS], od[MSL];
  int wj[KS], oj[MSL];
  // the obs row's neighbour columns p_j - p: the finish's own differences, kept
  // in registers to the row build instead of a second random ring gather (LDS bank conflicts)
  float nd[3 * S64_K];
  auto regather_nd = [&]() {
#pragma unroll
    for (int s = 0; s < S64_K; ++s) {
      const float4 q = s64_ring_gather(ring, wj[s] & (S64_N - 1), px, py, pz);
      nd[3 * s] = q.x - px; nd[3 * s + 1] = q.y - py; nd[3 * s + 2] = q.z - pz;
    }
  };
  auto select_topk = [&](bool dkey) {
    uint32_t fflags;
    // the nearest keys bound every survivor's squared distance from below: a d~ key >= 2^-47 (or
    // an s' key >= 2^-94; s' and d~ within 2^-20 of exact) and an exact obstacle key >= 2^-95 put
    // every exact s the finish takes the square root of above sqrt_rn's 2^-96 slow-path limit
    const bool big = SWARM_S64_BIGSQRT &&
                     __ballot(!(__uint_as_float(nk[0] & A->P.nb_keep) >= (dkey ? 0x1p-47f : 0x1p-94f) &&
                                __uint_as_float(ok[0] & A->P.ob_keep) >= 0x1p-95f)) == 0;
    if (big)
      fflags = s64_finish_fast<KS, MSL, true>(nk, ok, ring, obst, t, M, A->P.nb_keep, A->P.ob_keep, dkey, px, py, pz,
                                              wd, wj, od, oj, nd);
    else
      fflags = s64_finish_fast<KS, MSL>(nk, ok, ring, obst, t, M, A->P.nb_keep, A->P.ob_keep, dkey, px, py, pz, wd,
                                        wj, od, oj, nd);
    const uint64_t fails = __ballot(fflags != 0);
    if (fails == 0) return;
    bool slow_nb, slow_ob;
    s64_finish_general<KS, MSL>(fflags, nk, ok, ring, obst, t, M, A->P.nb_keep, A->P.ob_keep, dkey, px, py, pz, wd, wj,
                                od, oj, slow_nb, slow_ob);
    if (slow_nb) exact_select<KS, false>(ring, S64_N, t, S64_K, max_first(wd, S64_K), px, py, pz, wd, wj);
    if (slow_ob) exact_select<MSL, true>(obst, M, -1, S64_MS, max_first(od, S64_MS), px, py, pz, od, oj);
    regather_nd();  // the general finish may have re-ranked the neighbours
  };
  STAMP_AT(srec, 4);

  // ---- rewards / terminations: drone_swarm_env.py:120-172
  // The pair collision comes from the nearest key, not from the exact top-K: the finish runs
  // only for the observation that is emitted (after the reset decision), so a resetting env
  // pays one finish, not two.  Fast path: the nearest key bounds the exact nearest distance,
  // [key & keep, key | ~keep] x [FAST_LO, FAST_HI] (truncated d~ within 2^-21 of exact); only
  // a nearest distance inside that band (~1e-5 of the threshold) needs the exact scan.
  bool pcoll;
  float curr, rew = 0.f;
  bool reached = false, collided = false;
  bool term = false, trunc = false, cont = false, term_all = false, trunc_all = false;
  int new_step = stepc;
  if constexpr (DYN == DYN_PHYS) {
    // drone_physics_env.py:362-419 restated (swarm_kernel, DYN_PHYS): s' keys, every drone a
    // contact candidate (fast), the nearest key decides against the contact threshold
    const uint32_t keep = A->P.nb_keep;
    const float thr = A->P.s_phys_pair;
    pcoll = __uint_as_float(nk[0] | ~keep) * FAST_HI <= thr;
    if (!pcoll && __uint_as_float(nk[0] & keep) * FAST_LO <= thr)
      pcoll = key_zero_hit<false>(nk[0], keep, thr) || exact_pair_collision(ring, S64_N, t, px, py, pz, thr);
    const double dx = (double)px - (double)gx;
    const double dy = (double)py - (double)gy;
    const double dz = (double)pz - (double)gz;
    const double dist_phys = dsqrt_rn(((dx * dx) + (dy * dy)) + (dz * dz));
    curr = (float)dist_phys;
    collided = ocoll || pcoll || (pz <= A->P.ground_z);
    reached = dist_phys < A->P.goal_radius;
    if (act) {
      double r = (-dist_phys) * 0.1;
      if (collided) r = r - 10.0;
      else if (reached) r = r + 50.0;
      rew = (float)r;
    }
    const bool any_c = __ballot(act && collided) != 0;
    const bool any_notall = __ballot(act && !collided && !reached) != 0;
    new_step = stepc + 1;
    const bool tl = new_step >= A->P.max_steps;
    const bool done = any_c || !any_notall || tl;
    trunc_all = done && tl && !any_c && any_notall;
    term_all = done && !trunc_all;
    term = term_all;
    trunc = trunc_all;
    cont = true;
  } else {
    if (fast && !early) {
      const uint32_t keep = A->P.nb_keep;
      pcoll = __uint_as_float(nk[0] | ~keep) * FAST_HI <= A->P.thr_pair;
      if (!pcoll && __uint_as_float(nk[0] & keep) * FAST_LO <= A->P.thr_pair)
        pcoll = key_zero_hit<true>(nk[0], keep, A->P.s_pair) ||
                exact_pair_collision(ring, S64_N, t, px, py, pz, A->P.s_pair);
    } else {
      pcoll = smin <= A->P.thr_pair * FAST_LO;
      if (!pcoll && smin <= A->P.thr_pair * FAST_HI && act)
        pcoll = exact_pair_collision(ring, S64_N, t, px, py, pz, A->P.s_pair);
    }
    curr = sqrt_rn(sqsum_1d(gx - px, gy - py, gz - pz));
    if (act) {
      reached = (double)curr <= A->P.goal_radius;
      collided = ocoll || pcoll;
      double r = ((double)prev_d - (double)curr) * A->P.kp;
      if (n_active > 1) r = r + (-A->P.kf) * (fsum * inv_count(n_active - 1));
      if (reached) r = r + A->P.r_goal;
      if (collided) r = r + A->P.r_col;
      rew = (float)r;
    }
    const bool any_c = __ballot(act && collided) != 0;
    const bool any_cand = __ballot(act && !reached && !collided) != 0;
    if (n_active == 0) {  // drone_swarm_env.py:93-95
      term_all = true;
    } else {
      new_step = stepc + 1;
      const bool tl = new_step >= A->P.max_steps;
      term_all = (!any_cand && !any_c && !tl) || any_c;
      trunc_all = tl && !term_all;
      if (act) {
        const bool done_i = reached || collided;
        term = done_i;
        trunc = tl && !done_i;
        cont = !done_i && !tl && !any_c;
      }
    }
  }
  const bool do_reset = A->P.auto_reset && (term_all || trunc_all);
  (A->O.reward + ea)[t] = rew;
  if (A->O.dist_goal) (A->O.dist_goal + ea)[t] = curr;
  if (A->O.info_flags)
    (A->O.info_flags + ea)[t] = (uint8_t)((act ? SWARM_AGENT_STEPPED : 0u) | (act && reached ? SWARM_AGENT_REACHED : 0u) |
                                       (act && collided ? SWARM_AGENT_COLLISION : 0u) |
                                       (cont ? SWARM_AGENT_HAS_OBS : 0u));
  if (t == 0)
    A->O.env_done[env] = (uint8_t)((term_all ? SWARM_ENV_TERMINATED : 0u) | (trunc_all ? SWARM_ENV_TRUNCATED : 0u) |
                                (do_reset ? SWARM_ENV_RESET : 0u));
  const uint64_t m_term = __ballot(term), m_trunc = __ballot(trunc);
  bool ev_restart = false;  // fused eval: a live episode ended here and the env restarts
  if constexpr (EVAL) __builtin_amdgcn_sched_barrier(0);  // the finish's reads stay below the eval block
  if (EVAL && DYN == DYN_KIN && A->EV.status != nullptr) {
    // fused eval (out.eval, SWARM_EVAL_STEP_FUSED): everything swarm_eval_update does for one step
    // (swarm_eval.hip eval_update_kernel: the same arithmetic, the same f64 butterflies), with the
    // positions already in registers / LDS: episode reward += mean reward of the stepped agents,
    // steps, the first step all observed agents reached, the collision vote, path lengths, the
    // exact formation error of the observed drones, and at an episode's end its record
    const uint8_t status = A->EV.status[env];
    if (status & SWARM_EVAL_LIVE) {
      const bool coll = __ballot(cont && collided) != 0;
      const bool not_reached = __ballot(cont && !reached) != 0;
      const uint64_t m_obs = __ballot(cont);
      const int n_obs = __popcll(m_obs);
      if (cont) {
        // path length += |last - p| (evaluate_protocol.py's _distance: the sdot-double norm); last =
        // the position this step started from, still in the state (written back below): an agent
        // observed now was observed at the previous step or stands at its episode's start
        const float* po = A->S.pos + ea * 3 + t3;
        const float inc = sqrt_rn(sqsum_1d(po[0] - px, po[1] - py, po[2] - pz));
        double* tr = A->EV.traveled + ea + t;
        *tr = *tr + (double)inc;
      }
      // formation error (evaluate_protocol.py:103-116) of the observed drones: symmetric lane
      // rotations over the pair-pass ring (the emitted positions), each pair measured once,
      // 2 S_{r<32} + S_32 over n (n - 1) (eval_update_kernel's order, term for term); the wave
      // sums end uniform and are moved to SGPRs at once (short VGPR live ranges: the kernel runs
      // at 64 VGPRs)
      double fe = 0.0;
      if (n_obs > 1) {
        const double sp = A->EV.spacing;
        const bool all = n_obs == S64_N;
        // one pass: the square roots without sqrt_rn's per-call slow-path branch (a branch per
        // pair splits the loop into blocks the register allocator spills across); a coincident
        // pair (s' < 2^-96) on any lane redoes the pass with sqrt_rn, bit for bit the same terms
        // (a separate mask-free instance for the all-observed case measured much slower: more
        // dependency waits)
        auto pass = [&](auto sqrt_fn) -> double {
          // opaque ring base per pass: the two passes' reads must not be merged (96 values
          // would then stay live from the first pass into the second)
          // (an LDS-typed pointer: a plain `const float*` made opaque loses the address space and
          // every read became a flat load)
          s64_lds_cf* s0 = (s64_lds_cf*)(soa + t);
          asm volatile("" : "+v"(s0));
          double s_a = 0.0, s_b = 0.0;  // odd / even rotations (eval_update_kernel's two chains)
          // the term added under the lane's mask (|d - d*| as the add's source modifier: no
          // select, no zero); adding a skipped 0.0 never changed the sum, so the bits are the same
          auto add = [&](double& acc, int r) {
            const float d = sqrt_fn(sqsum_1d(px - s0[r], py - s0[S64_SOA + r], pz - s0[2 * S64_SOA + r]));
            const bool both = all || (cont && ((m_obs >> ((t + r) & (S64_N - 1))) & 1ull));
            if (both) acc += fabs((double)d - sp);
          };
#pragma unroll 1
          for (int r = 1; r < 31; r += 2) {
            add(s_a, r);
            add(s_b, r + 1);
          }
          add(s_a, 31);
          double s32 = 0.0;
          {
            const float d32 = sqrt_fn(sqsum_1d(px - s0[32], py - s0[S64_SOA + 32], pz - s0[2 * S64_SOA + 32]));
            const bool both32 = cont && ((m_obs >> ((t + 32) & (S64_N - 1))) & 1ull);
            if (both32) s32 = fabs((double)d32 - sp);
          }
          return 2.0 * (s_a + s_b) + s32;
        };
        double v;
        // no per-pair tiny-input test when the pair pass proves every pair is far from 0: its
        // nearest distance per lane (the nearest key's truncated d~, or the keyless pass's running
        // minimum) bounds every exact s from below (d~ >= 2^-47 gives s > 2^-95)
        const float near = early ? smin : __uint_as_float(nk[0] & A->P.nb_keep);
        if (fast && __ballot(!(near >= 0x1p-47f)) == 0) {
          v = pass([](float x) {
            bool unused = false;
            return sqrt_rn_nb(x, unused);
          });
        } else {
          bool tiny = false;
          v = pass([&](float x) { return sqrt_rn_nb(x, tiny); });
          if (__ballot(tiny) != 0) v = pass([](float x) { return sqrt_rn(x); });
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        fe = s64_uniform(v) / ((double)n_obs * (double)(n_obs - 1));
      }
      const bool ends = term_all || trunc_all;
      // path efficiency of an ending episode: mean over agents of |start - goal| / path length
      double pe = 0.0;
      if (ends) {
        const float* st0 = A->EV.start + (ea + t) * 3;
        const float* gl0 = A->EV.goal + (ea + t) * 3;
        const double tr = A->EV.traveled[ea + t];
        const float straight = sqrt_rn(sqsum_1d(st0[0] - gl0[0], st0[1] - gl0[1], st0[2] - gl0[2]));
        double q = tr > 1e-8 ? (double)straight / tr : 0.0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
        pe = s64_uniform(q) / (double)S64_N;
      }
      double rsum = (double)rew;  // 0 for agents without a reward entry
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) rsum += __shfl_xor(rsum, o);
      rsum = s64_uniform(rsum);
      if (t == 0) {
        const int steps = A->EV.ep_steps[env] + 1;
        int rs = A->EV.reached_step[env];
        if (!not_reached && rs < 0) rs = steps;
        const double ep_reward = A->EV.ep_reward[env] + (n_active > 0 ? rsum / (double)n_active : 0.0);
        const double fe_sum = A->EV.fe_sum[env] + fe;
        if (!ends) {
          A->EV.ep_reward[env] = ep_reward;
          A->EV.fe_sum[env] = fe_sum;
          A->EV.ep_steps[env] = steps;
          A->EV.reached_step[env] = rs;
          if (coll) A->EV.status[env] = (uint8_t)(status | SWARM_EVAL_COLLIDED);
        } else {
          // one record {env, success, collision-free, TTG, FE, PE, reward, steps, update}
          const bool coll_ep = coll || (status & SWARM_EVAL_COLLIDED);
          const long long genv = A->P.env_offset + env;
          const unsigned seg = (unsigned)(genv % SWARM_EVAL_SEGMENTS);
          const unsigned k = atomicAdd(A->EV.count + seg, 1u);
          const unsigned nseg = A->EV.segments > 0 ? (unsigned)A->EV.segments : (unsigned)SWARM_EVAL_SEGMENTS;
          const unsigned b = (seg + SWARM_EVAL_SEGMENTS - (unsigned)A->EV.seg_base % SWARM_EVAL_SEGMENTS) %
                             SWARM_EVAL_SEGMENTS;
          const unsigned cap = (unsigned)A->EV.capacity / nseg;
          if (b < nseg && k < cap) {
            double* rec = A->EV.records + ((size_t)b * cap + k) * SWARM_EVAL_RECORD;
            rec[0] = (double)genv;
            rec[1] = (!coll_ep && rs >= 0) ? 1.0 : 0.0;
            rec[2] = coll_ep ? 0.0 : 1.0;
            rec[3] = rs >= 0 ? (double)rs : __builtin_nan("");
            rec[4] = fe_sum / (double)steps;
            rec[5] = pe;
            rec[6] = ep_reward;
            rec[7] = (double)steps;
            rec[8] = (double)A->EV.update_index;
          }
          A->EV.ep_reward[env] = 0.0;
          A->EV.fe_sum[env] = 0.0;
          A->EV.ep_steps[env] = 0;
          A->EV.reached_step[env] = -1;
          A->EV.status[env] = do_reset ? (uint8_t)SWARM_EVAL_LIVE : (uint8_t)0;
        }
      }
      ev_restart = ends && do_reset;
    }
  }
  if constexpr (EVAL) __builtin_amdgcn_sched_barrier(0);
  STAMP_AT(srec, 5);
  A = s64_args<AOFF>();

  // ---- in-kernel auto-reset (wave-uniform): new episode, then its key passes
  uint32_t episode_new = episode0;
  if (do_reset) {
    const long long genv = A->P.env_offset + env;
    episode_new = episode0 + 1u;
    // two independent Philox chains per lane: drone t (block t), and obstacle t (block N + t) for
    // lanes t < M / the goal (block N + M) on lane M
    uint32_t w[4], wo[4];
    draw_block_k(A->P.seed_lo, A->P.seed_hi, genv, episode_new, (uint32_t)t, w);
    draw_block_k(A->P.seed_lo, A->P.seed_hi, genv, episode_new, (uint32_t)(S64_N + (t < M ? t : M)), wo);
    const float lo_w = A->P.neg_half_w, wd_w = A->P.width_w;
    px = uni(w[0], lo_w, wd_w);
    py = uni(w[1], lo_w, wd_w);
    pz = uni(w[2], lo_w, wd_w);
    vx = vy = vz = 0.f;
    act = true;
    const float ox = uni(wo[0], lo_w, wd_w), oy = uni(wo[1], lo_w, wd_w);
    float oz = uni(wo[2], lo_w, wd_w), goal_z = oz;
    if constexpr (DYN == DYN_PHYS) {  // drone_physics_env.py:205-242 ranges (swarm_kernel draw_env)
      pz = fmaxf(pz, 1.0f);
      damp = 0.5f * uni(w[3], 0.8f, 0.4f);
      goal_z = uni(wo[3], 0.5f, 1.5f);
      oz = fmaxf(oz, 0.5f);
    }
    wave_sync();  // every read of the old ring / obstacles is done
    if (t < M) s64_put_obst(obst, osoa, t, ox, oy, oz);
    gx = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(ox), M));
    gy = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(oy), M));
    gz = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(goal_z), M));
    s64_put(ring, soa, t, px, py, pz, 1.f);
    wave_sync();
#pragma unroll
    for (int s = 0; s < KS; ++s) nk[s] = KEY_EMPTY;
#pragma unroll
    for (int s = 0; s < MSL; ++s) ok[s] = KEY_EMPTY;
    bool c2 = false;
    float s2 = 0.f;
    double f2 = 0.0;
    pair_pass_s64<KS, 0, true>(soa, t, px, py, pz, true, A->P.nb_keep, 0.f, nk, s2, f2);
    obstacle_pass_s64<MSL, false>(osoa, M, px, py, pz, false, 0.f, A->P.ob_keep, ok, c2);
  }
  // one call site for both (the new episode's s' keys, the kinematic step pass's d~ keys; physics
  // ranks by s'): the finish and its general fallback are emitted once, not once per branch
  select_topk(DYN == DYN_KIN && !do_reset);

  STAMP_AT(srec, 6);
  A = s64_args<AOFF>();
  // ---- state write-back
  const bool new_act = do_reset || (DYN == DYN_PHYS ? (act && !(term_all || trunc_all)) : cont);
  float* __restrict__ posE = A->S.pos + ea * 3;
  float* __restrict__ velE = A->S.vel + ea * 3;
  posE[t3] = px; posE[t3 + 1] = py; posE[t3 + 2] = pz;
  velE[t3] = vx; velE[t3 + 1] = vy; velE[t3 + 2] = vz;
  {  // terminated, truncated, active: three 64-B rows of bytes built from wave ballots
    const uint64_t m_act = __ballot(new_act);
    // the three row pointers as uniform SGPR values: a lane-selected kernarg field would become
    // a per-lane load whose wait also drains every store issued before it
    // global-typed: made opaque, a plain pointer loses its address space and the row store becomes
    // a flat store, which every later `s_waitcnt lgkmcnt` (the obs stage) would also wait for
    s64_gu8* p_term = (s64_gu8*)A->O.terminated;
    s64_gu8* p_trunc = (s64_gu8*)A->O.truncated;
    s64_gu8* p_act = (s64_gu8*)A->S.active;
    asm volatile("" : "+s"(p_term), "+s"(p_trunc), "+s"(p_act));
    const int grp = t >> 4;
    if (grp < 3) {
      const uint64_t m = grp == 0 ? m_term : (grp == 1 ? m_trunc : m_act);
      const uint32_t nib = (uint32_t)(m >> (4 * (t & 15))) & 0xFu;
      const uint32_t word = (nib & 1u) | ((nib & 2u) << 7) | ((nib & 4u) << 14) | ((nib & 8u) << 21);
      s64_gu8* base = grp == 0 ? p_term : (grp == 1 ? p_trunc : p_act);
      *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(base + ea + 4 * (t & 15)) = word;
    }
  }
  if (t == 0) {
    A->S.step_count[env] = do_reset ? 0 : new_step;
    if (do_reset) {
      A->S.episode[env] = episode_new;
      A->S.goal[3 * env + 0] = gx; A->S.goal[3 * env + 1] = gy; A->S.goal[3 * env + 2] = gz;
    }
  }
  if (DYN == DYN_PHYS && do_reset) (A->S.damping + ea)[t] = damp;
  if (do_reset && t < M) {
    float* o = A->S.obstacles + ((size_t)env * M) * 3 + t3;
    const float4 q = obst[t];
    o[0] = q.x; o[1] = q.y; o[2] = q.z;
  }
  if (A->O.global_state) {
    float* gs = A->O.global_state + (size_t)env * (6 * S64_N + 3);
    gs[t3] = px; gs[t3 + 1] = py; gs[t3 + 2] = pz;
    gs[3 * S64_N + t3] = vx; gs[3 * S64_N + t3 + 1] = vy; gs[3 * S64_N + t3 + 2] = vz;
    if (t == 0) { gs[6 * S64_N + 0] = gx; gs[6 * S64_N + 1] = gy; gs[6 * S64_N + 2] = gz; }
  }
  if (EVAL && DYN == DYN_KIN && ev_restart) {
    // fused eval: the next episode opens from its first observation (eval_update_kernel's
    // restart: start = p, goal = p + obs[6:9] = p + (g - p), path length 0)
    float* st0 = A->EV.start + (ea + t) * 3;
    float* gl0 = A->EV.goal + (ea + t) * 3;
    st0[0] = px; st0[1] = py; st0[2] = pz;
    gl0[0] = px + (gx - px); gl0[1] = py + (gy - py); gl0[2] = pz + (gz - pz);
    A->EV.traveled[ea + t] = 0.0;
  }

  STAMP_AT(srec, 7);
  A = s64_args<AOFF>();
  // ---- observation row [p | v | g-p | K x (p_j-p, d) | Ms x (o_m-p, d)] (drone_swarm_env.py:226-291)
  float row[D];
  row[0] = px; row[1] = py; row[2] = pz;
  row[3] = vx; row[4] = vy; row[5] = vz;
  if constexpr (DYN == DYN_PHYS) {  // the obs velocity is clamped (drone_physics_env.py:438-442)
    const double dvx = (double)vx, dvy = (double)vy, dvz = (double)vz;
    const double nv = dsqrt_rn(((dvx * dvx) + (dvy * dvy)) + (dvz * dvz));
    if (nv > A->P.vmax_d) {
      row[3] = (float)((dvx / nv) * A->P.vmax_d);
      row[4] = (float)((dvy / nv) * A->P.vmax_d);
      row[5] = (float)((dvz / nv) * A->P.vmax_d);
    }
  }
  row[6] = gx - px; row[7] = gy - py; row[8] = gz - pz;
#pragma unroll
  for (int s = 0; s < S64_K; ++s) {
    row[9 + 4 * s] = nd[3 * s]; row[10 + 4 * s] = nd[3 * s + 1]; row[11 + 4 * s] = nd[3 * s + 2];
    row[12 + 4 * s] = wd[s];
  }
#pragma unroll
  for (int s = 0; s < S64_MS; ++s) {
    const float4 q = lds_f4(obst + (oj[s] & (S64_MMAX - 1)));
    row[21 + 4 * s] = q.x - px; row[22 + 4 * s] = q.y - py; row[23 + 4 * s] = q.z - pz; row[24 + 4 * s] = od[s];
  }
  constexpr int V4 = CH * D / 4;  // float4 per chunk
  wave_sync();  // the stage aliases ring / obstacles: every row-build read is issued before it
  const float4* s4 = reinterpret_cast<const float4*>(stage);
  float* srow = stage + (t % CH) * D;
#pragma unroll
  for (int ch = 0; ch < S64_N / CH; ++ch) {
    if (t / CH == ch) {
#pragma unroll
      for (int i = 0; i < D; ++i) srow[i] = row[i];
    }
    wave_sync();
    // all of the chunk's LDS reads in flight before the first store (a rolled `i += 64` loop
    // pays one LDS round trip per 1 KB).  The persistent loop (LANDED) has no registers to spare
    // for the 5 float4 and keeps the loop.
    if constexpr (LANDED) {
      for (int i = t; i < V4; i += 64) store_obs(A->O.obs + ea * D, S64_N * D * 4, 16u * (ch * V4 + i), s4[i]);
      wave_sync();
      continue;
    }
    constexpr int NF = V4 / 64, NR = V4 % 64;
    float4 v[NF + 1];
#pragma unroll
    for (int k = 0; k < NF; ++k) v[k] = s4[t + 64 * k];
    if (NR && t < NR) v[NF] = s4[t + 64 * NF];
#pragma unroll
    for (int k = 0; k < NF; ++k) store_obs(A->O.obs + ea * D, S64_N * D * 4, 16u * (ch * V4 + t + 64 * k), v[k]);
    if (NR && t < NR) store_obs(A->O.obs + ea * D, S64_N * D * 4, 16u * (ch * V4 + t + 64 * NF), v[NF]);
    wave_sync();
  }
  STAMP_AT(srec, 8);
  STAMP_END(srec, (threadIdx.x & 63) == 0);
}

// The kernel.  Without a work buffer (S.work == NULL): one env per workgroup.  With one: a
// persistent grid of G workgroups (waves_per_simd resident per SIMD).  Workgroups with
// blockIdx = x (mod H), H = min(8, G) — one XCD under the observed round-robin placement; that
// is locality only, never correctness — share the env range [E*x/H, E*(x+1)/H) and the queue
// head work[32x]: the k-th of them starts on env lo + k, every further env costs one returning
// device-scope atomicAdd on the head.  Every workgroup draws until its first failing ticket, so
// a launch draws exactly (envs beyond the first round) + (workgroups) tickets from each head, and
// the workgroup that draws the last one resets the head to 0 (the next launch on the stream sees
// it).  Envs are independent, so the env -> workgroup assignment never changes a result.
// Software pipeline: once env i has consumed its inputs (after integrate), the inputs of env i+1
// and the ticket of env i+2 are issued; they land while env i finishes, and env i's stores
// drain while env i+1 computes.

// One wave per env (the launch when the grid covers E): no loop, 8 waves per SIMD.  G envs per
// workgroup of G independent waves: 8192 one-wave workgroups take the dispatcher ~4 us to start,
// a quarter as many 4-wave ones about 1 us.
[[maybe_unused]] constexpr int S64_WG_ENVS = S64_WG_ENVS_C;
// The body of both one-wave-per-env kernels (kinematic / physics).
template <int CH, int G, int DYN, bool EVAL = false>
__device__ __forceinline__ void s64_once_body(const S64Hot& H) {
  __shared__ S64Lds<CH> lds[G];
  const int t = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int env = xcd_slot<SWARM_S64_XCD_MAP != 0>((int)blockIdx.x, (int)gridDim.x) * G + w;
  if (env >= H.E) return;  // whole wave (the last workgroup of a ragged E)
  S64In cur;
  s64_load<DYN>(s64_args<S64_HOT_BYTES>(), H, env, t, cur);
  s64_env<CH, false, void (*)(), DYN, EVAL, S64_HOT_BYTES>(env, H.M, cur, lds[w].w.ring, lds[w].w.obst,
                                                         reinterpret_cast<float*>(lds[w].stage), t, []() {});
}
// The once-kernels' leading arguments (S64Hot's fields, preloaded) and the S64Args block
#define S64_ONCE_PARAMS                                                                                          \
  const float *__restrict__ pos, const float *__restrict__ vel, const float *__restrict__ actions,              \
      const uint8_t *__restrict__ active, const uint32_t *__restrict__ goal, const uint8_t *__restrict__ amask, \
      int E, int M, const S64Args args
#define S64_ONCE_HOT S64Hot{pos, vel, actions, active, goal, amask, E, M}
}  // namespace swarm_dev
namespace {  // kernels: internal to this translation unit
template <int CH, int G>
__global__ void __launch_bounds__(64 * G) __attribute__((amdgpu_waves_per_eu(8)))
swarm_step64_once(S64_ONCE_PARAMS) {
  (void)args;  // read through s64_args<S64_HOT_BYTES>()
  s64_once_body<CH, G, DYN_KIN>(S64_ONCE_HOT);
}
}  // namespace
namespace swarm_dev {
// The physics restatement (DronePhysicsEnv, point mass) at the same shape: the
// same rings, passes, finish and obs staging, with the substep integrate, s' keys, contact
// thresholds, physics rewards / terminations, reset ranges and the clamped obs velocity of
// swarm_kernel<0, DYN_PHYS, 4, 5, 2>, bit for bit.
// The headline step with the evaluation protocol fused in (out.eval, SWARM_EVAL_STEP_FUSED):
// a separate instantiation, so the plain step's registers and schedule are untouched.
}  // namespace swarm_dev
namespace {  // kernels: internal to this translation unit
template <int CH, int G>
__global__ void __launch_bounds__(64 * G) __attribute__((amdgpu_waves_per_eu(S64_EVAL_WAVES)))
swarm_step64_eval_once(S64_ONCE_PARAMS) {
  (void)args;
  s64_once_body<CH, G, DYN_KIN, true>(S64_ONCE_HOT);
}
template <int CH, int G>
__global__ void __launch_bounds__(64 * G) __attribute__((amdgpu_waves_per_eu(8)))
swarm_step64_phys_once(S64_ONCE_PARAMS) {
  (void)args;
  s64_once_body<CH, G, DYN_PHYS>(S64_ONCE_HOT);
}
}  // namespace
namespace swarm_dev {

}  // namespace swarm_dev
namespace {  // kernels: internal to this translation unit
template <int CH>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(S64_MIN_WAVES)))
swarm_step64(const S64Args args) {
  (void)args;  // read through s64_args()
  __shared__ S64Lds<CH> lds;
  float4* const ring = lds.w.ring;
  float4* const obst = lds.w.obst;
  float* const stage = reinterpret_cast<float*>(lds.stage);
  const int t = threadIdx.x;
  uint32_t* head = nullptr;
  int env, base = 0;
  uint32_t n_dyn = 0, n_draws = 0;
  S64ArgPtr A = s64_args();
  const int M = A->P.M;
  if (A->S.work == nullptr) {
    env = blockIdx.x;
  } else {
    const int G = gridDim.x;
    const int H = G < S64_HEADS ? G : S64_HEADS;  // heads in use: every head has a workgroup
    const int x = blockIdx.x % H, k = blockIdx.x / H;
    const int lo = (int)(((long long)A->P.E * x) / H), hi = (int)(((long long)A->P.E * (x + 1)) / H);
    const int gx = (G - x + H - 1) / H;  // workgroups on this head
    const int n = hi - lo;
    env = k < n ? lo + k : -1;
    base = lo + gx;
    n_dyn = n > gx ? (uint32_t)(n - gx) : 0u;
    n_draws = n_dyn + (uint32_t)gx;
    head = A->S.work + S64_HEAD_STRIDE * x;
  }
  auto draw = [&]() -> uint32_t {  // issue only: the value is consumed one env later
    uint32_t v = 0xffffffffu;
    if (head != nullptr && t == 0) v = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
  };
  auto settle = [&](uint32_t v) -> int {
    if (head == nullptr) return -1;
    v = __builtin_amdgcn_readfirstlane(v);
    if (v == n_draws - 1u && t == 0) __hip_atomic_store(head, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v < n_dyn ? base + (int)v : -1;
  };
  S64In cur;
  const bool first = env >= 0;
  if (first) s64_load(A, s64_hot(A), env, t, cur);
  uint32_t ticket = draw();
  // the first env's inputs and ticket land here, so that no path into the loop header carries a
  // pending load (the in-loop ones are waited for mid-body, before any store): the header then
  // needs no vmcnt wait, which would also wait for the previous env's stores
  __builtin_amdgcn_s_waitcnt(0x0F70);
  while (env >= 0) {
    const int nxt = settle(ticket);
    s64_env<CH, true>(env, M, cur, ring, obst, stage, t, [&]() {
      if (nxt >= 0) {
        s64_load(s64_args(), s64_hot(s64_args()), nxt, t, cur);
        ticket = draw();
      }
    });
    env = nxt;
  }
  if (!first) settle(ticket);
}
}  // namespace
namespace swarm_dev {

// ------------------------------------------------------------------ step16q: config 2 (N = 16)
// BASELINE config 2 (N = 16 drones x E = 1024 envs) is a latency-bound launch: 1,024 envs of
// 16 drones fill a quarter of the SIMDs even as one env per wave, so the step time is the
// instruction latency of one wave, not the chip's throughput.  This specialisation puts one env
// in each 64-lane wave with FOUR lanes per drone (lane l = 4 d + q) and splits the per-drone work
// across the quarter q:
//  * pair pass: drone d's 15 partners are the symmetric rotations r = 1 .. 8 (r < 8 with a mirror
//    to drone d + r by ds_bpermute, r = 8 evaluated from both sides); quarter q takes r = q + 1
//    and q + 5, so a lane ranks 3-4 candidates instead of 15; the four partial top-4 lists are
//    merged across the quad with two DPP bitonic merges (12 min/max each), formation partial sums
//    and running minima with two DPP reductions;
//  * finish: quarter q computes the exact distance of neighbour slot q and obstacle slot q;
//  * observation row: quarter q stages its slots' 4-float groups, quarter 3 also p, v, g - p, in
//    LDS; the env's rows leave as coalesced 16-B stores.
// Three waves per env (192-thread workgroup): waves 0 and 1 both load and integrate the env, then
// wave 0 runs the formation / running-minimum pass, the obstacle collisions, rewards,
// terminations, flags and state, while wave 1 runs the keys pass, the exact finish and the
// observation rows of the continuing env; wave 2 prepares the next episode (q16_next_episode).
// One workgroup barrier hands wave 0's reset decision to waves 1 and 2.
// Integrate, obstacle pass, rewards and terminations run redundantly on the four lanes of a
// drone (identical values); every per-drone output is written by quarter 0.  Same numerics as
// swarm_kernel<0, 0, 4, 5, 1> (the generic kernel at N = 16), obs bit-identical
// (tests/test_gpu_step16.py).  Kinematic step, K = 3, Ms = 4, 4 <= M <= 16, no per-env records.
constexpr int Q_N = 16;
constexpr int Q_K = 3;
constexpr int Q_MS = 4;
constexpr int Q_D = 9 + 4 * Q_K + 4 * Q_MS;  // 37
constexpr int Q_MMAX = 16;
[[maybe_unused]] constexpr uint64_t Q_LEAD = 0x1111111111111111ull;  // quarter 0 of every drone

union Q16Lds {
  struct {
    float soa[4 * 32];  // x, y, z, eligibility planes; drone j at j and j + 16
    float4 ring[Q_N];
    float4 obst[Q_MMAX];
    float osoa[3 * Q_MMAX];
  };
  // the env's 16 obs rows (2,368 B), staged once the rows are in registers: the block leaves as
  // 148 aligned 16-B stores (whole 128-B lines) instead of 8-13 scattered dword stores per lane
  float4 stage[Q_N * Q_D / 4];
};

#if SWARM_HAS_PART(6)  // step16q's device code: its own translation unit
// step16q's leading kernel arguments: the addresses of the loads the integrate waits for, which
// the gfx950 kernarg preload puts in SGPRs at wave start (this translation unit is built with
// -amdgpu-kernarg-preload-count=16; 14 user SGPRs are left for it): those global loads issue
// without a scalar load of the kernarg segment first.  The S64Args block follows them at byte
// offset Q16_HOT_BYTES.  The launch is exactly E workgroups (no bounds test: it would wait for a
// kernarg load before the first global load).
struct Q16Hot {
  const float* pos;
  const float* vel;
  const float* actions;
  const uint8_t* active;
  const uint32_t* goal;
  const int32_t* step_count;
  const uint8_t* amask;  // NULL: every agent has an action
};
constexpr uint32_t Q16_HOT_BYTES = 56;
static_assert(alignof(S64Args) <= 8, "S64Args at kernarg offset 56");
__device__ __forceinline__ S64ArgPtr q16_args() {
  uint64_t v = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr()) + Q16_HOT_BYTES;
  asm volatile("" : "+s"(v));
  return reinterpret_cast<S64ArgPtr>(v);
}

// DPP quad permutations: xor 1, xor 2, broadcast of quad lane k
__device__ __forceinline__ uint32_t quad_xor1(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ uint32_t quad_xor2(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false); }
template <int K>
__device__ __forceinline__ float quad_bcast(float v) {
  constexpr int ctrl = K | (K << 2) | (K << 4) | (K << 6);
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xF, 0xF, false));
}
// Merge this lane's ascending 4-key list with the partner lane's (quad xor X): the 4 smallest of
// the union, ascending (bitonic: min(a_i, b_3-i), then a 4-element bitonic sort).
template <int X>
__device__ __forceinline__ void quad_merge4(uint32_t (&k)[4]) {
  uint32_t b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) b[i] = X == 1 ? quad_xor1(k[i]) : quad_xor2(k[i]);
  uint32_t c[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = min(k[i], b[3 - i]);
  const uint32_t c0 = min(c[0], c[2]), c2 = max(c[0], c[2]);
  const uint32_t c1 = min(c[1], c[3]), c3 = max(c[1], c[3]);
  k[0] = min(c0, c1); k[1] = max(c0, c1);
  k[2] = min(c2, c3); k[3] = max(c2, c3);
}
__device__ __forceinline__ float quad_sum(float v) {
  v = v + __uint_as_float(quad_xor1(__float_as_uint(v)));
  return v + __uint_as_float(quad_xor2(__float_as_uint(v)));
}
__device__ __forceinline__ float quad_min(float v) {
  v = fminf(v, __uint_as_float(quad_xor1(__float_as_uint(v))));
  return fminf(v, __uint_as_float(quad_xor2(__float_as_uint(v))));
}

// Exact (distance, index) keys for the quad-parallel fallback finish: the exact distance's float
// bits above the index, so one unsigned compare orders by distance, ties by index (the
// reference's stable order).
typedef unsigned long long q16_key;
__device__ __forceinline__ void q16_cx(q16_key& a, q16_key& b) {
  const q16_key lo = a < b ? a : b;
  b = a < b ? b : a;
  a = lo;
}
template <int X>
__device__ __forceinline__ q16_key quad_xor_key(q16_key v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  const uint32_t plo = X == 1 ? quad_xor1(lo) : quad_xor2(lo), phi = X == 1 ? quad_xor1(hi) : quad_xor2(hi);
  return ((q16_key)phi << 32) | plo;
}
// sort this lane's 4 keys, then two bitonic merges with the quad partners (as quad_merge4):
// every lane of the quad ends with the 4 smallest of the quad's 16 keys, ascending
__device__ __forceinline__ void q16_quad_select4(q16_key (&k)[4]) {
  q16_cx(k[0], k[1]); q16_cx(k[2], k[3]); q16_cx(k[0], k[2]); q16_cx(k[1], k[3]); q16_cx(k[1], k[2]);
#pragma unroll
  for (int x = 1; x <= 2; ++x) {
    q16_key c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const q16_key b = x == 1 ? quad_xor_key<1>(k[3 - i]) : quad_xor_key<2>(k[3 - i]);
      c[i] = k[i] < b ? k[i] : b;
    }
    q16_cx(c[0], c[2]); q16_cx(c[1], c[3]);
    q16_cx(c[0], c[1]); q16_cx(c[2], c[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) k[i] = c[i];
  }
}

// One quarter's share of the symmetric pair pass of drone d: rotations q + 1 and q + 5 (r = 8 has
// no mirror).  PASS 1: d~ values; PASS 0: s' keys only.  KEYS: the top-4 key list (merged over the
// quad); FORM (PASS 1): formation sum and running minimum (the minimum also on FAST passes without
// keys, where no nearest key decides the pair collision).
template <int PASS, bool FAST, bool KEYS = true, bool FORM = true>
__device__ __forceinline__ void q16_pair_pass(const float* __restrict__ soa, int d, int q, float px, float py, float pz,
                                              bool self, uint32_t keep, float ds, uint32_t (&nk)[4], float& smin,
                                              float& esum) {
  constexpr bool SUMS = PASS == 1 && FORM;
  constexpr bool MINS = SUMS && (!FAST || !KEYS);
  const uint32_t sflag = (FAST || self) ? 0u : 0x80000000u;
  const uint32_t keep_m = keep & 0x7fffffffu;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int r = q + 1 + 4 * it;
    const int j = d + r;  // ring index (wrap copy at j + 16)
    const float s = sqsum_rank(soa[j] - px, soa[32 + j] - py, soa[64 + j] - pz);
    const float v = PASS == 1 ? __builtin_amdgcn_sqrtf(s) : s;
    const bool el = FAST || (self && soa[96 + j] != 0.f);
    // the list starts empty: inserts 1 .. 4 of the pass skip the compares against KEY_EMPTY
    if constexpr (KEYS) kins_n<4>(nk, (__float_as_uint(v) & keep) | (uint32_t)r, 2 * it);
    if constexpr (MINS) smin = fminf(smin, el ? v : __builtin_inff());
    if constexpr (SUMS) esum += el ? fabsf(v - ds) : 0.f;
    // mirror: lane (d, q) receives drone (d - r)'s value of the pair (d - r, d) from lane 4(d - r) + q
    const int src = (((d - r) & (Q_N - 1)) << 2) | q;
    const uint32_t rcv = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)(__float_as_uint(v) | sflag));
    if (r < 8) {
      const float vm = __uint_as_float(rcv & 0x7fffffffu);
      const bool pr = FAST || (self && !(rcv >> 31));
      if constexpr (KEYS) kins_n<4>(nk, (rcv & keep_m) | (uint32_t)(Q_N - r), 2 * it + 1);
      if constexpr (MINS) smin = fminf(smin, pr ? vm : __builtin_inff());
      if constexpr (SUMS) esum += pr ? fabsf(vm - ds) : 0.f;
    }
  }
  if constexpr (KEYS) {
    quad_merge4<1>(nk);
    quad_merge4<2>(nk);
  }
  if constexpr (SUMS) esum = quad_sum(esum);
  if constexpr (MINS) smin = quad_min(smin);
}

// step16q's exact top-K of the emitted observation: quarter q measures neighbour slot q (q < 3)
// and obstacle slot q; near-ties / unproven bounds take the quad-parallel exact selection.
// dkey: the neighbour keys rank by d~ (PASS 1) instead of s' (PASS 0, a new episode's keys).
__device__ __forceinline__ void q16_finish(S64ArgPtr A, Q16Lds& L, int d, int q, int M, const uint32_t (&nk)[Q_K + 1],
                                           const uint32_t (&ok)[Q_MS + 1], bool dkey, float px, float py, float pz,
                                           float& nd, float& ndx, float& ndy, float& ndz, float& od, float& odx,
                                           float& ody, float& odz) {
  constexpr int KS = Q_K + 1, MSL = Q_MS + 1;
  const uint32_t nim = ~A->P.nb_keep, oim = ~A->P.ob_keep;
  {
    bool near_nb = false, near_ob = false;
#pragma unroll
    for (int s = 0; s + 1 < KS; ++s)
      near_nb = near_nb | (__uint_as_float(nk[s + 1] & A->P.nb_keep) <=
                           __uint_as_float((nk[s] & A->P.nb_keep) | nim) * FAST_HI);
#pragma unroll
    for (int s = 0; s + 1 < MSL; ++s)
      near_ob = near_ob | ((ok[s + 1] != KEY_EMPTY) & (__uint_as_float(ok[s + 1] & A->P.ob_keep) <=
                                                       __uint_as_float((ok[s] & A->P.ob_keep) | oim) * FAST_HI));
    // this quarter's slots (q = 3 has no neighbour slot: it repeats slot 2, unused)
    const uint32_t kn = q == 0 ? nk[0] : (q == 1 ? nk[1] : nk[2]);
    const int jn = (d + (int)(kn & nim)) & (Q_N - 1);
    const float4 qn = lds_f4(L.ring + jn);
    ndx = qn.x - px; ndy = qn.y - py; ndz = qn.z - pz;
    nd = sqrt_rn(sqsum_1d(ndx, ndy, ndz));
    const uint32_t ko = q == 0 ? ok[0] : (q == 1 ? ok[1] : (q == 2 ? ok[2] : ok[3]));
    const int jo = (int)(ko & oim) & (Q_MMAX - 1);
    const float4 qo = lds_f4(L.obst + jo);
    odx = qo.x - px; ody = qo.y - py; odz = qo.z - pz;
    od = sqrt_rn(sqsum_f(odx, ody, odz));
    // survivor bounds (finish_keys' tails) with slot K-1 / Ms-1 from quarters 2 / 3
    const float w2 = quad_bcast<2>(nd), w3 = quad_bcast<3>(od);
    const float nb_base = __uint_as_float(nk[Q_K] & A->P.nb_keep) * FAST_LO;
    const bool ok_nb = dkey ? nb_base > w2 : nb_base > (w2 * w2) * FAST_HI;
    const uint32_t last = ok[Q_MS];
    const bool ok_ob = last == KEY_EMPTY || (int)(last & oim) >= M ||
                       __uint_as_float(last & A->P.ob_keep) > (w3 * w3) * FAST_HI;
    // rare (near-ties, unproven bounds): an exact selection split over the quad — quarter q
    // measures neighbours d + q + 1 + 4i (obstacles q + 4i) exactly, then two DPP merges (what
    // exact_select does serially, in the reference's (distance, index) order); each side alone
    if (__ballot(near_nb || !ok_nb) != 0) {
      q16_key k4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = q + 1 + 4 * i;
        const int j = (d + r) & (Q_N - 1);
        const float4 pj = lds_f4(L.ring + j);
        const float dj = sqrt_rn(sqsum_1d(pj.x - px, pj.y - py, pj.z - pz));
        k4[i] = r < Q_N ? ((q16_key)__float_as_uint(dj) << 32) | (uint32_t)j : ~0ull;
      }
      q16_quad_select4(k4);
      const q16_key k2 = q == 0 ? k4[0] : (q == 1 ? k4[1] : k4[2]);
      nd = __uint_as_float((uint32_t)(k2 >> 32));
      const float4 qn2 = lds_f4(L.ring + ((int)k2 & (Q_N - 1)));
      ndx = qn2.x - px; ndy = qn2.y - py; ndz = qn2.z - pz;
    }
    if (__ballot(near_ob || !ok_ob) != 0) {
      q16_key k4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = q + 4 * i;
        const float4 om = lds_f4(L.obst + m);
        const float dm = sqrt_rn(sqsum_f(om.x - px, om.y - py, om.z - pz));
        k4[i] = m < M ? ((q16_key)__float_as_uint(dm) << 32) | (uint32_t)m : ~0ull;
      }
      q16_quad_select4(k4);
      const q16_key k2 = q == 0 ? k4[0] : (q == 1 ? k4[1] : (q == 2 ? k4[2] : k4[3]));
      od = __uint_as_float((uint32_t)(k2 >> 32));
      const float4 qo2 = lds_f4(L.obst + ((int)k2 & (Q_MMAX - 1)));
      odx = qo2.x - px; ody = qo2.y - py; odz = qo2.z - pz;
    }
  }
}

// step16q's observation rows [p | v | g-p | K x (p_j-p, d) | Ms x (o_m-p, d)]: the lanes' pieces
// into the LDS stage (aliasing the dead rings: every ring / obstacle read is issued before), then,
// by q16_store_obs, the env's block as 148 coalesced 16-B stores (whole 128-B lines)
__device__ __forceinline__ void q16_stage_row(Q16Lds& L, int d, int q, float px, float py, float pz, float vx, float vy,
                                              float vz, float gx, float gy, float gz, float nd, float ndx, float ndy,
                                              float ndz, float od, float odx, float ody, float odz) {
  wave_sync();
  float* row = reinterpret_cast<float*>(L.stage) + d * Q_D;
  if (q < 3) {
    row[9 + 4 * q] = ndx; row[10 + 4 * q] = ndy; row[11 + 4 * q] = ndz; row[12 + 4 * q] = nd;
  } else {
    row[0] = px; row[1] = py; row[2] = pz;
    row[3] = vx; row[4] = vy; row[5] = vz;
    row[6] = gx - px; row[7] = gy - py; row[8] = gz - pz;
  }
  row[21 + 4 * q] = odx; row[22 + 4 * q] = ody; row[23 + 4 * q] = odz; row[24 + 4 * q] = od;
  wave_sync();
}
__device__ __forceinline__ void q16_store_obs(S64ArgPtr A, const Q16Lds& L, size_t ea, int lane) {
  constexpr int V4 = Q_N * Q_D / 4;  // 148 float4: lanes take 64 + 64 + 20
  const float4 v0 = L.stage[lane], v1 = L.stage[lane + 64];
  const float4 v2 = L.stage[lane + 128 < V4 ? lane + 128 : V4 - 1];
  float* ob = A->O.obs + ea * Q_D;  // 16-B aligned: 2,368 B per env
  store_obs(ob, Q_N * Q_D * 4, 16u * (uint32_t)lane, v0);
  store_obs(ob, Q_N * Q_D * 4, 16u * (uint32_t)(lane + 64), v1);
  if (lane + 128 < V4) store_obs(ob, Q_N * Q_D * 4, 16u * (uint32_t)(lane + 128), v2);
}

// step16q's next-episode wave (wave 2 of an env's workgroup): a reset
// is deterministic before the step decides it — Philox4x32-10(seed, global env, episode + 1) —
// so while waves 0 and 1 step the env, this wave draws the next episode exactly as step16q's reset block
// does, runs its keys passes and exact finish and stages its observation rows.  At the decision
// (one workgroup barrier) it writes the new episode's state, global state and observations when
// the env resets, else it leaves.  The launch is latency-bound (one wave per SIMD): the reset's
// work comes off the critical path of the resetting envs' waves.
__device__ __forceinline__ void q16_next_episode(S64ArgPtr A, int env, int lane, Q16Lds& H,
                                                 const uint32_t* decision) {
  constexpr int MSL = Q_MS + 1;
  const int d = lane >> 2, q = lane & 3;
  const int M = A->P.M;
  const size_t ea = (size_t)env * Q_N;
  const size_t ag = ea + d;
  const uint32_t episode_new = A->S.episode[env] + 1u;
  const long long genv = A->P.env_offset + env;
  const uint32_t blk = q < 2 ? (uint32_t)d : (q == 2 ? (uint32_t)(Q_N + d) : (uint32_t)(Q_N + M));
  uint32_t wv[4];
  draw_block_k(A->P.seed_lo, A->P.seed_hi, genv, episode_new, blk, wv);
  const float lo_w = A->P.neg_half_w, wd_w = A->P.width_w;
  const float ux = uni(wv[0], lo_w, wd_w), uy = uni(wv[1], lo_w, wd_w), uz = uni(wv[2], lo_w, wd_w);
  const float px = quad_bcast<0>(ux), py = quad_bcast<0>(uy), pz = quad_bcast<0>(uz);
  const float gx = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(ux), 3));
  const float gy = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(uy), 3));
  const float gz = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(uz), 3));
  if (q == 2 && d < M) {
    H.obst[d] = make_float4(ux, uy, uz, 0.f);
    H.osoa[d] = ux; H.osoa[Q_MMAX + d] = uy; H.osoa[2 * Q_MMAX + d] = uz;
  }
  if (q == 0) {
    H.ring[d] = make_float4(px, py, pz, 1.f);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      H.soa[d + 16 * c] = px; H.soa[32 + d + 16 * c] = py; H.soa[64 + d + 16 * c] = pz;
      H.soa[96 + d + 16 * c] = 1.f;
    }
  }
  wave_sync();
  uint32_t nk[Q_K + 1], ok[MSL];
#pragma unroll
  for (int s = 0; s < Q_K + 1; ++s) nk[s] = KEY_EMPTY;
#pragma unroll
  for (int s = 0; s < MSL; ++s) ok[s] = KEY_EMPTY;
  float s2 = 0.f, e2 = 0.f;
  bool c2 = false;
  q16_pair_pass<0, true>(H.soa, d, q, px, py, pz, true, A->P.nb_keep, 0.f, nk, s2, e2);
  obstacle_pass_s64<MSL, false>(H.osoa, M, px, py, pz, false, 0.f, A->P.ob_keep, ok, c2);
  float nd, ndx, ndy, ndz, od, odx, ody, odz;
  q16_finish(A, H, d, q, M, nk, ok, false, px, py, pz, nd, ndx, ndy, ndz, od, odx, ody, odz);
  q16_stage_row(H, d, q, px, py, pz, 0.f, 0.f, 0.f, gx, gy, gz, nd, ndx, ndy, ndz, od, odx, ody, odz);
  __syncthreads();  // wave 0's decision
  if (*reinterpret_cast<const volatile uint32_t*>(decision) == 0u) return;
  A = q16_args();
  if (q == 0) {
    float* pe = A->S.pos + ag * 3;
    float* ve = A->S.vel + ag * 3;
    pe[0] = px; pe[1] = py; pe[2] = pz;
    ve[0] = 0.f; ve[1] = 0.f; ve[2] = 0.f;
  }
  if (lane == 0) {
    A->S.step_count[env] = 0;
    A->S.episode[env] = episode_new;
    A->S.goal[3 * env + 0] = gx; A->S.goal[3 * env + 1] = gy; A->S.goal[3 * env + 2] = gz;
  }
  if (q == 2 && d < M) {  // the obstacle this lane drew
    float* o = A->S.obstacles + ((size_t)env * M + d) * 3;
    o[0] = ux; o[1] = uy; o[2] = uz;
  }
  if (A->O.global_state && q == 0) {
    float* gs = A->O.global_state + (size_t)env * (6 * Q_N + 3);
    gs[3 * d] = px; gs[3 * d + 1] = py; gs[3 * d + 2] = pz;
    gs[3 * Q_N + 3 * d] = 0.f; gs[3 * Q_N + 3 * d + 1] = 0.f; gs[3 * Q_N + 3 * d + 2] = 0.f;
    if (d == 0) { gs[6 * Q_N + 0] = gx; gs[6 * Q_N + 1] = gy; gs[6 * Q_N + 2] = gz; }
  }
  q16_store_obs(A, H, ea, lane);
}

// One env's step inputs after the integrate (the step and observation waves hold the same values).
struct Q16Step {
  float px, py, pz, vx, vy, vz, gx, gy, gz, prev_d;
  int stepc, n_active;
  bool act, fast;
};
// One env's loaded words, not yet used (q16_load issues every load before anything waits for one)
struct Q16Raw {
  float ax, ay, az, ox, oy, oz;
  uint32_t gse, act, hm;
};

// Loads (the four lanes of a drone read the same words).
__device__ __forceinline__ void q16_load(S64ArgPtr A, const Q16Hot& H, int env, int lane, int M, Q16Step& st,
                                         Q16Raw& w) {
  // 32-bit element offsets (E <= SPEC_MAX_E, step16q_applies): 64-bit index arithmetic let the
  // register allocator tie an address's unused high half to the goal word's load register, a false
  // dependency that made every later load wait for that one
  const uint32_t ag = (uint32_t)env * Q_N + (uint32_t)(lane >> 2), ag3 = 3u * ag;
  w.gse = 0u;
  {
    const uint32_t* src = lane < 3 ? H.goal + 3u * (uint32_t)env + (uint32_t)lane
                                   : reinterpret_cast<const uint32_t*>(H.step_count) + (uint32_t)env;
    if (lane < 4) w.gse = *src;
  }
  w.ax = H.actions[ag3]; w.ay = H.actions[ag3 + 1]; w.az = H.actions[ag3 + 2];
  st.px = H.pos[ag3]; st.py = H.pos[ag3 + 1]; st.pz = H.pos[ag3 + 2];
  st.vx = H.vel[ag3]; st.vy = H.vel[ag3 + 1]; st.vz = H.vel[ag3 + 2];
  w.act = H.active[ag];
  // unconditional (a branch on the mask pointer made the later loads wait for every load above)
  w.hm = (H.amask != nullptr ? H.amask : H.active)[ag];
  // every load above is addressed from preloaded SGPRs: issue them all before the first wait for
  // a kernarg-segment scalar load (M and the obstacle base below)
  __builtin_amdgcn_sched_barrier(0);
  {  // obstacles (address from the kernarg segment): written to LDS after the integrate
    const int m = lane < M ? lane : M - 1;  // lanes >= M re-load the last obstacle (unused)
    const float* o = A->S.obstacles + 3u * ((uint32_t)env * (uint32_t)M + (uint32_t)m);
    w.ox = o[0]; w.oy = o[1]; w.oz = o[2];
  }
  __builtin_amdgcn_sched_barrier(0);
}

// Integrate (drone_swarm_env.py:98-117, swarm_kernel DYN_KIN), then this wave's rings.
__device__ __forceinline__ void q16_integrate(S64ArgPtr A, const Q16Hot& H, int lane, int M, Q16Lds& L, Q16Step& st,
                                              Q16Raw w) {
  const int d = lane >> 2, q = lane & 3;
  // the actions and the mask byte pinned here: left to the compiler, their loads sank into the
  // `act` branch below and issued only after the loads above had returned (a second round trip)
  asm volatile("" : "+v"(w.ax), "+v"(w.ay), "+v"(w.az), "+v"(w.hm));
  float ax = w.ax, ay = w.ay, az = w.az;
  const bool has = H.amask == nullptr || w.hm != 0u;
  st.act = w.act != 0u;
  st.gx = __uint_as_float(__builtin_amdgcn_readlane(w.gse, 0));
  st.gy = __uint_as_float(__builtin_amdgcn_readlane(w.gse, 1));
  st.gz = __uint_as_float(__builtin_amdgcn_readlane(w.gse, 2));
  st.stepc = (int)__builtin_amdgcn_readlane(w.gse, 3);
  st.n_active = __popcll(__ballot(st.act) & Q_LEAD);
  st.fast = (__ballot(st.act) & Q_LEAD) == Q_LEAD;
  const float ox = w.ox, oy = w.oy, oz = w.oz;
  float px = st.px, py = st.py, pz = st.pz, vx = st.vx, vy = st.vy, vz = st.vz;
  const float gx = st.gx, gy = st.gy, gz = st.gz;
  float prev_d = 0.f;
  if (st.act) {
    prev_d = sqrt_rn(sqsum_1d(gx - px, gy - py, gz - pz));
    zero_unless(has, ax, ay, az);
    ax = clampf(ax, -1.f, 1.f) * A->P.amax;
    ay = clampf(ay, -1.f, 1.f) * A->P.amax;
    az = clampf(az, -1.f, 1.f) * A->P.amax;
    vx = vx + ax * A->P.dt;
    vy = vy + ay * A->P.dt;
    vz = vz + az * A->P.dt;
    const float s_sp = sqsum_1d(vx, vy, vz);
    if (!(s_sp <= A->P.s_vmax)) {
      const float sp = sqrt_rn(s_sp);
      if (!(sp <= A->P.vmax || sp < (float)1e-8)) {
        vx = (vx / sp) * A->P.vmax;
        vy = (vy / sp) * A->P.vmax;
        vz = (vz / sp) * A->P.vmax;
      }
    }
    px = px + vx * A->P.dt;
    py = py + vy * A->P.dt;
    pz = pz + vz * A->P.dt;
  }
  if (st.n_active > 0) {
    px = clampf(px, A->P.neg_half_w, A->P.half_w);
    py = clampf(py, A->P.neg_half_w, A->P.half_w);
    pz = clampf(pz, A->P.neg_half_w, A->P.half_w);
  }
  if (lane < M) {
    L.obst[lane] = make_float4(ox, oy, oz, 0.f);
    L.osoa[lane] = ox; L.osoa[Q_MMAX + lane] = oy; L.osoa[2 * Q_MMAX + lane] = oz;
  }
  if (q == 0) {
    const float w_el = st.act ? 1.f : 0.f;
    L.ring[d] = make_float4(px, py, pz, w_el);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      L.soa[d + 16 * c] = px; L.soa[32 + d + 16 * c] = py; L.soa[64 + d + 16 * c] = pz;
      L.soa[96 + d + 16 * c] = w_el;
    }
  }
  st.px = px; st.py = py; st.pz = pz; st.vx = vx; st.vy = vy; st.vz = vz; st.prev_d = prev_d;
  wave_sync();
}

// step16q's observation wave (wave 1): the continuing env's observation — the keys pass on the
// post-step positions, the exact finish, the rows staged in LDS — while wave 0 computes rewards and
// terminations; stored once wave 0's reset decision says the env continues.
__device__ __forceinline__ void q16_obs_wave(S64ArgPtr A, int env, int lane, int M, Q16Lds& L, const Q16Step& st,
                                             const uint32_t* decision) {
  constexpr int KS = Q_K + 1, MSL = Q_MS + 1;
  const int d = lane >> 2, q = lane & 3;
  uint32_t nk[KS], ok[MSL];
#pragma unroll
  for (int s = 0; s < KS; ++s) nk[s] = KEY_EMPTY;
#pragma unroll
  for (int s = 0; s < MSL; ++s) ok[s] = KEY_EMPTY;
  float smin = __builtin_inff(), esum = 0.f;
  bool unused = false;
  if (st.fast) q16_pair_pass<1, true, true, false>(L.soa, d, q, st.px, st.py, st.pz, true, A->P.nb_keep, 0.f, nk, smin, esum);
  else q16_pair_pass<1, false, true, false>(L.soa, d, q, st.px, st.py, st.pz, st.act, A->P.nb_keep, 0.f, nk, smin, esum);
  obstacle_pass_s64<MSL, false>(L.osoa, M, st.px, st.py, st.pz, false, 0.f, A->P.ob_keep, ok, unused);
  STAMP_AT(env, 5);
  float nd, ndx, ndy, ndz, od, odx, ody, odz;
  q16_finish(A, L, d, q, M, nk, ok, true, st.px, st.py, st.pz, nd, ndx, ndy, ndz, od, odx, ody, odz);
  STAMP_AT(env, 6);
  q16_stage_row(L, d, q, st.px, st.py, st.pz, st.vx, st.vy, st.vz, st.gx, st.gy, st.gz, nd, ndx, ndy, ndz, od, odx,
                ody, odz);
  STAMP_AT(env, 7);
  A = q16_args();
  if (A->P.auto_reset) {
    __syncthreads();  // wave 0's decision
    if (*reinterpret_cast<const volatile uint32_t*>(decision) != 0u) return;
  }
  q16_store_obs(A, L, (size_t)env * Q_N, lane);
  STAMP_AT(env, 8);
  STAMP_END(env, lane == 0);
}

// step16q (one wave per SIMD, latency-bound) reads the kernarg segment through one pointer, so
// the compiler batches the parameter loads at the top instead of a dependent scalar round trip at
// each phase: 6.85 -> 6.80 us (step256 measured 46.8 -> 47.5-48.2 us that way and keeps step64's
// per-phase re-fetch).
// One env per 3-wave workgroup, the step's serial path split over two waves: wave 0 computes the
// rewards, terminations, flags and state (formation-only pair pass), wave 1 the continuing env's
// observation (keys-only pair pass, exact finish, rows), wave 2 the next episode
// (q16_next_episode); one workgroup barrier hands wave 0's reset decision to waves 1 and 2.
}  // namespace swarm_dev
namespace {  // kernels: internal to this translation unit
__global__ void __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(Q16_WAVES_PER_EU)))
swarm_step16q(const float* __restrict__ pos, const float* __restrict__ vel, const float* __restrict__ actions,
              const uint8_t* __restrict__ active, const uint32_t* __restrict__ goal,
              const int32_t* __restrict__ step_count, const uint8_t* __restrict__ amask, const S64Args args) {
  (void)args;  // read through q16_args()
  __shared__ Q16Lds ldsq[3];
  __shared__ uint32_t decision;  // wave 0's reset decision for waves 1 and 2
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  S64ArgPtr A = q16_args();
  const Q16Hot H{pos, vel, actions, active, goal, step_count, amask};
  const int env = xcd_slot((int)blockIdx.x, (int)gridDim.x);  // grid = E
  // the step's waves (the launch's critical path) issue ahead of the next-episode waves sharing
  // their SIMDs: 5.82-5.84 -> 5.71-5.73 us per step (priority 3 no better, r05aa)
  if (wv != 2) __builtin_amdgcn_s_setprio(1);
  if (wv == 2) {
    if (A->P.auto_reset) q16_next_episode(A, env, lane, ldsq[2], &decision);
    return;
  }
  Q16Lds& L = ldsq[wv];
  const int d = lane >> 2, q = lane & 3;
  const int M = A->P.M;
  const size_t ea = (size_t)env * Q_N;
  const size_t ag = ea + d;
  if (wv == 0) {
    STAMP_AT(env, 0);
    STAMP_BEGIN(env, lane == 0);
  }
  Q16Step st;
  Q16Raw w;
  q16_load(A, H, env, lane, M, st, w);
  if (wv == 0) STAMP_AT(env, 1);
  q16_integrate(A, H, lane, M, L, st, w);
  if (wv == 1) {
    q16_obs_wave(A, env, lane, M, L, st, &decision);
    return;
  }
  STAMP_AT(env, 2);
  Q16_FLAGS_DECL;
  const float px = st.px, py = st.py, pz = st.pz;
  const bool act = st.act;
  const int n_active = st.n_active;

  // ---- formation + running-minimum pass (no keys: wave 1 ranks the observation), obstacle
  // collisions
  uint32_t nk[4], ok[1] = {KEY_EMPTY};  // no neighbour keys in this pass (nk unused)
  float smin = __builtin_inff(), esum = 0.f;
  bool ocoll = false;
  if (st.fast) {
    q16_pair_pass<1, true, false, true>(L.soa, d, q, px, py, pz, true, A->P.nb_keep, A->P.ds_f, nk, smin, esum);
  } else {
    Q16_FLAG(8u);
    q16_pair_pass<1, false, false, true>(L.soa, d, q, px, py, pz, act, A->P.nb_keep, A->P.ds_f, nk, smin, esum);
  }
  obstacle_pass_s64<0, true>(L.osoa, M, px, py, pz, act, A->P.s_obst, A->P.ob_keep, ok, ocoll);
  STAMP_AT(env, 3);

  // ---- terminations first (drone_swarm_env.py:120-172, swarm_kernel DYN_KIN): the pair collision
  // from the running minimum of d~ (certain below the band, exact inside it), the goal test in
  // squared space ((double)sqrt_rn(s) <= goal_radius exactly when s <= s_goal), so the reset
  // decision reaches waves 1 and 2 before the reward's square root and f64 terms
  bool pcoll = smin <= A->P.thr_pair * FAST_LO;
  if (!pcoll && smin <= A->P.thr_pair * FAST_HI && act) {
    pcoll = exact_pair_collision(L.ring, Q_N, d, px, py, pz, A->P.s_pair);
    Q16_FLAG(2u);
  }
  const float s_goal = sqsum_1d(st.gx - px, st.gy - py, st.gz - pz);
  bool reached = false, collided = false, term = false, trunc = false, cont = false;
  bool term_all = false, trunc_all = false;
  int new_step = st.stepc;
  if (act) {
    reached = s_goal <= A->P.s_goal;
    collided = ocoll || pcoll;
  }
  const bool any_c = (__ballot(act && collided) & Q_LEAD) != 0;
  const bool any_cand = (__ballot(act && !reached && !collided) & Q_LEAD) != 0;
  if (n_active == 0) {
    term_all = true;
  } else {
    new_step = st.stepc + 1;
    const bool tl = new_step >= A->P.max_steps;
    term_all = (!any_cand && !any_c && !tl) || any_c;
    trunc_all = tl && !term_all;
    if (act) {
      const bool done_i = reached || collided;
      term = done_i;
      trunc = tl && !done_i;
      cont = !done_i && !tl && !any_c;
    }
  }
  const bool do_reset = A->P.auto_reset && (term_all || trunc_all);

  // ---- hand the reset decision to waves 1 (observation) and 2 (next episode)
  if (A->P.auto_reset) {
    if (lane == 0) decision = do_reset ? 1u : 0u;
    __syncthreads();
  }
  STAMP_AT(env, 4);
  A = q16_args();

  // ---- rewards and the per-agent / per-env outputs
  const float curr = sqrt_rn(s_goal);
  float rew = 0.f;
  if (act) {
    double r = ((double)st.prev_d - (double)curr) * A->P.kp;
    if (n_active > 1) r = r + (-A->P.kf) * ((double)esum * inv_count(n_active - 1));
    if (reached) r = r + A->P.r_goal;
    if (collided) r = r + A->P.r_col;
    rew = (float)r;
  }
  if (q == 0) {
    A->O.reward[ag] = rew;
    if (A->O.dist_goal) A->O.dist_goal[ag] = curr;
    if (A->O.info_flags)
      A->O.info_flags[ag] = (uint8_t)((act ? SWARM_AGENT_STEPPED : 0u) | (act && reached ? SWARM_AGENT_REACHED : 0u) |
                                      (act && collided ? SWARM_AGENT_COLLISION : 0u) | (cont ? SWARM_AGENT_HAS_OBS : 0u));
  }
  if (lane == 0)
    A->O.env_done[env] = (uint8_t)((term_all ? SWARM_ENV_TERMINATED : 0u) | (trunc_all ? SWARM_ENV_TRUNCATED : 0u) |
                                   (do_reset ? SWARM_ENV_RESET : 0u));
  const uint64_t m_term = __ballot(term), m_trunc = __ballot(trunc);

  // ---- the terminated / truncated / active rows: three dword rows built from ballots (a resetting
  // env's drones are all active again)
  {
    const uint64_t m_act = __ballot(do_reset || cont);
    // global-typed: made opaque, a plain pointer loses its address space and the row store becomes
    // a flat store, which every later `s_waitcnt lgkmcnt` would also wait for
    s64_gu8* p_term = (s64_gu8*)A->O.terminated;
    s64_gu8* p_trunc = (s64_gu8*)A->O.truncated;
    s64_gu8* p_act = (s64_gu8*)A->S.active;
    asm volatile("" : "+s"(p_term), "+s"(p_trunc), "+s"(p_act));
    const int grp = lane >> 2;  // lanes 0-3 terminated, 4-7 truncated, 8-11 active: dword lane & 3
    if (grp < 3) {
      const uint64_t m = grp == 0 ? m_term : (grp == 1 ? m_trunc : m_act);
      const uint32_t nib = (uint32_t)(m >> (16 * (lane & 3)));  // drones 4k .. 4k+3 at bits 0, 4, 8, 12
      const uint32_t word = (nib & 1u) | ((nib >> 4) & 1u) << 8 | ((nib >> 8) & 1u) << 16 | ((nib >> 12) & 1u) << 24;
      s64_gu8* base = grp == 0 ? p_term : (grp == 1 ? p_trunc : p_act);
      *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(base + ea + 4 * (lane & 3)) = word;
    }
  }

  // ---- state write-back of a continuing env (quarter 0), env scalars (lane 0); a resetting env's
  // new episode is wave 2's
  if (!do_reset) {
    if (q == 0) {
      float* pe = A->S.pos + ag * 3;
      float* ve = A->S.vel + ag * 3;
      pe[0] = px; pe[1] = py; pe[2] = pz;
      ve[0] = st.vx; ve[1] = st.vy; ve[2] = st.vz;
    }
    if (lane == 0) A->S.step_count[env] = new_step;
    if (A->O.global_state && q == 0) {
      float* gs = A->O.global_state + (size_t)env * (6 * Q_N + 3);
      gs[3 * d] = px; gs[3 * d + 1] = py; gs[3 * d + 2] = pz;
      gs[3 * Q_N + 3 * d] = st.vx; gs[3 * Q_N + 3 * d + 1] = st.vy; gs[3 * Q_N + 3 * d + 2] = st.vz;
      if (d == 0) { gs[6 * Q_N + 0] = st.gx; gs[6 * Q_N + 1] = st.gy; gs[6 * Q_N + 2] = st.gz; }
    }
  }
  Q16_FLAGS_END(env, lane);
}
}  // namespace
namespace swarm_dev {

#endif  // SWARM_HAS_PART(6)

// ------------------------------------------------------------------ step256: config 5 (N = 256)
// Specialisation of the step for one env of exactly 256 drones per 256-thread workgroup (wave w
// holds drones 64w .. 64w + 63, one per lane), kinematic dynamics + swarm reward, K = 3, Ms = 4,
// 4 <= M <= 16.  Observations, flags, state and global state equal
// swarm_kernel<0, 0, 4, 5, 0>'s bit for bit; rewards within the 1e-5 contract (formation partial
// sums in another order) — tests/test_gpu_step256.py.  The generic block team evaluates every
// pair twice (once per drone); here every pair is evaluated once and its value reaches the
// other drone by a lane rotation:
//  * block (w, w), the wave's own drones: step64's symmetric rotations r = 1 .. 32;
//  * block (w, w + 1): all 64 rotations; the mirror values belong to the next wave's drones;
//  * block (w, w + 2): half of it — rotations 0 .. 31 on waves 0 and 1, 1 .. 32 (the other half
//    seen from the far side) on waves 2 and 3.
// 128 rotations per wave instead of 255.  Mirror values travel: formation terms and minima as
// DPP wave rotations (a value added at rotation r has moved r lanes when the pass ends), keys by
// ds_bpermute; the ones that belong to another wave's drones are handed over through LDS after
// the pass.  Keys carry a partner code relative to the drone whose list holds them (block delta
// x 64 + lane offset, a compile-time constant per rotation), decoded to the drone index before
// the exact finish.  The keys' inserts are as many as before (each drone ranks 255 candidates);
// distances, square roots and formation terms halve.
constexpr int H_N = 256;
[[maybe_unused]] constexpr int H_K = 3;
[[maybe_unused]] constexpr int H_MS = 4;
constexpr int H_MMAX = 16;
constexpr int H_BL = 128;       // per-block plane segment: 64 drones + their wrap copy
constexpr int H_BATCH = H_BATCH_C;  // rotations per scheduling batch of the pair passes

struct H256Lds {
  // SoA planes per block: seg[b][plane][u], planes x, y, z, eligibility; drone 64b + u at u and
  // u + 64.  Lane t of a pass reads block b's rotation r at base + r with two bases (x / y and
  // z / eligibility), every plane within ds_read2_b32's 255-dword offset reach
  float seg[4][4][H_BL];
  float4 ring[H_N];                              // exact finish, obs rows, exact scans
  float4 obst[H_MMAX];
  float osoa[3 * H_MMAX];
  float4 goal;  // a new episode's goal (drawn by thread M)
  uint32_t red[4];  // per-wave vote bits of the reward phase
  union {
    struct {
      float sum[2][H_N];
      float mn[2][H_N];
    } p1;                      // formation sums / minima handed to another wave's drones
    uint32_t keys[2][4][H_N];  // neighbour key lists handed to another wave's drones
  } x;
};

// step256 on a 512-thread workgroup (SWARM_S256_WIDE): waves 0-3 (primary) and 4-7 (secondary)
// both hold drones 64b .. 64b + 63 of block b = wave & 3.  The primary evaluates blocks (b, b) and
// half of (b, b + 2), the secondary all of (b, b + 1): 64 rotations each instead of 128.  The
// secondary's own-side results come to the primary through LDS as the mirrors do.  Plane layout:
// per block and plane (x, y, z, eligibility) two copies of the 128-entry wrap segment, copy 0 at
// dword 0 and copy 1 shifted by one dword at H_C1 + 1 (H_C1 = 30 mod 64 apart: a ds_read_b64
// half-wave's two copies land on disjoint banks), so each lane reads aligned rotation pairs.
constexpr int H_C1 = 158;
constexpr int H_PS = 288;  // dwords per plane: copy 0 [0, 128), copy 1 [H_C1 + 1, H_C1 + 129)
static_assert(H_C1 % 64 == 30 && H_C1 % 2 == 0 && H_PS % 2 == 0 && H_C1 >= 2 * 64 && H_C1 + 1 + 2 * 64 <= H_PS,
              "two-copy plane layout: copy 1 even-based, 30 banks after copy 0, both copies inside the plane");
struct H256WLds {
  float seg2[4][4][H_PS];
  float4 ring[H_N];
  float4 obst[H_MMAX];
  float osoa[3 * H_MMAX];
  float4 goal;
  uint32_t red[4];
  union {
    struct {
      double dsum[H_N];          // the secondary's own formation sums
      float sum[3][H_N];         // mirror sums: [0] from block (b - 1, b), [1] from (b - 2, b), [2] the
                                 // primary's share of (b - 1, b) (SWARM_S256W_SPLIT1)
      float mn[4][H_N];          // mirror minima [0], [1]; the secondary's own minima [2]; [3] as sum[2]
    } p1;
    uint32_t keys[3][4][H_N];  // mirror lists [0] (b - 1, b), [1] (b - 2, b); the secondary's own [2]
  } x;
};

template <class LT>
__device__ __forceinline__ void h_put(LT& L, int w, int t, float x, float y, float z, float el) {
  L.seg[w][0][t] = x; L.seg[w][0][t + 64] = x;
  L.seg[w][1][t] = y; L.seg[w][1][t + 64] = y;
  L.seg[w][2][t] = z; L.seg[w][2][t + 64] = z;
  L.seg[w][3][t] = el; L.seg[w][3][t + 64] = el;
  L.ring[64 * w + t] = make_float4(x, y, z, el);
}

// Lane t's two read bases into block b's planes (x / y and z / eligibility) as opaque LDS
// addresses, so every rotation's read is an immediate offset of ds_read2_b32
template <int NP>
__device__ __forceinline__ void h_bases_p(float (*seg)[NP][H_BL], int b, int t, s64_lds_cf*& P0, s64_lds_cf*& P1) {
  P0 = (s64_lds_cf*)&seg[b][0][t];
  P1 = (s64_lds_cf*)&seg[b][2][t];
  asm volatile("" : "+v"(P0), "+v"(P1));
}
template <class LT>
__device__ __forceinline__ void h_bases(LT& L, int b, int t, s64_lds_cf*& P0, s64_lds_cf*& P1) {
  h_bases_p<4>(L.seg, b, t, P0, P1);
}
// Traveling minima are kept as float bits and reduced with v_min_u32 (every value is a
// non-negative float, whose bit patterns order like the floats): an integer min takes the
// rotated operand without the canonicalising v_max that v_min_f32 needs, so the DPP move folds
// into v_min_u32's DPP form (a full-wave rotation gives every lane a source: bound_ctrl changes
// nothing here)
__device__ __forceinline__ uint32_t wave_ror1_u(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x13C, 0xF, 0xF, true);
}

// Plane reads of the wide kernel's two-copy layout (H256WLds::seg2, PS dwords per plane): lane t's
// base addresses copy (t + PAR) & 1, in which the rotation pair (r - 1, r) of every r with
// r - 1 = PAR (mod 2) is 8-B aligned, so the pair is one ds_read_b64 (2 LDS cycles) instead of a
// ds_read2_b32 (4)
typedef const __attribute__((address_space(3))) s64_f2 s64_lds_cf2;
template <int PS>
__device__ __forceinline__ s64_f2 hw_ld2(s64_lds_cf* P, int plane, int r) {  // {X[r], X[r - 1]}
  const s64_f2 v = *(volatile s64_lds_cf2*)(P + plane * PS + r - 1);
  return v.yx;
}
template <int PS, int PAR>
__device__ __forceinline__ float hw_ld1(s64_lds_cf* P, int plane, int r) {  // X[r] from its aligned pair
  const int lo = (((r - 1) & 1) == PAR) ? r - 1 : r;
  const s64_f2 v = *(volatile s64_lds_cf2*)(P + plane * PS + lo);
  return lo == r ? v.x : v.y;
}

// Formation + minimum pass over rotations RHI, RHI - 1, .., RLO of one block (X/Y/Z/E = the
// block's plane segments at lane t).  Own side: formation partial sum `esum` (flushed into the
// f64 `fsum` every 8 rotations) and minimum `mn` of d~ = v_sqrt_f32(s') over eligible pairs.
// TRAVEL: the pair's value also enters the traveling sum / minimum (the partner's side).
// PS > 0: the two-copy layout (hw_ld2 / hw_ld1 from the base P0; P1 unused).
template <bool FAST, int RHI, int RLO, bool TRAVEL, int PS = 0, int PAR = 0>
__device__ __forceinline__ void h_seg1(s64_lds_cf* __restrict__ P0, s64_lds_cf* __restrict__ P1, bool self,
                                       float px, float py, float pz, float ds, double& fsum, float& mn, float& tsum,
                                       uint32_t& tmin) {
  s64_lds_cf* X = P0;
  s64_lds_cf* Y = P0 + H_BL;
  s64_lds_cf* Z = P1;
  s64_lds_cf* E = P1 + H_BL;
  static_assert(PS == 0 || RHI == RLO || ((RHI - 1) & 1) == PAR, "rotation pairs off the copy's alignment");
  float esum = 0.f;
  const float selff = self ? 1.f : 0.f;
#pragma unroll
  for (int r = RHI; r >= RLO; r -= 2) {
    const bool two = r - 1 >= RLO;
    float d[2];
    if (two) {
      s64_f2 XX, YY, ZZ;
      if constexpr (PS > 0) {
        XX = hw_ld2<PS>(P0, 0, r); YY = hw_ld2<PS>(P0, 1, r); ZZ = hw_ld2<PS>(P0, 2, r);
      } else {
        XX = s64_f2{X[r], X[r - 1]}; YY = s64_f2{Y[r], Y[r - 1]}; ZZ = s64_f2{Z[r], Z[r - 1]};
      }
      const s64_f2 dx = XX - px, dy = YY - py, dz = ZZ - pz;
      s64_f2 s = dx * dx;
      s = __builtin_elementwise_fma(dy, dy, s);
      s = __builtin_elementwise_fma(dz, dz, s);
      d[0] = __builtin_amdgcn_sqrtf(s.x);
      d[1] = __builtin_amdgcn_sqrtf(s.y);
    } else {
      if constexpr (PS > 0)
        d[0] = __builtin_amdgcn_sqrtf(sqsum_rank(hw_ld1<PS, PAR>(P0, 0, r) - px, hw_ld1<PS, PAR>(P0, 1, r) - py,
                                                 hw_ld1<PS, PAR>(P0, 2, r) - pz));
      else
        d[0] = __builtin_amdgcn_sqrtf(sqsum_rank(X[r] - px, Y[r] - py, Z[r] - pz));
      d[1] = 0.f;
    }
    float term[2];
    if (two) {
      const s64_f2 V = {d[0], d[1]};
      const s64_f2 Ed = V - ds;
      term[0] = fabsf(Ed.x);
      term[1] = fabsf(Ed.y);
    } else {
      term[0] = fabsf(d[0] - ds);
      term[1] = 0.f;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !two) break;
      const int rr = r - h;
      // masked pass: the pair's eligibility as a float factor (partner plane value 0 / 1 times
      // this drone's), so no per-rotation lane masks stay live; a masked pair's minimum value is
      // 3e38 (above every threshold) instead of inf
      float tv = term[h], dv = d[h];
      if constexpr (!FAST) {
        float er;
        if constexpr (PS > 0) er = hw_ld1<PS, PAR>(P0, 3, rr);
        else er = E[rr];
        const float ef = selff * er;
        tv = tv * ef;
        dv = fmaxf(dv, (1.f - ef) * 3e38f);
      }
      esum += tv;
      mn = fminf(mn, dv);
      if constexpr (TRAVEL) {
        tsum = wave_ror1(tsum) + tv;
        tmin = min(wave_ror1_u(tmin), __float_as_uint(dv));
      }
      if (((RHI - rr) & 7) == 7) {
        fsum += (double)esum;
        esum = 0.f;
      }
    }
    // batches of H_BATCH rotations: unbounded hoisting of the compile-time-offset LDS reads of a
    // whole segment costs registers (spills at 4 waves per SIMD)
    if (((RHI - r) % H_BATCH) == H_BATCH - 2) __builtin_amdgcn_sched_barrier(0);
  }
  fsum += (double)esum;
}

// Keys pass (s' keys) over rotations RHI .. RLO of one block: own keys into `nk` with partner
// code CO + r; MIRROR: the pair value goes by ds_bpermute to lane t + r, whose target list `mk`
// takes it with code CM + (64 - r) % 64 (lane offset back to this lane, block delta in CM).
template <int RHI, int RLO, int CO, int CM, bool MIRROR, int PS = 0, int PAR = 0>
__device__ __forceinline__ void h_seg0(s64_lds_cf* __restrict__ P0, s64_lds_cf* __restrict__ P1, uint32_t t4, float px,
                                       float py, float pz, uint32_t keep, uint32_t (&nk)[4], uint32_t (&mk)[4]) {
  s64_lds_cf* X = P0;
  s64_lds_cf* Y = P0 + H_BL;
  s64_lds_cf* Z = P1;
  // keep in a VGPR: (value & keep) | code is then one v_and_or_b32 with the code from an SGPR
  // (a VOP3 literal is not encodable on gfx9)
  static_assert(PS == 0 || RHI == RLO || ((RHI - 1) & 1) == PAR, "rotation pairs off the copy's alignment");
  uint32_t keepv = keep;
  asm volatile("" : "+v"(keepv));
#pragma unroll
  for (int r = RHI; r >= RLO; r -= 2) {
    const bool two = r - 1 >= RLO;
    float s[2];
    if (two) {
      s64_f2 XX, YY, ZZ;
      if constexpr (PS > 0) {
        XX = hw_ld2<PS>(P0, 0, r); YY = hw_ld2<PS>(P0, 1, r); ZZ = hw_ld2<PS>(P0, 2, r);
      } else {
        XX = s64_f2{X[r], X[r - 1]}; YY = s64_f2{Y[r], Y[r - 1]}; ZZ = s64_f2{Z[r], Z[r - 1]};
      }
      const s64_f2 dx = XX - px, dy = YY - py, dz = ZZ - pz;
      s64_f2 q = dx * dx;
      q = __builtin_elementwise_fma(dy, dy, q);
      q = __builtin_elementwise_fma(dz, dz, q);
      s[0] = q.x;
      s[1] = q.y;
    } else {
      if constexpr (PS > 0)
        s[0] = sqsum_rank(hw_ld1<PS, PAR>(P0, 0, r) - px, hw_ld1<PS, PAR>(P0, 1, r) - py, hw_ld1<PS, PAR>(P0, 2, r) - pz);
      else
        s[0] = sqsum_rank(X[r] - px, Y[r] - py, Z[r] - pz);
      s[1] = 0.f;
    }
    // the own key goes to the mirror as is; the mirror swaps its code CO + r for CM + (64 - r) % 64
    // with one full-rate v_xor_b32 (s' >= 0: the sign bit is clear on both sides)
    uint32_t key[2] = {0u, 0u}, rc[2] = {0u, 0u};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !two) break;
      key[h] = (__float_as_uint(s[h]) & keepv) | (uint32_t)(CO + r - h);
      if constexpr (MIRROR)
        rc[h] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(t4 + (uint32_t)(256 - 4 * (r - h))), (int)key[h]);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !two) break;
      const int rr = r - h;
      kins<4>(nk, key[h]);
      if constexpr (MIRROR) kins<4>(mk, rc[h] ^ ((uint32_t)(CO + rr) ^ (uint32_t)(CM + ((64 - rr) & 63))));
    }
    if (((RHI - r) % H_BATCH) == H_BATCH - 2) __builtin_amdgcn_sched_barrier(0);
  }
}

// The 4 smallest of two ascending 4-key lists (bitonic, as quad_merge4)
__device__ __forceinline__ void h_merge4(uint32_t (&k)[4], const uint32_t (&b)[4]) {
  uint32_t c[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = min(k[i], b[3 - i]);
  const uint32_t c0 = min(c[0], c[2]), c2 = max(c[0], c[2]);
  const uint32_t c1 = min(c[1], c[3]), c3 = max(c[1], c[3]);
  k[0] = min(c0, c1); k[1] = max(c0, c1);
  k[2] = min(c2, c3); k[3] = max(c2, c3);
}

// seg: the [block][x, y, z, eligibility][H_BL] planes; psum / pmn: the two handed-over sets
template <bool FAST>
__device__ __forceinline__ void h_pass1(float (*seg)[4][H_BL], float (*psum)[H_N], float (*pmn)[H_N], int w, int t,
                                        bool self, float px, float py, float pz, float ds, double& fsum, float& smin) {
  const int b1 = (w + 1) & 3, b2 = (w + 2) & 3;
  s64_lds_cf *A0, *A1, *B0, *B1, *C0, *C1;
  h_bases_p(seg, w, t, A0, A1);
  h_bases_p(seg, b1, t, B0, B1);
  h_bases_p(seg, b2, t, C0, C1);
  float ta = 0.f, dummy = 0.f;
  uint32_t tam = 0x7f800000u, dummym = 0x7f800000u;
  // own block: rotations 31 .. 1 with the traveling mirror, then 32 from both sides
  h_seg1<FAST, 31, 1, true>(A0, A1, self, px, py, pz, ds, fsum, smin, ta, tam);
  fsum += (double)wave_ror1(ta);
  smin = fminf(smin, __uint_as_float(wave_ror1_u(tam)));
  h_seg1<FAST, 32, 32, false>(A0, A1, self, px, py, pz, ds, fsum, smin, dummy, dummym);
  // block (w, w + 1): rotations 63 .. 0, mirror for wave w + 1's drones
  float tb = 0.f;
  uint32_t tbm = 0x7f800000u;
  h_seg1<FAST, 63, 0, true>(B0, B1, self, px, py, pz, ds, fsum, smin, tb, tbm);
  // block (w, w + 2): half, mirror for wave w + 2's drones
  float tc = 0.f;
  uint32_t tcm = 0x7f800000u;
  if (w < 2) {
    h_seg1<FAST, 31, 0, true>(C0, C1, self, px, py, pz, ds, fsum, smin, tc, tcm);
  } else {
    h_seg1<FAST, 32, 1, true>(C0, C1, self, px, py, pz, ds, fsum, smin, tc, tcm);
    tc = wave_ror1(tc);
    tcm = wave_ror1_u(tcm);
  }
  psum[0][64 * b1 + t] = tb;
  pmn[0][64 * b1 + t] = __uint_as_float(tbm);
  psum[1][64 * b2 + t] = tc;
  pmn[1][64 * b2 + t] = __uint_as_float(tcm);
}

__device__ __forceinline__ void h_pass0(H256Lds& L, int w, int t, float px, float py, float pz, uint32_t keep,
                                        uint32_t (&nk)[4]) {
  const int b1 = (w + 1) & 3, b2 = (w + 2) & 3;
  const uint32_t t4 = (uint32_t)t << 2;
  uint32_t kb[4], kc[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) { kb[s] = KEY_EMPTY; kc[s] = KEY_EMPTY; }
  // own block: codes r (own) and 64 - r (mirror, same block); rotation 32 from both sides
  s64_lds_cf *A0, *A1, *B0, *B1, *C0, *C1;
  h_bases(L, w, t, A0, A1);
  h_bases(L, b1, t, B0, B1);
  h_bases(L, b2, t, C0, C1);
  h_seg0<31, 1, 0, 0, true>(A0, A1, t4, px, py, pz, keep, nk, nk);
  h_seg0<32, 32, 0, 0, false>(A0, A1, t4, px, py, pz, keep, nk, nk);
  // block (w, w + 1): own code 64 + r (block delta 1); mirror code 192 + (64 - r) % 64 (delta -1)
  h_seg0<63, 0, 64, 192, true>(B0, B1, t4, px, py, pz, keep, nk, kb);
  // block (w, w + 2): own code 128 + r, mirror code 128 + (64 - r) % 64 (delta +-2)
  if (w < 2)
    h_seg0<31, 0, 128, 128, true>(C0, C1, t4, px, py, pz, keep, nk, kc);
  else
    h_seg0<32, 1, 128, 128, true>(C0, C1, t4, px, py, pz, keep, nk, kc);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    L.x.keys[0][s][64 * b1 + t] = kb[s];
    L.x.keys[1][s][64 * b2 + t] = kc[s];
  }
}

__device__ __forceinline__ void hw_put(H256WLds& L, int w, int t, float x, float y, float z, float el) {
  const float v[4] = {x, y, z, el};
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    L.seg2[w][p][t] = v[p]; L.seg2[w][p][t + 64] = v[p];
    L.seg2[w][p][H_C1 + 1 + t] = v[p]; L.seg2[w][p][H_C1 + 65 + t] = v[p];
  }
  L.ring[64 * w + t] = make_float4(x, y, z, el);
}
// Lane t's base into block b's planes for rotation pairs (r - 1, r) with r - 1 = PAR (mod 2)
template <int PAR>
__device__ __forceinline__ s64_lds_cf* hw_base(H256WLds& L, int b, int t) {
  const int c = (t + PAR) & 1;
  s64_lds_cf* P = (s64_lds_cf*)&L.seg2[b][0][(c ? H_C1 + 1 : 0) + t];
  asm volatile("" : "+v"(P));
  return P;
}

// The wide kernel's halves of h_pass1 / h_pass0.  Primary: block (w, w) and half of (w, w + 2);
// secondary: block (w, w + 1), its own side into fsum / smin / nk, the mirror into set [0].
// SWARM_S256W_SPLIT1 = S > 0: the formation pass's rotations S - 1 .. 0 of block (w, w + 1) move to
// the primary (mirror set [2] / [3]); the secondary's travelled values, which stop at rotation S,
// are rotated the remaining S lanes by one ds_bpermute each.
#ifndef SWARM_S256W_SPLIT1
#define SWARM_S256W_SPLIT1 16  // r06d / r06e: 36.07 / 35.81 / 36.03, 36.22 / 35.92 / 36.12 vs 35.97 / 36.41 / 36.37,
                               // 36.40 / 36.28 / 36.10 us (5 of 6 pairs); the primary's hand-over wait 4.9k -> 2.0k cycles
#endif
static_assert(SWARM_S256W_SPLIT1 % 2 == 0 && SWARM_S256W_SPLIT1 < 64, "split on the two-copy rotation pairs");
template <bool FAST, bool PRIMARY>
__device__ __forceinline__ void hw_pass1(H256WLds& L, int w, int t, bool self, float px, float py, float pz, float ds,
                                         double& fsum, float& smin) {
  const int b1 = (w + 1) & 3, b2 = (w + 2) & 3;
  s64_lds_cf* const none = nullptr;
  if constexpr (PRIMARY) {
    s64_lds_cf* P0 = hw_base<0>(L, w, t);
    float ta = 0.f, dummy = 0.f;
    uint32_t tam = 0x7f800000u, dummym = 0x7f800000u;
    h_seg1<FAST, 31, 1, true, H_PS, 0>(P0, none, self, px, py, pz, ds, fsum, smin, ta, tam);
    fsum += (double)wave_ror1(ta);
    smin = fminf(smin, __uint_as_float(wave_ror1_u(tam)));
    h_seg1<FAST, 32, 32, false, H_PS, 0>(P0, none, self, px, py, pz, ds, fsum, smin, dummy, dummym);
    float tc = 0.f;
    uint32_t tcm = 0x7f800000u;
    if (w < 2) {
      h_seg1<FAST, 31, 0, true, H_PS, 0>(hw_base<0>(L, b2, t), none, self, px, py, pz, ds, fsum, smin, tc, tcm);
    } else {
      h_seg1<FAST, 32, 1, true, H_PS, 1>(hw_base<1>(L, b2, t), none, self, px, py, pz, ds, fsum, smin, tc, tcm);
      tc = wave_ror1(tc);
      tcm = wave_ror1_u(tcm);
    }
    L.x.p1.sum[1][64 * b2 + t] = tc;
    L.x.p1.mn[1][64 * b2 + t] = __uint_as_float(tcm);
    if constexpr (SWARM_S256W_SPLIT1 > 0) {
      float tb = 0.f;
      uint32_t tbm = 0x7f800000u;
      h_seg1<FAST, SWARM_S256W_SPLIT1 - 1, 0, true, H_PS, 0>(hw_base<0>(L, b1, t), none, self, px, py, pz, ds, fsum,
                                                              smin, tb, tbm);
      L.x.p1.sum[2][64 * b1 + t] = tb;
      L.x.p1.mn[3][64 * b1 + t] = __uint_as_float(tbm);
    }
  } else {
    float tb = 0.f;
    uint32_t tbm = 0x7f800000u;
    h_seg1<FAST, 63, SWARM_S256W_SPLIT1, true, H_PS, 0>(hw_base<0>(L, b1, t), none, self, px, py, pz, ds, fsum, smin,
                                                         tb, tbm);
    if constexpr (SWARM_S256W_SPLIT1 > 0) {  // the travelled values' last S lanes
      const int src = (int)((((uint32_t)t - SWARM_S256W_SPLIT1) & 63u) << 2);
      tb = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(tb)));
      tbm = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)tbm);
    }
    L.x.p1.sum[0][64 * b1 + t] = tb;
    L.x.p1.mn[0][64 * b1 + t] = __uint_as_float(tbm);
    L.x.p1.dsum[64 * w + t] = fsum;
    L.x.p1.mn[2][64 * w + t] = smin;
  }
}

template <bool PRIMARY>
__device__ __forceinline__ void hw_pass0(H256WLds& L, int w, int t, float px, float py, float pz, uint32_t keep,
                                         uint32_t (&nk)[4]) {
  const int b1 = (w + 1) & 3, b2 = (w + 2) & 3;
  const uint32_t t4 = (uint32_t)t << 2;
  uint32_t km[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) km[s] = KEY_EMPTY;
  s64_lds_cf* const none = nullptr;
  if constexpr (PRIMARY) {
    s64_lds_cf* P0 = hw_base<0>(L, w, t);
    h_seg0<31, 1, 0, 0, true, H_PS, 0>(P0, none, t4, px, py, pz, keep, nk, nk);
    h_seg0<32, 32, 0, 0, false, H_PS, 0>(P0, none, t4, px, py, pz, keep, nk, nk);
    if (w < 2)
      h_seg0<31, 0, 128, 128, true, H_PS, 0>(hw_base<0>(L, b2, t), none, t4, px, py, pz, keep, nk, km);
    else
      h_seg0<32, 1, 128, 128, true, H_PS, 1>(hw_base<1>(L, b2, t), none, t4, px, py, pz, keep, nk, km);
#pragma unroll
    for (int s = 0; s < 4; ++s) L.x.keys[1][s][64 * b2 + t] = km[s];
  } else {
    h_seg0<63, 0, 64, 192, true, H_PS, 0>(hw_base<0>(L, b1, t), none, t4, px, py, pz, keep, nk, km);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      L.x.keys[0][s][64 * b1 + t] = km[s];
      L.x.keys[2][s][64 * w + t] = nk[s];
    }
  }
}

// partner code -> drone index, for the drone (w, t) whose list holds the key
__device__ __forceinline__ uint32_t h_decode(uint32_t key, int w, int t, uint32_t keep) {
  if (key == KEY_EMPTY) return key;
  const uint32_t c = key & ~keep;
  const uint32_t j = ((((uint32_t)w + (c >> 6)) & 3u) << 6) | (((uint32_t)t + c) & 63u);
  return (key & keep) | j;
}

// step64's straight-line finish (s64_finish_fast) with drone indices in the neighbour keys
__device__ __forceinline__ uint32_t h_finish_fast(const uint32_t (&nk)[4], const uint32_t (&ok)[5],
                                                  const float4* __restrict__ ring, const float4* __restrict__ obst,
                                                  int M, uint32_t nb_keep, uint32_t ob_keep, float px, float py,
                                                  float pz, float (&wd)[4], int (&wj)[4], float (&od)[5],
                                                  int (&oj)[5]) {
  constexpr int K = 3, MS = 4;
  const uint32_t nim = ~nb_keep, oim = ~ob_keep;
  bool near_nb = false, near_ob = false;
#pragma unroll
  for (int s = 0; s + 1 < 4; ++s)
    near_nb = near_nb | (__uint_as_float(nk[s + 1] & nb_keep) <= __uint_as_float((nk[s] & nb_keep) | nim) * FAST_HI);
#pragma unroll
  for (int s = 0; s + 1 < 5; ++s)
    near_ob = near_ob | ((ok[s + 1] != KEY_EMPTY) &
                         (__uint_as_float(ok[s + 1] & ob_keep) <= __uint_as_float((ok[s] & ob_keep) | oim) * FAST_HI));
#pragma unroll
  for (int s = 0; s < K; ++s) {
    const int j = (int)(nk[s] & nim) & (H_N - 1);
    const float4 q = lds_f4(ring + j);
    wd[s] = sqrt_rn(sqsum_1d(q.x - px, q.y - py, q.z - pz));
    wj[s] = j;
  }
  wd[K] = __builtin_inff();
  wj[K] = 0x7fffffff;
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    const int j = (int)(ok[s] & oim);
    const float4 q = lds_f4(obst + (j & (H_MMAX - 1)));
    od[s] = sqrt_rn(sqsum_f(q.x - px, q.y - py, q.z - pz));
    oj[s] = j;
  }
  od[MS] = __builtin_inff();
  oj[MS] = 0x7fffffff;
  // survivor bounds (finish_keys' tails: s' neighbour keys, exact obstacle keys)
  const float nb_base = __uint_as_float(nk[K] & nb_keep) * FAST_LO;
  const float wv = wd[K - 1];
  const bool ok_nb = nb_base > (wv * wv) * FAST_HI;
  const uint32_t last = ok[MS];
  const float wo = od[MS - 1];
  const bool ok_ob = last == KEY_EMPTY || (int)(last & oim) >= M ||
                     __uint_as_float(last & ob_keep) > (wo * wo) * FAST_HI;
  return (near_nb ? S64F_NEAR_NB : 0u) | (near_ob ? S64F_NEAR_OB : 0u) | (ok_nb ? 0u : S64F_BOUND_NB) |
         (ok_ob ? 0u : S64F_BOUND_OB);
}

// Phase stamps of step256 (diagnostic stamps build, tools/stamps.py with SWARM_STAMPS_KERNEL=n256):
// wave 0's view of each phase boundary, one record per env
#define STAMP256(i) STAMP_AT(threadIdx.x == 0 ? env : (1 << 16), i)

#if SWARM_HAS_PART(7)  // emitted in its own translation unit only
}  // namespace swarm_dev
namespace {  // kernels: internal to this translation unit
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) swarm_step256(S64_ONCE_PARAMS) {
  // (the leading arguments of the wide kernel's launch, unused here: everything from the args block)
  (void)pos; (void)vel; (void)actions; (void)active; (void)goal; (void)amask; (void)E;  // M: the launch's obstacle count
  (void)args;  // read through s64_args<S64_HOT_BYTES>()
  constexpr int KS = H_K + 1, MSL = H_MS + 1;
  __shared__ H256Lds L;
  const int i = threadIdx.x;  // drone
  const int w = __builtin_amdgcn_readfirstlane(i >> 6), t = i & 63;
  S64ArgPtr A = s64_args<S64_HOT_BYTES>();
  const int env = blockIdx.x;
  if (env >= A->P.E) return;  // whole block
  const size_t ag = (size_t)env * H_N + i;
  STAMP256(0);
  STAMP_BEGIN(env, i == 0);

  // ---- loads
  const float gx0 = A->S.goal[3 * env], gy0 = A->S.goal[3 * env + 1], gz0 = A->S.goal[3 * env + 2];
  const int stepc = A->S.step_count[env];
  const uint32_t episode0 = A->S.episode[env];
  float ax = A->actions[ag * 3], ay = A->actions[ag * 3 + 1], az = A->actions[ag * 3 + 2];
  float px = A->S.pos[ag * 3], py = A->S.pos[ag * 3 + 1], pz = A->S.pos[ag * 3 + 2];
  float vx = A->S.vel[ag * 3], vy = A->S.vel[ag * 3 + 1], vz = A->S.vel[ag * 3 + 2];
  bool act = A->S.active[ag] != 0;
  const bool has = A->amask == nullptr || A->amask[ag] != 0;
  if (i < M) {
    const float* o = A->S.obstacles + ((size_t)env * M + i) * 3;
    const float ox = o[0], oy = o[1], oz = o[2];
    L.obst[i] = make_float4(ox, oy, oz, 0.f);
    L.osoa[i] = ox; L.osoa[H_MMAX + i] = oy; L.osoa[2 * H_MMAX + i] = oz;
  }
  float gx = gx0, gy = gy0, gz = gz0;
  const int n_active = __syncthreads_count(act);
  STAMP256(1);
  A = s64_args<S64_HOT_BYTES>();

  // ---- integrate: drone_swarm_env.py:98-117 (swarm_kernel, DYN_KIN)
  float prev_d = 0.f;
  if (act) {
    prev_d = sqrt_rn(sqsum_1d(gx - px, gy - py, gz - pz));
    if (!has) { ax = 0.f; ay = 0.f; az = 0.f; }
    ax = clampf(ax, -1.f, 1.f) * A->P.amax;
    ay = clampf(ay, -1.f, 1.f) * A->P.amax;
    az = clampf(az, -1.f, 1.f) * A->P.amax;
    vx = vx + ax * A->P.dt;
    vy = vy + ay * A->P.dt;
    vz = vz + az * A->P.dt;
    const float s_sp = sqsum_1d(vx, vy, vz);
    if (!(s_sp <= A->P.s_vmax)) {
      const float sp = sqrt_rn(s_sp);
      if (!(sp <= A->P.vmax || sp < (float)1e-8)) {
        vx = (vx / sp) * A->P.vmax;
        vy = (vy / sp) * A->P.vmax;
        vz = (vz / sp) * A->P.vmax;
      }
    }
    px = px + vx * A->P.dt;
    py = py + vy * A->P.dt;
    pz = pz + vz * A->P.dt;
  }
  if (n_active > 0) {
    px = clampf(px, A->P.neg_half_w, A->P.half_w);
    py = clampf(py, A->P.neg_half_w, A->P.half_w);
    pz = clampf(pz, A->P.neg_half_w, A->P.half_w);
  }
  h_put(L, w, t, px, py, pz, act ? 1.f : 0.f);
  const bool fast = __syncthreads_and(act) != 0;  // also the barrier after the puts
  STAMP256(2);
  A = s64_args<S64_HOT_BYTES>();

  // ---- formation + minimum pass (every pair once), obstacle pass
  double fsum = 0.0;
  float smin = __builtin_inff();
  if (fast) h_pass1<true>(L.seg, L.x.p1.sum, L.x.p1.mn, w, t, true, px, py, pz, A->P.ds_f, fsum, smin);
  else h_pass1<false>(L.seg, L.x.p1.sum, L.x.p1.mn, w, t, act, px, py, pz, A->P.ds_f, fsum, smin);
  uint32_t ok[MSL];
#pragma unroll
  for (int s = 0; s < MSL; ++s) ok[s] = KEY_EMPTY;
  bool ocoll = false;
  obstacle_pass_s64<MSL, true>(L.osoa, M, px, py, pz, act, A->P.s_obst, A->P.ob_keep, ok, ocoll);
  STAMP256(3);
  __syncthreads();  // handed-over sums / minima written
  fsum += (double)L.x.p1.sum[0][i];
  fsum += (double)L.x.p1.sum[1][i];
  smin = fminf(smin, fminf(L.x.p1.mn[0][i], L.x.p1.mn[1][i]));
  A = s64_args<S64_HOT_BYTES>();

  STAMP256(4);
  // ---- rewards / terminations: drone_swarm_env.py:120-172 (swarm_kernel, DYN_KIN)
  bool pcoll = smin <= A->P.thr_pair * FAST_LO;
  if (!pcoll && smin <= A->P.thr_pair * FAST_HI && act)
    pcoll = exact_pair_collision(L.ring, H_N, i, px, py, pz, A->P.s_pair);
  const float curr = sqrt_rn(sqsum_1d(gx - px, gy - py, gz - pz));
  float rew = 0.f;
  bool reached = false, collided = false, term = false, trunc = false, cont = false;
  bool term_all = false, trunc_all = false;
  int new_step = stepc;
  bool p_coll = false, p_cand = false;
  if (act) {
    reached = (double)curr <= A->P.goal_radius;
    collided = ocoll || pcoll;
    p_coll = collided;
    p_cand = !reached && !collided;
    double r = ((double)prev_d - (double)curr) * A->P.kp;
    if (n_active > 1) r = r + (-A->P.kf) * (fsum * inv_count(n_active - 1));
    if (reached) r = r + A->P.r_goal;
    if (collided) r = r + A->P.r_col;
    rew = (float)r;
  }
  // both block votes through one barrier: wave ballots -> one word per wave
  {
    const bool wc = __ballot(p_coll) != 0, wd = __ballot(p_cand) != 0;
    if (t == 0) L.red[w] = (wc ? 1u : 0u) | (wd ? 2u : 0u);
  }
  __syncthreads();
  const uint32_t votes = L.red[0] | L.red[1] | L.red[2] | L.red[3];
  const bool any_c = (votes & 1u) != 0, any_cand = (votes & 2u) != 0;
  A = s64_args<S64_HOT_BYTES>();
  if (n_active == 0) {
    term_all = true;
  } else {
    new_step = stepc + 1;
    const bool tl = new_step >= A->P.max_steps;
    term_all = (!any_cand && !any_c && !tl) || any_c;
    trunc_all = tl && !term_all;
    if (act) {
      const bool done_i = reached || collided;
      term = done_i;
      trunc = tl && !done_i;
      cont = !done_i && !tl && !any_c;
    }
  }
  const bool do_reset = A->P.auto_reset && (term_all || trunc_all);
  A->O.reward[ag] = rew;
  A->O.terminated[ag] = term ? 1 : 0;
  A->O.truncated[ag] = trunc ? 1 : 0;
  if (A->O.dist_goal) A->O.dist_goal[ag] = curr;
  if (A->O.info_flags)
    A->O.info_flags[ag] = (uint8_t)((act ? SWARM_AGENT_STEPPED : 0u) | (act && reached ? SWARM_AGENT_REACHED : 0u) |
                                    (act && collided ? SWARM_AGENT_COLLISION : 0u) | (cont ? SWARM_AGENT_HAS_OBS : 0u));
  if (i == 0)
    A->O.env_done[env] = (uint8_t)((term_all ? SWARM_ENV_TERMINATED : 0u) | (trunc_all ? SWARM_ENV_TRUNCATED : 0u) |
                                   (do_reset ? SWARM_ENV_RESET : 0u));

  STAMP256(5);
  // ---- in-kernel auto-reset (block-uniform): the new episode, then its keys
  uint32_t episode_new = episode0;
  if (do_reset) {
    episode_new = episode0 + 1u;
    const long long genv = A->P.env_offset + env;
    uint32_t wd4[4], wo[4];
    draw_block_k(A->P.seed_lo, A->P.seed_hi, genv, episode_new, (uint32_t)i, wd4);
    const bool drawer = i <= M;  // obstacle i (i < M) or the goal (i == M)
    if (drawer) draw_block_k(A->P.seed_lo, A->P.seed_hi, genv, episode_new, (uint32_t)(H_N + i), wo);
    const float lo_w = A->P.neg_half_w, wd_w = A->P.width_w;
    px = uni(wd4[0], lo_w, wd_w);
    py = uni(wd4[1], lo_w, wd_w);
    pz = uni(wd4[2], lo_w, wd_w);
    vx = vy = vz = 0.f;
    act = true;
    __syncthreads();  // every read of the old planes / ring / obstacles is done
    if (drawer) {
      const float ox = uni(wo[0], lo_w, wd_w), oy = uni(wo[1], lo_w, wd_w), oz = uni(wo[2], lo_w, wd_w);
      if (i < M) {
        L.obst[i] = make_float4(ox, oy, oz, 0.f);
        L.osoa[i] = ox; L.osoa[H_MMAX + i] = oy; L.osoa[2 * H_MMAX + i] = oz;
      } else {
        L.goal = make_float4(ox, oy, oz, 0.f);
      }
    }
    h_put(L, w, t, px, py, pz, 1.f);
    __syncthreads();
    const float4 g4 = L.goal;
    gx = g4.x; gy = g4.y; gz = g4.z;
#pragma unroll
    for (int s = 0; s < MSL; ++s) ok[s] = KEY_EMPTY;
    bool c2 = false;
    obstacle_pass_s64<MSL, false>(L.osoa, M, px, py, pz, false, 0.f, A->P.ob_keep, ok, c2);
  }
  STAMP256(6);
  A = s64_args<S64_HOT_BYTES>();
  uint32_t nk[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) nk[s] = KEY_EMPTY;
  h_pass0(L, w, t, px, py, pz, A->P.nb_keep, nk);
  __syncthreads();  // handed-over key lists written
  {
    uint32_t kb[4], kc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) { kb[s] = L.x.keys[0][s][i]; kc[s] = L.x.keys[1][s][i]; }
    h_merge4(nk, kb);
    h_merge4(nk, kc);
#pragma unroll
    for (int s = 0; s < KS; ++s) nk[s] = h_decode(nk[s], w, t, A->P.nb_keep);
  }
  A = s64_args<S64_HOT_BYTES>();

  // ---- exact top-K of the emitted observation (keys rank by s', drone indices)
  float wd[KS], od[MSL];
  int wj[KS], oj[MSL];
  {
    const uint32_t ff = h_finish_fast(nk, ok, L.ring, L.obst, M, A->P.nb_keep, A->P.ob_keep, px, py, pz, wd, wj, od, oj);
    if (__ballot(ff != 0) != 0) {  // straight-line rest of finish_keys (s64_finish_general), then the scans
      bool slow_nb, slow_ob;
      s64_finish_general<KS, MSL, H_N, false, H_MMAX>(ff, nk, ok, L.ring, L.obst, i, M, A->P.nb_keep, A->P.ob_keep,
                                                      false, px, py, pz, wd, wj, od, oj, slow_nb, slow_ob);
      if (slow_nb) exact_select<KS, false>(L.ring, H_N, i, H_K, max_first(wd, H_K), px, py, pz, wd, wj);
      if (slow_ob) exact_select<MSL, true>(L.obst, M, -1, H_MS, max_first(od, H_MS), px, py, pz, od, oj);
    }
  }
  STAMP256(7);
  A = s64_args<S64_HOT_BYTES>();

  // ---- state write-back
  const bool new_act = do_reset || cont;
  A->S.pos[ag * 3] = px; A->S.pos[ag * 3 + 1] = py; A->S.pos[ag * 3 + 2] = pz;
  A->S.vel[ag * 3] = vx; A->S.vel[ag * 3 + 1] = vy; A->S.vel[ag * 3 + 2] = vz;
  A->S.active[ag] = new_act ? 1 : 0;
  if (i == 0) {
    A->S.step_count[env] = do_reset ? 0 : new_step;
    if (do_reset) {
      A->S.episode[env] = episode_new;
      A->S.goal[3 * env] = gx; A->S.goal[3 * env + 1] = gy; A->S.goal[3 * env + 2] = gz;
    }
  }
  if (do_reset && i < M) {
    float* o = A->S.obstacles + ((size_t)env * M + i) * 3;
    const float4 q = L.obst[i];
    o[0] = q.x; o[1] = q.y; o[2] = q.z;
  }
  if (A->O.global_state) {
    float* gs = A->O.global_state + (size_t)env * (6 * H_N + 3);
    gs[3 * i] = px; gs[3 * i + 1] = py; gs[3 * i + 2] = pz;
    gs[3 * H_N + 3 * i] = vx; gs[3 * H_N + 3 * i + 1] = vy; gs[3 * H_N + 3 * i + 2] = vz;
    if (i == 0) { gs[6 * H_N] = gx; gs[6 * H_N + 1] = gy; gs[6 * H_N + 2] = gz; }
  }
  A = s64_args<S64_HOT_BYTES>();

  // ---- observation row [p | v | g-p | K x (p_j-p, d) | Ms x (o_m-p, d)], straight from registers
  float* row = A->O.obs + ag * (9 + 4 * H_K + 4 * H_MS);
  row[0] = px; row[1] = py; row[2] = pz;
  row[3] = vx; row[4] = vy; row[5] = vz;
  row[6] = gx - px; row[7] = gy - py; row[8] = gz - pz;
#pragma unroll
  for (int s = 0; s < H_K; ++s) {
    const float4 q = lds_f4(L.ring + (wj[s] & (H_N - 1)));
    row[9 + 4 * s] = q.x - px; row[10 + 4 * s] = q.y - py; row[11 + 4 * s] = q.z - pz; row[12 + 4 * s] = wd[s];
  }
#pragma unroll
  for (int s = 0; s < H_MS; ++s) {
    const float4 q = lds_f4(L.obst + (oj[s] & (H_MMAX - 1)));
    row[21 + 4 * s] = q.x - px; row[22 + 4 * s] = q.y - py; row[23 + 4 * s] = q.z - pz; row[24 + 4 * s] = od[s];
  }
  STAMP256(8);
  STAMP_END(env, i == 0);
}

// The same step on 512 threads (H256WLds): the primary wave of block b runs every phase of
// swarm_step256 for drones 64b .. 64b + 63 except block (b, b + 1) of both pair passes, which
// its secondary wave (b + 4) evaluates at the same time; the secondary also loads, draws and
// writes the obstacles and draws the goal.  Results as swarm_step256's (formation sums in
// another order: rewards within 1e-5).
#ifndef SWARM_S256W_WAVES
#define SWARM_S256W_WAVES 6  // 80 VGPRs: three 512-thread workgroups per CU
#endif
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(SWARM_S256W_WAVES)))
swarm_step256w(S64_ONCE_PARAMS) {
  (void)args;  // read through s64_args<S64_HOT_BYTES>()
  // the leading arguments (preloaded into SGPRs, -amdgpu-kernarg-preload-count=16 for this unit):
  // the bound test and the primary's first loads issue without a scalar load of the kernarg segment
  const S64Hot H = S64_ONCE_HOT;
  constexpr int KS = H_K + 1, MSL = H_MS + 1;
  __shared__ H256WLds L;
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const bool primary = wv < 4;
  const int w = wv & 3, t = threadIdx.x & 63;
  const int i = 64 * w + t;  // drone
  const int env = xcd_slot((int)blockIdx.x, (int)gridDim.x);
  if (env >= H.E) return;  // whole block
  const size_t ag = (size_t)env * H_N + i;
  STAMP256(0);
  STAMP_BEGIN(env, threadIdx.x == 0);

  // ---- loads (the secondary: obstacles); 32-bit element offsets (step256_applies: E x 256 x 3 < 2^32)
  float gx = 0.f, gy = 0.f, gz = 0.f, ax = 0.f, ay = 0.f, az = 0.f;
  float px = 0.f, py = 0.f, pz = 0.f, vx = 0.f, vy = 0.f, vz = 0.f;
  bool act = false, has = true;
  if (primary) {
    // wave-uniform row bases (SGPRs) + 32-bit lane offsets: saddr-form loads, no 64-bit lane math
    const uint32_t wb = (uint32_t)env * H_N + 64u * (uint32_t)w, t3 = 3u * (uint32_t)t, g3 = 3u * (uint32_t)env;
    const float* __restrict__ pe = H.pos + 3u * wb;
    const float* __restrict__ ve = H.vel + 3u * wb;
    const float* __restrict__ ae = H.actions + 3u * wb;
    gx = __uint_as_float(H.goal[g3]); gy = __uint_as_float(H.goal[g3 + 1]); gz = __uint_as_float(H.goal[g3 + 2]);
    ax = ae[t3]; ay = ae[t3 + 1]; az = ae[t3 + 2];
    px = pe[t3]; py = pe[t3 + 1]; pz = pe[t3 + 2];
    vx = ve[t3]; vy = ve[t3 + 1]; vz = ve[t3 + 2];
    act = (H.active + wb)[t] != 0;
    has = H.amask == nullptr || (H.amask + wb)[t] != 0;
  }
  S64ArgPtr A = s64_args<S64_HOT_BYTES>();
  const int stepc = A->S.step_count[env];
  const uint32_t episode0 = A->S.episode[env];
  if (!primary && i < M) {
    const float* o = A->S.obstacles + ((size_t)env * M + i) * 3;
    const float ox = o[0], oy = o[1], oz = o[2];
    L.obst[i] = make_float4(ox, oy, oz, 0.f);
    L.osoa[i] = ox; L.osoa[H_MMAX + i] = oy; L.osoa[2 * H_MMAX + i] = oz;
  }
  const int n_active = __syncthreads_count(act);
  STAMP256(1);
  A = s64_args<S64_HOT_BYTES>();
  // SWARM_S256W_PRIO: issue priority of the secondary over the (older) primary that shares its
  // SIMD: 1 = during the formation pass, 2 = from here on (the oldest wave issues first otherwise)
#ifndef SWARM_S256W_PRIO
#define SWARM_S256W_PRIO 0
#endif
  if (SWARM_S256W_PRIO == 2 && !primary) __builtin_amdgcn_s_setprio(1);

  // ---- integrate: drone_swarm_env.py:98-117 (swarm_kernel, DYN_KIN)
  float prev_d = 0.f;
  if (primary) {
    if (act) {
      prev_d = sqrt_rn(sqsum_1d(gx - px, gy - py, gz - pz));
      zero_unless(has, ax, ay, az);
      ax = clampf(ax, -1.f, 1.f) * A->P.amax;
      ay = clampf(ay, -1.f, 1.f) * A->P.amax;
      az = clampf(az, -1.f, 1.f) * A->P.amax;
      vx = vx + ax * A->P.dt;
      vy = vy + ay * A->P.dt;
      vz = vz + az * A->P.dt;
      const float s_sp = sqsum_1d(vx, vy, vz);
      if (!(s_sp <= A->P.s_vmax)) {
        const float sp = sqrt_rn(s_sp);
        if (!(sp <= A->P.vmax || sp < (float)1e-8)) {
          vx = (vx / sp) * A->P.vmax;
          vy = (vy / sp) * A->P.vmax;
          vz = (vz / sp) * A->P.vmax;
        }
      }
      px = px + vx * A->P.dt;
      py = py + vy * A->P.dt;
      pz = pz + vz * A->P.dt;
    }
    if (n_active > 0) {
      px = clampf(px, A->P.neg_half_w, A->P.half_w);
      py = clampf(py, A->P.neg_half_w, A->P.half_w);
      pz = clampf(pz, A->P.neg_half_w, A->P.half_w);
    }
    hw_put(L, w, t, px, py, pz, act ? 1.f : 0.f);
  }
  const bool fast = __syncthreads_and(act || !primary) != 0;  // also the barrier after the puts
  STAMP256(2);
  A = s64_args<S64_HOT_BYTES>();

  // ---- formation + minimum pass (every pair once, split over the two waves), obstacle pass
  double fsum = 0.0;
  float smin = __builtin_inff();
  uint32_t ok[MSL];
#pragma unroll
  for (int s = 0; s < MSL; ++s) ok[s] = KEY_EMPTY;
  bool ocoll = false;
  if (primary) {
    if (fast) hw_pass1<true, true>(L, w, t, true, px, py, pz, A->P.ds_f, fsum, smin);
    else hw_pass1<false, true>(L, w, t, act, px, py, pz, A->P.ds_f, fsum, smin);
    obstacle_pass_s64<MSL, true>(L.osoa, M, px, py, pz, act, A->P.s_obst, A->P.ob_keep, ok, ocoll);
  } else {
    const float qx = L.seg2[w][0][t], qy = L.seg2[w][1][t], qz = L.seg2[w][2][t];
    const bool self = L.seg2[w][3][t] != 0.f;
    if (SWARM_S256W_PRIO == 1) __builtin_amdgcn_s_setprio(1);
    if (fast) hw_pass1<true, false>(L, w, t, true, qx, qy, qz, A->P.ds_f, fsum, smin);
    else hw_pass1<false, false>(L, w, t, self, qx, qy, qz, A->P.ds_f, fsum, smin);
    if (SWARM_S256W_PRIO == 1) __builtin_amdgcn_s_setprio(0);
  }
  STAMP256(3);
  __syncthreads();  // handed-over sums / minima written
  if (primary) {
    fsum += L.x.p1.dsum[i];
    fsum += (double)L.x.p1.sum[0][i];
    fsum += (double)L.x.p1.sum[1][i];
    smin = fminf(fminf(smin, L.x.p1.mn[2][i]), fminf(L.x.p1.mn[0][i], L.x.p1.mn[1][i]));
    if constexpr (SWARM_S256W_SPLIT1 > 0) {
      fsum += (double)L.x.p1.sum[2][i];
      smin = fminf(smin, L.x.p1.mn[3][i]);
    }
  }
  A = s64_args<S64_HOT_BYTES>();

  STAMP256(4);
  // ---- rewards / terminations: drone_swarm_env.py:120-172 (swarm_kernel, DYN_KIN)
  float curr = 0.f, rew = 0.f;
  bool reached = false, collided = false, term = false, trunc = false, cont = false;
  bool term_all = false, trunc_all = false;
  int new_step = stepc;
  if (primary) {
    bool pcoll = smin <= A->P.thr_pair * FAST_LO;
    if (!pcoll && smin <= A->P.thr_pair * FAST_HI && act)
      pcoll = exact_pair_collision(L.ring, H_N, i, px, py, pz, A->P.s_pair);
    curr = sqrt_rn(sqsum_1d(gx - px, gy - py, gz - pz));
    bool p_coll = false, p_cand = false;
    if (act) {
      reached = (double)curr <= A->P.goal_radius;
      collided = ocoll || pcoll;
      p_coll = collided;
      p_cand = !reached && !collided;
      double r = ((double)prev_d - (double)curr) * A->P.kp;
      if (n_active > 1) r = r + (-A->P.kf) * (fsum * inv_count(n_active - 1));
      if (reached) r = r + A->P.r_goal;
      if (collided) r = r + A->P.r_col;
      rew = (float)r;
    }
    const bool wc = __ballot(p_coll) != 0, wd = __ballot(p_cand) != 0;
    if (t == 0) L.red[w] = (wc ? 1u : 0u) | (wd ? 2u : 0u);
  }
  __syncthreads();
  const uint32_t votes = L.red[0] | L.red[1] | L.red[2] | L.red[3];
  const bool any_c = (votes & 1u) != 0, any_cand = (votes & 2u) != 0;
  A = s64_args<S64_HOT_BYTES>();
  if (n_active == 0) {
    term_all = true;
  } else {
    new_step = stepc + 1;
    const bool tl = new_step >= A->P.max_steps;
    term_all = (!any_cand && !any_c && !tl) || any_c;
    trunc_all = tl && !term_all;
    if (act) {
      const bool done_i = reached || collided;
      term = done_i;
      trunc = tl && !done_i;
      cont = !done_i && !tl && !any_c;
    }
  }
  const bool do_reset = A->P.auto_reset && (term_all || trunc_all);
  if (primary) {
    A->O.reward[ag] = rew;
    A->O.terminated[ag] = term ? 1 : 0;
    A->O.truncated[ag] = trunc ? 1 : 0;
    if (A->O.dist_goal) A->O.dist_goal[ag] = curr;
    if (A->O.info_flags)
      A->O.info_flags[ag] = (uint8_t)((act ? SWARM_AGENT_STEPPED : 0u) | (act && reached ? SWARM_AGENT_REACHED : 0u) |
                                      (act && collided ? SWARM_AGENT_COLLISION : 0u) | (cont ? SWARM_AGENT_HAS_OBS : 0u));
    if (i == 0)
      A->O.env_done[env] = (uint8_t)((term_all ? SWARM_ENV_TERMINATED : 0u) | (trunc_all ? SWARM_ENV_TRUNCATED : 0u) |
                                     (do_reset ? SWARM_ENV_RESET : 0u));
  }

  STAMP256(5);
  // ---- in-kernel auto-reset (block-uniform): the new episode, then its keys
  uint32_t episode_new = episode0;
  if (do_reset) {
    episode_new = episode0 + 1u;
    const long long genv = A->P.env_offset + env;
    const float lo_w = A->P.neg_half_w, wd_w = A->P.width_w;
    float ox = 0.f, oy = 0.f, oz = 0.f;
    if (primary) {
      uint32_t wd4[4];
      draw_block_k(A->P.seed_lo, A->P.seed_hi, genv, episode_new, (uint32_t)i, wd4);
      px = uni(wd4[0], lo_w, wd_w);
      py = uni(wd4[1], lo_w, wd_w);
      pz = uni(wd4[2], lo_w, wd_w);
      vx = vy = vz = 0.f;
      act = true;
    } else if (i <= M) {  // obstacle i (i < M) or the goal (i == M)
      uint32_t wo[4];
      draw_block_k(A->P.seed_lo, A->P.seed_hi, genv, episode_new, (uint32_t)(H_N + i), wo);
      ox = uni(wo[0], lo_w, wd_w); oy = uni(wo[1], lo_w, wd_w); oz = uni(wo[2], lo_w, wd_w);
      if (i < M) {  // the state row: the old one was read into LDS at the start
        float* o = A->S.obstacles + ((size_t)env * M + i) * 3;
        o[0] = ox; o[1] = oy; o[2] = oz;
      }
    }
    __syncthreads();  // every read of the old planes / ring / obstacles is done
    if (primary) {
      hw_put(L, w, t, px, py, pz, 1.f);
    } else if (i < M) {
      L.obst[i] = make_float4(ox, oy, oz, 0.f);
      L.osoa[i] = ox; L.osoa[H_MMAX + i] = oy; L.osoa[2 * H_MMAX + i] = oz;
    } else if (i == M) {
      L.goal = make_float4(ox, oy, oz, 0.f);
    }
    __syncthreads();
    if (primary) {
      const float4 g4 = L.goal;
      gx = g4.x; gy = g4.y; gz = g4.z;
#pragma unroll
      for (int s = 0; s < MSL; ++s) ok[s] = KEY_EMPTY;
      bool c2 = false;
      obstacle_pass_s64<MSL, false>(L.osoa, M, px, py, pz, false, 0.f, A->P.ob_keep, ok, c2);
    }
  }
  STAMP256(6);
  A = s64_args<S64_HOT_BYTES>();
  uint32_t nk[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) nk[s] = KEY_EMPTY;
  if (primary) {
    hw_pass0<true>(L, w, t, px, py, pz, A->P.nb_keep, nk);
  } else {
    const float qx = L.seg2[w][0][t], qy = L.seg2[w][1][t], qz = L.seg2[w][2][t];
    hw_pass0<false>(L, w, t, qx, qy, qz, A->P.nb_keep, nk);
  }
  __syncthreads();  // handed-over key lists written
  if (!primary) return;  // no barrier follows
  {
    uint32_t kb[4], kc[4], ks2[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kb[s] = L.x.keys[0][s][i];
      kc[s] = L.x.keys[1][s][i];
      ks2[s] = L.x.keys[2][s][i];
    }
    h_merge4(nk, ks2);
    h_merge4(nk, kb);
    h_merge4(nk, kc);
#pragma unroll
    for (int s = 0; s < KS; ++s) nk[s] = h_decode(nk[s], w, t, A->P.nb_keep);
  }
  A = s64_args<S64_HOT_BYTES>();

  // ---- exact top-K of the emitted observation (keys rank by s', drone indices)
  float wd[KS], od[MSL];
  int wj[KS], oj[MSL];
  {
    const uint32_t ff = h_finish_fast(nk, ok, L.ring, L.obst, M, A->P.nb_keep, A->P.ob_keep, px, py, pz, wd, wj, od, oj);
    if (__ballot(ff != 0) != 0) {  // straight-line rest of finish_keys (s64_finish_general), then the scans
      bool slow_nb, slow_ob;
      s64_finish_general<KS, MSL, H_N, false, H_MMAX>(ff, nk, ok, L.ring, L.obst, i, M, A->P.nb_keep, A->P.ob_keep,
                                                      false, px, py, pz, wd, wj, od, oj, slow_nb, slow_ob);
      if (slow_nb) exact_select<KS, false>(L.ring, H_N, i, H_K, max_first(wd, H_K), px, py, pz, wd, wj);
      if (slow_ob) exact_select<MSL, true>(L.obst, M, -1, H_MS, max_first(od, H_MS), px, py, pz, od, oj);
    }
  }
  STAMP256(7);
  A = s64_args<S64_HOT_BYTES>();

  // ---- state write-back
  const bool new_act = do_reset || cont;
  A->S.pos[ag * 3] = px; A->S.pos[ag * 3 + 1] = py; A->S.pos[ag * 3 + 2] = pz;
  A->S.vel[ag * 3] = vx; A->S.vel[ag * 3 + 1] = vy; A->S.vel[ag * 3 + 2] = vz;
  A->S.active[ag] = new_act ? 1 : 0;
  if (i == 0) {
    A->S.step_count[env] = do_reset ? 0 : new_step;
    if (do_reset) {
      A->S.episode[env] = episode_new;
      A->S.goal[3 * env] = gx; A->S.goal[3 * env + 1] = gy; A->S.goal[3 * env + 2] = gz;
    }
  }
  if (A->O.global_state) {
    float* gs = A->O.global_state + (size_t)env * (6 * H_N + 3);
    gs[3 * i] = px; gs[3 * i + 1] = py; gs[3 * i + 2] = pz;
    gs[3 * H_N + 3 * i] = vx; gs[3 * H_N + 3 * i + 1] = vy; gs[3 * H_N + 3 * i + 2] = vz;
    if (i == 0) { gs[6 * H_N] = gx; gs[6 * H_N + 1] = gy; gs[6 * H_N + 2] = gz; }
  }
  A = s64_args<S64_HOT_BYTES>();

  // ---- observation row [p | v | g-p | K x (p_j-p, d) | Ms x (o_m-p, d)]
  constexpr int D = 9 + 4 * H_K + 4 * H_MS;
#ifndef SWARM_S256W_STAGE
#define SWARM_S256W_STAGE 1  // r06c: 36.68 / 36.88 / 37.24 vs 38.10 / 38.21 / 38.58 us (config 5, graph, 4 groups)
#endif
#if SWARM_S256W_STAGE
  // staged like step64's rows: 16 rows at a time in this wave's (dead) plane segment, then stored
  // as coalesced 16-B write-through buffer stores of the wave's contiguous 64-row block — straight
  // from registers, every dword store touched 64 lines (148-B row stride), partial-line writes
  float row[D];
#else
  float* row = A->O.obs + ag * D;  // straight from registers
#endif
  row[0] = px; row[1] = py; row[2] = pz;
  row[3] = vx; row[4] = vy; row[5] = vz;
  row[6] = gx - px; row[7] = gy - py; row[8] = gz - pz;
#pragma unroll
  for (int s = 0; s < H_K; ++s) {
    const float4 q = lds_f4(L.ring + (wj[s] & (H_N - 1)));
    row[9 + 4 * s] = q.x - px; row[10 + 4 * s] = q.y - py; row[11 + 4 * s] = q.z - pz; row[12 + 4 * s] = wd[s];
  }
#pragma unroll
  for (int s = 0; s < H_MS; ++s) {
    const float4 q = lds_f4(L.obst + (oj[s] & (H_MMAX - 1)));
    row[21 + 4 * s] = q.x - px; row[22 + 4 * s] = q.y - py; row[23 + 4 * s] = q.z - pz; row[24 + 4 * s] = od[s];
  }
#if SWARM_S256W_STAGE
  {
    constexpr int CH = 16, V4 = CH * D / 4, NF = V4 / 64, NR = V4 % 64;
    static_assert(CH * D <= 4 * H_PS && (CH * D) % 4 == 0 && H_N % CH == 0, "stage chunk in the wave's planes");
    // this wave's planes are dead: every pass-0 read precedes the hand-over barrier
    float* stage = &L.seg2[w][0][0];
    const float4* s4 = reinterpret_cast<const float4*>(stage);
    float* srow = stage + (t % CH) * D;
    float* const ob = A->O.obs + ((size_t)env * H_N + 64 * w) * D;  // the wave's 64 rows, contiguous
#pragma unroll
    for (int ch = 0; ch < 64 / CH; ++ch) {
      if (t / CH == ch) {
#pragma unroll
        for (int k = 0; k < D; ++k) srow[k] = row[k];
      }
      wave_sync();
      float4 v[NF + 1];
#pragma unroll
      for (int k = 0; k < NF; ++k) v[k] = s4[t + 64 * k];
      if (NR && t < NR) v[NF] = s4[t + 64 * NF];
#pragma unroll
      for (int k = 0; k < NF; ++k) store_obs(ob, 64 * D * 4, 16u * (ch * V4 + t + 64 * k), v[k]);
      if (NR && t < NR) store_obs(ob, 64 * D * 4, 16u * (ch * V4 + t + 64 * NF), v[NF]);
      wave_sync();
    }
  }
#endif
  STAMP256(8);
  STAMP_END(env, threadIdx.x == 0);
}
}  // namespace
namespace swarm_dev {

#endif

// ------------------------------------------------------------------ host side
typedef void (*step64_fn)(const S64Args);
typedef void (*step64o_fn)(const float*, const float*, const float*, const uint8_t*, const uint32_t*, const uint8_t*, int,
                           int, const S64Args);
typedef void (*step16q_fn)(const float*, const float*, const float*, const uint8_t*, const uint32_t*, const int32_t*,
                           const uint8_t*, const S64Args);
typedef void (*kernel_fn)(const KParams, const swarm_state_t, const float*, const uint8_t*, const swarm_out_t,
                          const uint8_t*, int);

template <int KIND, int DYN, int KS, int LM>
kernel_fn pick_ms(int msl) {
  switch (msl) {
    case 0: return swarm_kernel<KIND, DYN, KS, 0, LM>;
    case 5: return swarm_kernel<KIND, DYN, KS, 5, LM>;
    case 9: return swarm_kernel<KIND, DYN, KS, 9, LM>;
    default: return swarm_kernel<KIND, DYN, KS, 17, LM>;
  }
}
template <int KIND, int DYN, int LM>
kernel_fn pick_ks(int ks, int msl) {
  switch (ks) {
    case 0: return pick_ms<KIND, DYN, 0, LM>(msl);
    case 4: return pick_ms<KIND, DYN, 4, LM>(msl);
    case 9: return pick_ms<KIND, DYN, 9, LM>(msl);
    default: return pick_ms<KIND, DYN, 17, LM>(msl);
  }
}
template <int KIND, int DYN>
void* pick_lm(int lm, int ks, int msl) {
#ifdef SWARM_DEV_HOT
  // diagnostic builds (tools/): only K = 3, Ms = 4 (the reset / observe of configs 2, 3 and 5)
  if (ks == 4 && msl == 5) {
    if (lm == 2) return reinterpret_cast<void*>(swarm_kernel<KIND, DYN, 4, 5, 2>);
    if (lm == 1) return reinterpret_cast<void*>(swarm_kernel<KIND, DYN, 4, 5, 1>);
    if (lm == 0) return reinterpret_cast<void*>(swarm_kernel<KIND, DYN, 4, 5, 0>);
  }
  return nullptr;
#else
  switch (lm) {
    case 0: return reinterpret_cast<void*>(pick_ks<KIND, DYN, 0>(ks, msl));
    case 1: return reinterpret_cast<void*>(pick_ks<KIND, DYN, 1>(ks, msl));
    default: return reinterpret_cast<void*>(pick_ks<KIND, DYN, 2>(ks, msl));
  }
#endif
}

}  // namespace swarm_dev

// kernel tables, one per translation unit (SWARM_PART); returns the host stub of the kernel
#define SWARM_PICK_DECL(k) __attribute__((visibility("hidden"))) void* swarm_pick_##k(int lm, int ks, int msl)
SWARM_PICK_DECL(0);
SWARM_PICK_DECL(1);
SWARM_PICK_DECL(2);
SWARM_PICK_DECL(3);
// the headline specialisation (SWARM_PART 5)
__attribute__((visibility("hidden"))) void* swarm_pick_step64(bool persistent, bool physics);
__attribute__((visibility("hidden"))) void* swarm_pick_step64_eval();
// the config-2 specialisation (SWARM_PART 6)
__attribute__((visibility("hidden"))) void* swarm_pick_step16q();
// the config-5 specialisation (SWARM_PART 7)
// (kernel, threads per workgroup, LDS bytes): swarm_step256w (512 threads) unless SWARM_S256_WIDE=0
__attribute__((visibility("hidden"))) void* swarm_pick_step256(int* threads, int* lds_bytes);
#if SWARM_HAS_PART(7)
#ifndef SWARM_S256_WIDE
#define SWARM_S256_WIDE 1
#endif
__attribute__((visibility("hidden"))) void* swarm_pick_step256(int* threads, int* lds_bytes) {
  if (SWARM_S256_WIDE) {
    *threads = 2 * swarm_dev::H_N;
    *lds_bytes = (int)sizeof(swarm_dev::H256WLds);
    return reinterpret_cast<void*>(swarm_step256w);
  }
  *threads = swarm_dev::H_N;
  *lds_bytes = (int)sizeof(swarm_dev::H256Lds);
  return reinterpret_cast<void*>(swarm_step256);
}
#endif
#if SWARM_HAS_PART(6)
__attribute__((visibility("hidden"))) void* swarm_pick_step16q() {
  return reinterpret_cast<void*>(swarm_step16q);
}
#endif
#if SWARM_HAS_PART(5)
__attribute__((visibility("hidden"))) void* swarm_pick_step64_eval() {
  return reinterpret_cast<void*>(swarm_step64_eval_once<S64_CH, S64_WG_ENVS>);
}
__attribute__((visibility("hidden"))) void* swarm_pick_step64(bool persistent, bool physics) {
  if (physics) return reinterpret_cast<void*>(swarm_step64_phys_once<S64_CH, S64_WG_ENVS>);
  return persistent ? reinterpret_cast<void*>(swarm_step64<S64_CH>)
                    : reinterpret_cast<void*>(swarm_step64_once<S64_CH, S64_WG_ENVS>);
}
#endif
#if SWARM_HAS_PART(0)
SWARM_PICK_DECL(0) { return pick_lm<KIND_STEP, DYN_KIN>(lm, ks, msl); }
#endif
#if SWARM_HAS_PART(1)
SWARM_PICK_DECL(1) { return pick_lm<KIND_STEP, DYN_PHYS>(lm, ks, msl); }
#endif
#if SWARM_HAS_PART(2)
SWARM_PICK_DECL(2) { return pick_lm<KIND_AUX, DYN_KIN>(lm, ks, msl); }
#endif
#if SWARM_HAS_PART(3)
SWARM_PICK_DECL(3) { return pick_lm<KIND_AUX, DYN_PHYS>(lm, ks, msl); }
#endif

#if SWARM_HAS_HOST
namespace {
thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// Largest float s >= 0 with sqrtf(s) <= T: lets the passes compare the exact float squared
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
// compile-time slot counts: K+1 (or more) neighbour keys, Ms_eff+1 obstacle keys
int neighbor_slots(int K) {
  if (K <= 0) return 0;
  if (K <= 3) return 4;
  if (K <= 8) return 9;
  return 17;
}
int obstacle_slots(int Ms, int M) {
  const int need = Ms < M ? Ms : M;
  if (need <= 0) return 0;
  if (need <= 4) return 5;
  if (need <= 8) return 9;
  return 17;
}

int obs_dim_of(const swarm_params_t* p) {
  return 9 + 4 * (p->neighbor_k > 0 ? p->neighbor_k : 0) + 4 * (p->sensed_obstacles > 0 ? p->sensed_obstacles : 0);
}

// The headline specialisation swarm_step64 covers N = 64, K = 3, Ms = 4, 4 <= M <= 16 in
// kinematic/swarm mode (buffer alignment is checked at launch).
// The specialisations' loads index with 32-bit element offsets (E x N x 3 and E x M x 3 < 2^32):
// batches above 2^22 envs take the generic kernel.
constexpr int SPEC_MAX_E = 1 << 22;
bool step64_applies(const swarm_params_t* p, const KParams& k) {
  return p->kernel_path == SWARM_PATH_AUTO && k.N == S64_N && k.K == S64_K && k.Ms == S64_MS && k.M >= S64_MS &&
         k.M <= S64_MMAX && k.E <= SPEC_MAX_E && (p->dynamics == DYN_KIN || p->dynamics == DYN_PHYS);
}

// The config-2 specialisation swarm_step16q covers N = 16, K = 3, Ms = 4, 4 <= M <= 16, kinematic.
bool step16q_applies(const swarm_params_t* p, const KParams& k) {
  return p->kernel_path == SWARM_PATH_AUTO && k.N == Q_N && k.K == Q_K && k.Ms == Q_MS && k.M >= Q_MS &&
         k.M <= Q_MMAX && k.E <= SPEC_MAX_E && p->dynamics == DYN_KIN;
}

// The config-5 specialisation swarm_step256 covers N = 256, K = 3, Ms = 4, 4 <= M <= 16, kinematic.
bool step256_applies(const swarm_params_t* p, const KParams& k) {
  return p->kernel_path == SWARM_PATH_AUTO && k.N == H_N && k.K == H_K && k.Ms == H_MS && k.M >= H_MS &&
         k.M <= H_MMAX && k.E <= SPEC_MAX_E && p->dynamics == DYN_KIN;  // E x 256 x 3 < 2^32: 32-bit offsets
}

// Persistent grid of swarm_step64: waves_per_simd x 4 SIMDs x the current device's CUs (E when
// no device is visible, e.g. host-only queries).
int step64_grid(const swarm_params_t* p, int E) {
  static std::atomic<int> cu_cache[64];
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return E;
  if (dev < 64) cus = cu_cache[dev].load(std::memory_order_relaxed);
  if (cus <= 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
      (void)hipGetLastError();
      return E;
    }
    if (dev < 64) cu_cache[dev].store(cus, std::memory_order_relaxed);
  }
  const int wps = p->waves_per_simd > 0 ? p->waves_per_simd : S64_WPS_DEFAULT;
  if (wps <= 0) return E;
  const long long g = (long long)cus * 4 * wps;
  return g < E ? (int)g : E;
}

int build_kparams_uncached(const swarm_params_t* p, KParams* kp, swarm_launch_info_t* info);
// Derived launch parameters of the last few params blocks (every step call derives them; an
// env-group step derives them once per group): a hit is one memcmp of the 240-B params block.
struct KpMemo {
  swarm_params_t p;
  KParams k;
  swarm_launch_info_t info;
  bool valid;
};
thread_local KpMemo g_kp_memo[4];
thread_local int g_kp_memo_next = 0;
int build_kparams(const swarm_params_t* p, KParams* kp, swarm_launch_info_t* info) {
  if (p) {
    for (const KpMemo& m : g_kp_memo) {
      if (m.valid && memcmp(&m.p, p, sizeof(*p)) == 0) {
        *kp = m.k;
        if (info) *info = m.info;
        return SWARM_OK;
      }
    }
  }
  swarm_launch_info_t li;
  const int rc = build_kparams_uncached(p, kp, &li);
  if (rc == SWARM_OK) {
    KpMemo& m = g_kp_memo[g_kp_memo_next];
    g_kp_memo_next = (g_kp_memo_next + 1) % 4;
    m.p = *p;
    m.k = *kp;
    m.info = li;
    m.valid = true;
    if (info) *info = li;
  }
  return rc;
}
int build_kparams_uncached(const swarm_params_t* p, KParams* kp, swarm_launch_info_t* info) {
  if (!p) return fail(SWARM_ENULL, "params is NULL");
  if (p->abi_version != SWARM_ABI_VERSION)
    return fail(SWARM_EINVAL, "abi_version %d != library %d", p->abi_version, SWARM_ABI_VERSION);
  if (p->num_envs < 0) return fail(SWARM_EINVAL, "num_envs must be >= 0 (got %d)", p->num_envs);
  if (p->num_drones < 1 || p->num_drones > MAX_N)
    return fail(SWARM_ELIMIT, "num_drones must be in [1, %d] (got %d)", MAX_N, p->num_drones);
  if (p->num_obstacles < 0 || p->num_obstacles > 65536) return fail(SWARM_EINVAL, "num_obstacles must be in [0, 65536]");
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
  if (p->kernel_path != SWARM_PATH_AUTO && p->kernel_path != SWARM_PATH_GENERIC)
    return fail(SWARM_EINVAL, "kernel_path must be SWARM_PATH_AUTO or SWARM_PATH_GENERIC (got %d)", p->kernel_path);
  if (p->waves_per_simd < 0 || p->waves_per_simd > 8)
    return fail(SWARM_EINVAL, "waves_per_simd must be in [0, 8] (got %d)", p->waves_per_simd);

  KParams k;
  memset(&k, 0, sizeof(k));
  k.E = p->num_envs;
  k.N = p->num_drones;
  k.M = p->num_obstacles;
  k.K = p->neighbor_k > 0 ? p->neighbor_k : 0;
  k.Ms = p->sensed_obstacles > 0 ? p->sensed_obstacles : 0;
  k.D = obs_dim_of(p);
  k.max_steps = p->max_steps;
  k.auto_reset = p->auto_reset ? 1 : 0;
  k.substeps = p->physics_substeps;
  k.damping_law = p->damping_law;
  const int lanes = next_pow2(k.N);
  k.log2_lanes = ilog2(lanes);
  const bool wave = lanes <= 64;
  const int threads = wave ? 64 : lanes;
  k.envs_per_block = threads / lanes;
  const int G = k.envs_per_block;
  k.ring = wave ? 2 * lanes : lanes;
  k.obst_stride = k.M + 1;
  k.off_obst = G * k.ring * 16;
  const long long obst_bytes = (long long)G * k.obst_stride * 16;
  k.off_stage = (int)(k.off_obst + obst_bytes);
  k.off_pair = 0;
  if (!wave && lanes == k.N) {  // block team, N a power of two: the rotation passes' pair ring
    k.off_pair = k.off_stage;
    k.off_stage = (int)(k.off_pair + 2LL * k.N * BLK_PAIR_STRIDE * 4);
  }
  const int rows = G * k.N;
  const long long row_bytes = 4LL * k.D;
  int rounds = (int)((rows * row_bytes + STAGE_BUDGET - 1) / STAGE_BUDGET);
  if (rounds < 1) rounds = 1;
  int ch = (rows + rounds - 1) / rounds;
  ch = (ch + 3) & ~3;  // multiple of 4 rows keeps every chunk 16-B aligned
  if (ch > rows) ch = rows;
  k.chunk_rows = ch;
  const long long lds = k.off_stage + (long long)ch * row_bytes;
  if (lds > LDS_LIMIT) return fail(SWARM_ELIMIT, "LDS footprint %lld B exceeds %d B (N=%d, M=%d)", lds, LDS_LIMIT, k.N, k.M);
  k.obs_vec4 = (((long long)rows * k.D) % 4 == 0 && ((long long)ch * k.D) % 4 == 0) ? 1 : 0;
  // Small launches of multi-team waves or block teams (<= 2048 workgroups) are latency-bound: rows
  // go straight from registers to memory (N=16: E=1024 14.0 -> 13.1 us per step, E=8192 18.4 ->
  // 18.2; N=256 x E=1024 in 2 groups 63.0 -> 60.6); larger ones keep the coalescing LDS stage
  // (N=16, E=32768: 33.1 vs 42.7 us direct).  One-env waves (lanes = 64) always stage.
  // SWARM_OBS_DIRECT=0/1 overrides (diagnostics).
  {
    const long long blocks = ((long long)k.E + G - 1) / G;
    k.obs_direct = (lanes != 64 && blocks <= 2048) ? 1 : 0;
    // read once per process: the derived parameters are memoised by the params bytes (KpMemo),
    // so an override set after the first launch would be ignored silently for a cached block
    static const int obs_direct_override = []() {
      const char* ov = getenv("SWARM_OBS_DIRECT");
      return (ov && (ov[0] == '0' || ov[0] == '1')) ? ov[0] - '0' : -1;
    }();
    if (obs_direct_override >= 0) k.obs_direct = obs_direct_override;
  }
  // neighbour keys carry the drone index (block) or the rotation offset in [1, L) (wave)
  const int nb_bits = k.log2_lanes;
  const int ob_bits = ilog2(k.M > 1 ? k.M : 2);
  k.nb_keep = nb_bits > 0 ? ~((1u << nb_bits) - 1u) : ~0u;
  k.ob_keep = ~((1u << ob_bits) - 1u);
  k.env_offset = p->env_offset;
  k.seed_lo = (unsigned)(p->seed & 0xffffffffull);
  k.seed_hi = (unsigned)(p->seed >> 32);
  k.half_w = (float)(p->world_size / 2.0);
  k.neg_half_w = (float)(-p->world_size / 2.0);
  k.width_w = (float)p->world_size;
  k.dt = (float)p->dt;
  k.vmax = (float)p->max_speed;
  k.s_vmax = s_threshold(k.vmax);
  k.amax = (float)p->max_accel;
  k.ds_f = (float)p->desired_spacing;
  k.thr_pair = (float)(2.0 * p->collision_radius);
  k.s_pair = s_threshold(k.thr_pair);
  k.s_obst = s_threshold((float)(p->collision_radius + p->obstacle_radius));
  k.thr_ppair = (float)(2.0 * p->drone_contact_radius);
  k.s_phys_pair = s_threshold(k.thr_ppair);
  k.s_phys_obst = s_threshold((float)(p->obstacle_radius + p->drone_contact_radius));
  k.ground_z = (float)p->ground_contact_height;
  k.h = (float)p->substep_dt;
  k.g = (float)p->gravity;
  k.gcomp = (float)p->gravity_comp;
  k.goal_radius = p->goal_radius;
  {  // the largest float <= goal_radius, then its squared-space threshold
    float gr = (float)p->goal_radius;
    if ((double)gr > p->goal_radius) gr = nextafterf(gr, -INFINITY);
    k.s_goal = s_threshold(gr);
  }
  k.kp = p->reward_progress_scale;
  k.r_goal = p->reward_goal;
  k.r_col = p->reward_collision;
  k.kf = p->reward_formation_scale;
  k.vmax_d = p->max_speed;
  *kp = k;
  if (info) {
    info->threads_per_block = threads;
    info->envs_per_block = G;
    info->lanes_per_env = lanes;
    info->blocks = (int)((k.E + G - 1) / G);
    info->lds_bytes = (int)lds;
    info->neighbor_slots = neighbor_slots(k.K);
    info->obstacle_slots = obstacle_slots(k.Ms, k.M);
    info->obs_dim = k.D;
    info->staged_obs = k.obs_direct ? 0 : 1;
    info->kernel_id = SWARM_KERNEL_GENERIC;
  }
  return SWARM_OK;
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
  if (s->env_cfg_next && !s->env_cfg) return fail(SWARM_ENULL, "state.env_cfg_next needs state.env_cfg");
  if (!o->obs) return fail(SWARM_ENULL, "out.obs is NULL");
  if (mode == MODE_STEP) {
    if (!actions) return fail(SWARM_ENULL, "actions is NULL");
    if (!o->reward || !o->terminated || !o->truncated || !o->env_done)
      return fail(SWARM_ENULL, "out.reward/terminated/truncated/env_done required by swarm_step");
  }
  if (((uintptr_t)o->obs) % 16 != 0) kp.obs_vec4 = 0;
  // ballot-packed byte outputs need N == 64 and dword-aligned bool tensors
  kp.pack_bytes = (kp.N == 64 && mode == MODE_STEP && ((uintptr_t)o->terminated | (uintptr_t)o->truncated |
                                                       (uintptr_t)s->active) % 4 == 0) ? 1 : 0;
  S64Eval ev{};
  // out.eval is a step-only input: reset / observe never touch the eval accumulators (a VecSwarm
  // passes the same out struct to every mode), so it is neither validated nor used there
  if (o->eval && mode == MODE_STEP) {
    // fused eval accumulation: the kinematic one-wave-per-env step64 launch only
    const swarm_eval_t* e = o->eval;
    const bool once = mode == MODE_STEP && step64_applies(p, kp) && kp.obs_vec4 && kp.pack_bytes && !s->env_cfg &&
                      p->dynamics == DYN_KIN && !(s->work && step64_grid(p, kp.E) < kp.E);
    if (!once)
      return fail(SWARM_EINVAL, "out.eval (fused eval accumulation) needs the kinematic swarm_step64 launch "
                                "(N = 64, K = 3, Ms = 4, no env_cfg, no persistent grid)");
    if (!(e->flags & SWARM_EVAL_STEP_FUSED)) return fail(SWARM_EINVAL, "out.eval without SWARM_EVAL_STEP_FUSED in its flags");
    if (!e->ep_reward || !e->ep_steps || !e->reached_step || !e->status || !e->traveled || !e->fe_sum || !e->start ||
        !e->goal || !e->records || !e->count)
      return fail(SWARM_ENULL, "out.eval: an eval state buffer is NULL");
    const int nseg = e->segments > 0 ? e->segments : SWARM_EVAL_SEGMENTS;
    if (e->segments < 0 || e->segments > SWARM_EVAL_SEGMENTS || e->seg_base < 0 || e->capacity < 0 ||
        e->capacity % nseg != 0)
      return fail(SWARM_EINVAL, "out.eval: bad capacity / segments / seg_base");
    ev = S64Eval{e->ep_reward, e->ep_steps, e->reached_step, e->status, e->traveled, e->fe_sum, e->start, e->goal,
                 e->records, e->count, e->capacity, e->update_index, e->seg_base, e->segments, p->desired_spacing};
  }
  if (mode == MODE_STEP && step64_applies(p, kp) && kp.obs_vec4 && kp.pack_bytes && !s->env_cfg) {
    swarm_state_t st = *s;
    const bool phys = p->dynamics == DYN_PHYS;  // physics: the one-wave-per-env launch only
    const int grid = phys ? kp.E : step64_grid(p, kp.E);
    if (grid >= kp.E) st.work = nullptr;  // one env per workgroup: nothing to dequeue
    const S64Args args{kp, st, actions, amask, *o, ev};
    if (st.work)
      hipLaunchKernelGGL(reinterpret_cast<step64_fn>(swarm_pick_step64(true, false)), dim3(grid), dim3(64), 0,
                         (hipStream_t)stream, args);
    else  // the first loads' addresses, E and M lead the arguments (preloaded into SGPRs)
      hipLaunchKernelGGL(reinterpret_cast<step64o_fn>(ev.status ? swarm_pick_step64_eval() : swarm_pick_step64(false, phys)),
                         dim3((kp.E + S64_WG_ENVS - 1) / S64_WG_ENVS), dim3(64 * S64_WG_ENVS), 0, (hipStream_t)stream,
                         (const float*)st.pos, (const float*)st.vel, actions, (const uint8_t*)st.active,
                         (const uint32_t*)st.goal, amask, kp.E, kp.M, args);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SWARM_EHIP, "kernel launch: %s", hipGetErrorString(e));
    return SWARM_OK;
  }
  if (mode == MODE_STEP && step16q_applies(p, kp) && !s->env_cfg && ((uintptr_t)o->obs) % 16 == 0 &&
      ((uintptr_t)o->terminated | (uintptr_t)o->truncated | (uintptr_t)s->active) % 4 == 0) {
    const S64Args args{kp, *s, actions, amask, *o, ev};
    // one env per 3-wave workgroup (rewards / observation / next episode); the first loads'
    // addresses lead the kernel arguments (preloaded into SGPRs)
    hipLaunchKernelGGL(reinterpret_cast<step16q_fn>(swarm_pick_step16q()), dim3(kp.E), dim3(192), 0,
                       (hipStream_t)stream, (const float*)s->pos, (const float*)s->vel, actions,
                       (const uint8_t*)s->active, (const uint32_t*)s->goal, (const int32_t*)s->step_count, amask,
                       args);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SWARM_EHIP, "kernel launch: %s", hipGetErrorString(e));
    return SWARM_OK;
  }
  // (16-B aligned obs: the wide kernel stages its rows and stores them as 16-B buffer stores)
  if (mode == MODE_STEP && step256_applies(p, kp) && !s->env_cfg && ((uintptr_t)o->obs) % 16 == 0) {
    const S64Args args{kp, *s, actions, amask, *o};
    int threads = 0, lds = 0;
    // the first loads' addresses, E and M lead the arguments (preloaded into SGPRs, as step64 / step16q)
    const step64o_fn k256 = reinterpret_cast<step64o_fn>(swarm_pick_step256(&threads, &lds));
    hipLaunchKernelGGL(k256, dim3(kp.E), dim3(threads), 0, (hipStream_t)stream, (const float*)s->pos,
                       (const float*)s->vel, actions, (const uint8_t*)s->active, (const uint32_t*)s->goal, amask, kp.E,
                       kp.M, args);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SWARM_EHIP, "kernel launch: %s", hipGetErrorString(e));
    return SWARM_OK;
  }
  const int lanes = 1 << kp.log2_lanes;
  const int lm = lanes > 64 ? 0 : (lanes == 64 ? 2 : 1);
  const int ks = info.neighbor_slots, msl = info.obstacle_slots;
  const bool kin = p->dynamics == DYN_KIN;
  void* fnp = (mode == MODE_STEP) ? (kin ? swarm_pick_0(lm, ks, msl) : swarm_pick_1(lm, ks, msl))
                                  : (kin ? swarm_pick_2(lm, ks, msl) : swarm_pick_3(lm, ks, msl));
  kernel_fn fn = reinterpret_cast<kernel_fn>(fnp);
  if (!fn) return fail(SWARM_ELIMIT, "no kernel instantiation for lanes=%d ks=%d msl=%d in this build", lanes, ks, msl);
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

// ---- per-env parameter records (swarm_env_cfg_set)
// s_threshold on the device: the same search with IEEE sqrt (llvm.sqrt) and one-ulp steps on
// the bit pattern (every argument here is finite and >= 0, so the patterns are ordered).
__device__ float s_threshold_dev(float T) {
  if (!(T >= 0.0f)) return -1.0f;
  if (__builtin_isinf(T)) return __builtin_inff();
  float s = T * T;
  while (s > 0.0f && __builtin_sqrtf(s) > T) s = __uint_as_float(__float_as_uint(s) - 1u);
  for (;;) {
    const float nx = __uint_as_float(__float_as_uint(s) + 1u);
    if (__builtin_isinf(nx) || __builtin_sqrtf(nx) > T) break;
    s = nx;
  }
  return s;
}

struct EnvCfgBase {
  int E, M, max_steps;
  double world_size, dt, max_speed, max_accel, obstacle_radius, collision_radius, drone_contact_radius;
};

// one thread per env; the derivations are build_kparams' (double -> float conversions included)
__global__ void __launch_bounds__(256) env_cfg_set_kernel(const EnvCfgBase B, const swarm_env_overrides_t ov,
                                                          const uint8_t* __restrict__ env_mask,
                                                          swarm_env_cfg_t* __restrict__ out) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B.E) return;
  if (env_mask != nullptr && env_mask[e] == 0) return;
  const double ws = ov.world_size ? ov.world_size[e] : B.world_size;
  const double dt = ov.dt ? ov.dt[e] : B.dt;
  const double vmax = ov.max_speed ? ov.max_speed[e] : B.max_speed;
  const double amax = ov.max_accel ? ov.max_accel[e] : B.max_accel;
  const double orad = ov.obstacle_radius ? ov.obstacle_radius[e] : B.obstacle_radius;
  swarm_env_cfg_t c;
  c.half_w = (float)(ws / 2.0);
  c.neg_half_w = (float)(-ws / 2.0);
  c.width_w = (float)ws;
  c.dt = (float)dt;
  c.max_speed = (float)vmax;
  c.max_accel = (float)amax;
  c.s_vmax = s_threshold_dev(c.max_speed);
  c.s_obst = s_threshold_dev((float)(B.collision_radius + orad));
  c.s_phys_obst = s_threshold_dev((float)(orad + B.drone_contact_radius));
  c.max_steps = ov.max_steps ? ov.max_steps[e] : B.max_steps;
  c.num_obstacles = clamp_obstacles(ov.num_obstacles ? ov.num_obstacles[e] : B.M, B.M);
  c.reserved = 0;
  c.max_speed_d = vmax;
  c.world_size = ws;
  out[e] = c;
}

}  // namespace

extern "C" {

int swarm_abi_version(void) { return SWARM_ABI_VERSION; }

#ifdef SWARM_STAMPS
int swarm_debug_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -1;
}
#endif

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
  p->kernel_path = SWARM_PATH_AUTO;
}

int swarm_obs_dim(const swarm_params_t* p) {
  if (!p) return fail(SWARM_ENULL, "params is NULL");
  return obs_dim_of(p);
}

int swarm_query_launch(const swarm_params_t* p, swarm_launch_info_t* info) {
  KParams kp;
  if (!info) return fail(SWARM_ENULL, "info is NULL");
  const int rc = build_kparams(p, &kp, info);
  if (rc == SWARM_OK && step16q_applies(p, kp)) {  // one env per 64-lane wave, 4 lanes per drone
    info->lanes_per_env = 64;
    info->threads_per_block = 192;  // waves 0 / 1 step the env (rewards / observation), wave 2 its next episode
    info->envs_per_block = 1;
    info->blocks = kp.E;
    info->lds_bytes = 3 * (int)sizeof(Q16Lds) + 4;
    info->staged_obs = 0;
    info->kernel_id = SWARM_KERNEL_STEP16Q;
  }
  if (rc == SWARM_OK && step256_applies(p, kp)) {  // one env per workgroup of 512 (or 256) threads
    int threads = 0, lds = 0;
    (void)swarm_pick_step256(&threads, &lds);
    info->lanes_per_env = H_N;
    info->threads_per_block = threads;
    info->envs_per_block = 1;
    info->blocks = kp.E;
    info->lds_bytes = lds;
    info->staged_obs = 0;
    info->kernel_id = SWARM_KERNEL_STEP256;
  }
  if (rc == SWARM_OK && step64_applies(p, kp)) {  // geometry of the step launch (reset/observe stay generic)
    const int grid = p->dynamics == DYN_PHYS ? kp.E : step64_grid(p, kp.E);
    const int lds_env = (int)sizeof(S64Lds<S64_CH>);
    info->lanes_per_env = 64;
    if (grid < kp.E) {  // persistent grid with env queues (launched when state.work is given)
      info->threads_per_block = 64;
      info->envs_per_block = 1;
      info->blocks = grid;
      info->lds_bytes = lds_env;
      info->kernel_id = SWARM_KERNEL_STEP64_PERSISTENT;
    } else {  // one wave per env, S64_WG_ENVS independent waves per workgroup
      info->threads_per_block = 64 * S64_WG_ENVS;
      info->envs_per_block = S64_WG_ENVS;
      info->blocks = (kp.E + S64_WG_ENVS - 1) / S64_WG_ENVS;
      info->lds_bytes = S64_WG_ENVS * lds_env;
      info->kernel_id = SWARM_KERNEL_STEP64;
    }
  }
  return rc;
}

int swarm_step(const swarm_params_t* p, const swarm_state_t* s, const float* actions, const uint8_t* action_mask,
               const swarm_out_t* o, void* hip_stream) {
  return launch(MODE_STEP, p, s, actions, action_mask, nullptr, o, hip_stream);
}

// Env groups in one call: group g = rows [lo_g, lo_g + group_envs[g]) of every [E, ...] buffer,
// stepped by its own launch on hip_streams[g] with env_offset + lo_g (so its device-RNG draws are
// those of the whole-batch launch).  The params are validated once, before any group launches.
int swarm_step_groups(const swarm_params_t* p, const swarm_state_t* s, const float* actions,
                      const uint8_t* action_mask, const swarm_out_t* o, int groups, const int32_t* group_envs,
                      void* const* hip_streams) {
  KParams kp;
  const int rc0 = build_kparams(p, &kp, nullptr);
  if (rc0) return rc0;
  if (!s || !o) return fail(SWARM_ENULL, "state/out is NULL");
  if (groups < 1) return fail(SWARM_EINVAL, "groups must be >= 1 (got %d)", groups);
  if (!group_envs || !hip_streams) return fail(SWARM_ENULL, "group_envs/hip_streams is NULL");
  long long total = 0;
  for (int g = 0; g < groups; ++g) {
    if (group_envs[g] < 0) return fail(SWARM_EINVAL, "group_envs[%d] = %d < 0", g, group_envs[g]);
    total += group_envs[g];
  }
  if (total != p->num_envs) return fail(SWARM_EINVAL, "group_envs sum to %lld, num_envs is %d", total, p->num_envs);
  const size_t N = (size_t)kp.N, M = (size_t)kp.M, D = (size_t)kp.D;
  size_t lo = 0;
  for (int g = 0; g < groups; ++g) {
    auto row = [lo](auto* ptr, size_t per_env) { return ptr ? ptr + lo * per_env : ptr; };
    swarm_params_t pg = *p;
    pg.num_envs = group_envs[g];
    pg.env_offset = p->env_offset + (int64_t)lo;
    swarm_state_t sg = *s;
    sg.pos = row(s->pos, 3 * N);
    sg.vel = row(s->vel, 3 * N);
    sg.goal = row(s->goal, 3);
    sg.obstacles = row(s->obstacles, 3 * M);
    sg.active = row(s->active, N);
    sg.step_count = row(s->step_count, 1);
    sg.episode = row(s->episode, 1);
    sg.damping = row(s->damping, N);
    sg.work = s->work ? s->work + (size_t)g * SWARM_WORK_WORDS : nullptr;
    sg.env_cfg = row(s->env_cfg, 1);
    sg.env_cfg_next = row(s->env_cfg_next, 1);
    swarm_out_t og = *o;
    swarm_eval_t eg;  // the eval accumulators of the group's rows (fused eval)
    if (o->eval) {
      eg = *o->eval;
      eg.ep_reward = row(eg.ep_reward, 1);
      eg.ep_steps = row(eg.ep_steps, 1);
      eg.reached_step = row(eg.reached_step, 1);
      eg.status = row(eg.status, 1);
      eg.traveled = row(eg.traveled, N);
      eg.fe_sum = row(eg.fe_sum, 1);
      eg.start = row(eg.start, 3 * N);
      eg.goal = row(eg.goal, 3 * N);
      eg.last = row(eg.last, 3 * N);
      og.eval = &eg;
    }
    og.obs = row(o->obs, N * D);
    og.reward = row(o->reward, N);
    og.terminated = row(o->terminated, N);
    og.truncated = row(o->truncated, N);
    og.env_done = row(o->env_done, 1);
    og.dist_goal = row(o->dist_goal, N);
    og.info_flags = row(o->info_flags, N);
    og.global_state = row(o->global_state, 6 * N + 3);
    const int rc = launch(MODE_STEP, &pg, &sg, row(actions, 3 * N), row(action_mask, N), nullptr, &og,
                          hip_streams[g]);
    if (rc) return rc;
    lo += (size_t)group_envs[g];
  }
  return SWARM_OK;
}

int swarm_reset(const swarm_params_t* p, const swarm_state_t* s, const uint8_t* env_mask, const swarm_out_t* o,
                void* hip_stream) {
  return launch(MODE_RESET, p, s, nullptr, nullptr, env_mask, o, hip_stream);
}

int swarm_observe(const swarm_params_t* p, const swarm_state_t* s, const uint8_t* env_mask, const swarm_out_t* o,
                  void* hip_stream) {
  return launch(MODE_OBSERVE, p, s, nullptr, nullptr, env_mask, o, hip_stream);
}

int swarm_env_cfg_set(const swarm_params_t* p, const swarm_env_overrides_t* ov, const uint8_t* env_mask,
                      swarm_env_cfg_t* cfg, void* hip_stream) {
  KParams kp;
  const int rc = build_kparams(p, &kp, nullptr);
  if (rc) return rc;
  if (!ov) return fail(SWARM_ENULL, "overrides is NULL");
  if (kp.E == 0) return SWARM_OK;
  if (!cfg) return fail(SWARM_ENULL, "env_cfg is NULL");
  EnvCfgBase b;
  b.E = kp.E;
  b.M = kp.M;
  b.max_steps = p->max_steps;
  b.world_size = p->world_size;
  b.dt = p->dt;
  b.max_speed = p->max_speed;
  b.max_accel = p->max_accel;
  b.obstacle_radius = p->obstacle_radius;
  b.collision_radius = p->collision_radius;
  b.drone_contact_radius = p->drone_contact_radius;
  hipLaunchKernelGGL(env_cfg_set_kernel, dim3((kp.E + 255) / 256), dim3(256), 0, (hipStream_t)hip_stream, b, *ov,
                     env_mask, cfg);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(SWARM_EHIP, "kernel launch: %s", hipGetErrorString(e));
  return SWARM_OK;
}

}  // extern "C"
#endif  // SWARM_HAS_HOST
