// swarm_eval.hip — on-device evaluation metrics for E envs.
//
// The reference evaluates a policy episode by episode on the host
// (scripts/evaluate_protocol.py:237-331 `_run_single_episode_multi_agent`, :103-116 formation
// error, :334-350 `_aggregate`), reading the dict outputs of DroneSwarmEnv.step.  Here the same
// per-episode quantities are accumulated on the device from the step kernel's dense outputs,
// one 64-lane workgroup per env (lane = agent, strided for N > 64), after every step launch:
//   * episode reward   += mean of the rewards of the agents stepped (the rewards dict),
//   * positions of the agents with an observation (obs[0:3]): path length += |last - p|,
//     formation error of that set (mean over agents of mean_j |d_ij - d*|),
//   * collision / all-reached votes from those agents' infos (none on the terminal step, whose
//     dict holds no observations: the all-reached test then passes vacuously — the
//     reference's behaviour, kept),
//   * at the episode's end one record {env, success, collision-free, time-to-goal, formation
//     error, path efficiency, reward, steps, update} is appended to one of 64 record segments
//     (vector atomic on that segment's counter);
//     an env auto-reset in the same launch starts its next episode from the new observations.
// Distances follow the reference's float(np.linalg.norm(a - b)) of float32 vectors (sdot: f32
// products, f64 sum, f32 sqrt); sums are f64.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include "swarm_mi355x.h"

#pragma clang fp contract(off)

namespace {

constexpr int EVAL_THREADS = 64;   // one wave per env
constexpr int EVAL_WG_ENVS = 4;    // independent waves per workgroup: a quarter of the workgroups
                                   // to dispatch (8192 one-wave workgroups cost the dispatcher ~4 us)
constexpr int EVAL_MAX_N = 1024;

__device__ __forceinline__ float norm1d(float x, float y, float z) {
  const float xx = x * x, yy = y * y, zz = z * z;
  return __builtin_sqrtf((float)(((double)xx + (double)yy) + (double)zz));  // IEEE sqrt
}

// The same float as norm1d, with the correctly rounded square root as swarm_kernel.hip's
// sqrt_rn (v_sqrt_f32 within 1 ulp + one correction step; OCML's scaling path below 2^-96).
__device__ __forceinline__ float norm1d_fast(float x, float y, float z) {
  const float xx = x * x, yy = y * y, zz = z * z;
  const float s = (float)(((double)xx + (double)yy) + (double)zz);
  if (__builtin_expect(__ballot(!(s >= 0x1p-96f || s == 0.0f)) != 0, 0)) return __builtin_sqrtf(s);
  float r = __builtin_amdgcn_sqrtf(s);
  const float rm = __uint_as_float(__float_as_uint(r) - 1u), rp = __uint_as_float(__float_as_uint(r) + 1u);
  const float em = __builtin_fmaf(-rm, r, s), ep = __builtin_fmaf(-rp, r, s);
  r = (em <= 0.0f) ? rm : r;
  r = (ep > 0.0f) ? rp : r;
  return r;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Row k of segment seg's record block: block (seg - seg_base) mod 64 of `segments` blocks of
// capacity / segments rows each; NULL once the block is full (or for a segment outside the
// tracker's live set, which no env of it maps to)
__device__ __forceinline__ double* record_slot(const swarm_eval_t& v, unsigned seg, unsigned k) {
  const unsigned nseg = v.segments > 0 ? (unsigned)v.segments : (unsigned)SWARM_EVAL_SEGMENTS;
  const unsigned b = (seg + SWARM_EVAL_SEGMENTS - (unsigned)v.seg_base % SWARM_EVAL_SEGMENTS) % SWARM_EVAL_SEGMENTS;
  const unsigned cap = (unsigned)v.capacity / nseg;
  if (b >= nseg || k >= cap) return nullptr;
  return v.records + ((size_t)b * cap + k) * SWARM_EVAL_RECORD;
}

struct EvalArgs {
  int E, N, D;
  long long env_offset;
  double spacing;
  swarm_eval_t ev;
  const float* obs;
  const float* reward;
  const uint8_t* info_flags;
  const uint8_t* env_done;
  const uint8_t* env_mask;
};

// Episode start of env e from its current observation rows (every agent).
// obs[0:3] and obs[6:9] of row r (agent i of env e): from the state (contiguous; bitwise the
// same floats: the step writes px and gx - px) when given, else from the obs row
__device__ __forceinline__ void obs_pos(const EvalArgs& a, size_t r, float& x, float& y, float& z) {
  if (a.ev.state_pos) {
    x = a.ev.state_pos[3 * r]; y = a.ev.state_pos[3 * r + 1]; z = a.ev.state_pos[3 * r + 2];
  } else {
    const float* o = a.obs + r * a.D;
    x = o[0]; y = o[1]; z = o[2];
  }
}
__device__ __forceinline__ void obs_goal_vec(const EvalArgs& a, int e, size_t r, float px, float py, float pz,
                                             float& x, float& y, float& z) {
  if (a.ev.state_pos) {
    x = a.ev.state_goal[3 * e] - px; y = a.ev.state_goal[3 * e + 1] - py; z = a.ev.state_goal[3 * e + 2] - pz;
  } else {
    const float* o = a.obs + r * a.D;
    x = o[6]; y = o[7]; z = o[8];
  }
}

__device__ void begin_env(const EvalArgs& a, int e, int t) {
  const swarm_eval_t& v = a.ev;
  for (int i = t; i < a.N; i += EVAL_THREADS) {
    const size_t r = (size_t)e * a.N + i;
    float px, py, pz, rx, ry, rz;
    obs_pos(a, r, px, py, pz);
    obs_goal_vec(a, e, r, px, py, pz, rx, ry, rz);
    v.start[3 * r] = px; v.start[3 * r + 1] = py; v.start[3 * r + 2] = pz;
    v.goal[3 * r] = px + rx; v.goal[3 * r + 1] = py + ry; v.goal[3 * r + 2] = pz + rz;
    v.last[3 * r] = px; v.last[3 * r + 1] = py; v.last[3 * r + 2] = pz;
    v.traveled[r] = 0.0;
  }
  if (t == 0) {
    v.ep_reward[e] = 0.0;
    v.fe_sum[e] = 0.0;
    v.ep_steps[e] = 0;
    v.reached_step[e] = -1;
    v.status[e] = SWARM_EVAL_LIVE;
  }
}

__global__ void __launch_bounds__(EVAL_THREADS * EVAL_WG_ENVS) eval_begin_kernel(const EvalArgs a) {
  const int e = blockIdx.x * EVAL_WG_ENVS + (threadIdx.x >> 6);
  if (e >= a.E || (a.env_mask && !a.env_mask[e])) return;
  begin_env(a, e, threadIdx.x & 63);
}

// One wave per env.  Every global load of the step is issued in one batch at the top (the env's
// accumulators, the agents' flags / reward / observed position / last position / path length,
// and — known from env_done before anything else — the start / goal rows of an ending episode and
// the goal columns of a restarting one): the kernel is latency-bound (all 8192 waves of the
// headline batch are resident at once), so the chain of dependent memory round trips, not the
// bytes, sets its time.  A restart writes the new episode's start rows in the same pass.
__global__ void __launch_bounds__(EVAL_THREADS * EVAL_WG_ENVS) eval_update_kernel(const EvalArgs a) {
  // agents with an observation this step (x, y, z, has); N float4 of dynamic LDS, so that the
  // LDS of a small swarm does not cap the waves per CU (a static EVAL_MAX_N array did: 16 KB)
  extern __shared__ float4 pos_all[];
  const int w = threadIdx.x >> 6;
  const int e = blockIdx.x * EVAL_WG_ENVS + w;
  const int t = threadIdx.x & 63;
  if (e >= a.E) return;  // whole wave
  float4* pos = pos_all + (size_t)w * a.N;  // this wave's slice: waves never share LDS
  const swarm_eval_t& v = a.ev;
  const uint8_t status = v.status[e];  // uniform
  const uint8_t done = a.env_done[e];
  const double ep_reward0 = v.ep_reward[e];
  const double fe_sum0 = v.fe_sum[e];
  const int steps0 = v.ep_steps[e];
  const int reached0 = v.reached_step[e];
  if (!(status & SWARM_EVAL_LIVE)) return;
  const bool ends = (done & (SWARM_ENV_TERMINATED | SWARM_ENV_TRUNCATED)) != 0;
  const bool restarts = ends && (done & SWARM_ENV_RESET) != 0;
  // SWARM_EVAL_STEP_FUSED: the step launch (out.eval) already added this step's reward, steps,
  // reached step, collision vote and path lengths (swarm_kernel.hip s64_env, the same arithmetic):
  // only the formation error and the episode ends are left here
  const bool fused = (v.flags & SWARM_EVAL_STEP_FUSED) != 0;
  // ---- per-agent votes, path length, observed positions; path efficiency and the next
  // episode's start rows when the episode ends here
  double rsum = 0.0, pe = 0.0;
  int n_st = 0, n_obs = 0, coll = 0, not_reached = 0;
  for (int i = t; i < a.N; i += EVAL_THREADS) {
    const size_t r = (size_t)e * a.N + i;
    const uint8_t fl = a.info_flags[r];
    float ox, oy, oz;
    obs_pos(a, r, ox, oy, oz);
    if (fused) {  // observed positions for the formation error; the ended episode's path efficiency
      const bool has = (fl & SWARM_AGENT_HAS_OBS) != 0;
      n_obs += has ? 1 : 0;
      pos[i] = has ? make_float4(ox, oy, oz, 1.f) : make_float4(0.f, 0.f, 0.f, 0.f);
      if (ends) {
        const double tr = v.traveled[r];
        const float straight = norm1d(v.start[3 * r] - v.goal[3 * r], v.start[3 * r + 1] - v.goal[3 * r + 1],
                                      v.start[3 * r + 2] - v.goal[3 * r + 2]);
        pe += tr > 1e-8 ? (double)straight / tr : 0.0;
      }
      if (restarts) {
        float rx, ry, rz;
        obs_goal_vec(a, e, r, ox, oy, oz, rx, ry, rz);
        v.start[3 * r] = ox; v.start[3 * r + 1] = oy; v.start[3 * r + 2] = oz;
        v.goal[3 * r] = ox + rx; v.goal[3 * r + 1] = oy + ry; v.goal[3 * r + 2] = oz + rz;
        v.traveled[r] = 0.0;
      }
      continue;
    }
    const float rw = a.reward[r];
    const float lx = v.last[3 * r], ly = v.last[3 * r + 1], lz = v.last[3 * r + 2];
    double tr = v.traveled[r];
    float sx = 0.f, sy = 0.f, sz = 0.f, gx = 0.f, gy = 0.f, gz = 0.f, rx = 0.f, ry = 0.f, rz = 0.f;
    if (ends) {
      sx = v.start[3 * r]; sy = v.start[3 * r + 1]; sz = v.start[3 * r + 2];
      gx = v.goal[3 * r]; gy = v.goal[3 * r + 1]; gz = v.goal[3 * r + 2];
    }
    if (restarts) obs_goal_vec(a, e, r, ox, oy, oz, rx, ry, rz);
    if (fl & SWARM_AGENT_STEPPED) {
      rsum += (double)rw;
      ++n_st;
    }
    const bool has = (fl & SWARM_AGENT_HAS_OBS) != 0;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (has) {
      p = make_float4(ox, oy, oz, 1.f);
      ++n_obs;
      coll |= (fl & SWARM_AGENT_COLLISION) ? 1 : 0;
      not_reached |= (fl & SWARM_AGENT_REACHED) ? 0 : 1;
      tr += (double)norm1d(lx - ox, ly - oy, lz - oz);
    }
    pos[i] = p;
    if (ends) {
      const float straight = norm1d(sx - gx, sy - gy, sz - gz);
      pe += tr > 1e-8 ? (double)straight / tr : 0.0;
    }
    if (restarts) {  // the obs rows are the new episode's first observation (every agent)
      v.start[3 * r] = ox; v.start[3 * r + 1] = oy; v.start[3 * r + 2] = oz;
      v.goal[3 * r] = ox + rx; v.goal[3 * r + 1] = oy + ry; v.goal[3 * r + 2] = oz + rz;
      v.last[3 * r] = ox; v.last[3 * r + 1] = oy; v.last[3 * r + 2] = oz;
      v.traveled[r] = 0.0;
    } else if (has) {
      v.traveled[r] = tr;
      v.last[3 * r] = ox; v.last[3 * r + 1] = oy; v.last[3 * r + 2] = oz;
    }
  }
  // LDS ordering within one wave: a compiler fence around the wave barrier suffices
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  rsum = wave_sum(rsum);
  n_st = wave_sum_i(n_st);
  n_obs = wave_sum_i(n_obs);
  coll = __any(coll) ? 1 : 0;
  not_reached = __any(not_reached) ? 1 : 0;
  // ---- formation error of the observed set (evaluate_protocol.py:103-116)
  double fe = 0.0;
  if (n_obs > 1 && a.N == EVAL_THREADS) {
    // one drone per lane: symmetric rotations.  At rotation r lane t measures the pair
    // (t, t+r); r = 1..31 covers every unordered pair except the 32 opposite ones once, r = 32
    // covers those twice (lanes t and t+32).  Distances are symmetric bit for bit (|a-b| = |b-a|
    // per component) and every observed drone divides by the same n_obs - 1, so the reference's
    // mean over drones of the mean over partners is (2 S_{r<32} + S_{32}) / (n (n - 1)): the same
    // terms, each measured once; only the f64 summation order differs (np.mean's pairwise order
    // is not reproduced: 1e-9 relative).
    const float4 p = pos[t];
    double s_a = 0.0, s_b = 0.0;  // two chains of dependent f64 adds instead of one
    if (n_obs == EVAL_THREADS) {  // every drone observed (the common step): no pair masks
#pragma unroll 8
      for (int r = 1; r < 32; ++r) {
        const float4 q = pos[(t + r) & (EVAL_THREADS - 1)];
        const double term = fabs((double)norm1d_fast(p.x - q.x, p.y - q.y, p.z - q.z) - a.spacing);
        if (r & 1) s_a += term; else s_b += term;
      }
    } else {
#pragma unroll 8
      for (int r = 1; r < 32; ++r) {
        const float4 q = pos[(t + r) & (EVAL_THREADS - 1)];
        const float d = norm1d_fast(p.x - q.x, p.y - q.y, p.z - q.z);
        const double term = (p.w != 0.f && q.w != 0.f) ? fabs((double)d - a.spacing) : 0.0;
        if (r & 1) s_a += term; else s_b += term;
      }
    }
    const float4 q = pos[(t + 32) & (EVAL_THREADS - 1)];
    const float d = norm1d_fast(p.x - q.x, p.y - q.y, p.z - q.z);
    const double opp = (p.w != 0.f && q.w != 0.f) ? fabs((double)d - a.spacing) : 0.0;
    fe = wave_sum(2.0 * (s_a + s_b) + opp) / ((double)n_obs * (double)(n_obs - 1));
  } else if (n_obs > 1 && a.N <= EVAL_THREADS / 2) {
    // small swarms (config 2: N = 16): P = 64 / next_pow2(N) lanes per drone, lane (i, q) takes
    // partners j = q, q + P, ... — every ordered pair once, spread over all 64 lanes instead of a
    // serial N - 1 chain on N lanes; every observed drone divides by the same n - 1, so the mean of
    // means is the pair sum over n (n - 1) (1e-9 relative: only the f64 summation order differs)
    int np2 = 1;
    while (np2 < a.N) np2 <<= 1;
    const int P = EVAL_THREADS / np2;
    const int i = t / P, q = t - i * P;
    double acc = 0.0;
    if (i < a.N) {
      const float4 p = pos[i];
      if (p.w != 0.f) {
        for (int j = q; j < a.N; j += P) {
          const float4 o = pos[j];
          if (j == i || o.w == 0.f) continue;
          acc += fabs((double)norm1d(p.x - o.x, p.y - o.y, p.z - o.z) - a.spacing);
        }
      }
    }
    fe = wave_sum(acc) / ((double)n_obs * (double)(n_obs - 1));
  } else if (n_obs > 1) {
    double acc = 0.0;
    for (int i = t; i < a.N; i += EVAL_THREADS) {
      const float4 p = pos[i];
      if (p.w == 0.f) continue;
      double s = 0.0;
      for (int j = 0; j < a.N; ++j) {
        const float4 q = pos[j];
        if (j == i || q.w == 0.f) continue;
        s += fabs((double)norm1d(p.x - q.x, p.y - q.y, p.z - q.z) - a.spacing);
      }
      acc += s / (double)(n_obs - 1);
    }
    fe = wave_sum(acc) / (double)n_obs;
  }
  if (ends) pe = wave_sum(pe) / (double)a.N;
  if (t != 0) return;
  const double ep_reward = fused ? ep_reward0 : ep_reward0 + (n_st > 0 ? rsum / (double)n_st : 0.0);
  const double fe_sum = fe_sum0 + fe;
  const int steps = fused ? steps0 : steps0 + 1;
  int reached = reached0;
  if (!fused && !not_reached && reached < 0) reached = steps;
  if (!ends) {
    v.fe_sum[e] = fe_sum;
    if (fused) return;
    v.ep_reward[e] = ep_reward;
    v.ep_steps[e] = steps;
    v.reached_step[e] = reached;
    if (coll) v.status[e] = status | SWARM_EVAL_COLLIDED;
    return;
  }
  // ---- episode end: one record; a restarting env opens its next episode
  const bool collided = coll || (status & SWARM_EVAL_COLLIDED);
  const long long genv = a.env_offset + e;
  const unsigned seg = (unsigned)(genv % SWARM_EVAL_SEGMENTS);
  const unsigned k = atomicAdd(v.count + seg, 1u);
  double* rec = record_slot(v, seg, k);
  if (rec) {
    rec[0] = (double)genv;  // global env index
    rec[1] = (!collided && reached >= 0) ? 1.0 : 0.0;
    rec[2] = collided ? 0.0 : 1.0;
    rec[3] = reached >= 0 ? (double)reached : __builtin_nan("");
    rec[4] = fe_sum / (double)steps;
    rec[5] = pe;
    rec[6] = ep_reward;
    rec[7] = (double)steps;
    rec[8] = (double)v.update_index;
  }
  v.ep_reward[e] = 0.0;
  v.fe_sum[e] = 0.0;
  v.ep_steps[e] = 0;
  v.reached_step[e] = -1;
  v.status[e] = restarts ? SWARM_EVAL_LIVE : 0;
}

// Single-agent protocol (evaluate_protocol.py:193-234): one thread per env of single-drone envs.
// The step ran without auto-reset, so the state still holds the terminal step's position; the
// terminal step's info (collision, reached_goal) counts, which the swarm protocol never sees.
__global__ void __launch_bounds__(256) eval_single_update_kernel(const EvalArgs a, uint8_t* __restrict__ reset_mask) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= a.E) return;
  const swarm_eval_t& v = a.ev;
  const uint8_t status = v.status[e];
  const uint8_t done = a.env_done[e];
  const uint8_t fl = a.info_flags[e];
  const float rw = a.reward[e];
  const float px = v.state_pos[3 * e], py = v.state_pos[3 * e + 1], pz = v.state_pos[3 * e + 2];
  const float lx = v.last[3 * e], ly = v.last[3 * e + 1], lz = v.last[3 * e + 2];
  const bool ends = (done & (SWARM_ENV_TERMINATED | SWARM_ENV_TRUNCATED)) != 0;
  reset_mask[e] = (ends && (status & SWARM_EVAL_LIVE)) ? 1 : 0;
  if (!(status & SWARM_EVAL_LIVE) || !(fl & SWARM_AGENT_STEPPED)) return;
  const double ep_reward = v.ep_reward[e] + (double)rw;  // episode_reward += float(reward)
  const double tr = v.traveled[e] + (double)norm1d(lx - px, ly - py, lz - pz);  // _distance(last, pos)
  const int steps = v.ep_steps[e] + 1;
  int reached = v.reached_step[e];
  if ((fl & SWARM_AGENT_REACHED) && reached < 0) reached = steps;
  const bool collided = (status & SWARM_EVAL_COLLIDED) || (fl & SWARM_AGENT_COLLISION);
  if (!ends) {
    v.ep_reward[e] = ep_reward;
    v.traveled[e] = tr;
    v.ep_steps[e] = steps;
    v.reached_step[e] = reached;
    v.last[3 * e] = px; v.last[3 * e + 1] = py; v.last[3 * e + 2] = pz;
    if (collided) v.status[e] = status | SWARM_EVAL_COLLIDED;
    return;
  }
  const float straight = norm1d(v.start[3 * e] - v.goal[3 * e], v.start[3 * e + 1] - v.goal[3 * e + 1],
                                v.start[3 * e + 2] - v.goal[3 * e + 2]);
  const long long genv = a.env_offset + e;
  const unsigned seg = (unsigned)(genv % SWARM_EVAL_SEGMENTS);
  const unsigned k = atomicAdd(v.count + seg, 1u);
  double* rec = record_slot(v, seg, k);
  if (rec) {
    rec[0] = (double)genv;
    rec[1] = (!collided && reached >= 0) ? 1.0 : 0.0;
    rec[2] = collided ? 0.0 : 1.0;
    rec[3] = reached >= 0 ? (double)reached : __builtin_nan("");
    rec[4] = 0.0;  // formation_error: one agent
    rec[5] = tr > 1e-8 ? (double)straight / tr : 0.0;
    rec[6] = ep_reward;
    rec[7] = (double)steps;
    rec[8] = (double)v.update_index;
  }
  v.status[e] = 0;  // reopened by swarm_eval_begin after the caller's reset
}

thread_local char g_eerr[256] = "";
int efail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_eerr, sizeof(g_eerr), fmt, ap);
  va_end(ap);
  return code;
}

int make_args(const swarm_params_t* p, const swarm_eval_t* ev, const swarm_out_t* o, EvalArgs* a) {
  if (!p || !ev || !o) return efail(SWARM_ENULL, "params/eval/out is NULL");
  if (p->abi_version != SWARM_ABI_VERSION) return efail(SWARM_EINVAL, "abi_version mismatch");
  if (p->num_envs < 0) return efail(SWARM_EINVAL, "num_envs < 0");
  if (p->num_drones < 1 || p->num_drones > EVAL_MAX_N) return efail(SWARM_ELIMIT, "num_drones must be in [1, %d]", EVAL_MAX_N);
  if (!o->obs) return efail(SWARM_ENULL, "out.obs is NULL");
  if (!ev->ep_reward || !ev->ep_steps || !ev->reached_step || !ev->status || !ev->fe_sum || !ev->start || !ev->goal ||
      !ev->last || !ev->traveled || !ev->records || !ev->count)
    return efail(SWARM_ENULL, "an eval state buffer is NULL");
  if ((ev->state_pos == nullptr) != (ev->state_goal == nullptr))
    return efail(SWARM_EINVAL, "state_pos and state_goal go together");
  if (ev->flags & ~SWARM_EVAL_STEP_FUSED) return efail(SWARM_EINVAL, "unknown eval flags 0x%x", (unsigned)ev->flags);
  if (ev->segments < 0 || ev->segments > SWARM_EVAL_SEGMENTS || ev->seg_base < 0)
    return efail(SWARM_EINVAL, "segments must be in [0, %d] and seg_base >= 0", SWARM_EVAL_SEGMENTS);
  const int nseg = ev->segments > 0 ? ev->segments : SWARM_EVAL_SEGMENTS;
  if (ev->capacity < 0 || ev->capacity % nseg != 0)
    return efail(SWARM_EINVAL, "capacity must be a non-negative multiple of segments (%d)", nseg);
  a->E = p->num_envs;
  a->N = p->num_drones;
  a->D = 9 + 4 * (p->neighbor_k > 0 ? p->neighbor_k : 0) + 4 * (p->sensed_obstacles > 0 ? p->sensed_obstacles : 0);
  a->spacing = p->desired_spacing;
  a->env_offset = p->env_offset;
  a->ev = *ev;
  a->obs = o->obs;
  a->reward = o->reward;
  a->info_flags = o->info_flags;
  a->env_done = o->env_done;
  a->env_mask = nullptr;
  return SWARM_OK;
}

}  // namespace

extern "C" {

int swarm_eval_begin(const swarm_params_t* p, const swarm_eval_t* ev, const swarm_out_t* o, const uint8_t* env_mask,
                     void* hip_stream) {
  EvalArgs a;
  const int rc = make_args(p, ev, o, &a);
  if (rc) return rc;
  if (a.E == 0) return SWARM_OK;
  a.env_mask = env_mask;
  hipLaunchKernelGGL(eval_begin_kernel, dim3((a.E + EVAL_WG_ENVS - 1) / EVAL_WG_ENVS), dim3(EVAL_THREADS * EVAL_WG_ENVS),
                     0, (hipStream_t)hip_stream, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? SWARM_OK : efail(SWARM_EHIP, "eval_begin launch: %s", hipGetErrorString(e));
}

int swarm_eval_update(const swarm_params_t* p, const swarm_eval_t* ev, const swarm_out_t* o, void* hip_stream) {
  EvalArgs a;
  const int rc = make_args(p, ev, o, &a);
  if (rc) return rc;
  if (!o->reward || !o->info_flags || !o->env_done)
    return efail(SWARM_ENULL, "out.reward/info_flags/env_done required (build the env with infos)");
  if (a.E == 0) return SWARM_OK;
  // SWARM_EVAL_STEP_FUSED: the step launches (out.eval) did this update's work already
  if (ev->flags & SWARM_EVAL_STEP_FUSED) return SWARM_OK;
  hipLaunchKernelGGL(eval_update_kernel, dim3((a.E + EVAL_WG_ENVS - 1) / EVAL_WG_ENVS), dim3(EVAL_THREADS * EVAL_WG_ENVS),
                     (unsigned)(EVAL_WG_ENVS * a.N * sizeof(float4)),
                     (hipStream_t)hip_stream, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? SWARM_OK : efail(SWARM_EHIP, "eval_update launch: %s", hipGetErrorString(e));
}

int swarm_eval_single_update(const swarm_params_t* p, const swarm_eval_t* ev, const swarm_out_t* o,
                             uint8_t* reset_mask, void* hip_stream) {
  EvalArgs a;
  const int rc = make_args(p, ev, o, &a);
  if (rc) return rc;
  if (p->num_drones != 1 || p->neighbor_k > 0)
    return efail(SWARM_EINVAL, "the single-agent protocol needs num_drones 1 and neighbor_k 0 (SingleDroneEnv)");
  if (p->auto_reset) return efail(SWARM_EINVAL, "the single-agent protocol needs auto_reset 0 (terminal positions)");
  if (!ev->state_pos) return efail(SWARM_ENULL, "state_pos / state_goal are required by the single-agent protocol");
  if (!o->reward || !o->info_flags || !o->env_done)
    return efail(SWARM_ENULL, "out.reward/info_flags/env_done required (build the env with infos)");
  if (!reset_mask) return efail(SWARM_ENULL, "reset_mask is NULL");
  if (a.E == 0) return SWARM_OK;
  hipLaunchKernelGGL(eval_single_update_kernel, dim3((a.E + 255) / 256), dim3(256), 0, (hipStream_t)hip_stream, a,
                     reset_mask);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? SWARM_OK : efail(SWARM_EHIP, "eval_single_update launch: %s", hipGetErrorString(e));
}

const char* swarm_eval_last_error(void) { return g_eerr; }

}  // extern "C"
