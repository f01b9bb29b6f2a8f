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
//     error, path efficiency, reward, steps} is appended (vector atomic on the record counter);
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

constexpr int EVAL_THREADS = 64;
constexpr int EVAL_MAX_N = 1024;

__device__ __forceinline__ float norm1d(float x, float y, float z) {
  const float xx = x * x, yy = y * y, zz = z * z;
  return __builtin_sqrtf((float)(((double)xx + (double)yy) + (double)zz));  // IEEE sqrt
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
__device__ void begin_env(const EvalArgs& a, int e, int t) {
  const swarm_eval_t& v = a.ev;
  for (int i = t; i < a.N; i += EVAL_THREADS) {
    const size_t r = (size_t)e * a.N + i;
    const float* o = a.obs + r * a.D;
    const float px = o[0], py = o[1], pz = o[2];
    v.start[3 * r] = px; v.start[3 * r + 1] = py; v.start[3 * r + 2] = pz;
    v.goal[3 * r] = px + o[6]; v.goal[3 * r + 1] = py + o[7]; v.goal[3 * r + 2] = pz + o[8];
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

__global__ void __launch_bounds__(EVAL_THREADS) eval_begin_kernel(const EvalArgs a) {
  const int e = blockIdx.x;
  if (a.env_mask && !a.env_mask[e]) return;
  begin_env(a, e, threadIdx.x);
}

__global__ void __launch_bounds__(EVAL_THREADS) eval_update_kernel(const EvalArgs a) {
  __shared__ float4 pos[EVAL_MAX_N];  // agents with an observation this step (x, y, z, has)
  const int e = blockIdx.x;
  const int t = threadIdx.x;
  const swarm_eval_t& v = a.ev;
  const uint8_t status = v.status[e];  // uniform
  if (!(status & SWARM_EVAL_LIVE)) return;
  const uint8_t done = a.env_done[e];
  // ---- per-agent votes and the observed positions
  double rsum = 0.0;
  int n_st = 0, n_obs = 0, coll = 0, not_reached = 0;
  for (int i = t; i < a.N; i += EVAL_THREADS) {
    const size_t r = (size_t)e * a.N + i;
    const uint8_t fl = a.info_flags[r];
    if (fl & SWARM_AGENT_STEPPED) {
      rsum += (double)a.reward[r];
      ++n_st;
    }
    const bool has = (fl & SWARM_AGENT_HAS_OBS) != 0;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (has) {
      const float* o = a.obs + r * a.D;
      p = make_float4(o[0], o[1], o[2], 1.f);
      ++n_obs;
      coll |= (fl & SWARM_AGENT_COLLISION) ? 1 : 0;
      not_reached |= (fl & SWARM_AGENT_REACHED) ? 0 : 1;
      v.traveled[r] += (double)norm1d(v.last[3 * r] - p.x, v.last[3 * r + 1] - p.y, v.last[3 * r + 2] - p.z);
      v.last[3 * r] = p.x; v.last[3 * r + 1] = p.y; v.last[3 * r + 2] = p.z;
    }
    pos[i] = p;
  }
  __syncthreads();
  rsum = wave_sum(rsum);
  n_st = wave_sum_i(n_st);
  n_obs = wave_sum_i(n_obs);
  coll = __any(coll) ? 1 : 0;
  not_reached = __any(not_reached) ? 1 : 0;
  // ---- formation error of the observed set (evaluate_protocol.py:103-116)
  double fe = 0.0;
  if (n_obs > 1) {
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
  int steps = 0, reached = -1;
  double ep_reward = 0.0, fe_sum = 0.0;
  if (t == 0) {
    ep_reward = v.ep_reward[e] + (n_st > 0 ? rsum / (double)n_st : 0.0);
    fe_sum = v.fe_sum[e] + fe;
    steps = v.ep_steps[e] + 1;
    reached = v.reached_step[e];
    if (!not_reached && reached < 0) reached = steps;
    v.ep_reward[e] = ep_reward;
    v.fe_sum[e] = fe_sum;
    v.ep_steps[e] = steps;
    v.reached_step[e] = reached;
    if (coll) v.status[e] = status | SWARM_EVAL_COLLIDED;
  }
  if (!(done & (SWARM_ENV_TERMINATED | SWARM_ENV_TRUNCATED))) return;
  // ---- episode end: path efficiency over every agent, one record
  double pe = 0.0;
  for (int i = t; i < a.N; i += EVAL_THREADS) {
    const size_t r = (size_t)e * a.N + i;
    const float straight = norm1d(v.start[3 * r] - v.goal[3 * r], v.start[3 * r + 1] - v.goal[3 * r + 1],
                                  v.start[3 * r + 2] - v.goal[3 * r + 2]);
    const double tr = v.traveled[r];
    pe += tr > 1e-8 ? (double)straight / tr : 0.0;
  }
  pe = wave_sum(pe) / (double)a.N;
  if (t == 0) {
    const bool collided = coll || (status & SWARM_EVAL_COLLIDED);
    const unsigned k = atomicAdd(v.count, 1u);
    if (k < (unsigned)v.capacity) {
      double* rec = v.records + (size_t)k * SWARM_EVAL_RECORD;
      rec[0] = (double)(a.env_offset + e);  // global env index
      rec[1] = (!collided && reached >= 0) ? 1.0 : 0.0;
      rec[2] = collided ? 0.0 : 1.0;
      rec[3] = reached >= 0 ? (double)reached : __builtin_nan("");
      rec[4] = fe_sum / (double)steps;
      rec[5] = pe;
      rec[6] = ep_reward;
      rec[7] = (double)steps;
    }
    v.status[e] = 0;
  }
  if (done & SWARM_ENV_RESET) {  // auto-reset in the same launch: the next episode starts now
    __syncthreads();
    begin_env(a, e, t);
  }
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
  if (ev->capacity < 0) return efail(SWARM_EINVAL, "capacity < 0");
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
  hipLaunchKernelGGL(eval_begin_kernel, dim3(a.E), dim3(EVAL_THREADS), 0, (hipStream_t)hip_stream, a);
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
  hipLaunchKernelGGL(eval_update_kernel, dim3(a.E), dim3(EVAL_THREADS), 0, (hipStream_t)hip_stream, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? SWARM_OK : efail(SWARM_EHIP, "eval_update launch: %s", hipGetErrorString(e));
}

const char* swarm_eval_last_error(void) { return g_eerr; }

}  // extern "C"
