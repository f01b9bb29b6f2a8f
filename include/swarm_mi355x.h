/*
 * swarm_mi355x.h — C-ABI of the MI355X-native vectorised drone-swarm step/observe/reward path.
 *
 * One call steps E independent swarm envs of N drones on the GPU (gfx950).  It replaces the
 * reference's per-env Python hot path:
 *
 *   swarm_step    <- DroneSwarmEnv.step            src/swarm_marl/envs/drone_swarm_env.py:92-174
 *                    (+ _clip_speed :179-183, _collision_mask :185-208,
 *                     _formation_penalties :210-224, _build_obs :226-243,
 *                     _nearest_neighbor_features :245-271, _nearest_obstacle_features :273-291,
 *                     _global_state :293-302)
 *                 <- DronePhysicsEnv.step          src/swarm_marl/envs/drone_physics_env.py:279-419
 *                    (point-mass restatement of the PyBullet force/substep loop :320-360,
 *                     _get_obs :421-462, _get_infos :540-583)
 *   swarm_reset   <- DroneSwarmEnv.reset           drone_swarm_env.py:65-90 (device RNG draws;
 *                    the seeded NumPy-stream reset stays on the host and uses swarm_observe)
 *                 <- DronePhysicsEnv.reset         drone_physics_env.py:174-263
 *   swarm_observe <- the observation/info half of reset(): drone_swarm_env.py:82-90
 *                    (_build_obs for every agent, distance_to_goal, global_state)
 *
 * Conventions
 *  - Every buffer is device memory owned by the caller (PyTorch tensors in the Python host
 *    package).  All buffers are dense, C-contiguous, and must not overlap each other.
 *  - Calls are asynchronous on `hip_stream` (a hipStream_t; NULL = the null stream).  No
 *    allocation, no host synchronisation, no exceptions cross the ABI: 0 on success, a negative
 *    SWARM_E* code otherwise; swarm_last_error() gives a thread-local message.
 *  - Reentrant for distinct state/out buffers.
 */
#ifndef SWARM_MI355X_H
#define SWARM_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWARM_ABI_VERSION 5

/* error codes */
#define SWARM_OK 0
#define SWARM_EINVAL -1    /* bad argument / unsupported configuration */
#define SWARM_ENULL -2     /* required pointer is NULL */
#define SWARM_ELIMIT -3    /* size exceeds a documented limit (N, K, Ms, LDS budget) */
#define SWARM_EHIP -4      /* HIP launch / runtime error */

/* dynamics modes */
#define SWARM_DYN_KINEMATIC 0         /* DroneSwarmEnv Euler integrator (drone_swarm_env.py:103-117) */
#define SWARM_DYN_POINTMASS_PHYSICS 1 /* DronePhysicsEnv force model as a point mass (drone_physics_env.py:320-360) */

/* reward modes */
#define SWARM_REW_SWARM 0    /* progress + formation + goal + collision (drone_swarm_env.py:137-172) */
#define SWARM_REW_PHYSICS 1  /* -0.1*dist, -10 collision, +50 goal (drone_physics_env.py:374-417) */

/* kernel selection (swarm_params_t.kernel_path) */
#define SWARM_PATH_AUTO 0     /* specialised kernels where they apply (swarm_step64 for the headline shape) */
#define SWARM_PATH_GENERIC 1  /* always the generic swarm_kernel (A/B parity checks, diagnostics) */

/* kernel actually launched (swarm_launch_info_t.kernel_id) */
#define SWARM_KERNEL_GENERIC 0  /* swarm_kernel<KIND, DYN, KS, MSL, LM> */
#define SWARM_KERNEL_STEP64 1   /* swarm_step64_once: N = 64, K = 3, Ms = 4, 4 <= M <= 16, kinematic step;
                                   one wave per env, 4 envs per workgroup (physics: swarm_step64_phys_once) */
#define SWARM_KERNEL_STEP64_PERSISTENT 2  /* swarm_step64: the same step on a persistent grid of
                                   waves_per_simd waves per SIMD with per-XCD env queues
                                   (E > grid; needs state.work, else STEP64 is launched) */
#define SWARM_KERNEL_STEP16Q 3  /* swarm_step16q: N = 16, K = 3, Ms = 4, 4 <= M <= 16, kinematic step; one
                                   env per 64-lane wave, four lanes per drone (BASELINE config 2) */
#define SWARM_KERNEL_STEP256 4  /* swarm_step256: N = 256, K = 3, Ms = 4, 4 <= M <= 16, kinematic step; one
                                   env per 256-thread workgroup, every pair evaluated once (BASELINE config 5) */

/* env_done bits ([E] u8) */
#define SWARM_ENV_TERMINATED 1u  /* terminated["__all__"] */
#define SWARM_ENV_TRUNCATED 2u   /* truncated["__all__"] */
#define SWARM_ENV_RESET 4u       /* the env was auto-reset in this call; obs/state are the new episode's */

/* info_flags bits ([E,N] u8) */
#define SWARM_AGENT_STEPPED 1u    /* agent had a reward/terminated/truncated entry this step */
#define SWARM_AGENT_REACHED 2u    /* infos["reached_goal"] */
#define SWARM_AGENT_COLLISION 4u  /* infos["collision"] */
#define SWARM_AGENT_HAS_OBS 8u    /* obs/infos entry emitted by the dict API (continuing agent) */

/*
 * Environment parameters.  Field meaning follows DroneEnvConfig (src/swarm_marl/envs/common.py:7-25)
 * plus `num_drones` (drone_swarm_env.py:32-34); floating fields are the Python (double) values,
 * the library derives the float32 constants the reference's NumPy code actually compares against.
 */
typedef struct swarm_params {
  int32_t abi_version;       /* must be SWARM_ABI_VERSION */
  int32_t num_envs;          /* E (local shard) */
  int32_t num_drones;        /* N, 1..1024 */
  int32_t num_obstacles;     /* M >= 0 */
  int32_t sensed_obstacles;  /* Ms (<= 16 supported); <= 0 -> no obstacle block in obs */
  int32_t neighbor_k;        /* K (<= 16 supported); <= 0 -> no neighbour block in obs */
  int32_t max_steps;
  int32_t dynamics;          /* SWARM_DYN_* */
  int32_t reward_mode;       /* SWARM_REW_* */
  int32_t auto_reset;        /* swarm_step: reset envs whose episode ended, in-kernel (device RNG) */
  int32_t physics_substeps;  /* physics: int(dt*240) (drone_physics_env.py:323) */
  int32_t damping_law;       /* physics: 0 = btMultiBody -d*(1+|v|)*v (default), 1 = btRigidBody v*=(1-d)^h */
  int64_t env_offset;        /* global index of local env 0 (RNG key; sharding across ranks) */
  uint64_t seed;             /* device-RNG key */
  double world_size;
  double dt;
  double max_speed;
  double max_accel;
  double collision_radius;
  double goal_radius;
  double obstacle_radius;
  double desired_spacing;
  double reward_progress_scale;
  double reward_goal;
  double reward_collision;
  double reward_formation_scale;
  /* physics-mode constants (drone_physics_env.py:135,343; drone.urdf geometry) */
  double gravity;            /* -9.81 */
  double gravity_comp;       /* 9.5 */
  double substep_dt;         /* 1/240 */
  double drone_contact_radius;    /* contact approximation radius of the 0.3x0.3x0.05 box */
  double ground_contact_height;   /* z at or below which the box touches the plane */
  int32_t kernel_path;       /* SWARM_PATH_* (default AUTO) */
  int32_t waves_per_simd;    /* 0 (default): swarm_step64_once, one wave per env; 1..8: persistent
                                swarm_step64 grid of that many waves per SIMD (needs state.work) */
} swarm_params_t;

/* Per-env state, device SoA blocks (all dense, C-contiguous). */
typedef struct swarm_state {
  float* pos;          /* [E,N,3] */
  float* vel;          /* [E,N,3] */
  float* goal;         /* [E,3] */
  float* obstacles;    /* [E,M,3] (may be NULL iff M == 0) */
  uint8_t* active;     /* [E,N]  agent still in env.agents */
  int32_t* step_count; /* [E] */
  uint32_t* episode;   /* [E]  device-RNG episode counter (incremented by every device reset) */
  float* damping;      /* [E,N] physics linear damping (NULL allowed in kinematic mode) */
  uint32_t* work;      /* [SWARM_WORK_WORDS] env-queue heads of the persistent swarm_step64: zeroed
                          once by the caller, left zeroed by every call; NULL = one workgroup per
                          env.  Belongs to this state: concurrent calls need distinct buffers. */
  struct swarm_env_cfg* env_cfg;             /* [E] per-env parameters (NULL: every env uses
                                                swarm_params_t); see swarm_env_cfg_set */
  const struct swarm_env_cfg* env_cfg_next;  /* [E] parameters of each env's NEXT episode: a reset
                                                (auto or swarm_reset) copies it into env_cfg before
                                                drawing.  NULL: episodes keep env_cfg.  Needs env_cfg. */
} swarm_state_t;

/*
 * Per-env parameters (curriculum stages configs/curriculum_v1.yaml:9-60 and
 * domain randomisation configs/domain_randomization_v1.yaml:9-57 as per-env tensors).  One 64-B
 * record per env, derived on the device by swarm_env_cfg_set from per-env values exactly as the
 * library derives the uniform constants from swarm_params_t, so that an env with record r behaves
 * bit-for-bit like a launch whose swarm_params_t carries r's values.  N, K, Ms, rewards and radii
 * other than the obstacle radius stay uniform (they fix the tensor shapes or are not randomised).
 * With env_cfg set, swarm_step launches the generic kernel (the step64 specialisation assumes
 * uniform parameters).
 */
typedef struct swarm_env_cfg {
  float half_w;          /* (float)(world_size / 2)  world clip and reset draw bounds */
  float neg_half_w;      /* (float)(-world_size / 2) */
  float width_w;         /* (float)world_size */
  float dt;              /* kinematic integrator step (physics: substeps stay uniform) */
  float max_speed;
  float max_accel;
  float s_vmax;          /* largest s with sqrtf(s) <= (float)max_speed */
  float s_obst;          /* same for (float)(collision_radius + obstacle_radius) */
  float s_phys_obst;     /* same for (float)(obstacle_radius + drone_contact_radius) */
  int32_t max_steps;
  int32_t num_obstacles; /* active obstacles, 0..swarm_params_t.num_obstacles (the state keeps M
                            slots; slots >= num_obstacles are zero and ignored) */
  int32_t reserved;
  double max_speed_d;    /* max_speed as given (physics observation clamp) */
  double world_size;     /* as given (for readers) */
} swarm_env_cfg_t;

/* Per-env values for swarm_env_cfg_set: each pointer is a device array [E] or NULL (= the
 * swarm_params_t value for every env). */
typedef struct swarm_env_overrides {
  const double* world_size;
  const double* dt;
  const double* max_speed;
  const double* max_accel;
  const double* obstacle_radius;
  const int32_t* max_steps;
  const int32_t* num_obstacles;  /* clamped to [0, swarm_params_t.num_obstacles] */
} swarm_env_overrides_t;

#define SWARM_WORK_WORDS 256  /* 8 dequeue heads (one per XCD), one 128-B line each */

/* Outputs.  Optional pointers may be NULL. */
typedef struct swarm_out {
  float* obs;            /* [E,N,D], D = 9 + 4*max(K,0) + 4*max(Ms,0) */
  float* reward;         /* [E,N]   (0 for agents without a reward entry) */
  uint8_t* terminated;   /* [E,N] */
  uint8_t* truncated;    /* [E,N] */
  uint8_t* env_done;     /* [E]     SWARM_ENV_* bits */
  float* dist_goal;      /* [E,N]   optional: infos["distance_to_goal"] */
  uint8_t* info_flags;   /* [E,N]   optional: SWARM_AGENT_* bits */
  float* global_state;   /* [E,6N+3] optional: concat(pos, vel, goal) (drone_swarm_env.py:293-302) */
  const struct swarm_eval* eval;  /* optional HOST pointer to an eval tracker's state (swarm_eval_t,
                             its `flags` holding SWARM_EVAL_STEP_FUSED): the step accumulates the
                             evaluation protocol's per-step terms in its write-back — episode reward,
                             steps, first all-reached step, collision vote, path length — and
                             swarm_eval_update then adds only the formation error and closes the
                             ended episodes.  Kinematic swarm_step64 launches only (SWARM_KERNEL_STEP64
                             from swarm_query_launch, no env_cfg): other launches return SWARM_EINVAL */
} swarm_out_t;

/* Launch geometry actually used (for tests / profiling). */
typedef struct swarm_launch_info {
  int32_t threads_per_block;
  int32_t envs_per_block;
  int32_t lanes_per_env;
  int32_t blocks;
  int32_t lds_bytes;
  int32_t neighbor_slots;   /* compile-time top-K slots of the chosen kernel variant */
  int32_t obstacle_slots;
  int32_t obs_dim;
  int32_t staged_obs;       /* 1: obs staged through LDS and stored coalesced; 0: rows stored from
                               registers (small latency-bound launches, lanes_per_env != 64) */
  int32_t kernel_id;        /* SWARM_KERNEL_* swarm_step launches for these params (aligned buffers) */
} swarm_launch_info_t;

int swarm_abi_version(void);
const char* swarm_last_error(void);

/* Fill swarm_params_t with DroneEnvConfig defaults (common.py:9-24), num_drones = 3. */
void swarm_params_default(swarm_params_t* p);

/* Observation width D for `p` (drone_swarm_env.py:41-45). */
int swarm_obs_dim(const swarm_params_t* p);

/* Geometry of the kernel `swarm_step` would launch for `p`. */
int swarm_query_launch(const swarm_params_t* p, swarm_launch_info_t* info);

/*
 * One env step for every env: integrate, clip, distances, collision, formation, rewards,
 * terminations, (auto-reset), kNN observation, optional infos/global_state.
 * actions: [E,N,3] f32.  action_mask: [E,N] u8 or NULL (= every agent supplied an action;
 * a missing action is a zero action in swarm mode, no thrust in physics mode).
 * obs/global_state describe the state AFTER the call (post-reset for auto-reset envs).
 */
int swarm_step(const swarm_params_t* p, const swarm_state_t* s, const float* actions,
               const uint8_t* action_mask, const swarm_out_t* o, void* hip_stream);

/*
 * swarm_step for a batch split into env groups, one launch per group in one call (the batch's
 * env groups overlap on their streams: one group's launch burst and tail run beside the others'
 * steady state).  p / s / o / actions / action_mask describe the whole batch of p->num_envs envs;
 * group g is rows [lo_g, lo_g + group_envs[g]) (lo_g = the sum of the earlier groups), stepped on
 * hip_streams[g] exactly as swarm_step would step those rows with env_offset + lo_g — results are
 * bitwise those of one swarm_step over the batch.  group_envs must sum to p->num_envs.  s->work
 * (persistent kernel only), if set, holds `groups` x SWARM_WORK_WORDS words, one block per group.
 * No ordering between the streams is added: the caller makes every stream wait for the inputs.
 * Replaces the per-group Python launch loop (one ctypes call per step instead of G).
 */
int swarm_step_groups(const swarm_params_t* p, const swarm_state_t* s, const float* actions,
                      const uint8_t* action_mask, const swarm_out_t* o, int groups,
                      const int32_t* group_envs, void* const* hip_streams);

/*
 * Device reset: draw a new episode (Philox4x32-10 keyed by seed, global env index and
 * episode counter) for the envs with env_mask[e] != 0 (NULL = all) and write their obs,
 * dist_goal, global_state.  Outputs of envs not in the mask are left untouched.
 */
int swarm_reset(const swarm_params_t* p, const swarm_state_t* s, const uint8_t* env_mask,
                const swarm_out_t* o, void* hip_stream);

/*
 * Observation only: obs / dist_goal / global_state for the current state of the masked envs
 * (NULL = all).  The state is not modified.  Used after a host-side seeded reset.
 */
int swarm_observe(const swarm_params_t* p, const swarm_state_t* s, const uint8_t* env_mask,
                  const swarm_out_t* o, void* hip_stream);


/*
 * On-device actor inference: the reference's exported policy
 * (scripts/export_onnx.py:120-141: RLlib TorchFC, fcnet_hiddens [256, 256], relu;
 * src/swarm_marl/training/config_builders.py:53-56, models.py:75-81)
 *     logits = W3 relu(W2 relu(W1 x + b1) + b2) + b3,   logits = [mean | log_std]
 * run on the GPU over the env's observation tensor, writing logits and/or the next actions
 * (RLlib TorchDiagGaussian: deterministic = mean; sampled = mean + exp(log_std) * N(0, 1)).
 * It replaces the policy forward the reference runs on the host per agent
 * (algo.compute_single_action / the ONNX graph, scripts/evaluate_protocol.py:152-170).
 */
#define SWARM_POLICY_HIDDEN 256
#define SWARM_POLICY_MAX_IN 47      /* obs dim (one pad column carries the layer-1 bias) */
#define SWARM_POLICY_MAX_OUT 12     /* logits (2 x action dim) */
#define SWARM_POLICY_BF16 0         /* v_mfma_f32_32x32x16_bf16: bf16 operands, f32 accumulation */
#define SWARM_POLICY_F32 1          /* v_mfma_f32_16x16x4_f32: f32 operands and sums */
#define SWARM_POLICY_F32X3 2        /* v_mfma_f32_32x32x16_f16, three passes: every f32 operand split
                                       into f16 hi + lo, products hi*hi + hi*lo + lo*hi (~2^-21
                                       relative per product: the f32 path's tolerance at f16-MFMA
                                       speed); obs, weights and activations must be < 65504 in
                                       magnitude (f16 range) */
#define SWARM_POLICY_ACT_MEAN 0     /* actions = mean (deterministic) */
#define SWARM_POLICY_ACT_SAMPLE 1   /* actions = mean + exp(log_std) * N(0,1), Philox(seed; row, counter) */

typedef struct swarm_policy {
  int32_t in_dim;        /* observation width D */
  int32_t out_dim;       /* logits width (even) */
  int32_t precision;     /* SWARM_POLICY_BF16 / SWARM_POLICY_F32 / SWARM_POLICY_F32X3 */
  int32_t reserved;
  const void* weights;   /* device copy of the swarm_policy_pack blob (16-B aligned) */
} swarm_policy_t;

/* Bytes of the packed weight blob (negative SWARM_E* code for unsupported dims). */
long long swarm_policy_packed_bytes(int in_dim, int out_dim, int precision);

/* Pack row-major f32 weights (PyTorch / ONNX Gemm transB layout: w1 [256,in], w2 [256,256],
 * w3 [out,256]) into the kernel's fragment-order blob at host_out (host memory). */
int swarm_policy_pack(int in_dim, int out_dim, int precision, const float* w1, const float* b1, const float* w2,
                      const float* b2, const float* w3, const float* b3, void* host_out);

/* logits [rows,out] (nullable) and/or actions [rows,out/2] (nullable) for obs [rows,in]; async on
 * hip_stream, no allocation, no sync. */
int swarm_policy_forward(const swarm_policy_t* p, const float* obs, long long rows, float* logits, float* actions,
                         int action_mode, unsigned long long seed, unsigned long long counter, void* hip_stream);

const char* swarm_policy_last_error(void);

/*
 * On-device evaluation metrics: the per-episode summary of
 * scripts/evaluate_protocol.py:237-331 (`_run_single_episode_multi_agent`; formation error
 * :103-116) accumulated on the device from a step's outputs (obs, reward, info_flags, env_done:
 * the env must be stepped with infos).  swarm_eval_update after every swarm_step appends one
 * record per finished episode; the host aggregates the records like `_aggregate` (:334-350).
 * Replaces the host-side per-agent loop over the dict outputs of every evaluation step.
 */
#define SWARM_EVAL_LIVE 1u       /* status: an episode is being accumulated */
#define SWARM_EVAL_COLLIDED 2u   /* status: an observed agent reported a collision */
#define SWARM_EVAL_STEP_FUSED 1  /* swarm_eval_t.flags: per-step accumulation done by the step (out.eval) */
#define SWARM_EVAL_RECORD 9      /* doubles per record: global env index, success, collision_free, time_to_goal
                                    (NaN if never all-reached), formation_error, path_efficiency,
                                    episode_reward, steps, update_index of the closing update */
#define SWARM_EVAL_SEGMENTS 64   /* record counters: an episode of global env g is appended to segment
                                    g % 64 (64 counters on distinct lines instead of one contended
                                    device-scope atomic) */

typedef struct swarm_eval {
  double* ep_reward;      /* [E] sum over steps of the mean reward of the stepped agents */
  int32_t* ep_steps;      /* [E] */
  int32_t* reached_step;  /* [E] first step whose observed agents all reached (-1: none yet) */
  uint8_t* status;        /* [E] SWARM_EVAL_* bits */
  double* fe_sum;         /* [E] sum over steps of the formation error */
  float* start;           /* [E,N,3] positions at the episode start */
  float* goal;            /* [E,N,3] start + obs[6:9] (the reference's goal estimate) */
  float* last;            /* [E,N,3] last observed positions */
  double* traveled;       /* [E,N]   path length */
  double* records;        /* [capacity, SWARM_EVAL_RECORD] finished episodes; segment s owns the row
                             block b = (s - seg_base) mod 64 (< segments): rows [b*C, (b+1)*C),
                             C = capacity / segments */
  uint32_t* count;        /* [SWARM_EVAL_SEGMENTS] records appended per segment (may exceed C: the
                             rest are dropped) */
  int32_t capacity;       /* a multiple of `segments` */
  int32_t update_index;   /* stamped into the records this update closes (the caller counts updates) */
  int32_t flags;          /* SWARM_EVAL_STEP_FUSED: the step launches carry this state in out.eval */
  int32_t seg_base;       /* segment of the tracker's first global env (its env_offset mod 64) */
  int32_t segments;       /* record segments that receive episodes: min(envs, 64) (0 = 64): a
                             batch of E < 64 envs holds only E row blocks */
  const float* state_pos;   /* [E,N,3] optional: the env state's positions after the step (bitwise
                               obs[..., 0:3]), read contiguously instead of from the obs rows */
  const float* state_goal;  /* [E,3] optional (with state_pos): the goal; obs[..., 6:9] = goal - pos */
} swarm_eval_t;

/* Start an episode in the masked envs (all if NULL) from the current obs (after a reset). */
int swarm_eval_begin(const swarm_params_t* p, const swarm_eval_t* ev, const swarm_out_t* out,
                     const uint8_t* env_mask, void* hip_stream);

/* Accumulate one step's outputs; close finished episodes (and open the next one of an env the
 * step auto-reset).  Async on hip_stream, no allocation, no sync. */
int swarm_eval_update(const swarm_params_t* p, const swarm_eval_t* ev, const swarm_out_t* out, void* hip_stream);

/* Single-agent protocol (scripts/evaluate_protocol.py:193-234 `_run_single_episode_single_agent`
 * over SingleDroneEnv): a batch of E single-drone envs (num_drones 1, neighbor_k 0, stepped with
 * infos and auto_reset 0, ev->state_pos / state_goal set).  Unlike the swarm protocol the
 * terminal step counts: its collision / reached_goal info and its position (the state, not yet
 * reset).  Per env and step: reward sum, path length, first reached step, any collision; at
 * terminated or truncated one record (formation_error 0) and reset_mask[e] = 1 (0 otherwise):
 * the caller then runs swarm_reset(reset_mask) and swarm_eval_begin(reset_mask) — the next
 * episode — without a host sync.  Replaces the reference's per-episode host loop. */
int swarm_eval_single_update(const swarm_params_t* p, const swarm_eval_t* ev, const swarm_out_t* out,
                             uint8_t* reset_mask, void* hip_stream);

const char* swarm_eval_last_error(void);

/*
 * Write the per-env parameter records cfg[e] (device, [E] swarm_env_cfg_t) of the masked envs
 * (env_mask NULL = all) from `ov` and the uniform fields of `p`.  Async on hip_stream.  Point
 * swarm_state_t.env_cfg (the current episode) or .env_cfg_next (the next episode, e.g. a domain
 * randomisation draw made after the step that reset the env) at the result.
 */
int swarm_env_cfg_set(const swarm_params_t* p, const swarm_env_overrides_t* ov, const uint8_t* env_mask,
                      swarm_env_cfg_t* cfg, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* SWARM_MI355X_H */
