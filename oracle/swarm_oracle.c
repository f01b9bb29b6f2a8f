/*
 * swarm_oracle.c — plain-C CPU restatement of the reference swarm step — TEST INFRASTRUCTURE.
 *
 * Used only by tests/ (cross-check against oracle/swarm_oracle.py and the golden fixtures) and
 * by bench.py's cpu_baseline leg (timed on the host cores).  Never linked into the product.
 *
 * It follows the reference's per-env, per-agent loop structure:
 *   step                         src/swarm_marl/envs/drone_swarm_env.py:92-174
 *   _clip_speed                  :179-183
 *   _collision_mask              :185-208   (obstacle pass with the axis=1 norm, pair pass i<j)
 *   _formation_penalties         :210-224   (np.mean = NumPy pairwise summation, reproduced)
 *   _build_obs / kNN             :226-291
 *   _global_state                :293-302
 *   physics (point mass)         src/swarm_marl/envs/drone_physics_env.py:279-462 (unpinned)
 * with the float32/float64 rounding sequence described in oracle/swarm_oracle.py.
 * Build: oracle/Makefile (-ffp-contract=off, no fast-math).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/swarm_mi355x.h"

#define MODE_STEP 0
#define MODE_RESET 1
#define MODE_OBSERVE 2

static float sqsum_1d(float x, float y, float z) {
  const float xx = x * x, yy = y * y, zz = z * z;
  return (float)(((double)xx + (double)yy) + (double)zz);
}
static float norm_1d(float x, float y, float z) { return sqrtf(sqsum_1d(x, y, z)); }
static float norm_axis(float x, float y, float z) { return sqrtf(((x * x) + (y * y)) + (z * z)); }

/* NumPy pairwise summation (numpy/_core/src/umath/loops_utils.h.src), PW_BLOCKSIZE 128 */
static double pairwise_sum(const double* a, long n) {
  if (n < 8) {
    double res = 0.0;
    for (long i = 0; i < n; ++i) res += a[i];
    return res;
  } else if (n <= 128) {
    double r[8];
    long i;
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    for (i = 8; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  } else {
    long n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
  }
}

/* ---------------------------------------------------------------- Philox4x32-10 */
static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
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
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  memcpy(out, ctr, 16);
  philox(out, key[0], key[1]);
}
static float uni(uint32_t x, float lo, float width) {
  const float u = (float)(x >> 8) * 0x1p-24f;
  return lo + u * width;
}

typedef struct {
  int N, M, K, Ms, D, phys;
  float hw, nhw, width, dt, vmax, amax, eps, thr_pair, thr_obst, thr_ppair, thr_pobst, ground, h, g, gc;
} derived_t;

static void derive(const swarm_params_t* p, derived_t* d) {
  d->N = p->num_drones;
  d->M = p->num_obstacles;
  d->K = p->neighbor_k > 0 ? p->neighbor_k : 0;
  d->Ms = p->sensed_obstacles > 0 ? p->sensed_obstacles : 0;
  d->D = 9 + 4 * d->K + 4 * d->Ms;
  d->phys = p->dynamics == SWARM_DYN_POINTMASS_PHYSICS;
  d->hw = (float)(p->world_size / 2.0);
  d->nhw = (float)(-p->world_size / 2.0);
  d->width = (float)p->world_size;
  d->dt = (float)p->dt;
  d->vmax = (float)p->max_speed;
  d->amax = (float)p->max_accel;
  d->eps = (float)1e-8;
  d->thr_pair = (float)(2.0 * p->collision_radius);
  d->thr_obst = (float)(p->collision_radius + p->obstacle_radius);
  d->thr_ppair = (float)(2.0 * p->drone_contact_radius);
  d->thr_pobst = (float)(p->obstacle_radius + p->drone_contact_radius);
  d->ground = (float)p->ground_contact_height;
  d->h = (float)p->substep_dt;
  d->g = (float)p->gravity;
  d->gc = (float)p->gravity_comp;
}

static void draw_env(const swarm_params_t* p, const derived_t* d, long long genv, uint32_t ep, float* pos,
                     float* goal, float* obst, float* damp) {
  const uint32_t k0 = (uint32_t)(p->seed & 0xffffffffu), k1 = (uint32_t)(p->seed >> 32);
  uint32_t w[4];
  for (int b = 0; b < d->N + d->M + 1; ++b) {
    w[0] = (uint32_t)b;
    w[1] = ep;
    w[2] = (uint32_t)((unsigned long long)genv & 0xffffffffu);
    w[3] = (uint32_t)((unsigned long long)genv >> 32);
    philox(w, k0, k1);
    float x = uni(w[0], d->nhw, d->width), y = uni(w[1], d->nhw, d->width), z = uni(w[2], d->nhw, d->width);
    if (b < d->N) {
      if (d->phys) {
        z = fmaxf(z, 1.0f);
        damp[b] = 0.5f * uni(w[3], 0.8f, 0.4f);
      }
      pos[3 * b] = x; pos[3 * b + 1] = y; pos[3 * b + 2] = z;
    } else if (b < d->N + d->M) {
      if (d->phys) z = fmaxf(z, 0.5f);
      float* o = obst + 3 * (b - d->N);
      o[0] = x; o[1] = y; o[2] = z;
    } else {
      goal[0] = x; goal[1] = y; goal[2] = d->phys ? uni(w[3], 0.5f, 1.5f) : z;
    }
  }
}

typedef struct { float d; int j; } nb_t;
static int nb_less(nb_t a, nb_t b) { return a.d < b.d || (a.d == b.d && a.j < b.j); }

/* kNN observation of agent i (drone_swarm_env.py:226-291), vel_obs = velocity written to the obs */
static void build_obs(const derived_t* d, const float* pos, const float* velobs, const float* goal,
                      const float* obst, int i, float* row, nb_t* scratch) {
  const float px = pos[3 * i], py = pos[3 * i + 1], pz = pos[3 * i + 2];
  row[0] = px; row[1] = py; row[2] = pz;
  row[3] = velobs[0]; row[4] = velobs[1]; row[5] = velobs[2];
  row[6] = goal[0] - px; row[7] = goal[1] - py; row[8] = goal[2] - pz;
  int col = 9;
  if (d->K > 0) {
    int cnt = 0;
    for (int j = 0; j < d->N; ++j) {
      if (j == i) continue;
      nb_t c = {norm_1d(pos[3 * j] - px, pos[3 * j + 1] - py, pos[3 * j + 2] - pz), j};
      int k = cnt < d->K ? cnt : d->K;
      if (cnt >= d->K && !nb_less(c, scratch[d->K - 1])) { ++cnt; continue; }
      if (cnt >= d->K) k = d->K - 1;
      while (k > 0 && nb_less(c, scratch[k - 1])) { scratch[k] = scratch[k - 1]; --k; }
      scratch[k] = c;
      ++cnt;
    }
    const int kk = cnt < d->K ? cnt : d->K;
    for (int s = 0; s < d->K; ++s) {
      float* f = row + col + 4 * s;
      if (s < kk) {
        const int j = scratch[s].j;
        f[0] = pos[3 * j] - px; f[1] = pos[3 * j + 1] - py; f[2] = pos[3 * j + 2] - pz; f[3] = scratch[s].d;
      } else {
        f[0] = f[1] = f[2] = f[3] = 0.f;
      }
    }
    col += 4 * d->K;
  }
  if (d->Ms > 0) {
    int cnt = 0;
    for (int m = 0; m < d->M; ++m) {
      const float* o = obst + 3 * m;
      nb_t c = {norm_axis(o[0] - px, o[1] - py, o[2] - pz), m};
      int k = cnt < d->Ms ? cnt : d->Ms;
      if (cnt >= d->Ms && !nb_less(c, scratch[d->Ms - 1])) { ++cnt; continue; }
      if (cnt >= d->Ms) k = d->Ms - 1;
      while (k > 0 && nb_less(c, scratch[k - 1])) { scratch[k] = scratch[k - 1]; --k; }
      scratch[k] = c;
      ++cnt;
    }
    const int kk = cnt < d->Ms ? cnt : d->Ms;
    for (int s = 0; s < d->Ms; ++s) {
      float* f = row + col + 4 * s;
      if (s < kk) {
        const float* o = obst + 3 * scratch[s].j;
        f[0] = o[0] - px; f[1] = o[1] - py; f[2] = o[2] - pz; f[3] = scratch[s].d;
      } else {
        f[0] = f[1] = f[2] = f[3] = 0.f;
      }
    }
  }
}

static void obs_velocity(const swarm_params_t* p, const derived_t* d, const float* v, float* out) {
  if (!d->phys) {
    out[0] = v[0]; out[1] = v[1]; out[2] = v[2];
    return;
  }
  const double x = v[0], y = v[1], z = v[2];
  const double n = sqrt(((x * x) + (y * y)) + (z * z));
  if (n > p->max_speed) {
    out[0] = (float)((x / n) * p->max_speed);
    out[1] = (float)((y / n) * p->max_speed);
    out[2] = (float)((z / n) * p->max_speed);
  } else {
    out[0] = v[0]; out[1] = v[1]; out[2] = v[2];
  }
}

typedef struct {
  double* dl;   /* [N] formation list */
  float* dist;  /* [N*N] pair distances */
  nb_t* nb;     /* [max(K,Ms)+1] */
  float* curr;  /* [N] */
  float* prev;  /* [N] */
  uint8_t* coll;
  uint8_t* reached;
  double* form;
} scratch_t;

static void env_one(const swarm_params_t* p, const derived_t* d, int mode, long long e, float* pos, float* vel,
                    float* goal, float* obst, uint8_t* active, int32_t* stepc, uint32_t* episode, float* damp,
                    const float* act, const uint8_t* amask, float* obs, double* reward, uint8_t* term,
                    uint8_t* trunc, uint8_t* env_done, float* dist, uint8_t* flags, float* gs, scratch_t* sc) {
  const int N = d->N, M = d->M;
  int term_all = 0, trunc_all = 0, do_reset = 0;
  if (mode == MODE_STEP) {
    int n_active = 0;
    for (int i = 0; i < N; ++i) n_active += active[i] != 0;
    for (int i = 0; i < N; ++i) {
      reward[i] = 0.0; term[i] = 0; trunc[i] = 0; if (flags) flags[i] = 0;
      sc->coll[i] = 0; sc->reached[i] = 0; sc->form[i] = 0.0;
    }
    if (!d->phys) {
      if (n_active == 0) {
        term_all = 1;
        for (int i = 0; i < N; ++i) if (dist) dist[i] = norm_1d(goal[0] - pos[3 * i], goal[1] - pos[3 * i + 1], goal[2] - pos[3 * i + 2]);
      } else {
        for (int i = 0; i < N; ++i) {
          if (!active[i]) continue;
          float* pi = pos + 3 * i;
          float* vi = vel + 3 * i;
          sc->prev[i] = norm_1d(goal[0] - pi[0], goal[1] - pi[1], goal[2] - pi[2]);
          float a[3];
          for (int c = 0; c < 3; ++c) {
            float x = (amask && !amask[i]) ? 0.f : act[3 * i + c];
            x = fminf(fmaxf(x, -1.f), 1.f);
            a[c] = x * d->amax;
          }
          for (int c = 0; c < 3; ++c) vi[c] = vi[c] + a[c] * d->dt;
          const float sp = norm_1d(vi[0], vi[1], vi[2]);
          if (!(sp <= d->vmax || sp < d->eps))
            for (int c = 0; c < 3; ++c) vi[c] = (vi[c] / sp) * d->vmax;
          for (int c = 0; c < 3; ++c) pi[c] = pi[c] + vi[c] * d->dt;
        }
        for (int i = 0; i < 3 * N; ++i) pos[i] = fminf(fmaxf(pos[i], d->nhw), d->hw);
        const int new_step = *stepc + 1;
        *stepc = new_step;
        for (int i = 0; i < N; ++i) {
          sc->curr[i] = norm_1d(goal[0] - pos[3 * i], goal[1] - pos[3 * i + 1], goal[2] - pos[3 * i + 2]);
          if (dist) dist[i] = sc->curr[i];
          if (active[i]) sc->reached[i] = (double)sc->curr[i] <= p->goal_radius;
        }
        /* _collision_mask: obstacle pass, then pair pass over active i<j */
        for (int i = 0; i < N; ++i) {
          if (!active[i]) continue;
          for (int m = 0; m < M; ++m) {
            const float* o = obst + 3 * m;
            if (norm_axis(pos[3 * i] - o[0], pos[3 * i + 1] - o[1], pos[3 * i + 2] - o[2]) <= d->thr_obst) {
              sc->coll[i] = 1;
              break;
            }
          }
        }
        for (int i = 0; i < N; ++i) {
          for (int j = 0; j < N; ++j) {
            sc->dist[i * N + j] = norm_1d(pos[3 * i] - pos[3 * j], pos[3 * i + 1] - pos[3 * j + 1], pos[3 * i + 2] - pos[3 * j + 2]);
          }
        }
        if (n_active > 1) {
          for (int i = 0; i < N; ++i) {
            if (!active[i]) continue;
            for (int j = i + 1; j < N; ++j)
              if (active[j] && sc->dist[i * N + j] <= d->thr_pair) sc->coll[i] = sc->coll[j] = 1;
          }
          for (int i = 0; i < N; ++i) {
            if (!active[i]) continue;
            long c = 0;
            for (int j = 0; j < N; ++j)
              if (j != i && active[j]) sc->dl[c++] = fabs((double)sc->dist[i * N + j] - p->desired_spacing);
            sc->form[i] = -p->reward_formation_scale * (pairwise_sum(sc->dl, c) / (double)c);
          }
        }
        int any_c = 0, n_cont = 0;
        for (int i = 0; i < N; ++i) if (active[i] && sc->coll[i]) any_c = 1;
        const int tl = new_step >= p->max_steps;
        for (int i = 0; i < N; ++i) {
          if (!active[i]) continue;
          double r = ((double)sc->prev[i] - (double)sc->curr[i]) * p->reward_progress_scale;
          r = r + sc->form[i];
          if (sc->reached[i]) r = r + p->reward_goal;
          if (sc->coll[i]) r = r + p->reward_collision;
          reward[i] = r;
          const int done_i = sc->reached[i] || sc->coll[i];
          term[i] = (uint8_t)done_i;
          trunc[i] = (uint8_t)(tl && !done_i);
          const int cont = !done_i && !tl && !any_c;
          n_cont += cont;
          if (flags)
            flags[i] = (uint8_t)(SWARM_AGENT_STEPPED | (sc->reached[i] ? SWARM_AGENT_REACHED : 0) |
                                 (sc->coll[i] ? SWARM_AGENT_COLLISION : 0) | (cont ? SWARM_AGENT_HAS_OBS : 0));
        }
        const int all_reached = n_cont == 0 && !any_c && !tl;
        term_all = all_reached || any_c;
        trunc_all = tl && !term_all;
        for (int i = 0; i < N; ++i) {
          const int cont = active[i] && !(sc->reached[i] || sc->coll[i]) && !tl && !any_c;
          active[i] = (uint8_t)cont;
        }
      }
    } else {
      /* point-mass physics (drone_physics_env.py:323-419) */
      for (int i = 0; i < N; ++i) {
        float* pi = pos + 3 * i;
        float* vi = vel + 3 * i;
        const int has = !amask || amask[i];
        const float cx = has ? act[3 * i] * d->amax : 0.f;
        const float cy = has ? act[3 * i + 1] * d->amax : 0.f;
        float cz = has ? act[3 * i + 2] * d->amax + d->gc : 0.f;
        cz = cz + d->g;
        float fac = 1.f;
        if (p->damping_law == 1) fac = (float)pow((double)(1.f - damp[i]), (double)d->h);
        for (int s = 0; s < p->physics_substeps; ++s) {
          const float sp = norm_1d(vi[0], vi[1], vi[2]);
          if (has && sp > d->vmax)
            for (int c = 0; c < 3; ++c) vi[c] = (vi[c] / sp) * d->vmax;
          if (p->damping_law == 0) {
            const float sp2 = norm_1d(vi[0], vi[1], vi[2]);
            const float cc = damp[i] * (1.f + sp2);
            vi[0] = vi[0] + d->h * (cx - cc * vi[0]);
            vi[1] = vi[1] + d->h * (cy - cc * vi[1]);
            vi[2] = vi[2] + d->h * (cz - cc * vi[2]);
          } else {
            vi[0] = (vi[0] + d->h * cx) * fac;
            vi[1] = (vi[1] + d->h * cy) * fac;
            vi[2] = (vi[2] + d->h * cz) * fac;
          }
          for (int c = 0; c < 3; ++c) pi[c] = pi[c] + d->h * vi[c];
        }
      }
      const int new_step = *stepc + 1;
      *stepc = new_step;
      int any_c = 0, not_all = 0;
      for (int i = 0; i < N; ++i) {
        const float* pi = pos + 3 * i;
        int c = pi[2] <= d->ground;
        for (int m = 0; m < M && !c; ++m) {
          const float* o = obst + 3 * m;
          if (norm_axis(o[0] - pi[0], o[1] - pi[1], o[2] - pi[2]) <= d->thr_pobst) c = 1;
        }
        for (int j = 0; j < N && !c; ++j)
          if (j != i && norm_1d(pi[0] - pos[3 * j], pi[1] - pos[3 * j + 1], pi[2] - pos[3 * j + 2]) <= d->thr_ppair) c = 1;
        const double dx = (double)pi[0] - (double)goal[0], dy = (double)pi[1] - (double)goal[1],
                     dz = (double)pi[2] - (double)goal[2];
        const double dd = sqrt(((dx * dx) + (dy * dy)) + (dz * dz));
        const int reached = dd < p->goal_radius;
        if (dist) dist[i] = (float)dd;
        if (active[i]) {
          double r = (-dd) * 0.1;
          if (c) { r = r - 10.0; any_c = 1; }
          else if (reached) r = r + 50.0;
          else not_all = 1;
          reward[i] = r;
        }
        if (flags)
          flags[i] = (uint8_t)((active[i] ? SWARM_AGENT_STEPPED : 0) | (active[i] && reached ? SWARM_AGENT_REACHED : 0) |
                               (active[i] && c ? SWARM_AGENT_COLLISION : 0) | SWARM_AGENT_HAS_OBS);
      }
      const int tl = new_step >= p->max_steps;
      const int all_goals = !not_all;
      const int done = any_c || all_goals || tl;
      trunc_all = done && tl && !any_c && !all_goals;
      term_all = done && !trunc_all;
      for (int i = 0; i < N; ++i) {
        term[i] = (uint8_t)term_all;
        trunc[i] = (uint8_t)trunc_all;
        if (done) active[i] = 0;
      }
    }
    do_reset = p->auto_reset && (term_all || trunc_all);
    if (env_done) *env_done = (uint8_t)((term_all ? SWARM_ENV_TERMINATED : 0) | (trunc_all ? SWARM_ENV_TRUNCATED : 0) |
                                        (do_reset ? SWARM_ENV_RESET : 0));
  } else if (mode == MODE_RESET) {
    do_reset = 1;
  }
  if (do_reset) {
    const uint32_t ep = *episode + 1u;
    *episode = ep;
    draw_env(p, d, p->env_offset + e, ep, pos, goal, obst, damp);
    for (int i = 0; i < 3 * N; ++i) vel[i] = 0.f;
    for (int i = 0; i < N; ++i) active[i] = 1;
    *stepc = 0;
  }
  if (mode != MODE_STEP && dist)
    for (int i = 0; i < N; ++i) dist[i] = norm_1d(goal[0] - pos[3 * i], goal[1] - pos[3 * i + 1], goal[2] - pos[3 * i + 2]);
  for (int i = 0; i < N; ++i) {
    float vo[3];
    obs_velocity(p, d, vel + 3 * i, vo);
    build_obs(d, pos, vo, goal, obst, i, obs + (size_t)i * d->D, sc->nb);
  }
  if (gs) {
    memcpy(gs, pos, sizeof(float) * 3 * N);
    memcpy(gs + 3 * N, vel, sizeof(float) * 3 * N);
    memcpy(gs + 6 * N, goal, sizeof(float) * 3);
  }
}

/*
 * Batched entry: mode 0 = step, 1 = reset (masked, Philox draws), 2 = observe.  Buffers as in
 * swarm_mi355x.h but host memory and reward in double.  nthreads <= 0: OpenMP default.
 */
int oracle_run(const swarm_params_t* p, int mode, float* pos, float* vel, float* goal, float* obst, uint8_t* active,
               int32_t* stepc, uint32_t* episode, float* damping, const float* actions, const uint8_t* amask,
               const uint8_t* env_mask, float* obs, double* reward, uint8_t* term, uint8_t* trunc, uint8_t* env_done,
               float* dist, uint8_t* flags, float* gs, int nthreads) {
  derived_t d;
  derive(p, &d);
  const long long E = p->num_envs;
  const int N = d.N, M = d.M;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
  int fail = 0;
#pragma omp parallel
  {
    scratch_t sc;
    const int nbmax = (d.K > d.Ms ? d.K : d.Ms) + 1;
    sc.dl = (double*)malloc(sizeof(double) * (N + 1));
    sc.dist = (float*)malloc(sizeof(float) * (size_t)N * N);
    sc.nb = (nb_t*)malloc(sizeof(nb_t) * nbmax);
    sc.curr = (float*)malloc(sizeof(float) * N);
    sc.prev = (float*)malloc(sizeof(float) * N);
    sc.coll = (uint8_t*)malloc(N);
    sc.reached = (uint8_t*)malloc(N);
    sc.form = (double*)malloc(sizeof(double) * N);
    if (!sc.dl || !sc.dist || !sc.nb || !sc.curr || !sc.prev || !sc.coll || !sc.reached || !sc.form) {
#pragma omp atomic write
      fail = 1;
    } else {
#pragma omp for schedule(dynamic, 16)
      for (long long e = 0; e < E; ++e) {
        if (mode != MODE_STEP && env_mask && !env_mask[e]) continue;
        env_one(p, &d, mode, e, pos + e * N * 3, vel + e * N * 3, goal + e * 3, obst ? obst + e * M * 3 : NULL,
                active + e * N, stepc + e, episode + e, damping ? damping + e * N : NULL,
                actions ? actions + e * N * 3 : NULL, amask ? amask + e * N : NULL, obs + e * (long long)N * d.D,
                reward ? reward + e * N : NULL, term ? term + e * N : NULL, trunc ? trunc + e * N : NULL,
                env_done ? env_done + e : NULL, dist ? dist + e * N : NULL, flags ? flags + e * N : NULL,
                gs ? gs + e * (6LL * N + 3) : NULL, &sc);
      }
    }
    free(sc.dl); free(sc.dist); free(sc.nb); free(sc.curr); free(sc.prev); free(sc.coll); free(sc.reached);
    free(sc.form);
  }
  return fail ? -1 : 0;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
