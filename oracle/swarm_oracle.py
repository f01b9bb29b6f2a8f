"""CPU restatement (ORACLE) of the reference swarm step/reset/observe path — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker.  The product path (swarm_marl_amd) never calls it.

Parity status
-------------
* kinematic dynamics + swarm reward (DroneSwarmEnv): PINNED — checked bit-exactly (obs, state,
  flags) and to 1e-9 (rewards) against golden fixtures recorded from the reference itself
  (tests/golden/*.npz, generator tests/golden/make_golden.py; tests/test_oracle_golden.py).
* pointmass_physics dynamics + physics reward (DronePhysicsEnv): parity UNPINNED — the reference
  runs PyBullet (pybullet>=3.2.5, unpinned, requirements.txt:4), which is not installed here.
  This restatement follows drone_physics_env.py:320-419 with the assumptions listed in
  DESIGN.md §4 and is pinned only by analytic known-answer tests.

Numerics (SURVEY.md §8a "parity spec"):
* `np.linalg.norm(v)` of a float32 3-vector is OpenBLAS sdot with a double accumulator of float
  products:  sqrtf((float)(((double)(x*x) + (double)(y*y)) + (double)(z*z)))   -> norm1d()
* `np.linalg.norm(A, axis=1)` is all-float32:  sqrtf(((x*x)+(y*y))+(z*z))        -> norm_axis()
* Python-float constants meet float32 arrays as float32 (NumPy 2 weak scalars, NEP 50).

Arrays are batched over E envs: pos/vel [E,N,3] f32, goal [E,3], obst [E,M,3], active [E,N] bool,
step [E] int32, episode [E] uint32, damping [E,N] f32.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32
f64 = np.float64
u32 = np.uint32
u64 = np.uint64

DEFAULTS = dict(  # DroneEnvConfig defaults, src/swarm_marl/envs/common.py:9-24
    world_size=20.0, dt=0.1, max_steps=400, max_speed=4.0, max_accel=2.0,
    collision_radius=0.5, goal_radius=0.8, num_obstacles=8, sensed_obstacles=4,
    neighbor_k=3, obstacle_radius=0.8, desired_spacing=2.5, reward_progress_scale=2.0,
    reward_goal=25.0, reward_collision=-25.0, reward_formation_scale=0.15,
)
PHYSICS_DEFAULTS = dict(  # drone_physics_env.py:135,197,323,343 ; assets/drone.urdf:5,7
    gravity=-9.81, gravity_comp=9.5, substep_dt=1.0 / 240.0, drone_contact_radius=0.15,
    ground_contact_height=0.025, damping_law=0,
)


def make_cfg(**kw) -> dict:
    cfg = dict(DEFAULTS)
    cfg.update(PHYSICS_DEFAULTS)
    cfg["num_drones"] = 3
    cfg.update(kw)
    return cfg


def obs_dim(cfg) -> int:
    return 9 + 4 * max(int(cfg["neighbor_k"]), 0) + 4 * max(int(cfg["sensed_obstacles"]), 0)


# ----------------------------------------------------------------------------- numerics
def norm1d(v):
    """np.linalg.norm(v) for float32 3-vectors (sdot, double accumulator)."""
    sq = v * v
    s = (sq[..., 0].astype(f64) + sq[..., 1].astype(f64)) + sq[..., 2].astype(f64)
    return np.sqrt(s.astype(f32))


def norm_axis(v):
    """np.linalg.norm(A, axis=-1) for float32 rows (float32 pairwise add of 3 terms)."""
    sq = v * v
    return np.sqrt((sq[..., 0] + sq[..., 1]) + sq[..., 2])


# ----------------------------------------------------------------------------- device RNG
PHILOX_M0, PHILOX_M1 = 0xD2511F53, 0xCD9E8D57
PHILOX_W0, PHILOX_W1 = 0x9E3779B9, 0xBB67AE85


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Salmon et al., SC'11; Random123 philox4x32_R with R=10)."""
    m32 = u64(0xFFFFFFFF)
    c = [np.asarray(x, dtype=u64) & m32 for x in (c0, c1, c2, c3)]
    k0 = np.asarray(k0, dtype=u64) & m32
    k1 = np.asarray(k1, dtype=u64) & m32
    for _ in range(10):
        p0 = u64(PHILOX_M0) * c[0]
        p1 = u64(PHILOX_M1) * c[2]
        hi0, lo0 = p0 >> u64(32), p0 & m32
        hi1, lo1 = p1 >> u64(32), p1 & m32
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = (k0 + u64(PHILOX_W0)) & m32
        k1 = (k1 + u64(PHILOX_W1)) & m32
    return [x.astype(u32) for x in c]


def _u01(x):
    return ((x >> u32(8)).astype(f32) * f32(2.0 ** -24)).astype(f32)


def _uni(x, lo, width):
    return (f32(lo) + _u01(x) * f32(width)).astype(f32)


def device_reset_draws(cfg, env_ids, episodes, seed, physics=False):
    """Philox draw layout of the in-kernel reset.

    key = (seed lo, seed hi); counter = (block, episode, global env lo, global env hi).
    drone i: block i words 0..2 -> pos (physics: z=max(1,z); word 3 -> damping);
    obstacle m: block N+m; goal: block N+M (physics: word 3 -> goal z ~ U(0.5,2.0)).
    Mirrors drone_swarm_env.py:72-80 / drone_physics_env.py:205-242 draw ranges.
    """
    n, m = int(cfg["num_drones"]), int(cfg["num_obstacles"])
    env_ids = np.asarray(env_ids, dtype=np.int64)
    e = env_ids.shape[0]
    k0, k1 = u64(seed & 0xFFFFFFFF), u64((seed >> 32) & 0xFFFFFFFF)
    blocks = np.arange(n + m + 1, dtype=u64)
    cb = np.broadcast_to(blocks[None, :], (e, n + m + 1))
    ce = np.broadcast_to(np.asarray(episodes, dtype=u64)[:, None], cb.shape)
    glo = np.broadcast_to((env_ids.astype(u64) & u64(0xFFFFFFFF))[:, None], cb.shape)
    ghi = np.broadcast_to((env_ids.astype(u64) >> u64(32))[:, None], cb.shape)
    w = philox4x32_10(cb, ce, glo, ghi, k0, k1)
    lo, width = -float(f32(cfg["world_size"] / 2.0)), float(f32(cfg["world_size"]))
    xyz = np.stack([_uni(w[c], lo, width) for c in range(3)], axis=-1)  # [E, n+m+1, 3]
    pos = xyz[:, :n].copy()
    obst = xyz[:, n:n + m].copy()
    goal = xyz[:, n + m].copy()
    damping = np.zeros((e, n), f32)
    if physics:
        pos[..., 2] = np.maximum(pos[..., 2], f32(1.0))
        obst[..., 2] = np.maximum(obst[..., 2], f32(0.5))
        goal[:, 2] = _uni(w[3][:, n + m], 0.5, 1.5)
        damping = (f32(0.5) * _uni(w[3][:, :n], 0.8, 0.4)).astype(f32)
    return pos, obst, goal, damping


# ----------------------------------------------------------------------------- observation
def observe(cfg, pos, vel, goal, obst, physics=False):
    """_build_obs for every agent (drone_swarm_env.py:226-291; drone_physics_env.py:421-538).

    Neighbours range over ALL drones (active or not; :252-257), sorted by (distance, index)
    (np.argsort; ties are measure-zero, index order chosen).  Zero padding when fewer than K
    neighbours / Ms obstacles exist.  Physics mode clamps the velocity in the obs only (:438-442).
    """
    e, n, _ = pos.shape
    k = int(cfg["neighbor_k"])
    ms = int(cfg["sensed_obstacles"])
    m = obst.shape[1]
    d = obs_dim(cfg)
    obs = np.zeros((e, n, d), f32)
    obs[:, :, 0:3] = pos
    if physics:
        vd = vel.astype(f64)
        sq = vd * vd
        nv = np.sqrt((sq[..., 0] + sq[..., 1]) + sq[..., 2])
        big = nv > float(cfg["max_speed"])
        with np.errstate(invalid="ignore", divide="ignore"):
            vc = (vd / nv[..., None]) * float(cfg["max_speed"])
        obs[:, :, 3:6] = np.where(big[..., None], vc, vd).astype(f32)
    else:
        obs[:, :, 3:6] = vel
    obs[:, :, 6:9] = goal[:, None, :] - pos
    col = 9
    if k > 0:
        if n > 1:
            rel = pos[:, None, :, :] - pos[:, :, None, :]  # [e,i,j] = p_j - p_i
            dist = norm1d(rel)
            key = dist.astype(f64)
            idx = np.arange(n)
            key[:, idx, idx] = np.inf
            order = np.argsort(key, axis=2, kind="stable")
            kk = min(k, n - 1)
            sel = order[:, :, :kk]
            ii = np.arange(n)[None, :, None]
            ee = np.arange(e)[:, None, None]
            feats = np.concatenate([rel[ee, ii, sel], dist[ee, ii, sel][..., None]], axis=-1)
            obs[:, :, col:col + 4 * kk] = feats.reshape(e, n, 4 * kk)
        col += 4 * k
    if ms > 0:
        if m > 0:
            rel = obst[:, None, :, :] - pos[:, :, None, :]  # o_m - p_i
            dist = norm_axis(rel)
            order = np.argsort(dist, axis=2, kind="stable")
            kk = min(ms, m)
            sel = order[:, :, :kk]
            ii = np.arange(n)[None, :, None]
            ee = np.arange(e)[:, None, None]
            feats = np.concatenate([rel[ee, ii, sel], dist[ee, ii, sel][..., None]], axis=-1)
            obs[:, :, col:col + 4 * kk] = feats.reshape(e, n, 4 * kk)
    return obs


def global_state(pos, vel, goal):
    """drone_swarm_env.py:293-302: concat(positions.ravel(), velocities.ravel(), goal)."""
    e = pos.shape[0]
    return np.concatenate([pos.reshape(e, -1), vel.reshape(e, -1), goal], axis=1).astype(f32)


def thresholds(cfg):
    return dict(
        obst=f32(cfg["collision_radius"] + cfg["obstacle_radius"]),  # drone_swarm_env.py:196-197
        pair=f32(2.0 * cfg["collision_radius"]),                       # :205
        phys_obst=f32(cfg["obstacle_radius"] + cfg["drone_contact_radius"]),
        phys_pair=f32(2.0 * cfg["drone_contact_radius"]),
        ground=f32(cfg["ground_contact_height"]),
    )


# ----------------------------------------------------------------------------- step
def _kinematic_integrate(cfg, pos, vel, actions, act):
    """drone_swarm_env.py:103-117 (+ _clip_speed :179-183)."""
    a = np.clip(actions, f32(-1.0), f32(1.0)).astype(f32)
    acc = a * f32(cfg["max_accel"])
    v = vel + acc * f32(cfg["dt"])
    sp = norm1d(v)
    keep = (sp <= f32(cfg["max_speed"])) | (sp < f32(1e-8))
    with np.errstate(invalid="ignore", divide="ignore"):
        vc = (v / sp[..., None]) * f32(cfg["max_speed"])
    v = np.where(keep[..., None], v, vc).astype(f32)
    p = pos + v * f32(cfg["dt"])
    return np.where(act[..., None], p, pos), np.where(act[..., None], v, vel)


def _physics_integrate(cfg, pos, vel, actions, has, damping):
    """Point-mass restatement of drone_physics_env.py:323-360 (DESIGN.md §4 assumptions)."""
    h = f32(cfg["substep_dt"])
    amax = f32(cfg["max_accel"])
    gc = f32(cfg["gravity_comp"])
    g = f32(cfg["gravity"])
    vmax = f32(cfg["max_speed"])
    law = int(cfg.get("damping_law", 0))
    p, v = pos.copy(), vel.copy()
    hasb = has[..., None]
    a_cmd = np.where(hasb, actions * amax, f32(0.0)).astype(f32)
    a_cmd[..., 2] = np.where(has, a_cmd[..., 2] + gc, f32(0.0))
    a_cmd[..., 2] = a_cmd[..., 2] + g
    if law == 1:
        fac = np.power((f32(1.0) - damping).astype(f64), float(h)).astype(f32)
    for _ in range(int(cfg.get("physics_substeps", int(float(cfg["dt"]) * 240)))):
        sp = norm1d(v)
        big = has & (sp > vmax)
        with np.errstate(invalid="ignore", divide="ignore"):
            vc = (v / sp[..., None]) * vmax
        v = np.where(big[..., None], vc, v).astype(f32)
        if law == 0:
            sp2 = norm1d(v)
            c = (damping * (f32(1.0) + sp2)).astype(f32)
            acc = (a_cmd - c[..., None] * v).astype(f32)
            v = (v + h * acc).astype(f32)
        else:
            v = (v + h * a_cmd).astype(f32)
            v = (v * fac[..., None]).astype(f32)
        p = (p + h * v).astype(f32)
    return p, v


def _numpy_mean_pairwise(vals: np.ndarray) -> float:
    return float(np.mean(vals))


def step(cfg, state, actions, action_mask=None, *, physics=False, auto_reset=False, seed=0,
         env_offset=0, exact_formation=True):
    """One step of every env.  Returns (new_state, out) with out arrays:
    obs [E,N,D] f32, reward [E,N] f64, terminated/truncated [E,N] bool, term_all/trunc_all [E],
    reset [E] bool, dist_goal [E,N] f32 (info), reached/collision/stepped/has_obs [E,N] bool,
    global_state [E,6N+3] f32.
    """
    pos = state["pos"].astype(f32).copy()
    vel = state["vel"].astype(f32).copy()
    goal = state["goal"].astype(f32).copy()
    obst = state["obst"].astype(f32).copy()
    act = state["active"].astype(bool).copy()
    stepc = state["step"].astype(np.int32).copy()
    episode = state.get("episode", np.zeros(pos.shape[0], u32)).astype(u32).copy()
    damping = state.get("damping", np.zeros(pos.shape[:2], f32)).astype(f32).copy()
    e, n, _ = pos.shape
    m = obst.shape[1]
    actions = np.asarray(actions, f32)
    has = np.ones((e, n), bool) if action_mask is None else np.asarray(action_mask, bool)
    thr = thresholds(cfg)
    eye = np.eye(n, dtype=bool)[None]

    n_active = act.sum(axis=1)
    no_active = n_active == 0
    reward = np.zeros((e, n), f64)
    term = np.zeros((e, n), bool)
    trunc = np.zeros((e, n), bool)
    reached = np.zeros((e, n), bool)
    collided = np.zeros((e, n), bool)
    has_obs = np.zeros((e, n), bool)

    if not physics:
        # ---------------- DroneSwarmEnv.step (drone_swarm_env.py:92-174)
        prev = norm1d(goal[:, None, :] - pos)                                     # :98-101
        moving = act & ~no_active[:, None]
        a = np.where(has[..., None], actions, f32(0.0)).astype(f32)              # :104
        p1, v1 = _kinematic_integrate(cfg, pos, vel, a, moving)                   # :103-111
        hw = f32(cfg["world_size"] / 2.0)
        p1 = np.clip(p1, -hw, hw).astype(f32)                                     # :113-117
        pos = np.where(no_active[:, None, None], pos, p1)
        vel = np.where(no_active[:, None, None], vel, v1)
        stepc = stepc + (~no_active).astype(np.int32)                             # :118
        curr = norm1d(goal[:, None, :] - pos)                                     # :120-123
        reached = act & (curr.astype(f64) <= float(cfg["goal_radius"]))           # :124-127
        if m > 0:                                                                 # :190-200
            do = norm_axis(pos[:, :, None, :] - obst[:, None, :, :])
            ohit = np.any(do <= thr["obst"], axis=2)
        else:
            ohit = np.zeros((e, n), bool)
        dpp = norm1d(pos[:, :, None, :] - pos[:, None, :, :])                     # :202-207
        pmask = act[:, :, None] & act[:, None, :] & ~eye
        phit = np.any(pmask & (dpp <= thr["pair"]), axis=2)
        collided = act & (ohit | phit)
        # _formation_penalties (:210-224): mean over active j != i of |d_ij - d*| (fp64)
        form = np.zeros((e, n), f64)
        ds = float(cfg["desired_spacing"])
        kf = float(cfg["reward_formation_scale"])
        if exact_formation:
            for ei in range(e):
                if n_active[ei] <= 1:
                    continue
                ids = np.nonzero(act[ei])[0]
                for i in ids:
                    others = ids[ids != i]
                    dl = dpp[ei, i, others].astype(f64)
                    form[ei, i] = -kf * _numpy_mean_pairwise(np.abs(dl - ds))
        else:
            err = np.where(pmask, np.abs(dpp.astype(f64) - ds), 0.0).sum(axis=2)
            cnt = np.maximum(n_active - 1, 1)[:, None]
            form = np.where((n_active > 1)[:, None] & act, -kf * (err / cnt), 0.0)
        any_coll = np.any(collided, axis=1)                                       # :137
        time_limit = stepc >= int(cfg["max_steps"])                               # :138
        r = (prev.astype(f64) - curr.astype(f64)) * float(cfg["reward_progress_scale"])
        r = r + form                                                              # :141-142
        r = np.where(reached, r + float(cfg["reward_goal"]), r)                   # :143-144
        r = np.where(collided, r + float(cfg["reward_collision"]), r)             # :145-146
        done_i = reached | collided
        reward = np.where(act, r, 0.0)
        term = act & done_i                                                       # :150-151
        trunc = act & time_limit[:, None] & ~done_i                               # :152
        has_obs = act & ~done_i & ~time_limit[:, None] & ~any_coll[:, None]       # :154
        n_cont = has_obs.sum(axis=1)
        all_reached = (n_cont == 0) & ~any_coll & ~time_limit                     # :164
        term_all = all_reached | any_coll                                         # :165-166
        trunc_all = time_limit & ~term_all                                        # :167
        term_all = np.where(no_active, True, term_all)                            # :93-95
        trunc_all = np.where(no_active, False, trunc_all)
        new_act = has_obs.copy()                                                  # :169-172
        stepped = act.copy()
        dist_out = np.where(act, curr, norm1d(goal[:, None, :] - pos))
    else:
        # ---------------- DronePhysicsEnv.step (drone_physics_env.py:279-419), point mass
        p1, v1 = _physics_integrate(cfg, pos, vel, actions, has, damping)        # :323-360
        pos, vel = p1, v1
        stepc = stepc + 1                                                         # :363
        pd = pos.astype(f64) - goal[:, None, :].astype(f64)
        sq = pd * pd
        dist = np.sqrt((sq[..., 0] + sq[..., 1]) + sq[..., 2])                    # :380-381
        coll = pos[..., 2] <= thr["ground"]                                       # :368-372
        if m > 0:
            do = norm_axis(obst[:, None, :, :] - pos[:, :, None, :])
            coll = coll | np.any(do <= thr["phys_obst"], axis=2)
        dpp = norm1d(pos[:, :, None, :] - pos[:, None, :, :])
        coll = coll | np.any(~eye & (dpp <= thr["phys_pair"]), axis=2)
        collided = coll
        reached = dist < float(cfg["goal_radius"])                                # :389, :579
        r = (-dist) * 0.1                                                          # :383
        r = np.where(collided, r - 10.0, np.where(reached, r + 50.0, r))          # :386-392
        reward = np.where(act, r, 0.0)
        any_coll = np.any(act & collided, axis=1)
        all_goals = ~np.any(act & ~collided & ~reached, axis=1)
        time_limit = stepc >= int(cfg["max_steps"])                               # :398
        done = any_coll | all_goals | time_limit                                  # :399
        trunc_all = done & time_limit & ~any_coll & ~all_goals                    # :403-410
        term_all = done & ~trunc_all
        term = np.broadcast_to(term_all[:, None], (e, n)).copy()
        trunc = np.broadcast_to(trunc_all[:, None], (e, n)).copy()
        new_act = act & ~done[:, None]                                            # :411
        stepped = act.copy()
        has_obs = np.ones((e, n), bool)
        dist_out = dist.astype(f32)

    done_env = term_all | trunc_all
    reset = done_env & bool(auto_reset)
    if reset.any():
        ids = np.nonzero(reset)[0]
        episode[ids] = episode[ids] + u32(1)
        rp, ro, rg, rd = device_reset_draws(cfg, env_offset + ids, episode[ids], seed,
                                            physics=physics)
        pos[ids] = rp
        vel[ids] = 0
        goal[ids] = rg
        if m > 0:
            obst[ids] = ro
        if physics:
            damping[ids] = rd
        new_act[ids] = True
        stepc[ids] = 0

    obs = observe(cfg, pos, vel, goal, obst, physics=physics)
    new_state = dict(pos=pos, vel=vel, goal=goal, obst=obst, active=new_act, step=stepc,
                     episode=episode, damping=damping)
    out = dict(obs=obs, reward=reward, terminated=term, truncated=trunc,
               term_all=term_all, trunc_all=trunc_all, reset=reset,
               dist_goal=dist_out.astype(f32), reached=reached, collision=collided,
               stepped=stepped, has_obs=has_obs,
               global_state=global_state(pos, vel, goal))
    return new_state, out


def reset_device(cfg, state, env_mask=None, *, physics=False, seed=0, env_offset=0):
    """swarm_reset: Philox draws for masked envs, then obs (drone_swarm_env.py:65-90)."""
    st = {k: np.array(v, copy=True) for k, v in state.items()}
    e = st["pos"].shape[0]
    mask = np.ones(e, bool) if env_mask is None else np.asarray(env_mask, bool)
    ids = np.nonzero(mask)[0]
    st["episode"][ids] = st["episode"][ids] + u32(1)
    rp, ro, rg, rd = device_reset_draws(cfg, env_offset + ids, st["episode"][ids], seed,
                                        physics=physics)
    st["pos"][ids] = rp
    st["vel"][ids] = 0
    st["goal"][ids] = rg
    if st["obst"].shape[1] > 0:
        st["obst"][ids] = ro
    if physics:
        st["damping"][ids] = rd
    st["active"][ids] = True
    st["step"][ids] = 0
    obs = observe(cfg, st["pos"], st["vel"], st["goal"], st["obst"], physics=physics)
    dist = norm1d(st["goal"][:, None, :] - st["pos"])
    return st, dict(obs=obs, dist_goal=dist, global_state=global_state(st["pos"], st["vel"],
                                                                        st["goal"]))


def empty_state(cfg, e):
    n, m = int(cfg["num_drones"]), int(cfg["num_obstacles"])
    return dict(pos=np.zeros((e, n, 3), f32), vel=np.zeros((e, n, 3), f32),
                goal=np.zeros((e, 3), f32), obst=np.zeros((e, m, 3), f32),
                active=np.ones((e, n), bool), step=np.zeros(e, np.int32),
                episode=np.zeros(e, u32), damping=np.zeros((e, n), f32))
