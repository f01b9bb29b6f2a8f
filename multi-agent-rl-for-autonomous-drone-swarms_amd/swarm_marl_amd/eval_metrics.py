"""On-device evaluation metrics for a VecSwarm.

The reference evaluates one episode at a time on the host: scripts/evaluate_protocol.py:237-331
walks the dict outputs of every step (path length, formation error, collision / all-reached
votes, reward) and :334-350 aggregates the episode summaries into success rate (SR),
collision-free rate (CFR), mean time to goal (TTG), formation error (FE), path efficiency (PE)
and the reward mean / std.  `EvalTracker` accumulates the same per-episode quantities on the
device for all E envs at once (swarm_eval_update, one launch after each step, no host sync) and
aggregates the finished-episode records on the host exactly like `_aggregate`:

    vec = VecSwarm(E, cfg, with_infos=True, auto_reset=True); vec.reset()
    ev = EvalTracker(vec); ev.begin()
    for t in range(T):
        vec.step(policy(vec.obs)); ev.update()
    ev.aggregate()   # {"success_rate": ..., "collision_free_rate": ..., ...}

Semantics kept from the reference, including that the terminal step (no observations,
drone_swarm_env.py:154) counts as "all reached" and carries no collision vote.
"""
from __future__ import annotations

import ctypes
import math
from statistics import mean, pstdev

import numpy as np
import torch

from . import _native as nat
from .vec_env import VecSwarm

FIELDS = ("env", "success", "collision_free", "time_to_goal", "formation_error", "path_efficiency",
          "episode_reward", "steps", "update")


def aggregate_records(rec: np.ndarray) -> dict:
    """evaluate_protocol.py:334-350 `_aggregate` over records [n, >= 8] (FIELDS order)."""
    if len(rec) == 0:
        return {"episodes": 0, "success_rate": 0.0, "collision_free_rate": 0.0, "mean_time_to_goal": math.nan,
                "formation_error": 0.0, "path_efficiency": 0.0, "episode_reward_mean": 0.0,
                "episode_reward_std": 0.0}
    ttg = [float(x) for x in rec[:, 3] if not math.isnan(x)]
    rw = [float(x) for x in rec[:, 6]]
    return {"episodes": int(len(rec)),
            "success_rate": float(mean(int(x) for x in rec[:, 1])),
            "collision_free_rate": float(mean(int(x) for x in rec[:, 2])),
            "mean_time_to_goal": float(mean(ttg)) if ttg else math.nan,
            "formation_error": float(mean(float(x) for x in rec[:, 4])),
            "path_efficiency": float(mean(float(x) for x in rec[:, 5])),
            "episode_reward_mean": float(mean(rw)),
            "episode_reward_std": float(pstdev(rw)) if len(rw) > 1 else 0.0}


class EvalTracker:
    """fused (default "auto"): where the step runs the kinematic swarm_step64 kernel (N = 64,
    K = 3, Ms = 4, no per-env records), the step itself does the whole update (out.eval,
    SWARM_EVAL_STEP_FUSED: swarm_step64_eval_once adds the episode reward, steps, reached step,
    collision vote, path lengths and the exact formation error, and writes the record of every
    episode that ends) — the same records, bit for bit (tests/test_gpu_eval.py) — and update()
    launches nothing: it counts the update (the record's update index).  Every step of the
    VecSwarm then updates, so call update() after every step (as without fusion); `detach()`
    ends the fusion."""

    def __init__(self, vec: VecSwarm, capacity: int = 65536, fused="auto"):
        if vec.info_flags is None:
            raise ValueError("EvalTracker needs a VecSwarm built with with_infos=True")
        if vec.dynamics != "kinematic":
            raise ValueError("EvalTracker follows the kinematic swarm protocol (evaluate_protocol.py)")
        self.vec = vec
        self.lib = vec.lib
        e, n, dev = vec.num_envs, vec.num_drones, vec.device
        f64 = dict(dtype=torch.float64, device=dev)
        self.ep_reward = torch.zeros(e, **f64)
        self.ep_steps = torch.zeros(e, dtype=torch.int32, device=dev)
        self.reached_step = torch.full((e,), -1, dtype=torch.int32, device=dev)
        self.status = torch.zeros(e, dtype=torch.uint8, device=dev)
        self.fe_sum = torch.zeros(e, **f64)
        self.start = torch.zeros((e, n, 3), dtype=torch.float32, device=dev)
        self.goal = torch.zeros_like(self.start)
        self.last = torch.zeros_like(self.start)
        self.traveled = torch.zeros((e, n), **f64)
        seg = nat.EVAL_SEGMENTS
        # segment s holds the episodes of global envs g with g % 64 == s: only min(E, 64) segments
        # are ever written (row blocks (s - seg_base) mod 64 < segments) and the busiest holds
        # ceil(E / 64) envs — every live block is sized for that one's share of `capacity`
        # episodes (capacity * ceil(E/64) / E), so `capacity` finished episodes fit whatever E is
        self.segments = min(e, seg) if e > 0 else seg
        seg_cap = max(1, -(-int(capacity) * (-(-e // seg)) // max(e, 1)))
        self.capacity = self.segments * seg_cap
        self.records_buf = torch.zeros((self.capacity, nat.EVAL_RECORD), **f64)
        self.count = torch.zeros(seg, dtype=torch.int32, device=dev)
        self.seg_base = int(vec.params.env_offset) % seg
        self.updates = 0
        c = nat.SwarmEval()
        for name in ("ep_reward", "ep_steps", "reached_step", "status", "fe_sum", "start", "goal", "last",
                     "traveled", "count"):
            setattr(c, name, getattr(self, name).data_ptr())
        c.records = self.records_buf.data_ptr()
        c.capacity = self.capacity
        c.seg_base, c.segments = self.seg_base, self.segments
        # positions / goal from the state tensors (contiguous) rather than the strided obs rows
        c.state_pos, c.state_goal = vec.pos.data_ptr(), vec.goal.data_ptr()
        self._c = c
        if fused == "auto":
            li = vec.group_launch_info[0]
            fused = (vec.dynamics == "kinematic" and vec.env_cfg is None and int(li.kernel_id) == nat.KERNEL_STEP64)
        self.fused = bool(fused)
        self._step_c = []
        if self.fused:
            c.flags = nat.EVAL_STEP_FUSED
            self._attach()

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.vec.device).cuda_stream

    def _attach(self) -> None:
        """Point every group's step launch at this tracker's accumulators (out.eval): group g's
        struct holds its row offsets (swarm_step_groups offsets group 0's by itself)."""
        vec = self.vec
        prev = getattr(vec, "_eval_owner", None)
        if prev is not None and prev is not self and prev.fused:
            # one fused tracker per VecSwarm: the previous owner goes back to unfused updates
            # (its update() launches swarm_eval_update again), so neither loses records
            prev.detach()
        # copies: _group_c(g) of one group is self._c, whose update index the launches of
        # begin() / update() rewrite
        self._step_c = [nat.SwarmEval.from_buffer_copy(self._group_c(g)) for g in range(vec.groups)]
        for g, sc in enumerate(self._step_c):
            sc.flags = nat.EVAL_STEP_FUSED
            vec._gout[g].eval = ctypes.addressof(sc)
        self._next_index()
        vec._eval_owner = self  # the structs and tensors stay alive while the VecSwarm writes them

    def detach(self) -> None:
        """Stop the fused accumulation (the steps no longer touch this tracker); update() then
        accumulates every per-step term itself again."""
        if not self.fused:
            return
        if getattr(self.vec, "_eval_owner", None) is self:
            # the group structs point at this tracker only while it owns them (a newer fused
            # tracker has re-pointed them: leave those alone)
            for g in range(self.vec.groups):
                self.vec._gout[g].eval = None
            self.vec._eval_owner = None
        self.vec.join()
        self.fused = False
        self._c.flags = 0
        self._step_c = []
        # unfused updates measure path increments from `last`, which the fused steps did not keep:
        # the state positions are where every agent observed next stands now
        self.last.copy_(self.vec.pos)

    def begin(self, env_mask: torch.Tensor | None = None) -> None:
        """Open an episode in the masked envs (all if None) from the current observations."""
        self.vec.join()
        mp = self.vec._mask_ptr(env_mask)
        for g, (lo, _) in enumerate(self.vec.group_slices):
            nat.check(self.lib.swarm_eval_begin(ctypes.byref(self.vec._gparams[g]), ctypes.byref(self._group_c(g)),
                                                ctypes.byref(self.vec._gout[g]), None if mp is None else mp + lo,
                                                self._stream()), self.lib, which="eval")

    def _next_index(self) -> None:
        """The update index the next fused step stamps into the records it closes."""
        for sc in self._step_c:
            sc.update_index = self.updates + 1

    def update(self) -> None:
        """Accumulate the last step (call after every VecSwarm.step)."""
        if self.fused:  # the step did the work
            self.updates += 1
            self._next_index()
            return
        self.vec.join()
        self.updates += 1
        for g in range(self.vec.groups):
            nat.check(self.lib.swarm_eval_update(ctypes.byref(self.vec._gparams[g]), ctypes.byref(self._group_c(g)),
                                                 ctypes.byref(self.vec._gout[g]), self._stream()), self.lib,
                      which="eval")

    def update_group(self, g: int) -> None:
        """Env group g's share of update(), on the current stream and without joining the
        groups: for callers that step each group on its own stream (bench.py --eval) and call
        this after the group's step, for every group once per step, group 0 first."""
        if g == 0:
            self.updates += 1
        if self.fused:
            if g == self.vec.groups - 1:
                self._next_index()
            return
        nat.check(self.lib.swarm_eval_update(ctypes.byref(self.vec._gparams[g]), ctypes.byref(self._group_c(g)),
                                             ctypes.byref(self.vec._gout[g]), self._stream()), self.lib,
                  which="eval")

    def _group_c(self, g: int) -> nat.SwarmEval:
        self._c.update_index = self.updates
        if self.vec.groups == 1:
            return self._c
        lo = self.vec.group_slices[g][0]
        c = nat.SwarmEval()
        for name in ("ep_reward", "ep_steps", "reached_step", "status", "fe_sum", "start", "goal", "last",
                     "traveled"):
            t = getattr(self, name)
            setattr(c, name, t.data_ptr() + lo * t.stride(0) * t.element_size())
        c.records, c.count, c.capacity = self.records_buf.data_ptr(), self.count.data_ptr(), self.capacity
        c.update_index = self.updates
        c.flags, c.seg_base, c.segments = self._c.flags, self.seg_base, self.segments
        v = self.vec
        c.state_pos = v.pos.data_ptr() + lo * v.pos.stride(0) * v.pos.element_size()
        c.state_goal = v.goal.data_ptr() + lo * v.goal.stride(0) * v.goal.element_size()
        return c

    def overflowed(self) -> bool:
        """True once a record segment has filled (further episodes of its envs are dropped by
        the kernel): one 256-B device read, for long runs to check every few thousand updates."""
        return int(self.count.max()) > self.capacity // self.segments

    def records(self) -> np.ndarray:
        """Finished-episode records [n, 9] (FIELDS), in completion order: by the update that
        closed them, then by global env index (deterministic)."""
        counts = self.count.cpu().numpy().astype(np.int64)
        seg_cap = self.capacity // self.segments
        if counts.max(initial=0) > seg_cap:
            raise RuntimeError(f"{int(counts.max())} episodes finished in one record segment, which holds "
                               f"{seg_cap} (EvalTracker capacity {self.capacity}); raise the capacity")
        buf = self.records_buf.cpu().numpy()
        blocks = []
        for s, c in enumerate(counts):
            if c:
                b = (s - self.seg_base) % nat.EVAL_SEGMENTS  # < segments for every written segment
                blocks.append(buf[b * seg_cap:b * seg_cap + int(c)])
        rec = np.concatenate(blocks, axis=0) if blocks else np.zeros((0, nat.EVAL_RECORD))
        return rec[np.lexsort((rec[:, 0], rec[:, 8]))]

    def aggregate(self) -> dict:
        return aggregate_records(self.records())

    def clear(self) -> None:
        self.count.zero_()


class SingleAgentEvalTracker(EvalTracker):
    """scripts/evaluate_protocol.py:193-234 (`_run_single_episode_single_agent`) for E
    single-drone envs at once — the SingleDroneEnv protocol, on the device:

        vec = VecSwarm(E, cfg, num_drones=1, with_infos=True, auto_reset=False)  # cfg neighbor_k=0
        vec.reset(); ev = SingleAgentEvalTracker(vec); ev.begin()
        for t in range(T):
            vec.step(policy(vec.obs)); ev.update()   # closes episodes, resets and reopens those envs
        ev.aggregate()

    Unlike the swarm protocol the terminal step's info and position count (SingleDroneEnv emits
    them), so SR = 0 / CFR = 0 / NaN TTG episodes occur.  The env must not auto-reset (the
    terminal position must still be in the state): `update()` runs swarm_eval_single_update,
    which closes the finished episodes and flags them, then swarm_reset and swarm_eval_begin of
    exactly those envs — three launches, no host sync."""

    def __init__(self, vec: VecSwarm, capacity: int = 65536):
        if vec.num_drones != 1 or int(vec.cfg.neighbor_k) != 0:
            raise ValueError("SingleAgentEvalTracker needs a single-drone VecSwarm (num_drones=1, neighbor_k=0)")
        if int(vec.params.auto_reset):
            raise ValueError("SingleAgentEvalTracker needs auto_reset=False (it resets the finished envs itself)")
        if vec.groups != 1:
            raise ValueError("SingleAgentEvalTracker runs on one env group")
        super().__init__(vec, capacity)
        self.reset_mask = torch.zeros(vec.num_envs, dtype=torch.uint8, device=vec.device)

    def update(self) -> None:
        """Accumulate the last step; finished episodes are recorded, reset and reopened."""
        v = self.vec
        self.updates += 1
        self._c.update_index = self.updates
        nat.check(self.lib.swarm_eval_single_update(ctypes.byref(v._gparams[0]), ctypes.byref(self._c),
                                                    ctypes.byref(v._gout[0]), self.reset_mask.data_ptr(),
                                                    self._stream()), self.lib, which="eval")
        v.reset(env_mask=self.reset_mask)
        self.begin(env_mask=self.reset_mask)
