"""VecSwarm — E independent swarm envs stepped by one HIP kernel launch per call.

This is the throughput API the dict-API envs (envs/*.py) sit on.  All state and outputs are
PyTorch tensors resident in HBM; a step is ONE asynchronous launch on the current HIP stream with
no host synchronisation.  Output tensors are persistent buffers overwritten by the next call
(clone them to keep them).

Semantics per env follow DroneSwarmEnv.step (src/swarm_marl/envs/drone_swarm_env.py:92-174) in
"kinematic" mode and DronePhysicsEnv.step (src/swarm_marl/envs/drone_physics_env.py:279-419,
point-mass restatement) in "physics" mode.  With auto_reset=True an env whose episode ended is
re-drawn in the same launch (Philox stream keyed by seed, global env index and episode number);
`obs` then holds the new episode's first observation — the reference emits no terminal obs
(drone_swarm_env.py:154), so nothing is lost.  env_done carries terminated/truncated["__all__"]
and a RESET bit.

Env groups (`groups=G`): the E envs are split into G contiguous blocks, each stepped by its own
launch on its own HIP stream (`group_streams`).  Envs are independent, so a group's step k+1
needs only that group's step k: with `step(..., join=False)` (or `step_group` on the group
streams) the launches of different groups overlap, and one group's load burst and completion
tail run under another group's steady state instead of idling the CUs.  Every env is still
stepped exactly once per step; results are bitwise those of G = 1 (the reset RNG is keyed by the
global env index).
"""
from __future__ import annotations

import ctypes
from dataclasses import asdict
from typing import Any

import torch

from . import _native as nat
from .envs.common import DroneEnvConfig

PHYSICS_DEFAULTS = dict(gravity=-9.81, gravity_comp=9.5, substep_dt=1.0 / 240.0,
                        drone_contact_radius=0.15, ground_contact_height=0.025, damping_law=0)


# torch's raw current-stream handle (what torch.cuda.current_stream(d).cuda_stream returns,
# without constructing a Stream object); the public call is the fallback
_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


# mapped packed I/O is for dict-API sized batches (one env of a few drones): the kernel's reads
# and writes then cross the host link, which only pays when the copies' fixed costs dominate
MAPPED_IO_MAX_AGENTS = 1024
_HIP = None


def _device_mapped(host_ptr: int) -> bool:
    """True when the HIP runtime maps this pinned host allocation into the device address space
    at the same address (hipHostGetDevicePointer), i.e. a kernel may dereference host_ptr."""
    global _HIP
    try:
        if _HIP is None:
            _HIP = ctypes.CDLL("libamdhip64.so")
            _HIP.hipHostGetDevicePointer.restype = ctypes.c_int
            _HIP.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                                     ctypes.c_uint]
        d = ctypes.c_void_p()
        rc = _HIP.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(host_ptr), 0)
        return rc == 0 and d.value == host_ptr
    except (OSError, AttributeError):
        return False


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


class VecSwarm:
    def __init__(self, num_envs: int, config: dict[str, Any] | DroneEnvConfig | None = None, *,
                 num_drones: int | None = None, dynamics: str = "kinematic",
                 auto_reset: bool = True, seed: int = 0, env_offset: int = 0,
                 device: str | torch.device | None = None, with_infos: bool = False,
                 with_global_state: bool = False, physics: dict[str, Any] | None = None,
                 kernel_path: str = "auto", persistent: bool = True, waves_per_simd: int = 0,
                 groups: int = 1, packed_io: bool = False, global_state_slots: int = 1):
        if isinstance(config, DroneEnvConfig):
            cfg, raw = config, {}
        else:
            raw = dict(config or {})
            cfg = DroneEnvConfig.from_dict({k: v for k, v in raw.items() if k != "num_drones"})
        n = int(num_drones if num_drones is not None else raw.get("num_drones", 3))
        if dynamics not in ("kinematic", "physics"):
            raise ValueError(f"dynamics must be 'kinematic' or 'physics', got {dynamics!r}")
        self.cfg = cfg
        self.num_envs = int(num_envs)
        self.num_drones = n
        self.dynamics = dynamics
        self.lib = nat.load_library()
        if device is None:
            if not torch.cuda.is_available():
                raise RuntimeError("VecSwarm needs a ROCm GPU (gfx950); none is visible")
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("VecSwarm state must live on a GPU device ('cuda' on ROCm)")

        phys = dict(PHYSICS_DEFAULTS)
        phys.update(physics or {})
        p = nat.SwarmParams()
        self.lib.swarm_params_default(ctypes.byref(p))
        p.num_envs = self.num_envs
        p.num_drones = n
        p.num_obstacles = int(cfg.num_obstacles)
        p.sensed_obstacles = int(cfg.sensed_obstacles)
        p.neighbor_k = int(cfg.neighbor_k)
        p.max_steps = int(cfg.max_steps)
        p.dynamics = nat.DYN_KINEMATIC if dynamics == "kinematic" else nat.DYN_POINTMASS_PHYSICS
        p.reward_mode = nat.REW_SWARM if dynamics == "kinematic" else nat.REW_PHYSICS
        p.auto_reset = 1 if auto_reset else 0
        p.physics_substeps = int(phys.get("substeps", int(float(cfg.dt) * 240)))  # :323
        p.damping_law = int(phys["damping_law"])
        p.env_offset = int(env_offset)
        p.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        if kernel_path not in ("auto", "generic"):
            raise ValueError(f"kernel_path must be 'auto' or 'generic', got {kernel_path!r}")
        p.kernel_path = nat.PATH_AUTO if kernel_path == "auto" else nat.PATH_GENERIC
        if not 0 <= int(waves_per_simd) <= 8:
            raise ValueError(f"waves_per_simd must be in [0, 8], got {waves_per_simd}")
        p.waves_per_simd = int(waves_per_simd)
        self.persistent = bool(persistent)
        for name in ("world_size", "dt", "max_speed", "max_accel", "collision_radius",
                     "goal_radius", "obstacle_radius", "desired_spacing", "reward_progress_scale",
                     "reward_goal", "reward_collision", "reward_formation_scale"):
            setattr(p, name, float(getattr(cfg, name)))
        for name in ("gravity", "gravity_comp", "substep_dt", "drone_contact_radius",
                     "ground_contact_height"):
            setattr(p, name, float(phys[name]))
        self.params = p
        self.launch_info = nat.SwarmLaunchInfo()
        nat.check(self.lib.swarm_query_launch(ctypes.byref(p), ctypes.byref(self.launch_info)),
                  self.lib)
        self.obs_dim = int(self.lib.swarm_obs_dim(ctypes.byref(p)))
        # ---- env groups: contiguous env blocks, one launch (and stream) each
        g_n = int(groups)
        if not 1 <= g_n <= max(1, self.num_envs):
            raise ValueError(f"groups must be in [1, num_envs], got {groups}")
        self.groups = g_n
        q, r = divmod(self.num_envs, g_n)
        bounds = [0]
        for g in range(g_n):
            bounds.append(bounds[-1] + q + (1 if g < r else 0))
        self.group_slices = [(bounds[g], bounds[g + 1]) for g in range(g_n)]
        self._gparams, self.group_launch_info = [], []
        for lo, hi in self.group_slices:
            pg = nat.SwarmParams()
            ctypes.memmove(ctypes.byref(pg), ctypes.byref(p), ctypes.sizeof(p))
            pg.num_envs = hi - lo
            pg.env_offset = int(env_offset) + lo
            li = nat.SwarmLaunchInfo()
            nat.check(self.lib.swarm_query_launch(ctypes.byref(pg), ctypes.byref(li)), self.lib)
            self._gparams.append(pg)
            self.group_launch_info.append(li)
        self.group_streams = ([torch.cuda.Stream(self.device) for _ in range(g_n)]
                              if g_n > 1 else None)
        self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self._swarm_step = self.lib.swarm_step
        self._swarm_step_groups = self.lib.swarm_step_groups
        self._gstream_h = [st.cuda_stream for st in self.group_streams] if self.group_streams else []
        # swarm_step_groups arguments: every group's env count and stream handle
        self._group_envs_c = (ctypes.c_int32 * g_n)(*[hi - lo for lo, hi in self.group_slices])
        self._gstreams_c = (ctypes.c_void_p * g_n)(*self._gstream_h) if g_n > 1 else None
        # fork / join events of the group launches, reused by every step (record overwrites)
        self._fork_ev = torch.cuda.Event() if g_n > 1 else None
        self._join_evs = [torch.cuda.Event() for _ in range(g_n)] if g_n > 1 else []

        e, m, d = self.num_envs, int(cfg.num_obstacles), self.obs_dim
        kw = dict(device=self.device)
        f32 = torch.float32
        # ---- state (SoA blocks, [E, ...] contiguous)
        self.pos = torch.zeros((e, n, 3), dtype=f32, **kw)
        self.vel = torch.zeros((e, n, 3), dtype=f32, **kw)
        self.goal = torch.zeros((e, 3), dtype=f32, **kw)
        self.obstacles = torch.zeros((e, m, 3), dtype=f32, **kw)
        # packed_io (the dict-API envs): the per-step inputs (an actions buffer and the active
        # mask) and all outputs are views of two flat device arenas, so that one step moves one
        # H2D and one D2H copy (in_layout / out_layout: name -> (byte offset, shape, dtype))
        if packed_io not in (False, True, "mapped"):
            raise ValueError(f"packed_io must be False, True or 'mapped', got {packed_io!r}")
        self.packed_io = bool(packed_io)
        # "mapped": the arenas are pinned host memory the kernel reads and writes in place (the
        # device address of a pinned allocation is its host address), so a dict-API step moves
        # no copies at all: the host fills the inputs, launches, synchronises and reads the
        # outputs.  Used only when the runtime confirms the mapping; otherwise device arenas.
        self.mapped_io = packed_io == "mapped" and self.num_envs * n <= MAPPED_IO_MAX_AGENTS
        self.in_arena = self.out_arena = None
        self.in_layout, self.out_layout = {}, {}
        if self.packed_io:
            self.in_arena, views = self._arena(self.in_layout, [
                ("actions", (e, n, 3), f32), ("active", (e, n), torch.bool),
                ("action_mask", (e, n), torch.uint8)], self.device, self.mapped_io)
            self.mapped_io = self.in_arena.device.type == "cpu"
            self.actions_in = views["actions"]
            self.action_mask_in = views["action_mask"]
            self.active = views["active"]
            self.active.fill_(True)
        else:
            self.actions_in = self.action_mask_in = None
            self.active = torch.ones((e, n), dtype=torch.bool, **kw)
        self.step_count = torch.zeros((e,), dtype=torch.int32, **kw)
        self.episode = torch.zeros((e,), dtype=torch.int32, **kw)  # read as uint32 by the kernel
        self.damping = torch.zeros((e, n), dtype=f32, **kw)
        # env-queue heads of the persistent step kernel, one row per group (zero, and left
        # zero by every launch)
        self.work = (torch.zeros((self.groups, nat.WORK_WORDS), dtype=torch.int32, **kw)
                     if self.persistent else None)
        # per-env parameter records ([E, 64] bytes of swarm_env_cfg_t; set_env_config)
        self.env_cfg = self.env_cfg_next = None
        # ---- outputs (persistent buffers)
        outs = [("obs", (e, n, d), f32), ("reward", (e, n), f32)]
        if with_infos:
            outs.append(("dist_goal", (e, n), f32))
        # global_state ring (CTDE gather overlap, distributed.GlobalStateGather): the step writes
        # slot `global_state_slot` of global_state_ring [R, E, 6N+3]; `global_state` is that slot
        self.global_state_ring = None
        self.global_state_slot = 0
        gs_slots = int(global_state_slots)
        if gs_slots < 1:
            raise ValueError(f"global_state_slots must be >= 1, got {global_state_slots}")
        if with_global_state and gs_slots > 1:
            if packed_io:
                raise ValueError("global_state_slots > 1 is not supported with packed_io")
            self.global_state_ring = torch.zeros((gs_slots, e, 6 * n + 3), dtype=f32, **kw)
        elif with_global_state:
            outs.append(("global_state", (e, 6 * n + 3), f32))
        outs += [("terminated", (e, n), torch.bool), ("truncated", (e, n), torch.bool),
                 ("env_done", (e,), torch.uint8)]
        if with_infos:
            outs.append(("info_flags", (e, n), torch.uint8))
        if self.packed_io:
            self.out_arena, views = self._arena(self.out_layout, outs, self.device, self.mapped_io)
            self.mapped_io = self.mapped_io and self.out_arena.device.type == "cpu"
        else:
            views = {name: torch.zeros(shape, dtype=dt, **kw) for name, shape, dt in outs}
        for name in ("obs", "reward", "terminated", "truncated", "env_done", "dist_goal",
                     "info_flags", "global_state"):
            setattr(self, name, views.get(name))
        if self.global_state_ring is not None:
            self.global_state = self.global_state_ring[0]
        self._bind()

    def close(self) -> None:
        """Wait for every launch that may still use this batch's buffers.  Needed for mapped
        arenas: they are blocks of torch's pinned-host caching allocator that the kernels use
        behind torch's back (no stream use is recorded on them), so dropping the VecSwarm while a
        step is in flight could hand a block that a kernel still writes to another pinned copy.
        Called by __del__ for mapped batches; device-resident batches need nothing."""
        if not getattr(self, "mapped_io", False):
            return
        try:
            torch.cuda.synchronize(self.device)
        except Exception:  # interpreter shutdown: the runtime may already be gone
            pass

    def __del__(self):
        self.close()

    # ------------------------------------------------------------------ plumbing
    @staticmethod
    def _arena(layout: dict, fields, device, mapped: bool = False):
        """One zeroed uint8 buffer holding `fields` (name, shape, dtype) at 16-B aligned offsets;
        returns (buffer, {name: typed view}) and fills `layout`.  mapped: pinned host memory
        whose device address equals its host address (else a device buffer)."""
        off = 0
        for name, shape, dt in fields:
            nbytes = torch.Size(shape).numel() * torch.empty((), dtype=dt).element_size()
            layout[name] = (off, tuple(shape), dt)
            off += (nbytes + 15) // 16 * 16
        buf = None
        if mapped:
            buf = torch.zeros((max(off, 16),), dtype=torch.uint8).pin_memory()
            if not _device_mapped(buf.data_ptr()):
                buf = None
        if buf is None:
            buf = torch.zeros((max(off, 16),), dtype=torch.uint8, device=device)
        return buf, VecSwarm.arena_views(buf, layout)

    @staticmethod
    def arena_views(buf: torch.Tensor, layout: dict) -> dict:
        """Typed views of an arena laid out by `layout` (device arena or a host mirror of it)."""
        out = {}
        for name, (off, shape, dt) in layout.items():
            nbytes = torch.Size(shape).numel() * torch.empty((), dtype=dt).element_size()
            out[name] = buf[off:off + nbytes].view(dt).view(shape)
        return out

    def _bind(self) -> None:
        """ctypes state/out blocks per group: row `lo` of every [E, ...] tensor onwards."""
        def off(t, lo):
            return None if t is None else t.data_ptr() + lo * t.stride(0) * t.element_size()

        self._gstate, self._gout = [], []
        for g, (lo, _) in enumerate(self.group_slices):
            s = nat.SwarmState()
            s.pos, s.vel, s.goal = off(self.pos, lo), off(self.vel, lo), off(self.goal, lo)
            s.obstacles = off(self.obstacles, lo) if self.obstacles.numel() else None
            s.active, s.step_count = off(self.active, lo), off(self.step_count, lo)
            s.episode, s.damping = off(self.episode, lo), off(self.damping, lo)
            s.work = None if self.work is None else _ptr(self.work[g])
            s.env_cfg, s.env_cfg_next = off(self.env_cfg, lo), off(self.env_cfg_next, lo)
            o = nat.SwarmOut()
            o.obs, o.reward = off(self.obs, lo), off(self.reward, lo)
            o.terminated, o.truncated = off(self.terminated, lo), off(self.truncated, lo)
            o.env_done = off(self.env_done, lo)
            o.dist_goal, o.info_flags = off(self.dist_goal, lo), off(self.info_flags, lo)
            o.global_state = off(self.global_state, lo)
            self._gstate.append(s)
            self._gout.append(o)
        self._state_c, self._out_c = self._gstate[0], self._gout[0]
        # per-launch plumbing built once (eager steps are host-bound at small E or with groups):
        # the three struct references and each group's row offsets into an [E,N,3] f32 actions
        # tensor / [E,N] u8 action mask (both validated contiguous by _actions)
        self._grefs = [(ctypes.byref(self._gparams[g]), ctypes.byref(self._gstate[g]), ctypes.byref(self._gout[g]))
                       for g in range(self.groups)]
        self._gact_off = [(lo * self.num_drones * 12, lo * self.num_drones) for lo, _ in self.group_slices]

    def select_global_state_slot(self, i: int) -> None:
        """Make the next launches write global_state into slot i of `global_state_ring` (and
        `global_state` that slot).  Launches already issued keep the slot they were given."""
        if self.global_state_ring is None:
            if i != 0:
                raise ValueError("this VecSwarm has one global_state buffer (global_state_slots=1)")
            return
        r = self.global_state_ring
        if not 0 <= i < r.shape[0]:
            raise ValueError(f"global_state slot {i} out of range [0, {r.shape[0]})")
        self.global_state_slot = int(i)
        self.global_state = r[i]
        base = self.global_state.data_ptr()
        row = self.global_state.stride(0) * self.global_state.element_size()
        for g, (lo, _) in enumerate(self.group_slices):
            self._gout[g].global_state = base + lo * row

    def _stream(self) -> int:
        if _RAW_STREAM is not None:  # the raw handle, no Stream object per call
            return _RAW_STREAM(self._dev_index)
        return torch.cuda.current_stream(self.device).cuda_stream

    def _check_tensor(self, name: str, t: torch.Tensor, shape: tuple, dtype) -> None:
        if not isinstance(t, torch.Tensor):
            raise ValueError(f"{name} must be a torch.Tensor")
        if not t.is_cuda or t.get_device() != self._dev_index:
            raise ValueError(f"{name} is on {t.device}, expected {self.device}")
        if t.dtype != dtype:
            raise ValueError(f"{name} has dtype {t.dtype}, expected {dtype}")
        if t.shape != shape:
            raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")

    def _mask_ptr(self, env_mask) -> int | None:
        if env_mask is None:
            return None
        mk = env_mask
        if mk.dtype != torch.uint8:
            mk = mk.to(torch.uint8)
        self._check_tensor("env_mask", mk, (self.num_envs,), torch.uint8)
        self._keep = mk
        return mk.data_ptr()

    # ------------------------------------------------------------------ API
    def _actions(self, actions, action_mask):
        if self.mapped_io and actions is self.actions_in and (action_mask is None or
                                                              action_mask is self.action_mask_in):
            return actions, action_mask  # the mapped arena's own views (host-resident, device-addressable)
        self._check_tensor("actions", actions, (self.num_envs, self.num_drones, 3), torch.float32)
        if action_mask is not None:
            if action_mask.dtype == torch.bool:
                action_mask = action_mask.view(torch.uint8)
            self._check_tensor("action_mask", action_mask, (self.num_envs, self.num_drones),
                               torch.uint8)
        return actions, action_mask

    def _launch_step(self, g: int, actions, action_mask, stream: int) -> None:
        pr, sr, orf = self._grefs[g]
        ao, mo = self._gact_off[g]
        rc = self._swarm_step(pr, sr, actions.data_ptr() + ao,
                              None if action_mask is None else action_mask.data_ptr() + mo, orf, stream)
        if rc:
            nat.check(rc, self.lib)

    def step(self, actions: torch.Tensor, action_mask: torch.Tensor | None = None, *,
             join: bool = True):
        """One step of all envs.  actions [E,N,3] float32 on the device.

        Returns (obs [E,N,D], reward [E,N] f32, terminated [E,N] bool, truncated [E,N] bool,
        env_done [E] u8 bits).  Views into persistent buffers.

        With env groups the launches fork from the current stream onto the group streams; with
        join=False they are not joined back (call `join()` before using the outputs on another
        stream), so consecutive steps of different groups overlap.
        """
        actions, action_mask = self._actions(actions, action_mask)
        if self.groups == 1:
            self._launch_step(0, actions, action_mask, self._stream())
            return self.obs, self.reward, self.terminated, self.truncated, self.env_done
        cur = torch.cuda.current_stream(self.device)
        fork = self._fork_ev
        fork.record(cur)
        for st in self.group_streams:
            st.wait_event(fork)
            if not join:  # the caller's tensors are in use on the group stream
                actions.record_stream(st)
                if action_mask is not None:
                    action_mask.record_stream(st)
        self._launch_groups(actions, action_mask)
        if join:
            self.join()
        return self.obs, self.reward, self.terminated, self.truncated, self.env_done

    def _launch_groups(self, actions, action_mask) -> None:
        pr, sr, orf = self._grefs[0]  # group 0's structs hold the batch's row-0 pointers
        rc = self._swarm_step_groups(ctypes.byref(self.params), sr, actions.data_ptr(),
                                     None if action_mask is None else action_mask.data_ptr(), orf,
                                     self.groups, self._group_envs_c, self._gstreams_c)
        if rc:
            nat.check(rc, self.lib)

    def step_groups(self, actions: torch.Tensor, action_mask: torch.Tensor | None = None):
        """One step of all envs, group g launched on group stream g by one native call
        (swarm_step_groups), with no fork from or join to the current stream: the caller orders
        the group streams after the inputs (e.g. once per rollout, `fork_groups()`) and before
        reading the outputs (`join()`).  Group g's steps follow each other on its stream, and
        groups share no rows, so consecutive steps need no ordering between the streams."""
        actions, action_mask = self._actions(actions, action_mask)
        if self.groups == 1:
            self._launch_step(0, actions, action_mask, self._stream())
        else:
            self._launch_groups(actions, action_mask)
        return self.obs, self.reward, self.terminated, self.truncated, self.env_done

    def fork_groups(self) -> None:
        """Make every group stream wait for the work issued so far on the current stream."""
        if self.group_streams is None:
            return
        self._fork_ev.record(torch.cuda.current_stream(self.device))
        for st in self.group_streams:
            st.wait_event(self._fork_ev)

    def step_group(self, g: int, actions: torch.Tensor, action_mask: torch.Tensor | None = None):
        """Step env group `g` only (rows group_slices[g] of the full-batch tensors) on the
        current stream — e.g. inside `torch.cuda.stream(vec.group_streams[g])` or a hipGraph
        capture on that stream.  actions is the full [E,N,3] tensor."""
        if not 0 <= g < self.groups:
            raise ValueError(f"group {g} out of range [0, {self.groups})")
        actions, action_mask = self._actions(actions, action_mask)
        self._launch_step(g, actions, action_mask, self._stream())
        return self.obs, self.reward, self.terminated, self.truncated, self.env_done

    def join(self) -> None:
        """Make the current stream wait for every group stream."""
        if self.group_streams is None:
            return
        cur = torch.cuda.current_stream(self.device)
        for st, ev in zip(self.group_streams, self._join_evs):
            ev.record(st)
            cur.wait_event(ev)

    def _aux(self, fn, env_mask) -> None:
        self.join()
        mp = self._mask_ptr(env_mask)
        for g, (lo, _) in enumerate(self.group_slices):
            rc = fn(ctypes.byref(self._gparams[g]), ctypes.byref(self._gstate[g]),
                    None if mp is None else mp + lo, ctypes.byref(self._gout[g]), self._stream())
            nat.check(rc, self.lib)

    def reset(self, env_mask: torch.Tensor | None = None) -> torch.Tensor:
        """Device reset (Philox draws) of the masked envs (all if None); returns obs."""
        self._aux(self.lib.swarm_reset, env_mask)
        return self.obs

    def observe(self, env_mask: torch.Tensor | None = None) -> torch.Tensor:
        """obs / dist_goal / global_state of the current state (no state change)."""
        self._aux(self.lib.swarm_observe, env_mask)
        return self.obs

    def set_state(self, *, pos=None, vel=None, goal=None, obstacles=None, active=None,
                  step_count=None, episode=None, damping=None) -> None:
        """Inject state (host or device arrays); shapes as the state tensors."""
        self.join()
        if self.mapped_io:  # `active` lives in the mapped arena: no kernel may still use it
            torch.cuda.current_stream(self.device).synchronize()
        for name, val in (("pos", pos), ("vel", vel), ("goal", goal), ("obstacles", obstacles),
                          ("active", active), ("step_count", step_count),
                          ("episode", episode), ("damping", damping)):
            if val is None:
                continue
            dst = getattr(self, name)
            src = torch.as_tensor(val)
            if tuple(src.shape) != tuple(dst.shape):
                raise ValueError(f"{name}: shape {tuple(src.shape)} != {tuple(dst.shape)}")
            dst.copy_(src.to(dtype=dst.dtype), non_blocking=False)

    # ------------------------------------------------------------------ per-env parameters
    def set_env_config(self, *, env_mask: torch.Tensor | None = None, next_episode: bool = False,
                       **values) -> None:
        """Per-env parameters (curriculum stages and domain randomisation as
        per-env tensors).  `values` maps any of world_size, dt, max_speed, max_accel,
        obstacle_radius (float), max_steps, num_obstacles (int, 0..num_obstacles of the batch) to a
        scalar or an [E] array; unnamed fields take the batch config.  The records of the masked
        envs (all if None) are derived on the device (swarm_env_cfg_set, no host sync).

        next_episode=False sets the CURRENT parameters (they apply from the next step / reset on;
        a curriculum mix keeps them across resets).  next_episode=True sets the parameters each
        env's NEXT episode starts with: every reset (auto or explicit) copies them in — the hook
        for per-episode randomisation (domain_randomization.py).  The step then runs the generic
        kernel."""
        unknown = set(values) - set(nat.ENV_OVERRIDE_FIELDS)
        if unknown:
            raise ValueError(f"unknown per-env parameters {sorted(unknown)}; "
                             f"supported: {nat.ENV_OVERRIDE_FIELDS}")
        if self.dynamics == "physics" and values.get("dt") is not None:
            raise ValueError("per-env dt applies to the kinematic integrator only (physics substeps are "
                             "uniform)")
        e = self.num_envs
        self.join()
        owner = getattr(self, "_eval_owner", None)
        if owner is not None and owner.fused:
            # per-env records move the step to the generic kernel, which has no fused eval: the
            # tracker goes back to unfused updates (its update() launches swarm_eval_update)
            owner.detach()
        rebind = False
        if self.env_cfg is None:
            self.env_cfg = torch.zeros((e, nat.ENV_CFG_BYTES), dtype=torch.uint8, device=self.device)
            self._env_cfg_write(self.env_cfg, {}, None)  # uniform records first
            rebind = True
        if next_episode and self.env_cfg_next is None:
            self.env_cfg_next = torch.zeros_like(self.env_cfg)
            self.env_cfg_next.copy_(self.env_cfg)
            rebind = True
        if rebind:
            self._bind()
        self._env_cfg_write(self.env_cfg_next if next_episode else self.env_cfg, values, env_mask)

    def _env_cfg_write(self, dst: torch.Tensor, values: dict, env_mask) -> None:
        e = self.num_envs
        ov = nat.SwarmEnvOverrides()
        keep = []
        for name in nat.ENV_OVERRIDE_FIELDS:
            v = values.get(name)
            if v is None:
                continue
            dt = torch.int32 if name in ("max_steps", "num_obstacles") else torch.float64
            t = torch.as_tensor(v, dtype=dt).to(self.device)
            if t.dim() == 0:
                t = t.expand(e)
            if tuple(t.shape) != (e,):
                raise ValueError(f"{name}: expected a scalar or shape ({e},), got {tuple(t.shape)}")
            t = t.contiguous()
            keep.append(t)
            setattr(ov, name, t.data_ptr())
        mp = self._mask_ptr(env_mask)
        for g, (lo, hi) in enumerate(self.group_slices):
            og = nat.SwarmEnvOverrides()
            for name in nat.ENV_OVERRIDE_FIELDS:
                ptr = getattr(ov, name)
                setattr(og, name, None if ptr is None else ptr + lo * (4 if name in ("max_steps", "num_obstacles")
                                                                        else 8))
            rc = self.lib.swarm_env_cfg_set(ctypes.byref(self._gparams[g]), ctypes.byref(og),
                                            None if mp is None else mp + lo,
                                            dst.data_ptr() + lo * nat.ENV_CFG_BYTES, self._stream())
            nat.check(rc, self.lib)
        self._keep_cfg = keep  # the launches read them asynchronously

    def env_config(self, next_episode: bool = False) -> dict[str, torch.Tensor] | None:
        """Per-env parameters as [E] tensors (views of the records), or None if unset."""
        rec = self.env_cfg_next if next_episode else self.env_cfg
        if rec is None:
            return None
        f = rec.view(torch.float32)
        i = rec.view(torch.int32)
        d = rec.view(torch.float64)
        return dict(world_size=d[:, 7], dt=f[:, 3], max_speed=d[:, 6], max_accel=f[:, 5],
                    max_steps=i[:, 9], num_obstacles=i[:, 10], half_w=f[:, 0], s_obst=f[:, 7])

    def state_dict(self) -> dict[str, torch.Tensor]:
        return dict(pos=self.pos, vel=self.vel, goal=self.goal, obstacles=self.obstacles,
                    active=self.active, step_count=self.step_count, episode=self.episode,
                    damping=self.damping)

    @property
    def config(self) -> dict[str, Any]:
        d = asdict(self.cfg)
        d["num_drones"] = self.num_drones
        return d

    def kernel_name(self) -> str:
        """Kernel the step launches: the headline specialisation swarm_step64_once<32, 4> (one
        wave per env, 4 per workgroup; swarm_step64_phys_once<32, 4> in physics mode) or its persistent form swarm_step64<32> (E larger than
        the resident grid, env queues in `work`), else the generic swarm_kernel<KIND, DYN, KS,
        MSL, LM> (KIND 0 = step; LM lane mode 0 block / 1 multi-team wave / 2 one team per wave).
        With env groups: the kernel of group 0."""
        li = self.group_launch_info[0]
        kid = int(li.kernel_id)
        if self.env_cfg is not None:
            # per-env parameters: launch() always takes the generic kernel, whose geometry the
            # AUTO query does not describe (it reports the specialisation's) — query it as such
            gp = nat.SwarmParams.from_buffer_copy(self._gparams[0])
            gp.kernel_path = nat.PATH_GENERIC
            li = nat.SwarmLaunchInfo()
            nat.check(self.lib.swarm_query_launch(ctypes.byref(gp), ctypes.byref(li)), self.lib)
            kid = nat.KERNEL_GENERIC
        if kid == nat.KERNEL_STEP64_PERSISTENT and self.persistent:
            return "swarm_step64<32>"
        if kid == nat.KERNEL_STEP16Q:
            return "swarm_step16q"
        if kid == nat.KERNEL_STEP256:  # 512 threads: the two-waves-per-block build (swarm_step256w)
            return "swarm_step256w" if int(li.threads_per_block) == 512 else "swarm_step256"
        if kid in (nat.KERNEL_STEP64, nat.KERNEL_STEP64_PERSISTENT):
            return "swarm_step64_phys_once<32, 4>" if self.dynamics == "physics" else "swarm_step64_once<32, 4>"
        lanes = int(li.lanes_per_env)
        lm = 0 if lanes > 64 else (2 if lanes == 64 else 1)
        return (f"swarm_kernel<0, {int(self.params.dynamics)}, {int(li.neighbor_slots)}, "
                f"{int(li.obstacle_slots)}, {lm}>")

    def algorithmic_bytes_per_step(self) -> int:
        """HBM bytes one step must move: per agent action 12 + pos/vel r/w 48 +
        active r/w 2 + obs 4D + reward 4 + terminated/truncated 2; per env goal 12 + obstacles
        12M + step r/w 8 + env_done 1 (+ optional infos / global_state)."""
        n, e, d, m = self.num_drones, self.num_envs, self.obs_dim, int(self.cfg.num_obstacles)
        per_agent = 12 + 48 + 2 + 4 * d + 4 + 2
        per_env = 12 + 12 * m + 8 + 1
        extra = 0
        if self.dist_goal is not None:
            per_agent += 5
        if self.global_state is not None:
            extra = e * (6 * n + 3) * 4
        if self.dynamics == "physics":
            per_agent += 4
        return e * (n * per_agent + per_env) + extra
