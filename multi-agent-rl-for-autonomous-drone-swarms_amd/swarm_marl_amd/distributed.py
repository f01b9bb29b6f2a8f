"""Env-parallel sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

The E envs are independent: rank r of P owns the contiguous block
[offset_r, offset_r + E_r) and steps it with no collective on the step path.  The device-reset
RNG is keyed by the GLOBAL env index (env_offset), so a sharded run draws the same episodes as a
single-GPU run of the whole batch.  The only exchange is the optional CTDE `global_state`
all-gather (all_gather_into_tensor; backend "nccl" is RCCL on ROCm).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(num_envs_global: int, world_size: int, rank: int) -> tuple[int, int]:
    """(env_offset, local_count) of `rank` for a contiguous balanced split."""
    if world_size < 1 or not (0 <= rank < world_size):
        raise ValueError(f"bad rank {rank} / world_size {world_size}")
    base, rem = divmod(int(num_envs_global), int(world_size))
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


class GlobalStateGather:
    """Periodic CTDE global_state all-gather, overlapped with the steps that follow it.

    The reference builds the critic input per step (drone_swarm_env.py:293-302, collected into
    the batch by training/callbacks.py:14-57; global_state_dim = 6N+3, config_builders.py:164).
    Here each step writes the state into slot k % R of a device ring `ring` [R, E_local, 6N+3]
    (`select_slot(i)` points the next launch at slot i: VecSwarm.select_global_state_slot).  A
    gather step's slot is all-gathered on a side stream once that step's launches are done,
    while the next steps run on their own streams; only the step that next rewrites the slot
    (R steps later) waits for the gather.  With R = 1 and no side stream this degenerates to
    the synchronous join-then-gather.

    Backends: "nccl" (RCCL over xGMI) gathers device tensors directly.  "gloo" (the CPU test
    backend and bench.py's one-GPU rehearsal) gathers host tensors: a device ring is staged
    through pinned host memory on the side stream (synchronously, so no overlap there).
    A CPU ring (tests) is gathered in place.

    Side stream (`stream`): "auto" (default) issues the gathers from the device's default stream
    when no step launches on it (the env-group case), else from a new stream.  A rank then keeps
    to the default stream, the G group streams and RCCL's own stream — 4 with 2 groups, within
    the box's GPU_MAX_HW_QUEUES = 4 (a fifth active stream shares a hardware queue and
    serialises behind it).  Anything else the caller queues on the side stream orders after the
    gathers issued before it.  "new" forces a fresh stream; a torch.cuda.Stream is used as given.

    Usage per step k:  g.before_step(streams); <launch step k on streams>; g.after_step(streams, k in sched)
    then g.wait() before reading `g.result(i)` of the i-th gather on the current stream.
    Buffer reuse: gather i + keep overwrites gather i's buffer.  It is ordered after every read
    queued, before it is issued (host order), on a stream that called wait() or result():
    each such stream records an event at that point and the side stream waits for it.
    """

    def __init__(self, ring: torch.Tensor, select_slot, *, group=None, keep: int = 2, stream="auto"):
        if ring.dim() != 3:
            raise ValueError("ring must be [slots, E_local, F]")
        self.ring, self.select_slot, self.group = ring, select_slot, group
        self.slots = int(ring.shape[0])
        self.dist = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.dist else 1
        self.backend = dist.get_backend(group) if self.dist else None
        self.cuda = ring.is_cuda
        self.staged = self.cuda and self.backend == "gloo"
        e, f = int(ring.shape[1]), int(ring.shape[2])
        # `keep` result buffers, used round robin: gather i lands in outs[i % keep]
        self.outs = [torch.empty((self.world * e, f), dtype=ring.dtype, device=ring.device)
                     for _ in range(max(1, keep))]
        self.k = 0        # steps seen
        self.count = 0    # gathers issued
        self.gathered_steps: list[int] = []
        if self.cuda:
            if not (stream in ("auto", "new") or isinstance(stream, torch.cuda.Stream)):
                raise ValueError(f"stream must be 'auto', 'new' or a torch.cuda.Stream, not {stream!r}")
            self._stream_mode = stream
            # the side stream: chosen at the first gather ("auto" needs the launch streams)
            self.stream = stream if isinstance(stream, torch.cuda.Stream) else None
            self._consumers: list = []  # streams that results were handed to (wait / result)
            self._consumer_evs: list = []
            self.slot_done = [torch.cuda.Event() for _ in range(self.slots)]
            self.slot_pending = [False] * self.slots
            self._step_evs: list = []
            if self.staged:
                self.h_in = torch.empty((e, f), dtype=ring.dtype).pin_memory()
                self.h_out = torch.empty((self.world * e, f), dtype=ring.dtype)

    def before_step(self, streams=()) -> int:
        """Point the next step at its slot; the streams that will rewrite a slot still being
        gathered wait for that gather first.  Returns the slot."""
        s = self.k % self.slots
        if self.cuda and self.slot_pending[s]:
            for st in streams:
                st.wait_event(self.slot_done[s])
            self.slot_pending[s] = False
        self.select_slot(s)
        return s

    def before_steps(self, n: int, streams=()) -> None:
        """before_step for the next n steps launched as one unit (a replayed graph segment that
        writes slots k .. k + n - 1 mod R, its slots baked in at capture): the streams wait for the
        pending gather of every one of those slots.  Follow with n after_step calls."""
        for i in range(n):
            s = (self.k + i) % self.slots
            if self.cuda and self.slot_pending[s]:
                for st in streams:
                    st.wait_event(self.slot_done[s])
                self.slot_pending[s] = False

    def after_step(self, streams=(), gather: bool = False) -> None:
        """Called after step k's launches were issued on `streams`; gathers its slot if asked."""
        s = self.k % self.slots
        step = self.k
        self.k += 1
        if not gather:
            return
        out = self.outs[self.count % len(self.outs)]
        self.count += 1
        self.gathered_steps.append(step)
        src = self.ring[s]
        if not self.cuda:
            self._gather(out, src)
            return
        if self.stream is None:
            self.stream = self._pick_stream(streams)
        if self.count > len(self.outs):
            # `out` held gather count - 1 - keep: reads of it queued so far on the consumer
            # streams finish before the gather rewrites it
            for st, ev in zip(self._consumers, self._consumer_evs):
                ev.record(st)
                self.stream.wait_event(ev)
        while len(self._step_evs) < len(streams):
            self._step_evs.append(torch.cuda.Event())
        for st, ev in zip(streams, self._step_evs):
            ev.record(st)
            self.stream.wait_event(ev)
        with torch.cuda.stream(self.stream):
            if self.staged:  # gloo: host tensors only
                self.h_in.copy_(src, non_blocking=True)
                self.stream.synchronize()
                self._gather(self.h_out, self.h_in)
                out.copy_(self.h_out, non_blocking=True)
            else:
                self._gather(out, src)
            self.slot_done[s].record(self.stream)
        self.slot_pending[s] = True

    def _gather(self, out: torch.Tensor, src: torch.Tensor) -> None:
        if self.dist:  # the collective even for one rank (the -m gpu test drives RCCL this way)
            dist.all_gather_into_tensor(out, src, group=self.group)
        else:
            out.copy_(src, non_blocking=True)

    def _pick_stream(self, streams) -> "torch.cuda.Stream":
        if self._stream_mode == "auto" and not self.staged:
            dflt = torch.cuda.default_stream(self.ring.device)
            if all(st != dflt for st in streams):
                return dflt
        return torch.cuda.Stream(self.ring.device)

    def _consumer(self) -> None:
        """Register the current stream as a reader of the results (see the class doc)."""
        if not self.cuda:
            return
        cur = torch.cuda.current_stream(self.ring.device)
        if self.stream is not None and cur == self.stream:
            return  # reads on the side stream are ordered before its next gather anyway
        if all(cur != st for st in self._consumers):
            self._consumers.append(cur)
            self._consumer_evs.append(torch.cuda.Event())

    def wait(self) -> None:
        """Make the current stream wait for every gather issued so far."""
        if self.cuda:
            self._consumer()
            if self.stream is not None:
                torch.cuda.current_stream(self.ring.device).wait_stream(self.stream)

    def result(self, i: int = -1) -> torch.Tensor:
        """Buffer of gather i (default: the latest).  Reads of it queued on the current stream
        before gather i + keep is issued are ordered before that gather overwrites it."""
        if self.count == 0:
            raise RuntimeError("no gather issued yet")
        i = self.count - 1 if i < 0 else i
        if not self.count - len(self.outs) <= i < self.count:
            raise IndexError(f"gather {i} was overwritten (keep={len(self.outs)})")
        self._consumer()
        return self.outs[i % len(self.outs)]


def gather_global_state(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather the per-env CTDE critic input [E_local, 6N+3] into [E_global, 6N+3].

    Requires equal local batch sizes (weak-scaling shards).  One collective per call — gather
    every K steps or at batch boundaries."""
    if not dist.is_available() or not dist.is_initialized():
        return local
    ws = dist.get_world_size(group)
    out = torch.empty((ws * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out
