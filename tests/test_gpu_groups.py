"""GPU: env groups (VecSwarm groups=G) — G contiguous env blocks stepped by G launches on G HIP
streams — are bitwise the single-launch run: obs, reward, flags, infos, global_state and state,
over steps with in-kernel resets, whether the steps join back per step, overlap (join=False),
or replay per-group hipGraphs on the group streams (the bench's timed path).
Reference semantics per env: src/swarm_marl/envs/drone_swarm_env.py:92-174.
"""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _pair(dev, e, n, g, **kw):
    from swarm_marl_amd import VecSwarm
    base = dict(device=dev, auto_reset=True, seed=13, with_infos=True, with_global_state=True, **kw)
    a = VecSwarm(e, {"num_drones": n}, **base)
    b = VecSwarm(e, {"num_drones": n}, groups=g, **base)
    a.reset()
    b.reset()
    return a, b


def _fields(v):
    return (v.obs, v.reward, v.terminated, v.truncated, v.env_done, v.dist_goal, v.info_flags,
            v.global_state, v.pos, v.vel, v.goal, v.obstacles, v.active, v.step_count, v.episode)


def _same(a, b, tag):
    for i, (x, y) in enumerate(zip(_fields(a), _fields(b))):
        assert torch.equal(x, y), (tag, i)


def _acts(dev, e, n, k):
    g = torch.Generator(device=dev).manual_seed(500 + k)
    return torch.rand((e, n, 3), device=dev, generator=g) * 2 - 1


@pytest.mark.parametrize("e,n,g", [(8192, 64, 4), (1000, 16, 3), (257, 64, 2), (96, 256, 4), (10, 5, 10)])
def test_groups_equal_single_launch(dev, e, n, g):
    a, b = _pair(dev, e, n, g)
    assert b.groups == g and sum(hi - lo for lo, hi in b.group_slices) == e
    _same(a, b, "reset")
    for k in range(8):
        act = _acts(dev, e, n, k)
        a.step(act)
        b.step(act, join=(k % 3 == 0))
        b.join()
        _same(a, b, k)
    assert int((a.env_done & 4).sum()) > 0 or n < 16  # resets happened in the compared steps


def test_groups_overlapped_graph_replay(dev):
    """Per-group hipGraphs on the group streams, replayed interleaved without per-step joins."""
    e, n, g, ring = 4096, 64, 4, 4
    a, b = _pair(dev, e, n, g)
    acts = [_acts(dev, e, n, k) for k in range(ring)]
    torch.cuda.synchronize()
    graphs = []
    for gi, st in enumerate(b.group_streams):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st), torch.cuda.graph(gr, stream=st):
            for k in range(ring):
                b.step_group(gi, acts[k])
        graphs.append(gr)
    torch.cuda.synchronize()  # capture runs nothing: a and b are still at the same reset state
    cur = torch.cuda.current_stream(dev)
    start = torch.cuda.Event()
    start.record(cur)
    for st in b.group_streams:
        st.wait_event(start)
    for _ in range(3):
        for gi, st in enumerate(b.group_streams):
            with torch.cuda.stream(st):
                graphs[gi].replay()
        for k in range(ring):
            a.step(acts[k])
    b.join()
    torch.cuda.synchronize()
    _same(a, b, "graph")


def test_groups_validation(dev):
    from swarm_marl_amd import VecSwarm
    with pytest.raises(ValueError):
        VecSwarm(4, {"num_drones": 8}, device=dev, groups=5)
    with pytest.raises(ValueError):
        VecSwarm(4, {"num_drones": 8}, device=dev, groups=0)
    v = VecSwarm(4, {"num_drones": 8}, device=dev, groups=2)
    with pytest.raises(ValueError):
        v.step_group(2, torch.zeros((4, 8, 3), device=dev))


@pytest.mark.parametrize("e,n,g,kw", [(8192, 64, 4, {}), (8192, 64, 3, {}), (1000, 16, 3, {}), (96, 256, 2, {}),
                                      (300, 64, 3, {"dynamics": "physics"}), (77, 5, 4, {})])
def test_step_groups_native_launch(dev, e, n, g, kw):
    """VecSwarm.step_groups (swarm_step_groups: one native call, group g on stream g, no fork or
    join per step) equals single launches bitwise, with and without an action mask."""
    a, b = _pair(dev, e, n, g, **kw)
    acts = [_acts(dev, e, n, k) for k in range(6)]
    gm = torch.Generator(device=dev).manual_seed(77)
    masks = [None if k % 2 == 0 else (torch.rand((e, n), device=dev, generator=gm) < 0.8).to(torch.uint8)
             for k in range(6)]
    torch.cuda.synchronize()
    b.fork_groups()
    for k in range(6):
        a.step(acts[k], masks[k])
        b.step_groups(acts[k], masks[k])
    b.join()
    torch.cuda.synchronize()
    _same(a, b, "step_groups")
