"""CPU: the env-queue protocol of the persistent swarm_step64 (csrc/swarm_kernel.hip,
`swarm_step64`), restated step for step in Python and run under random interleavings of the
workgroups' atomics.  Every env must be processed exactly once per launch, and every launch must
leave the queue heads at zero so the next launch on the stream starts from a clean queue.
"""
from __future__ import annotations

import random

import pytest

HEADS = 8  # S64_HEADS


def _program(b: int, E: int, G: int, heads: list, done: list):
    """One workgroup of swarm_step64, as a generator that yields before every atomic."""
    H = min(G, HEADS)                          # heads in use
    x, k = b % H, b // H
    lo, hi = (E * x) // H, (E * (x + 1)) // H
    gx = (G - x + H - 1) // H                  # workgroups sharing head x
    n = hi - lo
    env = lo + k if k < n else -1              # static first env
    base = lo + gx
    n_dyn = n - gx if n > gx else 0
    n_draws = n_dyn + gx                       # tickets drawn from head x per launch

    def settle(v):
        if v == n_draws - 1:                   # the last ticket of the launch: reset the head
            heads[x] = 0
        return base + v if v < n_dyn else -1

    first = env >= 0
    yield
    ticket = heads[x]; heads[x] += 1           # draw(): returning device-scope atomicAdd
    while env >= 0:
        yield
        nxt = settle(ticket)
        if nxt >= 0:                           # prefetch(): the next env's inputs + next ticket
            yield
            ticket = heads[x]; heads[x] += 1
        done.append(env)                       # s64_env(env)
        env = nxt
    if not first:
        yield
        settle(ticket)


def _launch(E: int, G: int, heads: list, rng: random.Random) -> list:
    done: list = []
    live = [_program(b, E, G, heads, done) for b in range(G)]
    while live:
        g = rng.randrange(len(live))
        try:
            next(live[g])
        except StopIteration:
            live.pop(g)
    return done


@pytest.mark.parametrize("E,G", [(1, 1), (7, 3), (8, 8), (9, 8), (100, 8), (100, 16), (1000, 64),
                                 (3000, 1024), (5, 40), (8192, 6144), (777, 13)])
def test_every_env_once_and_heads_reset(E, G):
    rng = random.Random(E * 7919 + G)
    heads = [0] * HEADS
    for _ in range(3):  # consecutive launches share the work buffer
        done = _launch(E, G, heads, rng)
        assert sorted(done) == list(range(E))
        assert heads == [0] * HEADS
