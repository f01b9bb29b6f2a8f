"""GPU: the RLlib batched-env bridge (swarm_marl_amd/rllib_bridge.py) against the batched tensor
API stepped with the same actions — MultiEnvDict values equal the kernel's tensors, terminal
steps carry no observations (drone_swarm_env.py:154), try_reset hands out the in-kernel reset's
first observation, removed agents get no reward — and the device global_state consumer resolves
every reference to the global state the reference would have copied into that info
(callbacks.py:14-57)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from swarm_marl_amd import _native as nat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("mode", ["info", "device"])
def test_bridge_matches_tensor_api(dev, mode):
    from swarm_marl_amd import VecSwarm
    from swarm_marl_amd.rllib_bridge import DeviceGlobalStateCallback, SwarmBaseEnv
    e, n, steps = 24, 8, 40
    br = SwarmBaseEnv(e, {"num_drones": n}, device=dev, seed=3, global_state=mode, ring_len=64)
    ref = VecSwarm(e, {"num_drones": n}, device=dev, auto_reset=True, seed=3, with_infos=True,
                   with_global_state=True)
    ref.reset()
    obs, rew, term, trunc, infos, _ = br.poll()
    assert set(obs) == set(range(e)) and all(len(o) == n for o in obs.values())
    for k in range(n):
        assert np.array_equal(obs[0][f"drone_{k}"], ref.obs[0, k].cpu().numpy())
    rng = np.random.default_rng(0)
    collected = []  # (info, expected global state) pairs, as a sampler would batch them
    active = np.ones((e, n), bool)
    resets = 0
    for t in range(steps):
        acts = rng.uniform(-1, 1, (e, n, 3)).astype(np.float32)
        br.send_actions({i: {f"drone_{k}": acts[i, k] for k in range(n) if active[i, k]} for i in range(e)})
        a_t = torch.as_tensor(acts * active[..., None], device=dev)
        ref.step(a_t)
        obs, rew, term, trunc, infos, _ = br.poll()
        flags = ref.info_flags.cpu().numpy()
        done = ref.env_done.cpu().numpy()
        r_obs, r_rew = ref.obs.cpu().numpy(), ref.reward.cpu().numpy()
        gs = ref.global_state.cpu().numpy()
        for i in range(e):
            stepped = [k for k in range(n) if flags[i, k] & nat.AGENT_STEPPED]
            assert sorted(rew[i]) == sorted(f"drone_{k}" for k in stepped)
            for k in stepped:
                assert rew[i][f"drone_{k}"] == float(r_rew[i, k])
            assert term[i]["__all__"] == bool(done[i] & nat.ENV_TERMINATED)
            if done[i] & nat.ENV_RESET:
                assert obs[i] == {}
                o2, inf2 = br.try_reset(i)
                resets += 1
                for k in range(n):
                    assert np.array_equal(o2[i][f"drone_{k}"], r_obs[i, k])
                collected += [(inf2[i][f"drone_{k}"], gs[i]) for k in range(n)]
                active[i] = True
            else:
                has = [k for k in range(n) if flags[i, k] & nat.AGENT_HAS_OBS]
                assert sorted(obs[i]) == sorted(f"drone_{k}" for k in has)
                for k in has:
                    assert np.array_equal(obs[i][f"drone_{k}"], r_obs[i, k])
                    collected.append((infos[i][f"drone_{k}"], gs[i]))
                active[i] = False
                active[i, has] = True
    assert resets > 0
    # GlobalStateCallback equivalent over the whole collected trajectory
    batch = {"infos": [c[0] for c in collected]}
    DeviceGlobalStateCallback().on_postprocess_trajectory(policy_id="p", policies={},
                                                          postprocessed_batch=batch)
    assert np.array_equal(batch["global_state"], np.stack([c[1] for c in collected]))
    if mode == "device":
        assert "global_state_ref" in collected[0][0] and "global_state" not in collected[0][0]
