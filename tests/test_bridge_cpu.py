"""CPU: host logic of the RLlib batched-env bridge (swarm_marl_amd/rllib_bridge.py) — action
packing from MultiEnvDicts, the continuing-agent mask, and the GlobalStateCallback equivalent
on per-agent copies (callbacks.py:14-57 semantics) and on references to a device ring."""
from __future__ import annotations

import numpy as np
import pytest

from swarm_marl_amd import _native as nat
from swarm_marl_amd import rllib_bridge as rb


def test_pack_actions_missing_and_unknown():
    idx = {"drone_0": 0, "drone_1": 1, "drone_2": 2}
    out = np.full((3, 3, 3), 7.0, np.float32)
    rb.pack_actions({0: {"drone_1": [1, 2, 3], "ghost": [9, 9, 9]}, 2: {"drone_0": np.ones(3)}}, idx, out)
    exp = np.zeros((3, 3, 3), np.float32)
    exp[0, 1] = [1, 2, 3]
    exp[2, 0] = 1
    assert np.array_equal(out, exp)


def test_next_active():
    fl = np.array([[nat.AGENT_HAS_OBS | nat.AGENT_STEPPED, nat.AGENT_STEPPED, 0],
                   [nat.AGENT_STEPPED, 0, 0]], np.uint8)
    done = np.array([0, nat.ENV_TERMINATED | nat.ENV_RESET], np.uint8)
    assert next_active_eq(rb.next_active(fl, done), [[True, False, False], [True, True, True]])


def next_active_eq(a, b):
    return np.array_equal(a, np.array(b, bool))


class _Batch(dict):
    def __init__(self, infos):
        super().__init__(infos=infos)
        self.count = len(infos)


class _Model:
    global_state_dim = 6 * 2 + 3


class _Policy:
    model = _Model()


def test_callback_copies_like_reference():
    infos = [{"global_state": np.full(15, k, np.float32)} for k in range(4)]
    b = _Batch(infos)
    rb.DeviceGlobalStateCallback().on_postprocess_trajectory(policy_id="shared_policy",
                                                             policies={"shared_policy": _Policy()},
                                                             postprocessed_batch=b)
    assert b["global_state"].shape == (4, 15) and b["global_state"][3, 0] == 3


def test_callback_zero_init_without_infos():
    b = _Batch([{}])
    rb.DeviceGlobalStateCallback().on_postprocess_trajectory(policy_id="p", policies={"p": _Policy()},
                                                             postprocessed_batch=b)
    assert b["global_state"].shape == (1, 15) and not b["global_state"].any()


def test_resolve_refs_to_missing_bridge():
    with pytest.raises(ValueError):
        rb.resolve_global_state([(10 ** 9, 0, 0)])
