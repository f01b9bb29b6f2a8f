"""GPU: on-device actor inference (csrc/swarm_policy.hip) through the C-ABI.

Oracle: the reference's exported actor graph (artifacts/policy.onnx, scripts/export_onnx.py:
120-141) evaluated in float32 NumPy by oracle/policy_oracle.py on the fixture observations
(tests/golden/policy_onnx.npz: random obs and real N=64 env obs).
Tolerances (stated per path):
  f32  (v_mfma_f32_16x16x4_f32): |logit error| <= 1e-4 + 1e-5 |logit|  (summation order only)
  f32x3 (three v_mfma_f32_32x32x16_f16 passes over f16 hi / lo splits): the same bound; its host
       emulation from the packed blob sits at 0.1 of it (tests/test_policy_cpu.py); its two kernels
       (two waves per SIMD, default; one wave pipelined) agree bit for bit
  bf16 (v_mfma_f32_32x32x16_bf16): within 0.02 of the NumPy emulation of the same bf16 arithmetic
       (tests/test_policy_cpu.py) and within 0.3 of the f32 graph (logits span about -37 .. 66).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def fx():
    from tests.test_policy_cpu import fixture_layers
    return fixture_layers()


def _pol(fx, dev, precision):
    from swarm_marl_amd.policy import PolicyMLP
    layers, _ = fx
    return PolicyMLP(layers, device=dev, precision=precision)


@pytest.mark.parametrize("precision", ["f32", "f32x3"])
def test_f32_logits_vs_graph(dev, fx, precision):
    layers, d = fx
    pol = _pol(fx, dev, precision)
    got = pol.logits(torch.as_tensor(d["obs"]).to(dev)).cpu().numpy()
    ref = d["logits"]
    assert np.all(np.abs(got - ref) <= 1e-4 + 1e-5 * np.abs(ref)), np.abs(got - ref).max()


def test_bf16_logits_vs_emulation_and_graph(dev, fx):
    from tests.test_policy_cpu import emulate_bf16_kernel
    layers, d = fx
    pol = _pol(fx, dev, "bf16")
    got = pol.logits(torch.as_tensor(d["obs"]).to(dev)).cpu().numpy()
    emu = emulate_bf16_kernel(pol.packed_host, d["obs"], 6)
    # the kernel against a host emulation of its own bf16 arithmetic (operand roundings, f32 sums):
    # measured 1.8e-4 (tools/policy_err.py), bound 1e-3
    assert np.abs(got - emu).max() <= 1e-3, np.abs(got - emu).max()
    # against the reference's f32 graph the bf16 operand rounding (2^-9 relative) shows: measured
    # 0.225 max / 0.018 mean on logits up to |66| (0.34 % of the range); bounds 0.3 / 0.03
    err = np.abs(got - d["logits"])
    assert err.max() <= 0.3 and err.mean() <= 0.03, (err.max(), err.mean())


@pytest.mark.parametrize("precision", ["bf16", "f32", "f32x3"])
def test_actions_are_gaussian_mean_and_ragged_rows(dev, fx, precision):
    layers, d = fx
    pol = _pol(fx, dev, precision)
    for rows in (1, 31, 33, 1000):  # ragged last tile
        obs = torch.as_tensor(d["obs"][:rows]).to(dev)
        lg = pol.logits(obs)
        act = pol.act(obs)
        torch.cuda.synchronize()
        assert act.shape == (rows, 3)
        assert torch.equal(act, lg[:, :3])


def test_headline_batch_f32_vs_float64(dev, fx):
    """E=8192 x N=64 observation rows of the real env, one launch."""
    from swarm_marl_amd import VecSwarm
    layers, _ = fx
    vec = VecSwarm(8192, {"num_drones": 64}, device=dev, auto_reset=True, seed=4)
    vec.reset()
    g = torch.Generator(device=dev).manual_seed(3)
    vec.step(torch.rand((8192, 64, 3), device=dev, generator=g) * 2 - 1)
    pol32, pol16, polx3 = _pol(fx, dev, "f32"), _pol(fx, dev, "bf16"), _pol(fx, dev, "f32x3")
    lg32 = pol32.logits(vec.obs).reshape(-1, 6)
    lg16 = pol16.logits(vec.obs).reshape(-1, 6)
    lgx3 = polx3.logits(vec.obs).reshape(-1, 6)
    idx = torch.randperm(lg32.shape[0], device=dev, generator=g)[:4096]
    x = vec.obs.reshape(-1, 37)[idx].double().cpu().numpy()
    for i, (w, b, relu) in enumerate(layers):
        x = x @ w.T.astype(np.float64) + b
        if relu:
            x = np.maximum(x, 0)
    got32 = lg32[idx].double().cpu().numpy()
    assert np.all(np.abs(got32 - x) <= 1e-4 + 1e-5 * np.abs(x)), np.abs(got32 - x).max()
    gotx3 = lgx3[idx].double().cpu().numpy()  # the three-pass f16 path meets the f32 tolerance
    assert np.all(np.abs(gotx3 - x) <= 1e-4 + 1e-5 * np.abs(x)), np.abs(gotx3 - x).max()
    assert np.abs(lg16[idx].double().cpu().numpy() - x).max() <= 0.3


def test_x3_two_waves_equals_pipelined_bitwise(dev, fx, monkeypatch):
    """policy_mlp_x3l (two waves per SIMD, the default f32x3 kernel) against policy_mlp_x3 (one
    wave, pipelined; SWARM_POLICY_X3_PIPELINED=1): the same MFMA sequence per accumulator and the
    same epilogues, so the logits agree bit for bit — full tiles, a ragged last tile, fewer rows
    than one workgroup's waves, and more tiles than waves in the grid."""
    layers, d = fx
    pol = _pol(fx, dev, "f32x3")
    g = torch.Generator(device=dev).manual_seed(11)
    for rows in (1, 33, 255, 70_001):
        obs = torch.randn((rows, 37), device=dev, generator=g) * 3
        monkeypatch.setenv("SWARM_POLICY_X3_PIPELINED", "1")
        ref = pol.logits(obs).clone()
        monkeypatch.delenv("SWARM_POLICY_X3_PIPELINED")
        got = pol.logits(obs)
        torch.cuda.synchronize()
        assert torch.equal(got, ref), (rows, (got - ref).abs().max().item())


def test_sampled_actions(dev, fx):
    layers, d = fx
    pol = _pol(fx, dev, "bf16")
    obs = torch.as_tensor(np.repeat(d["obs"][1024:1025], 200000, axis=0)).to(dev)
    lg = pol.logits(obs[:1])[0].cpu().numpy()
    a1 = pol.act(obs, deterministic=False, seed=5, counter=7)
    a2 = pol.act(obs, deterministic=False, seed=5, counter=7)
    a3 = pol.act(obs, deterministic=False, seed=5, counter=8)
    assert torch.equal(a1, a2) and not torch.equal(a1, a3)
    a = a1.double().cpu().numpy()
    mean, std = lg[:3], np.exp(lg[3:])
    assert np.all(np.abs(a.mean(0) - mean) < 5 * std / np.sqrt(len(a)) + 1e-3)
    assert np.all(np.abs(a.std(0) / std - 1) < 0.02)


def test_rollout_graph_policy_plus_step(dev, fx):
    """A captured rollout segment: policy on the obs tensor -> env step, 4 times, replayed."""
    from swarm_marl_amd import VecSwarm
    layers, _ = fx
    pol = _pol(fx, dev, "bf16")
    vec = VecSwarm(512, {"num_drones": 64}, device=dev, auto_reset=True, seed=9)
    vec.reset()
    acts = torch.zeros((512, 64, 3), device=dev)
    ref = VecSwarm(512, {"num_drones": 64}, device=dev, auto_reset=True, seed=9)
    ref.reset()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(4):
            pol.act(vec.obs, out=acts)
            vec.step(acts)
    for _ in range(3):
        graph.replay()
    for _ in range(12):  # the same 12 steps eagerly
        ref.step(pol.act(ref.obs))
    torch.cuda.synchronize()
    assert torch.equal(vec.obs, ref.obs) and torch.equal(vec.pos, ref.pos)
    assert bool(torch.isfinite(acts).all())
