"""On-device actor inference for the rollout loop.

The reference's actor is RLlib's TorchFC (fcnet_hiddens [256, 256], relu;
src/swarm_marl/training/config_builders.py:53-56, models.py:75-81), exported by
scripts/export_onnx.py:120-141 to artifacts/policy.onnx.  `PolicyMLP` runs that MLP with the
library's MFMA kernel (swarm_policy_forward, csrc/swarm_policy.hip) directly on a VecSwarm's
observation tensor and writes the next action tensor in place, so a rollout step is two kernel
launches (policy, env step) with no host round trip:

    pol = PolicyMLP.from_onnx("artifacts/policy.onnx", device="cuda")
    acts = pol.act(vec.obs)            # [E, N, 3]: RLlib TorchDiagGaussian mean (deterministic)
    vec.step(acts)

precision "bf16" (default): bf16 MFMA operands with f32 accumulation (~1e-2 relative on the
logits); "f32": f32 MFMA (within summation-order rounding of the f32 graph); "f32x3": the f32
graph's accuracy on f16 MFMA — every operand split into f16 hi + lo, three products per term
(hi*hi + hi*lo + lo*hi, ~2^-21 relative each); obs / weights / activations within the f16 range.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native as nat
from .onnx_weights import mlp_layers, read_onnx

_PRECISION = {"bf16": nat.POLICY_BF16, "f32": nat.POLICY_F32, "f32x3": nat.POLICY_F32X3}


def _fp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class PolicyMLP:
    def __init__(self, layers, *, device="cuda", precision: str = "bf16"):
        if precision not in _PRECISION:
            raise ValueError(f"precision must be one of {sorted(_PRECISION)}, got {precision!r}")
        if len(layers) != 3:
            raise ValueError("expected 3 dense layers (two 256-unit relu hidden layers + logits)")
        (w1, b1, r1), (w2, b2, r2), (w3, b3, r3) = layers
        h = nat.POLICY_HIDDEN
        if not (r1 and r2 and not r3):
            raise ValueError("expected relu after the two hidden layers and none after the logits")
        if w1.shape[0] != h or w2.shape != (h, h) or w3.shape[1] != h:
            raise ValueError(f"hidden layers must be {h} wide, got {w1.shape}, {w2.shape}, {w3.shape}")
        self.lib = nat.load_library()
        self.in_dim, self.out_dim = int(w1.shape[1]), int(w3.shape[0])
        self.precision = precision
        self.device = torch.device(device)
        prec = _PRECISION[precision]
        nb = int(self.lib.swarm_policy_packed_bytes(self.in_dim, self.out_dim, prec))
        if nb < 0:
            nat.check(nb, self.lib, policy=True)
        host = np.zeros(nb, np.uint8)
        arrs = [np.ascontiguousarray(a, np.float32) for a in (w1, b1, w2, b2, w3, b3)]
        nat.check(self.lib.swarm_policy_pack(self.in_dim, self.out_dim, prec, *map(_fp, arrs),
                                             host.ctypes.data_as(ctypes.c_void_p)), self.lib, policy=True)
        self.packed_host = host
        self.weights = torch.from_numpy(host).to(self.device)  # caching allocator: 256-B aligned
        self._c = nat.SwarmPolicy(self.in_dim, self.out_dim, prec, 0, self.weights.data_ptr())
        self.layers = [(np.asarray(w, np.float32), np.asarray(b, np.float32)) for w, b, _ in layers]

    @classmethod
    def from_onnx(cls, path_or_bytes, **kw) -> "PolicyMLP":
        """Weights and topology from an exported actor (scripts/export_onnx.py output)."""
        return cls(mlp_layers(read_onnx(path_or_bytes)), **kw)

    @classmethod
    def from_arrays(cls, w1, b1, w2, b2, w3, b3, **kw) -> "PolicyMLP":
        return cls([(w1, b1, True), (w2, b2, True), (w3, b3, False)], **kw)

    # ------------------------------------------------------------------ forward
    def _check_obs(self, obs: torch.Tensor) -> int:
        if not isinstance(obs, torch.Tensor) or obs.device != self.device or obs.dtype != torch.float32:
            raise ValueError(f"obs must be a float32 tensor on {self.device}")
        if obs.shape[-1] != self.in_dim or not obs.is_contiguous():
            raise ValueError(f"obs must be contiguous [..., {self.in_dim}], got {tuple(obs.shape)}")
        return int(obs.numel() // self.in_dim)

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def forward(self, obs: torch.Tensor, *, logits: torch.Tensor | None = None,
                actions: torch.Tensor | None = None, sample: bool = False, seed: int = 0,
                counter: int = 0) -> None:
        rows = self._check_obs(obs)
        for name, t, width in (("logits", logits, self.out_dim), ("actions", actions, self.out_dim // 2)):
            if t is not None and (t.device != self.device or t.dtype != torch.float32 or not t.is_contiguous()
                                  or t.numel() != rows * width):
                raise ValueError(f"{name} must be a contiguous float32 tensor of {rows} x {width} on {self.device}")
        mode = nat.POLICY_ACT_SAMPLE if sample else nat.POLICY_ACT_MEAN
        rc = self.lib.swarm_policy_forward(ctypes.byref(self._c), obs.data_ptr(), rows,
                                           None if logits is None else logits.data_ptr(),
                                           None if actions is None else actions.data_ptr(), mode,
                                           int(seed) & (2**64 - 1), int(counter) & (2**64 - 1), self._stream())
        nat.check(rc, self.lib, policy=True)

    def logits(self, obs: torch.Tensor) -> torch.Tensor:
        out = torch.empty(obs.shape[:-1] + (self.out_dim,), dtype=torch.float32, device=self.device)
        self.forward(obs, logits=out)
        return out

    def act(self, obs: torch.Tensor, out: torch.Tensor | None = None, *, deterministic: bool = True,
            seed: int = 0, counter: int = 0) -> torch.Tensor:
        """Actions [..., out/2]: the Gaussian mean, or mean + exp(log_std) * N(0, 1) (Philox keyed by
        (seed, row, counter)) with deterministic=False."""
        if out is None:
            out = torch.empty(obs.shape[:-1] + (self.out_dim // 2,), dtype=torch.float32, device=self.device)
        self.forward(obs, actions=out, sample=not deterministic, seed=seed, counter=counter)
        return out
