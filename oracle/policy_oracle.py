"""CPU evaluation of the exported actor graph — TEST INFRASTRUCTURE ONLY (the policy oracle).

Evaluates the node list of the reference's artifacts/policy.onnx (scripts/export_onnx.py:120-141:
the RLlib TorchFC actor, config_builders.py:53-56 fcnet_hiddens [256, 256] relu) in float32 NumPy
with ONNX operator semantics for the ops it contains (Cast, Shape, Constant, Gather, Unsqueeze,
Concat, Reshape, Gemm, Relu).  The graph and weights come from tests/golden/policy_onnx.npz,
extracted from the artifact as data by tests/golden/make_policy_fixture.py.  onnxruntime is not
installed, so parity is pinned to the graph's operator semantics, not to an ONNX runtime's bits.
Only tests/ (and smoke/bench checks) import this module.
"""
from __future__ import annotations

import json

import numpy as np


def load_fixture(path):
    d = np.load(path, allow_pickle=False)
    nodes = json.loads(str(d["nodes_json"]))
    tensors = {k[5:]: d[k] for k in d.files if k.startswith("init:")}
    tensors.update({k[6:]: d[k] for k in d.files if k.startswith("const:")})
    return nodes, tensors, d


def eval_graph(nodes, tensors, obs: np.ndarray, graph_input="observation") -> np.ndarray:
    env = dict(tensors)
    env[graph_input] = np.asarray(obs)
    out = None
    for nd in nodes:
        op, ins, outs, at = nd["op"], nd["inputs"], nd["outputs"], nd["attrs"]
        x = [env[i] for i in ins]
        if op == "Cast":
            y = x[0].astype(np.float32)  # to = FLOAT (1) in this graph
        elif op == "Shape":
            y = np.asarray(x[0].shape, np.int64)
        elif op == "Constant":
            y = env[outs[0]]
        elif op == "Gather":
            y = np.take(x[0], x[1], axis=int(at.get("axis", 0)))
        elif op == "Unsqueeze":
            y = np.expand_dims(x[0], tuple(int(a) for a in np.atleast_1d(x[1])))
        elif op == "Concat":
            y = np.concatenate([np.atleast_1d(v) for v in x], axis=int(at.get("axis", 0)))
        elif op == "Reshape":
            y = x[0].reshape(tuple(int(v) for v in x[1]))
        elif op == "Gemm":
            a = x[0].T if at.get("transA", 0) else x[0]
            b = x[1].T if at.get("transB", 0) else x[1]
            y = np.float32(at.get("alpha", 1.0)) * (a.astype(np.float32) @ b.astype(np.float32))
            if len(x) > 2:
                y = y + np.float32(at.get("beta", 1.0)) * x[2].astype(np.float32)
            y = y.astype(np.float32)
        elif op == "Relu":
            y = np.maximum(x[0], np.float32(0))
        else:
            raise NotImplementedError(op)
        env[outs[0]] = y
        out = y
    return out


def diag_gaussian_mean(logits: np.ndarray) -> np.ndarray:
    """Deterministic action of RLlib's TorchDiagGaussian: the first half of the logits."""
    return logits[:, : logits.shape[1] // 2]
