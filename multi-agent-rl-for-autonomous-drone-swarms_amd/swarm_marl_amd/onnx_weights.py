"""Weights of the reference's exported actor (artifacts/policy.onnx) without onnx/onnxruntime.

scripts/export_onnx.py:120-141 traces the RLlib actor (TorchFC, fcnet_hiddens [256, 256], relu;
config_builders.py:53-56, models.py:75-81) into an ONNX graph
    observation -> Cast -> Reshape(B, -1) -> Gemm(transB) -> Relu -> Gemm(transB) -> Relu
                -> Gemm(transB) -> action_logits
This module reads such a file as DATA: a protobuf wire-format walk (varints and length-delimited
fields only) that extracts the float32 initializers and the node list.  Nothing in the file is
executed.  The Gemm chain is then checked to be exactly the MLP the MI355X policy kernel runs.

ONNX field numbers (onnx.proto3): ModelProto.graph = 7; GraphProto.node = 1, initializer = 5,
input = 11, output = 12; NodeProto.input = 1, output = 2, op_type = 4, attribute = 5;
AttributeProto.name = 1, f = 2, i = 3, type = 20; TensorProto.dims = 1, data_type = 2,
float_data = 4, name = 8, raw_data = 9.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

_FLOAT = 1  # TensorProto.DataType.FLOAT


def _varint(b: bytes, i: int) -> tuple[int, int]:
    r = s = 0
    while True:
        if i >= len(b):
            raise ValueError("truncated varint")
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return r, i


def _fields(b: bytes) -> list[tuple[int, int, object]]:
    """(field number, wire type, value) of one protobuf message; value is int or bytes."""
    out, i = [], 0
    while i < len(b):
        key, i = _varint(b, i)
        f, w = key >> 3, key & 7
        if w == 0:
            v, i = _varint(b, i)
        elif w == 1:
            v, i = b[i:i + 8], i + 8
        elif w == 2:
            n, i = _varint(b, i)
            v, i = b[i:i + n], i + n
        elif w == 5:
            v, i = b[i:i + 4], i + 4
        else:
            raise ValueError(f"unsupported wire type {w}")
        out.append((f, w, v))
    return out


def _group(b: bytes) -> dict[int, list]:
    d: dict[int, list] = {}
    for f, _, v in _fields(b):
        d.setdefault(f, []).append(v)
    return d


def _tensor(b: bytes) -> tuple[str, np.ndarray]:
    t = _group(b)
    name = t[8][0].decode()
    dims = []
    for v in t.get(1, []):  # packed or unpacked int64 dims
        if isinstance(v, int):
            dims.append(v)
        else:
            i = 0
            while i < len(v):
                x, i = _varint(v, i)
                dims.append(x)
    dtype = t.get(2, [_FLOAT])[0]
    if dtype != _FLOAT:
        raise ValueError(f"initializer {name}: data_type {dtype} is not float32")
    if 9 in t:
        arr = np.frombuffer(t[9][0], dtype="<f4").copy()
    else:
        vals = []
        for v in t.get(4, []):
            if isinstance(v, (bytes, bytearray)) and len(v) % 4 == 0:
                vals.extend(struct.unpack(f"<{len(v) // 4}f", v))
        arr = np.asarray(vals, np.float32)
    return name, arr.reshape(dims)


@dataclass
class OnnxNode:
    op: str
    inputs: list[str]
    outputs: list[str]
    attrs: dict[str, object] = field(default_factory=dict)


@dataclass
class OnnxGraph:
    nodes: list[OnnxNode]
    inits: dict[str, np.ndarray]
    inputs: list[str]
    outputs: list[str]


def read_onnx(path_or_bytes) -> OnnxGraph:
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else Path(path_or_bytes).read_bytes()
    model = _group(bytes(data))
    if 7 not in model:
        raise ValueError("not an ONNX ModelProto (no graph)")
    g = _group(model[7][0])
    nodes = []
    for nb in g.get(1, []):
        n = _group(nb)
        attrs = {}
        for ab in n.get(5, []):
            a = _group(ab)
            nm = a[1][0].decode()
            if 2 in a:
                attrs[nm] = struct.unpack("<f", a[2][0])[0]
            elif 3 in a:
                v = a[3][0]
                attrs[nm] = v - (1 << 64) if v >= 1 << 63 else v
            elif 5 in a:  # tensor-valued (Constant): kept as raw bytes
                attrs[nm] = a[5][0]
        nodes.append(OnnxNode(n[4][0].decode(), [x.decode() for x in n.get(1, [])],
                              [x.decode() for x in n.get(2, [])], attrs))
    inits = dict(_tensor(tb) for tb in g.get(5, []))
    names = lambda key: [_group(v)[1][0].decode() for v in g.get(key, [])]  # noqa: E731
    return OnnxGraph(nodes, inits, names(11), names(12))


def mlp_layers(graph: OnnxGraph) -> list[tuple[np.ndarray, np.ndarray, bool]]:
    """The Gemm chain as [(W [out, in], b [out], relu_after)], validated against the graph:
    Gemm(alpha=1, beta=1, transB=1) nodes fed by the previous Gemm (optionally through a Relu),
    the first fed (through shape-only Cast/Reshape nodes) by the graph input."""
    layers: list[tuple[np.ndarray, np.ndarray, bool]] = []
    cur = graph.inputs[0] if graph.inputs else None
    for nd in graph.nodes:
        if nd.op in ("Cast", "Reshape") and nd.inputs and nd.inputs[0] == cur:
            cur = nd.outputs[0]
        elif nd.op == "Gemm":
            if nd.inputs[0] != cur:
                raise ValueError(f"Gemm input {nd.inputs[0]} is not the running activation {cur}")
            if nd.attrs.get("transB", 0) != 1 or nd.attrs.get("transA", 0) != 0:
                raise ValueError("expected Gemm(transA=0, transB=1)")
            if nd.attrs.get("alpha", 1.0) != 1.0 or nd.attrs.get("beta", 1.0) != 1.0:
                raise ValueError("expected Gemm alpha = beta = 1")
            w = graph.inits[nd.inputs[1]]
            b = graph.inits[nd.inputs[2]] if len(nd.inputs) > 2 else np.zeros(w.shape[0], np.float32)
            layers.append((w.astype(np.float32), b.astype(np.float32), False))
            cur = nd.outputs[0]
        elif nd.op == "Relu" and nd.inputs[0] == cur:
            w, b, _ = layers[-1]
            layers[-1] = (w, b, True)
            cur = nd.outputs[0]
    if not layers or cur not in graph.outputs:
        raise ValueError("graph is not a Gemm/Relu chain ending at the graph output")
    return layers
