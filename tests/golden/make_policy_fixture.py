"""Extract the reference's exported actor (artifacts/policy.onnx) into a data fixture.

Run only in the build container (reads /root/reference):  python tests/golden/make_policy_fixture.py
The ONNX file is read as DATA (protobuf wire format), never executed.

The decode here is deliberately INDEPENDENT of the product's reader (swarm_marl_amd.onnx_weights,
which the kernel's weights come through): a schema-table driven recursive-descent walker written
separately, that imports nothing from swarm_marl_amd.  A wire-format or layout bug in the product
reader therefore cannot hide in the fixture; tests/test_policy_cpu.py checks, where the reference
is present, that both decodes agree byte for byte on every initializer.

Writes tests/golden/policy_onnx.npz: the float32 initializers, the node list (JSON) with its
Constant tensors, and input/expected-output vectors evaluated by oracle/policy_oracle.py (a graph
interpreter over these arrays, not the product kernel): random observations and real N=64
observations from the reference rollout fixture.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))

from oracle.policy_oracle import eval_graph  # noqa: E402

SRC = Path("/root/reference/artifacts/policy.onnx")

# ------------------------------------------------------------------ independent wire decoder
# onnx.proto (ONNX IR): the fields this fixture needs, as {message: {field: (name, kind, repeated)}}.
# kinds: "msg:<Message>", "str", "bytes", "int" (varint, int64 two's complement), "f32" (fixed32),
# "ints" (repeated int64, packed or not).
SCHEMA = {
    "Model": {7: ("graph", "msg:Graph", False)},
    "Graph": {1: ("node", "msg:Node", True), 5: ("initializer", "msg:Tensor", True),
              11: ("input", "msg:ValueInfo", True), 12: ("output", "msg:ValueInfo", True)},
    "ValueInfo": {1: ("name", "str", False)},
    "Node": {1: ("input", "str", True), 2: ("output", "str", True), 4: ("op_type", "str", False),
             5: ("attribute", "msg:Attribute", True)},
    "Attribute": {1: ("name", "str", False), 2: ("f", "f32", False), 3: ("i", "int", False),
                  5: ("t", "msg:Tensor", False), 20: ("type", "int", False)},
    "Tensor": {1: ("dims", "ints", True), 2: ("data_type", "int", False), 4: ("float_data", "f32s", True),
               7: ("int64_data", "ints", True), 8: ("name", "str", False), 9: ("raw_data", "bytes", False)},
}


class Reader:
    """Cursor over one protobuf message body."""

    def __init__(self, data: bytes, lo: int = 0, hi: int | None = None):
        self.d, self.p, self.end = data, lo, len(data) if hi is None else hi

    def done(self) -> bool:
        return self.p >= self.end

    def uvarint(self) -> int:
        val, shift = 0, 0
        for _ in range(10):
            if self.p >= self.end:
                raise ValueError("varint runs past the message end")
            byte = self.d[self.p]
            self.p += 1
            val += (byte & 0x7F) << shift
            if byte < 0x80:
                return val
            shift += 7
        raise ValueError("varint longer than 10 bytes")

    def take(self, n: int) -> tuple[int, int]:
        lo = self.p
        if n < 0 or lo + n > self.end:
            raise ValueError("field runs past the message end")
        self.p = lo + n
        return lo, self.p


def decode(msg: str, data: bytes, lo: int = 0, hi: int | None = None) -> dict:
    spec = SCHEMA[msg]
    out: dict = {name: [] for name, _, rep in spec.values() if rep}
    r = Reader(data, lo, hi)
    while not r.done():
        tag = r.uvarint()
        fnum, wtype = tag >> 3, tag & 7
        if wtype == 0:
            raw = r.uvarint()
            payload = None
        elif wtype == 1:
            payload = r.take(8)
        elif wtype == 2:
            payload = r.take(r.uvarint())
        elif wtype == 5:
            payload = r.take(4)
        else:
            raise ValueError(f"{msg}: wire type {wtype} not expected in ONNX")
        if fnum not in spec:
            continue  # unneeded field
        name, kind, rep = spec[fnum]
        if kind.startswith("msg:"):
            val = decode(kind[4:], data, *payload)
        elif kind == "str":
            val = bytes(data[payload[0]:payload[1]]).decode("utf-8")
        elif kind == "bytes":
            val = bytes(data[payload[0]:payload[1]])
        elif kind == "int":
            val = raw - (1 << 64) if raw >> 63 else raw
        elif kind in ("f32", "f32s"):
            if wtype == 5:
                val = np.frombuffer(data, "<f4", 1, payload[0])[0]
            else:  # packed repeated floats
                val = np.frombuffer(data, "<f4", (payload[1] - payload[0]) // 4, payload[0])
        elif kind == "ints":
            if wtype == 0:
                val = [raw - (1 << 64) if raw >> 63 else raw]
            else:  # packed
                sub, val = Reader(data, *payload), []
                while not sub.done():
                    v = sub.uvarint()
                    val.append(v - (1 << 64) if v >> 63 else v)
        else:  # pragma: no cover
            raise AssertionError(kind)
        if rep:
            if isinstance(val, list):
                out[name].extend(val)
            elif kind == "f32s" and isinstance(val, np.ndarray) and val.ndim:
                out[name].extend(val.tolist())
            else:
                out[name].append(val)
        else:
            out[name] = val
    return out


DTYPES = {1: np.dtype("<f4"), 7: np.dtype("<i8")}  # TensorProto FLOAT, INT64


def tensor_array(t: dict) -> np.ndarray:
    dt = DTYPES[t.get("data_type", 1)]
    if "raw_data" in t:
        arr = np.frombuffer(t["raw_data"], dt).copy()
    elif dt.kind == "f":
        arr = np.asarray(t.get("float_data", []), dt)
    else:
        arr = np.asarray(t.get("int64_data", []), dt)
    dims = [int(x) for x in t.get("dims", [])]
    return arr.reshape(dims) if dims else arr.reshape(())


def read_model(data: bytes):
    """(nodes as JSON-able dicts, {'init:name' | 'const:output': array}, input name, output name)."""
    g = decode("Model", data)["graph"]
    nodes, arrays = [], {}
    for nd in g["node"]:
        attrs = {}
        for a in nd["attribute"]:
            if "t" in a:
                if nd["op_type"] == "Constant":
                    arrays["const:" + nd["output"][0]] = tensor_array(a["t"])
                continue
            if "f" in a:
                attrs[a["name"]] = float(a["f"])
            elif "i" in a:
                attrs[a["name"]] = int(a["i"])
        nodes.append(dict(op=nd["op_type"], inputs=nd["input"], outputs=nd["output"], attrs=attrs))
    for t in g["initializer"]:
        arrays["init:" + t["name"]] = tensor_array(t)
    return nodes, arrays, g["input"][0]["name"], g["output"][0]["name"]


def main() -> None:
    nodes, arrays, gin, gout = read_model(SRC.read_bytes())
    tensors = {k.split(":", 1)[1]: v for k, v in arrays.items()}
    rng = np.random.default_rng(2024)
    obs_rand = rng.uniform(-12, 12, (1024, 37)).astype(np.float32)
    roll = np.load(HERE / "rollout_n64.npz")
    obs_env = roll["out_obs"][roll["obs_present"]][:256].astype(np.float32)
    obs = np.concatenate([obs_rand, obs_env])
    logits = eval_graph(nodes, tensors, obs, gin)
    np.savez_compressed(HERE / "policy_onnx.npz", nodes_json=json.dumps(nodes),
                        graph_input=gin, graph_output=gout, obs=obs, logits=logits,
                        source=str(SRC), decoder="tests/golden/make_policy_fixture.py (independent)",
                        **arrays)
    print("wrote", HERE / "policy_onnx.npz", obs.shape, logits.shape,
          {k: v.shape for k, v in arrays.items() if k.startswith("init:")})


if __name__ == "__main__":
    main()
