"""CPU: the on-device policy's host side — ONNX weight reader, oracle, fragment packing.

* swarm_marl_amd.onnx_weights reads a protobuf-encoded ONNX graph as data (a synthetic model
  written here, and the reference artifact's node list / weights held in tests/golden/policy_onnx.npz).
* oracle/policy_oracle.py evaluates the reference's exported graph; it reproduces the fixture's
  logits and a float64 dense evaluation.
* swarm_policy_pack (C-ABI, host only): the packed bf16 blob, decoded with the MFMA fragment maps
  the kernel assumes (32x32x16 A/B lane maps, accumulator-as-operand k order), computes the same
  MLP in NumPy — the packing and the chaining permutation agree with each other; the GPU tests
  check the maps against the hardware.
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np
import pytest

from tests.conftest import GOLDEN


# ---------------------------------------------------------------- a tiny protobuf writer
def _vint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _fld(num: int, wire: int, payload) -> bytes:
    key = _vint((num << 3) | wire)
    if wire == 0:
        return key + _vint(payload)
    if wire == 5:
        return key + payload
    return key + _vint(len(payload)) + payload


def _tensor(name: str, arr: np.ndarray) -> bytes:
    b = b"".join(_fld(1, 0, d) for d in arr.shape) + _fld(2, 0, 1) + _fld(8, 2, name.encode())
    return b + _fld(9, 2, np.ascontiguousarray(arr, "<f4").tobytes())


def _node(op, ins, outs, attrs=()) -> bytes:
    b = b"".join(_fld(1, 2, i.encode()) for i in ins) + b"".join(_fld(2, 2, o.encode()) for o in outs)
    b += _fld(4, 2, op.encode())
    for name, kind, val in attrs:
        a = _fld(1, 2, name.encode())
        a += _fld(2, 5, struct.pack("<f", val)) if kind == "f" else _fld(3, 0, val)
        b += _fld(5, 2, a)
    return b


def _valueinfo(name):
    return _fld(1, 2, name.encode())


def synthetic_onnx(layers) -> bytes:
    nodes, inits, cur = [], [], "obs"
    gemm = [("alpha", "f", 1.0), ("beta", "f", 1.0), ("transB", "i", 1)]
    nodes.append(_node("Cast", [cur], ["c0"], [("to", "i", 1)]))
    cur = "c0"
    for i, (w, b, relu) in enumerate(layers):
        inits += [_tensor(f"w{i}", w), _tensor(f"b{i}", b)]
        nodes.append(_node("Gemm", [cur, f"w{i}", f"b{i}"], [f"g{i}"], gemm))
        cur = f"g{i}"
        if relu:
            nodes.append(_node("Relu", [cur], [f"r{i}"]))
            cur = f"r{i}"
    graph = b"".join(_fld(1, 2, n) for n in nodes) + b"".join(_fld(5, 2, t) for t in inits)
    graph += _fld(11, 2, _valueinfo("obs")) + _fld(12, 2, _valueinfo(cur))
    return _fld(1, 0, 8) + _fld(7, 2, graph)


def _random_layers(rng, d=37, out=6):
    return [(rng.normal(0, 0.2, (256, d)).astype(np.float32), rng.normal(0, 0.1, 256).astype(np.float32), True),
            (rng.normal(0, 0.06, (256, 256)).astype(np.float32), rng.normal(0, 0.1, 256).astype(np.float32), True),
            (rng.normal(0, 0.06, (out, 256)).astype(np.float32), rng.normal(0, 0.1, out).astype(np.float32), False)]


def test_onnx_reader_synthetic_model():
    from swarm_marl_amd.onnx_weights import mlp_layers, read_onnx
    layers = _random_layers(np.random.default_rng(0))
    g = read_onnx(synthetic_onnx(layers))
    assert [n.op for n in g.nodes] == ["Cast", "Gemm", "Relu", "Gemm", "Relu", "Gemm"]
    got = mlp_layers(g)
    for (w, b, r), (w2, b2, r2) in zip(layers, got):
        assert np.array_equal(w, w2) and np.array_equal(b, b2) and r == r2


def test_onnx_reader_rejects_non_mlp():
    from swarm_marl_amd.onnx_weights import mlp_layers, read_onnx
    layers = _random_layers(np.random.default_rng(1))
    raw = synthetic_onnx(layers).replace(b"transB", b"transX")
    with pytest.raises(ValueError):
        mlp_layers(read_onnx(raw))
    with pytest.raises(ValueError):
        read_onnx(b"\x08\x08")  # a ModelProto without a graph


def _independent():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_policy_fixture", GOLDEN / "make_policy_fixture.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_independent_decoder_agrees_on_synthetic_model():
    """The fixture's decoder (tests/golden/make_policy_fixture.py, imports nothing from
    swarm_marl_amd) and the product reader decode the same bytes to the same arrays."""
    from swarm_marl_amd.onnx_weights import read_onnx
    mod = _independent()
    raw = synthetic_onnx(_random_layers(np.random.default_rng(3)))
    nodes, arrays, gin, gout = mod.read_model(raw)
    g = read_onnx(raw)
    assert [n["op"] for n in nodes] == [n.op for n in g.nodes]
    assert (gin, gout) == (g.inputs[0], g.outputs[0])
    for name, arr in g.inits.items():
        ind = arrays["init:" + name]
        assert ind.dtype == arr.dtype and ind.shape == arr.shape and ind.tobytes() == arr.tobytes(), name


def test_fixture_weights_match_product_reader_on_reference_artifact():
    """Every initializer of the committed fixture (independent decode) equals, byte for byte,
    what the product reader extracts from the reference's artifacts/policy.onnx — and so what
    the GPU kernel is loaded with by PolicyMLP.from_onnx.  Needs /root/reference (build
    container only)."""
    from pathlib import Path
    from swarm_marl_amd.onnx_weights import mlp_layers, read_onnx
    src = Path("/root/reference/artifacts/policy.onnx")
    if not src.exists():
        pytest.skip("reference artifact not present (GPU box)")
    d = np.load(GOLDEN / "policy_onnx.npz")
    assert "independent" in str(d["decoder"])
    g = read_onnx(src)
    assert set("init:" + k for k in g.inits) == {k for k in d.files if k.startswith("init:")}
    for name, arr in g.inits.items():
        fx = d["init:" + name]
        assert fx.dtype == arr.dtype and fx.shape == arr.shape and fx.tobytes() == arr.tobytes(), name
    # and the Gemm chain the kernel runs is made of exactly those arrays
    gem = [n for n in g.nodes if n.op == "Gemm"]
    for (w, b, _), nd in zip(mlp_layers(g), gem):
        assert w.tobytes() == d["init:" + nd.inputs[1]].tobytes()
        assert b.tobytes() == d["init:" + nd.inputs[2]].tobytes()
    # the independent decode of the artifact is the committed fixture's
    _, arrays, _, _ = _independent().read_model(src.read_bytes())
    for k, v in arrays.items():
        assert v.tobytes() == d[k].tobytes(), k


def test_policy_oracle_reproduces_fixture():
    from oracle.policy_oracle import eval_graph, load_fixture
    nodes, tensors, d = load_fixture(GOLDEN / "policy_onnx.npz")
    assert [n["op"] for n in nodes if n["op"] in ("Gemm", "Relu")] == ["Gemm", "Relu", "Gemm", "Relu", "Gemm"]
    got = eval_graph(nodes, tensors, d["obs"], str(d["graph_input"]))
    assert np.array_equal(got, d["logits"])
    x = d["obs"].astype(np.float64)
    ws = [tensors[n["inputs"][1]] for n in nodes if n["op"] == "Gemm"]
    bs = [tensors[n["inputs"][2]] for n in nodes if n["op"] == "Gemm"]
    for i, (w, b) in enumerate(zip(ws, bs)):
        x = x @ w.T.astype(np.float64) + b
        if i < 2:
            x = np.maximum(x, 0)
    assert np.abs(x - d["logits"]).max() < 1e-3 * max(1.0, np.abs(x).max()) * 1e-1


def fixture_layers():
    from oracle.policy_oracle import load_fixture
    nodes, tensors, d = load_fixture(GOLDEN / "policy_onnx.npz")
    gem = [n for n in nodes if n["op"] == "Gemm"]
    return [(tensors[g["inputs"][1]], tensors[g["inputs"][2]], i < 2) for i, g in enumerate(gem)], d


def _pack(lib, layers, precision):
    (w1, b1, _), (w2, b2, _), (w3, b3, _) = layers
    nb = lib.swarm_policy_packed_bytes(w1.shape[1], w3.shape[0], precision)
    assert nb > 0
    buf = np.zeros(nb, np.uint8)
    fp = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa
    keep = [np.ascontiguousarray(a, np.float32) for a in (w1, b1, w2, b2, w3, b3)]
    rc = lib.swarm_policy_pack(w1.shape[1], w3.shape[0], precision, *[fp(a) for a in keep],
                               buf.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return buf


def _bf16(u16: np.ndarray) -> np.ndarray:
    return (u16.astype(np.uint32) << 16).view(np.float32)


def _to_bf16(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return _bf16(u.astype(np.uint16))


def emulate_bf16_kernel(buf: np.ndarray, x: np.ndarray, out: int) -> np.ndarray:
    """The bf16 kernel's arithmetic in NumPy, reading weights only from the packed blob through
    the fragment maps: A[row r][k = 8h + j] on lane l = 32h + r; B[k = 8h + j][col r];
    C[row (i&3) + 8(i>>2) + 4h][col r] in register i; chained operand element j of half h in
    k-step s = accumulator register 8s + j."""
    rows, d = x.shape
    w1f = _bf16(buf[:8 * 3 * 1024].view(np.uint16)).reshape(8, 3, 2, 32, 8)  # ob, ks, h, m, j
    off = 8 * 3 * 1024
    w2f = _bf16(buf[off:off + 8 * 16 * 1024].view(np.uint16)).reshape(8, 16, 2, 32, 8)
    off += 8 * 16 * 1024
    w3f = _bf16(buf[off:off + 16 * 2 * out * 16].view(np.uint16)).reshape(16, 2, out, 8)
    off += 16 * 2 * out * 16
    b2 = buf[off:off + 1024].view(np.float32)
    b3 = buf[off + 1024:off + 1024 + 4 * out].view(np.float32)
    xp = np.zeros((rows, 48), np.float32)
    xp[:, :d] = x
    xp[:, d] = 1.0
    xb = _to_bf16(xp).reshape(rows, 3, 2, 8)  # n, ks, h, j
    # accumulator register i of lane half h holds row (i & 3) + 8 (i >> 2) + 4 h
    reg_row = np.array([[(i & 3) + 8 * (i >> 2) + 4 * h for i in range(16)] for h in range(2)])

    def chain(c):  # c [ob, 32 rows, n] -> operand fragments [ks = 2 ob + s, h, n, j] (bf16, relu)
        obn = c.shape[0]
        frag = np.zeros((2 * obn, 2, c.shape[2], 8), np.float32)
        for ob in range(obn):
            for s in range(2):
                for h in range(2):
                    for j in range(8):
                        frag[2 * ob + s, h, :, j] = c[ob, reg_row[h, 8 * s + j], :]
        return _to_bf16(np.maximum(frag, 0))

    c1 = np.einsum("oshmj,nshj->omn", w1f.astype(np.float64), xb.astype(np.float64))
    h1 = chain(c1)
    c2 = np.einsum("okhmj,khnj->omn", w2f.astype(np.float64), h1.astype(np.float64))
    c2 += b2.reshape(8, 32, 1)
    h2 = chain(c2)
    c3 = np.einsum("khmj,khnj->mn", w3f.astype(np.float64), h2.astype(np.float64)) + b3[:, None]
    return c3.T


def test_pack_bf16_layout_computes_the_mlp():
    from oracle.policy_oracle import load_fixture
    from swarm_marl_amd import _native as nat
    lib = nat.load_library()
    layers, d = fixture_layers()
    buf = _pack(lib, layers, nat.POLICY_BF16)
    obs = d["obs"][::5]
    got = emulate_bf16_kernel(buf, obs, 6)
    ref = d["logits"][::5]
    err = np.abs(got - ref)
    assert err.max() < 0.05 * max(1.0, np.abs(ref).max()), err.max()
    # and the permutation matters: an unpermuted W2 gives a different function
    assert np.abs(got - ref).mean() < 0.05


def test_pack_f32_layout_roundtrip():
    from swarm_marl_amd import _native as nat
    lib = nat.load_library()
    layers, _ = fixture_layers()
    buf = _pack(lib, layers, nat.POLICY_F32).view(np.float32)
    (w1, b1, _), (w2, b2, _), (w3, b3, _) = layers
    kq1 = (37 + 1 + 3) // 4
    W1 = buf[:16 * kq1 * 64].reshape(16, kq1, 4, 16)  # ob, q, g, m
    assert np.array_equal(W1[2, 3, 1, 5], w1[2 * 16 + 5, 4 * 3 + 1])
    assert W1[0, 9, 1, 0] == b1[0]  # k == in_dim (37 = 4*9 + 1): the bias column
    off = 16 * kq1 * 64
    W2 = buf[off:off + 16 * 64 * 64].reshape(16, 64, 4, 16)  # ob, q, g, m
    for ob, q, g, m in [(0, 0, 0, 0), (3, 17, 2, 9), (15, 63, 3, 15)]:
        assert W2[ob, q, g, m] == w2[ob * 16 + m, (q >> 2) * 16 + 4 * g + (q & 3)]


def test_pack_rejects_bad_dims():
    from swarm_marl_amd import _native as nat
    lib = nat.load_library()
    assert lib.swarm_policy_packed_bytes(48, 6, 0) < 0
    assert lib.swarm_policy_packed_bytes(37, 14, 0) < 0
    assert lib.swarm_policy_packed_bytes(37, 5, 0) < 0
    assert lib.swarm_policy_packed_bytes(37, 6, 7) < 0


def _split16(x: np.ndarray):
    """f32 -> (hi, lo) f16 pieces as the f32x3 kernel splits its activations (RNE both; lo is
    (x - hi) scaled by 2^11)."""
    x = np.asarray(x, np.float32)
    hi = x.astype(np.float16)
    lo = ((x - hi.astype(np.float32)) * np.float32(2048)).astype(np.float16)
    return hi.astype(np.float64), lo.astype(np.float64)


def emulate_x3_kernel(buf: np.ndarray, x: np.ndarray, out: int) -> np.ndarray:
    """The f32x3 kernel's arithmetic in float64 from its packed blob (hi blob then lo blob, the
    bf16 blob's fragment maps with f16 elements): every layer sums hi*hi + hi*lo + lo*hi."""
    total = len(buf) // 2
    rows, d = x.shape

    def frags(part):
        b = buf[part * total:(part + 1) * total]
        w1 = b[:8 * 3 * 1024].view(np.float16).astype(np.float64).reshape(8, 3, 2, 32, 8)
        off = 8 * 3 * 1024
        w2 = b[off:off + 8 * 16 * 1024].view(np.float16).astype(np.float64).reshape(8, 16, 2, 32, 8)
        off += 8 * 16 * 1024
        w3 = b[off:off + 16 * 2 * out * 16].view(np.float16).astype(np.float64).reshape(16, 2, out, 8)
        off += 16 * 2 * out * 16
        return w1, w2, w3, b[off:off + 1024].view(np.float32), b[off + 1024:off + 1024 + 4 * out].view(np.float32)

    (w1h, w2h, w3h, b2, b3), (w1l, w2l, w3l, _, _) = frags(0), frags(1)
    xp = np.zeros((rows, 48), np.float32)
    xp[:, :d] = x
    xp[:, d] = 1.0
    xh, xl = _split16(xp)
    xh, xl = xh.reshape(rows, 3, 2, 8), xl.reshape(rows, 3, 2, 8)
    reg_row = np.array([[(i & 3) + 8 * (i >> 2) + 4 * h for i in range(16)] for h in range(2)])

    def chain(c):
        obn = c.shape[0]
        frag = np.zeros((2 * obn, 2, c.shape[2], 8), np.float32)
        for ob in range(obn):
            for s in range(2):
                for h in range(2):
                    for j in range(8):
                        frag[2 * ob + s, h, :, j] = c[ob, reg_row[h, 8 * s + j], :]
        return _split16(np.maximum(frag, 0))

    def x3(eq, ah, al, bh, bl):  # hi*hi + 2^-11 (hi*lo + lo*hi)
        return np.einsum(eq, ah, bh) + (np.einsum(eq, ah, bl) + np.einsum(eq, al, bh)) / 2048.0

    c1 = x3("oshmj,nshj->omn", w1h, w1l, xh, xl).astype(np.float32)
    h1h, h1l = chain(c1)
    c2 = (x3("okhmj,khnj->omn", w2h, w2l, h1h, h1l) + b2.reshape(8, 32, 1)).astype(np.float32)
    h2h, h2l = chain(c2)
    c3 = x3("khmj,khnj->mn", w3h, w3l, h2h, h2l) + b3[:, None]
    return c3.T


def test_pack_f32x3_split_and_emulation_meet_the_f32_tolerance():
    """The f32x3 blob: hi = f16(w) (RNE, as numpy), lo = f16(w - hi); its three-pass arithmetic
    (emulated in float64 from the blob) is within the f32 path's tolerance of the f32 graph."""
    from swarm_marl_amd import _native as nat
    lib = nat.load_library()
    layers, d = fixture_layers()
    buf = _pack(lib, layers, nat.POLICY_F32X3)
    assert len(buf) == 2 * lib.swarm_policy_packed_bytes(37, 6, nat.POLICY_BF16)
    (w1, b1, _), (w2, b2, _), _ = layers
    half = len(buf) // 2
    hi2 = buf[8 * 3 * 1024:8 * 19 * 1024].view(np.float16).reshape(8, 16, 2, 32, 8)
    lo2 = buf[half + 8 * 3 * 1024:half + 8 * 19 * 1024].view(np.float16).reshape(8, 16, 2, 32, 8)
    # out block 3, k-step 5, half 1, row 7, element 2 -> W2[3*32+7][chained_k(5, 1, 2)]
    ks, h, j = 5, 1, 2
    k = (ks >> 1) * 32 + 16 * (ks & 1) + 8 * (j >> 2) + 4 * h + (j & 3)
    w = np.float32(w2[3 * 32 + 7, k])
    assert hi2[3, ks, h, 7, j] == np.float16(w)
    assert lo2[3, ks, h, 7, j] == np.float16((w - np.float32(np.float16(w))) * np.float32(2048))
    rec = hi2.astype(np.float64) + lo2.astype(np.float64) / 2048.0
    w2perm = np.array([[w2[ob * 32 + m, (s >> 1) * 32 + 16 * (s & 1) + 8 * (jj >> 2) + 4 * hh + (jj & 3)]
                        for ob in range(8) for s in range(16) for hh in range(2) for m in range(32)
                        for jj in range(8)]], np.float64).reshape(rec.shape)
    big = np.abs(w2perm) > 1e-4
    assert np.all(np.abs(rec - w2perm)[big] <= 2.0 ** -21 * np.abs(w2perm)[big])
    obs = d["obs"][::3]
    got = emulate_x3_kernel(buf, obs, 6)
    ref = d["logits"][::3]
    assert np.all(np.abs(got - ref) <= 1e-4 + 1e-5 * np.abs(ref)), np.abs(got - ref).max()
