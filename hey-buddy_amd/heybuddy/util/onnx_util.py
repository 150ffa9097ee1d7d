"""Wake-word heads as ONNX files, without the onnx package (not in this image).

The reference ships its trained classifiers as ``src/js/models/*.onnx`` and
writes new ones with ``torch.onnx.export`` (wakeword.py:316-332, opset 19,
input ``input`` [1, 16, 96], output ``output`` [1, 1]). Those files are
plain protobuf: this module walks the wire format directly.

* ``read_initializers``: the named weight tensors (``TensorProto`` raw_data or
  typed data fields) -> numpy arrays. The exporter keeps state_dict names
  (``norm_in.weight``, ``mlp_in.hidden.weight``, ``layers.0.1.gate.bias`` ...),
  so they load into ``WakeWordMLPModel`` with strict=True.
* ``read_nodes``: (op_type, inputs, outputs) of the graph, for structure checks.
* ``read_model``: the whole graph -- nodes with their attributes, initializers
  (and Constant nodes' tensors), graph inputs / outputs with their shapes --
  for the importers of the reference's pretrained graphs
  (``heybuddy.embedding_graph.from_onnx``, ``heybuddy.spectrogram.mel_params_from_onnx``).
* ``write_wakeword_onnx``: the graph the exporter emits for the default
  gated-MLP head (Flatten, LayerNormalization, Gemm transB=1, Sigmoid, Mul),
  so heads trained here can be deployed where the reference's are.
* ``write_model``: any graph from (op, name, inputs, outputs, attributes)
  nodes and named initializers (the exporters of the embedding and mel graphs).

Host-side file IO only (the weights then live in the flat HBM buffer the HIP
kernels read).
"""
from __future__ import annotations

import struct
from collections import OrderedDict
from typing import Dict, Iterator, List, Mapping, Sequence, Tuple

import numpy as np

__all__ = ["read_initializers", "read_nodes", "read_model", "OnnxNode", "OnnxModel", "write_model",
           "write_wakeword_onnx", "sha256_of"]

# TensorProto.DataType -> numpy dtype (the ones a classifier head can hold)
_DTYPES = {1: np.float32, 6: np.int32, 7: np.int64, 10: np.float16, 11: np.float64}
_NP2ONNX = {np.dtype(v): k for k, v in _DTYPES.items()}


# -- wire format -------------------------------------------------------------
def _varint(buf: bytes, i: int) -> Tuple[int, int]:
    value = shift = 0
    while True:
        byte = buf[i]
        i += 1
        value |= (byte & 0x7F) << shift
        shift += 7
        if byte < 0x80:
            return value, i


def _fields(buf: bytes) -> Iterator[Tuple[int, int, object]]:
    """(field number, wire type, value) of one message; length-delimited values
    are memoryview slices, varints ints, fixed32 / fixed64 raw bytes."""
    buf = memoryview(buf)
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        field, wire = key >> 3, key & 7
        if wire == 0:
            value, i = _varint(buf, i)
        elif wire == 1:
            value, i = bytes(buf[i:i + 8]), i + 8
        elif wire == 5:
            value, i = bytes(buf[i:i + 4]), i + 4
        elif wire == 2:
            size, i = _varint(buf, i)
            value, i = buf[i:i + size], i + size
        else:
            raise ValueError(f"unsupported protobuf wire type {wire}")
        yield field, wire, value


def _packed_varints(value) -> List[int]:
    out, i = [], 0
    while i < len(value):
        v, i = _varint(value, i)
        out.append(v)
    return out


def _graph(path: str):
    with open(path, "rb") as fp:
        data = fp.read()
    for field, wire, value in _fields(data):
        if field == 7 and wire == 2:  # ModelProto.graph
            return value
    raise ValueError(f"{path}: no graph in this ONNX model")


def _tensor(msg) -> Tuple[str, np.ndarray]:
    name, dims, dtype, raw = "", [], 1, None
    typed: Dict[int, list] = {}
    for field, wire, value in _fields(msg):
        if field == 1:  # dims (int64, packed or not)
            dims.extend(_packed_varints(value) if wire == 2 else [value])
        elif field == 2:
            dtype = value
        elif field == 8:
            name = bytes(value).decode()
        elif field == 9:
            raw = bytes(value)
        elif field in (4, 5, 7, 10):  # float_data, int32_data, int64_data, double_data
            typed.setdefault(field, []).append((wire, value))
        elif field == 14:
            raise ValueError(f"initializer {name!r} stores its data externally")
    if dtype not in _DTYPES:
        raise ValueError(f"initializer {name!r}: unsupported ONNX data type {dtype}")
    np_dtype = np.dtype(_DTYPES[dtype]).newbyteorder("<")
    if raw is not None:
        arr = np.frombuffer(raw, dtype=np_dtype)
    elif 4 in typed:
        arr = np.concatenate([np.frombuffer(bytes(v), "<f4") if w == 2 else np.frombuffer(v, "<f4")
                              for w, v in typed[4]]).astype(np_dtype)
    elif 10 in typed:
        arr = np.concatenate([np.frombuffer(bytes(v), "<f8") if w == 2 else np.frombuffer(v, "<f8")
                              for w, v in typed[10]]).astype(np_dtype)
    elif 5 in typed or 7 in typed:
        vals = []
        for w, v in typed.get(5, []) + typed.get(7, []):
            vals.extend(_packed_varints(v) if w == 2 else [v])
        vals = [x - (1 << 64) if x >= 1 << 63 else x for x in vals]
        if dtype == 10:  # float16 travels as its bit pattern in int32_data
            arr = np.array(vals, dtype=np.uint16).view(np.float16)
        else:
            arr = np.array(vals, dtype=np_dtype)
    else:
        arr = np.zeros(0, dtype=np_dtype)
    count = int(np.prod(dims)) if dims else 1
    if arr.size != count:
        raise ValueError(f"initializer {name!r}: {arr.size} values for shape {tuple(dims)}")
    return name, arr.reshape(dims).astype(np_dtype.newbyteorder("="), copy=True)


def read_initializers(path: str) -> "OrderedDict[str, np.ndarray]":
    """All initializers of an ONNX model, in file order."""
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for field, wire, value in _fields(_graph(path)):
        if field == 5 and wire == 2:  # GraphProto.initializer
            name, arr = _tensor(value)
            out[name] = arr
    return out


def read_nodes(path: str) -> List[Tuple[str, Tuple[str, ...], Tuple[str, ...]]]:
    """(op_type, inputs, outputs) of every node, in graph order."""
    nodes = []
    for field, wire, value in _fields(_graph(path)):
        if field == 1 and wire == 2:  # GraphProto.node
            op, ins, outs = "", [], []
            for f, _, v in _fields(value):
                if f == 1:
                    ins.append(bytes(v).decode())
                elif f == 2:
                    outs.append(bytes(v).decode())
                elif f == 4:
                    op = bytes(v).decode()
            nodes.append((op, tuple(ins), tuple(outs)))
    return nodes


# -- whole-graph reader ----------------------------------------------------------
class OnnxNode:
    """One NodeProto: op_type, name, inputs, outputs, attributes (name -> int,
    float, bytes, numpy array (tensor), list of ints / floats)."""

    __slots__ = ("op", "name", "inputs", "outputs", "attrs")

    def __init__(self, op: str, name: str, inputs: Sequence[str], outputs: Sequence[str], attrs: Dict[str, object]):
        self.op, self.name, self.inputs, self.outputs, self.attrs = op, name, tuple(inputs), tuple(outputs), attrs

    def __repr__(self) -> str:
        return f"OnnxNode({self.op} {self.name!r}: {self.inputs} -> {self.outputs})"


class OnnxModel:
    """The graph of one ONNX file: nodes in graph order, initializers (Constant
    nodes' values included), graph inputs / outputs as (name, dims) with None
    for a symbolic dimension, and the default-domain opset."""

    def __init__(self, nodes: List[OnnxNode], initializers: "OrderedDict[str, np.ndarray]",
                 inputs: List[Tuple[str, Tuple]], outputs: List[Tuple[str, Tuple]], opset: int) -> None:
        self.nodes, self.initializers, self.inputs, self.outputs, self.opset = nodes, initializers, inputs, outputs, opset

    def consumers(self, name: str) -> List[OnnxNode]:
        return [n for n in self.nodes if name in n.inputs]

    def producer(self, name: str):
        return next((n for n in self.nodes if name in n.outputs), None)


def _attribute(msg) -> Tuple[str, object]:
    name, typ, vals = "", 0, {}
    ints: List[int] = []
    floats: List[float] = []
    for field, wire, value in _fields(msg):
        if field == 1:
            name = bytes(value).decode()
        elif field == 20:
            typ = value
        elif field == 2:
            vals["f"] = struct.unpack("<f", value)[0]
        elif field == 3:
            vals["i"] = value - (1 << 64) if value >= 1 << 63 else value
        elif field == 4:
            vals["s"] = bytes(value)
        elif field == 5:
            vals["t"] = _tensor(value)[1]
        elif field == 7:
            floats.extend(np.frombuffer(bytes(value), "<f4").tolist() if wire == 2 else [struct.unpack("<f", value)[0]])
        elif field == 8:
            ints.extend(_packed_varints(value) if wire == 2 else [value])
    ints = [x - (1 << 64) if x >= 1 << 63 else x for x in ints]
    # AttributeProto.AttributeType: FLOAT 1, INT 2, STRING 3, TENSOR 4, FLOATS 6, INTS 7
    by_type = {1: vals.get("f"), 2: vals.get("i"), 3: vals.get("s"), 4: vals.get("t"), 6: floats, 7: ints}
    if typ in by_type:
        return name, by_type[typ]
    if typ == 0:  # untyped (old writers): the field that is present
        for k in ("t", "s", "f", "i"):
            if k in vals:
                return name, vals[k]
        return name, ints or floats
    raise ValueError(f"attribute {name!r}: unsupported attribute type {typ}")


def _value_info_shape(msg) -> Tuple[str, Tuple]:
    name, dims = "", []
    for field, _, value in _fields(msg):
        if field == 1:
            name = bytes(value).decode()
        elif field == 2:  # TypeProto
            for f2, _, v2 in _fields(value):
                if f2 == 1:  # tensor_type
                    for f3, _, v3 in _fields(v2):
                        if f3 == 2:  # TensorShapeProto
                            for f4, _, v4 in _fields(v3):
                                if f4 == 1:  # Dimension: dim_value 1 | dim_param 2
                                    d = None
                                    for f5, _, v5 in _fields(v4):
                                        if f5 == 1:
                                            d = v5
                                    dims.append(d)
    return name, tuple(dims)


def read_model(path: str) -> OnnxModel:
    """The graph of an ONNX file (no external data, no subgraphs)."""
    with open(path, "rb") as fp:
        data = fp.read()
    graph, opset = None, 0
    for field, wire, value in _fields(data):
        if field == 7 and wire == 2:
            graph = value
        elif field == 8 and wire == 2:  # OperatorSetIdProto: domain 1, version 2
            dom, ver = "", 0
            for f, _, v in _fields(value):
                if f == 1:
                    dom = bytes(v).decode()
                elif f == 2:
                    ver = v
            if dom in ("", "ai.onnx"):
                opset = ver
    if graph is None:
        raise ValueError(f"{path}: no graph in this ONNX model")
    nodes: List[OnnxNode] = []
    inits: "OrderedDict[str, np.ndarray]" = OrderedDict()
    inputs: List[Tuple[str, Tuple]] = []
    outputs: List[Tuple[str, Tuple]] = []
    for field, wire, value in _fields(graph):
        if field == 1 and wire == 2:
            op, name, ins, outs, attrs = "", "", [], [], {}
            for f, _, v in _fields(value):
                if f == 1:
                    ins.append(bytes(v).decode())
                elif f == 2:
                    outs.append(bytes(v).decode())
                elif f == 3:
                    name = bytes(v).decode()
                elif f == 4:
                    op = bytes(v).decode()
                elif f == 5:
                    k, a = _attribute(v)
                    attrs[k] = a
                elif f == 7 and bytes(v).decode() not in ("", "ai.onnx"):
                    raise ValueError(f"node {name!r}: op {op!r} of domain {bytes(v).decode()!r} is not supported")
            if op == "Constant":
                if "value" not in attrs:
                    raise ValueError(f"Constant {name!r}: only tensor-valued constants are supported")
                inits[outs[0]] = np.asarray(attrs["value"])
                continue
            nodes.append(OnnxNode(op, name, ins, outs, attrs))
        elif field == 5 and wire == 2:
            n, arr = _tensor(value)
            inits[n] = arr
        elif field == 11 and wire == 2:
            inputs.append(_value_info_shape(value))
        elif field == 12 and wire == 2:
            outputs.append(_value_info_shape(value))
    inputs = [(n, s) for n, s in inputs if n not in inits]  # old exporters list initializers as inputs
    return OnnxModel(nodes, inits, inputs, outputs, opset)


def sha256_of(path: str) -> str:
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as fp:
        for chunk in iter(lambda: fp.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


# -- writer --------------------------------------------------------------------
def _enc_varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _f_varint(field: int, v: int) -> bytes:
    return _enc_varint(field << 3) + _enc_varint(v)


def _f_bytes(field: int, payload: bytes) -> bytes:
    return _enc_varint(field << 3 | 2) + _enc_varint(len(payload)) + payload


def _f_str(field: int, s: str) -> bytes:
    return _f_bytes(field, s.encode())


def _attr_int(name: str, v: int) -> bytes:
    return _f_str(1, name) + _f_varint(3, v) + _f_varint(20, 2)  # AttributeProto.INT


def _attr_float(name: str, v: float) -> bytes:
    return _f_str(1, name) + _enc_varint(2 << 3 | 5) + struct.pack("<f", v) + _f_varint(20, 1)  # FLOAT


def _node(op: str, name: str, ins: Sequence[str], outs: Sequence[str], attrs: Sequence[bytes] = ()) -> bytes:
    body = b"".join(_f_str(1, i) for i in ins) + b"".join(_f_str(2, o) for o in outs)
    body += _f_str(3, name) + _f_str(4, op) + b"".join(_f_bytes(5, a) for a in attrs)
    return _f_bytes(1, body)


def _initializer(name: str, arr: np.ndarray) -> bytes:
    arr = np.asarray(arr, order="C")  # (not ascontiguousarray: it makes a 0-d scalar 1-d)
    body = b"".join(_f_varint(1, d) for d in arr.shape) + _f_varint(2, _NP2ONNX[arr.dtype])
    body += _f_str(8, name) + _f_bytes(9, arr.astype(arr.dtype.newbyteorder("<")).tobytes())
    return _f_bytes(5, body)


def _value_info(field: int, name: str, shape: Sequence[int]) -> bytes:
    dims = b"".join(_f_bytes(1, _f_varint(1, d)) for d in shape)
    tensor = _f_varint(1, 1) + _f_bytes(2, dims)  # elem_type FLOAT, shape
    return _f_bytes(field, _f_str(1, name) + _f_bytes(2, _f_bytes(1, tensor)))


def _attr(name: str, v: object) -> bytes:
    """AttributeProto for an int, float, string, list of ints / floats or tensor."""
    if isinstance(v, (bool, int, np.integer)):
        return _attr_int(name, int(v))
    if isinstance(v, (float, np.floating)):
        return _attr_float(name, float(v))
    if isinstance(v, (str, bytes)):
        return _f_str(1, name) + _f_bytes(4, v.encode() if isinstance(v, str) else v) + _f_varint(20, 3)
    if isinstance(v, np.ndarray):
        t = _initializer("", v)
        return _f_str(1, name) + _f_bytes(5, _fields_payload(t)) + _f_varint(20, 4)
    v = list(v)
    if all(isinstance(x, (int, np.integer)) for x in v):
        return _f_str(1, name) + _f_bytes(8, b"".join(_enc_varint(int(x)) for x in v)) + _f_varint(20, 7)
    return _f_str(1, name) + _f_bytes(7, np.asarray(v, "<f4").tobytes()) + _f_varint(20, 6)


def _fields_payload(wrapped: bytes) -> bytes:
    """The payload of a single length-delimited field (strip its key and length)."""
    (_, _, value), = list(_fields(wrapped))
    return bytes(value)


def write_model(path: str, nodes: Sequence[Tuple[str, str, Sequence[str], Sequence[str], Mapping[str, object]]],
                initializers: Mapping[str, np.ndarray], inputs: Sequence[Tuple[str, Sequence]],
                outputs: Sequence[Tuple[str, Sequence]], opset_version: int = 13,
                producer: str = "heybuddy-amd", graph_name: str = "main_graph") -> None:
    """Write a graph: ``nodes`` as (op, name, inputs, outputs, attributes),
    float initializers, inputs / outputs as (name, dims) (a str or None dim is
    symbolic)."""
    body = b"".join(_node(op, name, ins, outs, [_attr(k, v) for k, v in attrs.items()])
                    for op, name, ins, outs, attrs in nodes)
    body += _f_str(2, graph_name)
    body += b"".join(_initializer(k, np.asarray(v)) for k, v in initializers.items())

    def vi(field: int, name: str, shape: Sequence) -> bytes:
        dims = b"".join(_f_bytes(1, _f_varint(1, d) if isinstance(d, (int, np.integer)) else
                                 _f_str(2, str(d or "N"))) for d in shape)
        tensor = _f_varint(1, 1) + _f_bytes(2, dims)
        return _f_bytes(field, _f_str(1, name) + _f_bytes(2, _f_bytes(1, tensor)))

    body += b"".join(vi(11, n, s) for n, s in inputs) + b"".join(vi(12, n, s) for n, s in outputs)
    model = _f_varint(1, 8) + _f_str(2, producer) + _f_str(3, "0.1.0") + _f_bytes(7, body)
    model += _f_bytes(8, _f_varint(2, opset_version))
    with open(path, "wb") as fp:
        fp.write(model)


def write_wakeword_onnx(path: str, state_dict: Mapping[str, np.ndarray], num_layers: int,
                        input_shape: Tuple[int, int] = (16, 96), opset_version: int = 19,
                        eps: float = 1e-5) -> None:
    """The default head (flatten > LN > gated MLP > [LN > gated MLP] x L > LN >
    gated MLP > sigmoid) in the node / tensor naming of torch.onnx.export of the
    reference module (wakeword.py:316-332), weights from ``state_dict``."""
    nodes: List[bytes] = []

    def ln(src: str, prefix: str, scope: str) -> str:
        out = f"{scope}/LayerNormalization_output_0"
        nodes.append(_node("LayerNormalization", f"{scope}/LayerNormalization",
                           [src, f"{prefix}.weight", f"{prefix}.bias"], [out],
                           [_attr_int("axis", -1), _attr_float("epsilon", eps)]))
        return out

    def gemm(src: str, prefix: str, scope: str) -> str:
        out = f"{scope}/Gemm_output_0"
        nodes.append(_node("Gemm", f"{scope}/Gemm", [src, f"{prefix}.weight", f"{prefix}.bias"], [out],
                           [_attr_float("alpha", 1.0), _attr_float("beta", 1.0), _attr_int("transB", 1)]))
        return out

    def gmlp(src: str, prefix: str, scope: str) -> str:
        h = gemm(src, f"{prefix}.hidden", f"{scope}/hidden")
        s = f"{scope}/activation/Sigmoid_output_0"
        nodes.append(_node("Sigmoid", f"{scope}/activation/Sigmoid", [h], [s]))
        a = f"{scope}/activation/Mul_output_0"
        nodes.append(_node("Mul", f"{scope}/activation/Mul", [h, s], [a]))
        g = gemm(src, f"{prefix}.gate", f"{scope}/gate")
        m = f"{scope}/Mul_output_0"
        nodes.append(_node("Mul", f"{scope}/Mul", [a, g], [m]))
        return gemm(m, f"{prefix}.output", f"{scope}/output")

    flat = "/flatten/Flatten_output_0"
    nodes.append(_node("Flatten", "/flatten/Flatten", ["input"], [flat], [_attr_int("axis", 1)]))
    x = gmlp(ln(flat, "norm_in", "/norm_in"), "mlp_in", "/mlp_in")
    for l in range(num_layers):
        x = ln(x, f"layers.{l}.0", f"/layers.{l}/layers.{l}.0")
        x = gmlp(x, f"layers.{l}.1", f"/layers.{l}/layers.{l}.1")
    x = gmlp(ln(x, "norm_out", "/norm_out"), "mlp_out", "/mlp_out")
    nodes.append(_node("Sigmoid", "/sigmoid/Sigmoid", [x], ["output"]))

    inits = b"".join(_initializer(k, np.asarray(v, dtype=np.float32)) for k, v in state_dict.items())
    graph = b"".join(nodes) + _f_str(2, "main_graph") + inits
    graph += _value_info(11, "input", (1, *input_shape)) + _value_info(12, "output", (1, 1))
    model = _f_varint(1, 9) + _f_str(2, "heybuddy-amd") + _f_str(3, "0.1.0") + _f_bytes(7, graph)
    model += _f_bytes(8, _f_varint(2, opset_version))
    with open(path, "wb") as fp:
        fp.write(model)
