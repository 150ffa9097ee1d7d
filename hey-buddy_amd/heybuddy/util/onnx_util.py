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
* ``write_wakeword_onnx``: the graph the exporter emits for the default
  gated-MLP head (Flatten, LayerNormalization, Gemm transB=1, Sigmoid, Mul),
  so heads trained here can be deployed where the reference's are.

Host-side file IO only (the weights then live in the flat HBM buffer the HIP
kernels read).
"""
from __future__ import annotations

import struct
from collections import OrderedDict
from typing import Dict, Iterator, List, Mapping, Sequence, Tuple

import numpy as np

__all__ = ["read_initializers", "read_nodes", "write_wakeword_onnx"]

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
    arr = np.ascontiguousarray(arr)
    body = b"".join(_f_varint(1, d) for d in arr.shape) + _f_varint(2, _NP2ONNX[arr.dtype])
    body += _f_str(8, name) + _f_bytes(9, arr.astype(arr.dtype.newbyteorder("<")).tobytes())
    return _f_bytes(5, body)


def _value_info(field: int, name: str, shape: Sequence[int]) -> bytes:
    dims = b"".join(_f_bytes(1, _f_varint(1, d)) for d in shape)
    tensor = _f_varint(1, 1) + _f_bytes(2, dims)  # elem_type FLOAT, shape
    return _f_bytes(field, _f_str(1, name) + _f_bytes(2, _f_bytes(1, tensor)))


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
