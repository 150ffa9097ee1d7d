"""The speech-embedding graph as runtime data.

The reference runs Google's speech_embedding network as an opaque ONNX file
(SpeechEmbeddingModel, embeddings.py:23-42; I/O ``input_1`` [n,76,32,1] ->
``conv2d_19`` [n,1,1,96], src/js/src/models/speech-embedding.js:125-146)
that is downloaded at run time and absent offline. Its topology and weights
are therefore NOT known here. This module describes the network as a list of
ops (Keras Conv2D 'valid' / LeakyReLU / MaxPool2D, NHWC) that libhbk.so
executes generically; ``se20_graph()`` is a 20-conv stand-in with the same
I/O signature and the same last node name, with seeded weights.

``from_onnx(path)`` reads the reference's own file (sha256 70d16429...,
embeddings.py:29-30) -- or any graph in the Keras / tf2onnx layout: NHWC
input ``input_1`` [n, 76, 32, 1], Transpose to NCHW, Conv (+ bias, or a bias
Add), LeakyRelu / Relu, MaxPool, Transpose back, Reshape / Squeeze to
``conv2d_19`` -- into this form, and raises on any op or attribute the HIP
kernels do not implement. ``to_onnx(graph, path)`` writes a graph in that
layout (so a graph trained or edited here deploys where the reference's does).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Union

import numpy as np

__all__ = ["Conv", "MaxPool", "Graph", "se20_graph", "from_onnx", "to_onnx", "WINDOW_STARTS", "LEAKY_ALPHA"]

LEAKY_ALPHA = 0.2

# Global start frame (in unique-frame coordinates of a 1.44 s clip) of each of
# the reference's 16 embedding windows, in output-slot order: slot 4 w + q
# starts at 12 w + 8 q (audio window w at 1,920 samples = 12 frames,
# embeddings.py:190; embedding window q at stride 8, embeddings.py:136-143).
WINDOW_STARTS = tuple(12 * w + 8 * q for w in range(4) for q in range(4))


@dataclass
class Conv:
    kh: int
    kw: int
    cin: int
    cout: int
    weight: np.ndarray  # [kh, kw, cin, cout] f32 (Keras HWIO)
    bias: np.ndarray    # [cout] f32
    act: Optional[str] = "leaky_relu"
    alpha: float = LEAKY_ALPHA
    name: str = ""

    def __post_init__(self):
        self.weight = np.ascontiguousarray(self.weight, dtype=np.float32)
        self.bias = np.ascontiguousarray(self.bias, dtype=np.float32)
        assert self.weight.shape == (self.kh, self.kw, self.cin, self.cout)
        assert self.bias.shape == (self.cout,)


@dataclass
class MaxPool:
    ph: int
    pw: int
    name: str = ""


Op = Union[Conv, MaxPool]


@dataclass
class Graph:
    ops: List[Op]
    in_shape: tuple = (76, 32, 1)
    name: str = "graph"

    def shapes(self) -> list:
        """Output shape (H, W, C) after every op for one input window."""
        h, w, c = self.in_shape
        out = []
        for op in self.ops:
            if isinstance(op, Conv):
                assert op.cin == c, (op.name, op.cin, c)
                h, w, c = h - op.kh + 1, w - op.kw + 1, op.cout
            else:
                h, w = h // op.ph, w // op.pw
            assert h > 0 and w > 0, f"{op.name} collapses the image"
            out.append((h, w, c))
        return out

    @property
    def out_dim(self) -> int:
        h, w, c = self.shapes()[-1]
        assert h == 1 and w == 1
        return c

    def macs_per_window(self) -> int:
        h, w, c = self.in_shape
        total = 0
        for op, (ho, wo, co) in zip(self.ops, self.shapes()):
            if isinstance(op, Conv):
                total += ho * wo * co * op.kh * op.kw * op.cin
        return total

    def n_params(self) -> int:
        return sum(op.weight.size + op.bias.size for op in self.ops if isinstance(op, Conv))


# (kind, kh, kw, cout) — SE20: 20 convs in 5 groups, 3 max-pools
_SE20 = [
    ("conv", 3, 3, 24), ("conv", 1, 3, 24), ("conv", 3, 1, 24), ("pool", 2, 2, 0),
    ("conv", 1, 3, 32), ("conv", 3, 1, 32), ("conv", 1, 3, 32), ("conv", 3, 1, 32), ("pool", 2, 2, 0),
    ("conv", 1, 3, 48), ("conv", 3, 1, 48), ("conv", 1, 3, 48), ("conv", 3, 1, 48), ("pool", 2, 1, 0),
    ("conv", 3, 1, 64), ("conv", 1, 1, 64), ("conv", 3, 1, 64), ("conv", 1, 1, 64),
    ("conv", 2, 1, 96), ("conv", 1, 1, 96), ("conv", 1, 1, 96), ("conv", 1, 1, 96), ("conv", 1, 1, 96),
]


def se20_graph(seed: int = 1234) -> Graph:
    """Seeded stand-in for the speech-embedding graph: [76,32,1] -> [1,1,96],
    20 convs named conv2d ... conv2d_19 (the last has no activation)."""
    rng = np.random.default_rng(seed)
    ops: List[Op] = []
    cin = 1
    n_conv = sum(1 for s in _SE20 if s[0] == "conv")
    i_conv = 0
    for kind, kh, kw, cout in _SE20:
        if kind == "pool":
            ops.append(MaxPool(kh, kw, name=f"max_pooling2d_{len([o for o in ops if isinstance(o, MaxPool)])}"))
            continue
        fan_in = kh * kw * cin
        w = rng.standard_normal((kh, kw, cin, cout)) * np.sqrt(2.0 / fan_in) * 0.9
        b = rng.standard_normal(cout) * 0.05
        last = i_conv == n_conv - 1
        ops.append(Conv(kh, kw, cin, cout, w.astype(np.float32), b.astype(np.float32),
                        act=None if last else "leaky_relu",
                        name="conv2d" if i_conv == 0 else f"conv2d_{i_conv}"))
        cin = cout
        i_conv += 1
    g = Graph(ops, (76, 32, 1), name="se20")
    assert g.out_dim == 96
    return g


# -- ONNX (Keras / tf2onnx layout) ---------------------------------------------------
_TO_NCHW = (0, 3, 1, 2)
# integer shape arithmetic a Reshape's computed target may come from
_SHAPE_OPS = ("Shape", "Gather", "Slice", "Unsqueeze", "Squeeze", "Concat", "Cast", "Mul", "Div", "Add", "Sub",
              "ReduceProd", "Identity")
_TO_NHWC = (0, 2, 3, 1)


def to_onnx(graph: Graph, path: str, input_name: str = "input_1", opset_version: int = 13) -> None:
    """Write ``graph`` as tf2onnx writes a Keras Conv2D stack: NHWC input
    [n, H, W, C] -> Transpose -> (Conv [Cout, Cin, kh, kw] + bias, LeakyRelu |
    MaxPool)* -> Transpose -> output named after the last conv ([n, 1, 1, out])."""
    from heybuddy.util.onnx_util import write_model
    nodes, inits = [], {}
    x = f"{input_name}__0"
    nodes.append(("Transpose", "transpose_in", [input_name], [x], {"perm": list(_TO_NCHW)}))
    last = max(i for i, op in enumerate(graph.ops) if isinstance(op, Conv))
    n_pool = 0
    for i, op in enumerate(graph.ops):
        if isinstance(op, MaxPool):
            name = op.name or f"max_pooling2d_{n_pool}"
            n_pool += 1
            y = f"{name}/MaxPool"
            nodes.append(("MaxPool", y, [x], [y], {"kernel_shape": [op.ph, op.pw], "strides": [op.ph, op.pw]}))
            x = y
            continue
        name = op.name or f"conv2d_{i}"
        w, b = f"{name}/kernel", f"{name}/bias"
        inits[w] = np.ascontiguousarray(op.weight.transpose(3, 2, 0, 1))  # HWIO -> OIHW
        inits[b] = op.bias
        y = f"{name}/BiasAdd"
        nodes.append(("Conv", y, [x, w, b], [y], {"kernel_shape": [op.kh, op.kw], "strides": [1, 1],
                                                  "dilations": [1, 1], "group": 1, "pads": [0, 0, 0, 0]}))
        x = y
        if op.act == "leaky_relu":
            y = f"{name}/LeakyRelu"
            nodes.append(("LeakyRelu", y, [x], [y], {"alpha": float(op.alpha)}))
            x = y
        if i == last:
            out = name
    h, w_, c = graph.shapes()[-1]
    nodes.append(("Transpose", "transpose_out", [x], [out], {"perm": list(_TO_NHWC)}))
    write_model(path, nodes, inits, [(input_name, ["unk__n", *graph.in_shape])], [(out, ["unk__n", h, w_, c])],
                opset_version=opset_version, producer="tf2onnx-layout (heybuddy-amd)")


def from_onnx(path: str, name: Optional[str] = None) -> Graph:
    """The speech-embedding graph of an ONNX file as runtime data for the HIP
    kernels (the reference's ``speech-embedding.onnx``, embeddings.py:23-42; I/O
    ``input_1`` [n, 76, 32, 1] -> ``conv2d_19`` [n, 1, 1, 96],
    speech-embedding.js:125-146). The graph must be one chain from the input:
    layout Transposes (NHWC <-> NCHW), Conv (stride 1, dilation 1, group 1, no
    padding) with its bias as the Conv's third input or a following Add of a
    [C] / [1, C, 1, 1] constant, per-channel Mul / Add (a BatchNorm folded by
    the exporter) and BatchNormalization (inference form) after a conv --
    folded into its weights and bias --, LeakyRelu / Relu after a conv, MaxPool
    (kernel = stride, no padding), and trailing Reshape / Squeeze / Flatten /
    Identity to the output. A Reshape's target shape may be computed (tf2onnx's
    Shape -> Gather / Slice -> Unsqueeze -> Concat subgraphs): side consumers of
    a chain tensor are allowed when they only feed such shape arithmetic ending
    in a Reshape's shape input. Anything else raises ValueError naming the node."""
    from heybuddy.util.onnx_util import read_model
    m = read_model(path)
    if len(m.inputs) != 1 or len(m.outputs) != 1:
        raise ValueError(f"{path}: expected one graph input and one output, got {m.inputs} / {m.outputs}")
    (in_name, in_dims), (out_name, _) = m.inputs[0], m.outputs[0]
    dims = tuple(in_dims[1:])
    if len(dims) != 3 or any(d is None for d in dims):
        raise ValueError(f"{path}: input {in_name!r} must be [n, H, W, C] (or [n, C, H, W]), got {in_dims}")
    inits = m.initializers
    ops: List[Op] = []
    # the chain from the input; the layout of the tensor "x" (NHWC as Keras, or NCHW)
    nchw = dims[0] == 1 and dims[2] != 1  # [n, 1, H, W]: a one-channel NCHW input
    in_shape = (dims[1], dims[2], dims[0]) if nchw else dims
    x = in_name
    terminal = False

    def const(name_: str) -> np.ndarray:
        if name_ not in inits:
            raise ValueError(f"{path}: {name_!r} must be a constant (initializer) for the HIP kernels")
        return np.asarray(inits[name_], dtype=np.float32)

    def shape_only(node, seen=None) -> bool:
        """node (a Shape of a chain tensor) and everything downstream only compute a
        Reshape's target shape (integer shape arithmetic, no data)."""
        seen = set() if seen is None else seen
        if node.name in seen:
            return True
        seen.add(node.name)
        if node.op not in _SHAPE_OPS:
            return False
        for t in node.outputs:
            for u in m.consumers(t):
                if u.op == "Reshape" and len(u.inputs) > 1 and u.inputs[1] == t and u.inputs[0] != t:
                    continue
                if not shape_only(u, seen):
                    return False
        return True

    def channel_vec(b: np.ndarray, cout: int, where: str) -> np.ndarray:
        """A per-channel constant of a conv's output ([C], [1, C, 1, 1] in NCHW,
        [.., C] in NHWC, or a scalar) as [C]."""
        ok = (b.size == 1 or (b.size == cout and (b.ndim == 1 or (nchw and b.shape[-3:] == (cout, 1, 1))
                                                   or (not nchw and b.shape[-1] == cout))))
        if not ok:
            raise ValueError(f"{where}: constant of shape {b.shape} does not broadcast over {cout} channels")
        return np.broadcast_to(b.reshape(-1), (cout,)).astype(np.float32)

    def conv_before(where: str, what: str) -> "Conv":
        prev = ops[-1] if ops else None
        if not isinstance(prev, Conv) or prev.act is not None:
            raise ValueError(f"{where}: {what} is supported only right after a conv (before its activation)")
        return prev

    while x != out_name:
        users = m.consumers(x)
        data = [u for u in users if not (u.op == "Shape" and shape_only(u))]
        if len(data) != 1:
            raise ValueError(f"{path}: tensor {x!r} feeds {len(data)} nodes; only a single chain is supported")
        node = data[0]
        a = node.attrs
        where = f"{path}: node {node.name!r} ({node.op})"
        if terminal and node.op not in ("Reshape", "Squeeze", "Flatten", "Identity"):
            raise ValueError(f"{where}: after a reshape only reshapes may follow")
        if node.op == "Transpose":
            perm = tuple(a.get("perm", ()))
            if perm == _TO_NCHW and not nchw:
                nchw = True
            elif perm == _TO_NHWC and nchw:
                nchw = False
            else:
                raise ValueError(f"{where}: unsupported permutation {perm}")
        elif node.op == "Conv":
            if not nchw:
                raise ValueError(f"{where}: Conv on an NHWC tensor")
            w = const(node.inputs[1])
            if w.ndim != 4:
                raise ValueError(f"{where}: only 2-D convolutions are supported")
            co, ci, kh, kw = w.shape
            if (tuple(a.get("strides", (1, 1))) != (1, 1) or tuple(a.get("dilations", (1, 1))) != (1, 1)
                    or int(a.get("group", 1)) != 1 or any(a.get("pads", (0, 0, 0, 0)))
                    or a.get("auto_pad", b"NOTSET") not in (b"NOTSET", b"VALID")):
                raise ValueError(f"{where}: only stride-1, undilated, ungrouped 'valid' convolutions run on the "
                                 f"HIP kernels (attributes {a})")
            b = const(node.inputs[2]).reshape(-1) if len(node.inputs) > 2 and node.inputs[2] else np.zeros(co, np.float32)
            ops.append(Conv(kh, kw, ci, co, w.transpose(2, 3, 1, 0), b, act=None,
                            name=(node.name.split("/")[0] or f"conv2d_{len(ops)}")))
        elif node.op in ("Add", "Sub"):
            prev = conv_before(where, f"an {node.op} of a per-channel constant")
            if node.op == "Sub" and node.inputs[0] != x:
                raise ValueError(f"{where}: only x - constant is supported")
            other = node.inputs[1] if node.inputs[0] == x else node.inputs[0]
            b = channel_vec(const(other), prev.cout, where)
            prev.bias = np.ascontiguousarray(prev.bias + (b if node.op == "Add" else -b), dtype=np.float32)
        elif node.op == "Mul":  # a per-channel scale (BatchNorm folded as Mul / Add): into W and b
            prev = conv_before(where, "a Mul by a per-channel constant")
            other = node.inputs[1] if node.inputs[0] == x else node.inputs[0]
            sc = channel_vec(const(other), prev.cout, where)
            prev.weight = np.ascontiguousarray(prev.weight * sc, dtype=np.float32)
            prev.bias = np.ascontiguousarray(prev.bias * sc, dtype=np.float32)
        elif node.op == "BatchNormalization":  # inference form: y = (x - mean) / sqrt(var + eps) * g + b
            prev = conv_before(where, "a BatchNormalization")
            if not nchw or len(node.outputs) > 1 and any(node.outputs[1:]) or int(a.get("training_mode", 0)):
                raise ValueError(f"{where}: only the inference form over NCHW channels is supported")
            g_, b_, mu, var = (channel_vec(const(t), prev.cout, where) for t in node.inputs[1:5])
            sc = (g_.astype(np.float64) / np.sqrt(var.astype(np.float64) + float(a.get("epsilon", 1e-5))))
            prev.weight = np.ascontiguousarray(prev.weight * sc, dtype=np.float32)
            prev.bias = np.ascontiguousarray((prev.bias - mu) * sc + b_, dtype=np.float32)
        elif node.op in ("LeakyRelu", "Relu"):
            prev = conv_before(where, "an activation")
            prev.act = "leaky_relu"
            prev.alpha = float(np.float32(a.get("alpha", 0.01))) if node.op == "LeakyRelu" else 0.0
        elif node.op == "MaxPool":
            if not nchw:
                raise ValueError(f"{where}: MaxPool on an NHWC tensor")
            k = tuple(a.get("kernel_shape", ()))
            s = tuple(a.get("strides", k))
            if (len(k) != 2 or s != k or any(a.get("pads", (0, 0, 0, 0)))
                    or a.get("auto_pad", b"NOTSET") not in (b"NOTSET", b"VALID")
                    or int(a.get("ceil_mode", 0)) or tuple(a.get("dilations", (1, 1))) != (1, 1)):
                raise ValueError(f"{where}: only non-overlapping unpadded max-pools are supported ({a})")
            ops.append(MaxPool(k[0], k[1], name=node.name.split("/")[0]))
        elif node.op in ("Reshape", "Squeeze", "Flatten", "Identity"):
            terminal = node.op != "Identity" or terminal
        else:
            raise ValueError(f"{where}: op {node.op!r} is not supported by the HIP embedding kernels")
        x = node.outputs[0]
    if not any(isinstance(o, Conv) for o in ops):
        raise ValueError(f"{path}: no convolution on the path from {in_name!r} to {out_name!r}")
    g = Graph(ops, tuple(int(d) for d in in_shape), name=name or out_name)
    h, w_, _ = g.shapes()[-1]  # also checks the channel chain
    if (h, w_) != (1, 1):
        raise ValueError(f"{path}: the graph ends at {g.shapes()[-1]}, not a [1, 1, C] embedding")
    return g
