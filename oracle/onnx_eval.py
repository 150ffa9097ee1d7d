"""A small numpy interpreter for ONNX graphs -- TEST INFRASTRUCTURE ONLY.

Runs the graphs the importers read (heybuddy.embedding_graph.from_onnx,
heybuddy.spectrogram.mel_params_from_onnx) so that tests can check an import
against the file's own semantics: the ONNX operator definitions (opset 13-19)
restated in float64 numpy. It stands in for ONNX Runtime, which the reference
uses to run these graphs (src/python/heybuddy/util/onnx_util.py:63-96) and
which is not installed here. Only tests/ import it; the product never does.

Operators: Transpose, Conv (1-D / 2-D, pads, strides, group 1), LeakyRelu,
Relu, MaxPool, Reshape, Squeeze, Unsqueeze, Flatten, Identity, Cast, Add, Sub,
Mul, Div, Pow, Max, Min, Sqrt, Abs, Log, Exp, Neg, Clip, MatMul, ReduceSum,
Concat, Slice, STFT, and the shape / normalisation ops of tf2onnx exports:
Shape, Gather, ReduceProd, BatchNormalization (inference form).
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np
from numpy.lib.stride_tricks import sliding_window_view

__all__ = ["run"]


def _axes(node, vals, k=1):
    if "axes" in node.attrs:
        return [int(a) for a in node.attrs["axes"]]
    if len(node.inputs) > k and node.inputs[k]:
        return [int(a) for a in np.asarray(vals[node.inputs[k]]).reshape(-1)]
    return None


def _conv(x, w, b, a):
    nd = w.ndim - 2
    strides = list(a.get("strides", [1] * nd))
    pads = list(a.get("pads", [0] * (2 * nd)))
    if any(d != 1 for d in a.get("dilations", [1] * nd)) or int(a.get("group", 1)) != 1:
        raise NotImplementedError("dilated / grouped Conv")
    x = np.pad(x, [(0, 0), (0, 0)] + [(pads[i], pads[i + nd]) for i in range(nd)])
    k = w.shape[2:]
    win = sliding_window_view(x, k, axis=tuple(range(2, 2 + nd)))
    win = win[(slice(None), slice(None)) + tuple(slice(None, None, s) for s in strides)]
    if nd == 1:
        y = np.einsum("ncok,mck->nmo", win, w)
    else:
        y = np.einsum("ncopkl,mckl->nmop", win, w)
    if b is not None:
        y = y + b.reshape((1, -1) + (1,) * nd)
    return y


def _maxpool(x, a):
    k = list(a["kernel_shape"])
    s = list(a.get("strides", k))
    if any(a.get("pads", [0] * 2 * len(k))):
        raise NotImplementedError("padded MaxPool")
    win = sliding_window_view(x, k, axis=tuple(range(2, 2 + len(k))))
    win = win[(slice(None), slice(None)) + tuple(slice(None, None, t) for t in s)]
    return win.max(axis=tuple(range(-len(k), 0)))


def _stft(node, vals):
    sig = np.asarray(vals[node.inputs[0]])
    step = int(np.asarray(vals[node.inputs[1]]).reshape(-1)[0])
    win = np.asarray(vals[node.inputs[2]]) if len(node.inputs) > 2 and node.inputs[2] else None
    n = (int(np.asarray(vals[node.inputs[3]]).reshape(-1)[0]) if len(node.inputs) > 3 and node.inputs[3]
         else win.size)
    if sig.shape[-1] != 1:
        raise NotImplementedError("complex STFT input")
    s = sig[..., 0]
    frames = sliding_window_view(s, n, axis=-1)[:, ::step]  # [b, F, n]
    if win is not None:
        frames = frames * win
    spec = np.fft.rfft(frames, axis=-1) if int(node.attrs.get("onesided", 1)) else np.fft.fft(frames, axis=-1)
    return np.stack([spec.real, spec.imag], axis=-1)


def _slice(node, vals, x):
    starts = np.asarray(vals[node.inputs[1]]).reshape(-1)
    ends = np.asarray(vals[node.inputs[2]]).reshape(-1)
    axes = (np.asarray(vals[node.inputs[3]]).reshape(-1) if len(node.inputs) > 3 and node.inputs[3]
            else np.arange(len(starts)))
    steps = (np.asarray(vals[node.inputs[4]]).reshape(-1) if len(node.inputs) > 4 and node.inputs[4]
             else np.ones(len(starts), np.int64))
    sl = [slice(None)] * x.ndim
    for s, e, ax, st in zip(starts, ends, axes, steps):
        sl[int(ax)] = slice(int(s), int(e), int(st))
    return x[tuple(sl)]


def run(model, feeds: Dict[str, np.ndarray], outputs: Sequence[str] = ()) -> Dict[str, np.ndarray]:
    """Evaluate ``model`` (an onnx_util.OnnxModel or a path) on ``feeds``
    (name -> array) in float64; returns the graph outputs (or ``outputs``)."""
    if isinstance(model, str):
        from heybuddy.util.onnx_util import read_model
        model = read_model(model)
    vals: Dict[str, np.ndarray] = {k: (np.asarray(v, np.float64) if np.asarray(v).dtype.kind == "f" else np.asarray(v))
                                   for k, v in model.initializers.items()}
    vals.update({k: np.asarray(v, np.float64) for k, v in feeds.items()})
    for node in model.nodes:
        a, op = node.attrs, node.op
        ins = [vals[i] if i else None for i in node.inputs]
        x = ins[0] if ins else None
        if op == "Transpose":
            y = np.transpose(x, a.get("perm"))
        elif op == "Conv":
            y = _conv(x, ins[1], ins[2] if len(ins) > 2 else None, a)
        elif op == "LeakyRelu":
            y = np.where(x >= 0, x, x * float(a.get("alpha", 0.01)))
        elif op == "Relu":
            y = np.maximum(x, 0.0)
        elif op == "MaxPool":
            y = _maxpool(x, a)
        elif op == "Reshape":
            shape = [int(s) for s in np.asarray(ins[1]).reshape(-1)]
            shape = [x.shape[i] if s == 0 else s for i, s in enumerate(shape)]
            y = x.reshape(shape)
        elif op == "Squeeze":
            ax = _axes(node, vals)
            y = np.squeeze(x, axis=None if ax is None else tuple(ax))
        elif op == "Unsqueeze":
            y = x
            ax = _axes(node, vals)
            for d in sorted(int(v) % (x.ndim + len(ax)) for v in ax):
                y = np.expand_dims(y, d)
        elif op == "Flatten":
            ax = int(a.get("axis", 1))
            y = x.reshape(int(np.prod(x.shape[:ax])), -1)
        elif op in ("Identity", "Cast"):
            y = x
        elif op in ("Add", "Sub", "Mul", "Div", "Pow"):
            f = {"Add": np.add, "Sub": np.subtract, "Mul": np.multiply, "Div": np.divide, "Pow": np.power}[op]
            y = f(x, ins[1])
        elif op in ("Max", "Min"):
            y = ins[0]
            for v in ins[1:]:
                y = (np.maximum if op == "Max" else np.minimum)(y, v)
        elif op in ("Sqrt", "Abs", "Log", "Exp", "Neg"):
            y = {"Sqrt": np.sqrt, "Abs": np.abs, "Log": np.log, "Exp": np.exp, "Neg": np.negative}[op](x)
        elif op == "Clip":
            lo = a.get("min", ins[1] if len(ins) > 1 and ins[1] is not None else -np.inf)
            hi = a.get("max", ins[2] if len(ins) > 2 and ins[2] is not None else np.inf)
            y = np.clip(x, lo, hi)
        elif op == "MatMul":
            y = np.matmul(x, ins[1])
        elif op == "ReduceSum":
            ax = _axes(node, vals)
            y = np.sum(x, axis=None if ax is None else tuple(ax), keepdims=bool(int(a.get("keepdims", 1))))
        elif op == "Concat":
            y = np.concatenate(ins, axis=int(a["axis"]))
        elif op == "Slice":
            y = _slice(node, vals, x)
        elif op == "STFT":
            y = _stft(node, vals)
        elif op == "Shape":
            shp = np.asarray(x.shape, np.int64)
            y = shp[int(a.get("start", 0)):a.get("end", None)]
        elif op == "Gather":
            y = np.take(x, np.asarray(ins[1]).astype(np.int64), axis=int(a.get("axis", 0)))
        elif op == "ReduceProd":
            y = np.asarray(np.prod(x), dtype=x.dtype).reshape([1] * x.ndim if int(a.get("keepdims", 1)) else [])
        elif op == "BatchNormalization":  # inference form over axis 1
            c = (1, -1) + (1,) * (x.ndim - 2)
            g_, b_, mu, var = (np.asarray(v, np.float64).reshape(c) for v in ins[1:5])
            y = (x - mu) / np.sqrt(var + float(a.get("epsilon", 1e-5))) * g_ + b_
        else:
            raise NotImplementedError(f"onnx_eval: operator {op}")
        vals[node.outputs[0]] = y
    names = list(outputs) or [n for n, _ in model.outputs]
    return {n: vals[n] for n in names}
