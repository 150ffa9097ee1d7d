"""Speech-embedding oracle (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Restates what ``SpeechEmbeddingModel.__call__`` (reference
src/python/heybuddy/embeddings.py:32-42) computes: the ONNX graph applied to
each [76, 32, 1] mel window independently -> [96], then ``.squeeze()``.
The graph is given as runtime data (heybuddy.embedding_graph: Keras-style
valid Conv2D + LeakyReLU + MaxPool2D, NHWC); the true graph is absent offline,
so parity is against this executor (PARITY UNPINNED vs the real network).
Evaluated per window exactly as the reference does — no prefix sharing — so
it also checks the HIP path's shared-prefix deduplication.
"""
from __future__ import annotations

import numpy as np


def conv2d_valid(x: np.ndarray, w: np.ndarray, b: np.ndarray, dtype=np.float64) -> np.ndarray:
    """x [n, H, W, C], w [kh, kw, C, O] -> [n, H-kh+1, W-kw+1, O] (im2col GEMM)."""
    n, H, W, C = x.shape
    kh, kw, _, O = w.shape
    ho, wo = H - kh + 1, W - kw + 1
    cols = np.empty((n, ho, wo, kh, kw, C), dtype=dtype)
    for dh in range(kh):
        for dw in range(kw):
            cols[:, :, :, dh, dw, :] = x[:, dh:dh + ho, dw:dw + wo, :]
    y = cols.reshape(n * ho * wo, kh * kw * C) @ w.reshape(kh * kw * C, O).astype(dtype)
    return (y + b.astype(dtype)).reshape(n, ho, wo, O)


def maxpool(x: np.ndarray, ph: int, pw: int) -> np.ndarray:
    n, H, W, C = x.shape
    ho, wo = H // ph, W // pw
    x = x[:, :ho * ph, :wo * pw, :].reshape(n, ho, ph, wo, pw, C)
    return x.max(axis=(2, 4))


def run_graph(graph, windows: np.ndarray, dtype=np.float64, batch: int = 256) -> np.ndarray:
    """windows [n, 76, 32] or [n, 76, 32, 1] -> [n, out_dim] (in ``dtype``)."""
    from heybuddy.embedding_graph import Conv
    x = np.asarray(windows)
    if x.ndim == 3:
        x = x[..., None]
    outs = []
    for s in range(0, x.shape[0], batch):
        h = x[s:s + batch].astype(dtype)
        for op in graph.ops:
            if isinstance(op, Conv):
                h = conv2d_valid(h, op.weight, op.bias, dtype)
                if op.act == "leaky_relu":
                    h = np.where(h >= 0, h, h * dtype(op.alpha) if dtype is not None else h * op.alpha)
            else:
                h = maxpool(h, op.ph, op.pw)
        outs.append(h.reshape(h.shape[0], -1))
    return np.concatenate(outs, axis=0) if outs else np.zeros((0, graph.out_dim), dtype)


def speech_embedding_model(graph, spectrograms: np.ndarray) -> np.ndarray:
    """SpeechEmbeddingModel.__call__: [n,76,32,1] -> [n,1,1,96] -> squeeze."""
    out = run_graph(graph, spectrograms, dtype=np.float32)
    return out.reshape(out.shape[0], 1, 1, -1).squeeze()
