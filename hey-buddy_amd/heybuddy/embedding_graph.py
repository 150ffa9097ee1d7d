"""The speech-embedding graph as runtime data.

The reference runs Google's speech_embedding network as an opaque ONNX file
(SpeechEmbeddingModel, embeddings.py:23-42; I/O ``input_1`` [n,76,32,1] ->
``conv2d_19`` [n,1,1,96], src/js/src/models/speech-embedding.js:125-146)
that is downloaded at run time and absent offline. Its topology and weights
are therefore NOT known here. This module describes the network as a list of
ops (Keras Conv2D 'valid' / LeakyReLU / MaxPool2D, NHWC) that libhbk.so
executes generically; ``se20_graph()`` is a 20-conv stand-in with the same
I/O signature and the same last node name, with seeded weights. A graph read
from the real ONNX file (sha256 70d16429..., embeddings.py:30) can be passed in
the same form once it is supplied out of band.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Union

import numpy as np

__all__ = ["Conv", "MaxPool", "Graph", "se20_graph", "WINDOW_STARTS", "LEAKY_ALPHA"]

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
