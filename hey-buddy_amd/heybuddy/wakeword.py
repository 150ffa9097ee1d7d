"""Drop-in for heybuddy.wakeword's default classifier (reference
src/python/heybuddy/wakeword.py:171-348).

``WakeWordMLPModel`` keeps the reference's constructor, state_dict names and
shapes (checkpoints and the shipped src/js/models/*.onnx heads load with
strict=True, through heybuddy.util.onnx_util), ``from_file``, ``predict``,
``predict_timecodes`` and ``save_onnx``, but its parameters are views into
ONE flat f32 buffer laid out for libhbk.so, and ``forward`` runs the fused HIP
forward (hbk_mlp_forward). Training goes through the fused HIP train step
(heybuddy.trainer), not autograd. Only the default architecture is on the MI355X
path: gated MLP (DEFAULT_USE_GATING), no half layers, SiLU.
"""
from __future__ import annotations

import random
from collections import OrderedDict
from typing import Any, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
import torch.nn as nn

from heybuddy import _native
from heybuddy.constants import (DEFAULT_LAYER_DIM, DEFAULT_LAYERS, DEFAULT_USE_GATING,
                                DEFAULT_USE_HALF_LAYERS)
from heybuddy.kernels import MlpPlan

__all__ = ["WakeWordMLPModel", "get_normalized_dim"]


def get_normalized_dim(dim: int, multiple_of: int = 8, down_ratio: float = 2 / 3) -> int:
    """modeling_util.py:42-72: int(dim * 2/3) rounded up to a multiple of 8."""
    v = int(dim * down_ratio)
    return v if v % multiple_of == 0 else v + multiple_of - v % multiple_of


class _Affine(nn.Module):
    """Holds a weight and a bias (LayerNorm / Linear slots of the reference)."""

    def __init__(self, w: torch.Tensor, b: torch.Tensor) -> None:
        super().__init__()
        self.weight = nn.Parameter(w)
        self.bias = nn.Parameter(b)


class _Gmlp(nn.Module):
    def __init__(self, views, prefix: str) -> None:
        super().__init__()
        self.hidden = _Affine(views[f"{prefix}.hidden.weight"], views[f"{prefix}.hidden.bias"])
        self.output = _Affine(views[f"{prefix}.output.weight"], views[f"{prefix}.output.bias"])
        self.gate = _Affine(views[f"{prefix}.gate.weight"], views[f"{prefix}.gate.bias"])


class WakeWordMLPModel(nn.Module):
    """input > dropout > flatten > LN > gated MLP > [LN > gated MLP] x L > LN >
    gated MLP > sigmoid (wakeword.py:334-348). Input [B, 16, 96] -> [B, 1]."""

    def __init__(self, input_shape: Tuple[int, int] = (16, 96), layer_dim: int = DEFAULT_LAYER_DIM,
                 num_layers: int = DEFAULT_LAYERS, use_gating: bool = DEFAULT_USE_GATING,
                 use_half_layers: bool = DEFAULT_USE_HALF_LAYERS, dropout: float = 0.1,
                 activation: Optional[str] = "silu") -> None:
        super().__init__()
        if not use_gating or use_half_layers or activation not in ("silu", "swish"):
            raise NotImplementedError("the MI355X path implements the default architecture: gated MLP, "
                                      "no half layers, SiLU")
        self.input_shape = tuple(input_shape)
        self.input_features = input_shape[0] * input_shape[1]
        self.use_gating = use_gating
        self.use_half_layers = use_half_layers
        self.layer_dim = layer_dim
        self.num_layers = num_layers
        self.plan = MlpPlan(self.input_features, layer_dim, get_normalized_dim(layer_dim), num_layers)
        self.dropout = nn.Dropout(dropout)
        flat = torch.zeros(self.plan.n_params, dtype=torch.float32)
        self._bind(flat, build=True)
        self._reset_parameters()

    # -- flat parameter buffer ------------------------------------------------
    def _bind(self, flat: torch.Tensor, build: bool = False) -> None:
        views = self.plan.views(flat)
        if build:
            self.norm_in = _Affine(views["norm_in.weight"], views["norm_in.bias"])
            self.mlp_in = _Gmlp(views, "mlp_in")
            self.layers = nn.ModuleList(
                nn.ModuleList([_Affine(views[f"layers.{l}.0.weight"], views[f"layers.{l}.0.bias"]),
                               _Gmlp(views, f"layers.{l}.1")]) for l in range(self.num_layers))
            self.norm_out = _Affine(views["norm_out.weight"], views["norm_out.bias"])
            self.mlp_out = _Gmlp(views, "mlp_out")
        else:
            params = dict(self.named_parameters())
            for name, view in views.items():
                params[name].data = view
        self._flat = flat

    @property
    def flat_parameters(self) -> torch.Tensor:
        """All parameters as one contiguous f32 tensor (the kernels' layout)."""
        return self._flat

    def _apply(self, fn, recurse=True):
        flat = fn(self._flat)
        if flat.data_ptr() != self._flat.data_ptr() or flat.device != self._flat.device:
            self._bind(flat.contiguous())
        for p in self.parameters():
            if p.grad is not None:
                p.grad = fn(p.grad)
        return self

    @torch.no_grad()
    def _reset_parameters(self) -> None:
        """nn.Linear / nn.LayerNorm default initialisation (fan-in uniform)."""
        for name, p in self.named_parameters():
            if ".hidden." in name or ".output." in name or ".gate." in name:
                lin = name.rsplit(".", 1)[0]
                fan_in = dict(self.named_parameters())[f"{lin}.weight"].shape[1]
                bound = 1.0 / np.sqrt(fan_in)
                p.uniform_(-bound, bound)
            elif name.endswith("weight"):
                p.fill_(1.0)
            else:
                p.zero_()

    @property
    def device(self) -> torch.device:
        return self._flat.device

    @property
    def dtype(self) -> torch.dtype:
        return self._flat.dtype

    # -- inference ---------------------------------------------------------
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """[B, 16, 96] -> [B, 1] probabilities on the HIP path. In training mode
        the input dropout is applied, as in the reference (it never calls
        .eval(), so its validation passes run with dropout too)."""
        if self._flat.device.type != "cuda":
            raise _native.HBKUnavailable("WakeWordMLPModel runs on a HIP device: call .to('cuda') first")
        x = x.to(device=self._flat.device, dtype=torch.float32)
        p = self.dropout.p if self.training else 0.0
        prob = self.plan.forward(self._flat, x.reshape(x.shape[0], -1), dropout_p=p,
                                 seed=random.getrandbits(63))
        return prob.unsqueeze(1)

    def logits(self, x: torch.Tensor) -> torch.Tensor:
        """Pre-sigmoid outputs [B] (dropout off)."""
        x = x.to(device=self._flat.device, dtype=torch.float32)
        _, z = self.plan.forward(self._flat, x.reshape(x.shape[0], -1), logits=True)
        return z

    @classmethod
    def from_file(cls, path: str, device: Optional[torch.device] = None) -> "WakeWordMLPModel":
        """wakeword.py:249-276: infer layer_dim / num_layers from the state_dict.
        ``.onnx`` heads (the reference's shipped src/js/models/*.onnx, or
        ``save_onnx`` output) load from their initializers."""
        if str(path).lower().endswith(".onnx"):
            from heybuddy.util.onnx_util import read_initializers
            state_dict = {k: torch.from_numpy(v) for k, v in read_initializers(path).items()}
        else:
            state_dict = torch.load(path, weights_only=True, map_location="cpu")
        layer_dim = state_dict["norm_out.weight"].shape[0]
        num_layers = 0
        while f"layers.{num_layers}.0.weight" in state_dict:
            num_layers += 1
        model = cls(layer_dim=layer_dim, num_layers=num_layers)
        model.load_state_dict(state_dict)
        if device is not None:
            model.to(device)
        return model

    def save_onnx(self, path: str, opset_version: int = 19) -> None:
        """wakeword.py:316-332: the head as an ONNX file with the exporter's
        graph (input ``input`` [1, 16, 96], output ``output`` [1, 1])."""
        from heybuddy.util.onnx_util import write_wakeword_onnx
        sd = OrderedDict((k, v.detach().float().cpu().numpy()) for k, v in self.state_dict().items())
        write_wakeword_onnx(path, sd, self.num_layers, self.input_shape, opset_version=opset_version)

    # -- WakeWordInferenceMixin.predict (wakeword.py:129-169) ---------------
    @property
    def speech_embeddings(self):
        from heybuddy.embeddings import get_speech_embeddings
        if not hasattr(self, "_speech_embeddings"):
            idx = self.device.index if self.device.type == "cuda" else None
            self._speech_embeddings = get_speech_embeddings(device_id=idx)
        return self._speech_embeddings

    @torch.no_grad()
    def predict(self, audio: Any, threshold: float = 0.5, embedding_spectrogram_batch_size: int = 32,
                embedding_batch_size: int = 32, return_scores: bool = False,
                min_frames: int = 23040) -> Union[Tuple[bool, ...], Tuple[float, ...]]:
        from heybuddy.util import audio_to_bct_tensor
        audio_tensor, _ = audio_to_bct_tensor(audio, sample_rate=16000)
        n, c, t = audio_tensor.shape
        if t < min_frames:
            pad = min_frames - t
            left = int(pad / 2)
            audio_tensor = torch.cat([torch.zeros(n, c, left, dtype=audio_tensor.dtype), audio_tensor,
                                      torch.zeros(n, c, pad - left, dtype=audio_tensor.dtype)], dim=-1)
        emb = self.speech_embeddings(audio_tensor, embedding_batch_size=embedding_batch_size,
                                     spectrogram_batch_size=embedding_spectrogram_batch_size)
        pred = self(torch.tensor(emb, device=self.device, dtype=torch.float32)).cpu().numpy()
        if return_scores:
            return tuple(pred.flatten())
        return tuple(pred > threshold)

    @staticmethod
    def timecode_windows(audio_tensor: torch.Tensor) -> torch.Tensor:
        """wakeword.py:59-90: mono [t] -> 2-s windows every 1 s [n, 1, 32000]
        (padded to whole seconds, 1 s of silence on both ends)."""
        if audio_tensor.dim() == 3:
            _, c, _ = audio_tensor.shape
            audio_tensor = audio_tensor[0, 0, :] if c == 1 else audio_tensor[0, :, :].mean(dim=0)
        t = audio_tensor.shape[0]
        rem = t % 16000
        z = lambda n: torch.zeros(n, dtype=audio_tensor.dtype, device=audio_tensor.device)  # noqa: E731
        if rem > 0:
            audio_tensor = torch.cat([audio_tensor, z(16000 - rem)])
        audio_tensor = torch.cat([z(16000), audio_tensor, z(16000)])
        starts = range(0, audio_tensor.shape[0] - 16000, 16000)
        return torch.stack([audio_tensor[i:i + 32000] for i in starts]).unsqueeze(1)

    @staticmethod
    def timecodes(predictions: Sequence[bool]) -> List[float]:
        """wakeword.py:99-110: a positive window i is reported at i + 0.5 when
        window i + 1 is positive too, skipped when it is the last window and
        follows a positive one, else at i."""
        out: List[float] = []
        n = len(predictions)
        for i, hit in enumerate(predictions):
            if not hit:
                continue
            if i < n - 1 and predictions[i + 1]:
                out.append(i + 0.5)
            elif i == n - 1 and predictions[i - 1]:
                continue
            else:
                out.append(i)
        return out

    @torch.no_grad()
    def window_scores(self, windows: torch.Tensor) -> torch.Tensor:
        """Score of each audio window [n, 1, T]: a 2-s window yields more
        embedding rows (32) than the head takes (16), which the reference's
        predict() passes to the head unchanged (its LayerNorm(1536) then
        rejects the 3072-wide input). Here the head scores every 16-row run of
        the window's embeddings (the JS detector's rolling buffer,
        src/js/src/hey-buddy.js:88, wakeWordEmbeddingFrames = 16) and the window
        keeps the highest score."""
        x = windows.reshape(windows.shape[0], -1).to(self.device, torch.float32)
        emb = self.speech_embeddings.featurize(x)  # [n, m, 96] on the device
        rows = self.input_shape[0]
        n, m, d = emb.shape
        if m < rows:
            raise ValueError(f"windows of {x.shape[1]} samples give {m} < {rows} embedding rows")
        runs = emb.unfold(1, rows, 1).permute(0, 1, 3, 2).reshape(-1, rows, d)  # [n * (m - rows + 1), rows, d]
        return self(runs.contiguous()).reshape(n, m - rows + 1).amax(dim=1)

    @torch.no_grad()
    def predict_timecodes(self, audio: Any, threshold: float = 0.5, embedding_spectrogram_batch_size: int = 32,
                          embedding_batch_size: int = 32) -> List[float]:
        """Per-second detections in one clip (wakeword.py:50-110): 2-s windows
        every second, all featurized and scored in one batch on the device
        (window_scores), then the reference's timecode rule."""
        from heybuddy.util import audio_to_bct_tensor
        audio_tensor, _ = audio_to_bct_tensor(audio, sample_rate=16000)
        scores = self.window_scores(self.timecode_windows(audio_tensor))
        return self.timecodes((scores > threshold).tolist())
