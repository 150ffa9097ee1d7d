"""torch-facing wrappers over the libhbk.so C ABI (include/hbk.h).

Each wrapper validates shapes on the host (the kernels assume them), passes
raw device pointers and torch's current stream, and is registered as a
``torch.library`` custom op under the ``hbk`` namespace
(``torch.ops.hbk.mel_frames`` ...), so callers can treat it like any other
torch op. Nothing here computes on the CPU.
"""
from __future__ import annotations

import ctypes
import itertools
import threading
from typing import Dict

import numpy as np
import torch

from heybuddy import _native
from heybuddy._native import check, lib, ptr, stream_ptr

__all__ = ["MelPlan", "mel_frames"]

_plans: Dict[int, "MelPlan"] = {}
_plan_ids = itertools.count(1)
_plans_lock = threading.Lock()


class MelPlan:
    """Device tables for hbk_mel_frames (window, twiddles, sparse filterbank).

    Built once per (window, fbank, scaling); see hbk_mel_plan_create.
    """

    def __init__(self, window: np.ndarray, fbank: np.ndarray, hop: int = 160,
                 in_scale: float = 32767.0, log_floor: float = 1e-10,
                 out_div: float = 10.0, out_add: float = 2.0,
                 device: torch.device | int | None = None) -> None:
        self.device = _native.require_device(device)
        window = np.ascontiguousarray(window, dtype=np.float32)
        fbank = np.ascontiguousarray(fbank, dtype=np.float32)
        if window.ndim != 1 or fbank.ndim != 2 or fbank.shape[0] != window.shape[0] // 2 + 1:
            raise ValueError(f"bad window {window.shape} / fbank {fbank.shape}")
        self.n_fft = int(window.shape[0])
        self.hop = int(hop)
        self.n_mels = int(fbank.shape[1])
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().hbk_mel_plan_create(
                window.ctypes.data, fbank.ctypes.data, self.n_fft, self.hop, self.n_mels,
                float(in_scale), float(log_floor), float(out_div), float(out_add),
                ctypes.byref(handle)), "hbk_mel_plan_create")
        self._handle = handle
        with _plans_lock:
            self.id = next(_plan_ids)
            _plans[self.id] = self

    def n_frames(self, n_samples: int) -> int:
        return 0 if n_samples < self.n_fft else (n_samples - self.n_fft) // self.hop + 1

    def __call__(self, pcm: torch.Tensor, n_frames: int | None = None) -> torch.Tensor:
        return mel_frames(pcm, self, n_frames)

    def __del__(self) -> None:
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            try:
                lib().hbk_mel_plan_destroy(h)
            except Exception:
                pass
            self._handle = None


@torch.library.custom_op("hbk::mel_frames", mutates_args=())
def _mel_frames_op(pcm: torch.Tensor, n_frames: int, plan_id: int) -> torch.Tensor:
    plan = _plans[plan_id]
    n_clips = pcm.shape[0]
    out = torch.empty((n_clips, n_frames, plan.n_mels), dtype=torch.float32, device=pcm.device)
    check(lib().hbk_mel_frames(plan._handle, ptr(pcm), n_clips, pcm.stride(0), n_frames,
                               ptr(out), stream_ptr(pcm.device)), "hbk_mel_frames")
    return out


@_mel_frames_op.register_fake
def _(pcm, n_frames, plan_id):
    plan = _plans[plan_id]
    return pcm.new_empty((pcm.shape[0], n_frames, plan.n_mels))


def mel_frames(pcm: torch.Tensor, plan: MelPlan, n_frames: int | None = None) -> torch.Tensor:
    """Unique log-mel frames of every clip: pcm [B, T] f32 on the plan's device
    -> [B, n_frames, n_mels] f32 (frame f = samples [hop f, hop f + 512))."""
    if pcm.dim() != 2 or pcm.dtype != torch.float32 or pcm.device != plan.device:
        raise ValueError(f"pcm must be [B, T] float32 on {plan.device}, got "
                         f"{tuple(pcm.shape)} {pcm.dtype} {pcm.device}")
    if pcm.stride(1) != 1 or pcm.stride(0) % 2 or pcm.data_ptr() % 8:
        pcm = _aligned_copy(pcm)
    max_frames = plan.n_frames(pcm.shape[1])
    n_frames = max_frames if n_frames is None else int(n_frames)
    if n_frames < 0 or n_frames > max_frames:
        raise ValueError(f"n_frames {n_frames} outside [0, {max_frames}] for T={pcm.shape[1]}")
    return torch.ops.hbk.mel_frames(pcm, n_frames, plan.id)


def _aligned_copy(x: torch.Tensor) -> torch.Tensor:
    """Contiguous copy with an even row stride (the kernel loads float2)."""
    t = x.shape[1]
    buf = torch.empty((x.shape[0], t + (t & 1)), dtype=x.dtype, device=x.device)
    buf[:, :t].copy_(x)
    return buf[:, :t]
