"""Loader for libhbk.so — the C ABI declared in include/hbk.h.

The HIP kernels are the only compute path: if the library or a GPU is
missing, every entry point raises ``HBKUnavailable``. There is no CPU
fallback in this package (the CPU restatement lives in ``oracle/`` and is
test infrastructure only).

Tensors cross the boundary as raw device pointers (``tensor.data_ptr()``)
plus sizes; work is enqueued on torch's current HIP stream.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch  # noqa: F401  (loads the process' HIP runtime before libhbk.so)

__all__ = ["HBKError", "HBKUnavailable", "lib", "check", "stream_ptr", "require_device",
           "LIB_PATH"]

LIB_PATH = os.environ.get(
    "HBK_LIB",
    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libhbk.so"),
)


class HBKError(RuntimeError):
    """A libhbk.so entry point returned a non-zero status."""


class HBKUnavailable(HBKError):
    """libhbk.so (or a HIP device) is not available: the HIP path cannot run."""


_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None

_c_int64 = ctypes.c_int64
_c_int = ctypes.c_int
_c_float = ctypes.c_float
_vp = ctypes.c_void_p

# name -> (restype, argtypes); must match include/hbk.h
_PROTOS = {
    "hbk_version": (ctypes.c_char_p, []),
    "hbk_last_error": (ctypes.c_char_p, []),
    "hbk_device_count": (_c_int, [ctypes.POINTER(_c_int)]),
    "hbk_stream_create_cu_mask": (_c_int, [_vp, _c_int, ctypes.POINTER(_vp)]),
    "hbk_stream_destroy": (_c_int, [_vp]),
    "hbk_profile_mark": (_c_int, [ctypes.c_int32, _vp]),
    "hbk_mel_plan_create": (_c_int, [_vp, _vp, _c_int, _c_int, _c_int, _c_float, _c_float,
                                     _c_float, _c_float, ctypes.POINTER(_vp)]),
    "hbk_mel_plan_destroy": (_c_int, [_vp]),
    "hbk_mel_set_variant": (_c_int, [_vp, ctypes.c_int32]),
    "hbk_mel_frames": (_c_int, [_vp, _vp, _c_int64, _c_int64, _c_int64, _vp, _vp]),
    "hbk_embed_plan_create": (_c_int, [_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _vp,
                                       ctypes.c_int32, ctypes.POINTER(_vp)]),
    "hbk_embed_plan_create_ex": (_c_int, [_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _vp,
                                          ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(_vp)]),
    "hbk_embed_plan_destroy": (_c_int, [_vp]),
    "hbk_embed_plan_info": (_c_int, [_vp, ctypes.POINTER(ctypes.c_int32),
                                     ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                     ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_int32)]),
    "hbk_embed_workspace_size": (_c_int, [_vp, _c_int64, ctypes.POINTER(_c_int64)]),
    "hbk_embed_clips": (_c_int, [_vp, _vp, _c_int64, _c_int64, _vp, _vp, _c_int64, _vp]),
    "hbk_embed_split_info": (_c_int, [_vp, ctypes.c_int32, ctypes.POINTER(_c_int64)]),
    "hbk_embed_clips_front": (_c_int, [_vp, _vp, _c_int64, _c_int64, ctypes.c_int32, _vp, _vp, _c_int64, _vp]),
    "hbk_embed_clips_back": (_c_int, [_vp, _vp, _c_int64, ctypes.c_int32, _vp, _vp, _c_int64, _vp]),
    "hbk_embed_windows": (_c_int, [_vp, _vp, _c_int64, _vp, _vp, _c_int64, _vp]),
    "hbk_nan_rows_workspace_size": (_c_int64, [_c_int64]),
    "hbk_nan_rows_fix": (_c_int, [_vp, _c_int64, _c_int64, ctypes.c_uint64, _vp, _c_int64, _vp]),
    "hbk_embed_range_status": (_c_int, [_vp, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32, _vp]),
    "hbk_reverb_plan_create": (_c_int, [_c_int64, ctypes.POINTER(_vp)]),
    "hbk_reverb_plan_destroy": (_c_int, [_vp]),
    "hbk_reverb_spectrum": (_c_int, [_vp, _vp, _c_int64, _c_int64, _vp, _vp]),
    "hbk_augment": (_c_int, [_vp, _vp, _c_int64, _c_int64, _vp, _c_int64, _vp, _vp, _vp, _vp, _vp,
                             _vp, _c_int64, _vp]),
    "hbk_colored_noise": (_c_int, [_vp, _vp, _c_int64, _c_int64, _vp, _c_int64, ctypes.c_uint64, _c_int64, _vp,
                                   _vp, _c_float, _vp, _c_int64, _vp, _c_int64, _vp]),
    "hbk_augment_colored": (_c_int, [_vp, _vp, _c_int64, _c_int64, _vp, _c_int64, _vp, _vp, _vp, _vp, _vp,
                                     _vp, _c_int64, ctypes.c_uint64, _c_int64, _vp, _vp, _c_float, _vp, _c_int64,
                                     _vp, _c_int64, _vp, _c_int64, _vp]),
    "hbk_colored_noise_workspace_size": (_c_int64, [_c_int64, _c_int64]),
    "hbk_colored_noise_ws": (_c_int, [_vp, _vp, _c_int64, _c_int64, _vp, _c_int64, ctypes.c_uint64, _c_int64, _vp,
                                      _vp, _c_float, _vp, _c_int64, _vp, _c_int64, _vp, _c_int64, _vp]),
    "hbk_tanh_distortion": (_c_int, [_vp, _c_int64, _c_int64, _vp, _vp, _c_int64, _vp, _c_int64, _vp]),
    "hbk_band_stop_workspace_size": (_c_int64, [_c_int64, ctypes.c_int32, ctypes.c_int32, _vp]),
    "hbk_band_stop": (_c_int, [_vp, _vp, _c_int64, _c_int64, _vp, _vp, ctypes.c_int32, _vp, _vp, _vp, _vp,
                               ctypes.c_int32, _vp, _vp, _vp, _c_int64, _vp, _c_int64, _vp]),
    "hbk_pitch_shift_workspace_size": (_c_int64, [_c_int64, _c_int64, ctypes.c_int32, ctypes.c_int32,
                                                  ctypes.c_int32]),
    "hbk_pitch_shift": (_c_int, [_vp, _c_int64, _c_int64, _vp, _c_int64, ctypes.c_int32, ctypes.c_int32,
                                 ctypes.c_int32, _vp, _c_int64, _vp, _c_int64, _vp]),
    "hbk_seven_band_eq": (_c_int, [_vp, _c_int64, _c_int64, _vp, _vp, _c_int64, _vp, _c_int64, _vp]),
    "hbk_place_clips": (_c_int, [_vp, _c_int64, _c_int64, _vp, _vp, _vp, _c_int64, _c_int64, _vp]),
    "hbk_mlp_set_step_scalars": (_c_int, [_vp, _vp]),
    "hbk_mlp_plan_create": (_c_int, [ctypes.c_int32] * 4 + [ctypes.POINTER(_vp)]),
    "hbk_mlp_plan_destroy": (_c_int, [_vp]),
    "hbk_mlp_layout": (_c_int, [_vp, ctypes.POINTER(_c_int64), _vp, ctypes.c_int32]),
    "hbk_mlp_workspace_size": (_c_int, [_vp, _c_int64, ctypes.POINTER(_c_int64)]),
    "hbk_mlp_forward": (_c_int, [_vp, _vp, _vp, _c_int64, _vp, _vp, _c_float, ctypes.c_uint64,
                                 _vp, _c_int64, _vp]),
    "hbk_mlp_train_fwd_bwd": (_c_int, [_vp, _vp, _vp, _vp, _c_int64, _c_float, _c_float, _c_float,
                                       _c_float, ctypes.c_uint64, _vp, _vp, _vp, _c_int64, _vp]),
    "hbk_mlp_gate_adam": (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int32,
                                   _c_float, _c_float, _c_float, _c_float, _vp]),
    "hbk_mlp_fused_supported": (_c_int, [_vp, ctypes.POINTER(ctypes.c_int32)]),
    "hbk_mlp_step_fwd_bwd": (_c_int, [_vp, _vp, _vp, _c_int64, _vp, _c_int64, _vp, _c_int64, _vp, _c_int64,
                                      _c_int64, _vp, ctypes.c_int32, _vp, _c_int64, _c_float, _c_float,
                                      _c_float, _c_float, ctypes.c_uint64, _vp, _vp, _c_int64, ctypes.c_int32,
                                      _vp, _c_int64, _vp]),
    "hbk_mlp_step_update": (_c_int, [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int32, _vp, _c_int64, _c_float,
                                     _c_float, _c_float, _c_float, _vp, ctypes.c_int32, _vp, _c_int64, _vp]),
    "hbk_mlp_eval_workspace_size": (_c_int, [_vp, _c_int64, ctypes.POINTER(_c_int64)]),
    "hbk_mlp_eval_prepare": (_c_int, [_vp, _vp, _vp, _c_int64, _vp]),
    "hbk_mlp_eval_count_multi": (_c_int, [_vp, _vp, ctypes.c_int32, _vp, ctypes.c_int32, _vp, _vp, _vp, _vp, _vp,
                                          _vp, _c_float, _c_float, _vp, _c_int64, _vp]),
    "hbk_mlp_eval_count": (_c_int, [_vp, _vp, _vp, ctypes.c_int32, _c_int64, _vp, _c_int64, _c_int64,
                                    ctypes.c_int32, _c_float, _c_float, ctypes.c_uint64, _vp, _vp, _vp, _c_int64,
                                    _vp]),
    "hbk_mlp_eval_finish": (_c_int, [_vp, _vp, ctypes.POINTER(ctypes.c_double), _c_float, _c_float, _vp,
                                     _c_int64, _c_int64, _vp, _vp]),
}


class GraphOp(ctypes.Structure):
    """hbk_graph_op (include/hbk.h)."""
    _fields_ = [
        ("kind", ctypes.c_int32), ("kh", ctypes.c_int32), ("kw", ctypes.c_int32),
        ("cin", ctypes.c_int32), ("cout", ctypes.c_int32), ("act", ctypes.c_int32),
        ("alpha", ctypes.c_float), ("weight", _vp), ("bias", _vp),
    ]


def exported_symbols() -> list[str]:
    return list(_PROTOS)


def lib() -> ctypes.CDLL:
    """Load (once) and return libhbk.so with typed prototypes."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise HBKUnavailable(
                f"libhbk.so not found at {LIB_PATH}; build it with "
                "`python hey-buddy_amd/build.py` (the HIP path has no fallback)")
        try:
            handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise HBKUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in _PROTOS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
        return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().hbk_last_error().decode(errors="replace")
        raise HBKError(f"{what}: status {rc}: {msg}")


def require_device(device: Optional[torch.device | int] = None) -> torch.device:
    """Resolve the HIP device the hot path runs on; raise if there is none."""
    lib()
    if not torch.cuda.is_available():
        raise HBKUnavailable("no HIP device visible: the hey-buddy MI355X path needs a GPU")
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    if isinstance(device, int):
        return torch.device("cuda", device)
    device = torch.device(device)
    if device.type != "cuda":
        raise HBKUnavailable(f"device {device} is not a HIP device")
    return device if device.index is not None else torch.device("cuda", torch.cuda.current_device())


def stream_ptr(device: Optional[torch.device] = None) -> int:
    """Raw hipStream_t of torch's current stream on ``device``."""
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor) -> int:
    return t.data_ptr()
