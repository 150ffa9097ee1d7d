"""torch-facing wrappers over the libhbk.so C ABI (include/hbk.h).

Each wrapper validates shapes on the host (the kernels assume them), passes
raw device pointers and torch's current stream, and is registered as a
``torch.library`` custom op under the ``hbk`` namespace
(``torch.ops.hbk.mel_frames`` ...), so callers can treat it like any other
torch op. Nothing here computes on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import itertools
import threading
from typing import Dict

import numpy as np
import torch

from heybuddy import _native
from heybuddy._native import check, lib, ptr, stream_ptr

__all__ = ["MelPlan", "mel_frames"]

_plans: Dict[int, object] = {}
_plan_ids = itertools.count(1)
_plans_lock = threading.Lock()


def _register(plan) -> int:
    """Plans are handed to the torch.library ops by id (ops take no opaque objects)."""
    with _plans_lock:
        pid = next(_plan_ids)
        _plans[pid] = plan
    return pid


def _u64_to_i64(v: int) -> int:
    v &= 2 ** 64 - 1
    return v - 2 ** 64 if v >= 2 ** 63 else v


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
        self.id = _register(self)

    def n_frames(self, n_samples: int) -> int:
        return 0 if n_samples < self.n_fft else (n_samples - self.n_fft) // self.hop + 1

    def set_variant(self, variant: int) -> "MelPlan":
        """The filterbank stage (hbk_mel_set_variant): 0 = sparse per-lane dot
        products on the VALU (default), 1 = the dense split-f16 MFMA product."""
        check(lib().hbk_mel_set_variant(self._handle, int(variant)), "hbk_mel_set_variant")
        return self

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


EMBED_PRECISIONS = {"split": 0, "exact": 1}  # hbk_precision


def default_embed_precision() -> str:
    """HEYBUDDY_EMBED_PRECISION: 'split' (fp16 hi/lo pairs on the f16 MFMA,
    ~2^-21 relative; default) or 'exact' (f32 MFMA, bitwise fmaf chain)."""
    p = os.environ.get("HEYBUDDY_EMBED_PRECISION", "split")
    if p not in EMBED_PRECISIONS:
        raise ValueError(f"HEYBUDDY_EMBED_PRECISION must be one of {sorted(EMBED_PRECISIONS)}")
    return p


class EmbedPlan:
    """Device plan of the speech-embedding graph (hbk_embed_plan_create_ex).

    ``graph`` is a heybuddy.embedding_graph.Graph; ``starts`` are the window
    start frames of the clip path (the reference's 16 windows by default);
    ``precision`` is 'split' or 'exact' (see include/hbk.h, hbk_precision).
    """

    def __init__(self, graph, starts=None, device: torch.device | int | None = None,
                 precision: str | None = None) -> None:
        from heybuddy.embedding_graph import WINDOW_STARTS, Conv
        self.device = _native.require_device(device)
        self.precision = default_embed_precision() if precision is None else precision
        if self.precision not in EMBED_PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(EMBED_PRECISIONS)}")
        self.graph = graph
        self.starts = tuple(WINDOW_STARTS if starts is None else starts)
        ops = (_native.GraphOp * len(graph.ops))()
        self._keep = []  # host arrays referenced by ops during create
        for i, op in enumerate(graph.ops):
            if isinstance(op, Conv):
                w = np.ascontiguousarray(op.weight, dtype=np.float32)
                b = np.ascontiguousarray(op.bias, dtype=np.float32)
                self._keep += [w, b]
                ops[i] = _native.GraphOp(0, op.kh, op.kw, op.cin, op.cout,
                                         1 if op.act == "leaky_relu" else 0, float(op.alpha),
                                         w.ctypes.data, b.ctypes.data)
            else:
                ops[i] = _native.GraphOp(1, op.ph, op.pw, 0, 0, 0, 0.0, None, None)
        st = (ctypes.c_int32 * len(self.starts))(*self.starts)
        h, w, _ = graph.in_shape
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().hbk_embed_plan_create_ex(ops, len(graph.ops), h, w, st, len(self.starts),
                                                 EMBED_PRECISIONS[self.precision], ctypes.byref(handle)),
                  "hbk_embed_plan_create_ex")
        self._handle = handle
        self._keep = []
        od, npre, nch, sf = (ctypes.c_int32() for _ in range(4))
        pm, tm = ctypes.c_double(), ctypes.c_double()
        check(lib().hbk_embed_plan_info(handle, ctypes.byref(od), ctypes.byref(npre),
                                        ctypes.byref(nch), ctypes.byref(pm), ctypes.byref(tm),
                                        ctypes.byref(sf)), "hbk_embed_plan_info")
        self.out_dim = od.value
        self.n_prefix_ops = npre.value
        self.n_chains = nch.value
        self.prefix_macs_per_clip = pm.value
        self.tail_macs_per_window = tm.value
        self.seq_frames = sf.value
        self.in_h, self.in_w = h, w
        self._ws: torch.Tensor | None = None
        self.id = _register(self)

    def range_tripped(self, reset: bool = True) -> bool:
        """Range guard of a 'split' plan (hbk_embed_range_status): True if a
        kernel of this plan split an activation with |x| >= 65504 since the
        last reset, i.e. outputs since then are not f32-accurate. Waits for the
        current stream. An 'exact' plan never trips."""
        t = ctypes.c_int32()
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
            check(lib().hbk_embed_range_status(self._handle, ctypes.byref(t), int(reset), ctypes.c_void_p(stream)),
                  "hbk_embed_range_status")
        return bool(t.value)

    @property
    def macs_per_clip(self) -> float:
        """Algorithmic MACs of the clip path (shared prefix + per-window tail)."""
        return self.prefix_macs_per_clip + len(self.starts) * self.tail_macs_per_window

    def workspace(self, n: int, slot: int = 0) -> torch.Tensor:
        """The plan's workspace for n clips; slot 1 is a second one, for the
        back half of a split call running beside a front half (clips_back)."""
        need = ctypes.c_int64()
        check(lib().hbk_embed_workspace_size(self._handle, int(n), ctypes.byref(need)),
              "hbk_embed_workspace_size")
        attr = "_ws" if slot == 0 else "_ws_back"
        ws = getattr(self, attr, None)
        if ws is None or ws.numel() < need.value:
            ws = torch.empty(need.value, dtype=torch.uint8, device=self.device)
            setattr(self, attr, ws)
        return ws

    def mid_floats(self, n_front: int) -> int:
        """Floats per clip of the front half's output (hbk_embed_split_info)."""
        v = ctypes.c_int64()
        check(lib().hbk_embed_split_info(self._handle, int(n_front), ctypes.byref(v)), "hbk_embed_split_info")
        return v.value

    def clips_front(self, mel: torch.Tensor, n_front: int, mid: torch.Tensor) -> torch.Tensor:
        """The first n_front fused chains of the clip path (hbk_embed_clips_front)
        on the current stream: mel [B, F, n_mels] -> mid [B, mid_floats(n_front)]."""
        n = mel.shape[0]
        if not (mel.is_cuda and mel.dtype == torch.float32 and mel.stride(-1) == 1 and mid.is_contiguous()
                and mid.dtype == torch.float32 and mid.numel() >= n * self.mid_floats(n_front)):
            raise ValueError("clips_front: bad mel / mid tensors")
        ws = self.workspace(n)
        check(lib().hbk_embed_clips_front(self._handle, ptr(mel), n, mel.stride(0), int(n_front), ptr(mid), ptr(ws),
                                          ws.numel(), stream_ptr(mel.device)), "hbk_embed_clips_front")
        return mid

    def clips_back(self, mid: torch.Tensor, n: int, n_front: int, out: torch.Tensor) -> torch.Tensor:
        """The remaining chains (hbk_embed_clips_back) on the current stream, with
        the plan's second workspace: mid -> out [n, n_windows, out_dim]."""
        if not (mid.is_cuda and mid.is_contiguous() and out.is_contiguous() and out.dtype == torch.float32
                and out.shape == (n, len(self.starts), self.out_dim)):
            raise ValueError("clips_back: bad mid / out tensors")
        ws = self.workspace(n, slot=1)
        check(lib().hbk_embed_clips_back(self._handle, ptr(mid), n, int(n_front), ptr(out), ptr(ws), ws.numel(),
                                         stream_ptr(mid.device)), "hbk_embed_clips_back")
        return out

    def clips(self, mel: torch.Tensor) -> torch.Tensor:
        return embed_clips(mel, self)

    def windows(self, windows: torch.Tensor) -> torch.Tensor:
        return embed_windows(windows, self)

    def __del__(self) -> None:
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            try:
                lib().hbk_embed_plan_destroy(h)
            except Exception:
                pass
            self._handle = None


@torch.library.custom_op("hbk::embed_clips", mutates_args=())
def _embed_clips_op(mel: torch.Tensor, plan_id: int) -> torch.Tensor:
    plan = _plans[plan_id]
    n = mel.shape[0]
    out = torch.empty((n, len(plan.starts), plan.out_dim), dtype=torch.float32, device=mel.device)
    ws = plan.workspace(n)
    check(lib().hbk_embed_clips(plan._handle, ptr(mel), n, mel.stride(0), ptr(out), ptr(ws),
                                ws.numel(), stream_ptr(mel.device)), "hbk_embed_clips")
    return out


@_embed_clips_op.register_fake
def _(mel, plan_id):
    plan = _plans[plan_id]
    return mel.new_empty((mel.shape[0], len(plan.starts), plan.out_dim))


@torch.library.custom_op("hbk::embed_windows", mutates_args=())
def _embed_windows_op(windows: torch.Tensor, plan_id: int) -> torch.Tensor:
    plan = _plans[plan_id]
    n = windows.shape[0]
    out = torch.empty((n, plan.out_dim), dtype=torch.float32, device=windows.device)
    ws = plan.workspace(n)
    check(lib().hbk_embed_windows(plan._handle, ptr(windows), n, ptr(out), ptr(ws), ws.numel(),
                                  stream_ptr(windows.device)), "hbk_embed_windows")
    return out


@_embed_windows_op.register_fake
def _(windows, plan_id):
    plan = _plans[plan_id]
    return windows.new_empty((windows.shape[0], plan.out_dim))


@torch.library.custom_op("hbk::embed_clips_out", mutates_args=("out",))
def _embed_clips_out_op(mel: torch.Tensor, plan_id: int, out: torch.Tensor) -> None:
    plan = _plans[plan_id]
    n = mel.shape[0]
    ws = plan.workspace(n)
    check(lib().hbk_embed_clips(plan._handle, ptr(mel), n, mel.stride(0), ptr(out), ptr(ws),
                                ws.numel(), stream_ptr(mel.device)), "hbk_embed_clips")


def embed_clips(mel: torch.Tensor, plan: EmbedPlan, out: torch.Tensor | None = None) -> torch.Tensor:
    """Unique mel frames [B, F >= seq_frames, n_mels] -> embeddings
    [B, n_windows, out_dim] in the reference's slot order (into ``out`` if
    given: a contiguous f32 tensor of that shape on the device)."""
    if mel.dim() != 3 or mel.dtype != torch.float32 or mel.device != plan.device:
        raise ValueError(f"mel must be [B, F, {plan.in_w}] float32 on {plan.device}")
    if mel.shape[2] != plan.in_w or mel.shape[1] < plan.seq_frames:
        raise ValueError(f"mel {tuple(mel.shape)}: need >= {plan.seq_frames} frames of {plan.in_w}")
    if mel.stride(2) != 1 or mel.stride(1) != plan.in_w:
        mel = mel.contiguous()
    if out is not None:
        if (tuple(out.shape) != (mel.shape[0], len(plan.starts), plan.out_dim) or out.dtype != torch.float32
                or out.device != mel.device or not out.is_contiguous()):
            raise ValueError("out must be a contiguous f32 [B, n_windows, out_dim] tensor on the device")
        torch.ops.hbk.embed_clips_out(mel, plan.id, out)
        return out
    return torch.ops.hbk.embed_clips(mel, plan.id)


def embed_windows(windows: torch.Tensor, plan: EmbedPlan) -> torch.Tensor:
    """Reference per-window API: [n, in_h, in_w] (or [n, in_h, in_w, 1]) -> [n, out_dim]."""
    if windows.dim() == 4 and windows.shape[3] == 1:
        windows = windows[..., 0]
    if (windows.dim() != 3 or tuple(windows.shape[1:]) != (plan.in_h, plan.in_w)
            or windows.dtype != torch.float32 or windows.device != plan.device):
        raise ValueError(f"windows must be [n, {plan.in_h}, {plan.in_w}] float32 on {plan.device}")
    return torch.ops.hbk.embed_windows(windows.contiguous(), plan.id)


class MlpPlan:
    """The gated-MLP classifier on the HIP path (hbk_mlp_*): flat parameter
    layout, forward, and the two halves of a train step."""

    N_STATS = 8

    def __init__(self, d_in: int = 1536, layer_dim: int = 96, hidden: int = 64, n_layers: int = 2) -> None:
        handle = ctypes.c_void_p()
        check(lib().hbk_mlp_plan_create(d_in, layer_dim, hidden, n_layers, ctypes.byref(handle)),
              "hbk_mlp_plan_create")
        self._handle = handle
        self.d_in, self.layer_dim, self.hidden, self.n_layers = d_in, layer_dim, hidden, n_layers
        n = ctypes.c_int64()
        n_off = 2 + 4 * (n_layers + 2) + 2 * (n_layers + 1)
        offs = (ctypes.c_int64 * n_off)()
        check(lib().hbk_mlp_layout(handle, ctypes.byref(n), offs, n_off), "hbk_mlp_layout")
        self.n_params = n.value
        self.offsets = list(offs)
        self._ws: Dict[torch.device, torch.Tensor] = {}
        self.id = _register(self)

    def views(self, flat: torch.Tensor) -> "Dict[str, torch.Tensor]":
        """state_dict-named views (reference names and shapes) into ``flat``."""
        from collections import OrderedDict
        H, L, D = self.hidden, self.layer_dim, self.d_in
        o = self.offsets
        out = OrderedDict()

        def v(off, *shape):
            n = int(np.prod(shape))
            return flat[off:off + n].view(*shape)

        out["norm_in.weight"] = v(o[0], D)
        out["norm_in.bias"] = v(o[1], D)
        gm = o[2:2 + 4 * (self.n_layers + 2)]
        ln = o[2 + 4 * (self.n_layers + 2):]

        def gmlp(prefix, k, din, dout):
            w_hg, b_hg, w_o, b_o = gm[4 * k:4 * k + 4]
            out[f"{prefix}.hidden.weight"] = v(w_hg, H, din)
            out[f"{prefix}.hidden.bias"] = v(b_hg, H)
            out[f"{prefix}.output.weight"] = v(w_o, dout, H)
            out[f"{prefix}.output.bias"] = v(b_o, dout)
            out[f"{prefix}.gate.weight"] = v(w_hg + H * din, H, din)
            out[f"{prefix}.gate.bias"] = v(b_hg + H, H)

        gmlp("mlp_in", 0, D, L)
        for l in range(self.n_layers):
            out[f"layers.{l}.0.weight"] = v(ln[2 * l], L)
            out[f"layers.{l}.0.bias"] = v(ln[2 * l + 1], L)
            gmlp(f"layers.{l}.1", l + 1, L, L)
        out["norm_out.weight"] = v(ln[2 * self.n_layers], L)
        out["norm_out.bias"] = v(ln[2 * self.n_layers + 1], L)
        gmlp("mlp_out", self.n_layers + 1, L, 1)
        return out

    def set_step_scalars(self, scalars: torch.Tensor | None) -> None:
        """Device float64 [lr, neg_weight, seed] that train launches read instead of
        their arguments (hbk_mlp_set_step_scalars; None = off). The pointer is
        taken at launch time, so a graph captured while it is set keeps it."""
        if scalars is not None and (scalars.dtype != torch.float64 or scalars.numel() < 3
                                    or scalars.device.type != "cuda"):
            raise ValueError("step scalars must be a float64 [3] device tensor")
        check(lib().hbk_mlp_set_step_scalars(self._handle, ptr(scalars) if scalars is not None else None),
              "hbk_mlp_set_step_scalars")

    def workspace_bytes(self, batch: int) -> int:
        need = ctypes.c_int64()
        check(lib().hbk_mlp_workspace_size(self._handle, int(batch), ctypes.byref(need)),
              "hbk_mlp_workspace_size")
        return need.value

    def workspace(self, batch: int, device: torch.device) -> torch.Tensor:
        """Shared eager workspace (grown on demand). Captured graphs own their
        workspace instead: a growth here frees the old buffer."""
        need = ctypes.c_int64()
        check(lib().hbk_mlp_workspace_size(self._handle, int(batch), ctypes.byref(need)),
              "hbk_mlp_workspace_size")
        ws = self._ws.get(device)
        if ws is None or ws.numel() < need.value:
            ws = torch.empty(need.value, dtype=torch.uint8, device=device)
            self._ws[device] = ws
        return ws

    def _check(self, params: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        if params.numel() != self.n_params or params.dtype != torch.float32 or not params.is_contiguous():
            raise ValueError("params must be the contiguous flat f32 buffer")
        x = x.reshape(x.shape[0], -1)
        if x.shape[1] != self.d_in or x.dtype != torch.float32 or x.device != params.device:
            raise ValueError(f"x must be [B, {self.d_in}] f32 on {params.device}")
        return x.contiguous()

    def forward(self, params: torch.Tensor, x: torch.Tensor, dropout_p: float = 0.0, seed: int = 0,
                logits: bool = False):
        x = self._check(params, x)
        ws = self.workspace(x.shape[0], x.device)
        prob, logit = torch.ops.hbk.mlp_forward(params, x, ws, float(dropout_p), _u64_to_i64(seed), self.id)
        return (prob, logit) if logits else prob

    def train_fwd_bwd(self, params: torch.Tensor, x: torch.Tensor, y: torch.Tensor, bucket: torch.Tensor,
                      neg_weight: float, threshold: float = 1e-4, activation_threshold: float = 0.5,
                      dropout_p: float = 0.0, seed: int = 0, prob: torch.Tensor | None = None,
                      workspace: torch.Tensor | None = None) -> None:
        x = self._check(params, x)
        b = x.shape[0]
        y = y.to(device=x.device, dtype=torch.float32).contiguous()
        if y.numel() != b or bucket.numel() != self.n_params + self.N_STATS:
            raise ValueError("bad y / bucket size")
        ws = self.workspace(b, x.device) if workspace is None else workspace
        check(lib().hbk_mlp_train_fwd_bwd(self._handle, ptr(params), ptr(x), ptr(y), b, float(neg_weight),
                                          float(threshold), float(activation_threshold), float(dropout_p),
                                          int(seed) & (2 ** 64 - 1), ptr(bucket),
                                          ptr(prob) if prob is not None else None, ptr(ws), ws.numel(),
                                          stream_ptr(x.device)), "hbk_mlp_train_fwd_bwd")

    # -- fused train step (hbk_mlp_step_*) -------------------------------
    @property
    def fused(self) -> bool:
        """True when hbk_mlp_step_* cover this architecture (the default one)."""
        if not hasattr(self, "_fused"):
            ok = ctypes.c_int32()
            check(lib().hbk_mlp_fused_supported(self._handle, ctypes.byref(ok)), "hbk_mlp_fused_supported")
            self._fused = bool(ok.value)
        return self._fused

    @staticmethod
    def new_state(device, adam_t: float = 0.0, salt: int = 0) -> torch.Tensor:
        """Device step state, both halves [0, 1, adam_t, 0, salt, 0, 0, 0]."""
        half = [0.0, 1.0, float(adam_t), 0.0, float(salt % (1 << 24)), 0.0, 0.0, 0.0]
        return torch.tensor(half * 2, dtype=torch.float32, device=device)

    def step_fwd_bwd(self, params: torch.Tensor, bucket: torch.Tensor, state: torch.Tensor, parity: int,
                     y: torch.Tensor, batch: int, pool32: torch.Tensor | None = None,
                     pool16: torch.Tensor | None = None, idx: torch.Tensor | None = None,
                     idx_stride: int = 0, y_stride: int = 0, sched: torch.Tensor | None = None,
                     neg_weight: float = 1.0, threshold: float = 1e-4, activation_threshold: float = 0.5,
                     dropout_p: float = 0.0, seed: int = 0, prob: torch.Tensor | None = None,
                     workspace: torch.Tensor | None = None, xhat_ready: bool = False,
                     prefetch_next: bool = False, idx_steps: int | None = None,
                     weights_ready: bool = False, defer_partials: bool = False) -> None:
        """Forward / filter / BCE / backward of one step into ``bucket``
        (hbk_mlp_step_fwd_bwd). Rows come from pool32 [n, 1536] f32 and pool16
        [n, 1536] f16 by ``idx`` (int32, >= 0 -> pool32, < 0 -> pool16 row -i-1;
        None -> pool32 rows 0..batch-1); y: 0/1 float32 labels on the device.
        ``prefetch_next``: also gather + normalise step + 1's rows (idx row
        step + 1 < idx_steps, default idx.numel() // idx_stride) during this
        step; ``xhat_ready``: the previous call on this workspace did that for
        this step; ``weights_ready``: the previous step_update got this
        workspace, so its weight cache is current (else it is refreshed);
        ``defer_partials``: the weight gradients' per-split slabs stay in the
        workspace for the next step_update, which must get it (one process, no
        all-reduce in between); else they are summed into ``bucket`` here."""
        dev = params.device
        if params.numel() != self.n_params or bucket.numel() != self.n_params + self.N_STATS:
            raise ValueError("params / bucket do not match the plan")
        for t, dt, name in ((pool32, torch.float32, "pool32"), (pool16, torch.float16, "pool16")):
            if t is not None and (t.dtype != dt or t.device != dev or not t.is_contiguous()
                                  or t.reshape(t.shape[0], -1).shape[1] != self.d_in):
                raise ValueError(f"{name} must be a contiguous [n, {self.d_in}] {dt} tensor on {dev}")
        if idx is not None and (idx.dtype != torch.int32 or idx.device != dev or not idx.is_contiguous()):
            raise ValueError("idx must be a contiguous int32 device tensor")
        if idx is None and (pool32 is None or pool32.shape[0] < batch):
            raise ValueError("without idx, pool32 must hold the batch rows")
        if y.dtype != torch.float32 or y.device != dev or not y.is_contiguous():
            raise ValueError("y must be contiguous float32 labels on the device")
        if state.numel() != 16 or state.dtype != torch.float32 or state.device != dev:
            raise ValueError("state must be the float32 [16] device state (MlpPlan.new_state)")
        if sched is not None and (sched.dtype != torch.float32 or sched.shape[-1] != 2 or sched.device != dev):
            raise ValueError("sched must be float32 [n, 2] (lr, neg_weight) on the device")
        ws = self.workspace(batch, dev) if workspace is None else workspace
        if idx_steps is None:
            idx_steps = idx.numel() // idx_stride if idx is not None and idx_stride > 0 else 1
        flags = (1 if xhat_ready else 0) | (2 if prefetch_next and idx is not None else 0) | (
            4 if weights_ready else 0) | (8 if defer_partials else 0)
        torch.ops.hbk.mlp_step_fwd_bwd(params, bucket, state, int(parity), y, int(batch), pool32, pool16, idx,
                                       int(idx_stride), int(y_stride), sched, float(neg_weight), float(threshold),
                                       float(activation_threshold), float(dropout_p), _u64_to_i64(seed), prob, ws,
                                       int(idx_steps), int(flags), self.id)

    def step_update(self, params: torch.Tensor, bucket: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                    state: torch.Tensor, parity: int, sched: torch.Tensor | None = None, lr: float = 1e-3,
                    beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8,
                    history: torch.Tensor | None = None, workspace: torch.Tensor | None = None) -> None:
        """Gate + Adam + bucket zeroing (hbk_mlp_step_update); with the step's
        ``workspace`` it also keeps the weight cache there current, so the next
        step_fwd_bwd on it may pass weights_ready."""
        torch.ops.hbk.mlp_step_update(params, bucket, m, v, state, int(parity), sched, float(lr), float(beta1),
                                      float(beta2), float(eps), history, workspace, self.id)

    # -- evaluation passes (hbk_mlp_eval_*) ---------------------------------
    def eval_workspace_bytes(self, rows: int) -> int:
        need = ctypes.c_int64()
        check(lib().hbk_mlp_eval_workspace_size(self._handle, int(rows), ctypes.byref(need)),
              "hbk_mlp_eval_workspace_size")
        return need.value

    def eval_prepare(self, params: torch.Tensor, ws: torch.Tensor) -> None:
        """The pass's weight planes from ``params`` (hbk_mlp_eval_prepare): once per
        pass, before any eval_count."""
        torch.ops.hbk.mlp_eval_prepare_(params, ws, self.id)

    def eval_count(self, params: torch.Tensor, pool: torch.Tensor, rows: int, label: int, counts: torch.Tensor,
                   ws: torch.Tensor, idx: torch.Tensor | None = None, row_offset: int = 0,
                   activation_threshold: float = 0.5, dropout_p: float = 0.0, seed: int = 0,
                   prob: torch.Tensor | None = None) -> None:
        """Forward ``rows`` rows of ONE pool ([n, 1536] f32 or f16; row r = pool
        row idx[r], or (row_offset + r) % n without idx), all labelled ``label``,
        into ``counts`` [4] f32 (hbk_mlp_eval_count): counts[2 label] +=
        #(p >= threshold), counts[2 label + 1] += #(p > threshold)."""
        dev = params.device
        flat = pool.reshape(pool.shape[0], -1)
        if flat.shape[1] != self.d_in or pool.dtype not in (torch.float32, torch.float16) or pool.device != dev \
                or not pool.is_contiguous():
            raise ValueError(f"pool must be a contiguous [n, {self.d_in}] f32 / f16 tensor on {dev}")
        if idx is not None and (idx.dtype != torch.int32 or idx.device != dev or not idx.is_contiguous()
                                or idx.numel() < rows):
            raise ValueError("idx must be a contiguous int32 device tensor of >= rows entries")
        if counts.dtype != torch.float32 or counts.numel() < 4 or counts.device != dev:
            raise ValueError("counts must be a float32 [4] device tensor")
        if prob is not None and (prob.dtype != torch.float32 or prob.numel() < rows or prob.device != dev):
            raise ValueError("prob must be a float32 device tensor of >= rows entries")
        torch.ops.hbk.mlp_eval_count_(params, pool, idx, int(rows), int(row_offset), int(label),
                                      float(activation_threshold), float(dropout_p), _u64_to_i64(seed), counts, prob,
                                      ws, self.id)

    def eval_count_multi(self, params: torch.Tensor, parts, counts: torch.Tensor, ws: torch.Tensor,
                         activation_threshold: float = 0.5, dropout_p: float = 0.0) -> None:
        """eval_count for up to 4 pools of one dtype in ONE launch (hbk_mlp_eval_count_multi):
        ``parts`` = [(pool, rows, row_offset, label, which, seed)], pool i counted into
        counts[which] ([2, 4] f32), each exactly as its own eval_count (no idx, no prob)."""
        dev = params.device
        if not 0 < len(parts) <= 4:
            raise ValueError("1 to 4 pools per launch")
        dt = parts[0][0].dtype
        for pool, rows, _, label, which, _ in parts:
            if pool.dtype != dt or pool.dtype not in (torch.float32, torch.float16) or pool.device != dev \
                    or not pool.is_contiguous() or pool.reshape(pool.shape[0], -1).shape[1] != self.d_in:
                raise ValueError(f"pools must be contiguous [n, {self.d_in}] tensors of one dtype on {dev}")
            if label not in (0, 1) or which not in (0, 1) or rows < 0:
                raise ValueError("label / which must be 0 or 1, rows >= 0")
        if counts.dtype != torch.float32 or counts.shape != (2, 4) or counts.device != dev \
                or not counts.is_contiguous():
            raise ValueError("counts must be a contiguous float32 [2, 4] device tensor")
        torch.ops.hbk.mlp_eval_count_multi_(
            params, [q[0] for q in parts], [int(q[1]) for q in parts], [int(q[2]) for q in parts],
            [int(q[3]) for q in parts], [int(q[4]) for q in parts], [_u64_to_i64(q[5]) for q in parts],
            float(activation_threshold), float(dropout_p), counts, ws, self.id)

    @staticmethod
    def eval_finish(counts_val: torch.Tensor | None, counts_test: torch.Tensor | None, sizes, out: torch.Tensor,
                    target: float = 1.5, ratio: float = 0.0, sched: torch.Tensor | None = None,
                    next_step: int = 0) -> None:
        """The reference's bookkeeping after the passes (hbk_mlp_eval_finish):
        out [8] = (validation false positives / hour, validation recall, testing
        false-positive rate, testing recall, testing accuracy, new negative weight,
        weight before, 0); ratio > 0 writes the new negative weight into sched
        rows next_step .. (the dynamic negative weight, trainer.py:531-536)."""
        torch.ops.hbk.mlp_eval_finish_(counts_val, counts_test, [float(v) for v in sizes], float(target),
                                       float(ratio), sched, int(next_step), out)

    def gate_adam(self, params, bucket, m, v, state, ctrl, history, lr, beta1=0.9, beta2=0.999,
                  eps=1e-8) -> None:
        cap = 0 if history is None else history.shape[0]
        check(lib().hbk_mlp_gate_adam(self._handle, ptr(params), ptr(bucket), ptr(m), ptr(v), ptr(state),
                                      ptr(ctrl), ptr(history) if history is not None else None, cap,
                                      float(lr), float(beta1), float(beta2), float(eps),
                                      stream_ptr(params.device)), "hbk_mlp_gate_adam")


@torch.library.custom_op("hbk::mlp_forward", mutates_args=("ws",))
def _mlp_forward_op(params: torch.Tensor, x: torch.Tensor, ws: torch.Tensor, dropout_p: float, seed: int,
                    plan_id: int) -> tuple[torch.Tensor, torch.Tensor]:
    plan = _plans[plan_id]
    b = x.shape[0]
    prob = torch.empty(b, dtype=torch.float32, device=x.device)
    logit = torch.empty(b, dtype=torch.float32, device=x.device)
    check(lib().hbk_mlp_forward(plan._handle, ptr(params), ptr(x), b, ptr(prob), ptr(logit), float(dropout_p),
                                int(seed) & (2 ** 64 - 1), ptr(ws), ws.numel(), stream_ptr(x.device)),
          "hbk_mlp_forward")
    return prob, logit


@_mlp_forward_op.register_fake
def _(params, x, ws, dropout_p, seed, plan_id):
    return x.new_empty(x.shape[0]), x.new_empty(x.shape[0])


@torch.library.custom_op("hbk::mlp_step_fwd_bwd", mutates_args=("bucket", "prob", "ws"))
def _mlp_step_fwd_bwd_op(params: torch.Tensor, bucket: torch.Tensor, state: torch.Tensor, parity: int,
                         y: torch.Tensor, batch: int, pool32: torch.Tensor | None, pool16: torch.Tensor | None,
                         idx: torch.Tensor | None, idx_stride: int, y_stride: int, sched: torch.Tensor | None,
                         neg_weight: float, threshold: float, activation_threshold: float, dropout_p: float,
                         seed: int, prob: torch.Tensor | None, ws: torch.Tensor, idx_steps: int, flags: int,
                         plan_id: int) -> None:
    plan = _plans[plan_id]
    opt = lambda t: ptr(t) if t is not None else None  # noqa: E731
    check(lib().hbk_mlp_step_fwd_bwd(
        plan._handle, ptr(params), opt(pool32), pool32.shape[0] if pool32 is not None else 0, opt(pool16),
        pool16.shape[0] if pool16 is not None else 0, opt(idx), idx_stride, ptr(y), y_stride, batch, ptr(state),
        parity, opt(sched), sched.shape[0] if sched is not None else 0, neg_weight, threshold,
        activation_threshold, dropout_p, seed & (2 ** 64 - 1), ptr(bucket), opt(prob), idx_steps, flags, ptr(ws),
        ws.numel(), stream_ptr(params.device)), "hbk_mlp_step_fwd_bwd")


@torch.library.custom_op("hbk::mlp_step_update",
                         mutates_args=("params", "bucket", "m", "v", "state", "history", "ws"))
def _mlp_step_update_op(params: torch.Tensor, bucket: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                        state: torch.Tensor, parity: int, sched: torch.Tensor | None, lr: float, beta1: float,
                        beta2: float, eps: float, history: torch.Tensor | None, ws: torch.Tensor | None,
                        plan_id: int) -> None:
    plan = _plans[plan_id]
    cap = 0 if history is None else history.shape[0]
    check(lib().hbk_mlp_step_update(
        plan._handle, ptr(params), ptr(bucket), ptr(m), ptr(v), ptr(state), parity,
        ptr(sched) if sched is not None else None, sched.shape[0] if sched is not None else 0, lr, beta1, beta2,
        eps, ptr(history) if history is not None else None, cap, ptr(ws) if ws is not None else None,
        ws.numel() if ws is not None else 0, stream_ptr(params.device)), "hbk_mlp_step_update")


@torch.library.custom_op("hbk::mlp_eval_prepare_", mutates_args=("ws",))
def _mlp_eval_prepare_op(params: torch.Tensor, ws: torch.Tensor, plan_id: int) -> None:
    plan = _plans[plan_id]
    check(lib().hbk_mlp_eval_prepare(plan._handle, ptr(params), ptr(ws), ws.numel(), stream_ptr(params.device)),
          "hbk_mlp_eval_prepare")


@torch.library.custom_op("hbk::mlp_eval_count_", mutates_args=("counts", "prob", "ws"))
def _mlp_eval_count_op(params: torch.Tensor, pool: torch.Tensor, idx: torch.Tensor | None, rows: int,
                       row_offset: int, label: int, activation_threshold: float, dropout_p: float, seed: int,
                       counts: torch.Tensor, prob: torch.Tensor | None, ws: torch.Tensor, plan_id: int) -> None:
    plan = _plans[plan_id]
    check(lib().hbk_mlp_eval_count(
        plan._handle, ptr(params), ptr(pool), 1 if pool.dtype == torch.float16 else 0, pool.shape[0],
        ptr(idx) if idx is not None else None, rows, row_offset, label, activation_threshold, dropout_p,
        seed & (2 ** 64 - 1), ptr(counts), ptr(prob) if prob is not None else None, ptr(ws), ws.numel(),
        stream_ptr(params.device)), "hbk_mlp_eval_count")


@torch.library.custom_op("hbk::mlp_eval_count_multi_", mutates_args=("counts", "ws"))
def _mlp_eval_count_multi_op(params: torch.Tensor, pools: list[torch.Tensor], rows: list[int],
                             row_offsets: list[int], labels: list[int], which: list[int], seeds: list[int],
                             activation_threshold: float, dropout_p: float, counts: torch.Tensor, ws: torch.Tensor,
                             plan_id: int) -> None:
    plan = _plans[plan_id]
    n = len(pools)
    arr = lambda ct, vals: (ct * n)(*vals)  # noqa: E731
    check(lib().hbk_mlp_eval_count_multi(
        plan._handle, ptr(params), n, arr(ctypes.c_void_p, [ptr(q) for q in pools]),
        1 if pools[0].dtype == torch.float16 else 0, arr(ctypes.c_int64, [q.shape[0] for q in pools]),
        arr(ctypes.c_int64, rows), arr(ctypes.c_int64, row_offsets), arr(ctypes.c_int32, labels),
        arr(ctypes.c_uint64, [v & (2 ** 64 - 1) for v in seeds]),
        arr(ctypes.c_void_p, [counts.data_ptr() + 16 * w for w in which]), activation_threshold, dropout_p,
        ptr(ws), ws.numel(), stream_ptr(params.device)), "hbk_mlp_eval_count_multi")


@torch.library.custom_op("hbk::mlp_eval_finish_", mutates_args=("sched", "out"))
def _mlp_eval_finish_op(counts_val: torch.Tensor | None, counts_test: torch.Tensor | None, sizes: list[float],
                        target: float, ratio: float, sched: torch.Tensor | None, next_step: int,
                        out: torch.Tensor) -> None:
    sz = (ctypes.c_double * 4)(*sizes[:4])
    check(lib().hbk_mlp_eval_finish(
        ptr(counts_val) if counts_val is not None else None, ptr(counts_test) if counts_test is not None else None,
        sz, target, ratio, ptr(sched) if sched is not None else None, sched.shape[0] if sched is not None else 0,
        next_step, ptr(out), stream_ptr(out.device)), "hbk_mlp_eval_finish")


@torch.library.custom_op("hbk::nan_rows_fix_", mutates_args=("rows", "ws"))
def _nan_rows_fix_op(rows: torch.Tensor, seed: int, ws: torch.Tensor) -> None:
    n = rows.shape[0]
    check(lib().hbk_nan_rows_fix(ptr(rows), n, rows.numel() // max(n, 1), seed & (2 ** 64 - 1), ptr(ws), ws.numel(),
                                 stream_ptr(rows.device)), "hbk_nan_rows_fix")


def nan_rows_fix(rows: torch.Tensor, seed: int = 0, ws: torch.Tensor | None = None) -> torch.Tensor:
    """In place (hbk_nan_rows_fix): every row of rows [n, ...] (f32, contiguous, a multiple of
    4 elements per row) holding a NaN takes a uniformly drawn NaN-free row (a hash of (seed,
    row)), or zeros when every row holds a NaN; no host synchronisation. ``ws``: a uint8
    device tensor of >= hbk_nan_rows_workspace_size(n) bytes (allocated when None)."""
    _native.require_device(rows.device)
    n = rows.shape[0]
    if rows.dtype != torch.float32 or not rows.is_contiguous() or (n and (rows.numel() // n) % 4):
        raise ValueError("rows must be a contiguous float32 [n, ...] tensor with a multiple of 4 values per row")
    if n == 0:
        return rows
    need = int(lib().hbk_nan_rows_workspace_size(n))
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.uint8, device=rows.device)
    torch.ops.hbk.nan_rows_fix_(rows, _u64_to_i64(seed), ws)
    return rows


@torch.library.custom_op("hbk::place_clips", mutates_args=())
def _place_clips_op(src: torch.Tensor, src_len: torch.Tensor, pre: torch.Tensor, T: int) -> torch.Tensor:
    n = src.shape[0]
    out = torch.empty((n, T), dtype=torch.float32, device=src.device)
    if n:
        check(lib().hbk_place_clips(ptr(src), n, src.stride(0), ptr(src_len), ptr(pre), ptr(out), T, T,
                                    stream_ptr(src.device)), "hbk_place_clips")
    return out


@_place_clips_op.register_fake
def _(src, src_len, pre, T):
    return src.new_empty((src.shape[0], T))


def place_clips(src: torch.Tensor, src_len, pre, T: int = 23040) -> torch.Tensor:
    """AugmentedAudioGenerator.to_target_length on the device (hbk_place_clips):
    src [n, S] f32 rows holding src_len[i] valid samples -> [n, T] with clip i
    shifted right by pre[i] zeros and cut at T."""
    dev = _native.require_device(src.device)
    if src.dim() != 2 or src.dtype != torch.float32 or src.stride(1) != 1:
        raise ValueError("src must be [n, S] float32 rows on the device")
    n = src.shape[0]

    def per_clip(v) -> torch.Tensor:
        t = torch.as_tensor(v, dtype=torch.int32).reshape(-1).contiguous()
        if t.numel() != n:
            raise ValueError("src_len / pre must have n entries")
        if t.device.type == "cpu":
            if bool((t < 0).any()):
                raise ValueError("src_len / pre must be >= 0")
            return t.pin_memory().to(dev, non_blocking=True)
        return t.to(dev)

    if torch.is_tensor(src_len) and src_len.device.type != "cpu":
        src_len = src_len.clamp(0, src.shape[1])  # the kernel reads src[i, :min(len, T)]
    elif int(np.max(np.asarray(src_len), initial=0)) > src.shape[1]:
        raise ValueError(f"src_len exceeds the {src.shape[1]} source columns")
    src_len, pre = per_clip(src_len), per_clip(pre)
    return torch.ops.hbk.place_clips(src, src_len, pre, int(T))


def _active_rows(values: torch.Tensor) -> torch.Tensor | None:
    """int32 rows whose per-clip parameter is not NaN (a host tensor: the
    indexed, balanced launch), or None for a device tensor (every row)."""
    if values.device.type != "cpu":
        return None
    return torch.from_numpy(np.flatnonzero(~np.isnan(values.numpy())).astype(np.int32))


def tanh_distortion(x: torch.Tensor, amount: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """audiomentations TanhDistortion per clip on x [n, >= 23040] -> out [n, 23040]
    (hbk_tanh_distortion); amount per clip, NaN leaves the clip unchanged. A
    host ``amount`` launches over the clips it switches on only."""
    T = ReverbPlan.T
    dev = _native.require_device(x.device)
    n = x.shape[0]
    if x.dim() != 2 or x.shape[1] < T or x.stride(1) != 1 or x.dtype != torch.float32:
        raise ValueError(f"x must be [n, >= {T}] f32 rows on the device")
    amount = amount.to(dtype=torch.float32).reshape(-1).contiguous()
    if amount.numel() != n:
        raise ValueError("amount must have n entries")
    rows = _active_rows(amount)
    amount = amount.pin_memory().to(dev, non_blocking=True) if amount.device.type == "cpu" else amount.to(dev)
    if out is None:
        out = torch.empty((n, T), dtype=torch.float32, device=dev)
    if rows is not None:
        if out.data_ptr() != x.data_ptr():
            out.copy_(x[:, :T])  # the indexed launch writes the listed rows only
            x = out
        if rows.numel() == 0:
            return out
        rows = rows.pin_memory().to(dev, non_blocking=True)
    torch.ops.hbk.tanh_distortion_(x, amount, rows, out)
    return out


PITCH_SHIFT_CHUNK = 16384  # clips per hbk_pitch_shift call (~0.1 MB of workspace each)
# workspace per (device, stream): calls on one stream are ordered, so they may
# share one; a call on another stream gets its own (no cross-stream reuse)
_PS_WS: dict = {}


def pitch_shift(x: torch.Tensor, idx: torch.Tensor, num: int, den: int, out: torch.Tensor | None = None,
                sample_rate: int = 16000) -> torch.Tensor:
    """torch_pitch_shift.pitch_shift(x[idx], Fraction(num, den), sample_rate)
    (hbk_pitch_shift; torch_audiomentations PitchShift per batch,
    dataset/augmented.py:93-100) on rows idx of x [n, >= 23040] -> out [n, 23040].
    Rows not listed are copied from x when out is a different buffer."""
    T = ReverbPlan.T
    dev = _native.require_device(x.device)
    if x.dim() != 2 or x.shape[1] < T or x.stride(1) != 1 or x.dtype != torch.float32:
        raise ValueError(f"x must be [n, >= {T}] f32 rows on the device")
    n = x.shape[0]
    if out is None:
        out = torch.empty((n, T), dtype=torch.float32, device=dev)
    if out.data_ptr() != x.data_ptr():
        out.copy_(x[:, :T])
        x = out
    idx = idx.to(dtype=torch.int32).reshape(-1)
    if idx.numel() == 0:
        return out
    if idx.device.type == "cpu":
        if int(idx.min()) < 0 or int(idx.max()) >= n:
            raise ValueError("idx out of range")
        idx = idx.pin_memory().to(dev, non_blocking=True)
    chunk = min(PITCH_SHIFT_CHUNK, idx.numel())
    need = int(lib().hbk_pitch_shift_workspace_size(chunk, T, sample_rate, num, den))
    if need <= 0:
        raise ValueError(f"unsupported pitch shift {num}/{den} at {sample_rate} Hz")
    key = (dev, stream_ptr(dev))
    ws = _PS_WS.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.uint8, device=dev)  # allocated on this stream: no record_stream needed
        _PS_WS[key] = ws
    for c0 in range(0, idx.numel(), chunk):
        torch.ops.hbk.pitch_shift_(x, idx[c0:c0 + chunk], num, den, sample_rate, out, ws)
    return out


@torch.library.custom_op("hbk::pitch_shift_", mutates_args=("out", "workspace"))
def _pitch_shift_op(x: torch.Tensor, idx: torch.Tensor, num: int, den: int, sample_rate: int, out: torch.Tensor,
                    workspace: torch.Tensor) -> None:
    check(lib().hbk_pitch_shift(ptr(x), x.stride(0), idx.numel(), ptr(idx), ReverbPlan.T, sample_rate, num, den,
                                ptr(out), out.stride(0), ptr(workspace), workspace.numel(), stream_ptr(x.device)),
          "hbk_pitch_shift")


def seven_band_eq(x: torch.Tensor, coef: torch.Tensor, out: torch.Tensor | None = None,
                  idx: torch.Tensor | None = None) -> torch.Tensor:
    """audiomentations SevenBandParametricEQ per clip (hbk_seven_band_eq).
    Without ``idx``: every clip of x [n, >= 23040] -> out [n, 23040], coef
    [n, 7, 5] float64 (b0, b1, b2, a1, a2 of the low shelf, five peaks and high
    shelf, normalised by a0), a NaN coef[i, 0, 0] copies clip i. With ``idx``
    (int32 [m]): only clips idx[j] with coef [m, 7, 5], written into out
    (default: in place into x)."""
    T = ReverbPlan.T
    dev = _native.require_device(x.device)
    n = x.shape[0]
    if x.dim() != 2 or x.shape[1] < T or x.stride(1) != 1 or x.dtype != torch.float32:
        raise ValueError(f"x must be [n, >= {T}] f32 rows on the device")
    if x.stride(0) % 4 or x.data_ptr() % 16:
        raise ValueError("x rows must be 16-B aligned")

    def to_dev(t: torch.Tensor) -> torch.Tensor:
        return (t if t.is_pinned() else t.pin_memory()).to(dev, non_blocking=True) if t.device.type == "cpu" else t.to(dev)

    m = n if idx is None else int(idx.numel())
    coef = to_dev(coef.to(dtype=torch.float64).reshape(m, 7, 5).contiguous())
    if idx is not None:
        idx = idx.to(dtype=torch.int32).reshape(-1).contiguous()
        if idx.device.type == "cpu" and m and (int(idx.min()) < 0 or int(idx.max()) >= n):
            raise ValueError("idx out of range")
        idx = to_dev(idx)
        if out is None:
            out = x
    elif out is None:
        out = torch.empty((n, T), dtype=torch.float32, device=dev)
    if m:
        torch.ops.hbk.seven_band_eq_(x, coef, idx, out)
    return out


@torch.library.custom_op("hbk::seven_band_eq_", mutates_args=("out",))
def _seven_band_eq_op(x: torch.Tensor, coef: torch.Tensor, idx: torch.Tensor | None, out: torch.Tensor) -> None:
    check(lib().hbk_seven_band_eq(ptr(x), x.shape[0], x.stride(0), ptr(coef), ptr(idx) if idx is not None else None,
                                  idx.numel() if idx is not None else x.shape[0], ptr(out), out.stride(0),
                                  stream_ptr(x.device)), "hbk_seven_band_eq")


@torch.library.custom_op("hbk::tanh_distortion_", mutates_args=("out",))
def _tanh_distortion_op(x: torch.Tensor, amount: torch.Tensor, rows: torch.Tensor | None, out: torch.Tensor) -> None:
    check(lib().hbk_tanh_distortion(ptr(x), x.shape[0], x.stride(0), ptr(amount),
                                    ptr(rows) if rows is not None else None, rows.numel() if rows is not None else 0,
                                    ptr(out), out.stride(0), stream_ptr(x.device)), "hbk_tanh_distortion")


BAND_STOP_CIRCULAR_MAX_HALF = 512  # HBK_BAND_STOP_CIRCULAR_MAX_HALF (include/hbk.h)


class ReverbPlan:
    """Batch augmentation on the HIP path (hbk_reverb_* / hbk_augment):
    background-noise mix + IR reverb for clips of 23,040 samples."""

    T = 23040
    # colored noise: the group path (one coloured second per group, 64 KB of
    # workspace each) only for groups of at least this many clips
    COLORED_GROUP_MIN = 8

    def __init__(self, device: torch.device | int | None = None) -> None:
        self.device = _native.require_device(device)
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().hbk_reverb_plan_create(self.T, ctypes.byref(handle)), "hbk_reverb_plan_create")
        self._handle = handle
        self._bs_ws: torch.Tensor | None = None  # band-stop workspace (grows)
        self._cn_ws: torch.Tensor | None = None  # colored-noise group seconds (grows)
        self.id = _register(self)

    @staticmethod
    def rotated_kernel(ir: torch.Tensor, T: int = 23040) -> torch.Tensor:
        """speechbrain convolve1d(use_fft=True, rotation_index=argmax|ir|):
        [ir[d:], zeros(T - L), ir[:d]] with ir truncated to T first."""
        ir = ir.reshape(-1).to(torch.float32)
        d = int(torch.argmax(ir.abs()).item())
        if ir.shape[0] > T:
            ir = ir[:T]
        z = torch.zeros(T - ir.shape[0], dtype=ir.dtype, device=ir.device)
        return torch.cat([ir[d:], z, ir[:d]])

    SLOTS = 11536  # HBK_REVERB_SPECTRUM_SLOTS: bin k at slot (k % 16) * 721 + k // 16

    def spectra(self, kernels: torch.Tensor) -> torch.Tensor:
        """[n, T] rotated kernels -> [n, SLOTS, 2] f32 (complex interleaved), rfft
        bin k at slot (k % 16) * 721 + k // 16 (natural_spectrum() undoes it)."""
        kernels = kernels.to(self.device, torch.float32).contiguous()
        n = kernels.shape[0]
        out = torch.zeros((n, self.SLOTS, 2), dtype=torch.float32, device=self.device)
        torch.ops.hbk.reverb_spectrum_(kernels, out, self.id)
        return out

    @classmethod
    def natural_spectrum(cls, spectra: torch.Tensor) -> torch.Tensor:
        """[n, SLOTS, 2] slot layout -> [n, T/2 + 1, 2] in bin order."""
        n = spectra.shape[0]
        rows = spectra.reshape(n, 16, cls.SLOTS // 16, 2)
        return rows.transpose(1, 2).reshape(n, cls.SLOTS, 2)[:, :cls.T // 2 + 1]

    def augment(self, x: torch.Tensor, ring: torch.Tensor | None, noise_off: torch.Tensor,
                snr_db: torch.Tensor, spectra: torch.Tensor | None, spec_idx: torch.Tensor,
                out: torch.Tensor | None = None, gain: torch.Tensor | None = None,
                colored: tuple | None = None) -> torch.Tensor:
        """x [n, >= T] -> out [n, T]; per clip gain (linear factor, if given), then
        noise (noise_off >= 0), then reverb (spec_idx >= 0). ``colored`` =
        (f_decay, snr_db, seed, clips_per_noise) runs colored_noise() with the
        generated white noise first, in the same pass (hbk_augment_colored:
        bit-identical to the two calls, each clip read and written once)."""
        n = x.shape[0]
        if x.dim() != 2 or x.shape[1] < self.T or x.stride(1) != 1 or x.device != self.device:
            raise ValueError(f"x must be [n, >= {self.T}] f32 rows on {self.device}")
        if out is None:
            out = torch.empty((n, self.T), dtype=torch.float32, device=self.device)
        # Host-side per-clip arrays (the BatchAugmenter path) are checked on the
        # host and sent through pinned memory without a device sync; device
        # tensors are checked on the device (a sync per check).
        def per_clip(t: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
            t = t.to(dtype=dtype).reshape(-1).contiguous()
            if t.numel() != n:
                raise ValueError("per-clip arrays must have n entries")
            return t

        noise_off = per_clip(noise_off, torch.int64)
        spec_idx = per_clip(spec_idx, torch.int32)
        snr_db = per_clip(snr_db, torch.float32)
        if gain is not None:
            gain = per_clip(gain, torch.float32)
        if spectra is not None and (spectra.dim() != 3 or spectra.shape[1:] != (self.SLOTS, 2)):
            raise ValueError(f"spectra must be [n, {self.SLOTS}, 2] (ReverbPlan.spectra's slot layout)")
        ring_n = 0 if ring is None else ring.numel()
        if bool((noise_off >= 0).any()) and ring_n == 0:
            raise ValueError("noise requested without a noise ring")
        if ring_n and bool((noise_off >= ring_n).any()):
            raise ValueError("noise_off must be < the ring length")
        if spectra is not None and bool((spec_idx >= spectra.shape[0]).any()):
            raise ValueError("spec_idx out of range")

        def to_dev(t: torch.Tensor) -> torch.Tensor:
            if t.device.type == "cpu":
                return t.pin_memory().to(self.device, non_blocking=True)
            return t.to(self.device)

        noise_off, spec_idx, snr_db = to_dev(noise_off), to_dev(spec_idx), to_dev(snr_db)
        if gain is not None:
            gain = to_dev(gain)
        if colored is None:
            torch.ops.hbk.augment_(x, ring, noise_off, snr_db, spectra, spec_idx, gain, out, self.id)
            return out
        f_decay, c_snr, seed, clips_per_noise = colored
        f_decay, c_snr = per_clip(f_decay, torch.float32), per_clip(c_snr, torch.float32)
        if clips_per_noise < 1:
            raise ValueError("clips_per_noise must be >= 1")
        if out.data_ptr() != x.data_ptr():
            lo_o, hi_o = out.data_ptr(), out.data_ptr() + out.stride(0) * 4 * n
            lo_x, hi_x = x.data_ptr(), x.data_ptr() + x.stride(0) * 4 * n
            if lo_o < hi_x and lo_x < hi_o:
                raise ValueError("out overlaps x without being x")
        ws = self._colored_workspace(n, clips_per_noise)
        # the clips the group path does not cover (a batch whose first clip drew no noise, or
        # an f_decay other than its group's first clip's): coloured per clip before the pass
        rows = None
        if c_snr.device.type == "cpu" and f_decay.device.type == "cpu":
            on = ~torch.isnan(c_snr)
            if ws is not None:
                first = (torch.arange(n) // clips_per_noise) * clips_per_noise
                on &= torch.isnan(c_snr[first]) | (f_decay != f_decay[first])
            rows = torch.nonzero(on).reshape(-1).to(torch.int32)
        n_rows = -1 if rows is None else rows.numel()  # -1: the kernel scans every clip
        if n_rows == 0:
            rows = torch.zeros(1, dtype=torch.int32)  # a valid pointer with no entries
        if rows is not None:
            rows = rows.pin_memory().to(self.device, non_blocking=True)
        torch.ops.hbk.augment_colored_(x, ring, noise_off, snr_db, spectra, spec_idx, gain, to_dev(f_decay),
                                       to_dev(c_snr), _u64_to_i64(seed), int(clips_per_noise), rows, n_rows, out,
                                       ws, self.id)
        return out

    def _colored_workspace(self, n: int, clips_per_noise: int) -> torch.Tensor | None:
        ws_bytes = int(lib().hbk_colored_noise_workspace_size(n, int(clips_per_noise)))
        if (os.environ.get("HBK_COLORED_NO_GROUP") or ws_bytes > (1 << 30)
                or int(clips_per_noise) < self.COLORED_GROUP_MIN):
            return None  # A/B switch; small groups are not worth 64 KB of resident workspace each
        if ws_bytes <= 0:
            return None
        ws = self._cn_ws
        if ws is None or ws.numel() < ws_bytes:
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=self.device)
            self._cn_ws = ws
        return ws

    def colored_noise(self, x: torch.Tensor, f_decay: torch.Tensor, snr_db: torch.Tensor,
                      white: torch.Tensor | None = None, seed: int = 0, out: torch.Tensor | None = None,
                      sample_rate: int = 16000, clips_per_noise: int = 1) -> torch.Tensor:
        """torch_audiomentations AddColoredNoise on x [n, >= T] -> out [n, T]
        (hbk_colored_noise): per clip f_decay and snr (dB; NaN leaves the clip
        unchanged); one second of white noise per group of ``clips_per_noise``
        consecutive clips (per_batch mode shares one vector across the batch;
        [ceil(n / clips_per_noise), >= 16000] N(0,1)) if given, else the
        kernel's counter-based stream from ``seed``; the coloured second is
        tiled to T as _gen_noise does."""
        n = x.shape[0]
        if x.dim() != 2 or x.shape[1] < self.T or x.stride(1) != 1 or x.device != self.device:
            raise ValueError(f"x must be [n, >= {self.T}] f32 rows on {self.device}")
        groups = (n + clips_per_noise - 1) // max(1, clips_per_noise)
        if clips_per_noise < 1:
            raise ValueError("clips_per_noise must be >= 1")
        if white is not None and (white.dim() != 2 or white.shape[0] != groups or white.shape[1] < 16000
                                  or white.stride(1) != 1 or white.device != self.device
                                  or white.dtype != torch.float32):
            raise ValueError(f"white must be [{groups}, >= 16000] f32 rows on {self.device}")
        if out is None:
            out = torch.empty((n, self.T), dtype=torch.float32, device=self.device)

        def per_clip(t: torch.Tensor) -> torch.Tensor:
            t = t.to(dtype=torch.float32).reshape(-1).contiguous()
            if t.numel() != n:
                raise ValueError("per-clip arrays must have n entries")
            return t

        f_decay, snr_db = per_clip(f_decay), per_clip(snr_db)
        rows = _active_rows(snr_db)  # host snr: launch over the clips whose batch drew noise only
        if rows is not None:
            if out.data_ptr() != x.data_ptr():
                out.copy_(x[:, :self.T])  # the indexed launch writes the listed rows only
                x = out
            if rows.numel() == 0:
                return out
            rows = rows.pin_memory().to(self.device, non_blocking=True)

        def to_dev(t: torch.Tensor) -> torch.Tensor:
            return t.pin_memory().to(self.device, non_blocking=True) if t.device.type == "cpu" else t.to(self.device)

        # clips_per_noise > 1: each group's coloured second is made once (hbk_colored_noise_ws)
        ws = self._colored_workspace(n, clips_per_noise)
        torch.ops.hbk.colored_noise_(x, white, to_dev(f_decay), to_dev(snr_db), _u64_to_i64(seed),
                                     int(clips_per_noise), float(sample_rate), rows, out, ws, self.id)
        return out

    def band_stop(self, x: torch.Tensor, idx: torch.Tensor, cut_lo: torch.Tensor, cut_hi: torch.Tensor,
                  out: torch.Tensor | None = None) -> torch.Tensor:
        """torch_audiomentations BandStopFilter on rows idx of x [n, >= T] ->
        out [n, T] (hbk_band_stop): out[idx[e]] = x[idx[e]] - julius
        bandpass(cut_lo[e], cut_hi[e]) (fractions of the sample rate); other
        rows of out are left as they are (out may be x)."""
        n = x.shape[0]
        if x.dim() != 2 or x.shape[1] < self.T or x.stride(1) != 1 or x.device != self.device:
            raise ValueError(f"x must be [n, >= {self.T}] f32 rows on {self.device}")
        if out is None:
            out = x[:, :self.T].clone()
        e = idx.numel()
        if cut_lo.numel() != e or cut_hi.numel() != e:
            raise ValueError("idx, cut_lo and cut_hi must have one entry per filtered clip")
        if e == 0:
            return out
        lo_h = cut_lo.detach().to("cpu", torch.float32).reshape(-1)
        hi_h = cut_hi.detach().to("cpu", torch.float32).reshape(-1)
        if not bool(((lo_h > 0) & (lo_h <= hi_h) & (hi_h <= 0.5)).all()):
            raise ValueError("band-stop cutoffs must satisfy 0 < cut_lo <= cut_hi <= 0.5")
        idx_h = idx.detach().to("cpu", torch.int32).reshape(-1)
        if bool(((idx_h < 0) | (idx_h >= n)).any()):
            raise ValueError("idx out of range")
        # one filter per distinct cutoff pair (a batch's clips share theirs)
        pairs, filt = np.unique(np.stack([lo_h.numpy(), hi_h.numpy()], 1), axis=0, return_inverse=True)
        # julius LowPassFilters.half_size = int(zeros / min(cutoffs) / 2), zeros = 8
        half = np.array([int(8 / float(c) / 2) for c in pairs[:, 0].tolist()], dtype=np.int32)
        nspec = np.where(half <= BAND_STOP_CIRCULAR_MAX_HALF, 1, (2 * half + 1 + 11520) // 11521).astype(np.int32)
        spec0 = np.concatenate([[0], np.cumsum(nspec)[:-1]]).astype(np.int32)
        s_filt = np.repeat(np.arange(len(pairs), dtype=np.int32), nspec)
        s_part = np.concatenate([[-1] if h <= BAND_STOP_CIRCULAR_MAX_HALF else np.arange(k)
                                 for h, k in zip(half, nspec)]).astype(np.int32)

        def to_dev(a) -> torch.Tensor:
            return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(self.device, non_blocking=True)

        nf, ns = len(pairs), int(nspec.sum())
        ws_bytes = int(lib().hbk_band_stop_workspace_size(e, nf, ns, stream_ptr(self.device)))
        if self._bs_ws is None or self._bs_ws.numel() < ws_bytes:
            self._bs_ws = torch.empty(ws_bytes, dtype=torch.uint8, device=self.device)
        torch.ops.hbk.band_stop_(x, to_dev(idx_h.numpy()), to_dev(filt.astype(np.int32).reshape(-1)),
                                 to_dev(pairs[:, 0].astype(np.float32)), to_dev(pairs[:, 1].astype(np.float32)),
                                 to_dev(half), to_dev(spec0), to_dev(s_filt), to_dev(s_part), out, self._bs_ws,
                                 self.id)
        return out

    def __del__(self) -> None:
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            try:
                lib().hbk_reverb_plan_destroy(h)
            except Exception:
                pass
            self._handle = None


@torch.library.custom_op("hbk::reverb_spectrum_", mutates_args=("out",))
def _reverb_spectrum_op(kernels: torch.Tensor, out: torch.Tensor, plan_id: int) -> None:
    plan = _plans[plan_id]
    check(lib().hbk_reverb_spectrum(plan._handle, ptr(kernels), kernels.shape[0], kernels.stride(0), ptr(out),
                                    stream_ptr(kernels.device)), "hbk_reverb_spectrum")


@torch.library.custom_op("hbk::augment_", mutates_args=("out",))
def _augment_op(x: torch.Tensor, ring: torch.Tensor | None, noise_off: torch.Tensor, snr_db: torch.Tensor,
                spectra: torch.Tensor | None, spec_idx: torch.Tensor, gain: torch.Tensor | None, out: torch.Tensor,
                plan_id: int) -> None:
    plan = _plans[plan_id]
    opt = lambda t: ptr(t) if t is not None else None  # noqa: E731
    check(lib().hbk_augment(plan._handle, ptr(x), x.shape[0], x.stride(0), opt(ring),
                            0 if ring is None else ring.numel(), ptr(noise_off), ptr(snr_db), opt(spectra),
                            ptr(spec_idx), opt(gain), ptr(out), out.stride(0), stream_ptr(x.device)), "hbk_augment")


@torch.library.custom_op("hbk::augment_colored_", mutates_args=("out", "workspace"))
def _augment_colored_op(x: torch.Tensor, ring: torch.Tensor | None, noise_off: torch.Tensor, snr_db: torch.Tensor,
                        spectra: torch.Tensor | None, spec_idx: torch.Tensor, gain: torch.Tensor | None,
                        f_decay: torch.Tensor, c_snr: torch.Tensor, seed: int, clips_per_noise: int,
                        rows: torch.Tensor | None, n_rows: int, out: torch.Tensor, workspace: torch.Tensor | None,
                        plan_id: int) -> None:
    plan = _plans[plan_id]
    opt = lambda t: ptr(t) if t is not None else None  # noqa: E731
    check(lib().hbk_augment_colored(plan._handle, ptr(x), x.shape[0], x.stride(0), opt(ring),
                                    0 if ring is None else ring.numel(), ptr(noise_off), ptr(snr_db), opt(spectra),
                                    ptr(spec_idx), opt(gain), None, 0, seed & (2 ** 64 - 1), clips_per_noise,
                                    ptr(f_decay), ptr(c_snr), 16000.0, opt(rows) if n_rows >= 0 else None,
                                    max(n_rows, 0), ptr(out), out.stride(0),
                                    opt(workspace), workspace.numel() if workspace is not None else 0,
                                    stream_ptr(x.device)), "hbk_augment_colored")


@torch.library.custom_op("hbk::colored_noise_", mutates_args=("out", "workspace"))
def _colored_noise_op(x: torch.Tensor, white: torch.Tensor | None, f_decay: torch.Tensor, snr_db: torch.Tensor,
                      seed: int, clips_per_noise: int, sample_rate: float, rows: torch.Tensor | None,
                      out: torch.Tensor, workspace: torch.Tensor | None, plan_id: int) -> None:
    plan = _plans[plan_id]
    check(lib().hbk_colored_noise_ws(plan._handle, ptr(x), x.shape[0], x.stride(0),
                                     ptr(white) if white is not None else None,
                                     white.stride(0) if white is not None else 0, seed & (2 ** 64 - 1),
                                     clips_per_noise, ptr(f_decay),
                                     ptr(snr_db), sample_rate, ptr(rows) if rows is not None else None,
                                     rows.numel() if rows is not None else 0, ptr(out), out.stride(0),
                                     ptr(workspace) if workspace is not None else None,
                                     workspace.numel() if workspace is not None else 0,
                                     stream_ptr(x.device)), "hbk_colored_noise_ws")


@torch.library.custom_op("hbk::band_stop_", mutates_args=("out", "workspace"))
def _band_stop_op(x: torch.Tensor, idx: torch.Tensor, filt: torch.Tensor, f_lo: torch.Tensor, f_hi: torch.Tensor,
                  f_half: torch.Tensor, f_spec0: torch.Tensor, s_filt: torch.Tensor, s_part: torch.Tensor,
                  out: torch.Tensor, workspace: torch.Tensor, plan_id: int) -> None:
    plan = _plans[plan_id]
    check(lib().hbk_band_stop(plan._handle, ptr(x), x.stride(0), idx.numel(), ptr(idx), ptr(filt), f_lo.numel(),
                              ptr(f_lo), ptr(f_hi), ptr(f_half), ptr(f_spec0), s_filt.numel(), ptr(s_filt),
                              ptr(s_part), ptr(out), out.stride(0), ptr(workspace), workspace.numel(),
                              stream_ptr(x.device)), "hbk_band_stop")
