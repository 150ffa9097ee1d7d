"""Drop-in for heybuddy.spectrogram (reference src/python/heybuddy/spectrogram.py).

``MelSpectrogramModel.__call__`` keeps the reference contract (numpy
[b, t] int16-range audio in, numpy [b, frames, 32] log-mel out, already
``/10 + 2``-scaled, squeezed) but runs the fused STFT + mel HIP kernel
(hbk_mel_frames) instead of an ONNX Runtime session. The mel parameters are
runtime data (window, filterbank); the defaults are hypothesis H0 of
SURVEY.md §8a-3 (torchaudio MelSpectrogram, n_fft 512, win 400, hop 160,
60-3800 Hz, 32 HTK mels, 10 log10(max(P, 1e-10))).

The reference's own graph (``mel-spectrogram.onnx``, sha256 ba2b0e0f...,
spectrogram.py:20-21: "an ONNX version of the PyTorch model from the
torchaudio library") replaces H0 when it is present: ``mel_params_from_onnx``
reads the window, hop, filterbank, log floor and output scaling out of the
graph, ``MelSpectrogramModel.load`` picks the file up from the pretrained
directory (sha-checked), ``set_mel_parameters`` installs any parameters.
``mel_graph_to_onnx`` writes the front end as such a graph.
"""
from __future__ import annotations

import math
import os
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from heybuddy import _native
from heybuddy.kernels import MelPlan

__all__ = ["MelSpectrogramModel", "get_mel_spectrogram_model", "mel_parameters", "MelParams",
           "default_mel_plan", "set_mel_parameters", "mel_params_from_onnx", "mel_graph_to_onnx",
           "pretrained_dir", "REFERENCE_MEL_SHA256"]

SAMPLE_RATE = 16000
N_FFT = 512
WIN_LENGTH = 400
HOP = 160
F_MIN = 60.0
F_MAX = 3800.0
N_MELS = 32


def _hann_window(win_length: int = WIN_LENGTH, n_fft: int = N_FFT) -> np.ndarray:
    n = np.arange(win_length, dtype=np.float64)
    w = 0.5 - 0.5 * np.cos(2.0 * np.pi * n / win_length)  # periodic Hann
    out = np.zeros(n_fft, dtype=np.float64)
    left = (n_fft - win_length) // 2                         # torch.stft centring
    out[left:left + win_length] = w
    return out.astype(np.float32)


def _mel_fbank(n_freqs: int = N_FFT // 2 + 1, f_min: float = F_MIN, f_max: float = F_MAX,
               n_mels: int = N_MELS, sample_rate: int = SAMPLE_RATE) -> np.ndarray:
    hz2mel = lambda f: 2595.0 * np.log10(1.0 + np.asarray(f, np.float64) / 700.0)  # noqa: E731
    mel2hz = lambda m: 700.0 * (10.0 ** (np.asarray(m, np.float64) / 2595.0) - 1.0)  # noqa: E731
    all_freqs = np.linspace(0, sample_rate // 2, n_freqs)
    f_pts = mel2hz(np.linspace(hz2mel(f_min), hz2mel(f_max), n_mels + 2))
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    fb = np.maximum(0.0, np.minimum(-slopes[:, :-2] / f_diff[:-1], slopes[:, 2:] / f_diff[1:]))
    return fb.astype(np.float32)


class MelParams:
    """Everything the fused mel kernel needs of a mel graph: the window [n_fft]
    (zero outside its support), hop, filterbank [n_fft / 2 + 1, n_mels] applied
    to the power spectrum, the log floor, and the graph's output as
    ``scale * 10 log10(max(P, floor)) + offset`` of the power P of the input
    times ``in_scale``. The reference then applies ``/ 10 + 2`` on the host
    (spectrogram.py:32), folded into the plan's out_div / out_add."""

    def __init__(self, window: np.ndarray, fbank: np.ndarray, hop: int = HOP, log_floor: float = 1e-10,
                 scale: float = 1.0, offset: float = 0.0, in_scale: float = 1.0, source: str = "H0") -> None:
        self.window = np.ascontiguousarray(window, dtype=np.float32)
        self.fbank = np.ascontiguousarray(fbank, dtype=np.float32)
        if self.window.ndim != 1 or self.fbank.shape[0] != self.window.shape[0] // 2 + 1:
            raise ValueError(f"window {self.window.shape} and filterbank {self.fbank.shape} do not match")
        self.hop, self.log_floor = int(hop), float(log_floor)
        self.scale, self.offset, self.in_scale = float(scale), float(offset), float(in_scale)
        self.source = source

    @property
    def n_fft(self) -> int:
        return int(self.window.shape[0])

    def plan_args(self) -> Dict[str, float]:
        """MelPlan keyword arguments for the reference's host scaling (/10 + 2)."""
        return {"hop": self.hop, "log_floor": self.log_floor, "out_div": 10.0 / self.scale,
                "out_add": 2.0 + self.offset / 10.0}


def mel_parameters() -> Tuple[np.ndarray, np.ndarray]:
    """(window [512], filterbank [257, 32]) of the current mel graph (H0
    unless set_mel_parameters / MelSpectrogramModel.load installed another)."""
    p = current_mel_params()
    return p.window, p.fbank


_PARAMS: List[Optional[MelParams]] = [None]
_PLANS: Dict[Tuple[int, float], MelPlan] = {}


def current_mel_params() -> MelParams:
    """The installed parameters; at first use the reference's graph if
    ``mel-spectrogram.onnx`` with its sha256 is in pretrained_dir() (never
    downloaded), else H0."""
    if _PARAMS[0] is None:
        path = find_pretrained(REFERENCE_MEL_FILE, REFERENCE_MEL_SHA256)
        params = None
        if path is not None:
            # the importer's parity with the real graph is unpinned (the file is not in the
            # reference tree): a graph it cannot map, or one with other frame geometry, falls
            # back to H0 with a warning instead of failing every featurize call
            try:
                params = mel_params_from_onnx(path)
                set_mel_parameters(params)
            except ValueError as e:
                logger.warning("%s could not be used (%s); using the H0 mel parameters", path, e)
                params = None
        if params is None:
            _PARAMS[0] = MelParams(_hann_window(), _mel_fbank())
    return _PARAMS[0]


def set_mel_parameters(params: Optional[MelParams]) -> None:
    """Install the mel graph's parameters (None: back to H0). The featurizer's
    frame geometry is the reference's (512-sample frames at hop 160,
    embeddings.py:67 / :190), so other frame sizes are refused."""
    if params is not None and (params.n_fft != N_FFT or params.hop != HOP):
        raise ValueError(f"the featurizer needs {N_FFT}-sample frames at hop {HOP} (embeddings.py:67); "
                         f"this graph has {params.n_fft} / {params.hop}")
    _PARAMS[0] = params
    _PLANS.clear()


def default_mel_plan(device: torch.device, in_scale: float = 32767.0) -> MelPlan:
    """Cached plan per (device, input scale) of the current mel parameters."""
    key = (device.index, float(in_scale))
    if key not in _PLANS:
        p = current_mel_params()
        _PLANS[key] = MelPlan(p.window, p.fbank, in_scale=in_scale * p.in_scale, device=device, **p.plan_args())
    return _PLANS[key]


# -- the reference's pretrained graph ---------------------------------------------------
REFERENCE_MEL_FILE = "mel-spectrogram.onnx"  # spectrogram.py:20
REFERENCE_MEL_SHA256 = "ba2b0e0f8b7b875369a2c89cb13360ff53bac436f2895cced9f479fa65eb176f"  # spectrogram.py:21


def pretrained_dir() -> str:
    """Where the reference caches its downloads (util/pretrained_util.py:5:
    the package's ``pretrained/``), or $HEYBUDDY_PRETRAINED_DIR. Nothing is
    downloaded here: a file the user copied there is used."""
    return os.environ.get("HEYBUDDY_PRETRAINED_DIR") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                     "pretrained")


def find_pretrained(file_name: str, sha256: str) -> Optional[str]:
    """The reference's pretrained file in pretrained_dir() if its sha256 is the
    reference's (file_util.py:207 checks the same sum); None if absent; a file
    with another sum is not used (warned once)."""
    from heybuddy.util import logger
    from heybuddy.util.onnx_util import sha256_of
    path = os.path.join(pretrained_dir(), file_name)
    if not os.path.isfile(path):
        return None
    got = sha256_of(path)
    if got != sha256:
        logger.warning(f"heybuddy: {path} has sha256 {got}, not the reference's {sha256}; not used")
        return None
    return path


def mel_graph_to_onnx(path: str, params: Optional[MelParams] = None, layout: str = "conv",
                      opset_version: int = 17) -> None:
    """Write the mel front end as an ONNX graph, input ``input`` [b, t] -> output
    [b, 1, frames, n_mels] = scale * 10 log10(max(P, floor)) + offset, the way
    torchaudio's MelSpectrogram exports: ``layout`` "stft" (torch.stft as the
    opset-17 STFT op, Pow + ReduceSum power, MatMul filterbank, Clip, Log, Div
    ln 10, Mul) or "conv" (the DFT as a cos and a sin Conv1d of the windowed
    basis, stride hop, as exporters without STFT emit; Mul / Add power, Max
    floor, Log, one Mul)."""
    from heybuddy.util.onnx_util import write_model
    p = current_mel_params() if params is None else params
    n, k = p.n_fft, p.n_fft // 2 + 1
    nodes: list = []
    inits: Dict[str, np.ndarray] = {"mel_fb": p.fbank}
    x = "input"
    if p.in_scale != 1.0:
        inits["in_scale"] = np.array(p.in_scale, np.float32)
        nodes.append(("Mul", "scale_in", [x, "in_scale"], ["x_scaled"], {}))
        x = "x_scaled"
    if layout == "stft":
        inits.update({"axes_2": np.array([2], np.int64), "hop": np.array(p.hop, np.int64), "window": p.window,
                      "frame_length": np.array(n, np.int64), "two": np.array(2.0, np.float32),
                      "axes_3": np.array([3], np.int64)})
        nodes += [("Unsqueeze", "unsqueeze_sig", [x, "axes_2"], ["sig"], {}),
                  ("STFT", "stft", ["sig", "hop", "window", "frame_length"], ["spec"], {"onesided": 1}),
                  ("Pow", "pow", ["spec", "two"], ["spec_sq"], {}),
                  ("ReduceSum", "power", ["spec_sq", "axes_3"], ["pw"], {"keepdims": 0}),  # [b, F, K]
                  ("MatMul", "mel", ["pw", "mel_fb"], ["mel"], {})]
        inits.update({"amin": np.array(p.log_floor, np.float32), "ln10": np.array(math.log(10.0), np.float32),
                      "ten": np.array(10.0 * p.scale, np.float32)})
        nodes += [("Clip", "clamp", ["mel", "amin"], ["mel_c"], {}),
                  ("Log", "log", ["mel_c"], ["ln"], {}),
                  ("Div", "log10", ["ln", "ln10"], ["l10"], {}),
                  ("Mul", "db", ["l10", "ten"], ["db"], {})]
    elif layout == "conv":
        t = np.arange(n, dtype=np.float64)
        ang = 2.0 * np.pi * np.outer(np.arange(k), t) / n
        w = p.window.astype(np.float64)
        inits["dft_re"] = (np.cos(ang) * w).astype(np.float32)[:, None, :]
        inits["dft_im"] = (-np.sin(ang) * w).astype(np.float32)[:, None, :]
        inits["axes_1"] = np.array([1], np.int64)
        conv = {"kernel_shape": [n], "strides": [p.hop], "pads": [0, 0], "dilations": [1], "group": 1}
        nodes += [("Unsqueeze", "unsqueeze_ch", [x, "axes_1"], ["sig"], {}),
                  ("Conv", "stft_re", ["sig", "dft_re"], ["re"], conv),
                  ("Conv", "stft_im", ["sig", "dft_im"], ["im"], conv),
                  ("Mul", "re2", ["re", "re"], ["re_sq"], {}),
                  ("Mul", "im2", ["im", "im"], ["im_sq"], {}),
                  ("Add", "power", ["re_sq", "im_sq"], ["pw_kf"], {}),          # [b, K, F]
                  ("Transpose", "to_fk", ["pw_kf"], ["pw"], {"perm": [0, 2, 1]}),
                  ("MatMul", "mel", ["pw", "mel_fb"], ["mel"], {})]
        inits.update({"amin": np.array(p.log_floor, np.float32),
                      "db_per_ln": np.array(10.0 * p.scale / math.log(10.0), np.float32)})
        nodes += [("Max", "clamp", ["mel", "amin"], ["mel_c"], {}),
                  ("Log", "log", ["mel_c"], ["ln"], {}),
                  ("Mul", "db", ["ln", "db_per_ln"], ["db"], {})]
    else:
        raise ValueError(f"unknown layout {layout!r}")
    y = "db"
    if p.offset:
        inits["offset"] = np.array(p.offset, np.float32)
        nodes.append(("Add", "db_offset", [y, "offset"], ["db_o"], {}))
        y = "db_o"
    inits["axes_1o"] = np.array([1], np.int64)
    nodes.append(("Unsqueeze", "unsqueeze_out", [y, "axes_1o"], ["output"], {}))
    write_model(path, nodes, inits, [("input", ["batch", "samples"])],
                [("output", ["batch", 1, "frames", p.fbank.shape[1]])], opset_version=opset_version,
                producer=f"heybuddy-amd mel ({layout})")


_SHAPE_OPS = ("Unsqueeze", "Squeeze", "Reshape", "Transpose", "Identity", "Flatten")


def mel_params_from_onnx(path: str) -> MelParams:
    """The mel front end of an ONNX graph as MelParams. The graph must be one
    path from its single input to its single output of: shape-only ops
    (Unsqueeze / Squeeze / Reshape / Transpose / Identity / Flatten, Cast to
    float); an input scale (Mul / Div by a scalar constant); the short-time DFT
    as the opset-17 STFT op (window input, frame_step, frame_length; onesided)
    or as a pair of Conv1d's of one input whose kernels are window * cos and
    window * (-)sin of the DFT basis (checked entry by entry), stride = hop;
    the power (Pow 2 / Mul x x, summed over the re / im pair); the filterbank
    as a MatMul with a [n_fft / 2 + 1, n_mels] constant (or its transpose on
    the left); the floor as Clip(min) / Max with a scalar constant; Log, and
    the dB scaling and offset as scalar Mul / Div / Add / Sub. Anything else,
    or the stages out of that order, raises ValueError naming the node."""
    from heybuddy.util.onnx_util import read_model
    m = read_model(path)
    if len(m.inputs) != 1 or len(m.outputs) != 1:
        raise ValueError(f"{path}: expected one graph input and one output")
    inits = m.initializers
    out_name = m.outputs[0][0]

    def scalar(name_: str, where: str) -> float:
        if name_ not in inits or np.asarray(inits[name_]).size != 1:
            raise ValueError(f"{where}: {name_!r} must be a scalar constant")
        return float(np.asarray(inits[name_]).reshape(-1)[0])

    def single_user(x_: str) -> "object":
        users = m.consumers(x_)
        if len(users) != 1:
            raise ValueError(f"{path}: tensor {x_!r} feeds {len(users)} nodes")
        return users[0]

    in_scale, window, hop, fbank, floor = 1.0, None, None, None, None
    mult, offset = 1.0, 0.0  # the graph output = mult * ln(max(P, floor)) + offset, after "Log"
    stage = "input"  # input -> spectrum -> power -> mel -> floored -> log
    x = m.inputs[0][0]
    while x != out_name:
        users = m.consumers(x)
        where = f"{path}: tensor {x!r}"
        if stage == "input" and len(users) == 2 and all(u.op == "Conv" for u in users):
            kern = []
            for u in users:
                w = inits.get(u.inputs[1])
                if w is None or w.ndim != 3 or w.shape[1] != 1 or (len(u.inputs) > 2 and u.inputs[2]):
                    raise ValueError(f"{path}: Conv {u.name!r} is not a bias-free single-channel Conv1d DFT")
                a = u.attrs
                if any(a.get("pads", (0, 0))) or tuple(a.get("dilations", (1,))) != (1,) or int(a.get("group", 1)) != 1:
                    raise ValueError(f"{path}: Conv {u.name!r}: padded / dilated / grouped DFT convs are not supported")
                kern.append((w[:, 0, :].astype(np.float64), int(tuple(a.get("strides", (1,)))[0]), u))
            (k0, s0, u0), (k1, s1, u1) = kern
            if s0 != s1 or k0.shape != k1.shape:
                raise ValueError(f"{path}: the two DFT convs differ in stride or shape")
            if np.abs(k0[0]).max() < np.abs(k1[0]).max():  # the cos kernel's bin 0 is the window itself
                (k0, u0), (k1, u1) = (k1, u1), (k0, u0)
            n = k0.shape[1]
            kk = np.arange(k0.shape[0])
            if k0.shape[0] != n // 2 + 1:
                raise ValueError(f"{path}: {k0.shape[0]} DFT rows for {n}-sample frames (expected {n // 2 + 1})")
            win = k0[0]
            ang = 2.0 * np.pi * np.outer(kk, np.arange(n)) / n
            tol = 1e-5 * max(np.abs(win).max(), 1e-30)
            if (np.abs(k0 - np.cos(ang) * win).max() > tol
                    or min(np.abs(k1 - np.sin(ang) * win).max(), np.abs(k1 + np.sin(ang) * win).max()) > tol):
                raise ValueError(f"{path}: Conv kernels {u0.name!r} / {u1.name!r} are not window x DFT basis")
            window, hop = win.astype(np.float32), s0
            # the power: Mul(re, re) / Pow(re, 2) for each, then their Add
            sq = []
            for u in (u0, u1):
                v = single_user(u.outputs[0])
                if not ((v.op == "Mul" and v.inputs[0] == v.inputs[1])
                        or (v.op == "Pow" and scalar(v.inputs[1], f"{path}: {v.name!r}") == 2.0)):
                    raise ValueError(f"{path}: node {v.name!r} ({v.op}) does not square the DFT output")
                sq.append(v.outputs[0])
            add = single_user(sq[0])
            if add.op != "Add" or set(add.inputs) != set(sq):
                raise ValueError(f"{path}: node {add.name!r} ({add.op}) does not add the squared re / im parts")
            x, stage = add.outputs[0], "power"
            continue
        node = single_user(x)
        a = node.attrs
        where = f"{path}: node {node.name!r} ({node.op})"
        nxt = node.outputs[0]
        if node.op in _SHAPE_OPS or (node.op == "Cast" and int(a.get("to", 1)) == 1):
            pass
        elif stage == "input" and node.op in ("Mul", "Div") and any(i in inits for i in node.inputs):
            c = scalar(next(i for i in node.inputs if i in inits), where)
            if node.op == "Div" and node.inputs[1] not in inits:
                raise ValueError(f"{where}: a constant divided by the signal")
            in_scale *= c if node.op == "Mul" else 1.0 / c
        elif stage == "input" and node.op == "STFT":
            if int(a.get("onesided", 1)) != 1:
                raise ValueError(f"{where}: only the onesided STFT is supported")
            hop = int(scalar(node.inputs[1], where))
            if len(node.inputs) < 3 or node.inputs[2] not in inits:
                raise ValueError(f"{where}: the STFT window must be a constant input")
            window = np.asarray(inits[node.inputs[2]], np.float32).reshape(-1)
            if len(node.inputs) > 3 and node.inputs[3] and int(scalar(node.inputs[3], where)) != window.size:
                raise ValueError(f"{where}: frame_length differs from the window length")
            # |X|^2: Pow(X, 2) then ReduceSum over the re / im axis
            v = single_user(nxt)
            if not ((v.op == "Pow" and scalar(v.inputs[1], f"{path}: {v.name!r}") == 2.0)
                    or (v.op == "Mul" and v.inputs[0] == v.inputs[1])):
                raise ValueError(f"{path}: node {v.name!r} ({v.op}) does not square the STFT output")
            r = single_user(v.outputs[0])
            axes = r.attrs.get("axes") or (inits[r.inputs[1]].tolist() if len(r.inputs) > 1 and r.inputs[1] else None)
            if r.op != "ReduceSum" or list(axes or []) not in ([-1], [3]) or int(r.attrs.get("keepdims", 1)):
                raise ValueError(f"{path}: node {r.name!r} ({r.op}) does not sum the re / im axis of the STFT")
            nxt, stage = r.outputs[0], "power"
        elif stage == "power" and node.op == "MatMul":
            if node.inputs[1] in inits:
                fb = np.asarray(inits[node.inputs[1]], np.float32)
            elif node.inputs[0] in inits:
                fb = np.asarray(inits[node.inputs[0]], np.float32).T
            else:
                raise ValueError(f"{where}: the filterbank must be a constant operand")
            if fb.ndim != 2 or window is None or fb.shape[0] != window.size // 2 + 1:
                raise ValueError(f"{where}: filterbank of shape {fb.shape} for a {None if window is None else window.size}-point DFT")
            fbank, stage = fb, "mel"
        elif stage == "mel" and node.op in ("Clip", "Max"):
            if node.op == "Clip":
                lo = a.get("min")
                if lo is None:
                    lo = scalar(node.inputs[1], where) if len(node.inputs) > 1 and node.inputs[1] else None
                if lo is None or (len(node.inputs) > 2 and node.inputs[2]) or "max" in a:
                    raise ValueError(f"{where}: only a lower clamp is supported")
                floor = float(lo)
            else:
                other = [i for i in node.inputs if i != x]
                if len(other) != 1:
                    raise ValueError(f"{where}: Max of more than the spectrum and one constant")
                floor = scalar(other[0], where)
            stage = "floored"
        elif stage in ("mel", "floored") and node.op == "Log":
            if floor is None:
                raise ValueError(f"{where}: log of an unclamped mel power (no floor) is not supported")
            stage = "log"
        elif stage == "log" and node.op in ("Mul", "Div", "Add", "Sub") and len([i for i in node.inputs if i in inits]) == 1:
            ci = next(i for i in node.inputs if i in inits)
            c = scalar(ci, where)
            if node.op == "Mul":
                mult, offset = mult * c, offset * c
            elif node.op == "Div":
                if node.inputs[1] != ci:
                    raise ValueError(f"{where}: a constant divided by the log-mel")
                mult, offset = mult / c, offset / c
            elif node.op == "Add":
                offset += c
            elif node.inputs[1] == ci:
                offset -= c
            else:
                raise ValueError(f"{where}: a constant minus the log-mel")
        else:
            raise ValueError(f"{where}: not supported at the {stage!r} stage of a mel front end")
        x = nxt
    if stage != "log":
        raise ValueError(f"{path}: the graph ends at the {stage!r} stage (expected a log-mel output)")
    # mult * ln(v) = (mult * ln 10 / 10) * 10 log10(v)
    return MelParams(window, fbank, hop=hop, log_floor=floor, scale=mult * math.log(10.0) / 10.0, offset=offset,
                     in_scale=in_scale, source=path)


class MelSpectrogramModel:
    """Compute the log-mel spectrogram of int16-range audio (spectrogram.py:11-32).

    ``device_id`` picks the HIP device (None = the current one); there is no
    CPU execution provider: without a GPU the call raises HBKUnavailable.
    """

    def __init__(self, device_id: Optional[int] = None, load: bool = False) -> None:
        self.device_id = device_id
        self.loaded = False
        if load:
            self.load()

    @property
    def device(self) -> torch.device:
        return _native.require_device(self.device_id)

    def load(self) -> None:
        """The reference loads its pretrained graph (onnx_util.py:63-81): here the
        graph's parameters (current_mel_params: the reference's file from
        pretrained_dir() when present, else H0) become a device plan."""
        default_mel_plan(self.device, 1.0)
        self.loaded = True

    def unload(self) -> None:
        self.loaded = False

    def __call__(self, audio: np.ndarray[Any, Any]) -> np.ndarray[Any, Any]:
        assert isinstance(audio, np.ndarray)
        if audio.ndim == 1:
            audio = audio[np.newaxis, :]
        assert audio.ndim == 2, f"Audio must be a 1D or 2D array, got {audio.ndim}D"
        dev = self.device
        plan = default_mel_plan(dev, 1.0)  # input already in int16 range
        x = torch.from_numpy(np.ascontiguousarray(audio, dtype=np.float32)).to(dev)
        out = plan(x)
        return np.squeeze(out.cpu().numpy())


GLOBAL_MEL_MODELS: Dict[Optional[int], MelSpectrogramModel] = {}


def get_mel_spectrogram_model(device_id: Optional[int] = None) -> MelSpectrogramModel:
    if device_id not in GLOBAL_MEL_MODELS:
        GLOBAL_MEL_MODELS[device_id] = MelSpectrogramModel(device_id=device_id, load=True)
    return GLOBAL_MEL_MODELS[device_id]
