"""Drop-in for heybuddy.embeddings (reference src/python/heybuddy/embeddings.py).

Same classes and signatures as the reference — ``SpeechEmbeddingModel``,
``SpeechEmbeddings`` (``audio_to_spectrograms``, ``spectrograms_to_embeddings``,
``__call__``) and ``get_speech_embeddings`` — with every numeric op on the
MI355X through libhbk.so:

* ``__call__`` (embeddings.py:153-234) computes each UNIQUE mel frame of a
  clip once (the reference recomputes 4 x 105 = 420 frames for 141 unique
  ones, embeddings.py:190) and each embedding window's shared conv prefix once
  per clip (14 of the 16 windows are unique and they overlap), then cuts the
  reference's 16 windows in its slot order (slot 4 w + q <- frame 12 w + 8 q).
  Results equal the reference's per-window evaluation (see tests/).
* ``featurize`` is the device-resident form of ``__call__`` (torch tensors in
  and out, nothing copied to the host) used by the feature generator and the
  benchmark.
"""
from __future__ import annotations

import os
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from heybuddy import _native
from heybuddy.embedding_graph import Graph, from_onnx, se20_graph
from heybuddy.kernels import EmbedPlan, default_embed_precision, embed_clips, embed_windows, mel_frames
from heybuddy.spectrogram import HOP, MelSpectrogramModel, N_FFT, default_mel_plan, find_pretrained
from heybuddy.util import audio_to_bct_tensor, logger

__all__ = ["SpeechEmbeddingModel", "SpeechEmbeddings", "get_speech_embeddings", "default_graph",
           "set_default_graph", "REFERENCE_EMBED_SHA256"]

_GRAPH: Optional[Graph] = None


REFERENCE_EMBED_FILE = "speech-embedding.onnx"  # embeddings.py:29
REFERENCE_EMBED_SHA256 = "70d164290c1d095d1d4ee149bc5e00543250a7316b59f31d056cff7bd3075c1f"  # embeddings.py:30


def default_graph() -> Graph:
    """The speech-embedding graph. The reference downloads an ONNX file
    (embeddings.py:29-30); nothing is downloaded here. If that file -- the
    reference's sha256 -- is in the pretrained directory
    (``heybuddy.spectrogram.pretrained_dir()``), it is imported
    (``embedding_graph.from_onnx``); a graph registered with
    ``set_default_graph`` wins; otherwise the seeded SE20 stand-in.

    The stand-in has the reference graph's shapes and cost but seeded random
    weights: its embeddings are NOT those of the reference's speech-embedding
    model, so classifiers trained by the reference (e.g. the shipped
    ``src/js/models/*.onnx`` heads) score meaningless values on them. A
    warning says so once per process."""
    global _GRAPH
    if _GRAPH is None:
        path = find_pretrained(REFERENCE_EMBED_FILE, REFERENCE_EMBED_SHA256)
        if path is not None:
            _GRAPH = from_onnx(path)
            logger.info(f"heybuddy: speech-embedding graph imported from {path}")
            return _GRAPH
        seed = int(os.environ.get("HEYBUDDY_EMBEDDING_SEED", "1234"))
        _GRAPH = se20_graph(seed)
        logger.warning(
            "heybuddy: no speech-embedding weights registered (set_default_graph); using the seeded SE20 "
            "stand-in graph. Its embeddings are not reference-compatible: performance and pipeline "
            "behaviour match, model outputs do not.")
    return _GRAPH


def set_default_graph(graph: Optional[Graph]) -> None:
    """Use ``graph`` (e.g. ``embedding_graph.from_onnx(path)``) for every later
    call; None: back to the default (the pretrained file or SE20)."""
    global _GRAPH
    _GRAPH = graph
    _EMBED_PLANS.clear()


_EMBED_PLANS: Dict[Tuple[int, Tuple[int, ...], int, str], EmbedPlan] = {}


def embed_plan(device: torch.device, starts: Sequence[int], graph: Optional[Graph] = None,
               precision: Optional[str] = None) -> EmbedPlan:
    graph = default_graph() if graph is None else graph
    precision = default_embed_precision() if precision is None else precision
    key = (device.index, tuple(starts), id(graph), precision)
    if key not in _EMBED_PLANS:
        _EMBED_PLANS[key] = EmbedPlan(graph, starts=tuple(starts), device=device, precision=precision)
    return _EMBED_PLANS[key]


class SpeechEmbeddingModel:
    """Compute speech embeddings from spectrograms (embeddings.py:23-42)."""

    def __init__(self, device_id: Optional[int] = None, load: bool = False,
                 graph: Optional[Graph] = None) -> None:
        self.device_id = device_id
        self.graph = graph
        self.loaded = False
        if load:
            self.load()

    @property
    def device(self) -> torch.device:
        return _native.require_device(self.device_id)

    def plan(self, starts: Sequence[int] = (0,), precision: Optional[str] = None) -> EmbedPlan:
        return embed_plan(self.device, starts, self.graph, precision)

    def load(self) -> None:
        self.plan()
        self.loaded = True

    def unload(self) -> None:
        self.loaded = False

    def __call__(self, spectrograms: np.ndarray[Any, Any]) -> np.ndarray[Any, Any]:
        x = torch.as_tensor(np.ascontiguousarray(spectrograms, dtype=np.float32), device=self.device)
        x = x.reshape(x.shape[0], x.shape[1], x.shape[2])
        out = range_checked(lambda prec: embed_windows(x, self.plan(precision=prec)),
                            lambda: [self.plan()])
        return out.reshape(out.shape[0], 1, 1, -1).cpu().numpy().squeeze()


def range_checked(run: Callable[[Optional[str]], Any], plans: Callable[[], List[EmbedPlan]]) -> Any:
    """run(None) on the default plans; if a split-f16 plan's range guard
    tripped (an activation reached fp16's 65504, include/hbk.h
    hbk_embed_range_status), warn and return run('exact') instead. Waits for
    the device: for the host-returning entry points only."""
    out = run(None)
    tripped = [p.range_tripped() for p in plans() if p.precision == "split"]
    if any(tripped):
        logger.warning("speech embedding: an activation left the split-f16 range (|x| >= 65504); "
                       "recomputing this call in exact f32")
        out = run("exact")
    return out


class SpeechEmbeddings:
    """A class to compute embeddings from audio (embeddings.py:44-234)."""

    def __init__(self, device_id: Optional[int] = None, load: bool = False) -> None:
        self.device_id = device_id
        self.spectrogram = MelSpectrogramModel(device_id=device_id, load=load)
        self.embeddings = SpeechEmbeddingModel(device_id=device_id, load=load)

    @property
    def device(self) -> torch.device:
        return _native.require_device(self.device_id)

    # --- reference building blocks (kept for API parity) -------------------
    def audio_to_spectrograms(self, audio: torch.Tensor, batch_size: int = 128, mel_bins: int = 32,
                              on_progress: Optional[Callable[[int, int], None]] = None
                              ) -> np.ndarray[Any, Any]:
        """[b, t] int16-range audio -> [b, ceil(t/160 - 3), mel_bins] (embeddings.py:56-84)."""
        b, t = audio.shape
        n_frames = int(np.ceil(t / 160 - 3))
        dev = self.device
        x = torch.as_tensor(audio, device=dev).to(torch.float32)
        mel = mel_frames(x.contiguous(), default_mel_plan(dev, 1.0))
        if mel.shape[1] != n_frames or mel.shape[2] != mel_bins:
            raise ValueError(f"could not broadcast input array from shape {tuple(mel.shape)} "
                             f"into shape ({b},{n_frames},{mel_bins})")
        if on_progress is not None:
            on_progress(b * n_frames, b * n_frames)
        return mel.cpu().numpy()

    def spectrograms_to_embeddings(self, spectrograms: np.ndarray[Any, Any], batch_size: int = 128,
                                   embedding_dim: int = 96, window_size: int = 76,
                                   window_stride: int = 8,
                                   on_progress: Optional[Callable[[int, int], None]] = None
                                   ) -> np.ndarray[Any, Any]:
        """[b, t, m] -> [b, (t - window_size)//stride + 1, embedding_dim] (embeddings.py:86-151)."""
        b, t, m = spectrograms.shape
        assert t >= window_size, f"Time dimension {t} must be at least {window_size}"
        n = (t - window_size) // window_stride + 1
        x = torch.as_tensor(np.ascontiguousarray(spectrograms, dtype=np.float32), device=self.device)
        wins = x.unfold(1, window_size, window_stride)[:, :n]        # [b, n, m, ws]
        wins = wins.permute(0, 1, 3, 2).reshape(b * n, window_size, m)
        out = range_checked(lambda prec: embed_windows(wins, self.embeddings.plan(precision=prec)),
                            lambda: [self.embeddings.plan()])
        if on_progress is not None:
            on_progress(b * n, b * n)
        return out.reshape(b, n, embedding_dim).cpu().numpy()

    # --- device-resident hot path -----------------------------------------
    @staticmethod
    def window_plan(t: int, audio_window_size: int = 17280, audio_window_stride: int = 1920,
                    window_size: int = 76, window_stride: int = 8) -> Tuple[List[int], int, int]:
        """Global start frame of every embedding window (slot order), frames per
        audio window, and the unique frames the clip needs."""
        if audio_window_stride % HOP:
            raise ValueError("audio_window_stride must be a multiple of the 160-sample hop")
        n_aw = len(range(0, t - audio_window_size + 1, audio_window_stride))
        f_aw = (audio_window_size - N_FFT) // HOP + 1
        q = (f_aw - window_size) // window_stride + 1
        step = audio_window_stride // HOP
        starts = [step * w + window_stride * j for w in range(n_aw) for j in range(q)]
        return starts, f_aw, (n_aw - 1) * step + f_aw if n_aw else 0

    def featurize(self, audio: torch.Tensor, audio_window_size: int = 17280,
                  audio_window_stride: int = 1920, window_size: int = 76, window_stride: int = 8,
                  in_scale: float = 32767.0, remove_nan: bool = True,
                  return_frames: bool = False, out: Optional[torch.Tensor] = None,
                  check_range: bool = False):
        """audio [B, T] float in [-1, 1] on the device -> embeddings [B, n, 96]
        (and the unique mel frames [B, F, 32] if ``return_frames``); ``out``:
        an optional [B, n, 96] f32 destination (kept when no NaN row needs
        replacing). ``check_range``: wait for the device and recompute in exact
        f32 if a split-f16 kernel saw |x| >= 65504 (range_checked)."""
        dev = audio.device
        b, t = audio.shape
        starts, f_aw, f_total = self.window_plan(t, audio_window_size, audio_window_stride,
                                                 window_size, window_stride)
        if not starts:
            raise ValueError("need at least one array to concatenate")
        mplan = default_mel_plan(dev, in_scale)
        frames = mel_frames(audio, mplan, f_total)
        groups = [starts[s0:s0 + 32] for s0 in range(0, len(starts), 32)]  # hbk plans take <= 32 windows

        def run(prec: Optional[str]) -> torch.Tensor:
            if len(groups) == 1:  # one plan covers every window: write straight into the output
                off = min(starts)
                plan = embed_plan(dev, [s - off for s in starts], precision=prec)
                return embed_clips(frames[:, off:off + plan.seq_frames], plan, out=out)
            emb = out if out is not None else torch.empty((b, len(starts), 96), dtype=torch.float32, device=dev)
            for s0, st in zip(range(0, len(starts), 32), groups):
                off = min(st)
                plan = embed_plan(dev, [s - off for s in st], precision=prec)
                emb[:, s0:s0 + len(st)] = embed_clips(frames[:, off:off + plan.seq_frames], plan)
            return emb

        if check_range:
            emb = range_checked(run, lambda: [embed_plan(dev, [s - min(st) for s in st]) for st in groups])
        else:
            emb = run(None)
        if remove_nan:
            emb = _replace_nan_rows(emb)
        return (emb, frames) if return_frames else emb

    def __call__(self, audio: Any, spectrogram_batch_size: int = 32, mel_bins: int = 32,
                 embedding_batch_size: int = 32, embedding_dim: int = 96, window_size: int = 76,
                 window_stride: int = 8, audio_window_size: int = 17280,
                 audio_window_stride: int = 1920,
                 on_spectrogram_progress: Optional[Callable[[int, int], None]] = None,
                 on_embedding_progress: Optional[Callable[[int, int], None]] = None,
                 remove_nan: bool = True, return_spectrograms: bool = False):
        audio_tensor, _ = audio_to_bct_tensor(audio, sample_rate=16000)
        dev = self.device
        x = audio_tensor.to(dev)
        if x.shape[1] > 1 or x.dtype != torch.float32:
            # reference order: scale to int16 range, then channel mean (embeddings.py:182-184)
            x = (x * 32767.0).mean(dim=1).to(torch.float32)
            scale = 1.0
        else:
            x = x[:, 0, :]
            scale = 32767.0
        if mel_bins != 32 or embedding_dim != 96:
            raise ValueError("the MI355X featurizer is built for 32 mel bins and 96-d embeddings")
        emb, frames = self.featurize(x.contiguous(), audio_window_size, audio_window_stride,
                                     window_size, window_stride, in_scale=scale,
                                     remove_nan=False, return_frames=True, check_range=True)
        b, n = emb.shape[0], emb.shape[1]
        if on_spectrogram_progress is not None:
            on_spectrogram_progress(b, b)
        if on_embedding_progress is not None:
            on_embedding_progress(b * n, b * n)
        embeddings = emb.cpu().numpy()
        if remove_nan:
            embeddings = _replace_nan_rows_host(embeddings)
            if embeddings is None:
                return np.zeros(emb.shape, dtype=np.float32)
        if return_spectrograms:
            starts, f_aw, _ = self.window_plan(x.shape[1], audio_window_size, audio_window_stride,
                                               window_size, window_stride)
            step = audio_window_stride // HOP
            n_aw = len(range(0, x.shape[1] - audio_window_size + 1, audio_window_stride))
            idx = torch.cat([torch.arange(f_aw) + step * w for w in range(n_aw)]).to(dev)
            spect = frames.index_select(1, idx)
            t = spect.shape[1]
            truncated_t = t - ((t - window_size) % window_stride)
            return embeddings, spect[:, :truncated_t].cpu().numpy()
        return embeddings


def _replace_nan_rows(emb: torch.Tensor) -> torch.Tensor:
    """Device form of the reference's NaN replacement (embeddings.py:213-227)."""
    bad = torch.isnan(emb).flatten(1).any(dim=1)
    if not bool(bad.any()):
        return emb
    host = _replace_nan_rows_host(emb.cpu().numpy())
    if host is None:
        return torch.zeros_like(emb)
    return torch.from_numpy(host).to(emb.device)


def replace_nan_rows_device(emb: torch.Tensor, out: torch.Tensor,
                            generator: Optional[torch.Generator] = None, zero_row: bool = False) -> torch.Tensor:
    """The NaN replacement of embeddings.py:213-227 with no host
    synchronisation, for pipelined featurization: every clip (row of emb
    [n, ...]) holding a NaN takes the embeddings of a uniformly drawn NaN-free
    clip (device RNG in place of np.random.choice), all zeros when every clip
    is NaN; the result is gathered into out (same shape, not emb). The
    reference's warning needs the count on the host and is not emitted here
    (_replace_nan_rows is the logging form). zero_row=True: emb carries one
    extra row (n + 1 rows for out's n) that the CALLER keeps all zero; the
    all-NaN case then gathers it instead of a masked fill over the whole output
    (one pass less)."""
    n = out.shape[0]
    ext = bool(zero_row)
    if emb.shape[0] != n + (1 if ext else 0):
        raise ValueError("emb must have out's rows (plus the zero row when zero_row=True)")
    rows = emb.reshape(emb.shape[0], -1)
    bad = rows[:n].amax(dim=1).isnan()  # amax propagates NaN: one reduction pass, no bool plane
    order = torch.argsort(bad.to(torch.uint8), stable=True)  # NaN-free clips first
    n_good = n - bad.sum()
    r = (torch.rand(n, device=emb.device, generator=generator) * n_good).long().clamp_(max=n - 1)
    pick = order[r]
    if ext:
        pick = torch.where(n_good > 0, pick, torch.full_like(pick, n))
    src = torch.where(bad, pick, torch.arange(n, device=emb.device))
    torch.index_select(rows, 0, src, out=out.view(n, -1))
    if ext:
        return out
    return out.masked_fill_((n_good == 0).reshape([1] * out.dim()), 0.0)


def _replace_nan_rows_host(embeddings: np.ndarray) -> Optional[np.ndarray]:
    """Any clip with a NaN gets a random non-NaN clip's embeddings
    (np.random.choice, as embeddings.py:227); None if every clip is NaN."""
    bad = [i for i, e in enumerate(embeddings) if np.isnan(e).any()]
    if not bad:
        return embeddings
    logger.warning(f"Replacing {len(bad)} NaN embeddings with random embeddings.")
    keep = np.setdiff1d(np.arange(len(embeddings)), bad)
    if keep.size == 0:
        logger.warning("All embeddings are NaN, returning zero embeddings.")
        return None
    for i in bad:
        embeddings[i] = embeddings[np.random.choice(keep)]
    return embeddings


GLOBAL_EMBEDDINGS: Dict[Optional[int], SpeechEmbeddings] = {}


def get_speech_embeddings(device_id: Optional[int] = None) -> SpeechEmbeddings:
    """Cached SpeechEmbeddings per device (embeddings.py:236-243)."""
    if device_id not in GLOBAL_EMBEDDINGS:
        GLOBAL_EMBEDDINGS[device_id] = SpeechEmbeddings(device_id=device_id)
    return GLOBAL_EMBEDDINGS[device_id]
