"""Featurizer orchestration oracle (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Restates SpeechEmbeddings.__call__ (reference src/python/heybuddy/embeddings.py
:153-234) with its cost structure: for every 17,280-sample audio window at
stride 1,920 (:190) the mel graph is run on the window (:56-84, batch
``spectrogram_batch_size``), then every 76-frame window at stride 8 of that
window's 105 frames goes through the embedding graph (:86-151, batch
``embedding_batch_size``); results are concatenated along time (:209), NaN
clips replaced (:213-227) and the spectrograms truncated (:229-232).
Pinned against the reference itself (tests/golden/featurizer_*.npz).
Also the CPU baseline of bench.py (``cpu_featurize``).
"""
from __future__ import annotations

import numpy as np

from oracle import embed as oemb
from oracle import mel as omel


def featurize(audio: np.ndarray, graph, spectrogram_batch_size: int = 32,
              embedding_batch_size: int = 32, window_size: int = 76, window_stride: int = 8,
              audio_window_size: int = 17280, audio_window_stride: int = 1920,
              return_spectrograms: bool = False, mel_fn=None, embed_fn=None):
    """audio [B, T] float32 in [-1, 1] -> embeddings [B, n, 96] (numpy)."""
    mel_fn = mel_fn or omel.mel_spectrogram_model
    embed_fn = embed_fn or (lambda w: oemb.speech_embedding_model(graph, w))
    audio = np.asarray(audio, dtype=np.float32) * np.float32(32767.0)
    b, t = audio.shape
    embs, specs = [], []
    for i in range(0, t - audio_window_size + 1, audio_window_stride):
        win = audio[:, i:i + audio_window_size]
        nf = int(np.ceil(audio_window_size / 160 - 3))
        spec = np.empty((b, nf, 32), dtype=np.float32)
        for s in range(0, max(b, spectrogram_batch_size), spectrogram_batch_size):
            if s >= b:
                break
            spec[s:s + spectrogram_batch_size] = np.asarray(mel_fn(win[s:s + spectrogram_batch_size])
                                                            ).reshape(-1, nf, 32)
        n = (nf - window_size) // window_stride + 1
        out = np.empty((b, n, 96), dtype=np.float32)
        jobs = [(c, j) for c in range(b) for j in range(0, nf, window_stride) if j + window_size <= nf]
        for s in range(0, len(jobs), embedding_batch_size):
            chunk = jobs[s:s + embedding_batch_size]
            w = np.stack([spec[c, j:j + window_size, :, None] for c, j in chunk])
            r = np.asarray(embed_fn(w)).reshape(len(chunk), -1)
            for x, (c, j) in enumerate(chunk):
                out[c, j // window_stride] = r[x]
        embs.append(out)
        specs.append(spec)
    emb = np.concatenate(embs, axis=1)
    if return_spectrograms:
        spec = np.concatenate(specs, axis=1)
        tt = spec.shape[1]
        return emb, spec[:, :tt - ((tt - window_size) % window_stride)]
    return emb


def cpu_featurize(audio: np.ndarray, graph, batch: int = 64, threads: int | None = None):
    """Timed CPU baseline: the reference's cost structure (4 audio windows x 105
    mel frames, 16 embedding windows per clip, batch 64 = the CPU autoconfigure,
    features.py:203-208) with an fp32 mel (numpy rfft) and an fp32 conv graph
    (torch CPU conv2d, NHWC->NCHW) — what ONNX Runtime's CPU provider runs."""
    import torch
    if threads:
        torch.set_num_threads(threads)
    layers = _torch_layers(graph)

    def mel_fn(x):
        x = np.asarray(x, dtype=np.float32)
        nf = (x.shape[1] - 512) // 160 + 1
        idx = np.arange(nf)[:, None] * 160 + np.arange(512)[None, :]
        fr = x[:, idx] * omel.hann_window()
        spec = np.fft.rfft(fr, axis=-1)
        p = (spec.real ** 2 + spec.imag ** 2).astype(np.float32)
        mel = p @ omel.mel_fbank()
        return 10.0 * np.log10(np.maximum(mel, 1e-10)) / 10.0 + 2.0

    def embed_fn(w):
        with torch.no_grad():
            h = torch.from_numpy(np.ascontiguousarray(w[..., 0])).unsqueeze(1)  # [n,1,76,32]
            for kind, a, b in layers:
                if kind == "conv":
                    h = torch.nn.functional.conv2d(h, a, b)
                elif kind == "lrelu":
                    h = torch.nn.functional.leaky_relu(h, a)
                else:
                    h = torch.nn.functional.max_pool2d(h, a)
            return h.reshape(h.shape[0], -1).numpy()

    return featurize(audio, graph, spectrogram_batch_size=batch, embedding_batch_size=batch,
                     mel_fn=mel_fn, embed_fn=embed_fn)


def _torch_layers(graph):
    import torch
    from heybuddy.embedding_graph import Conv
    layers = []
    for op in graph.ops:
        if isinstance(op, Conv):
            w = torch.from_numpy(np.ascontiguousarray(op.weight.transpose(3, 2, 0, 1)))  # OIHW
            layers.append(("conv", w, torch.from_numpy(op.bias)))
            if op.act == "leaky_relu":
                layers.append(("lrelu", op.alpha, None))
        else:
            layers.append(("pool", (op.ph, op.pw), None))
    return layers


def _mel_batch(x: np.ndarray) -> np.ndarray:
    """fp32 mel graph of a batch of 17,280-sample windows -> [b, 105, 32]
    (the ONNX mel graph's work, spectrogram.py:23-32, with the H0 parameters)."""
    x = np.asarray(x, dtype=np.float32) * np.float32(32767.0)
    nf = (x.shape[1] - 512) // 160 + 1
    idx = np.arange(nf)[:, None] * 160 + np.arange(512)[None, :]
    fr = x[:, idx] * omel.hann_window().astype(np.float32)
    spec = np.fft.rfft(fr, axis=-1)
    p = (spec.real ** 2 + spec.imag ** 2).astype(np.float32)
    mel = p @ omel.mel_fbank().astype(np.float32)
    return 10.0 * np.log10(np.maximum(mel, 1e-10)) / 10.0 + 2.0


def cpu_mel_windows(audio: np.ndarray, batch: int = 64, threads: int = 1) -> np.ndarray:
    """configs[0]'s CPU path: SpeechEmbeddings.audio_to_spectrograms' cost
    structure (embeddings.py:56-84, :190): every clip's 4 audio windows of
    17,280 samples (stride 1,920) through the mel graph in batches of ``batch``
    windows (the CPU autoconfigure, features.py:203-208) -> [n, 420, 32].
    ``threads`` workers take whole batches (numpy's FFT releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    audio = np.asarray(audio, dtype=np.float32)
    n = audio.shape[0]
    wins = np.stack([audio[:, s:s + 17280] for s in range(0, 5761, 1920)], axis=1).reshape(n * 4, 17280)
    chunks = [wins[i:i + batch] for i in range(0, wins.shape[0], batch)]
    if threads > 1:
        from threadpoolctl import threadpool_limits
        with threadpool_limits(limits=1), ThreadPoolExecutor(threads) as ex:
            outs = list(ex.map(_mel_batch, chunks))
    else:
        outs = [_mel_batch(c) for c in chunks]
    return np.concatenate(outs).reshape(n, 4 * 105, 32)
