"""Synthetic inputs that stand in for TTS speech, the MIT IR survey and the
background-noise datasets (none are available offline). SURVEY.md §8d.

Generated with torch on the target device (input preparation, outside any
timed region), seeded per (config, rank) so every rank's shard is fixed.
"""
from __future__ import annotations

import math

import torch

SAMPLE_RATE = 16000
CLIP_SAMPLES = 24000  # 1.5 s synthetic clips; the featurizer reads [0, 23040)


def seed_for(config: int, rank: int = 0) -> int:
    return 20251015 + 1000 * config + rank


def synthetic_clips(n: int, length: int = CLIP_SAMPLES, seed: int = 0,
                    device: torch.device | str = "cpu", chunk: int = 4096,
                    out: torch.Tensor | None = None) -> torch.Tensor:
    """[n, length] f32 clips in [-1, 1]: 0.25 * sum of 6 sinusoids (80-4000 Hz)
    under a Hann burst of 0.3-1.0 s at a random offset, + 0.01 N(0, 1)."""
    device = torch.device(device)
    g = torch.Generator(device=device).manual_seed(seed)
    if out is None:
        out = torch.empty((n, length), dtype=torch.float32, device=device)
    t = torch.arange(length, device=device, dtype=torch.float32) / SAMPLE_RATE
    dur_total = length / SAMPLE_RATE
    for s in range(0, n, chunk):
        b = min(chunk, n - s)
        f = torch.rand((b, 6, 1), generator=g, device=device) * (4000.0 - 80.0) + 80.0
        ph = torch.rand((b, 6, 1), generator=g, device=device) * (2 * math.pi)
        dur = torch.rand((b, 1), generator=g, device=device) * 0.7 + 0.3
        off = torch.rand((b, 1), generator=g, device=device) * (dur_total - dur)
        u = ((t[None, :] - off) / dur).clamp(0.0, 1.0)
        env = 0.5 - 0.5 * torch.cos(2 * math.pi * u)
        tones = torch.sin(2 * math.pi * f * t[None, None, :] + ph).sum(dim=1)
        x = 0.25 * tones * env + 0.01 * torch.randn((b, length), generator=g, device=device)
        out[s:s + b] = x.clamp_(-1.0, 1.0)
    return out


def edge_clips(length: int = CLIP_SAMPLES, device: torch.device | str = "cpu") -> torch.Tensor:
    """All-zeros, DC 0.5, full-scale 440 Hz square, unit impulse."""
    t = torch.arange(length, dtype=torch.float64) / SAMPLE_RATE
    z = torch.zeros(length, dtype=torch.float64)
    dc = torch.full((length,), 0.5, dtype=torch.float64)
    sq = torch.sign(torch.sin(2 * math.pi * 440.0 * t))
    imp = torch.zeros(length, dtype=torch.float64)
    imp[length // 3] = 1.0
    return torch.stack([z, dc, sq, imp]).to(torch.float32).to(device)


def impulse_responses(n: int = 32, seed: int = 0, min_len: int = 4000, max_len: int = 16000,
                      device: torch.device | str = "cpu") -> list[torch.Tensor]:
    """Exponentially decaying noise IRs (RT60 0.2-1.0 s) with a direct-path
    spike at index U[0, 200]."""
    g = torch.Generator().manual_seed(seed)
    irs = []
    for _ in range(n):
        L = int(torch.randint(min_len, max_len + 1, (1,), generator=g))
        rt60 = float(torch.rand((1,), generator=g)) * 0.8 + 0.2
        tt = torch.arange(L, dtype=torch.float32) / SAMPLE_RATE
        ir = torch.randn((L,), generator=g) * torch.exp(-6.91 * tt / rt60) * 0.3
        d = int(torch.randint(0, 201, (1,), generator=g))
        ir[d] = 1.0
        irs.append(ir.to(device))
    return irs


def noise_bank(n: int = 64, seed: int = 0, device: torch.device | str = "cpu") -> list[torch.Tensor]:
    """3-10 s colored noise (1/f^beta, beta ~ U[-1, 2]), RMS-normalised to 0.1."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        L = int(torch.randint(3 * SAMPLE_RATE, 10 * SAMPLE_RATE + 1, (1,), generator=g))
        beta = float(torch.rand((1,), generator=g)) * 3.0 - 1.0
        spec = torch.fft.rfft(torch.randn((L,), generator=g, dtype=torch.float64))
        freqs = torch.fft.rfftfreq(L, d=1.0 / SAMPLE_RATE, dtype=torch.float64)
        freqs[0] = freqs[1]
        x = torch.fft.irfft(spec / freqs.pow(beta / 2.0), n=L)
        x = x / x.pow(2).mean().sqrt() * 0.1
        out.append(x.to(torch.float32).to(device))
    return out


def phrase_clips(phrase: str, n: int, length: int = CLIP_SAMPLES, seed: int = 0,
                 device: torch.device | str = "cpu") -> torch.Tensor:
    """[n, length] stand-ins for TTS renderings of one phrase: a sequence of
    4-7 tone "syllables" whose pitches and durations are fixed by the phrase
    text, rendered per clip with a random onset, tempo (0.85-1.15x), pitch
    shift (+-5%), gain and 0.01 N(0, 1) noise. Distinct phrases give distinct
    templates, so a classifier can learn one against synthetic_clips()."""
    import zlib
    device = torch.device(device)
    h = torch.Generator().manual_seed(zlib.crc32(phrase.encode("utf-8")))
    k = int(torch.randint(4, 8, (1,), generator=h))
    f0 = torch.rand((k,), generator=h) * 1500.0 + 200.0        # syllable pitch
    d0 = torch.rand((k,), generator=h) * 0.08 + 0.06           # syllable seconds
    g = torch.Generator(device=device).manual_seed(seed)
    t = torch.arange(length, device=device, dtype=torch.float32) / SAMPLE_RATE
    tempo = torch.rand((n, 1), generator=g, device=device) * 0.3 + 0.85
    shift = torch.rand((n, 1), generator=g, device=device) * 0.1 + 0.95
    total = float(d0.sum()) * 1.15
    onset = torch.rand((n, 1), generator=g, device=device) * max(length / SAMPLE_RATE - total - 0.05, 0.0)
    gain = torch.rand((n, 1), generator=g, device=device) * 0.3 + 0.2
    x = torch.zeros((n, length), device=device)
    start = onset.clone()
    for j in range(k):
        dur = float(d0[j]) * tempo
        u = ((t[None, :] - start) / dur)
        env = torch.where((u >= 0) & (u <= 1), 0.5 - 0.5 * torch.cos(2 * math.pi * u.clamp(0, 1)),
                          torch.zeros_like(u))
        f = float(f0[j]) * shift
        x += env * (torch.sin(2 * math.pi * f * t[None, :]) + 0.5 * torch.sin(4 * math.pi * f * t[None, :]))
        start = start + dur
    x = gain * x + 0.01 * torch.randn((n, length), generator=g, device=device)
    return x.clamp_(-1.0, 1.0)


def _syllables(phrase: str):
    """Pitch (Hz) and duration (s) of the tone "syllables" of a phrase template
    (fixed by the text: distinct phrases give distinct templates)."""
    import zlib
    h = torch.Generator().manual_seed(zlib.crc32(phrase.encode("utf-8")))
    k = int(torch.randint(4, 8, (1,), generator=h))
    f0 = torch.rand((k,), generator=h) * 1500.0 + 200.0
    d0 = torch.rand((k,), generator=h) * 0.08 + 0.06
    return f0, d0


def speech_clips(phrase: str, n: int, seed: int = 0, device: torch.device | str = "cpu",
                 adversarial: bool = False, num_phrases: int = 250, max_len: int = CLIP_SAMPLES,
                 chunk: int = 4096):
    """Stand-in for the Piper TTS generator (PiperSpeechGenerator, dataset/piper.py,
    out of scope offline): variable-length utterances as the reference's
    to_target_length receives them. Returns (clips [n, max_len] f32 with clip i
    valid in [0, lengths[i]) and zero after, lengths int32 numpy [n]).

    Positive clips render the phrase's template; adversarial clips render one
    of ``num_phrases`` other templates ("phrase#k"), per clip, with the same
    random tempo (0.85-1.15x), pitch shift (+-5 %), gain, 20-80 ms margins and
    0.01 N(0, 1) noise inside the utterance."""
    device = torch.device(device)
    g = torch.Generator(device=device).manual_seed(seed)
    gh = torch.Generator().manual_seed(seed + 1)
    names = [phrase] if not adversarial else [f"{phrase}#adv{k}" for k in range(num_phrases)]
    temps = [_syllables(s) for s in names]
    kmax = max(int(f.shape[0]) for f, _ in temps)
    F = torch.zeros((len(names), kmax))
    D = torch.zeros((len(names), kmax))
    for i, (f, d) in enumerate(temps):
        F[i, :f.shape[0]] = f
        D[i, :d.shape[0]] = d
    which = torch.randint(0, len(names), (n,), generator=gh)
    F, D = F[which].to(device), D[which].to(device)
    out = torch.zeros((n, max_len), dtype=torch.float32, device=device)
    lengths = torch.empty(n, dtype=torch.int32, device=device)
    t = torch.arange(max_len, device=device, dtype=torch.float32) / SAMPLE_RATE
    for s in range(0, n, chunk):
        b = min(chunk, n - s)
        f_all, d_all = F[s:s + b], D[s:s + b]
        tempo = torch.rand((b, 1), generator=g, device=device) * 0.3 + 0.85
        shift = torch.rand((b, 1), generator=g, device=device) * 0.1 + 0.95
        gain = torch.rand((b, 1), generator=g, device=device) * 0.3 + 0.2
        lead = torch.rand((b, 1), generator=g, device=device) * 0.06 + 0.02
        tail = torch.rand((b, 1), generator=g, device=device) * 0.06 + 0.02
        x = torch.zeros((b, max_len), device=device)
        start = lead.clone()
        for j in range(kmax):
            dur = d_all[:, j:j + 1] * tempo
            u = (t[None, :] - start) / dur.clamp_min(1e-6)
            on = (u >= 0) & (u <= 1) & (dur > 0)
            env = torch.where(on, 0.5 - 0.5 * torch.cos(2 * math.pi * u.clamp(0, 1)), torch.zeros_like(u))
            f = f_all[:, j:j + 1] * shift
            x += env * (torch.sin(2 * math.pi * f * t[None, :]) + 0.5 * torch.sin(4 * math.pi * f * t[None, :]))
            start = start + dur
        length = ((start + tail) * SAMPLE_RATE).floor().clamp(1, max_len)
        inside = torch.arange(max_len, device=device)[None, :] < length
        x = gain * x + 0.01 * torch.randn((b, max_len), generator=g, device=device)
        out[s:s + b] = torch.where(inside, x.clamp_(-1.0, 1.0), torch.zeros_like(x))
        lengths[s:s + b] = length[:, 0].to(torch.int32)
    return out, lengths.cpu().numpy()
