"""The headline workload (BASELINE configs[4], bench.py config 5) stage by stage
against the oracle: the `heybuddy train` hot path of the reference
(__main__.py:245-429 -> features.py:492-535 -> trainer.py:764-1007) on seeded
synthetic utterances.

  placement (to_target_length)   bit-exact vs the numpy restatement
  7-band EQ, tanh, pitch shift,  each stage's HIP output against the oracle
  band-stop, colored noise,      applied to the HIP output of the stage before
  gain + noise + reverb          (so an error is attributed to its stage), in
                                 the reference's order (augmented.py:79-121,
                                 :368-392); pitch shift first in the batch chain
  mel frames                     1e-4 vs oracle.mel on the augmented clips
  speech embedding               1e-4 (1 + |ref|) vs oracle.embed on the HIP mel
  NaN replacement                the device gather leaves finite rows alone
  3 fused train steps            B = 1,100 in the bench's composition (50 pos +
                                 50 adv of these clips + 1,000 f16 negatives),
                                 vs oracle.mlp forward / filter / BCE /
                                 backward / Adam on the same rows

Every augmentation runs at p = 1 here (the bench draws the reference's
probabilities). PARITY UNPINNED where the oracle restates a third-party
package (see oracle/augment.py); the classifier oracle is pinned by
tests/golden/classifier*.npz.
"""
import numpy as np
import pytest
import torch

from oracle import augment as oaug
from oracle import embed as oemb
from oracle import mel as omel
from oracle import mlp as omlp

pytestmark = pytest.mark.gpu

T = 23040
N = 300                  # 150 positive + 150 adversarial utterances
N_FRAMES = 141


def _close_aug(out, ref, inp=None):
    """max |err| <= 2e-5 max |ref| and rms(err) <= 2e-6 rms(ref); with inp, the
    scale is the larger of the output's and the input's (band-stop: y = x - bp(x)
    loses most of a clip whose energy sits in the stop band, while the
    convolution's rounding stays relative to x)."""
    err = np.abs(out - ref)
    mx, rms = np.abs(ref).max(), np.sqrt((ref ** 2).mean())
    if inp is not None:
        mx, rms = max(mx, np.abs(inp).max()), max(rms, np.sqrt((inp ** 2).mean()))
    r_max = err.max() / mx
    r_rms = np.sqrt((err ** 2).mean()) / rms
    return r_max <= 2e-5 and r_rms <= 2e-6, f"max |diff| {err.max():.3e} ({r_max:.2e} of max |ref|), rms {r_rms:.2e}"


def _check_stage(name, out, ref, rows, inp=None):
    for i in rows:
        ok, worst = _close_aug(out[i], ref[i], None if inp is None else inp[i])
        assert ok, f"{name}: clip {i}: {worst}"


def test_headline_pipeline_stagewise():
    from heybuddy.dataset.augmented import bandstop_cutoffs, eq_coefficients, eq_parameters, target_length_offsets
    from heybuddy.embedding_graph import WINDOW_STARTS, se20_graph
    from heybuddy.embeddings import embed_plan, replace_nan_rows_device
    from heybuddy.kernels import (ReverbPlan, embed_clips, mel_frames, pitch_shift, place_clips, seven_band_eq,
                                  tanh_distortion)
    from heybuddy.spectrogram import default_mel_plan
    from heybuddy.synthetic import impulse_responses, noise_bank, speech_clips
    from heybuddy.trainer import WakeWordTrainer

    dev = torch.device("cuda", 0)
    np.random.seed(2024)
    torch.manual_seed(2024)  # the band-stop cutoffs come from torch's CPU generator
    pos, pos_len = speech_clips("hello world", N // 2, seed=11, device=dev)
    adv, adv_len = speech_clips("hello world", N - N // 2, seed=12, device=dev, adversarial=True)
    src = torch.cat([pos, adv])
    lens = np.concatenate([pos_len, adv_len]).astype(np.int32)
    src_h = src.cpu().numpy()
    rows = list(range(0, N, 23)) + [N - 1]

    # 1) placement: crop, or shift right by the drawn leading silence
    pre = target_length_offsets(lens, T)
    x = place_clips(src, torch.from_numpy(lens), torch.from_numpy(pre.astype(np.int32)), T)
    ref = np.zeros((N, T), np.float32)
    for i in range(N):
        L = min(int(lens[i]), T - int(pre[i]))
        ref[i, pre[i]:pre[i] + L] = src_h[i, :L]
    np.testing.assert_array_equal(x.cpu().numpy(), ref)

    # 2) per-clip chain: 7-band EQ, then tanh distortion (every clip)
    params = eq_parameters(N, 6.0)
    coef = eq_coefficients(params)
    x_in = x.cpu().numpy()
    x = seven_band_eq(x, torch.from_numpy(coef).to(dev))
    sos = np.concatenate([coef[..., :3], np.ones(coef.shape[:-1] + (1,)), coef[..., 3:]], axis=-1)
    _check_stage("eq", x.cpu().numpy(), oaug.seven_band_eq(x_in, sos), rows)
    amount = np.random.uniform(1e-4, 0.1, N).astype(np.float32)
    x_in = x.cpu().numpy()
    x = tanh_distortion(x, torch.from_numpy(amount).to(dev))
    _check_stage("tanh", x.cpu().numpy(), oaug.tanh_distortion(x_in, amount), rows)

    # 3) batch chain (augmented.py:93-121): pitch shift first, one fast shift per batch of 128
    #    (batch 0: 125/128, batch 1: 128/125, batch 2: unshifted), vs the float64 restatement at
    #    the pitch tests' bound (per clip L2 <= 1e-4 of the reference's, max <= 1e-3 of its peak)
    x_in = x.cpu().numpy()
    shifted = {}
    for (num, den), b in (((125, 128), 0), ((128, 125), 1)):
        sel = np.arange(b * 128, min(N, (b + 1) * 128), dtype=np.int32)
        x = pitch_shift(x, torch.from_numpy(sel), num, den, out=x)
        for i in rows:
            if sel[0] <= i <= sel[-1]:
                shifted[i] = (num, den)
    out_h = x.cpu().numpy()
    for i in rows:
        if i not in shifted:
            np.testing.assert_array_equal(out_h[i], x_in[i])
            continue
        r = oaug.pitch_shift(x_in[i:i + 1].astype(np.float64), *shifted[i])[0]
        l2 = np.sqrt(((out_h[i] - r) ** 2).sum()) / np.sqrt((r ** 2).sum())
        mx = np.abs(out_h[i] - r).max() / np.abs(r).max()
        assert l2 <= 1e-4 and mx <= 1e-3, f"pitch shift {shifted[i]}: clip {i}: L2 {l2:.2e}, max {mx:.2e}"
    assert len(shifted) >= 8

    #    then band-stop (one cutoff pair per batch of 128), colored noise, gain + noise + reverb
    plan = ReverbPlan(dev)
    lo_b, hi_b = bandstop_cutoffs(3)
    batch = np.arange(N) // 128
    lo, hi = lo_b[batch], hi_b[batch]
    x_in = x.cpu().numpy()
    x = plan.band_stop(x, torch.arange(N, dtype=torch.int32), torch.from_numpy(lo), torch.from_numpy(hi), out=x)
    _check_stage("band-stop", x.cpu().numpy(), oaug.band_stop(x_in, lo, hi), rows, inp=x_in)
    g = torch.Generator(device="cpu").manual_seed(5)
    white = torch.randn((N, 16000), generator=g)
    fd = np.random.uniform(-1.0, 2.0, N).astype(np.float32)
    csnr = np.random.uniform(10.0, 30.0, N).astype(np.float32)
    x_in = x.cpu().numpy()
    x = plan.colored_noise(x, torch.from_numpy(fd), torch.from_numpy(csnr), white=white.to(dev), out=x)
    cref = oaug.colored_noise(x_in.astype(np.float64), white.numpy().astype(np.float64), fd, csnr)
    _check_stage("colored noise", x.cpu().numpy(), cref, rows)
    noises = [t.numpy() for t in noise_bank(6, seed=31)]
    irs = [t.numpy() for t in impulse_responses(3, seed=32)]
    ring = np.concatenate(noises).astype(np.float32)
    noise_off = (np.arange(N) * 977) % (ring.size - T)
    snr = np.random.uniform(-10.0, 15.0, N)
    spec_idx = (np.arange(N) // 128 % len(irs)).astype(np.int32)
    gain = np.random.uniform(0.2, 1.5, N).astype(np.float32)
    H = plan.spectra(torch.stack([ReverbPlan.rotated_kernel(torch.from_numpy(ir), T) for ir in irs]).to(dev))
    x_in = x.cpu().numpy()
    x = plan.augment(x, torch.from_numpy(ring).to(dev), torch.from_numpy(noise_off), torch.from_numpy(snr), H,
                     torch.from_numpy(spec_idx), gain=torch.from_numpy(gain))
    out_h = x.cpu().numpy()
    for i in rows:
        nz = ring[noise_off[i]:noise_off[i] + T].astype(np.float64)[None]
        r = oaug.augment_batch(x_in[i:i + 1].astype(np.float64), nz, snr[i:i + 1], irs[spec_idx[i]],
                               gain=gain[i:i + 1].astype(np.float64))[0]
        ok, worst = _close_aug(out_h[i], r)
        assert ok, f"gain + noise + reverb: clip {i}: {worst}"

    # 4) mel frames of the augmented clips (the featurizer's x 32767 folded into the window)
    frames = mel_frames(x, default_mel_plan(dev, 32767.0), N_FRAMES)
    mel_ref, _, _ = omel.mel_frames(out_h[rows], N_FRAMES)
    np.testing.assert_allclose(frames.cpu().numpy()[rows], mel_ref, rtol=1e-4, atol=1e-4)

    # 5) speech embedding of the HIP mel frames, and the NaN replacement (no NaN rows: a copy)
    eplan = embed_plan(dev, WINDOW_STARTS)
    raw = embed_clips(frames, eplan)
    pool = torch.empty_like(raw)
    replace_nan_rows_device(raw, out=pool)
    assert torch.equal(pool, raw)
    sub = rows[:6]
    mel_h = frames.cpu().numpy()[sub]
    wins = np.stack([mel_h[:, s:s + 76] for s in WINDOW_STARTS], axis=1)
    eref = oemb.run_graph(se20_graph(), wins.reshape(-1, 76, 32)).reshape(len(sub), len(WINDOW_STARTS), -1)
    err = np.abs(raw.cpu().numpy()[sub] - eref)
    assert (err <= 1e-4 * (1.0 + np.abs(eref))).all(), err.max()

    # 6) three fused train steps on these embeddings in the bench's composition
    P, A, NEG = 50, 50, 1000
    S = 3
    gneg = torch.Generator(device=dev).manual_seed(7)
    neg = torch.randn((3000, 16, 96), generator=gneg, device=dev).half()
    rng = np.random.default_rng(8)
    idx = np.empty((S, P + A + NEG), np.int32)
    for s in range(S):
        idx[s, :P] = rng.permutation(N // 2)[:P]
        idx[s, P:P + A] = N // 2 + rng.permutation(N - N // 2)[:A]
        idx[s, P + A:] = -1 - rng.permutation(3000)[:NEG]
    y = np.concatenate([np.ones(P), np.zeros(A + NEG)]).astype(np.float32)
    lrs = [omlp.learning_rate(s, 1, 1, S) for s in range(S)]
    sched = torch.tensor([[lr, 1.0] for lr in lrs], dtype=torch.float32, device=dev)
    tr = WakeWordTrainer(checkpoint_dir="/tmp/hb_e2e_ck", device=dev)
    tr.model.dropout.p = 0.0
    params0 = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in tr.model.state_dict().items()}
    tr._reset_accumulation()
    tr.train_indexed(torch.from_numpy(idx).to(dev), torch.from_numpy(y).to(dev), sched, pool32=pool, pool16=neg,
                     steps_per_graph=S)
    torch.cuda.synchronize()
    # the oracle on the same rows (f16 negatives widened to f32), reference optimisation path
    pool_h = pool.cpu().numpy().reshape(N, -1).astype(np.float64)
    neg_h = neg.float().cpu().numpy().reshape(3000, -1).astype(np.float64)
    batches = []
    for s in range(S):
        xs = np.where((idx[s] >= 0)[:, None], pool_h[np.clip(idx[s], 0, None)], neg_h[np.clip(-1 - idx[s], 0, None)])
        batches.append((xs.reshape(-1, 16, 96), y.astype(np.int64)))
    p_ref, hist = omlp.train_epoch(params0, batches, num_steps=S, warmup_steps=1, hold_steps=1)
    assert all(hist["updated"]), hist["updated"]
    sd = tr.model.state_dict()
    diffs = np.concatenate([np.abs(sd[k].cpu().numpy() - p_ref[k]).ravel() for k in p_ref])
    moved = np.concatenate([np.abs(p_ref[k] - params0[k]).ravel() for k in p_ref])
    assert moved.max() > 1e-4  # the steps did update the classifier
    assert (diffs > 2e-4).mean() <= 5e-3, (diffs > 2e-4).mean()
    assert diffs.max() <= 2 * sum(lrs) + 1e-6, diffs.max()
