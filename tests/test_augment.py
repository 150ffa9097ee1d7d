"""Background-noise mix + IR reverb: oracle properties (CPU), HIP parity (GPU).

PARITY UNPINNED at the third-party boundary: torchaudio.add_noise and
speechbrain.reverberate are not installed and the reference holds no fixture
for them; oracle/augment.py restates their published algorithms. The CPU
tests check that restatement against size-independent properties (linearity,
circularity, the SNR definition, the rotation by argmax |ir|); the GPU tests
check the HIP kernel against it. Tolerance: fp32 FFT of length 11,520 vs fp64,
|diff| <= 2e-5 * max|ref| and RMS(diff) <= 2e-6 * RMS(ref).
"""
import numpy as np
import pytest
import torch

from oracle import augment as oaug

T = 23040


def _clips(n, seed=0):
    from heybuddy.synthetic import synthetic_clips
    return synthetic_clips(n, length=T, seed=seed).numpy().astype(np.float64)


def _bank(seed=1):
    from heybuddy.synthetic import impulse_responses, noise_bank
    return ([x.numpy() for x in noise_bank(6, seed=seed)],
            [x.numpy() for x in impulse_responses(4, seed=seed)])


def test_add_noise_hits_requested_snr():
    x = _clips(3)
    rng = np.random.default_rng(0)
    n = rng.standard_normal((3, T)) * 0.1
    snr = np.array([-10.0, 0.0, 15.0])
    y = oaug.add_noise(x, n, snr)
    scaled = y - x
    got = 10 * np.log10((x ** 2).sum(1) / (scaled ** 2).sum(1))
    np.testing.assert_allclose(got, snr, atol=1e-9)
    # zero-energy noise -> NaN, zero-energy clip -> unchanged (torchaudio semantics)
    z = oaug.add_noise(np.zeros((1, T)), n[:1], np.zeros(1))
    assert np.all(z == 0)
    assert np.isnan(oaug.add_noise(x[:1], np.zeros((1, T)), np.zeros(1))).all()


def test_noise_segments_follow_the_dataset_order():
    bank = [np.full(40000, float(i)) for i in range(3)]
    seg, nxt = oaug.noise_segments(bank, 1, 4, T)
    assert seg.shape == (4, T) and nxt == 1 + 3  # 3 clips of 40000 >= 4*23040
    assert seg[0, 0] == 1 and seg[1, -1] == 2 and seg[3, -1] == 0


def test_reverb_kernel_rotation_and_circularity():
    ir = np.zeros(5000)
    ir[37] = 2.0
    ir[100] = 0.5
    k = oaug.reverb_kernel(ir, T)
    assert k.shape == (T,) and k[0] == 2.0 and k[63] == 0.5 and k[-37:].sum() == 0
    # a pure delta at the direct path = identity (up to the mean-amplitude rescale)
    x = _clips(2)
    y = oaug.reverberate(x, np.eye(1, 300, 120)[0])
    np.testing.assert_allclose(y, x, atol=1e-12)
    # circular, not linear: a delayed tap wraps around the clip end
    d = np.zeros(300)
    d[0], d[200] = 1.0, 0.9
    y = oaug.reverberate(x, d)
    ref = x + 0.9 * np.roll(x, 200, axis=1)
    ref *= np.abs(x).mean(1, keepdims=True) / np.abs(ref).mean(1, keepdims=True)
    np.testing.assert_allclose(y, ref, atol=1e-9)


def test_spectrum_slot_layout_round_trip():
    """hbk_reverb_spectrum stores bin k at slot (k % 16) * 721 + k // 16
    (include/hbk.h); natural_spectrum() restores bin order."""
    from heybuddy.kernels import ReverbPlan
    k = np.arange(T // 2 + 1)
    slots = torch.zeros((1, ReverbPlan.SLOTS, 2))
    slots[0, (k % 16) * 721 + k // 16, 0] = torch.from_numpy(k).float()
    nat = ReverbPlan.natural_spectrum(slots)
    assert nat.shape == (1, T // 2 + 1, 2)
    np.testing.assert_array_equal(nat[0, :, 0].numpy(), k)


def _close(out, ref):
    err = np.abs(out - ref)
    return (err.max() <= 2e-5 * np.abs(ref).max()
            and np.sqrt((err ** 2).mean()) <= 2e-6 * np.sqrt((ref ** 2).mean())), err.max()


@pytest.mark.gpu
def test_reverb_spectrum_matches_rfft():
    from heybuddy.kernels import ReverbPlan
    plan = ReverbPlan()
    _, irs = _bank()
    ks = torch.stack([ReverbPlan.rotated_kernel(torch.from_numpy(ir), T) for ir in irs])
    H = ReverbPlan.natural_spectrum(plan.spectra(ks.cuda())).cpu().numpy()
    ref = np.fft.rfft(ks.numpy().astype(np.float64), axis=1)
    got = H[..., 0] + 1j * H[..., 1]
    assert np.abs(got - ref).max() <= 2e-5 * np.abs(ref).max()


@pytest.mark.gpu
def test_augment_noise_and_reverb_parity():
    from heybuddy.kernels import ReverbPlan
    plan = ReverbPlan()
    x = _clips(6, seed=4)
    noises, irs = _bank(seed=5)
    ring = np.concatenate(noises)
    starts = np.cumsum([0] + [len(n) for n in noises])[:-1]
    # clips 0-2: noise + reverb (IR 0); 3: reverb only (IR 1); 4: noise only; 5: untouched
    seg, _ = oaug.noise_segments(noises, 2, 3, T)
    noise_off = np.array([starts[2], starts[2] + T, starts[2] + 2 * T, -1, starts[4], -1])
    snr = np.array([-10.0, 3.0, 15.0, 0.0, 7.5, 0.0])
    spec_idx = np.array([0, 0, 0, 1, -1, -1])
    ks = torch.stack([ReverbPlan.rotated_kernel(torch.from_numpy(irs[i]), T) for i in range(2)]).cuda()
    H = plan.spectra(ks)
    out = plan.augment(torch.from_numpy(x).float().cuda(), torch.from_numpy(ring).float().cuda(),
                       torch.from_numpy(noise_off), torch.from_numpy(snr), H,
                       torch.from_numpy(spec_idx)).cpu().numpy()
    xf = x.astype(np.float32).astype(np.float64)
    ref = np.empty_like(xf)
    ref[:3] = oaug.reverberate(oaug.add_noise(xf[:3], seg, snr[:3]), irs[0])
    ref[3] = oaug.reverberate(xf[3:4], irs[1])[0]
    n4 = np.asarray(noises[4], np.float64)[:T]
    ref[4] = oaug.add_noise(xf[4:5], n4[None], snr[4:5])[0]
    ref[5] = xf[5]
    for i in range(6):
        ok, worst = _close(out[i], ref[i])
        assert ok, f"clip {i}: max |diff| {worst}"


@pytest.mark.gpu
def test_augment_ring_wraparound_and_long_ir():
    """A noise segment that wraps the end of the ring, and an IR longer than
    the clip (truncated to T before rotation, augmented.py -> convolve1d)."""
    from heybuddy.kernels import ReverbPlan
    plan = ReverbPlan()
    x = _clips(2, seed=8)
    rng = np.random.default_rng(3)
    ring = rng.standard_normal(30000) * 0.05
    long_ir = rng.standard_normal(30000) * np.exp(-np.arange(30000) / 3000.0)
    long_ir[5] = 10.0
    H = plan.spectra(ReverbPlan.rotated_kernel(torch.from_numpy(long_ir), T)[None].cuda())
    off = np.array([20000, 29999])
    out = plan.augment(torch.from_numpy(x).float().cuda(), torch.from_numpy(ring).float().cuda(),
                       torch.from_numpy(off), torch.tensor([0.0, 5.0]), H,
                       torch.tensor([0, 0])).cpu().numpy()
    idx = (off[:, None] + np.arange(T)[None]) % ring.size
    xf = x.astype(np.float32).astype(np.float64)
    ref = oaug.reverberate(oaug.add_noise(xf, ring.astype(np.float32)[idx], np.array([0.0, 5.0])), long_ir)
    for i in range(2):
        ok, worst = _close(out[i], ref[i])
        assert ok, f"clip {i}: max |diff| {worst}"


def test_gain_precedes_and_commutes_with_noise_and_reverb():
    """torch_audiomentations Gain runs before the noise mix and the reverb
    (augmented.py:114-118, :383-392); both are scale-equivariant (the SNR is
    relative to the gained clip, the reverb rescales to mean |input|), so the
    chain with gain g equals g times the chain without it."""
    x = _clips(3, seed=6)
    noises, irs = _bank(seed=7)
    seg, _ = oaug.noise_segments(noises, 0, 3, T)
    snr = np.array([-5.0, 2.0, 12.0])
    g = oaug.db_to_amplitude([-18.0, 0.0, 6.0])
    np.testing.assert_allclose(g, [10 ** -0.9, 1.0, 10 ** 0.3])
    y = oaug.augment_batch(x, seg, snr, irs[1], gain=g)
    ref = g[:, None] * oaug.augment_batch(x, seg, snr, irs[1])
    np.testing.assert_allclose(y, ref, rtol=1e-9, atol=1e-12 * np.abs(ref).max())
    np.testing.assert_allclose(oaug.augment_batch(x, gain=g), g[:, None] * x, rtol=0, atol=0)


@pytest.mark.gpu
def test_augment_gain_parity():
    from heybuddy.kernels import ReverbPlan
    plan = ReverbPlan()
    x = _clips(4, seed=12)
    noises, irs = _bank(seed=13)
    ring = np.concatenate(noises)
    # clip 0: gain + noise + reverb; 1: gain + reverb; 2: gain only; 3: gain + noise
    noise_off = np.array([0, -1, -1, T])
    snr = np.array([4.0, 0.0, 0.0, -3.0])
    spec_idx = np.array([0, 0, -1, -1])
    gain_db = np.array([-18.0, 6.0, -7.25, 1.5], dtype=np.float32)
    gain = torch.pow(10.0, torch.from_numpy(gain_db) / 20.0)
    H = plan.spectra(ReverbPlan.rotated_kernel(torch.from_numpy(irs[0]), T)[None].cuda())
    out = plan.augment(torch.from_numpy(x).float().cuda(), torch.from_numpy(ring).float().cuda(),
                       torch.from_numpy(noise_off), torch.from_numpy(snr), H,
                       torch.from_numpy(spec_idx), gain=gain).cpu().numpy()
    xf = x.astype(np.float32).astype(np.float64)
    g = gain.numpy().astype(np.float64)
    r32 = ring.astype(np.float32).astype(np.float64)
    ref = np.empty_like(xf)
    ref[0] = oaug.augment_batch(xf[:1], r32[None, :T], snr[:1], irs[0], gain=g[:1])[0]
    ref[1] = oaug.augment_batch(xf[1:2], ir=irs[0], gain=g[1:2])[0]
    ref[2] = oaug.augment_batch(xf[2:3], gain=g[2:3])[0]
    ref[3] = oaug.augment_batch(xf[3:4], r32[None, T:2 * T], snr[3:4], gain=g[3:4])[0]
    for i in range(4):
        ok, worst = _close(out[i], ref[i])
        assert ok, f"clip {i}: max |diff| {worst}"


@pytest.mark.gpu
def test_batch_augmenter_gain_is_per_batch():
    """mode="per_batch": one gain per batch of 128, 10^(g/20) with g in
    [-18, 6] dB; gain_prob 0 leaves the clips untouched."""
    from heybuddy.dataset.augmented import BatchAugmenter
    x = torch.from_numpy(_clips(300, seed=14)).float().cuda()
    np.random.seed(5)
    aug = BatchAugmenter(device=0, batch_size=128, background_noise_prob=0.0, reverb_prob=0.0,
                         colored_noise_prob=0.0, tanh_distortion_prob=0.0, seven_band_prob=0.0,
                         band_stop_prob=0.0, pitch_shift_prob=0.0)
    out = aug(x)
    ratio = (out / x).cpu().numpy()
    xs = x.cpu().numpy()
    for b0 in range(0, 300, 128):
        blk = ratio[b0:b0 + 128][np.abs(xs[b0:b0 + 128]) > 1e-3]
        g = np.median(blk)
        np.testing.assert_allclose(blk, g, rtol=1e-6)
        assert 10 ** (-18 / 20) * (1 - 1e-6) <= g <= 10 ** (6 / 20) * (1 + 1e-6)
    off = BatchAugmenter(device=0, background_noise_prob=0.0, reverb_prob=0.0, gain_prob=0.0,
                         colored_noise_prob=0.0, tanh_distortion_prob=0.0, seven_band_prob=0.0,
                         band_stop_prob=0.0, pitch_shift_prob=0.0)
    assert torch.equal(off(x), x)


def test_batch_plan_consumes_whole_noise_clips_per_batch():
    """Host bookkeeping of BatchAugmenter (no device): each noisy batch takes
    consecutive T-sample segments of the noise stream starting at the current
    clip and then skips every clip it touched (augmented.py:246-267); one IR
    per reverb batch, in order (:188-192); one gain per batch."""
    from heybuddy.dataset.augmented import BatchAugmenter
    aug = object.__new__(BatchAugmenter)
    aug.batch_size, aug.p_gain, aug.gain_min_db, aug.gain_max_db = 128, 1.0, -18.0, 6.0
    aug.p_noise = aug.p_reverb = 1.0
    aug.p_colored, aug.colored_snr, aug.colored_decay = 0.5, (10.0, 30.0), (-1.0, 2.0)
    aug.p_tanh, aug.tanh_range = 0.25, (1e-4, 0.1)
    aug.lengths = [48000 + 997 * i for i in range(40)]
    aug.starts = list(np.cumsum([0] + aug.lengths[:-1]))
    aug.ring, aug.spectra = object(), np.zeros((7, 1))
    aug.noise_idx = aug.ir_idx = 0
    aug._advance = {}
    n = 1000
    noise_off, spec_idx, gain_db = aug.plan_batches(n)
    idx, ir = 0, 0
    for b0 in range(0, n, 128):
        nb = min(128, n - b0)
        np.testing.assert_array_equal(noise_off[b0:b0 + nb], aug.starts[idx] + np.arange(nb) * T)
        covered = 0
        while covered < nb * T:
            covered += aug.lengths[idx]
            idx = (idx + 1) % len(aug.lengths)
        assert (spec_idx[b0:b0 + nb] == ir).all()
        ir = (ir + 1) % 7
        assert len(set(gain_db[b0:b0 + nb])) == 1 and -18 <= gain_db[b0] <= 6
        c_snr, c_fd = aug._colored[0][b0:b0 + nb], aug._colored[1][b0:b0 + nb]
        assert len(set(c_fd)) == 1 and -1 <= c_fd[0] <= 2
        assert np.isnan(c_snr).all() or (len(set(c_snr)) == 1 and 10 <= c_snr[0] <= 30)
    assert aug.noise_idx == idx and aug.ir_idx == ir
    amt = aug._tanh  # per clip: NaN (off) or U[1e-4, 0.1]
    on = ~np.isnan(amt)
    assert 0.15 < on.mean() < 0.35 and ((amt[on] >= 1e-4) & (amt[on] <= 0.1)).all()


# ---- colored noise (torch_audiomentations AddColoredNoise, augmented.py:107-113) ----
# PARITY UNPINNED at the third-party boundary (torch_audiomentations is not
# installed, no fixture): oracle/augment.py restates AddColoredNoise; the white
# noise is an explicit input on both sides. Same tolerance as above.

N1 = 16000  # torch_audiomentations _gen_noise: ONE second of noise, tiled to the clip


def test_colored_noise_oracle_properties():
    rng = np.random.default_rng(21)
    x = _clips(3, seed=21)
    w = rng.standard_normal((3, N1))
    snr = np.array([10.0, 20.0, 30.0])
    rms = lambda v: np.sqrt((v * v).mean(axis=-1))
    # f_decay 0: the noise is the white second, rms-normalised, tiled to T
    y = oaug.colored_noise(x, w, np.zeros(3), snr)
    n = (y - x) / (rms(x) / 10 ** (snr / 20))[:, None]
    wn = w / (rms(w)[:, None] + 1e-8)
    np.testing.assert_allclose(n[:, :N1], wn, atol=1e-9)
    np.testing.assert_allclose(n[:, N1:], wn[:, :T - N1], atol=1e-9)
    # any f_decay: period 16,000, and the first second sits exactly snr dB below the clip
    fd = np.array([-1.0, 0.7, 2.0])
    y = oaug.colored_noise(x, w, fd, snr)
    d = y - x
    np.testing.assert_allclose(d[:, N1:], d[:, :T - N1], rtol=0, atol=1e-12)
    np.testing.assert_allclose(20 * np.log10(rms(x) / rms(d[:, :N1])), snr, atol=1e-6)
    # the noise spectrum is the white spectrum shaped by linspace(1, sqrt(8000), 8001)^-f_decay
    lin = np.linspace(1.0, np.sqrt(8000.0), N1 // 2 + 1)
    ratio = np.abs(np.fft.rfft(d[:, :N1])) / np.abs(np.fft.rfft(w))
    for i in range(3):
        shape = ratio[i] / ratio[i, 1]
        np.testing.assert_allclose(shape[1:], (lin[1:] / lin[1]) ** -fd[i], rtol=1e-6)


@pytest.mark.gpu
def test_colored_noise_parity():
    from heybuddy.kernels import ReverbPlan
    plan = ReverbPlan()
    x = _clips(5, seed=22)
    w = np.random.default_rng(23).standard_normal((5, N1)).astype(np.float32)
    fd = np.array([-1.0, 0.0, 0.5, 1.3, 2.0], dtype=np.float32)
    snr = np.array([10.0, 15.0, 20.0, 25.0, 30.0], dtype=np.float32)
    out = plan.colored_noise(torch.from_numpy(x).float().cuda(), torch.from_numpy(fd), torch.from_numpy(snr),
                             white=torch.from_numpy(w).cuda()).cpu().numpy()
    ref = oaug.colored_noise(x.astype(np.float32), w, fd, snr)
    for i in range(5):
        ok, worst = _close(out[i], ref[i])
        assert ok, f"clip {i}: max |diff| {worst}"
    # the added noise repeats with the 16,000-sample period of torch_audiomentations' one-second noise
    d = out - x.astype(np.float32)
    np.testing.assert_allclose(d[:, N1:], d[:, :T - N1], rtol=0, atol=2e-6 * np.abs(d).max())
    # per_batch sharing: clips_per_noise = 2 -> groups {0, 1}, {2, 3}, {4} read white rows 0, 1, 2
    out2 = plan.colored_noise(torch.from_numpy(x).float().cuda(), torch.from_numpy(fd), torch.from_numpy(snr),
                              white=torch.from_numpy(w[:3]).cuda(), clips_per_noise=2).cpu().numpy()
    ref2 = oaug.colored_noise(x.astype(np.float32), w[[0, 0, 1, 1, 2]], fd, snr)
    for i in range(5):
        ok, worst = _close(out2[i], ref2[i])
        assert ok, f"shared noise, clip {i}: max |diff| {worst}"
    # group path (hbk_colored_noise_ws): f_decay shared within each group -> one coloured second per
    # group, bit-identical to colouring each clip's own copy of its group's noise
    xt = torch.from_numpy(x).float().cuda()
    plan.COLORED_GROUP_MIN = 1  # the product takes the group path from 8 clips per group
    fd_g = torch.tensor([0.5, 0.5, 1.3, 1.3, -1.0])
    out3 = plan.colored_noise(xt, fd_g, torch.from_numpy(snr), white=torch.from_numpy(w[:3]).cuda(),
                              clips_per_noise=2)
    out4 = plan.colored_noise(xt, fd_g, torch.from_numpy(snr), white=torch.from_numpy(w[[0, 0, 1, 1, 2]]).cuda())
    assert torch.equal(out3, out4)
    # the same for the generated stream: the group path against the per-clip call (hbk_colored_noise)
    from heybuddy._native import lib
    from heybuddy.kernels import ptr, stream_ptr
    out5 = plan.colored_noise(xt, fd_g, torch.from_numpy(snr), seed=11, clips_per_noise=2)
    out6 = torch.empty_like(xt)
    fd_d, snr_d = fd_g.cuda(), torch.from_numpy(snr).cuda()
    assert lib().hbk_colored_noise(plan._handle, ptr(xt), 5, xt.stride(0), None, 0, 11, 2, ptr(fd_d), ptr(snr_d),
                                   16000.0, None, 0, ptr(out6), out6.stride(0), stream_ptr(xt.device)) == 0
    assert torch.equal(out5, out6)


@pytest.mark.gpu
def test_colored_noise_nan_snr_skips_and_generated_stream():
    from heybuddy.kernels import ReverbPlan
    plan = ReverbPlan()
    x = torch.from_numpy(_clips(4, seed=24)).float().cuda()
    fd = torch.tensor([0.0, 1.0, 0.0, -1.0])
    snr = torch.tensor([12.0, float("nan"), 25.0, float("nan")])
    out = plan.colored_noise(x, fd, snr, seed=7)
    assert torch.equal(out[1], x[1]) and torch.equal(out[3], x[3])
    again = plan.colored_noise(x, fd, snr, seed=7)
    other = plan.colored_noise(x, fd, snr, seed=8)
    assert torch.equal(out, again) and not torch.equal(out[0], other[0])
    xs, os_ = x.cpu().double().numpy(), out.cpu().double().numpy()
    rms = lambda v: np.sqrt((v * v).mean())
    for i, s in ((0, 12.0), (2, 25.0)):
        n = os_[i] - xs[i]
        assert abs(20 * np.log10(rms(xs[i]) / rms(n[:N1])) - s) < 1e-3
        # f_decay 0: the generated stream itself, normalised: ~N(0, 1) moments
        z = n / rms(n)
        assert abs(z.mean()) < 0.03 and abs((z ** 4).mean() - 3.0) < 0.2
    # in place (out = x) leaves NaN-snr clips untouched too
    y = x.clone()
    plan.colored_noise(y, fd, snr, seed=7, out=y)
    assert torch.equal(y, out)


@pytest.mark.gpu
def test_augment_colored_fold_is_bit_identical():
    """hbk_augment_colored (the colored mix folded into augment_kernel's prologue) equals
    hbk_colored_noise_ws followed by hbk_augment bit for bit: group-path clips, a group
    whose first clip drew no noise (its other clips take the per-clip path), a clip whose
    f_decay differs from its group's first, NaN-snr clips; gain, noise, reverb; in place and
    out of place."""
    from heybuddy.kernels import ReverbPlan
    plan = ReverbPlan()
    plan.COLORED_GROUP_MIN = 1
    n, g = 12, 4
    x = torch.from_numpy(_clips(n, seed=41)).float().cuda()
    noises, irs = _bank(seed=42)
    ring = torch.from_numpy(np.concatenate(noises)).float().cuda()
    rng = np.random.default_rng(43)
    noise_off = torch.from_numpy(np.where(rng.random(n) < 0.7, rng.integers(0, ring.numel(), n), -1))
    snr = torch.from_numpy(rng.uniform(0, 20, n)).float()
    spec_idx = torch.from_numpy(np.where(rng.random(n) < 0.7, rng.integers(0, 2, n), -1)).int()
    gain = torch.from_numpy(rng.uniform(0.5, 2.0, n)).float()
    H = plan.spectra(torch.stack([ReverbPlan.rotated_kernel(torch.from_numpy(irs[i]), T) for i in range(2)]).cuda())
    # groups of 4: {0-3} group path with clip 2's f_decay differing; {4-7} first clip NaN, the
    # rest coloured per clip; {8-11} NaN (no colored noise)
    fd = torch.tensor([0.5, 0.5, 1.5, 0.5, -1.0, 2.0, 2.0, 2.0, 0.0, 0.0, 0.0, 0.0])
    c_snr = torch.tensor([12.0, 12.0, 12.0, 12.0, float("nan"), 20.0, 20.0, 20.0] + [float("nan")] * 4)
    for seed in (5, 6):
        ref = plan.colored_noise(x, fd, c_snr, seed=seed, clips_per_noise=g)
        ref = plan.augment(ref, ring, noise_off, snr, H, spec_idx, gain=gain)
        got = plan.augment(x, ring, noise_off, snr, H, spec_idx, gain=gain, colored=(fd, c_snr, seed, g))
        assert torch.equal(got, ref)
        y = x.clone()
        got2 = plan.augment(y, ring, noise_off, snr, H, spec_idx, out=y, gain=gain, colored=(fd, c_snr, seed, g))
        assert got2.data_ptr() == y.data_ptr() and torch.equal(y, ref)
    assert not torch.equal(got[0], plan.augment(x, ring, noise_off, snr, H, spec_idx, gain=gain)[0])
    # the batch driver with the fold (HBK_AUG_COLORED_FOLD=1) and without (=0): same output
    import os
    from heybuddy.dataset.augmented import BatchAugmenter
    xb = torch.from_numpy(_clips(300, seed=44)).float().cuda()
    outs = []
    for fold in (True, False):
        os.environ["HBK_AUG_COLORED_FOLD"] = "1" if fold else "0"
        try:
            np.random.seed(9)
            torch.manual_seed(9)
            aug = BatchAugmenter([torch.from_numpy(v).float() for v in noises],
                                 [torch.from_numpy(v).float() for v in irs], device=0, batch_size=128,
                                 colored_noise_prob=1.0, tanh_distortion_prob=0.0,
                                 seven_band_prob=0.0, band_stop_prob=0.0, pitch_shift_prob=0.0)
            outs.append(aug(xb))
        finally:
            os.environ.pop("HBK_AUG_COLORED_FOLD", None)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.gpu
def test_batch_augmenter_colored_noise_is_per_batch():
    """mode="per_batch": one (snr, f_decay) AND one noise vector per batch of 128
    (torch_audiomentations runs the transform on the batch reshaped to
    (1, batch, T)); snr in [10, 30] dB."""
    from heybuddy.dataset.augmented import BatchAugmenter
    x = torch.from_numpy(_clips(300, seed=25)).float().cuda()
    np.random.seed(6)
    aug = BatchAugmenter(device=0, batch_size=128, background_noise_prob=0.0, reverb_prob=0.0, gain_prob=0.0,
                         colored_noise_prob=1.0, tanh_distortion_prob=0.0, seven_band_prob=0.0,
                         band_stop_prob=0.0, pitch_shift_prob=0.0)
    out = aug(x)
    xs, os_ = x.cpu().double().numpy(), out.cpu().double().numpy()
    rms = lambda v: np.sqrt((v * v).mean(axis=-1))
    snr = 20 * np.log10(rms(xs) / rms((os_ - xs)[:, :N1]))  # the noise's first (normalised) second
    for b0 in range(0, 300, 128):
        blk = snr[b0:b0 + 128]
        assert blk.max() - blk.min() < 1e-3
        assert 10.0 - 1e-3 <= blk[0] <= 30.0 + 1e-3
        # the normalised noise is the same vector for every clip of the batch
        z = (os_ - xs)[b0:b0 + 128]
        z = z / rms(z)[:, None]
        np.testing.assert_allclose(z, np.broadcast_to(z[:1], z.shape), rtol=0, atol=1e-4 * np.abs(z).max())
    assert not np.allclose((os_ - xs)[0] / rms(os_ - xs)[0], (os_ - xs)[128] / rms(os_ - xs)[128])
    off = BatchAugmenter(device=0, background_noise_prob=0.0, reverb_prob=0.0, gain_prob=0.0,
                         colored_noise_prob=0.0, tanh_distortion_prob=0.0, seven_band_prob=0.0,
                         band_stop_prob=0.0, pitch_shift_prob=0.0)
    assert torch.equal(off(x), x)


# ---- tanh distortion (audiomentations TanhDistortion, augmented.py:79-90) ----
# PARITY UNPINNED at the third-party boundary (audiomentations is not
# installed); oracle/augment.py restates TanhDistortion.apply.

def _tanh_clips():
    x = _clips(6, seed=31).astype(np.float32)
    x[3] = 0.0                                                # silent: no post-gain
    x[4] = np.round(x[4] * 64) / 64                           # heavy ties around the percentile
    x[5, :100] = 0.9; x[5, 100:] = 1e-3                       # percentile inside a tie run
    return x


def test_tanh_distortion_oracle_properties():
    x = _tanh_clips()
    amt = np.array([1e-4, 0.05, 0.1, 0.07, 0.1, 0.004])
    y = oaug.tanh_distortion(x, amt)
    rms = lambda v: np.sqrt(np.mean(np.square(v.astype(np.float64)), axis=-1))
    live = rms(x) > 1e-9
    np.testing.assert_allclose(rms(y)[live], rms(x)[live], rtol=1e-5)
    assert not y[3].any()
    # monotone, odd map of x
    i = np.argsort(x[0])
    assert (np.diff(y[0][i]) >= -1e-7).all()


@pytest.mark.gpu
def test_tanh_distortion_parity():
    from heybuddy.kernels import tanh_distortion
    x = _tanh_clips()
    amt = np.array([1e-4, 0.05, 0.1, 0.07, 0.1, 0.004], dtype=np.float32)
    out = tanh_distortion(torch.from_numpy(x).cuda(), torch.from_numpy(amt)).cpu().numpy()
    ref = oaug.tanh_distortion(x, amt.astype(np.float64))
    # f32 tanh / rms on both sides: 1e-5 of the clip's peak
    for i in range(6):
        err = np.abs(out[i] - ref[i]).max()
        assert err <= 1e-5 * max(np.abs(ref[i]).max(), 1e-30), f"clip {i}: max |diff| {err}"
    # NaN amount: untouched (out of place and in place)
    nan_amt = torch.tensor([float("nan"), 0.05, float("nan"), 0.1, float("nan"), 0.01])
    xs = torch.from_numpy(x).cuda()
    o2 = tanh_distortion(xs, nan_amt)
    assert torch.equal(o2[0], xs[0]) and torch.equal(o2[2], xs[2]) and torch.equal(o2[4], xs[4])
    y = xs.clone()
    tanh_distortion(y, nan_amt, out=y)
    assert torch.equal(y, o2)


# ---------------------------------------------------------------------------
# Seven-band parametric EQ (audiomentations SevenBandParametricEQ, parity unpinned)
def test_eq_coefficients_match_oracle_and_gains():
    """The product's RBJ coefficients equal the oracle's, and each filter's
    gain at its center frequency (peaks) / far side (shelves) is the drawn gain."""
    import scipy.signal as ss
    from heybuddy.dataset.augmented import eq_coefficients
    rng = np.random.default_rng(3)
    prm = oaug.eq_draw(rng, 5, 6.0)
    ours = eq_coefficients(prm)
    sos = oaug.eq_sos(prm)
    np.testing.assert_allclose(ours, sos[..., [0, 1, 2, 4, 5]], rtol=1e-12, atol=1e-14)
    for i in range(5):
        for k in range(1, 6):  # peaks: |H(f0)| = gain
            _, h = ss.sosfreqz(sos[i, k][None], worN=[prm[i, k, 0]], fs=16000)
            np.testing.assert_allclose(20 * np.log10(abs(h[0])), prm[i, k, 1], atol=1e-6)
        _, h = ss.sosfreqz(sos[i, 0][None], worN=[1e-3], fs=16000)  # low shelf at DC
        np.testing.assert_allclose(20 * np.log10(abs(h[0])), prm[i, 0, 1], atol=1e-3)
        _, h = ss.sosfreqz(sos[i, 6][None], worN=[7999.0], fs=16000)  # high shelf near Nyquist
        np.testing.assert_allclose(20 * np.log10(abs(h[0])), prm[i, 6, 1], atol=0.05)
    assert (prm[:, 6, 0] <= 7600.0).all() and (prm[:, :, 2] >= 0.5).all() and (prm[:, :, 2] <= 1.33).all()


@pytest.mark.gpu
def test_seven_band_eq_kernel_matches_oracle():
    from heybuddy.dataset.augmented import eq_coefficients, eq_parameters
    from heybuddy.kernels import seven_band_eq
    rng = np.random.default_rng(4)
    n = 70  # a full 64-clip wave and a ragged one
    x = (rng.standard_normal((n, 24000)) * 0.2).astype(np.float32)
    np.random.seed(9)
    coef = eq_coefficients(eq_parameters(n, 6.0))
    coef[[3, 65], 0, 0] = np.nan  # coin tails: copied
    sos = np.concatenate([coef[..., :3], np.ones_like(coef[..., :1]), coef[..., 3:]], axis=-1)
    ref = oaug.seven_band_eq(x[:, :23040], sos)
    out = seven_band_eq(torch.from_numpy(x).cuda(), torch.from_numpy(coef)).cpu().numpy()
    scale = np.abs(ref).max(axis=1, keepdims=True)
    np.testing.assert_allclose(out / scale, ref / scale, rtol=0, atol=2e-6)
    np.testing.assert_array_equal(out[[3, 65]], x[[3, 65], :23040])
    # indexed, in place: only the listed clips change
    sel = np.array([5, 0, 69, 40], dtype=np.int32)
    xd = torch.from_numpy(x).cuda()
    got = seven_band_eq(xd, torch.from_numpy(coef[sel]), idx=torch.from_numpy(sel)).cpu().numpy()
    keep = np.setdiff1d(np.arange(n), sel)
    np.testing.assert_array_equal(got[keep], x[keep])
    np.testing.assert_allclose(got[sel, :23040] / scale[sel], ref[sel] / scale[sel], rtol=0, atol=2e-6)


# ---- band-stop (torch_audiomentations BandStopFilter, augmented.py:101-105) ----
# PARITY UNPINNED at the third-party boundary (torch_audiomentations / julius are
# not installed); oracle/augment.py restates julius' bandpass_filter.

def test_bandstop_oracle_properties():
    """The restated filter: each lowpass sums to 1 (a constant clip passes the
    band-stop unchanged), an in-band tone is removed, an out-of-band one kept,
    and the half size is julius' int(8 / cut_lo / 2)."""
    assert oaug.bandstop_half_size(0.1) == 40
    assert oaug.bandstop_half_size(np.float32(0.1)) == 39  # the float32 cutoff is 0.1000000015
    for c, h in ((0.03, 133), (0.3, 40)):
        np.testing.assert_allclose(oaug.lowpass_taps(c, h).astype(np.float64).sum(), 1.0, rtol=1e-6)
    n = np.arange(T)
    x = np.stack([np.full(T, 0.3), np.sin(2 * np.pi * 1000 / 16000 * n), np.sin(2 * np.pi * 3000 / 16000 * n)])
    lo, hi = np.float32(700 / 16000), np.float32(1400 / 16000)
    y = oaug.band_stop(x.astype(np.float32), np.full(3, lo), np.full(3, hi))
    np.testing.assert_allclose(y[0], x[0], atol=1e-6)
    assert np.abs(y[1, 4000:-4000]).max() < 2e-3
    np.testing.assert_allclose(y[2, 4000:-4000], x[2, 4000:-4000], atol=2e-3)
    r = np.random.default_rng(3)
    lo, hi = oaug.bandstop_draw(r, 1000)
    assert (lo > 0).all() and (lo <= hi).all() and (hi < 0.5).all()


@pytest.mark.gpu
@pytest.mark.parametrize("inplace", [False, True])
def test_band_stop_matches_oracle(inplace):
    """hbk_band_stop against the oracle over filter lengths from 43 taps to
    the longest the reference draws (half size 64,000: 12 partitions of the
    overlap-save scheme), a step clip (replicate padding) and an unlisted clip."""
    from heybuddy.kernels import ReverbPlan
    x = _clips(10, seed=41).astype(np.float32)
    x[6] = np.where(np.arange(T) < T // 3, 0.4, -0.2)          # step: the padded edges matter
    x[8] = np.where(np.arange(T) > T - 300, 0.5, x[8])         # a step inside the last h samples
    # half sizes 21, 133 (circular path), 2000, 6666, 12121, 30769 (1, 2, 3, 6
    # overlap-save partitions), 400 (circular), -, 512 (largest circular), 513
    cut_lo = np.array([0.1875, 0.03, 2.0e-3, 6.0e-4, 3.3e-4, 1.3e-4, 0.01, np.nan, 0.0078125, 0.00779],
                      np.float32)
    cut_hi = np.array([0.45, 0.2, 0.1, 0.05, 2.0e-3, 0.4987, 0.03, np.nan, 0.02, 0.3], np.float32)
    sel = np.flatnonzero(~np.isnan(cut_lo)).astype(np.int32)   # clip 7 is not listed
    ref = oaug.band_stop(x, cut_lo, cut_hi)
    plan = ReverbPlan(0)
    xd = torch.from_numpy(x).cuda()
    out = plan.band_stop(xd, torch.from_numpy(sel), torch.from_numpy(cut_lo[sel]), torch.from_numpy(cut_hi[sel]),
                         out=xd if inplace else None).cpu().numpy()
    assert [oaug.bandstop_half_size(c) for c in cut_lo[8:]] == [512, 513]
    for i in range(10):
        tol = 2e-5 * max(np.abs(x[i]).max(), np.abs(ref[i]).max())
        err = np.abs(out[i] - ref[i]).max()
        assert err <= tol, f"clip {i} (half size {oaug.bandstop_half_size(cut_lo[i]) if i != 7 else 0}): {err} > {tol}"
    np.testing.assert_array_equal(out[7], x[7])


@pytest.mark.gpu
def test_batch_augmenter_band_stop_is_per_batch():
    """BatchAugmenter: band-stop per batch of 128 (one cutoff pair per batch
    whose coin came up) between the per-clip chain and the colored noise; the
    device result equals the oracle on the drawn cutoffs."""
    from heybuddy.dataset.augmented import BatchAugmenter
    x = torch.from_numpy(_clips(300, seed=43)).float().cuda()
    np.random.seed(9)
    aug = BatchAugmenter(device=0, batch_size=128, background_noise_prob=0.0, reverb_prob=0.0, gain_prob=0.0,
                         colored_noise_prob=0.0, tanh_distortion_prob=0.0, seven_band_prob=0.0,
                         band_stop_prob=1.0, pitch_shift_prob=0.0)
    pr = aug.prepare(300)
    idx, lo, hi = (t.numpy() for t in pr["bandstop"])
    np.testing.assert_array_equal(idx, np.arange(300))
    for b0 in range(0, 300, 128):
        assert np.unique(lo[b0:b0 + 128]).size == 1 and np.unique(hi[b0:b0 + 128]).size == 1
    out = aug(x, prepared=pr).cpu().numpy()
    xs = x.cpu().numpy()
    pick = [0, 127, 128, 299]
    ref = oaug.band_stop(xs[pick], lo[pick], hi[pick])
    for j, i in enumerate(pick):
        assert np.abs(out[i] - ref[j]).max() <= 2e-5 * np.abs(xs[i]).max()
    off = BatchAugmenter(device=0, background_noise_prob=0.0, reverb_prob=0.0, gain_prob=0.0,
                         colored_noise_prob=0.0, tanh_distortion_prob=0.0, seven_band_prob=0.0,
                         band_stop_prob=0.0, pitch_shift_prob=0.0)
    assert off.prepare(300)["bandstop"] is None


# ------------------------------------------------------------------ pitch shift

def test_pitch_shift_oracle_properties():
    """The restated torch_pitch_shift: the fast shifts at 16 kHz within +-3
    semitones, the frame / resampler geometry, and a tone moving by the ratio."""
    from fractions import Fraction
    assert oaug.pitch_fast_shifts(16000, 3) == [Fraction(125, 128), Fraction(128, 125)]
    g = oaug.pitch_shift_geometry(T, 128, 125)
    assert (g["f_in"], g["f_out"], g["l1"], g["orig"], g["new"], g["width"], g["target"]) == \
        (3292, 3372, 23597, 128, 125, 7, 23044)
    g = oaug.pitch_shift_geometry(T, 125, 128)
    assert (g["f_out"], g["l1"], g["orig"], g["new"], g["target"]) == (3215, 22498, 125, 128, 23038)
    taps, w = oaug.resample_taps(128, 125)
    assert taps.shape == (125, 2 * w + 128) and taps.dtype == np.float32
    np.testing.assert_allclose(taps.sum(axis=1), 1.0, rtol=2e-2)   # ~unit DC gain per output phase
    t = np.arange(T) / 16000.0
    for num, den in ((128, 125), (125, 128)):
        y = oaug.pitch_shift(0.5 * np.sin(2 * np.pi * 1000.0 * t), num, den)[0]
        s = np.abs(np.fft.rfft(y[2000:18384] * np.hanning(16384)))
        assert abs(np.argmax(s) * 16000 / 16384 - 1000.0 * num / den) < 1.5
    assert not oaug.pitch_shift(np.zeros(T), 128, 125).any()


def test_pitch_shift_workspace_geometry():
    """hbk_pitch_shift_workspace_size (host only): 0 for an unsupported rate
    or ratio, ~0.2 MB per clip at 23,040 samples (no spectrogram is stored)."""
    from heybuddy._native import lib
    h = lib()
    one = h.hbk_pitch_shift_workspace_size(1, T, 16000, 128, 125)
    assert 100_000 < one < 400_000
    assert h.hbk_pitch_shift_workspace_size(4, T, 16000, 125, 128) > 2 * one
    assert h.hbk_pitch_shift_workspace_size(1, T, 22050, 128, 125) == 0
    assert h.hbk_pitch_shift_workspace_size(1, T, 16000, 3, 2) == 0      # 16000 -> 10666: not a fast shift


def _pitch_clips():
    x = _clips(8, seed=57).astype(np.float32)
    t = np.arange(T) / 16000.0
    x[1] = 0.3 * np.sin(2 * np.pi * 440.0 * t) + 0.1 * np.sin(2 * np.pi * 3100.0 * t)
    x[2, :9000] = 0.0                   # leading silence (all-zero frames: angle 0 in the FFT)
    x[3, 15000:] = 0.0                  # trailing silence
    x[4] = 0.0                          # silent clip stays silent
    # a chirp. (No piecewise-constant clip: its constant frames have exactly zero
    # energy off DC, so the vocoder phase carried across a step is rounding noise
    # in every implementation, the reference's float32 FFT included.)
    x[6] = 0.3 * np.sin(2 * np.pi * (100.0 + 1500.0 * t) * t)
    x[5, 8000:12000] = 0.0              # an exact-zero gap inside a clip (all-zero frames mid-clip)
    return x


@pytest.mark.gpu
@pytest.mark.parametrize("num,den,inplace", [(128, 125, False), (125, 128, True)])
def test_pitch_shift_matches_oracle(num, den, inplace):
    """hbk_pitch_shift against the float64 restatement for both fast shifts:
    speech-like clips, two tones, leading / trailing silence, a silent clip, an
    exact-zero gap inside a clip, a chirp, and an unlisted clip (7) left
    untouched. The kernel's sliding DFT keeps a float64 state with float32
    increments (a direct float64 DFT every 1024 frames; exact zeros kept exact),
    its phase float64, its synthesis float32: per clip, L2 error <= 1e-4 of the
    reference's L2 and max error <= 1e-3 of its peak (measured worst: 6.5e-5 /
    2.6e-4, on the chirp, whose quiet frames carry the increments' rounding
    into the accumulated phase; the reference's own float32 torch.stft path
    differs from the float64 restatement by up to 5e-4, see
    test_pitch_shift_oracle_vs_torch_stft_restatement)."""
    from heybuddy.kernels import pitch_shift
    x = _pitch_clips()
    sel = np.array([0, 1, 2, 3, 4, 5, 6], np.int32)
    ref = oaug.pitch_shift(x[sel], num, den)
    xd = torch.from_numpy(x).cuda()
    out = pitch_shift(xd, torch.from_numpy(sel), num, den, out=xd if inplace else None).cpu().numpy()
    worst = (0.0, 0.0)
    for j, i in enumerate(sel):
        r = ref[j]
        if not r.any():
            assert not out[i].any(), f"clip {i}: silent input, non-zero output"
            continue
        l2 = np.sqrt(((out[i] - r) ** 2).sum()) / np.sqrt((r ** 2).sum())
        mx = np.abs(out[i] - r).max() / np.abs(r).max()
        worst = (max(worst[0], l2), max(worst[1], mx))
        assert l2 <= 1e-4 and mx <= 1e-3, f"clip {i}: rel L2 {l2:.2e}, rel max {mx:.2e}"
    print(f"pitch shift {num}/{den}: worst rel L2 {worst[0]:.2e}, worst rel max {worst[1]:.2e}")
    np.testing.assert_array_equal(out[7], x[7])


def test_fast_shifts_match_oracle():
    """The package's fast-shift list (BatchAugmenter's draw set) equals the
    oracle's restatement of torch_pitch_shift.get_fast_shifts."""
    from heybuddy.dataset.augmented import fast_shifts
    for sr, semi in ((16000, 3), (16000, 12), (22050, 2), (8000, 5)):
        assert fast_shifts(sr, semi) == oaug.pitch_fast_shifts(sr, semi)


@pytest.mark.gpu
def test_batch_augmenter_pitch_shift_is_per_batch():
    """BatchAugmenter: pitch shift per batch of 128 (one fast shift per batch
    whose coin came up), first in the batch chain; the device result equals
    the oracle on the drawn shift."""
    from heybuddy.dataset.augmented import BatchAugmenter
    x = torch.from_numpy(_clips(300, seed=61)).float().cuda()
    np.random.seed(13)
    aug = BatchAugmenter(device=0, batch_size=128, background_noise_prob=0.0, reverb_prob=0.0, gain_prob=0.0,
                         colored_noise_prob=0.0, tanh_distortion_prob=0.0, seven_band_prob=0.0,
                         band_stop_prob=0.0, pitch_shift_prob=1.0)
    pr = aug.prepare(300)
    groups = pr["pitch"]
    assert sorted(np.concatenate([g[2].numpy() for g in groups]).tolist()) == list(range(300))
    shift_of = {}
    for num, den, clips in groups:
        assert (num, den) in ((125, 128), (128, 125))
        for c in clips.numpy():
            shift_of[int(c)] = (num, den)
    for b0 in range(0, 300, 128):
        assert len({shift_of[c] for c in range(b0, min(b0 + 128, 300))}) == 1
    out = aug(x, prepared=pr).cpu().numpy()
    xs = x.cpu().numpy()
    for i in (0, 127, 128, 299):
        r = oaug.pitch_shift(xs[i], *shift_of[i])[0]
        assert np.sqrt(((out[i] - r) ** 2).sum() / (r ** 2).sum()) <= 1e-4
    off = BatchAugmenter(device=0, background_noise_prob=0.0, reverb_prob=0.0, gain_prob=0.0,
                         colored_noise_prob=0.0, tanh_distortion_prob=0.0, seven_band_prob=0.0,
                         band_stop_prob=0.0, pitch_shift_prob=0.0)
    assert off.prepare(300)["pitch"] == []


def test_pitch_shift_oracle_vs_torch_stft_restatement():
    """Cross-check of the float64 pitch-shift restatement against one built on
    torch.stft / torch.istft (the functions torch_pitch_shift itself calls), in
    float32 as the reference runs them (oracle.augment.pitch_shift_torch, also
    the CPU baseline's pitch shift): both fast shifts agree to the reference's
    own float32 rounding: relative L2 < 1e-3 (measured 0.8e-4 to 5.2e-4; the
    float32 phase cumsum dominates, so the HIP kernel's 1e-4 bound against the
    float64 restatement is tighter than the reference's own error)."""
    x = _pitch_clips()[[0, 1, 2, 5, 6]]
    for num, den in ((128, 125), (125, 128)):
        a = oaug.pitch_shift(x.astype(np.float64), num, den)
        b = oaug.pitch_shift_torch(x, num, den)
        for i in range(len(x)):
            assert np.linalg.norm(a[i] - b[i]) <= 1e-3 * np.linalg.norm(a[i]), (num, den, i)


def test_resample_taps_match_oracle():
    """util.resample's polyphase filters (torchaudio _get_sinc_resample_kernel,
    float32 phase offsets as with dtype=None) equal oracle.augment.resample_taps,
    and util.resample equals the oracle's polyphase resampling."""
    from heybuddy.util.audio_util import _sinc_kernel, resample
    for orig, new in ((125, 128), (128, 125), (3, 2), (441, 160)):
        k, w = _sinc_kernel(orig, new)
        kr, wr = oaug.resample_taps(orig, new)
        assert w == wr
        np.testing.assert_array_equal(k[:, 0].numpy(), kr)
    x = _clips(2, seed=71)[:, :5000].astype(np.float32)
    y = resample(torch.from_numpy(x), 128, 125).numpy()
    taps, w = oaug.resample_taps(128, 125)
    xp = np.pad(x.astype(np.float64), ((0, 0), (w, w + 128)))
    nfr = 5000 // 128 + 1
    win = 128 * np.arange(nfr)[:, None] + np.arange(2 * w + 128)[None]
    ref = np.einsum("nfq,pq->nfp", xp[:, win], taps.astype(np.float64)).reshape(2, -1)[:, :y.shape[1]]
    np.testing.assert_allclose(y, ref, rtol=0, atol=2e-6)
