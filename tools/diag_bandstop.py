"""Band-stop determinism / tolerance probe on the headline test's inputs
(tests/test_e2e_gpu.py stages 1-3), printing per checked row the two
tolerance ratios of _close_aug and whether repeated launches agree bit for bit.
usage: python tools/diag_bandstop.py"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..",
                                                                             "hey-buddy_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import augment as oaug  # noqa: E402
from heybuddy.dataset.augmented import bandstop_cutoffs, eq_coefficients, eq_parameters, target_length_offsets  # noqa: E402,E501
from heybuddy.kernels import ReverbPlan, pitch_shift, place_clips, seven_band_eq, tanh_distortion  # noqa: E402
from heybuddy.synthetic import speech_clips  # noqa: E402

T, N = 23040, 300
dev = torch.device("cuda", 0)
np.random.seed(2024)
pos, pos_len = speech_clips("hello world", N // 2, seed=11, device=dev)
adv, adv_len = speech_clips("hello world", N - N // 2, seed=12, device=dev, adversarial=True)
src = torch.cat([pos, adv])
lens = np.concatenate([pos_len, adv_len]).astype(np.int32)
rows = list(range(0, N, 23)) + [N - 1]
pre = target_length_offsets(lens, T)
x = place_clips(src, torch.from_numpy(lens), torch.from_numpy(pre.astype(np.int32)), T)
coef = eq_coefficients(eq_parameters(N, 6.0))
x = seven_band_eq(x, torch.from_numpy(coef).to(dev))
amount = np.random.uniform(1e-4, 0.1, N).astype(np.float32)
x = tanh_distortion(x, torch.from_numpy(amount).to(dev))
pre_pitch = x.clone()
outs = []
for rep in range(3):
    y = pre_pitch.clone()
    for (num, den), b in (((125, 128), 0), ((128, 125), 1)):
        sel = np.arange(b * 128, min(N, (b + 1) * 128), dtype=np.int32)
        y = pitch_shift(y, torch.from_numpy(sel), num, den, out=y)
    outs.append(y.cpu().numpy())
print("pitch repeat bit-equal:", all(np.array_equal(outs[0], o) for o in outs[1:]),
      "max diff", max(np.abs(outs[0] - o).max() for o in outs[1:]), flush=True)
x_in = outs[0]
plan = ReverbPlan(dev)
lo_b, hi_b = bandstop_cutoffs(3)
batch = np.arange(N) // 128
lo, hi = lo_b[batch], hi_b[batch]
print("cutoffs", lo_b, hi_b, "half", [int(8 / float(c) / 2) for c in lo_b])
bs = []
for rep in range(3):
    xx = torch.from_numpy(x_in).to(dev)
    bs.append(plan.band_stop(xx, torch.arange(N, dtype=torch.int32), torch.from_numpy(lo), torch.from_numpy(hi),
                             out=xx).cpu().numpy())
print("band-stop repeat bit-equal:", all(np.array_equal(bs[0], o) for o in bs[1:]), flush=True)
ref = oaug.band_stop(x_in, lo, hi)
for i in rows:
    err = np.abs(bs[0][i] - ref[i])
    r1 = err.max() / (np.abs(ref[i]).max() + 1e-30)
    r2 = np.sqrt((err ** 2).mean()) / (np.sqrt((ref[i] ** 2).mean()) + 1e-30)
    flag = "FAIL" if (r1 > 2e-5 or r2 > 2e-6) else "ok"
    print(f"row {i:3d} max|ref| {np.abs(ref[i]).max():.3e} rms {np.sqrt((ref[i]**2).mean()):.3e} "
          f"max|err| {err.max():.2e} maxratio {r1:.2e} rmsratio {r2:.2e} nz {np.count_nonzero(x_in[i])} {flag}")
