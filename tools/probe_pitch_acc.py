"""Pitch-shift accuracy on the headline test's inputs (tests/test_e2e_gpu.py
stages 1-3): per checked row the relative L2 and max error of hbk_pitch_shift
against the float64 oracle, for the library HBK_LIB names (A/B of vocoder builds).
usage: python tools/probe_pitch_acc.py [stride]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..",
                                                                             "hey-buddy_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import augment as oaug  # noqa: E402
from heybuddy.dataset.augmented import eq_coefficients, eq_parameters, target_length_offsets  # noqa: E402
from heybuddy.kernels import pitch_shift, place_clips, seven_band_eq, tanh_distortion  # noqa: E402
from heybuddy.synthetic import speech_clips  # noqa: E402

T, N = 23040, 256
stride = int(sys.argv[1]) if len(sys.argv) > 1 else 23
dev = torch.device("cuda", 0)
np.random.seed(2024)
torch.manual_seed(2024)
pos, pos_len = speech_clips("hello world", N // 2, seed=11, device=dev)
adv, adv_len = speech_clips("hello world", N - N // 2, seed=12, device=dev, adversarial=True)
src = torch.cat([pos, adv])
lens = np.concatenate([pos_len, adv_len]).astype(np.int32)
pre = target_length_offsets(lens, T)
x = place_clips(src, torch.from_numpy(lens), torch.from_numpy(pre.astype(np.int32)), T)
coef = eq_coefficients(eq_parameters(N, 6.0))
x = seven_band_eq(x, torch.from_numpy(coef).to(dev))
amount = np.random.uniform(1e-4, 0.1, N).astype(np.float32)
x = tanh_distortion(x, torch.from_numpy(amount).to(dev))
x_in = x.cpu().numpy()
worst = []
for (num, den), b in (((125, 128), 0), ((128, 125), 1)):
    sel = np.arange(b * 128, (b + 1) * 128, dtype=np.int32)
    y = pitch_shift(x.clone(), torch.from_numpy(sel), num, den).cpu().numpy()
    for i in sel[::stride]:
        r = oaug.pitch_shift(x_in[i:i + 1].astype(np.float64), num, den)[0]
        l2 = np.sqrt(((y[i] - r) ** 2).sum()) / np.sqrt((r ** 2).sum())
        mx = np.abs(y[i] - r).max() / np.abs(r).max()
        worst.append(l2)
        print(f"{num}/{den} clip {i:3d}: L2 {l2:.2e} max {mx:.2e}", flush=True)
print(f"L2 max {max(worst):.3e} mean {np.mean(worst):.3e} ({os.environ.get('HBK_LIB', 'libhbk.so')})")
