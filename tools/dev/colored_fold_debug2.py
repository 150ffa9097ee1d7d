"""Dev probe: which part of the fold differs from colored_noise + augment (300 clips, groups of 128)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
from test_augment import _clips, _bank
from heybuddy.kernels import ReverbPlan
plan = ReverbPlan()
n, g = 300, 128
x = torch.from_numpy(_clips(n, seed=44)).float().cuda()
noises, irs = _bank(seed=42)
ring = torch.from_numpy(np.concatenate(noises)).float().cuda()
H = plan.spectra(torch.stack([ReverbPlan.rotated_kernel(torch.from_numpy(irs[i]), 23040) for i in range(2)]).cuda())
rng = np.random.default_rng(1)
fd = torch.full((n,), 0.723)
csnr = torch.from_numpy(np.repeat(rng.uniform(3, 30, 3), g)[:n]).float()
seed = 3686776903862026525
off = torch.full((n,), -1, dtype=torch.int64)
noff = torch.from_numpy(rng.integers(0, ring.numel(), n))
sidx_off = torch.full((n,), -1, dtype=torch.int32)
sidx = torch.from_numpy(rng.integers(0, 2, n)).int()
snr = torch.from_numpy(rng.uniform(0, 20, n)).float()
gain = torch.from_numpy(rng.uniform(0.1, 1, n)).float()
c = plan.colored_noise(x, fd, csnr, seed=seed, clips_per_noise=g)
for name, no, si, gn in (("colored only", off, sidx_off, None), ("+gain", off, sidx_off, gain),
                         ("+noise", noff, sidx_off, None), ("+reverb", off, sidx, None), ("all", noff, sidx, gain)):
    ref = plan.augment(c, ring, no, snr, H, si, gain=gn)
    got = plan.augment(x, ring, no, snr, H, si, gain=gn, colored=(fd, csnr, seed, g))
    d = (ref - got).abs()
    rows = torch.nonzero(d.amax(1) > 0).reshape(-1).tolist()
    print(name, "max", float(d.max()), "rows", len(rows), rows[:8])
