"""Dev probe: time hbk_mel_frames on N clips with HIP events."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
import torch
from oracle import mel as omel
from heybuddy.kernels import MelPlan
from heybuddy.synthetic import synthetic_clips
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
plan = MelPlan(omel.hann_window(), omel.mel_fbank())
x = synthetic_clips(n, seed=1, device="cuda")
torch.cuda.synchronize()
for _ in range(3):
    y = plan(x, 141)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 10
e0.record()
for _ in range(reps):
    y = plan(x, 141)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
bytes_ = n * (22912 * 4 + 141 * 32 * 4)
print(f"mel: {n} clips {ms:.3f} ms  {n/ms*1e3:.3e} clips/s  {bytes_/ms/1e6:.1f} GB/s")
