"""Dev probe: time hbk_colored_noise (generated white noise) on N clips with HIP events:
per-clip parameters (every clip colours its own second) and per_batch parameters
(one f_decay / snr per batch of 128: the group path, hbk_colored_noise_ws).
usage: python tools/probe_colored.py [n]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
import torch
from heybuddy.kernels import ReverbPlan
from heybuddy.synthetic import synthetic_clips
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
plan = ReverbPlan(0)
x = synthetic_clips(n, length=23040, seed=1, device="cuda")
out = torch.empty_like(x)
nb = (n + 127) // 128
for label, fd, snr, cpn in (("per-clip f_decay, noise per clip", torch.rand(n) * 3 - 1, torch.rand(n) * 20 + 10, 1),
                            ("per-batch f_decay, noise per batch of 128",
                             (torch.rand(nb) * 3 - 1).repeat_interleave(128)[:n],
                             (torch.rand(nb) * 20 + 10).repeat_interleave(128)[:n], 128)):
    for _ in range(2):
        plan.colored_noise(x, fd, snr, seed=3, out=out, clips_per_noise=cpn)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        plan.colored_noise(x, fd, snr, seed=3, out=out, clips_per_noise=cpn)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    bytes_ = n * 23040 * 4 * 2
    print(f"colored ({label}): {n} clips {ms:.3f} ms  {n/ms*1e3:.3e} clips/s  "
          f"{bytes_/ms/1e6:.1f} GB/s (x read + y written)", flush=True)
