"""k4 (gate + Adam) timing with and without keeping the weight cache (tuning aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
import torch  # noqa: E402

from heybuddy.kernels import MlpPlan  # noqa: E402

dev = torch.device("cuda", 0)
plan = MlpPlan()
n = plan.n_params
params = torch.randn(n, device=dev) * 0.05
bucket = torch.randn(n + plan.N_STATS, device=dev) * 1e-3
m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
state = plan.new_state(dev) if hasattr(plan, "new_state") else torch.zeros(16, device=dev)
ws = plan.workspace(1100, dev)
for fire in (True, False):
    for use_ws in (False, True):
        times = []
        for rep in range(3):
            bucket[n:] = 0.0
            bucket[n] = 200.0 if fire else 0.0  # n_sel: the gate fires once 128 samples have accumulated
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(200):
                plan.step_update(params, bucket, m, v, state, i & 1, lr=1e-4, workspace=ws if use_ws else None)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / 200)
        print(f"k4 fire={fire} cache={use_ws}: {min(times):.2f} us per call")
