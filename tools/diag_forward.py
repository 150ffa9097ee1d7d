"""Diagnostic (not a test): fused HIP forward vs the oracle at several batch
sizes; prints max |dp| and how many probabilities sit within 1e-5 of 0.5."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import golden_classifier as gc  # noqa: E402
from oracle import mlp as omlp  # noqa: E402
from heybuddy.wakeword import WakeWordMLPModel  # noqa: E402

params = gc.golden_inputs()[0]
m = WakeWordMLPModel()
m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=True)
m = m.cuda().eval()
pools, val, test = gc.stage_inputs()
for x, y in val[:2]:
    p = m(torch.from_numpy(x).cuda()).cpu().numpy().ravel()
    po, _, _ = omlp.forward(params, x)
    print("val batch", x.shape[0], "max|dp|", float(np.abs(p - po).max()), "near 0.5:", int((np.abs(po - 0.5) < 1e-5).sum()))
rng = np.random.default_rng(0)
for B in (1, 17, 273, 550, 1000, 1100, 2000):
    x = rng.standard_normal((B, 16, 96)).astype(np.float32)
    p = m(torch.from_numpy(x).cuda()).cpu().numpy().ravel()
    po, _, _ = omlp.forward(params, x)
    print("B", B, "max|dp|", float(np.abs(p - po).max()))
