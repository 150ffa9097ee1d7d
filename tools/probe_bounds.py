"""Bounds-checked run of the fused train step (tuning / debugging aid, not a test).

HBK_LIB=hey-buddy_amd/lib/libhbk_bounds.so python tools/probe_bounds.py
runs the eager step on the classifier fixture's inputs, then a graph-replayed
indexed stage (tools/probe_mlp.py's setup) at a few batch sizes, and after each
prints the first out-of-range global access the step kernels recorded
(source line of hbk_mlp_fused.hip, block, thread, address), or 'clean'.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
os.environ.setdefault("HBK_LIB", os.path.join(ROOT, "hey-buddy_amd", "lib", "libhbk_bounds.so"))

import torch  # noqa: E402

from heybuddy._native import lib  # noqa: E402


def report(what):
    out = (ctypes.c_ulonglong * 4)()
    rc = lib().hbk_debug_bounds(out)
    if rc != 0:
        print(f"{what}: hbk_debug_bounds rc {rc}")
    elif out[0] == 0:
        print(f"{what}: clean")
    else:
        print(f"{what}: OUT OF RANGE at hbk_mlp_fused.hip:{out[0]} block {out[1]} thread {out[2]} addr {out[3]:#x}")
    sys.stdout.flush()


def eager():
    from oracle import golden_classifier as gc
    from heybuddy.wakeword import WakeWordMLPModel
    params, x, y, _ = gc.golden_inputs()
    m = WakeWordMLPModel()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=True)
    m.dropout.p = 0.0
    m = m.cuda()
    plan = m.plan
    for B in (len(x), 17, 1):
        bucket = torch.zeros(plan.n_params + plan.N_STATS, device="cuda")
        state = plan.new_state("cuda")
        xs = torch.as_tensor(x[:B]).cuda().reshape(B, -1).float().contiguous()
        ys = torch.as_tensor(y[:B]).cuda().to(torch.float32)
        plan.step_fwd_bwd(m.flat_parameters, bucket, state, 0, ys, B, pool32=xs, neg_weight=2.0)
        report(f"eager step B={B}")
        plan.forward(m.flat_parameters, xs)
        report(f"forward B={B}")


def indexed():
    sys.argv = [sys.argv[0]]
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import probe_mlp as pm
    for B in (1100, 550, 273, 138, 16):
        pm.BATCH = B
        tr, pos, neg, idx, y, sched = pm.setup(8, B=B)
        hist = torch.zeros((8, 8), device="cuda")
        tr._reset_accumulation()
        tr.train_indexed(idx, y, sched, pool32=pos, pool16=neg, history=hist, graphs=False)
        report(f"train_indexed B={B}")


if __name__ == "__main__":
    eager()
    indexed()
