"""Evaluation-pass probe (tuning aid, not a test): the bench's validation +
testing pass (EvalPasses: 25,000 f32 positives + 500,000 f16 negative rows,
25,000 + 25,000 f32 testing rows, dropout on) timed per pass on the whole GPU
and on a stream masked to N CUs.

  python tools/probe_eval.py [--cus=64] [passes]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]

import torch  # noqa: E402

from heybuddy.trainer import EvalPasses, WakeWordTrainer  # noqa: E402


def run(passes, n_cus=0):
    dev = torch.device("cuda", 0)
    if n_cus:
        from heybuddy.pipeline import masked_stream, train_cu_set
        ms = masked_stream(dev, train_cu_set(torch.cuda.get_device_properties(0).multi_processor_count, n_cus))
        with torch.cuda.stream(ms.stream):
            run(passes)
        torch.cuda.synchronize()
        print(f"  (above: stream masked to {n_cus} CUs)")
        return
    g = torch.Generator(device=dev).manual_seed(0)
    n = 25_000
    vpos = torch.randn((n, 16, 96), generator=g, device=dev) + 0.3
    vneg = torch.randn((n, 16, 96), generator=g, device=dev).half()
    tpos = torch.randn((n, 16, 96), generator=g, device=dev) + 0.3
    tadv = torch.randn((n, 16, 96), generator=g, device=dev)
    tr = WakeWordTrainer(checkpoint_dir="/tmp/probe_ck", device=dev)
    tr.model.train()
    ev = EvalPasses(tr, vpos, vneg, tpos, tadv)
    sched = torch.tensor([[1e-3, 1.0]] * 100, device=dev)
    for _ in range(2):
        ev.run(sched, 1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(passes):
        ev.run(sched, 1)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / passes
    print(f"{ms:.3f} ms per pass of {ev.rows_per_pass} rows ({ev.rows_per_pass / ms / 1e3:.1f} M rows/s); "
          f"history {ev.history[ev.n - 1].tolist()}")


if __name__ == "__main__":
    cus = next((int(a[6:]) for a in sys.argv[1:] if a.startswith("--cus=")), 0)
    run(int(next((a for a in sys.argv[1:] if a.isdigit()), 10)), cus)
