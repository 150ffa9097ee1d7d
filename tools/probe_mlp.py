"""Fused classifier train step probe (tuning aid, not a test).

  python tools/probe_mlp.py [steps]          µs per step over `steps` graph-replayed
                                             steps of B = 1100 (bench composition)
  python tools/probe_mlp.py --trace          s_memtime stage timeline of block 0's
                                             waves in k1 / k2 / k3 (libhbk_trace.so)
  options: --cus=N (a stream masked to N CUs), --batch=B (the stage-1 mix
  scaled to B rows), --reduce (a one-rank RCCL group with
  HBK_DP_REDUCE_ALWAYS=1: every step's bucket all-reduce captured into the
  graph, as the data-parallel path runs it)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
TRACE = "--trace" in sys.argv
if TRACE:
    os.environ["HBK_LIB"] = os.path.join(ROOT, "hey-buddy_amd", "lib", "libhbk_trace.so")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from heybuddy.trainer import WakeWordTrainer  # noqa: E402


BATCH = next((int(a[8:]) for a in sys.argv[1:] if a.startswith("--batch=")), 1100)


def setup(S, B=None, P=None, A=None):
    B = BATCH if B is None else B
    P = max(1, 50 * B // 1100) if P is None else P
    A = max(1, 50 * B // 1100) if A is None else A
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    pos = torch.randn((50_000, 16, 96), generator=g, device=dev) + 0.3
    neg = torch.randn((200_000, 16, 96), generator=g, device=dev).half()
    idx = torch.empty((S, B), dtype=torch.int32, device=dev)
    idx[:, :P + A] = torch.randint(0, 50_000, (S, P + A), device=dev, dtype=torch.int32)
    idx[:, P + A:] = -1 - torch.randint(0, 200_000, (S, B - P - A), device=dev, dtype=torch.int32)
    y = torch.cat([torch.ones(P), torch.zeros(B - P)]).to(dev)
    sched = torch.tensor([[1e-3, 1.0]] * S, device=dev)
    tr = WakeWordTrainer(checkpoint_dir="/tmp/probe_ck", device=dev)
    tr.model.train()
    return tr, pos, neg, idx, y, sched


def timing(S, n_cus=0):
    """n_cus > 0: on a stream masked to that many CUs (heybuddy.pipeline)."""
    if n_cus:
        from heybuddy.pipeline import masked_stream, train_cu_set
        ms = masked_stream(torch.device("cuda", 0), train_cu_set(torch.cuda.get_device_properties(0).multi_processor_count, n_cus))
        with torch.cuda.stream(ms.stream):
            timing(S)
        torch.cuda.synchronize()
        print(f"  (above: stream masked to {n_cus} CUs)")
        return
    tr, pos, neg, idx, y, sched = setup(S)
    hist = torch.zeros((S, 8), device="cuda")
    for _ in range(2):
        tr._reset_accumulation()
        tr.train_indexed(idx, y, sched, pool32=pos, pool16=neg, history=hist, steps_per_graph=50)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        tr._reset_accumulation()
        tr.train_indexed(idx, y, sched, pool32=pos, pool16=neg, history=hist, steps_per_graph=50)
    e1.record()
    torch.cuda.synchronize()
    print(f"{e0.elapsed_time(e1) * 1e3 / (3 * S):.2f} us per train step (B={BATCH}, {S} steps x 3"
          f"{', captured 1-rank all-reduce' if '--reduce' in sys.argv else ''})")


def trace():
    from heybuddy._native import lib
    tr, pos, neg, idx, y, sched = setup(4)
    fn = lib().hbk_debug_mlp_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * (6 * 4 * 128))()
    cnt = (ctypes.c_int * 24)()
    tr._reset_accumulation()
    tr.train_indexed(idx[:2], y, sched, pool32=pos, pool16=neg, graphs=False)
    torch.cuda.synchronize()
    fn(buf, cnt)  # reset
    tr.train_indexed(idx[2:3], y, sched, pool32=pos, pool16=neg, graphs=False)
    torch.cuda.synchronize()
    fn(buf, cnt)
    for k, name in enumerate(("k1a (standalone only)", "k2_rows", "k3_wgrad", "k1b_gemm", "k4 tile block 0",
                              "k4 first non-tile block")):
        evs = []
        for w in range(4):
            n = cnt[k * 4 + w]
            evs.append([(int(buf[(k * 4 + w) * 128 + i]) >> 56, int(buf[(k * 4 + w) * 128 + i]) & ((1 << 56) - 1))
                        for i in range(n)])
        if not any(evs):
            print(f"--- {name}: no marks")
            continue
        t0 = min(e[0][1] for e in evs if e)
        print(f"--- {name} (block 0; cycles from the first mark)")
        for w, e in enumerate(evs):
            print(f"  wave {w}: " + " ".join(f"{m}@{t - t0}" for m, t in e))
    if hasattr(lib(), "hbk_debug_spans"):  # k3s (v2 step): per-block spans, 100 MHz ticks
        sp = (ctypes.c_ulonglong * (1024 * 3))()
        lib().hbk_debug_spans(sp)
        rows = [(sp[3 * b], sp[3 * b + 1], sp[3 * b + 2] >> 32, sp[3 * b + 2] & 0xFFFFFFFF) for b in range(1024)
                if sp[3 * b] and sp[3 * b + 1] >= sp[3 * b]]
        if rows:
            t0 = min(r[0] for r in rows)
            print("--- k3s block spans (us from the first start): job split start end")
            by = {}
            for r in rows:
                by.setdefault(r[2], []).append(((r[0] - t0) / 100, (r[1] - t0) / 100, r[3]))
            for jb, v in sorted(by.items()):
                print(f"  job {jb}: {len(v)} blocks, start {min(x[0] for x in v):.2f}..{max(x[0] for x in v):.2f}, "
                      f"end {min(x[1] for x in v):.2f}..{max(x[1] for x in v):.2f}, "
                      f"mean dur {sum(x[1] - x[0] for x in v) / len(v):.2f}")


if __name__ == "__main__":
    if "--reduce" in sys.argv:
        import torch.distributed as dist
        os.environ.update(HBK_DP_REDUCE_ALWAYS="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="29533",
                          HSA_ENABLE_IPC_MODE_LEGACY="0")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    cus = next((int(a[6:]) for a in sys.argv[1:] if a.startswith("--cus=")), 0)
    if TRACE:
        if cus:
            from heybuddy.pipeline import masked_stream, train_cu_set
            ms = masked_stream(torch.device("cuda", 0),
                               train_cu_set(torch.cuda.get_device_properties(0).multi_processor_count, cus))
            with torch.cuda.stream(ms.stream):
                trace()
            print(f"  (above: stream masked to {cus} CUs)")
        else:
            trace()
    else:
        timing(int(next((a for a in sys.argv[1:] if a.isdigit()), 200)), cus)
