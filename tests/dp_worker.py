"""Child process of tests/test_dp_gpu.py (never imported by pytest): one rank of
WakeWordTrainer.train_indexed through the fused HIP train step on cuda:0.

usage: python tests/dp_worker.py MODE RANK WORLD PORT OUT.npz
  MODE single : no process group, the whole batch (the reference's run)
  MODE gloo   : torch.distributed gloo, WORLD ranks sharing cuda:0; each rank
                trains on its class-stratified slice idx[:, rank::WORLD] and the
                bucket is all-reduced every step (eager: gloo stages through
                the host and cannot be captured)
  MODE nccl1  : RCCL with one rank and HBK_DP_REDUCE_ALWAYS=1: the all-reduce
                runs inside the captured hipGraphs of the steps
  DP_BIG=1    : the reference's stage-1 batch (50 + 50 + 1,000 = 1,100 rows)
  DP_MASK64=1 : the steps on a stream masked to 64 CUs (the pipelined train partition: with
                DP_BIG the v2 kernels, k3s's slabs folded before the all-reduce)
Writes the final flat parameters and the per-step history rows.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]

S, P, A, N = 24, 10, 10, 90   # steps; positives, adversarials, negatives per global batch
if os.environ.get("DP_BIG") == "1":
    S, P, A, N = 20, 50, 50, 1000
B = P + A + N


def inputs():
    import numpy as np
    rng = np.random.default_rng(2024)
    u = rng.standard_normal((16, 96)).astype(np.float32)
    u /= np.linalg.norm(u)
    pool32 = np.concatenate([rng.standard_normal((200, 16, 96)) + 0.5 * u,
                             rng.standard_normal((200, 16, 96)) - 0.25 * u]).astype(np.float32)
    pool16 = rng.standard_normal((max(1000, 2 * N), 16, 96)).astype(np.float16)
    idx = np.concatenate([rng.integers(0, 200, (S, P)), 200 + rng.integers(0, 200, (S, A)),
                          -1 - rng.integers(0, pool16.shape[0], (S, N))], 1).astype(np.int32)
    y = np.concatenate([np.ones(P), np.zeros(A + N)]).astype(np.float32)
    lr = (1e-3 * (1.0 + np.arange(S) / S)).astype(np.float32)
    sched = np.stack([lr, np.full(S, 1.5, np.float32)], 1)
    return pool32, pool16, idx, y, sched


def main():
    mode, rank, world, port, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port, "RANK": str(rank),
                       "WORLD_SIZE": str(world)})
    import numpy as np
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if mode == "gloo":
        dist.init_process_group("gloo", rank=rank, world_size=world)
    elif mode == "nccl1":
        os.environ["HBK_DP_REDUCE_ALWAYS"] = "1"
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from heybuddy.trainer import WakeWordTrainer
    calls = [0]
    real = dist.all_reduce

    def counted(*a, **k):  # host calls: one per eager step, one per step while capturing a graph
        calls[0] += 1
        return real(*a, **k)

    dist.all_reduce = counted
    pool32, pool16, idx, y, sched = inputs()
    if mode == "gloo":
        idx, y = idx[:, rank::world], y[rank::world]
    torch.manual_seed(7)  # the same initial weights on every rank
    tr = WakeWordTrainer(checkpoint_dir="/tmp/hb_dp_ck", device=dev)
    tr.model.dropout.p = 0.0
    hist = torch.zeros((S, 8), dtype=torch.float32, device=dev)
    tr._reset_accumulation()
    args = (torch.from_numpy(np.ascontiguousarray(idx)).to(dev), torch.from_numpy(y).to(dev),
            torch.from_numpy(sched).to(dev))
    kw = dict(pool32=torch.from_numpy(pool32).to(dev), pool16=torch.from_numpy(pool16).to(dev), history=hist,
              steps_per_graph=8)
    if os.environ.get("DP_MASK64") == "1":
        from heybuddy.pipeline import masked_stream, train_cu_set
        ms = masked_stream(dev, train_cu_set(torch.cuda.get_device_properties(0).multi_processor_count, 64))
        ms.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(ms.stream):
            tr.train_indexed(*args, **kw)
    else:
        tr.train_indexed(*args, **kw)
    torch.cuda.synchronize()
    np.savez(out, flat=tr.model.flat_parameters.detach().cpu().numpy(), hist=hist.cpu().numpy(),
             reduce_calls=np.array(calls[0]))
    if dist.is_initialized():
        dist.destroy_process_group()
    print("dp worker ok", mode, rank, world, flush=True)


if __name__ == "__main__":
    main()
