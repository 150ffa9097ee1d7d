"""Data-parallel design on CPU (gloo, world size 2).

The trainer's exchange step is: each rank computes the UNNORMALISED gradient
bucket of its class-stratified batch slice, one all-reduce sums the buckets,
and the gate + normalisation use the global statistics. Here the oracle
stands in for the HIP kernel on each rank (no GPU in this container); the
test checks that the reduced, normalised gradient equals the single-process
gradient of the whole batch, using the same sharding / reduce helpers the
trainer calls (heybuddy.distributed).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from heybuddy import distributed as hd
    from oracle import mlp as omlp
    params = omlp.init_params(seed=3)
    rng = np.random.default_rng(9)
    B = 150
    y = np.concatenate([np.ones(50, np.int64), np.zeros(100, np.int64)])
    x = rng.standard_normal((B, 16, 96)).astype(np.float32)
    xs, ys = hd.shard_batch(torch.from_numpy(x), torch.from_numpy(y), rank, world)
    g, st = omlp.flat_bucket(params, xs.numpy(), ys.numpy(), neg_weight=2.0)
    bucket = torch.from_numpy(np.concatenate([g, st]))
    hd.reduce_bucket(bucket)
    lo, hi = hd.clip_range(1003, rank, world)
    q.put((rank, bucket.numpy(), (lo, hi), int(xs.shape[0]), int((ys == 1).sum())))
    dist.destroy_process_group()


def test_dp_bucket_allreduce_equals_full_batch():
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
    from oracle import mlp as omlp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    b0, b1 = res[0][1], res[1][1]
    np.testing.assert_array_equal(b0, b1)  # every rank holds the same reduced bucket
    # single process, whole batch
    params = omlp.init_params(seed=3)
    rng = np.random.default_rng(9)
    y = np.concatenate([np.ones(50, np.int64), np.zeros(100, np.int64)])
    x = rng.standard_normal((150, 16, 96)).astype(np.float32)
    g, st = omlp.flat_bucket(params, x, y, neg_weight=2.0)
    n = st[0]
    np.testing.assert_allclose(b0[-8:], st, rtol=1e-12)
    np.testing.assert_allclose(b0[:-8] / n, g / n, rtol=1e-9, atol=1e-14)
    # normalised = the reference's dL/dtheta of BCE_mean over the selected set
    prob, z, cache = omlp.forward(params, x)
    loss, n_sel, dz = omlp.step_loss_and_dz(prob, y, 2.0)
    ref = np.concatenate([v.reshape(-1) for v in omlp.backward(params, cache, dz).values()])
    np.testing.assert_allclose(b0[:-8] / n, ref, rtol=1e-6, atol=1e-12)
    # stratified shards and a complete clip partition
    assert res[0][3] + res[1][3] == 150 and res[0][4] == res[1][4] == 25
    assert res[0][2] == (0, 501) and res[1][2] == (501, 1003)


def _init_worker(rank, world, port, q, tmp):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(1234)
    np.random.seed(1234)
    from heybuddy.dataset.features import _sharded
    from heybuddy.trainer import WakeWordTrainer

    def fn(m):  # a shard's draws: how many depends on the shard (and the rank)
        torch.rand(1000 * (rank + 1) + m)
        np.random.rand(37 * (rank + 1))
        return torch.zeros((m, 16, 96))

    feats = _sharded(fn, 11)
    after = (torch.rand(4).tolist(), float(np.random.rand()))
    tr = WakeWordTrainer(checkpoint_dir=os.path.join(tmp, f"ck{rank}"), device="cpu")
    flat_shared = tr.model.flat_parameters.clone()
    # a rank whose generator differs on its own: the broadcast from rank 0 still aligns the weights
    torch.manual_seed(99 + rank)
    tr2 = WakeWordTrainer(checkpoint_dir=os.path.join(tmp, f"ck{rank}b"), device="cpu")
    own = tr2.model.flat_parameters.clone().numpy()  # construction is rank-local: no collective
    tr2._ensure_synced()  # what the first data-parallel train call runs
    assert tr2._weights_synced
    q.put((rank, feats.shape, after, flat_shared.numpy(), tr2.model.flat_parameters.clone().numpy(), own))
    dist.destroy_process_group()


def test_dp_ranks_start_from_the_same_weights(tmp_path):
    """the sharded feature generation restores every global
    RNG stream (numpy, torch CPU, python) it offset per rank, and the trainer
    broadcasts rank 0's initial parameters, so data-parallel ranks start from
    identical weights."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_init_worker, args=(r, 2, port, q, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1] == (11, 16, 96)
    assert res[0][2] == res[1][2]  # the callers' RNG streams are the same after the sharded call
    np.testing.assert_array_equal(res[0][3], res[1][3])
    np.testing.assert_array_equal(res[0][4], res[1][4])
    assert np.abs(res[0][4]).sum() > 0
    assert np.abs(res[0][5] - res[1][5]).max() > 0  # before the sync the ranks' weights differed
    np.testing.assert_array_equal(res[1][4], res[0][5])  # ... and rank 0's won


def _eval_worker(rank, world, port, q):
    """EvalPasses.run on CPU with a stand-in plan whose eval_count is the
    oracle forward (the kernels need a GPU): which rows each rank evaluates,
    the reduced counts and the negative weight written into sched."""
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from heybuddy.trainer import EvalPasses
    q.put((rank, *_run_eval_passes(EvalPasses)))
    if world > 1:
        dist.destroy_process_group()


class _OraclePlan:
    """eval_* of the HIP plan restated on the host (test infrastructure)."""

    def __init__(self, params):
        self.params = params
        self.seen = []

    def eval_workspace_bytes(self, rows):
        return 0

    def eval_prepare(self, flat, ws):
        pass

    def eval_count(self, flat, pool, rows, label, counts, ws, row_offset=0, activation_threshold=0.5,
                   dropout_p=0.0, seed=0):
        from oracle import mlp as omlp
        n = pool.shape[0]
        r = (row_offset + np.arange(rows)) % n
        self.seen.append((id(pool), r))
        prob, _, _ = omlp.forward(self.params, pool[r].float().numpy())
        counts[2 * label] += float((prob >= activation_threshold).sum())
        counts[2 * label + 1] += float((prob > activation_threshold).sum())

    @staticmethod
    def eval_finish(cv, ct, sizes, out, target=1.5, ratio=0.0, sched=None, next_step=0):
        fph = float(cv[1]) / (sizes[0] * 1.44 / 3600)  # negatives predicted positive per hour
        w0 = float(sched[next_step - 1, 1]) if next_step > 0 else 1.0
        w = w0 * ratio if fph > target else max(1.0, w0 / ratio)
        out[0], out[5], out[6] = fph, w, w0
        sched[next_step:, 1] = w


def _run_eval_passes(EvalPasses):
    from oracle import mlp as omlp
    params = omlp.init_params(seed=4)
    rng = np.random.default_rng(3)
    pools = [torch.from_numpy(rng.standard_normal((n, 16, 96)).astype(np.float32) + off)
             for n, off in ((130, 0.3), (410, 0.0), (90, 0.2), (95, -0.1))]
    pools[1] = pools[1].half()

    class _Model:
        training = False
        dropout = type("D", (), {"p": 0.0})()
        flat_parameters = torch.zeros(1)
        plan = _OraclePlan(params)

    class _Trainer:
        device = torch.device("cpu")
        model = _Model()

    tr = _Trainer()
    ev = EvalPasses(tr, pools[0], pools[1], pools[2], pools[3], validation_batch=(20, 100),
                    testing_batch=(20, 20), adjust_ratio=2.0, target_false_positive_rate=1e9)
    sched = torch.ones((12, 2))
    ev.run(sched, next_step=4)
    ev.run(sched, next_step=8)
    seen = [(next(i for i, p in enumerate(pools) if id(p) == pid), r) for pid, r in tr.model.plan.seen]
    return ev.counts.numpy().copy(), sched.numpy().copy(), ev.history[:2].numpy().copy(), seen


def test_eval_passes_shard_rows_and_agree_on_the_weight():
    """data-parallel evaluation passes. Every rank
    evaluates a contiguous share of each pass's rows (the shares partition the
    pass), the counts are all-reduced before the bookkeeping, so both ranks
    hold the counts of the whole pass and write the same negative weight into
    sched -- the same as one process evaluating every row."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_eval_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
    from heybuddy.trainer import EvalPasses
    c1, s1, h1, seen1 = _run_eval_passes(EvalPasses)  # one process
    for r in res:
        np.testing.assert_array_equal(r[1], c1)
        np.testing.assert_array_equal(r[2], s1)
        np.testing.assert_array_equal(r[3], h1)
    # the ranks' rows partition the single process's rows, call by call
    assert len(res[0][4]) == len(res[1][4]) == len(seen1)
    for (p0, r0), (p1, r1), (p, r) in zip(res[0][4], res[1][4], seen1):
        assert p0 == p1 == p
        np.testing.assert_array_equal(np.concatenate([r0, r1]), r)
        assert abs(len(r0) - len(r1)) <= 1
    assert s1[4:, 1].max() == 0.5 or s1[4:, 1].min() >= 1.0  # the weight was written from step 4 on
