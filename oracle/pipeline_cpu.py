"""Host-CPU baseline of the config-5 pipeline (TEST / BENCH INFRASTRUCTURE ONLY,
see oracle/__init__.py): placement + the reference's augmentation chain
(oracle.augment.augment_chain) + featurization at the reference's cost
structure (oracle.featurizer.cpu_featurize), spread over a process pool.

The reference runs its feature generation in worker processes too (chunks of
25,000 clips, one ProcessPoolExecutor child each: hb/dataset/features.py:
492-535). Here the unit of work is one augmentation batch of 128 clips (the
per-batch coins of hb/dataset/augmented.py:297-394), decided for the whole
sample up front (stratified: each per-batch augmentation on exactly
round(p * batches) batches) and handed to single-threaded workers, so the
16-process wall time and the 1-thread figure (the sum of the workers' busy
times) cover exactly the same work, augmentation mix included.
"""
from __future__ import annotations

import os
import time

import numpy as np

_W = {}  # per worker process: noise bank, IRs, graph


def _init(noise_bank, irs, graph):
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch
    torch.set_num_threads(1)
    _W.update(noise_bank=noise_bank, irs=irs, graph=graph)


def _warm(_):
    import torch  # noqa: F401
    from oracle import augment, featurizer  # noqa: F401
    return os.getpid()


def _batch(job):
    """One 128-clip batch: augment (its given coins) + featurize, one thread."""
    from threadpoolctl import threadpool_limits
    from oracle.augment import augment_chain
    from oracle.featurizer import cpu_featurize
    xs, ls, coins, b, seed = job
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        rng = np.random.default_rng(seed)
        xa, cnt = augment_chain(xs, ls, rng, _W["noise_bank"], _W["irs"], batch=len(xs), stratify=False,
                                fast_pitch=True, coins_given=coins, batch0=b)
        emb = cpu_featurize(xa, _W["graph"], threads=1)
        el = time.perf_counter() - t0
    return emb, el, cnt


def featurize_pool(src, lens, noise_bank, irs, graph, workers: int, batch: int = 128, seed: int = 0,
                   job_clips: int = 32):
    """src [m, >= T] utterances -> ([m, 16, 96] embeddings, wall s, sum of the
    workers' busy s, applied counts). A job is ``job_clips`` clips of one
    128-clip batch with that batch's coins (the per-batch parameters are drawn
    per job: the same cost; a pitch-shifted batch is ~7x the work of another,
    so whole batches would leave most workers idle behind it). The pool is
    started and warmed before the clock starts (a worker's interpreter start
    is not pipeline work); jobs are handed out longest first."""
    import multiprocessing as mp
    from oracle.augment import COIN_KINDS, stratified_coins
    m = len(src)
    nb = (m + batch - 1) // batch
    coins = stratified_coins(np.random.default_rng(seed), nb)
    jobs = [(src[j:j + job_clips], lens[j:j + job_clips], {k: coins[k][j // batch:j // batch + 1] for k in COIN_KINDS},
             j // batch, seed + 1 + j) for j in range(0, m, job_clips)]
    ctx = mp.get_context("spawn")  # children start clean: no inherited device runtime
    saved = {k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
    os.environ["HIP_VISIBLE_DEVICES"] = os.environ["CUDA_VISIBLE_DEVICES"] = ""  # the workers never touch a GPU
    try:
        pool = ctx.Pool(workers, initializer=_init, initargs=(noise_bank, irs, graph))
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    # longest first (a pitch-shifted batch is ~7x another's work): the pool's
    # tail is then the cheap jobs, not one expensive job started last
    cost = [7.0 if int(j[2]["pitch"][0]) else 1.0 for j in jobs]
    order = sorted(range(len(jobs)), key=lambda i: -cost[i])
    try:
        pool.map(_warm, range(workers), chunksize=1)
        t0 = time.perf_counter()
        res_o = pool.map(_batch, [jobs[i] for i in order], chunksize=1)
        wall = time.perf_counter() - t0
        res = [None] * len(jobs)
        for i, r in zip(order, res_o):
            res[i] = r
    finally:
        pool.close()
        pool.join()
    emb = np.concatenate([r[0] for r in res])
    busy = float(sum(r[1] for r in res))
    counts = {"batches": nb, "eq_clips": 0, "tanh_clips": 0}
    for r in res:
        counts["eq_clips"] += r[2]["eq_clips"]
        counts["tanh_clips"] += r[2]["tanh_clips"]
    for k in COIN_KINDS:
        counts[k + "_batches"] = int(coins[k].sum())
    return emb, wall, busy, counts
