"""Data-parallel train step on the GPU, through
the fused HIP kernels and the per-step bucket all-reduce, each rank a FRESH
child process (tests/dp_worker.py; never a re-exec of the pytest process):

* 2 ranks sharing cuda:0 over gloo (RCCL cannot put two ranks on one GPU),
  each on its class-stratified half of every batch, against one process on
  the whole batch: the reduced bucket makes every rank take the identical
  Adam step, so both ranks end with the same parameters and those equal the
  single-process run up to summation order;
* one RCCL rank with the all-reduce forced on (HBK_DP_REDUCE_ALWAYS=1): the
  collective is captured into the train step's hipGraphs and replayed (the
  path N > 1 ranks take on RCCL) and must give the single-process result.

Bounds: parameters after 24 Adam steps; summation order differs between a
split and a whole batch, and Adam's update is ~lr * sign(m / sqrt(v)), so a
gradient at the fp32 noise floor can flip one lr-sized step: >= 99.5 % of the
elements within 1e-5, every element within 2 * sum(lr) (the stages test's
rule); statistics rows (selected counts, accumulation) exact.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dp_worker.py")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return str(p)


def _run(mode, world, tmp_path, **extra_env):
    port = _port()
    tag = "".join(f"_{k}{v}" for k, v in sorted(extra_env.items()))
    outs = [str(tmp_path / f"{mode}{tag}_{r}.npz") for r in range(world)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **extra_env)
    procs = [subprocess.Popen([sys.executable, WORKER, mode, str(r), str(world), port, outs[r]], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
    logs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(out)
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    return [np.load(o) for o in outs]


def _close(a, b, lr_sum):
    d = np.abs(a - b)
    assert float(np.mean(d <= 1e-5)) >= 0.995, float(np.mean(d <= 1e-5))
    assert float(d.max()) <= 2 * lr_sum, (float(d.max()), 2 * lr_sum)


def test_dp_two_ranks_equal_single_process(tmp_path):
    sys.path[:0] = [os.path.join(ROOT, "tests")]
    import dp_worker
    single = _run("single", 1, tmp_path)[0]
    r0, r1 = _run("gloo", 2, tmp_path)
    np.testing.assert_array_equal(r0["flat"], r1["flat"])  # identical Adam step on every rank
    assert int(r0["reduce_calls"]) == dp_worker.S            # gloo: eager, one all-reduce per step
    lr_sum = float(dp_worker.inputs()[4][:, 0].sum())
    _close(r0["flat"], single["flat"], lr_sum)
    # per-step records (n_sel, accumulation steps, fired, loss, n_neg, fp, n_pos, tp): the
    # counts are global sums of per-sample decisions, so exact; the loss to summation order
    cols = [0, 1, 2, 4, 5, 6, 7]
    np.testing.assert_array_equal(r0["hist"][:, cols], single["hist"][:, cols])
    np.testing.assert_allclose(r0["hist"][:, 3], single["hist"][:, 3], rtol=2e-4)
    assert single["hist"][:, 2].sum() >= 1  # Adam fired


def test_rccl_allreduce_captured_in_train_graph(tmp_path):
    sys.path[:0] = [os.path.join(ROOT, "tests")]
    import dp_worker
    single = _run("single", 1, tmp_path)[0]
    cap = _run("nccl1", 1, tmp_path)[0]
    # a one-rank sum is the identity: the captured graphs replay the same steps (the weight-
    # gradient column sums use float atomics, so two runs agree to summation order, not bitwise)
    lr_sum = float(dp_worker.inputs()[4][:, 0].sum())
    _close(cap["flat"], single["flat"], lr_sum)
    cols = [0, 1, 2, 4, 5, 6, 7]
    np.testing.assert_array_equal(cap["hist"][:, cols], single["hist"][:, cols])
    # the collective ran inside replayed graphs: fewer host all_reduce calls than steps
    # (24 steps: 1 eager first step, an 8-step graph captured once and replayed twice, a
    # 6-step tail graph, 1 eager step -> 16 calls), while the gloo ranks call it every step
    assert int(cap["reduce_calls"]) < dp_worker.S, int(cap["reduce_calls"])
    r0 = np.load(str(tmp_path / "gloo_0.npz")) if (tmp_path / "gloo_0.npz").exists() else None
    assert r0 is None or int(r0["reduce_calls"]) == dp_worker.S


def test_rccl_allreduce_with_the_v2_step_on_the_train_partition(tmp_path):
    """The DP per-rank mode's train step as the pipelined headline runs it at N > 1: B = 1,100
    on a 64-CU stream (the v2 kernels), the weight-gradient slabs folded into the bucket
    before the captured RCCL all-reduce -- against the single process on the whole GPU (v1,
    slabs summed by the update)."""
    sys.path[:0] = [os.path.join(ROOT, "tests")]
    single = _run("single", 1, tmp_path, DP_BIG="1")[0]
    cap = _run("nccl1", 1, tmp_path, DP_BIG="1", DP_MASK64="1")[0]
    assert cap["flat"].shape == single["flat"].shape
    S = single["hist"].shape[0]  # (lr sum from the worker's schedule)
    lr_sum = float((1e-3 * (1.0 + np.arange(S) / S)).astype(np.float32).sum())
    _close(cap["flat"], single["flat"], lr_sum)
    cols = [0, 1, 2, 4, 5, 6, 7]
    np.testing.assert_array_equal(cap["hist"][:, cols], single["hist"][:, cols])
    assert int(cap["reduce_calls"]) < S
