"""The evaluation passes of train_epoch on the GPU (hbk_mlp_eval_*,
kv_gemm_kernel (input GEMM + network) + kv_finish_kernel): the validation /
testing forwards of trainer.py:496-566 reduced to prediction counts, and the
post-validation bookkeeping (false positives per hour, recall, testing rates,
dynamic negative weight, trainer.py:509-536).

Oracle: oracle/mlp.py (float64 forward, the counter-based dropout mask
restated, eval_counts / eval_finish). The classifier forward itself is pinned
against the reference (tests/golden/classifier.npz, test_mlp_fused_gpu.py);
here the input LayerNorm is folded into the GEMM's epilogue and the rows run
through the throughput kernel. Tolerance: probabilities 2e-5 absolute (the
split-f16 products are ~2^-22 relative; the fold adds ~|mean / std| of that);
counts exact against the kernel's own probabilities, and against the oracle's
away from the threshold.
"""
import numpy as np
import pytest
import torch

from oracle import mlp as omlp

pytestmark = pytest.mark.gpu


def _model(params):
    from heybuddy.wakeword import WakeWordMLPModel
    m = WakeWordMLPModel()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=True)
    return m.cuda()


def _pools(seed=0, n32=300, n16=500):
    rng = np.random.default_rng(seed)
    p32 = (rng.standard_normal((n32, 16, 96)) * 1.5 + 0.3).astype(np.float32)
    p16 = (rng.standard_normal((n16, 16, 96)) - 0.2).astype(np.float16)
    return p32, p16


def _run(plan, flat, pool, rows, label, p=0.0, seed=0, row_offset=0, idx=None):
    ws = torch.empty(plan.eval_workspace_bytes(rows), dtype=torch.uint8, device="cuda")
    plan.eval_prepare(flat, ws)
    counts = torch.zeros(4, device="cuda")
    prob = torch.zeros(rows, device="cuda")
    plan.eval_count(flat, pool, rows, label, counts, ws, idx=idx, row_offset=row_offset, dropout_p=p, seed=seed,
                    prob=prob)
    return counts.cpu().numpy(), prob.cpu().numpy()


def test_eval_probabilities_and_counts_match_oracle():
    params = omlp.init_params(seed=5)
    p32, p16 = _pools()
    # centre the output bias so that the f16 rows' predictions straddle the threshold
    _, z, _ = omlp.forward(params, p16.astype(np.float32))
    params["mlp_out.output.bias"] = (params["mlp_out.output.bias"] - np.median(z) + 1e-3).astype(np.float32)
    m = _model(params)
    # positives from an f32 pool, every row once
    c, pr = _run(m.plan, m.flat_parameters, torch.from_numpy(p32).cuda(), 300, 1)
    ref, _, _ = omlp.forward(params, p32)
    np.testing.assert_allclose(pr, ref, atol=2e-5, rtol=0)
    np.testing.assert_array_equal(c, omlp.eval_counts(pr, 1))
    # negatives from an f16 pool, 1,000 rows wrapping around its 500 (row r = pool row r % 500)
    c16, pr16 = _run(m.plan, m.flat_parameters, torch.from_numpy(p16).cuda(), 1000, 0)
    ref16, _, _ = omlp.forward(params, p16.astype(np.float32))
    np.testing.assert_allclose(pr16[:500], ref16, atol=2e-5, rtol=0)
    np.testing.assert_allclose(pr16[500:], pr16[:500], atol=1e-6, rtol=0)  # no dropout: independent of r
    np.testing.assert_array_equal(c16, omlp.eval_counts(pr16, 0))
    # against the oracle's counts: exact but for predictions within the tolerance of the threshold
    allref = np.concatenate([ref16, ref16])
    near = int((np.abs(allref - 0.5) <= 2e-5).sum())
    assert np.abs(c16 - omlp.eval_counts(allref, 0)).max() <= near
    assert 0 < c16[0] < 1000  # the seeded weights put predictions on both sides


def test_eval_dropout_mask_and_indexed_rows():
    """Dropout p = 0.1 (the reference keeps it on in validation): the mask is
    the counter hash of (seed, row_offset + r, element), restated in the
    oracle; rows by an index array."""
    params = omlp.init_params(seed=6)
    m = _model(params)
    p32, p16 = _pools(seed=1)
    rng = np.random.default_rng(2)
    idx = rng.integers(0, 500, 700).astype(np.int32)
    seed, off = 0x1234_5678_9ABC, 4242
    c, pr = _run(m.plan, m.flat_parameters, torch.from_numpy(p16).cuda(), 700, 0, p=0.1, seed=seed, row_offset=off,
                 idx=torch.from_numpy(idx).cuda())
    keep = omlp.dropout_keep(seed, off + np.arange(700), p=0.1)
    x = p16[idx].astype(np.float32).reshape(700, -1) * keep / np.float32(0.9)
    ref, _, _ = omlp.forward(params, x.reshape(700, 16, 96))
    np.testing.assert_allclose(pr, ref, atol=2e-5, rtol=0)
    np.testing.assert_array_equal(c, omlp.eval_counts(pr, 0))
    # f32 rows with dropout
    c, pr = _run(m.plan, m.flat_parameters, torch.from_numpy(p32).cuda(), 300, 1, p=0.1, seed=seed + 1)
    keep = omlp.dropout_keep(seed + 1, np.arange(300), p=0.1)
    ref, _, _ = omlp.forward(params, (p32.reshape(300, -1) * keep / np.float32(0.9)).reshape(300, 16, 96))
    np.testing.assert_allclose(pr, ref, atol=2e-5, rtol=0)


def test_eval_chunk_boundary_and_ragged_tiles():
    """More rows than one launch chunk (131,072) and a ragged last tile."""
    params = omlp.init_params(seed=7)
    m = _model(params)
    _, p16 = _pools(seed=3, n16=333)
    rows = 131072 + 301
    c, pr = _run(m.plan, m.flat_parameters, torch.from_numpy(p16).cuda(), rows, 0, row_offset=5)
    ref, _, _ = omlp.forward(params, p16.astype(np.float32))
    np.testing.assert_allclose(pr, ref[(5 + np.arange(rows)) % 333], atol=2e-5, rtol=0)
    np.testing.assert_array_equal(c, omlp.eval_counts(pr, 0))


def test_eval_count_multi_equals_separate_launches():
    """hbk_mlp_eval_count_multi: three f32 pools (ragged row counts, offsets, both labels, two
    counter sets, dropout on) in one launch give exactly the counts of three hbk_mlp_eval_count
    launches; the counts against the kernel's own probabilities (exact) and the oracle's."""
    params = omlp.init_params(seed=8)
    rng = np.random.default_rng(9)
    host = [(rng.standard_normal((n, 16, 96)) * 1.3 + 0.2).astype(np.float32) for n in (301, 129, 77)]
    # centre the output bias so that the predictions straddle the threshold (non-trivial counts)
    _, z, _ = omlp.forward(params, np.concatenate(host))
    params["mlp_out.output.bias"] = (params["mlp_out.output.bias"] - np.median(z) + 1e-3).astype(np.float32)
    m = _model(params)
    pools = [torch.from_numpy(h).cuda() for h in host]
    parts = [(pools[0], 333, 7, 1, 0, 0x51), (pools[1], 129, 0, 1, 1, 0x52), (pools[2], 200, 40, 0, 1, 0x53)]
    ws = torch.empty(m.plan.eval_workspace_bytes(400), dtype=torch.uint8, device="cuda")
    m.plan.eval_prepare(m.flat_parameters, ws)
    multi = torch.zeros((2, 4), device="cuda")
    m.plan.eval_count_multi(m.flat_parameters, parts, multi, ws, dropout_p=0.1)
    sep = torch.zeros((2, 4), device="cuda")
    for pool, rows, off, label, which, seed in parts:
        m.plan.eval_count(m.flat_parameters, pool, rows, label, sep[which], ws, row_offset=off, dropout_p=0.1,
                          seed=seed)
    torch.testing.assert_close(multi, sep, rtol=0, atol=0)
    for pool, rows, off, label, which, seed in parts:  # each part's share against its own probabilities
        c, pr = _run(m.plan, m.flat_parameters, pool, rows, label, p=0.1, seed=seed, row_offset=off)
        n = pool.shape[0]
        keep = omlp.dropout_keep(seed, off + np.arange(rows), p=0.1)
        x = pool.cpu().numpy().reshape(n, -1)[(off + np.arange(rows)) % n] * keep / np.float32(0.9)
        ref, _, _ = omlp.forward(params, x.reshape(rows, 16, 96))
        np.testing.assert_allclose(pr, ref, atol=2e-5, rtol=0)
        np.testing.assert_array_equal(c, omlp.eval_counts(pr, label))
    assert 0 < multi[:, 0].sum() < 333 + 129 + 200  # both sides of the threshold


def test_eval_finish_matches_reference_bookkeeping():
    from heybuddy.kernels import MlpPlan
    sizes = (500_000.0, 25_000.0, 25_000.0, 25_000.0)
    cv = np.array([310.0, 309.0, 24_000.0, 23_990.0], np.float32)
    ct = np.array([120.0, 118.0, 20_000.0, 19_876.0], np.float32)
    for cv0, nw0 in ((310.0, 1.0), (100.0, 4.0), (10.0, 1.0), (0.0, 8.0)):
        cv[0] = cv0
        sched = torch.tensor([[1e-3, nw0]] * 10, device="cuda")
        out = torch.zeros(8, device="cuda")
        MlpPlan.eval_finish(torch.from_numpy(cv).cuda(), torch.from_numpy(ct).cuda(), sizes, out, target=1.5,
                            ratio=2.0, sched=sched, next_step=4)
        ref = omlp.eval_finish(cv, ct, sizes, nw0, 1.5, 2.0)
        np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-6)
        s = sched.cpu().numpy()
        assert (s[:4, 1] == nw0).all() and (s[4:, 1] == np.float32(ref[5])).all()


def test_train_epoch_with_device_eval_passes_matches_host_batches(tmp_path):
    """train_epoch takes an EvalPasses over HBM pools as
    its validation (the device passes, one host read per validation step)
    and reports the same validation / testing histories and dynamic negative
    weight as the same rows fed as host (x, y) batches through the HIP
    forward (_predict_all). Dropout off; the pools are whole batches, so both
    paths see exactly the same rows."""
    from heybuddy.trainer import EvalPasses, WakeWordTrainer
    rng = np.random.default_rng(21)
    vpos = torch.from_numpy((rng.standard_normal((100, 16, 96)) + 0.4).astype(np.float32)).cuda()
    vneg = torch.from_numpy(rng.standard_normal((400, 16, 96)).astype(np.float16)).cuda()
    tpos = torch.from_numpy((rng.standard_normal((60, 16, 96)) + 0.4).astype(np.float32)).cuda()
    tadv = torch.from_numpy((rng.standard_normal((60, 16, 96)) - 0.1).astype(np.float32)).cuda()
    xb = [torch.from_numpy(rng.standard_normal((64, 16, 96)).astype(np.float32) + 0.1 * (i % 2)) for i in range(9)]
    yb = [torch.cat([torch.ones(20), torch.zeros(44)]).long() for _ in range(9)]
    training = list(zip(xb, yb))
    # the same rows as host batches: validation 2 x (50 positives + 200 negatives), testing 3 x (20 + 20)
    val = [(torch.cat([vpos[50 * i:50 * i + 50], vneg[200 * i:200 * i + 200].float()]).cpu(),
            torch.cat([torch.ones(50), torch.zeros(200)]).long()) for i in range(2)]
    tst = [(torch.cat([tpos[20 * i:20 * i + 20], tadv[20 * i:20 * i + 20]]).cpu(),
            torch.cat([torch.ones(20), torch.zeros(20)]).long()) for i in range(3)]
    out = {}
    for mode in ("host", "device"):
        torch.manual_seed(3)
        tr = WakeWordTrainer(checkpoint_dir=str(tmp_path / mode), device="cuda")
        tr.model.dropout.p = 0.0
        kw = dict(num_steps=9, warmup_steps=2, hold_steps=2, validation_steps=4, negative_weight_schedule=2.0,
                  negative_weight_adjust_ratio=2.0, target_false_positive_rate=1e6)
        if mode == "host":
            h = tr.train_epoch(training, validation=val, testing=tst, **kw)
        else:
            ev = EvalPasses(tr, vpos, vneg, tpos, tadv, validation_batch=(50, 200), testing_batch=(20, 20))
            assert ev.rows_per_pass == 500 + 120
            h = tr.train_epoch(training, validation=ev, **kw)
        out[mode] = h
    for i in (1, 6, 7, 8, 9, 10):  # nw, vfp, vrecall, tacc, trecall, tfp
        np.testing.assert_allclose(out["device"][i].numpy(), out["host"][i].numpy(), rtol=1e-6, atol=1e-6)
    assert out["device"][1][-1] < 2.0  # the weight halved at the validations (fph under the target)
