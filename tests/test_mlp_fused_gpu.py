"""The fused classifier train step (hbk_mlp_step_*, hbk_mlp_fused.hip) on the
GPU: against the reference's own outputs (tests/golden/classifier.npz), against
the generic GEMM path at the stage batch sizes 1100 / 550 / 273 (and ragged
ones), and the index-gathered multi-step graph (train_indexed) against eager
steps.

Tolerances: gradients 1e-4 of each tensor's max |g| (f32, summation order
and float-atomic order differ from torch's); loss 1e-5 relative.
"""
import numpy as np
import pytest
import torch

from oracle import golden_classifier as gc

pytestmark = pytest.mark.gpu

GOLD = "tests/golden/classifier.npz"


def _model(params):
    from heybuddy.wakeword import WakeWordMLPModel
    m = WakeWordMLPModel()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=True)
    m.dropout.p = 0.0
    return m.cuda()


def _fused_grads(model, x, y, neg_weight=2.0):
    plan = model.plan
    flat = model.flat_parameters
    bucket = torch.zeros(plan.n_params + plan.N_STATS, device="cuda")
    state = plan.new_state("cuda")
    xs = torch.as_tensor(x).cuda().reshape(len(x), -1).contiguous()
    ys = torch.as_tensor(y).cuda().to(torch.float32)
    prob = torch.zeros(len(x), device="cuda")
    plan.step_fwd_bwd(flat, bucket, state, 0, ys, len(x), pool32=xs, neg_weight=neg_weight, prob=prob)
    return bucket, prob


def test_fused_supported():
    from heybuddy.kernels import MlpPlan
    assert MlpPlan().fused
    assert not MlpPlan(layer_dim=64, hidden=48).fused


def test_fused_grads_match_reference():
    params, x, y, _ = gc.golden_inputs()
    gold = np.load(GOLD)
    m = _model(params)
    bucket, prob = _fused_grads(m, x, y)
    plan = m.plan
    stats = bucket[plan.n_params:].cpu().numpy()
    n_sel = int(gold["n_sel"])
    assert int(stats[0]) == n_sel
    np.testing.assert_allclose(stats[1] / n_sel, float(gold["loss"]), rtol=1e-5)
    np.testing.assert_allclose(prob.cpu().numpy(), gold["prob"], rtol=1e-4, atol=1e-6)
    g = plan.views(bucket[:plan.n_params] / n_sel)
    for k in params:
        ref = gold[f"grad/{k}"]
        scale = np.abs(ref).max() + 1e-12
        np.testing.assert_allclose(g[k].cpu().numpy() / scale, ref / scale, rtol=0, atol=1e-4, err_msg=k)


@pytest.mark.parametrize("B", [1100, 1000, 550, 500, 273, 100, 17, 1])
def test_fused_matches_generic_path(B):
    """Same step through the generic kernels (hbk_mlp_train_fwd_bwd) and the
    fused ones, at the reference's stage batch sizes, ragged tails and every
    K-split of the input GEMM (KS 8 / 12 / 16 / 24 at B 1100 / 550 / 500 / 273)."""
    params = gc.golden_inputs()[0]
    m = _model(params)
    rng = np.random.default_rng(B)
    y = (rng.random(B) < 0.1).astype(np.int64)
    x = (rng.standard_normal((B, 16, 96)) + np.where(y[:, None, None] == 1, 0.8, -0.2)).astype(np.float32)
    fused, _ = _fused_grads(m, x, y, neg_weight=1.5)
    plan = m.plan
    ref = torch.zeros_like(fused)
    plan.train_fwd_bwd(m.flat_parameters, torch.from_numpy(x).cuda().reshape(B, -1), torch.from_numpy(y), ref,
                       neg_weight=1.5)
    fs, rs = fused[plan.n_params:].cpu().numpy(), ref[plan.n_params:].cpu().numpy()
    np.testing.assert_array_equal(fs[[0, 2, 3, 4, 5, 6]], rs[[0, 2, 3, 4, 5, 6]])
    np.testing.assert_allclose(fs[1], rs[1], rtol=1e-5)
    gf, gr = plan.views(fused[:plan.n_params]), plan.views(ref[:plan.n_params])
    for k in gf:
        a, b = gf[k].cpu().numpy(), gr[k].cpu().numpy()
        scale = np.abs(b).max() + 1e-12
        np.testing.assert_allclose(a / scale, b / scale, rtol=0, atol=1e-4, err_msg=k)


def test_fused_update_matches_gate_adam():
    """hbk_mlp_step_update = hbk_mlp_gate_adam on the same bucket, and it
    zeroes the bucket and advances the ping-pong state."""
    params, x, y, _ = gc.golden_inputs()
    m = _model(params)
    plan = m.plan
    bucket, _ = _fused_grads(m, x, y)
    b2 = bucket.clone()
    p0 = m.flat_parameters.clone()
    mm, vv = torch.zeros_like(p0), torch.zeros_like(p0)
    state = plan.new_state("cuda")
    state[0] = 128.0  # earlier samples accumulated: the gate fires
    hist = torch.zeros((4, 8), device="cuda")
    plan.step_update(m.flat_parameters, bucket, mm, vv, state, 0, lr=1e-3, history=hist)
    new = m.flat_parameters.clone()
    # reference: the generic single-thread gate + Adam
    m.flat_parameters.copy_(p0)
    st2 = torch.tensor([128.0, 1.0, 0.0, 0.0], device="cuda")
    ctrl = torch.zeros(4, device="cuda")
    hist2 = torch.zeros((4, 8), device="cuda")
    plan.gate_adam(m.flat_parameters, b2, torch.zeros_like(p0), torch.zeros_like(p0), st2, ctrl, hist2, 1e-3)
    torch.testing.assert_close(new, m.flat_parameters, rtol=0, atol=0)
    torch.testing.assert_close(hist[0], hist2[0])
    assert float(bucket[:plan.n_params].abs().max()) == 0.0
    s = state.cpu().numpy()
    assert s[8 + 3] == 1.0 and s[8 + 2] == 1.0 and s[8 + 0] == 0.0 and s[8 + 1] == 1.0


def test_train_indexed_equals_eager_steps(tmp_path):
    """12 steps gathered by index from an f32 positive pool and an f16
    negative pool, as one 4-step graph replayed 3 times, against the same
    batches stepped eagerly from host tensors."""
    from heybuddy.trainer import WakeWordTrainer
    params = gc.golden_inputs()[0]
    rng = np.random.default_rng(5)
    S, npos, nneg = 12, 20, 80
    pos = torch.from_numpy(rng.standard_normal((300, 16, 96)).astype(np.float32) + 0.7)
    neg = torch.from_numpy(rng.standard_normal((500, 16, 96)).astype(np.float32)).half()
    ip = np.stack([rng.choice(300, npos, replace=False) for _ in range(S)])
    ineg = np.stack([rng.choice(500, nneg, replace=False) for _ in range(S)])
    idx = np.concatenate([ip, -ineg - 1], axis=1).astype(np.int32)
    y = np.concatenate([np.ones(npos), np.zeros(nneg)]).astype(np.float32)
    lr = np.linspace(1e-4, 1e-3, S).astype(np.float32)
    nw = np.tile([1.0, 2.0, 0.5], S // 3).astype(np.float32)
    runs = []
    for mode in ("indexed", "eager"):
        tr = WakeWordTrainer(checkpoint_dir=str(tmp_path / mode), device="cuda")
        tr.model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=True)
        tr.model.dropout.p = 0.0
        tr._reset_accumulation()
        hist = torch.zeros((S, 8), device="cuda")
        if mode == "indexed":
            sched = torch.from_numpy(np.stack([lr, nw], 1)).cuda()
            tr.train_indexed(torch.from_numpy(idx).cuda(), torch.from_numpy(y).cuda(), sched, pool32=pos.cuda(),
                             pool16=neg.cuda(), history=hist, steps_per_graph=4)
        else:
            for s in range(S):
                x = torch.cat([pos[ip[s]], neg[ineg[s]].float()])
                tr._step(x, torch.from_numpy(y).long(), float(lr[s]), float(nw[s]), 1e-4, 0.5, hist, s)
        torch.cuda.synchronize()
        runs.append((tr.model.flat_parameters.clone(), hist.clone(), tr._fstate.clone()))
    (p1, h1, s1), (p0, h0, s0) = runs
    np.testing.assert_allclose(h1[:, [0, 2, 4, 5, 6, 7]].cpu().numpy(), h0[:, [0, 2, 4, 5, 6, 7]].cpu().numpy())
    np.testing.assert_allclose(h1[:, 3].cpu().numpy(), h0[:, 3].cpu().numpy(), rtol=1e-4)
    d = (p1 - p0).abs()
    assert float((d > 1e-5).float().mean()) < 1e-3 and float(d.max()) <= 2e-2
    torch.testing.assert_close(s1, s0)


def test_train_indexed_split_with_eval_between_equals_one_call(tmp_path):
    """the headline splits every train chunk around the
    evaluation passes with train_indexed(n_steps=..., continued=True), whose
    first step relies on the previous call's last step having gathered its rows
    and refreshed the weight cache. S steps in one call against the same S
    steps split at k (an odd and an even split, each with an EvalPasses.run in
    between that does not touch sched: ratio 0), dropout on."""
    from heybuddy.trainer import EvalPasses, WakeWordTrainer
    params = gc.golden_inputs()[0]
    rng = np.random.default_rng(11)
    S, npos, nneg = 14, 24, 100
    pos = torch.from_numpy(rng.standard_normal((300, 16, 96)).astype(np.float32) + 0.7).cuda()
    neg = torch.from_numpy(rng.standard_normal((500, 16, 96)).astype(np.float32)).half().cuda()
    ip = np.stack([rng.choice(300, npos, replace=False) for _ in range(S)])
    ineg = np.stack([rng.choice(500, nneg, replace=False) for _ in range(S)])
    idx = torch.from_numpy(np.concatenate([ip, -ineg - 1], axis=1).astype(np.int32)).cuda()
    y = torch.from_numpy(np.concatenate([np.ones(npos), np.zeros(nneg)]).astype(np.float32)).cuda()
    lr = np.linspace(1e-4, 1e-3, S).astype(np.float32)
    sched0 = torch.from_numpy(np.stack([lr, np.full(S, 1.5, np.float32)], 1)).cuda()
    runs = {}
    for split in (None, (5,), (4, 9)):
        tr = WakeWordTrainer(checkpoint_dir=str(tmp_path / str(split)), device="cuda")
        tr.model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=True)
        tr.model.train()  # dropout 0.1 on: the prefetched rows carry the next step's mask
        tr._seed_base_v = 12345
        tr._reset_accumulation()
        hist = torch.zeros((S, 8), device="cuda")
        sched = sched0.clone()
        if split is None:
            tr.train_indexed(idx, y, sched, pool32=pos, pool16=neg, history=hist, steps_per_graph=4)
        else:
            ev = EvalPasses(tr, pos[:100], neg[:200], pos[100:150], pos[150:200], validation_batch=(10, 50),
                            testing_batch=(10, 10), adjust_ratio=0.0)
            done = 0
            for k in split:
                tr.train_indexed(idx, y, sched, pool32=pos, pool16=neg, history=hist, steps_per_graph=4,
                                 n_steps=k - done, continued=done > 0)
                done = k
                ev.run(sched, next_step=done)
            tr.train_indexed(idx, y, sched, pool32=pos, pool16=neg, history=hist, steps_per_graph=4,
                             n_steps=S - done, continued=True)
            torch.testing.assert_close(sched, sched0, rtol=0, atol=0)  # ratio 0: the passes leave sched alone
        torch.cuda.synchronize()
        runs[split] = (tr.model.flat_parameters.clone(), hist.clone(), tr._fstate.clone())
    p0, h0, s0 = runs[None]
    for split in ((5,), (4, 9)):
        p1, h1, s1 = runs[split]
        # as test_train_indexed_equals_eager_steps: counts / gate / selection, loss and parameters
        # to the float-atomic summation order (a wrong first step after a split moves them all)
        np.testing.assert_allclose(h1[:, [0, 2, 4, 5, 6, 7]].cpu().numpy(), h0[:, [0, 2, 4, 5, 6, 7]].cpu().numpy())
        np.testing.assert_allclose(h1[:, 3].cpu().numpy(), h0[:, 3].cpu().numpy(), rtol=1e-4)
        d = (p1 - p0).abs()
        assert float((d > 1e-5).float().mean()) < 1e-3 and float(d.max()) <= 2e-2
        torch.testing.assert_close(s1, s0)


@pytest.mark.parametrize("B", [1, 100, 273, 500, 550, 1000, 1100, 2000, 5000])
def test_fused_forward_matches_oracle(B):
    """Inference (hbk_mlp_forward: k1a + k1b + k2) against the oracle forward
    at every K-split of the input GEMM; probabilities within 1e-6."""
    from oracle import mlp as omlp
    params = gc.golden_inputs()[0]
    m = _model(params).eval()
    x = (np.random.default_rng(B).standard_normal((B, 16, 96)) * 1.3 + 0.2).astype(np.float32)
    p = m(torch.from_numpy(x).cuda()).cpu().numpy().ravel()
    po, _, _ = omlp.forward(params, x)
    np.testing.assert_allclose(p, po, rtol=0, atol=1e-6)


@pytest.mark.parametrize("B", [1100, 273])
def test_narrow_stream_weight_gradients_match(B):
    """On a stream masked to <= 96 CUs (the pipelined schedule's train stream)
    k3 runs with 128-row batch splits instead of 288, and from 800 rows the
    library switches to the v2 kernels (k1s / k1c / k3s: the input rows
    recomputed from the pool rows, no xhat^T); the gradients equal the wide
    (v1) launch's up to the split-K summation order."""
    from heybuddy.pipeline import masked_stream, train_cu_set
    params = gc.golden_inputs()[0]
    m = _model(params)
    rng = np.random.default_rng(7 + B)
    y = (rng.random(B) < 0.1).astype(np.int64)
    x = (rng.standard_normal((B, 16, 96)) + np.where(y[:, None, None] == 1, 0.8, -0.2)).astype(np.float32)
    wide, _ = _fused_grads(m, x, y, neg_weight=1.5)
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    ms = masked_stream(torch.device("cuda", 0), train_cu_set(n_cu, 64))
    with torch.cuda.stream(ms.stream):
        narrow, _ = _fused_grads(m, x, y, neg_weight=1.5)
    torch.cuda.synchronize()
    plan = m.plan
    ws_, ns_ = wide[plan.n_params:].cpu().numpy(), narrow[plan.n_params:].cpu().numpy()
    np.testing.assert_array_equal(ws_[[0, 2, 3, 4, 5, 6]], ns_[[0, 2, 3, 4, 5, 6]])
    gw, gn = plan.views(wide[:plan.n_params]), plan.views(narrow[:plan.n_params])
    for k in gw:
        a, b = gn[k].cpu().numpy(), gw[k].cpu().numpy()
        scale = np.abs(b).max() + 1e-12
        np.testing.assert_allclose(a / scale, b / scale, rtol=0, atol=1e-5, err_msg=k)


def test_v2_step_on_the_train_partition_equals_v1(tmp_path):
    """The v2 step (k1s / k1c / k3s, picked for >= 800 rows on a <= 128-CU stream:
    the pipelined headline's train partition) against v1 (the whole GPU) over 6
    graph-replayed train_indexed steps of B = 1,100 rows gathered from an f32 and
    an f16 pool, dropout on (k1s draws the same mask bits as k1a): counts, gate
    and selection exact, loss 1e-4, parameters to the summation order."""
    from heybuddy.pipeline import masked_stream, train_cu_set
    from heybuddy.trainer import WakeWordTrainer
    params = gc.golden_inputs()[0]
    rng = np.random.default_rng(23)
    S, npos, nneg = 6, 100, 1000
    pos = torch.from_numpy(rng.standard_normal((2000, 16, 96)).astype(np.float32) + 0.6).cuda()
    neg = torch.from_numpy(rng.standard_normal((4000, 16, 96)).astype(np.float32)).half().cuda()
    ip = np.stack([rng.choice(2000, npos, replace=False) for _ in range(S)])
    ineg = np.stack([rng.choice(4000, nneg, replace=False) for _ in range(S)])
    idx = torch.from_numpy(np.concatenate([ip, -ineg - 1], axis=1).astype(np.int32)).cuda()
    y = torch.from_numpy(np.concatenate([np.ones(npos), np.zeros(nneg)]).astype(np.float32)).cuda()
    sched = torch.from_numpy(np.stack([np.linspace(2e-4, 1e-3, S), np.full(S, 1.5)], 1).astype(np.float32)).cuda()
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    ms = masked_stream(torch.device("cuda", 0), train_cu_set(n_cu, 64))
    runs = {}
    for mode in ("v1", "v2"):
        tr = WakeWordTrainer(checkpoint_dir=str(tmp_path / mode), device="cuda")
        tr.model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=True)
        tr.model.train()
        tr._seed_base_v = 777
        tr._reset_accumulation()
        hist = torch.zeros((S, 8), device="cuda")
        if mode == "v2":
            ms.stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(ms.stream):
                tr.train_indexed(idx, y, sched, pool32=pos, pool16=neg, history=hist, steps_per_graph=4)
        else:
            tr.train_indexed(idx, y, sched, pool32=pos, pool16=neg, history=hist, steps_per_graph=4)
        torch.cuda.synchronize()
        runs[mode] = (tr.model.flat_parameters.clone(), hist.clone(), tr._fstate.clone())
    (p0, h0, s0), (p1, h1, s1) = runs["v1"], runs["v2"]
    np.testing.assert_allclose(h1[:, [0, 2, 4, 5, 6, 7]].cpu().numpy(), h0[:, [0, 2, 4, 5, 6, 7]].cpu().numpy())
    np.testing.assert_allclose(h1[:, 3].cpu().numpy(), h0[:, 3].cpu().numpy(), rtol=1e-4)
    d = (p1 - p0).abs()
    assert float((d > 1e-5).float().mean()) < 1e-3 and float(d.max()) <= 2e-2
    torch.testing.assert_close(s1, s0)


def test_train_epoch_device_iterator_runs_indexed_and_equals_eager(tmp_path, monkeypatch):
    """train_epoch over the CLI's device-pool iterators runs the
    measured path (the stage's rows drawn up front as pool indices, train_indexed
    hipGraph segments between the validation points, the validation / testing
    iterators as one EvalPasses each) and gives what the per-batch loop gives
    (HBK_TRAIN_EAGER=1: x gathered on the host side of the step, _predict_all over
    the iterators). Dropout off; the validation / testing pools are whole numbers of
    batches, so both evaluate the same rows. Tolerances as
    test_train_indexed_equals_eager_steps (the f16 rows' LayerNorm sums run in
    another order)."""
    from heybuddy.dataset.training import WakeWordTrainingDatasetIterator
    from heybuddy import trainer as trm
    params = gc.golden_inputs()[0]
    rng = np.random.default_rng(8)
    dev = torch.device("cuda")
    pos = torch.from_numpy(rng.standard_normal((300, 16, 96)).astype(np.float32) + 0.7).to(dev)
    adv = torch.from_numpy(rng.standard_normal((300, 16, 96)).astype(np.float32) - 0.2).to(dev)
    neg = torch.from_numpy(rng.standard_normal((2000, 16, 96)).astype(np.float32)).half().to(dev)
    vpos = torch.from_numpy(rng.standard_normal((100, 16, 96)).astype(np.float32) + 0.4).to(dev)
    vneg = torch.from_numpy(rng.standard_normal((400, 16, 96)).astype(np.float32)).half().to(dev)
    tpos = torch.from_numpy(rng.standard_normal((60, 16, 96)).astype(np.float32) + 0.4).to(dev)
    tadv = torch.from_numpy(rng.standard_normal((60, 16, 96)).astype(np.float32) - 0.1).to(dev)
    runs = {}
    for mode in ("fast", "eager"):
        monkeypatch.setenv("HBK_TRAIN_EAGER", "1" if mode == "eager" else "0")
        tr = trm.WakeWordTrainer(checkpoint_dir=str(tmp_path / mode), device="cuda")
        tr.model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=True)
        tr.model.dropout.p = 0.0
        training = WakeWordTrainingDatasetIterator(positive=[(pos, 20)], negative=[(adv, 20), (neg, 100)],
                                                   device=dev, seed=5)
        val = WakeWordTrainingDatasetIterator(positive=[(vpos, 50)], negative=[(vneg, 200)], device=dev, seed=6,
                                              max_samples=2)
        tst = WakeWordTrainingDatasetIterator(positive=[(tpos, 20)], negative=[(tadv, 20)], device=dev, seed=7,
                                              max_samples=3)
        called = []
        orig = trm.WakeWordTrainer.train_indexed
        monkeypatch.setattr(trm.WakeWordTrainer, "train_indexed",
                            lambda self, *a, **k: (called.append(k.get("n_steps")), orig(self, *a, **k))[1])
        h = tr.train_epoch(training, validation=val, testing=tst, num_steps=13, warmup_steps=3, hold_steps=3,
                           validation_steps=5, checkpoint_steps=1000, negative_weight_schedule=2.0,
                           negative_weight_adjust_ratio=2.0, target_false_positive_rate=1e6)
        torch.cuda.synchronize()
        runs[mode] = (h, tr.model.flat_parameters.clone(), called)
    (hf, pf, cf), (he, pe, ce) = runs["fast"], runs["eager"]
    assert cf == [6, 5, 2] and ce == []  # segments up to the validations after steps 5 and 10, then the rest
    for i in (0, 1):  # lr, negative weight
        np.testing.assert_allclose(hf[i].numpy(), he[i].numpy(), rtol=1e-6)
    np.testing.assert_allclose(hf[2].numpy(), he[2].numpy(), rtol=2e-4)  # loss
    for i in (6, 7, 8, 9, 10):  # validation fp/h, recall; testing accuracy, recall, fp rate
        np.testing.assert_allclose(hf[i].numpy(), he[i].numpy(), rtol=1e-5, atol=1e-5)
    d = (pf - pe).abs()
    assert float((d > 1e-5).float().mean()) < 1e-3 and float(d.max()) <= 2e-2
