"""Classifier oracle pinned to the reference (CPU).

tests/golden/classifier.npz holds the reference's own outputs
(WakeWordMLPModel forward, the trainer's filtered weighted BCE + autograd
gradients, one torch.optim.Adam step, a 24-step WakeWordTrainer.train_epoch)
on inputs regenerated here from seeds (oracle.golden_classifier.golden_inputs).
"""
import os

import numpy as np
import pytest

from oracle import golden_classifier as gc
from oracle import mlp as omlp

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "classifier.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


@pytest.fixture(scope="module")
def inputs():
    return gc.golden_inputs()


def test_param_count_and_names(inputs):
    params = inputs[0]
    assert sum(v.size for v in params.values()) == 256417
    assert list(params)[:3] == ["norm_in.weight", "norm_in.bias", "mlp_in.hidden.weight"]


def test_forward_logits(gold, inputs):
    params, x, y, _ = inputs
    prob, z, _ = omlp.forward(params, x)
    np.testing.assert_allclose(z, gold["logit"], rtol=0, atol=1e-4)   # north star: logits 1e-4
    np.testing.assert_allclose(prob, gold["prob"], rtol=1e-5, atol=1e-6)


def test_filtered_bce_and_gradients(gold, inputs):
    params, x, y, _ = inputs
    prob, z, cache = omlp.forward(params, x)
    loss, n, dz = omlp.step_loss_and_dz(prob, y, neg_weight=2.0)
    assert n == int(gold["n_sel"])
    np.testing.assert_allclose(loss, float(gold["loss"]), rtol=1e-5)
    grads = omlp.backward(params, cache, dz)
    for k, g in grads.items():
        ref = gold[f"grad/{k}"]
        scale = np.abs(ref).max() + 1e-12
        np.testing.assert_allclose(g / scale, ref / scale, rtol=0, atol=2e-5, err_msg=k)


def test_adam_step(gold, inputs):
    params, x, y, _ = inputs
    grads = {k: gold[f"grad/{k}"].astype(np.float64) for k in params}
    new = omlp.Adam(params).step({k: v.astype(np.float64) for k, v in params.items()}, grads)
    for k in params:
        np.testing.assert_allclose(new[k], gold[f"adam1/{k}"], rtol=0, atol=1e-6, err_msg=k)


def test_learning_rate_schedule(gold):
    lr = [omlp.learning_rate(s, 4, 8, 24, 1e-3) for s in range(24)]
    np.testing.assert_allclose(lr, gold["epoch/lr"], rtol=1e-6, atol=1e-12)


def test_train_epoch_histories(gold, inputs):
    params, _, _, batches = inputs
    final, hist = omlp.train_epoch(params, batches, 24, 4, 8)
    assert len(hist["loss"]) == len(gold["epoch/loss"])
    np.testing.assert_allclose(hist["high_loss_rate"], gold["epoch/hlr"], rtol=1e-6)
    np.testing.assert_allclose(hist["loss"], gold["epoch/loss"], rtol=2e-4, atol=1e-6)
    # the gate both skipped and fired in this schedule
    assert 0 < sum(hist["updated"]) < 24
    for k in params:
        ref = gold[f"epoch_final/{k}"]
        np.testing.assert_allclose(final[k], ref, rtol=0, atol=2e-4, err_msg=k)
