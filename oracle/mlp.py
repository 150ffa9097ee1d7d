"""Wake-word classifier oracle (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

numpy (fp64 by default) restatement of:
  * WakeWordMLPModel.forward (reference src/python/heybuddy/wakeword.py:334-348)
    with GatedMultiLayerPerceptron (modules/multi_layer_perceptron.py:76-124):
    x -> flatten -> LN(1536) -> GMLP_in -> [LN(96) -> GMLP]*L -> LN(96) ->
    GMLP_out -> sigmoid; GMLP(x) = W_o (silu(W_h x + b_h) * (W_g x + b_g)) + b_o;
    hidden = get_normalized_dim(layer_dim) (modeling_util.py:42-72), LN eps 1e-5.
  * the train step of WakeWordTrainer.train_epoch (trainer.py:380-494): high-loss
    filter (negatives with p >= thr, then positives with p < 1 - thr), weighted
    BCE (torch binary_cross_entropy: log clamped at -100), the < 128-sample
    accumulation gate, backward (torch's BCE / sigmoid backward formulas) and
    torch.optim.Adam (betas 0.9/0.999, eps 1e-8, no weight decay, trainer.py:45).
  * Trainer.get_learning_rate (trainer.py:127-156).
Pinned against the reference itself (tests/golden/classifier.npz).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np

LN_EPS = 1e-5


def normalized_dim(dim: int, multiple_of: int = 8, down_ratio: float = 2 / 3) -> int:
    v = int(dim * down_ratio)
    return v if v % multiple_of == 0 else v + multiple_of - v % multiple_of


def param_shapes(input_shape=(16, 96), layer_dim: int = 96, num_layers: int = 2):
    """state_dict names and shapes of WakeWordMLPModel (gated, no half layers)."""
    d_in = input_shape[0] * input_shape[1]
    hid = normalized_dim(layer_dim)
    shapes = OrderedDict()
    shapes["norm_in.weight"] = (d_in,)
    shapes["norm_in.bias"] = (d_in,)

    def gmlp(prefix, i, o):
        shapes[f"{prefix}.hidden.weight"] = (hid, i)
        shapes[f"{prefix}.hidden.bias"] = (hid,)
        shapes[f"{prefix}.output.weight"] = (o, hid)
        shapes[f"{prefix}.output.bias"] = (o,)
        shapes[f"{prefix}.gate.weight"] = (hid, i)
        shapes[f"{prefix}.gate.bias"] = (hid,)

    gmlp("mlp_in", d_in, layer_dim)
    for l in range(num_layers):
        shapes[f"layers.{l}.0.weight"] = (layer_dim,)
        shapes[f"layers.{l}.0.bias"] = (layer_dim,)
        gmlp(f"layers.{l}.1", layer_dim, layer_dim)
    shapes["norm_out.weight"] = (layer_dim,)
    shapes["norm_out.bias"] = (layer_dim,)
    gmlp("mlp_out", layer_dim, 1)
    return shapes


def init_params(seed: int = 0, input_shape=(16, 96), layer_dim=96, num_layers=2, scale=1.0):
    """Seeded weights (nn.Linear-like uniform fan-in init; LN affine near 1/0)."""
    rng = np.random.default_rng(seed)
    p = OrderedDict()
    for name, shp in param_shapes(input_shape, layer_dim, num_layers).items():
        if name.endswith(".weight") and len(shp) == 1:      # LayerNorm gamma
            p[name] = 1.0 + 0.1 * rng.standard_normal(shp)
        elif name.endswith(".bias") and ("norm" in name or name.endswith(".0.bias")):
            p[name] = 0.1 * rng.standard_normal(shp)
        else:
            fan_in = shp[-1] if len(shp) == 2 else shp[0]
            b = 1.0 / math.sqrt(fan_in)
            p[name] = rng.uniform(-b, b, shp) * scale
    return OrderedDict((k, v.astype(np.float32)) for k, v in p.items())


def _silu(x):
    return x / (1.0 + np.exp(-x))


def _ln(x, g, b):
    mu = x.mean(axis=1, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=1, keepdims=True)
    rstd = 1.0 / np.sqrt(var + LN_EPS)
    xh = (x - mu) * rstd
    return xh * g + b, xh, rstd


def _gmlp(p, prefix, x, cache):
    h = x @ p[f"{prefix}.hidden.weight"].T + p[f"{prefix}.hidden.bias"]
    g = x @ p[f"{prefix}.gate.weight"].T + p[f"{prefix}.gate.bias"]
    u = _silu(h) * g
    out = u @ p[f"{prefix}.output.weight"].T + p[f"{prefix}.output.bias"]
    cache[prefix] = (x, h, g, u)
    return out


def forward(params, x, num_layers=None, dtype=np.float64):
    """x [B, 16, 96] -> (p [B], z [B] pre-sigmoid logits, cache)."""
    p = {k: np.asarray(v, dtype=dtype) for k, v in params.items()}
    if num_layers is None:
        num_layers = sum(1 for k in p if k.startswith("layers.") and k.endswith(".0.weight"))
    x = np.asarray(x, dtype=dtype).reshape(x.shape[0], -1)
    cache = {}
    xn, xh, rs = _ln(x, p["norm_in.weight"], p["norm_in.bias"])
    cache["norm_in"] = (xh, rs)
    s = _gmlp(p, "mlp_in", xn, cache)
    for l in range(num_layers):
        xn, xh, rs = _ln(s, p[f"layers.{l}.0.weight"], p[f"layers.{l}.0.bias"])
        cache[f"layers.{l}.0"] = (xh, rs)
        s = _gmlp(p, f"layers.{l}.1", xn, cache)
    xn, xh, rs = _ln(s, p["norm_out.weight"], p["norm_out.bias"])
    cache["norm_out"] = (xh, rs)
    z = _gmlp(p, "mlp_out", xn, cache)[:, 0]
    prob = 1.0 / (1.0 + np.exp(-z))
    cache["num_layers"] = num_layers
    return prob, z, cache


def select_high_loss(prob, y, threshold=1e-4):
    """trainer.py:407-424: indices of negatives with p >= thr, then positives
    with p < 1 - thr (in that order)."""
    neg = np.nonzero((y == 0) & (prob >= threshold))[0]
    pos = np.nonzero((y == 1) & (prob < 1 - threshold))[0]
    return np.concatenate([neg, pos])


def bce_terms(prob, y):
    """torch binary_cross_entropy per element (log clamped at -100)."""
    lp = np.maximum(np.log(prob), -100.0)
    l1p = np.maximum(np.log(1.0 - prob), -100.0)
    return -(y * lp + (1.0 - y) * l1p)


def _gmlp_back(p, grads, prefix, dout, cache):
    x, h, g, u = cache[prefix]
    grads[f"{prefix}.output.weight"] = dout.T @ u
    grads[f"{prefix}.output.bias"] = dout.sum(axis=0)
    du = dout @ p[f"{prefix}.output.weight"]
    sig = 1.0 / (1.0 + np.exp(-h))
    dh = du * g * (sig * (1.0 + h * (1.0 - sig)))
    dg = du * h * sig
    grads[f"{prefix}.hidden.weight"] = dh.T @ x
    grads[f"{prefix}.hidden.bias"] = dh.sum(axis=0)
    grads[f"{prefix}.gate.weight"] = dg.T @ x
    grads[f"{prefix}.gate.bias"] = dg.sum(axis=0)
    return dh @ p[f"{prefix}.hidden.weight"] + dg @ p[f"{prefix}.gate.weight"]


def _ln_back(grads, name, dy, gamma, cache):
    xh, rstd = cache[name]
    grads[f"{name}.weight"] = (dy * xh).sum(axis=0)
    grads[f"{name}.bias"] = dy.sum(axis=0)
    dxh = dy * gamma
    d = dxh.shape[1]
    return rstd * (dxh - dxh.mean(axis=1, keepdims=True) - xh * (dxh * xh).mean(axis=1, keepdims=True))


def backward(params, cache, dz, dtype=np.float64):
    """Gradients of sum_i dz_i * z_i w.r.t. every parameter (dz [B] = dL/dz)."""
    p = {k: np.asarray(v, dtype=dtype) for k, v in params.items()}
    grads = OrderedDict()
    L = cache["num_layers"]
    ds = _gmlp_back(p, grads, "mlp_out", dz[:, None], cache)
    ds = _ln_back(grads, "norm_out", ds, p["norm_out.weight"], cache)
    for l in reversed(range(L)):
        ds = _gmlp_back(p, grads, f"layers.{l}.1", ds, cache)
        ds = _ln_back(grads, f"layers.{l}.0", ds, p[f"layers.{l}.0.weight"], cache)
    ds = _gmlp_back(p, grads, "mlp_in", ds, cache)
    _ln_back(grads, "norm_in", ds, p["norm_in.weight"], cache)
    return OrderedDict((k, grads[k]) for k in params)


def step_loss_and_dz(prob, y, neg_weight=1.0, threshold=1e-4, acc_steps=1):
    """Filtered weighted BCE of one step and dL/dz for every sample of the
    batch (0 for the unselected). Returns (loss, n_sel, dz [B])."""
    sel = select_high_loss(prob, y, threshold)
    n = sel.size
    dz = np.zeros_like(prob)
    if n == 0:
        return 0.0, 0, dz
    ps, ys = prob[sel], y[sel].astype(prob.dtype)
    w = np.where(ys == 1, 1.0, neg_weight)
    loss = float((w * bce_terms(ps, ys)).mean() / acc_steps)
    # torch: dL/dp = w (p - y) / max(p (1 - p), 1e-12) / n; sigmoid backward * p (1 - p)
    dp = w * (ps - ys) / np.maximum((1.0 - ps) * ps, 1e-12) / n / acc_steps
    dz[sel] = dp * (1.0 - ps) * ps
    return loss, n, dz


class Adam:
    """torch.optim.Adam, single-tensor (foreach) semantics, amsgrad False."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.m = OrderedDict((k, np.zeros_like(v, dtype=np.float64)) for k, v in params.items())
        self.v = OrderedDict((k, np.zeros_like(v, dtype=np.float64)) for k, v in params.items())
        self.t = 0

    def step(self, params, grads, lr=None):
        lr = self.lr if lr is None else lr
        self.t += 1
        bc1 = 1.0 - self.b1 ** self.t
        bc2 = 1.0 - self.b2 ** self.t
        out = OrderedDict()
        for k, p in params.items():
            g = grads[k]
            self.m[k] = self.b1 * self.m[k] + (1 - self.b1) * g
            self.v[k] = self.b2 * self.v[k] + (1 - self.b2) * g * g
            denom = np.sqrt(self.v[k]) / math.sqrt(bc2) + self.eps
            out[k] = p - (lr / bc1) * self.m[k] / denom
        return out


def learning_rate(step, warmup_steps=0, hold_steps=0, total_steps=0, target=1e-3):
    """Trainer.get_learning_rate (trainer.py:127-156)."""
    lr = 0.5 * target * (1 + np.cos(np.pi * (step - warmup_steps - hold_steps)
                                    / float(total_steps - warmup_steps - hold_steps)))
    warm = target * (step / warmup_steps) if warmup_steps > 0 else 0.0
    if hold_steps > 0:
        lr = np.where(step > warmup_steps + hold_steps, lr, target)
    return float(np.where(step < warmup_steps, warm, lr))


def train_epoch(params, batches, num_steps, warmup_steps, hold_steps, learning_rate_target=1e-3,
                neg_weight=1.0, threshold=1e-4, dtype=np.float64, last_loss=0.0):
    """Restatement of WakeWordTrainer.train_epoch's optimisation path and its
    loss-history bookkeeping (trainer.py:380-494; no validation / testing /
    checkpoints). Returns (params, history dict)."""
    params = OrderedDict((k, np.asarray(v, dtype=dtype)) for k, v in params.items())
    opt = Adam(params)
    acc_steps, acc_samples = 1, 0
    hist = {"lr": [], "loss": [], "high_loss_rate": [], "updated": []}
    for step, (x, y) in enumerate(batches):
        if step >= num_steps:
            break
        lr = learning_rate(step, warmup_steps, hold_steps, num_steps, learning_rate_target)
        hist["lr"].append(lr)
        prob, z, cache = forward(params, x, dtype=dtype)
        sel = select_high_loss(prob, y, threshold)
        hist["high_loss_rate"].append(sel.size / prob.shape[0])
        updated = False
        if sel.size:
            loss, n, dz = step_loss_and_dz(prob, y, neg_weight, threshold, acc_steps)
            acc_samples += n
            if acc_samples < 128:
                acc_steps += 1
                if hist["loss"]:
                    hist["loss"].append(hist["loss"][-1])
            else:
                grads = backward(params, cache, dz, dtype)
                params = opt.step(params, grads, lr)
                acc_steps, acc_samples = 1, 0
                hist["loss"].append(loss)
                updated = True
        elif hist["loss"]:
            hist["loss"].append(hist["loss"][-1])
        else:
            hist["loss"].append(last_loss)
        hist["updated"].append(updated)
    return params, hist


def flat_bucket(params, x, y, neg_weight=1.0, threshold=1e-4, act_thr=0.5):
    """What hbk_mlp_train_fwd_bwd leaves in its bucket: the UNNORMALISED
    gradient sum over the selected samples of w * dl/dz (state_dict order,
    flattened) and the 8 statistics [n_sel, sum w*l, n_neg_sel, fp_sel,
    n_pos_sel, tp_sel, batch, 0]."""
    prob, z, cache = forward(params, x)
    sel = select_high_loss(prob, y, threshold)
    dz = np.zeros_like(prob)
    stats = np.zeros(8)
    stats[6] = prob.shape[0]
    if sel.size:
        ps, ys = prob[sel], y[sel].astype(np.float64)
        w = np.where(ys == 1, 1.0, neg_weight)
        dz[sel] = w * (ps - ys)
        stats[0] = sel.size
        stats[1] = float((w * bce_terms(ps, ys)).sum())
        neg = ys == 0
        stats[2] = neg.sum()
        stats[3] = (neg & (ps >= act_thr)).sum()
        stats[4] = (~neg).sum()
        stats[5] = ((~neg) & (ps > act_thr)).sum()
    grads = backward(params, cache, dz)
    return np.concatenate([g.reshape(-1) for g in grads.values()]), stats


# ------------------------------------------------------------ evaluation ----
def dropout_keep(seed: int, row_ids, d: int = 1536, p: float = 0.1) -> np.ndarray:
    """The counter-based input-dropout mask of the HIP kernels (k1a_tile /
    kv_gemm_kernel, hbk_mlp_fused.hip: drop_hash): element c of row r is dropped
    iff a 16-bit uniform from hash(seed, r * d / 2 + c / 2) (low half for even c,
    high half for odd c) is below round(p * 65536). [n, d] bool (True = kept).
    The reference draws torch's Philox mask instead; only the rate matches."""
    m32 = np.uint64(0xFFFFFFFF)
    s0 = np.uint64(seed) & m32
    s1 = ((np.uint64(seed) >> np.uint64(32)) * np.uint64(0x27D4EB2F)) & m32
    r = np.asarray(row_ids, dtype=np.uint64)[:, None]
    i = (r * np.uint64(d // 2) + np.arange(d // 2, dtype=np.uint64)[None, :]) & m32
    h = (i * np.uint64(0x9E3779B1) + s0) & m32
    h ^= s1
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & m32
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & m32
    h ^= h >> np.uint64(16)
    thr = np.uint64(int(p * 65536.0 + 0.5))
    keep = np.empty((r.shape[0], d), dtype=bool)
    keep[:, 0::2] = (h & np.uint64(0xFFFF)) >= thr
    keep[:, 1::2] = (h >> np.uint64(16)) >= thr
    return keep


def eval_counts(prob, label: int, activation_threshold: float = 0.5) -> np.ndarray:
    """counts [4] of one labelled set: [2 label] = #(p >= thr), [2 label + 1] = #(p > thr)."""
    c = np.zeros(4)
    c[2 * label] = float((prob >= activation_threshold).sum())
    c[2 * label + 1] = float((prob > activation_threshold).sum())
    return c


def eval_finish(cv, ct, sizes, nw_before: float, target: float = 1.5, ratio: float = 2.0):
    """trainer.py:511-536, :552-561 on the counts: validation false positives per
    hour (an integer count tensor / a Python float -> float32), recall
    (preds > threshold over the positives), the testing false-positive rate,
    recall and accuracy, and the dynamic negative weight."""
    n_neg_v, n_pos_v, n_neg_t, n_pos_t = sizes
    hours = np.float32(n_neg_v * 1.44 / 3600)
    with np.errstate(divide="ignore", invalid="ignore"):
        fph = np.float32(cv[0]) / hours
    rec = cv[3] / n_pos_v if n_pos_v > 0 else 0.0
    nw = nw_before
    if ratio > 0:
        nw = nw_before * ratio if fph > target else max(1.0, nw_before / ratio)
    out = [float(fph), rec]
    if ct is not None:
        out += [ct[0] / max(n_neg_t, 1.0), ct[3] / n_pos_t if n_pos_t > 0 else 0.0,
                (ct[3] + (n_neg_t - ct[1])) / max(n_neg_t + n_pos_t, 1.0)]
    else:
        out += [0.0, 0.0, 0.0]
    return np.array(out + [nw, nw_before, 0.0])
