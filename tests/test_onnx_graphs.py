"""Importing the reference's own pretrained graphs.

The reference runs ``speech-embedding.onnx`` and ``mel-spectrogram.onnx``
through ONNX Runtime (src/python/heybuddy/embeddings.py:23-42,
spectrogram.py:12-32, util/onnx_util.py:63-96). Neither file is in this
container, so the importers are checked on graphs the repo's own writers emit
in the layouts those files come in (Keras / tf2onnx for the embedding, the
torch export of torchaudio's MelSpectrogram -- STFT op or Conv1d DFT -- for the
mel front end):

* round trip: write -> import gives bit-identical weights / window / filterbank;
* semantics: oracle/onnx_eval.py (float64 numpy restatement of the ONNX ops,
  standing in for ONNX Runtime) runs the FILE, and its output matches the
  oracle run on the IMPORTED parameters (embedding 1e-9 relative in float64;
  mel 1e-4 absolute after the reference's /10 + 2, as the mel tests);
* hand-built variants (bias as an Add, Relu, NHWC transposes around every
  conv; an input scale, a dB offset) import to the right semantics;
* unsupported ops and attributes raise;
* the sha-checked pickup from the pretrained directory;
* on the GPU: the HIP kernels on the imported graph give the same output as on
  the original.
"""
import os

import numpy as np
import pytest
import torch

from oracle import embed as oembed
from oracle import mel as omel
from oracle import onnx_eval


def _se20():
    from heybuddy.embedding_graph import se20_graph
    return se20_graph(1234)


def _same_graph(g, h):
    from heybuddy.embedding_graph import Conv
    assert len(g.ops) == len(h.ops) and g.in_shape == h.in_shape
    for a, b in zip(g.ops, h.ops):
        assert type(a) is type(b)
        if isinstance(a, Conv):
            assert (a.kh, a.kw, a.cin, a.cout, a.act) == (b.kh, b.kw, b.cin, b.cout, b.act)
            np.testing.assert_array_equal(a.weight, b.weight)
            np.testing.assert_array_equal(a.bias, b.bias)
            assert np.float32(a.alpha) == np.float32(b.alpha) or a.act is None
        else:
            assert (a.ph, a.pw) == (b.ph, b.pw)


def test_embedding_graph_round_trip_and_semantics(tmp_path):
    from heybuddy.embedding_graph import from_onnx, to_onnx
    g = _se20()
    p = str(tmp_path / "speech-embedding.onnx")
    to_onnx(g, p)
    h = from_onnx(p)
    _same_graph(g, h)
    assert h.name == "conv2d_19" and h.out_dim == 96 and h.macs_per_window() == g.macs_per_window()
    x = np.random.default_rng(0).standard_normal((5, 76, 32, 1)) * 2.0 + 1.0
    got = onnx_eval.run(p, {"input_1": x})["conv2d_19"]  # the file, [n, 1, 1, 96]
    assert got.shape == (5, 1, 1, 96)
    ref = oembed.run_graph(h, x)
    np.testing.assert_allclose(got.reshape(5, 96), ref, rtol=1e-9, atol=1e-9 * np.abs(ref).max())


def _write_keras_variant(path, g, bias_as_add=True, relu=False, transpose_each=True):
    """SE20 as a less tidy tf2onnx export: biases as separate Adds ([1, C, 1, 1]),
    Relu / LeakyRelu applied in NHWC between transpose pairs, Squeeze + Reshape
    at the end."""
    from heybuddy.embedding_graph import Conv
    from heybuddy.util.onnx_util import write_model
    nodes, inits = [], {}
    x, nchw, k = "input_1", False, 0

    def t(perm):
        nonlocal x, k
        y = f"t{k}"
        k += 1
        nodes.append(("Transpose", y, [x], [y], {"perm": list(perm)}))
        x = y

    for i, op in enumerate(g.ops):
        if not nchw:
            t((0, 3, 1, 2))
            nchw = True
        if isinstance(op, Conv):
            inits[f"w{i}"] = np.ascontiguousarray(op.weight.transpose(3, 2, 0, 1))
            if bias_as_add:
                nodes.append(("Conv", f"conv{i}", [x, f"w{i}"], [f"c{i}"], {"kernel_shape": [op.kh, op.kw]}))
                inits[f"b{i}"] = op.bias.reshape(1, -1, 1, 1)
                nodes.append(("Add", f"badd{i}", [f"c{i}", f"b{i}"], [f"cb{i}"], {}))
                x = f"cb{i}"
            else:
                inits[f"b{i}"] = op.bias
                nodes.append(("Conv", f"conv{i}", [x, f"w{i}", f"b{i}"], [f"c{i}"], {"kernel_shape": [op.kh, op.kw]}))
                x = f"c{i}"
            if op.act == "leaky_relu":
                if transpose_each:
                    t((0, 2, 3, 1))
                    nchw = False
                if relu:
                    nodes.append(("Relu", f"act{i}", [x], [f"a{i}"], {}))
                else:
                    nodes.append(("LeakyRelu", f"act{i}", [x], [f"a{i}"], {"alpha": float(op.alpha)}))
                x = f"a{i}"
        else:
            nodes.append(("MaxPool", f"pool{i}", [x], [f"p{i}"], {"kernel_shape": [op.ph, op.pw],
                                                                  "strides": [op.ph, op.pw]}))
            x = f"p{i}"
    if nchw:
        t((0, 2, 3, 1))
    inits["shape"] = np.array([-1, 96], np.int64)
    nodes.append(("Reshape", "flat", [x, "shape"], ["emb"], {}))
    write_model(path, nodes, inits, [("input_1", ["n", 76, 32, 1])], [("emb", ["n", 96])])


@pytest.mark.parametrize("relu", [False, True])
def test_embedding_graph_keras_variants(tmp_path, relu):
    from heybuddy.embedding_graph import Conv, from_onnx
    g = _se20()
    p = str(tmp_path / "variant.onnx")
    _write_keras_variant(p, g, bias_as_add=not relu, relu=relu)
    h = from_onnx(p)
    for a, b in zip(g.ops, h.ops):
        if isinstance(a, Conv):
            np.testing.assert_array_equal(a.weight, b.weight)
            np.testing.assert_array_equal(a.bias, b.bias)
            if a.act:
                assert b.act == "leaky_relu" and b.alpha == (0.0 if relu else np.float32(a.alpha))
    x = np.random.default_rng(1).standard_normal((3, 76, 32, 1))
    got = onnx_eval.run(p, {"input_1": x})["emb"]
    np.testing.assert_allclose(got, oembed.run_graph(h, x), rtol=1e-9, atol=1e-12)


def _write_tf2onnx_variant(path, g, seed=0):
    """SE20 as tf2onnx exports a Keras model with BatchNorm layers: conv weights
    pre-scaled, each BatchNorm either folded by the exporter into a per-channel
    Mul + Add ([1, C, 1, 1]) after a bias-less Conv or left as a
    BatchNormalization node, and the final Reshape's target computed from the
    tensor's own Shape (Shape -> Gather -> Unsqueeze -> Concat)."""
    from heybuddy.embedding_graph import Conv
    from heybuddy.util.onnx_util import write_model
    rng = np.random.default_rng(seed)
    nodes, inits = [("Transpose", "t_in", ["input_1"], ["x0"], {"perm": [0, 3, 1, 2]})], {}
    x = "x0"
    for i, op in enumerate(g.ops):
        if not isinstance(op, Conv):
            nodes.append(("MaxPool", f"pool{i}", [x], [f"p{i}"], {"kernel_shape": [op.ph, op.pw],
                                                                  "strides": [op.ph, op.pw]}))
            x = f"p{i}"
            continue
        inits[f"w{i}"] = np.ascontiguousarray(op.weight.transpose(3, 2, 0, 1))
        c = op.cout
        if i % 2 == 0:  # folded: Conv (no bias) -> Mul s -> Add t
            nodes.append(("Conv", f"conv{i}", [x, f"w{i}"], [f"c{i}"], {"kernel_shape": [op.kh, op.kw]}))
            inits[f"s{i}"] = rng.uniform(0.5, 1.5, (1, c, 1, 1)).astype(np.float32)
            inits[f"t{i}"] = rng.standard_normal((1, c, 1, 1)).astype(np.float32) * 0.1
            nodes.append(("Mul", f"bnmul{i}", [f"c{i}", f"s{i}"], [f"m{i}"], {}))
            nodes.append(("Add", f"bnadd{i}", [f"m{i}", f"t{i}"], [f"n{i}"], {}))
        else:  # Conv (+ bias) -> BatchNormalization
            inits[f"b{i}"] = op.bias
            nodes.append(("Conv", f"conv{i}", [x, f"w{i}", f"b{i}"], [f"c{i}"], {"kernel_shape": [op.kh, op.kw]}))
            for k, v in (("g", rng.uniform(0.5, 1.5, c)), ("be", rng.standard_normal(c) * 0.1),
                         ("mu", rng.standard_normal(c) * 0.1), ("var", rng.uniform(0.5, 2.0, c))):
                inits[f"{k}{i}"] = v.astype(np.float32)
            nodes.append(("BatchNormalization", f"bn{i}", [f"c{i}", f"g{i}", f"be{i}", f"mu{i}", f"var{i}"],
                          [f"n{i}"], {"epsilon": 1e-3}))
        x = f"n{i}"
        if op.act == "leaky_relu":
            nodes.append(("LeakyRelu", f"act{i}", [x], [f"a{i}"], {"alpha": float(op.alpha)}))
            x = f"a{i}"
    nodes.append(("Transpose", "t_out", [x], ["xo"], {"perm": [0, 2, 3, 1]}))
    inits["i0"] = np.array(0, np.int64)
    inits["ax0"] = np.array([0], np.int64)
    inits["rest"] = np.array([-1], np.int64)
    nodes += [("Shape", "shp", ["xo"], ["shp_o"], {}),
              ("Gather", "gat", ["shp_o", "i0"], ["n_o"], {"axis": 0}),
              ("Unsqueeze", "unsq", ["n_o", "ax0"], ["cnt1"], {}),
              ("Concat", "cat", ["cnt1", "rest"], ["tgt"], {"axis": 0}),
              ("Reshape", "flat", ["xo", "tgt"], ["emb"], {})]
    write_model(path, nodes, inits, [("input_1", ["n", 76, 32, 1])], [("emb", ["n", 96])])


def test_embedding_graph_tf2onnx_batchnorm_and_computed_reshape(tmp_path):
    """BatchNorm (folded Mul / Add, or the op) is folded into the
    conv it follows, and a Reshape whose shape is computed from the tensor's Shape
    imports; the imported graph computes what the file computes."""
    from heybuddy.embedding_graph import from_onnx
    g = _se20()
    p = str(tmp_path / "tf2onnx_bn.onnx")
    _write_tf2onnx_variant(p, g)
    h = from_onnx(p)
    assert [type(o) for o in h.ops] == [type(o) for o in g.ops] and h.out_dim == 96
    x = np.random.default_rng(2).standard_normal((3, 76, 32, 1))
    got = onnx_eval.run(p, {"input_1": x})["emb"]
    assert got.shape == (3, 96)
    ref = oembed.run_graph(h, x)
    # (the fold rounds the scaled weights to f32: relative 1e-6, not the 1e-9 of an exact import)
    np.testing.assert_allclose(got, ref, rtol=2e-5, atol=2e-5 * np.abs(ref).max())


def test_embedding_graph_rejects_a_shape_branch_that_feeds_data(tmp_path):
    """A Shape side branch is allowed only when it ends in a Reshape's shape input."""
    from heybuddy.embedding_graph import from_onnx
    from heybuddy.util.onnx_util import read_model, write_model
    p = str(tmp_path / "tf2onnx_bn.onnx")
    _write_tf2onnx_variant(p, _se20())
    m = read_model(p)
    nodes = [(n.op, n.name, list(n.inputs), list(n.outputs), dict(n.attrs)) for n in m.nodes]
    # the computed count also scales the data: Shape -> ... -> Cast -> Mul into the chain
    k = next(i for i, n in enumerate(nodes) if n[0] == "Reshape")
    nodes[k:k] = [("Cast", "cst", ["n_o"], ["n_f"], {"to": 1}), ("Mul", "scale", ["xo", "n_f"], ["xs"], {})]
    nodes[-1] = ("Reshape", "flat", ["xs", "tgt"], ["emb"], {})
    q = str(tmp_path / "bad.onnx")
    write_model(q, nodes, dict(m.initializers), [(n, list(s)) for n, s in m.inputs],
                [(n, list(s)) for n, s in m.outputs])
    with pytest.raises(ValueError):
        from_onnx(q)


def _edit(tmp_path, mutate):
    """SE20's ONNX nodes through ``mutate(nodes, inits)``, rewritten."""
    from heybuddy.util.onnx_util import read_model, write_model
    from heybuddy.embedding_graph import to_onnx
    p = str(tmp_path / "base.onnx")
    to_onnx(_se20(), p)
    m = read_model(p)
    nodes = [(n.op, n.name, list(n.inputs), list(n.outputs), dict(n.attrs)) for n in m.nodes]
    inits = dict(m.initializers)
    mutate(nodes, inits)
    q = str(tmp_path / "edited.onnx")
    write_model(q, nodes, inits, [(n, list(s)) for n, s in m.inputs], [(n, list(s)) for n, s in m.outputs])
    return q


@pytest.mark.parametrize("case", ["unknown_op", "padded_conv", "strided_conv", "overlapping_pool", "branch"])
def test_embedding_graph_rejects_what_the_kernels_cannot_run(tmp_path, case):
    from heybuddy.embedding_graph import from_onnx

    def mutate(nodes, inits):
        i = next(k for k, n in enumerate(nodes) if n[0] == "LeakyRelu")
        if case == "unknown_op":
            nodes[i] = ("Sigmoid", nodes[i][1], nodes[i][2], nodes[i][3], {})
        elif case == "padded_conv":
            c = next(n for n in nodes if n[0] == "Conv")
            c[4]["pads"] = [1, 1, 1, 1]
        elif case == "strided_conv":
            c = next(n for n in nodes if n[0] == "Conv")
            c[4]["strides"] = [2, 1]
        elif case == "overlapping_pool":
            c = next(n for n in nodes if n[0] == "MaxPool")
            c[4]["strides"] = [1, 1]
        else:  # a second consumer of an activation
            nodes.insert(i + 1, ("Identity", "side", [nodes[i][3][0]], ["side_out"], {}))

    with pytest.raises(ValueError):
        from_onnx(_edit(tmp_path, mutate))


def _probe_audio(n=3, t=17280, seed=0):
    rng = np.random.default_rng(seed)
    tt = np.arange(t) / 16000.0
    x = 0.3 * np.sin(2 * np.pi * rng.uniform(100, 3000, (n, 1)) * tt) + 0.05 * rng.standard_normal((n, t))
    return (x * 32767.0).astype(np.float32)


@pytest.mark.parametrize("layout", ["stft", "conv"])
def test_mel_graph_round_trip_and_semantics(tmp_path, layout):
    from heybuddy.spectrogram import MelParams, mel_graph_to_onnx, mel_params_from_onnx, mel_parameters
    window, fbank = mel_parameters()
    p = str(tmp_path / f"mel-{layout}.onnx")
    mel_graph_to_onnx(p, MelParams(window, fbank), layout=layout)
    q = mel_params_from_onnx(p)
    if layout == "stft":
        np.testing.assert_array_equal(q.window, window)
    else:  # the window read back from the cos kernel's bin 0 (window * cos 0), exactly
        np.testing.assert_array_equal(q.window, window)
    np.testing.assert_array_equal(q.fbank, fbank)
    assert q.hop == 160 and q.n_fft == 512 and np.float32(q.log_floor) == np.float32(1e-10)
    assert abs(q.scale - 1.0) < 1e-6 and q.offset == 0.0 and q.in_scale == 1.0
    kw = q.plan_args()
    assert abs(kw["out_div"] - 10.0) < 1e-5 and kw["out_add"] == 2.0
    audio = _probe_audio()
    graph_out = onnx_eval.run(p, {"input": audio})["output"]  # [b, 1, 105, 32]
    assert graph_out.shape == (3, 1, 105, 32)
    host = np.squeeze(graph_out) / 10 + 2  # MelSpectrogramModel.__call__ (spectrogram.py:32)
    ref = omel.mel_spectrogram_model(audio, window=q.window, fbank=q.fbank, hop=q.hop, log_floor=q.log_floor)
    np.testing.assert_allclose(host, ref, atol=1e-4)


def test_mel_graph_input_scale_and_db_offset(tmp_path):
    """A graph that scales its input and offsets its dB output (the shapes an
    exporter of AmplitudeToDB with a reference level produces): the folded
    plan arguments reproduce the file's output."""
    from heybuddy.spectrogram import MelParams, mel_graph_to_onnx, mel_params_from_onnx, mel_parameters
    window, fbank = mel_parameters()
    p = str(tmp_path / "mel-scaled.onnx")
    mel_graph_to_onnx(p, MelParams(window, fbank, in_scale=0.5, offset=-3.0, scale=2.0), layout="conv")
    q = mel_params_from_onnx(p)
    assert q.in_scale == 0.5 and abs(q.offset + 3.0) < 1e-6 and abs(q.scale - 2.0) < 1e-6
    audio = _probe_audio(2, seed=1)
    host = np.squeeze(onnx_eval.run(p, {"input": audio})["output"]) / 10 + 2
    kw = q.plan_args()
    ref, _, _ = omel.mel_frames(audio, in_scale=q.in_scale, window=q.window, fbank=q.fbank, hop=q.hop,
                                log_floor=q.log_floor, out_div=kw["out_div"], out_add=kw["out_add"])
    np.testing.assert_allclose(host, ref, atol=1e-4)


@pytest.mark.parametrize("case", ["magnitude", "two_sided", "floor_before_fbank", "no_floor", "unknown_op",
                                  "not_dft"])
def test_mel_graph_rejects_what_the_kernel_cannot_run(tmp_path, case):
    from heybuddy.spectrogram import MelParams, mel_graph_to_onnx, mel_params_from_onnx, mel_parameters
    from heybuddy.util.onnx_util import read_model, write_model
    window, fbank = mel_parameters()
    p = str(tmp_path / "mel.onnx")
    mel_graph_to_onnx(p, MelParams(window, fbank), layout="conv" if case == "not_dft" else "stft")
    m = read_model(p)
    nodes = [(n.op, n.name, list(n.inputs), list(n.outputs), dict(n.attrs)) for n in m.nodes]
    inits = dict(m.initializers)
    idx = {n[1]: i for i, n in enumerate(nodes)}
    if case == "magnitude":  # sqrt of the power before the filterbank
        i = idx["mel"]
        nodes.insert(i, ("Sqrt", "mag", ["pw"], ["pw_mag"], {}))
        nodes[i + 1][2][0] = "pw_mag"
    elif case == "two_sided":
        nodes[idx["stft"]][4]["onesided"] = 0
    elif case == "floor_before_fbank":
        i = idx["mel"]
        nodes.insert(i, ("Clip", "early", ["pw", "amin"], ["pw_c"], {}))
        nodes[i + 1][2][0] = "pw_c"
    elif case == "no_floor":
        i = idx["clamp"]
        nodes[i + 1][2][0] = "mel"
        del nodes[i]
    elif case == "unknown_op":
        i = idx["log"]
        nodes[i] = ("Tanh", "log", nodes[i][2], nodes[i][3], {})
    else:  # a Conv kernel that is not window x DFT basis
        inits["dft_im"] = inits["dft_im"] * 1.01
    q = str(tmp_path / "bad.onnx")
    write_model(q, nodes, inits, [(n, list(s)) for n, s in m.inputs], [(n, list(s)) for n, s in m.outputs],
                opset_version=17)
    with pytest.raises(ValueError):
        mel_params_from_onnx(q)


def test_pretrained_files_are_picked_up_by_sha(tmp_path, monkeypatch):
    """MelSpectrogramModel / SpeechEmbeddingModel load the reference's files from
    the pretrained directory when their sha256 is the reference's (patched here
    to the sums of the files this test writes); a file with another sum is not
    used and the H0 / SE20 defaults stay."""
    from heybuddy import embeddings, spectrogram
    from heybuddy.embedding_graph import Graph, se20_graph, to_onnx
    from heybuddy.spectrogram import MelParams, mel_graph_to_onnx, mel_parameters
    from heybuddy.util.onnx_util import sha256_of
    monkeypatch.setenv("HEYBUDDY_PRETRAINED_DIR", str(tmp_path))
    g = se20_graph(77)  # weights that differ from the default SE20
    to_onnx(g, str(tmp_path / "speech-embedding.onnx"))
    window, fbank = mel_parameters()
    fb2 = fbank * np.float32(0.5)
    mel_graph_to_onnx(str(tmp_path / "mel-spectrogram.onnx"), MelParams(window, fb2), layout="stft")
    for sha_ok in (False, True):
        monkeypatch.setattr(embeddings, "_GRAPH", None)
        monkeypatch.setattr(spectrogram, "_PARAMS", [None])
        monkeypatch.setattr(embeddings, "REFERENCE_EMBED_SHA256",
                            sha256_of(str(tmp_path / "speech-embedding.onnx")) if sha_ok else "0" * 64)
        monkeypatch.setattr(spectrogram, "REFERENCE_MEL_SHA256",
                            sha256_of(str(tmp_path / "mel-spectrogram.onnx")) if sha_ok else "0" * 64)
        got = embeddings.default_graph()
        assert isinstance(got, Graph)
        w77 = g.ops[0].weight
        assert np.array_equal(got.ops[0].weight, w77) == sha_ok
        np.testing.assert_array_equal(spectrogram.mel_parameters()[1], fb2 if sha_ok else fbank)
    monkeypatch.setattr(embeddings, "_GRAPH", None)
    monkeypatch.setattr(spectrogram, "_PARAMS", [None])


@pytest.mark.gpu
def test_hip_output_on_imported_graphs_equals_original(tmp_path):
    """The HIP kernels on the imported graph / mel parameters against the same
    kernels on the originals: embedding bit-identical (identical plans), mel
    within 1e-6 (the dB scale read back from a float32 constant may move
    out_div by an ulp)."""
    from heybuddy.embedding_graph import WINDOW_STARTS, from_onnx, to_onnx
    from heybuddy.kernels import EmbedPlan, MelPlan, embed_clips, mel_frames
    from heybuddy.spectrogram import MelParams, mel_graph_to_onnx, mel_params_from_onnx, mel_parameters
    from heybuddy.synthetic import synthetic_clips
    dev = torch.device("cuda", 0)
    g = _se20()
    p = str(tmp_path / "se.onnx")
    to_onnx(g, p)
    h = from_onnx(p)
    clips = synthetic_clips(64, seed=5, device=dev)
    window, fbank = mel_parameters()
    base = MelPlan(window, fbank, in_scale=32767.0, device=dev)
    frames = mel_frames(clips, base, 141)
    outs = []
    for graph in (g, h):
        plan = EmbedPlan(graph, starts=WINDOW_STARTS, device=dev)
        outs.append(embed_clips(frames, plan))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    for layout in ("stft", "conv"):
        q = str(tmp_path / f"mel-{layout}.onnx")
        mel_graph_to_onnx(q, MelParams(window, fbank), layout=layout)
        prm = mel_params_from_onnx(q)
        plan = MelPlan(prm.window, prm.fbank, in_scale=32767.0 * prm.in_scale, device=dev, **prm.plan_args())
        got = mel_frames(clips, plan, 141)
        torch.testing.assert_close(got, frames, rtol=0, atol=1e-6)
