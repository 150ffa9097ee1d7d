"""The reference's shipped wake-word heads (src/js/models/*.onnx) through
heybuddy.util.onnx_util and the HIP forward.

Fixture tests/golden/onnx_heads.npz (oracle/make_golden.py --only onnx) holds
the reference WakeWordMLPModel's outputs for every shipped head on zeros (the
wake-word.js:33-47 KAT input) and, for two heads, their weights and outputs on
seeded embeddings. Tolerance: probabilities rtol 1e-4, atol 1e-6 (f32 forward,
different summation order).
"""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import mlp as omlp

GOLD = "tests/golden/onnx_heads.npz"
MODELS = "/root/reference/src/js/models"
HEADS = ("hey-buddy", "okay-buddy")


def _weights(gold, name):
    pre = f"w/{name}/"
    return {k[len(pre):]: gold[k] for k in gold.files if k.startswith(pre)}


def test_fixture_pins_the_oracle_forward():
    gold = np.load(GOLD)
    for name in HEADS:
        p, _, _ = omlp.forward(_weights(gold, name), gold["x"])
        np.testing.assert_allclose(p, gold[f"prob/{name}"], rtol=1e-5, atol=1e-7, err_msg=name)
        assert 0.0 <= float(gold[f"zeros/{name}"][0]) <= 1.0


@pytest.mark.skipif(not os.path.isdir(MODELS), reason="reference ONNX heads only in the build container")
def test_reader_on_shipped_heads(tmp_path):
    from heybuddy.util.onnx_util import read_initializers, read_nodes
    from heybuddy.wakeword import WakeWordMLPModel
    gold = np.load(GOLD)
    paths = sorted(glob.glob(os.path.join(MODELS, "*.onnx")))
    assert len(paths) == 7
    for path in paths:
        name = os.path.basename(path)[:-5]
        sd = read_initializers(path)
        model = WakeWordMLPModel.from_file(path)  # strict load, shapes from the file
        ours = model.state_dict()
        assert list(sd) == list(ours)
        for k, v in sd.items():
            assert v.dtype == np.float32 and tuple(v.shape) == tuple(ours[k].shape), k
            np.testing.assert_array_equal(ours[k].numpy(), v)
        p, _, _ = omlp.forward(sd, np.zeros((1, 16, 96), np.float32))
        np.testing.assert_allclose(p, gold[f"zeros/{name}"], rtol=1e-5, err_msg=name)
        if name in HEADS:
            for k, v in _weights(gold, name).items():
                np.testing.assert_array_equal(sd[k], v)
        # save_onnx writes the exporter's graph: same nodes, same tensors
        out = str(tmp_path / f"{name}.onnx")
        model.save_onnx(out)
        assert read_nodes(out) == read_nodes(path)
        back = read_initializers(out)
        assert list(back) == list(sd) and all(np.array_equal(back[k], sd[k]) for k in sd)


def test_writer_reader_roundtrip(tmp_path):
    from heybuddy.util.onnx_util import read_initializers, read_nodes, write_wakeword_onnx
    sd = omlp.init_params(seed=3, num_layers=1)
    sd = {k: np.asarray(v, np.float32) for k, v in sd.items()}
    path = str(tmp_path / "h.onnx")
    write_wakeword_onnx(path, sd, num_layers=1)
    back = read_initializers(path)
    assert set(back) == set(sd)
    for k in sd:
        np.testing.assert_array_equal(back[k], sd[k])
    ops = [n[0] for n in read_nodes(path)]
    assert ops[0] == "Flatten" and ops[-1] == "Sigmoid" and ops.count("LayerNormalization") == 3
    assert ops.count("Gemm") == 3 * 3


def test_timecodes_rule():
    from heybuddy.wakeword import WakeWordMLPModel
    tc = WakeWordMLPModel.timecodes
    assert tc([False, True, True, False]) == [1.5, 2]  # the reference rule, wakeword.py:99-110
    assert tc([True, False, True]) == [0, 2]
    assert tc([False, True, True]) == [1.5]  # last window after a positive one: skipped
    assert tc([True]) == []  # predictions[i - 1] wraps to itself in the reference: skipped
    w = WakeWordMLPModel.timecode_windows(torch.arange(40000, dtype=torch.float32))
    # 40000 -> padded to 48000, + 1 s each side = 80000 -> starts 0, 16000, 32000, 48000
    assert tuple(w.shape) == (4, 1, 32000)
    assert float(w[0, 0, 16000]) == 0.0 and float(w[1, 0, 1]) == 1.0 and float(w[3, 0, 0]) == 32000.0


@pytest.mark.gpu
def test_shipped_heads_on_hip():
    from heybuddy.wakeword import WakeWordMLPModel
    gold = np.load(GOLD)
    x = torch.from_numpy(gold["x"]).cuda()
    for name in HEADS:
        m = WakeWordMLPModel()
        m.load_state_dict({k: torch.from_numpy(v) for k, v in _weights(gold, name).items()}, strict=True)
        m = m.cuda().eval()
        p = m(x).cpu().numpy().reshape(-1)
        np.testing.assert_allclose(p, gold[f"prob/{name}"], rtol=1e-4, atol=1e-6, err_msg=name)
        z = float(m(torch.zeros(1, 16, 96, device="cuda"))[0, 0])  # the JS KAT
        assert 0.0 <= z <= 1.0
        np.testing.assert_allclose(z, gold[f"zeros/{name}"][0], rtol=1e-4, atol=1e-7)
