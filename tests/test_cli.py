"""``heybuddy train`` drop-in (reference src/python/heybuddy/__main__.py:171-429).

CPU: the command keeps the reference's option names and defaults; the
synthetic phrase generator is deterministic and phrase-specific.
GPU: a short two-stage run end to end (augment -> featurize -> train ->
validate -> test -> checkpoint) learns the phrase against adversarial clips.
"""
import os

import pytest
import torch
from click.testing import CliRunner

from heybuddy.__main__ import main, safe_name
from heybuddy.synthetic import phrase_clips

# Options of the reference's `train` on the hot path (__main__.py:171-300).
REFERENCE_OPTIONS = [
    "--additional-phrase", "--wandb-entity", "--perceptron", "--transformer", "--use-half-layers",
    "--use-gating", "--layer-dim", "--num-layers", "--steps", "--stages", "--threshold",
    "--learning-rate", "--high-loss-threshold", "--target-false-positive-rate",
    "--dynamic-negative-weight", "--negative-weight", "--augmentation-background-noise-prob",
    "--augmentation-background-noise-min-snr-db", "--augmentation-background-noise-max-snr-db",
    "--augmentation-reverb-prob", "--augmentation-gain-prob", "--logging-steps", "--validation-steps", "--checkpoint-steps",
    "--positive-samples", "--adversarial-samples", "--positive-batch-size", "--negative-batch-size",
    "--adversarial-batch-size", "--validation-samples", "--testing-positive-samples",
    "--testing-adversarial-samples", "--resume", "--debug",
]


def test_train_help_lists_reference_options():
    res = CliRunner().invoke(main, ["train", "--help"])
    assert res.exit_code == 0, res.output
    for opt in REFERENCE_OPTIONS:
        assert opt in res.output, opt


def test_safe_name():
    assert safe_name("Hey Buddy!") == "hey_buddy"
    assert safe_name("  OK, computer ") == "ok_computer"


def test_phrase_clips_deterministic_and_distinct():
    a = phrase_clips("hey buddy", 4, seed=3)
    b = phrase_clips("hey buddy", 4, seed=3)
    c = phrase_clips("hello world", 4, seed=3)
    assert a.shape == (4, 24000) and a.dtype == torch.float32
    assert torch.equal(a, b)
    assert not torch.allclose(a, c)
    assert float(a.abs().max()) <= 1.0


@pytest.mark.gpu
def test_train_cli_short_run(tmp_path):
    ckpt = tmp_path / "ckpt"
    args = ["train", "hey buddy", "--steps", "40", "--stages", "2", "--validation-steps", "20",
            "--checkpoint-steps", "40", "--positive-samples", "3000", "--adversarial-samples", "3000",
            "--negative-samples", "6000", "--validation-samples", "2000",
            "--testing-positive-samples", "1000", "--testing-adversarial-samples", "1000",
            "--logging-steps", "20", "--checkpoint-dir", str(ckpt), "--seed", "5"]
    res = CliRunner().invoke(main, args, catch_exceptions=False)
    assert res.exit_code == 0, res.output
    files = os.listdir(ckpt)
    assert any(f.startswith("hey_buddy") and f.endswith(".pt") and not f.endswith("_optimizer.pt")
               for f in files), files


def test_combine_half_and_delete(tmp_path):
    """`heybuddy combine A B target --half --delete` (__main__.py:112-169): sorted
    file order, f16, sources removed."""
    import numpy as np
    rng = np.random.default_rng(0)
    parts = {}
    for d in ("a", "b"):
        os.makedirs(tmp_path / d)
        for k in range(3):
            x = rng.standard_normal((5 + k, 16, 96)).astype(np.float32)
            np.save(tmp_path / d / f"{k}.npy", x)
            parts[str(tmp_path / d / f"{k}.npy")] = x
    res = CliRunner().invoke(main, ["combine", "a", "b", "all.npy", "--directory", str(tmp_path), "--half",
                                    "--delete", "--batch-size", "2"])
    assert res.exit_code == 0, res.output
    got = np.load(tmp_path / "all.npy")
    want = np.concatenate([parts[k] for k in sorted(parts)]).astype(np.float16)
    assert got.dtype == np.float16
    np.testing.assert_array_equal(got, want)
    assert not (tmp_path / "a").exists() and not (tmp_path / "b").exists()


def test_new_commands_listed():
    res = CliRunner().invoke(main, ["--help"])
    for cmd in ("train", "extract", "combine", "predict", "convert"):
        assert cmd in res.output, cmd


@pytest.mark.gpu
def test_extract_files_match_featurize(tmp_path):
    """extract: 1.44-s windows (last one right-padded), featurized on the device,
    files flushed at the reference's points (buffer >= samples_per_file after a
    process batch)."""
    import numpy as np
    from heybuddy.dataset.precalculated import PrecalculatedTrainingDatasetGenerator
    from heybuddy.embeddings import SpeechEmbeddings
    rng = np.random.default_rng(1)
    clips = [(rng.standard_normal(n) * 0.1).astype(np.float32) for n in (50000, 23040, 7000, 99999)]
    ds = [{"audio": {"array": c, "sampling_rate": 16000}} for c in clips]
    gen = PrecalculatedTrainingDatasetGenerator("local", process_batch_size=3, device_id=0)
    files = gen("x", output_dir=str(tmp_path), samples_per_file=4, dataset=ds)
    wins = []
    for c in clips:
        for i in range(0, len(c), 23040):
            w = c[i:i + 23040]
            wins.append(np.pad(w, (0, 23040 - len(w))))
    want = SpeechEmbeddings(device_id=0).featurize(torch.from_numpy(np.stack(wins)).cuda(), remove_nan=False)
    got = np.concatenate([np.load(f) for f in files])
    np.testing.assert_allclose(got, want.cpu().numpy(), rtol=1e-5, atol=1e-5)
    # 3 + 1 + 1 + 5 = 10 windows in batches of 3: flushes after batches 2 (6 rows), 4 (4 rows)
    assert [np.load(f).shape[0] for f in files] == [6, 4]


@pytest.mark.gpu
def test_convert_and_predict_commands(tmp_path):
    import numpy as np
    from heybuddy.wakeword import WakeWordMLPModel
    m = WakeWordMLPModel()
    ck = str(tmp_path / "head.pt")
    torch.save(m.state_dict(), ck)
    res = CliRunner().invoke(main, ["convert", ck])
    assert res.exit_code == 0, res.output
    back = WakeWordMLPModel.from_file(str(tmp_path / "head.onnx"))
    for k, v in m.state_dict().items():
        assert torch.equal(back.state_dict()[k], v), k
    wav = str(tmp_path / "a.npy")
    np.save(wav, (np.random.default_rng(0).standard_normal(40000) * 0.05).astype(np.float32))
    res = CliRunner().invoke(main, ["predict", str(tmp_path / "head.onnx"), wav, "--threshold", "2.0"])
    assert res.exit_code == 0, res.output
    assert "No wake-word utterances detected" in res.output
