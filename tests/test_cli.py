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
