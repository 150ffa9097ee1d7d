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

GOLDEN_OPTIONS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cli_train_options.json")


def _train_params():
    from heybuddy.__main__ import train
    out = {}
    for p in train.params:
        for f in list(p.opts) + list(p.secondary_opts):
            out[f] = p
    return out


def test_train_has_every_reference_option_with_its_default():
    """The reference's `train` surface (__main__.py:171-244), read from its
    decorators into tests/golden/cli_train_options.json (oracle/make_cli_fixture.py):
    every flag, the same destination for the architecture / dataset-size flag
    groups, and the same default (expressions over DEFAULT_* evaluated against
    this package's constants, which must equal the reference's values)."""
    import json
    import heybuddy.constants as C
    gold = json.load(open(GOLDEN_OPTIONS))
    for name, val in gold["constants"].items():
        mine = getattr(C, name)
        assert (list(mine) if isinstance(mine, tuple) else mine) == val, name
    params = _train_params()
    from heybuddy.__main__ import train
    assert [p.name for p in train.params if p.param_type_name == "argument"] == gold["arguments"]
    for opt in gold["options"]:
        for flag in opt["flags"]:
            for f in flag.split("/"):
                assert f in params, f
        p = params[opt["flags"][0].split("/")[0]]
        if opt["dest"]:
            assert p.name == opt["dest"], (opt["flags"], p.name)
        if opt["flag_value"] is not None:
            assert p.flag_value == opt["flag_value"], opt["flags"]
        assert bool(p.multiple) == opt["multiple"], opt["flags"]
        if opt["default"] is not None and opt["flag_value"] is None:
            want = eval(opt["default"], {"__builtins__": {}}, vars(C))
            got = p.default
            assert got == want or (got is None and want is None), (opt["flags"], got, want)
        if opt["flag_value"] is not None:  # the group's default member
            want = eval(opt["default"], {"__builtins__": {}}, vars(C))
            assert bool(p.default) == bool(want), opt["flags"]


def test_train_routes_through_dataset_iterator_all(monkeypatch):
    """`heybuddy train PHRASE` builds its data exactly as the reference does
    (__main__.py:294-386): WakeWordTrainingDatasetIterator.all with the
    reference's keyword mapping (the tanh pair, dataset-size flags, phrase
    words, default background / impulse datasets), then WakeWordTrainer."""
    import heybuddy.constants as C
    from heybuddy.dataset.training import WakeWordTrainingDatasetIterator
    seen = {}

    class Stop(Exception):
        pass

    def fake_all(**kw):
        seen.update(kw)
        raise Stop()

    monkeypatch.setattr(WakeWordTrainingDatasetIterator, "all", staticmethod(fake_all))
    args = ["train", "hey buddy", "--augmentation-tanh-distortion-min", "0.01", "--augmentation-tanh-distortion-max",
            "0.2", "--training-large-default-dataset", "--augment-phrase-word", "yo", "--adversarial-phrases", "7",
            "--augmentation-no-default-impulse-dataset", "--augmentation-impulse-dataset", "my/irs",
            "--testing-positive-batch-size", "20"]
    res = CliRunner().invoke(main, args)
    assert isinstance(res.exception, Stop), res.output
    assert seen["wake_phrase"] == "hey buddy"
    assert seen["augment_tanh_min_distortion"] == 0.01 and seen["augment_tanh_max_distortion"] == 0.2
    assert seen["large_training"] and not seen["medium_training"]
    assert seen["phrase_augment_words"] == list(C.DEFAULT_AUGMENT_PHRASE_WORDS) + ["yo"]
    assert seen["augment_background_dataset"] == list(C.DEFAULT_BACKGROUND_DATASET)
    assert seen["augment_impulse_dataset"] == ["my/irs"]
    assert seen["num_adversarial_phrases"] == 7 and seen["testing_positive_per_batch"] == 20
    assert seen["negative_per_batch"] == C.DEFAULT_NEGATIVE_BATCH_SIZE
    assert seen["validation_num_positive_samples"] == C.DEFAULT_VALIDATION_SAMPLES
    seen.clear()
    res = CliRunner().invoke(main, ["train", "hey buddy"])  # no dataset-size flag: the full default set
    assert isinstance(res.exception, Stop) and seen["large_training"] and seen["medium_training"]


def test_train_help_lists_reference_options():
    res = CliRunner().invoke(main, ["train", "--help"])
    assert res.exit_code == 0, res.output
    assert "--augmentation-tanh-distortion-min" in res.output and "--training-no-default-dataset" in res.output


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
def test_train_cli_short_run(tmp_path, monkeypatch):
    ckpt = tmp_path / "ckpt"
    from heybuddy.dataset import precalculated as pc
    monkeypatch.setattr(pc, "LOCAL_DIR", str(tmp_path / "precalculated"))  # feature cache + offline negatives
    args = ["train", "hey buddy", "--steps", "40", "--stages", "2", "--validation-steps", "20",
            "--checkpoint-steps", "40", "--positive-samples", "3000", "--adversarial-samples", "3000",
            "--negative-samples", "6000", "--validation-negative-samples", "2000", "--validation-samples", "500",
            "--testing-positive-samples", "1000", "--testing-adversarial-samples", "1000",
            "--logging-steps", "20", "--checkpoint-dir", str(ckpt), "--seed", "5"]
    res = CliRunner().invoke(main, args, catch_exceptions=False)
    assert res.exit_code == 0, res.output
    files = os.listdir(ckpt)
    assert any(f.startswith("hey_buddy") and f.endswith(".pt") and not f.endswith("_optimizer.pt")
               for f in files), files
    # the reference's feature caches (features.py:686-760): positives, adversarials, testing, validation
    cached = set(os.listdir(pc.LOCAL_DIR))
    for f in ("hey_buddy.npy", "hey_buddy_adv.npy", "hey_buddy_tst.npy", "hey_buddy_tst_adv.npy", "hey_buddy_val.npy",
              "synthetic-large.npy", "synthetic-medium.npy", "synthetic-validation.npy"):
        assert f in cached, (f, cached)
    import numpy as np
    assert np.load(os.path.join(pc.LOCAL_DIR, "hey_buddy.npy"), mmap_mode="r").shape == (3000, 16, 96)
    assert np.load(os.path.join(pc.LOCAL_DIR, "hey_buddy_val.npy"), mmap_mode="r").shape == (500, 16, 96)


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
