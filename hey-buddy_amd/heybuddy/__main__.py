"""``heybuddy train`` on the MI355X hot path (reference src/python/heybuddy/__main__.py:171-429).

Same command and option names for the hot-path settings. The data sources the
reference downloads or synthesizes with TTS (Piper positives and adversarial
phrases, HF background-noise and impulse-response datasets, the hosted 72 GB
negative embeddings) are unavailable offline, so this command builds them
synthetically on the device (heybuddy.synthetic) and runs the reference's
pipeline on them: augment (noise mix + reverb) -> featurize (mel + embedding)
-> 3-stage classifier training with validation and testing. Under
torch.distributed.run every rank featurizes its shard of the clips, the
embedding pools are all-gathered, and training is data-parallel with one
gradient all-reduce per step.
"""
from __future__ import annotations

import os
import re
from typing import List, Optional

import click
import torch

from heybuddy.constants import *  # noqa: F401,F403
from heybuddy.constants import (DEFAULT_ACTIVATION_THRESHOLD, DEFAULT_ADVERSARIAL_BATCH_SIZE,
                                DEFAULT_ADVERSARIAL_SAMPLES, DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB,
                                DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB,
                                DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB, DEFAULT_AUGMENT_GAIN_PROB,
                                DEFAULT_AUGMENT_REVERB_PROB,
                                DEFAULT_CHECKPOINT_STEPS, DEFAULT_HIGH_LOSS_THRESHOLD, DEFAULT_LAYER_DIM,
                                DEFAULT_LAYERS, DEFAULT_LEARNING_RATE, DEFAULT_LOGGING_STEPS,
                                DEFAULT_NEGATIVE_BATCH_SIZE, DEFAULT_NEGATIVE_WEIGHT,
                                DEFAULT_POSITIVE_BATCH_SIZE, DEFAULT_POSITIVE_SAMPLES, DEFAULT_STAGES,
                                DEFAULT_STEPS, DEFAULT_TARGET_FALSE_POSITIVE_RATE,
                                DEFAULT_TESTING_ADVERSARIAL_SAMPLES, DEFAULT_TESTING_POSITIVE_SAMPLES,
                                DEFAULT_USE_GATING, DEFAULT_USE_HALF_LAYERS, DEFAULT_VALIDATION_SAMPLES,
                                DEFAULT_VALIDATION_STEPS)


def safe_name(name: str) -> str:
    """util/string_util.py:145-151: lower-case, non-alphanumerics -> '_'."""
    return re.sub(r"[^a-z0-9]+", "_", name.lower()).strip("_")


@click.group()
def main() -> None:
    """hey-buddy (MI355X hot path)."""


def build_embeddings(n: int, seed: int, device: torch.device, augmenter=None, chunk: int = 65536,
                     kind: str = "positive", phrase: str = "") -> torch.Tensor:
    """Synthetic clips of one class -> [n, 16, 96] embeddings on the device,
    featurized (and augmented, if given) in chunks, sharded over the ranks.
    positive: phrase_clips(phrase); adversarial: random tone bursts;
    negative: the same at 0.3x level."""
    from heybuddy import distributed as hd
    from heybuddy.embeddings import SpeechEmbeddings
    from heybuddy.synthetic import phrase_clips, synthetic_clips
    rank, world = hd.world()
    lo, hi = hd.clip_range(n, rank, world)
    se = SpeechEmbeddings(device_id=device.index)
    parts = []
    for s in range(lo, hi, chunk):
        m = min(chunk, hi - s)
        if kind == "positive":
            clips = phrase_clips(phrase, m, seed=seed * 7919 + s, device=device)
        else:
            clips = synthetic_clips(m, seed=seed * 7919 + s, device=device)
        if kind == "negative":  # noise-like negatives: random tones at low level, no burst
            clips.mul_(0.3)
        if augmenter is not None:
            clips = augmenter(clips)
        parts.append(se.featurize(clips))
    local = torch.cat(parts) if parts else torch.empty((0, 16, 96), device=device)
    if world == 1:
        return local
    sizes = [hd.clip_range(n, r, world) for r in range(world)]
    buf = [torch.empty((b - a, 16, 96), device=device) for a, b in sizes]
    torch.distributed.all_gather(buf, local.contiguous())
    return torch.cat(buf)


@main.command()
@click.argument("phrase", type=str, nargs=1)
@click.option("--additional-phrase", type=str, default=None, multiple=True)
@click.option("--wandb-entity", type=str, default=None)
@click.option("--perceptron", "architecture", flag_value="perceptron", default=True)
@click.option("--transformer", "architecture", flag_value="transformer")
@click.option("--use-half-layers/--no-use-half-layers", default=DEFAULT_USE_HALF_LAYERS)
@click.option("--use-gating/--no-use-gating", default=DEFAULT_USE_GATING)
@click.option("--layer-dim", type=int, default=DEFAULT_LAYER_DIM, show_default=True)
@click.option("--num-layers", type=int, default=DEFAULT_LAYERS, show_default=True)
@click.option("--steps", type=int, default=DEFAULT_STEPS, show_default=True)
@click.option("--stages", type=int, default=DEFAULT_STAGES, show_default=True)
@click.option("--threshold", type=float, default=DEFAULT_ACTIVATION_THRESHOLD, show_default=True)
@click.option("--learning-rate", type=float, default=DEFAULT_LEARNING_RATE, show_default=True)
@click.option("--high-loss-threshold", type=float, default=DEFAULT_HIGH_LOSS_THRESHOLD, show_default=True)
@click.option("--target-false-positive-rate", type=float, default=DEFAULT_TARGET_FALSE_POSITIVE_RATE, show_default=True)
@click.option("--dynamic-negative-weight/--no-dynamic-negative-weight", default=True)
@click.option("--negative-weight", type=float, default=DEFAULT_NEGATIVE_WEIGHT, show_default=True)
@click.option("--augmentation-background-noise-prob", type=float, default=DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB, show_default=True)
@click.option("--augmentation-background-noise-min-snr-db", type=float, default=DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB, show_default=True)
@click.option("--augmentation-background-noise-max-snr-db", type=float, default=DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB, show_default=True)
@click.option("--augmentation-reverb-prob", type=float, default=DEFAULT_AUGMENT_REVERB_PROB, show_default=True)
@click.option("--augmentation-gain-prob", type=float, default=DEFAULT_AUGMENT_GAIN_PROB, show_default=True)
@click.option("--augmentation-tanh-distortion-prob", type=float, default=DEFAULT_AUGMENT_TANH_DISTORTION_PROB, show_default=True)
@click.option("--augmentation-tanh-min-distortion", type=float, default=DEFAULT_AUGMENT_TANH_MIN_DISTORTION, show_default=True)
@click.option("--augmentation-tanh-max-distortion", type=float, default=DEFAULT_AUGMENT_TANH_MAX_DISTORTION, show_default=True)
@click.option("--augmentation-colored-noise-prob", type=float, default=DEFAULT_AUGMENT_COLORED_NOISE_PROB, show_default=True)
@click.option("--augmentation-colored-noise-min-snr-db", type=float, default=DEFAULT_AUGMENT_COLORED_NOISE_MIN_SNR_DB, show_default=True)
@click.option("--augmentation-colored-noise-max-snr-db", type=float, default=DEFAULT_AUGMENT_COLORED_NOISE_MAX_SNR_DB, show_default=True)
@click.option("--augmentation-colored-noise-min-f-decay", type=float, default=DEFAULT_AUGMENT_COLORED_NOISE_MIN_F_DECAY, show_default=True)
@click.option("--augmentation-colored-noise-max-f-decay", type=float, default=DEFAULT_AUGMENT_COLORED_NOISE_MAX_F_DECAY, show_default=True)
@click.option("--logging-steps", type=int, default=DEFAULT_LOGGING_STEPS, show_default=True)
@click.option("--validation-steps", type=int, default=DEFAULT_VALIDATION_STEPS, show_default=True)
@click.option("--checkpoint-steps", type=int, default=DEFAULT_CHECKPOINT_STEPS, show_default=True)
@click.option("--positive-samples", type=int, default=DEFAULT_POSITIVE_SAMPLES, show_default=True)
@click.option("--adversarial-samples", type=int, default=DEFAULT_ADVERSARIAL_SAMPLES, show_default=True)
@click.option("--negative-samples", type=int, default=200_000, show_default=True,
              help="Synthetic negatives featurized in place of the hosted precalculated sets.")
@click.option("--positive-batch-size", type=int, default=DEFAULT_POSITIVE_BATCH_SIZE, show_default=True)
@click.option("--negative-batch-size", type=int, default=DEFAULT_NEGATIVE_BATCH_SIZE, show_default=True)
@click.option("--adversarial-batch-size", type=int, default=DEFAULT_ADVERSARIAL_BATCH_SIZE, show_default=True)
@click.option("--validation-samples", type=int, default=DEFAULT_VALIDATION_SAMPLES, show_default=True)
@click.option("--testing-positive-samples", type=int, default=DEFAULT_TESTING_POSITIVE_SAMPLES, show_default=True)
@click.option("--testing-adversarial-samples", type=int, default=DEFAULT_TESTING_ADVERSARIAL_SAMPLES, show_default=True)
@click.option("--checkpoint-dir", type=str, default="./checkpoints", show_default=True)
@click.option("--seed", type=int, default=0, show_default=True)
@click.option("--resume/--no-resume", default=False)
@click.option("--debug/--no-debug", default=False)
def train(phrase: str, additional_phrase: List[str], wandb_entity: Optional[str], architecture: str,
          use_half_layers: bool, use_gating: bool, layer_dim: int, num_layers: int, steps: int, stages: int,
          threshold: float, learning_rate: float, high_loss_threshold: float,
          target_false_positive_rate: float, dynamic_negative_weight: bool, negative_weight: float,
          augmentation_background_noise_prob: float, augmentation_background_noise_min_snr_db: float,
          augmentation_background_noise_max_snr_db: float, augmentation_reverb_prob: float,
          augmentation_gain_prob: float, augmentation_colored_noise_prob: float,
          augmentation_colored_noise_min_snr_db: float, augmentation_colored_noise_max_snr_db: float,
          augmentation_colored_noise_min_f_decay: float, augmentation_colored_noise_max_f_decay: float,
          augmentation_tanh_distortion_prob: float, augmentation_tanh_min_distortion: float,
          augmentation_tanh_max_distortion: float,
          logging_steps: int, validation_steps: int, checkpoint_steps: int, positive_samples: int,
          adversarial_samples: int, negative_samples: int, positive_batch_size: int,
          negative_batch_size: int, adversarial_batch_size: int, validation_samples: int,
          testing_positive_samples: int, testing_adversarial_samples: int, checkpoint_dir: str, seed: int,
          resume: bool, debug: bool) -> None:
    """Trains a wake word detection model (synthetic data on the device)."""
    import numpy as np
    from heybuddy import distributed as hd
    from heybuddy.dataset.augmented import BatchAugmenter
    from heybuddy.dataset.training import DevicePool, TrainingDatasetIterator, WakeWordTrainingDatasetIterator
    from heybuddy.synthetic import impulse_responses, noise_bank
    from heybuddy.trainer import WakeWordTrainer
    from heybuddy.util import logger

    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1 and not torch.distributed.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(seed)
    np.random.seed(seed)
    if additional_phrase:
        logger.warning("additional phrases need TTS; the synthetic positives stand in for every phrase")
    if wandb_entity:
        logger.warning("wandb logging is outside the MI355X hot path; ignored")
    aug = BatchAugmenter(noise_bank(64, seed=seed + 11, device=device),
                         impulse_responses(32, seed=seed + 12, device=device), device=device,
                         batch_size=128, background_noise_prob=augmentation_background_noise_prob,
                         background_noise_min_snr_db=augmentation_background_noise_min_snr_db,
                         background_noise_max_snr_db=augmentation_background_noise_max_snr_db,
                         reverb_prob=augmentation_reverb_prob, gain_prob=augmentation_gain_prob,
                         colored_noise_prob=augmentation_colored_noise_prob,
                         colored_noise_min_snr_db=augmentation_colored_noise_min_snr_db,
                         colored_noise_max_snr_db=augmentation_colored_noise_max_snr_db,
                         colored_noise_min_f_decay=augmentation_colored_noise_min_f_decay,
                         colored_noise_max_f_decay=augmentation_colored_noise_max_f_decay,
                         tanh_distortion_prob=augmentation_tanh_distortion_prob,
                         tanh_min_distortion=augmentation_tanh_min_distortion,
                         tanh_max_distortion=augmentation_tanh_max_distortion)
    pos = build_embeddings(positive_samples, seed + 1, device, aug, kind="positive", phrase=phrase)
    adv = build_embeddings(adversarial_samples, seed + 2, device, aug, kind="adversarial")
    neg = build_embeddings(negative_samples, seed + 3, device, aug, kind="negative").half()
    vpos = build_embeddings(validation_samples // 10 or 1, seed + 4, device, aug, kind="positive", phrase=phrase)
    vneg = build_embeddings(validation_samples, seed + 5, device, aug, kind="negative")
    tpos = build_embeddings(testing_positive_samples, seed + 6, device, aug, kind="positive", phrase=phrase)
    tadv = build_embeddings(testing_adversarial_samples, seed + 7, device, aug, kind="adversarial")
    g = torch.Generator(device=device).manual_seed(seed + 99)  # identical batches on every rank
    half = int(negative_samples * 2 / 3)
    training = WakeWordTrainingDatasetIterator.default(
        pos, adv, neg[:half], neg[half:], positive_per_batch=positive_batch_size,
        adversarial_per_batch=adversarial_batch_size, negative_per_batch=negative_batch_size, generator=g)

    def fixed(xs, ys, bs=1000):
        x = torch.cat(xs)
        y = torch.cat(ys)
        return [(x[i:i + bs], y[i:i + bs]) for i in range(0, x.shape[0], bs)]

    validation = fixed([vpos, vneg], [torch.ones(vpos.shape[0], dtype=torch.int64, device=device),
                                      torch.zeros(vneg.shape[0], dtype=torch.int64, device=device)])
    testing = fixed([tpos, tadv], [torch.ones(tpos.shape[0], dtype=torch.int64, device=device),
                                   torch.zeros(tadv.shape[0], dtype=torch.int64, device=device)])
    rank, world = hd.world()
    trainer = WakeWordTrainer(checkpoint_dir=checkpoint_dir, architecture=architecture,
                              use_half_layers=use_half_layers, use_gating=use_gating, layer_dim=layer_dim,
                              num_layers=num_layers, device=device)
    name = safe_name(phrase)
    if resume:
        trainer.resume(name)
    trainer(training=training, validation=validation, testing=testing, activation_threshold=threshold,
            checkpoint_steps=checkpoint_steps, dynamic_negative_weight=dynamic_negative_weight,
            high_loss_threshold=high_loss_threshold, learning_rate=learning_rate,
            max_negative_weight=negative_weight, name=name if rank == 0 else f"{name}_rank{rank}",
            num_stages=stages, num_steps=steps, target_false_positive_rate=target_false_positive_rate,
            validation_steps=validation_steps, logging_steps=logging_steps)
    if world > 1:
        torch.distributed.destroy_process_group()


@main.command()
@click.argument("name", type=str, nargs=1)
@click.argument("repo_id", type=str, nargs=1)
@click.option("--directory", default=None, help="Directory to save the embeddings to (default: precalculated/).")
@click.option("--config", type=str, default=None)
@click.option("--split", type=str, default="train", show_default=True)
@click.option("--audio-key", type=str, default="audio", show_default=True)
@click.option("--audio-array-key", type=str, default="array", show_default=True)
@click.option("--audio-sample-rate-key", type=str, default="sampling_rate", show_default=True)
@click.option("--transcript-key", type=str, default=None,
              help="Write labeled [N, 17, 96] files (needs a local tokenizer: --tokenizer).")
@click.option("--tokenizer", type=str, default=None, help="Local transformers tokenizer directory.")
@click.option("--streaming/--no-streaming", default=True)
@click.option("--trust-remote-code/--no-trust-remote-code", default=False)
@click.option("--hours", type=float, default=1000.0, show_default=True)
@click.option("--samples-per-file", type=int, default=10000, show_default=True)
@click.option("--device-id", type=int, default=None)
@click.option("--sample-rate", type=int, default=16000, show_default=True)
@click.option("--seconds-per-batch", type=float, default=1.44, show_default=True)
@click.option("--process-batch-size", default=100, show_default=True)
@click.option("--embedding-batch-size", default=32, show_default=True)
@click.option("--tokenizer-max-length", default=96, show_default=True)
@click.option("--debug/--no-debug", default=False)
def extract(name: str, repo_id: str, directory: Optional[str], config: Optional[str], split: str, audio_key: str,
            audio_array_key: str, audio_sample_rate_key: str, transcript_key: Optional[str],
            tokenizer: Optional[str], streaming: bool, trust_remote_code: bool, hours: float,
            samples_per_file: int, device_id: Optional[int], sample_rate: int, seconds_per_batch: float,
            process_batch_size: int, embedding_batch_size: int, tokenizer_max_length: int, debug: bool) -> None:
    """Creates a dataset of speech embeddings from an audio dataset (__main__.py:40-110);
    REPO_ID is anything datasets.load_dataset opens offline (a local path)."""
    from heybuddy.dataset import precalculated as pc
    kw = dict(config_name=config, split=split, audio_key=audio_key, audio_array_key=audio_array_key,
              audio_sample_rate_key=audio_sample_rate_key, device_id=device_id, sample_rate=sample_rate,
              seconds_per_batch=seconds_per_batch, process_batch_size=process_batch_size,
              embedding_batch_size=embedding_batch_size)
    if transcript_key is not None:
        tok = None
        if tokenizer is not None:
            from transformers import AutoTokenizer
            t = AutoTokenizer.from_pretrained(tokenizer, local_files_only=True)
            tok = lambda text: t(text, padding="max_length", truncation=True,  # noqa: E731
                                 max_length=tokenizer_max_length)["input_ids"]
        gen = pc.PrecalculatedLabeledTrainingDatasetGenerator(repo_id, transcript_key=transcript_key,
                                                              tokenizer_max_length=tokenizer_max_length,
                                                              tokenizer=tok, **kw)
    else:
        gen = pc.PrecalculatedTrainingDatasetGenerator(repo_id, **kw)
    files = gen(name=name, output_dir=directory or pc.LOCAL_DIR, max_hours=hours, dataset_streaming=streaming,
                trust_remote_code=trust_remote_code, samples_per_file=samples_per_file)
    click.echo(f"Wrote {len(files)} file(s) to {os.path.join(directory or pc.LOCAL_DIR, name)}")


@main.command()
@click.argument("source", type=str, nargs=-1)
@click.argument("target", type=str, nargs=1)
@click.option("--directory", default=None, help="Directory of the embeddings (default: precalculated/).")
@click.option("--reset/--no-reset", default=True, help="Reset the target file if it already exists.")
@click.option("--half/--no-half", default=False, help="Store f16 embeddings.")
@click.option("--delete/--no-delete", default=False, help="Delete source embeddings after combining.")
@click.option("--batch-size", default=10, show_default=True, help="Files read per append.")
@click.option("--debug/--no-debug", default=False)
def combine(source: List[str], target: str, directory: Optional[str], reset: bool, half: bool, delete: bool,
            batch_size: int, debug: bool) -> None:
    """Combines the .npy files of one or more extract directories into one
    appendable .npy (__main__.py:112-169); --half stores f16 (the trainer's
    f16 negative pool)."""
    import numpy as np
    from heybuddy.dataset.precalculated import LOCAL_DIR
    from heybuddy.util.numpy_util import AppendableNumpyArrayFile
    directory = directory or LOCAL_DIR
    target_path = os.path.join(directory, target)
    if reset and os.path.exists(target_path):
        os.remove(target_path)
    dirs = [os.path.join(directory, s) for s in source]
    files = sorted(os.path.join(d, f) for d in dirs for f in os.listdir(d) if f.endswith(".npy"))
    with AppendableNumpyArrayFile(target_path, dtype=np.float16 if half else None) as out:
        for i in range(0, len(files), max(1, batch_size)):
            group = files[i:i + max(1, batch_size)]
            out.append(np.concatenate([np.load(f) for f in group], axis=0))
            if delete:
                for f in group:
                    os.remove(f)
    if delete:
        for d in dirs:
            os.rmdir(d)
    click.echo(f"Combined {len(files)} file(s) into {target_path}")


@main.command()
@click.argument("checkpoint", type=click.Path(exists=True, dir_okay=False, file_okay=True), nargs=1)
@click.argument("audio", type=click.Path(exists=True, dir_okay=False, file_okay=True), nargs=1)
@click.option("--threshold", type=float, default=DEFAULT_ACTIVATION_THRESHOLD, show_default=True)
@click.option("--device-id", type=int, default=None)
@click.option("--debug/--no-debug", default=False)
def predict(checkpoint: str, audio: str, threshold: float, device_id: Optional[int], debug: bool) -> None:
    """Predicts wake word times in an audio file (__main__.py:431-464). AUDIO:
    a .npy / .wav (PCM) file at 16 kHz or any rate (resampled)."""
    import numpy as np
    from heybuddy.wakeword import WakeWordMLPModel
    device = torch.device("cuda", device_id or 0)
    model = WakeWordMLPModel.from_file(checkpoint, device=device).eval()
    if audio.endswith(".npy"):
        wav, rate = np.load(audio), 16000
    else:
        import wave
        with wave.open(audio, "rb") as w:
            rate, width, ch = w.getframerate(), w.getsampwidth(), w.getnchannels()
            raw = np.frombuffer(w.readframes(w.getnframes()), dtype={1: np.uint8, 2: np.int16, 4: np.int32}[width])
        wav = raw.reshape(-1, ch).T.astype(np.float32)
        wav = (wav - 128) / 128 if width == 1 else wav / float(2 ** (8 * width - 1))
    from heybuddy.util import audio_to_bct_tensor
    x, _ = audio_to_bct_tensor(np.asarray(wav, dtype=np.float32), sample_rate=rate, target_sample_rate=16000)
    times = model.predict_timecodes(x, threshold=threshold)
    if not times:
        click.echo("No wake-word utterances detected")
    elif len(times) == 1:
        click.echo(f"Wake-word utterance detected at {times[0]:.1f} second(s)")
    else:
        click.echo(f"{len(times)} wake-word utterances detected at the following times:")
        for t in times:
            click.echo(f"  {t:.1f} second(s)")


@main.command()
@click.argument("checkpoint", type=click.Path(exists=True, dir_okay=False, file_okay=True), nargs=1)
@click.option("-v", "--opset-version", type=int, default=19, show_default=True)
@click.option("-o", "--output", type=click.Path(exists=False, dir_okay=False, file_okay=True), default=None)
def convert(checkpoint: str, opset_version: int, output: Optional[str]) -> None:
    """Converts a checkpoint to ONNX (__main__.py:599-625)."""
    from heybuddy.wakeword import WakeWordMLPModel
    dest = output or os.path.join(os.path.dirname(checkpoint),
                                  os.path.splitext(os.path.basename(checkpoint))[0] + ".onnx")
    if os.path.exists(dest):
        os.remove(dest)
    WakeWordMLPModel.from_file(checkpoint).save_onnx(dest, opset_version=opset_version)
    click.echo(f"Model saved to {dest}")


if __name__ == "__main__":
    main()
