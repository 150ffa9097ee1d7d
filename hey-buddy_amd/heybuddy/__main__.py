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
from heybuddy.dataset.training import OFFLINE_NEGATIVE_SAMPLES, OFFLINE_VALIDATION_NEGATIVE_SAMPLES
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


@main.command()
@click.argument("phrase", type=str, nargs=1)
@click.option("--additional-phrase", type=str, default=None, multiple=True, help="Additional phrases to use for training.", show_default=True)
@click.option("--wandb-entity", type=str, default=None, help="W&B entity to use for logging (outside the hot path: ignored).", show_default=True)
@click.option("--perceptron", "architecture", flag_value="perceptron", default=DEFAULT_ARCHITECTURE == "perceptron", help="Use a perceptron architecture.", show_default=True)
@click.option("--transformer", "architecture", flag_value="transformer", default=DEFAULT_ARCHITECTURE == "transformer", help="Use a transformer architecture (not implemented on the MI355X path).", show_default=True)
@click.option("--use-half-layers/--no-use-half-layers", default=DEFAULT_USE_HALF_LAYERS, is_flag=True, help="Use enumerated striped-attention layers for the perceptron model.", show_default=True)
@click.option("--use-gating/--no-use-gating", default=DEFAULT_USE_GATING, is_flag=True, help="Use gated MLP layers for the perceptron model.", show_default=True)
@click.option("--layer-dim", type=int, default=DEFAULT_LAYER_DIM, help="Dimension of the linear layers to use for the model.", show_default=True)
@click.option("--num-layers", type=int, default=DEFAULT_LAYERS, help="The number of perceptron blocks.", show_default=True)
@click.option("--num-heads", type=int, default=DEFAULT_HEADS, help="The number of attention heads to use when using the transformer model.", show_default=True)
@click.option("--steps", type=int, default=DEFAULT_STEPS, help="Number of optimization steps to take.", show_default=True)
@click.option("--stages", type=int, default=DEFAULT_STAGES, help="Number of training stages.", show_default=True)
@click.option("--threshold", type=float, default=DEFAULT_ACTIVATION_THRESHOLD, help="Threshold to use for wake-word detection.", show_default=True)
@click.option("--learning-rate", type=float, default=DEFAULT_LEARNING_RATE, help="Learning rate for the optimizer.", show_default=True)
@click.option("--high-loss-threshold", type=float, default=DEFAULT_HIGH_LOSS_THRESHOLD, help="Threshold for high loss values.", show_default=True)
@click.option("--target-false-positive-rate", type=float, default=DEFAULT_TARGET_FALSE_POSITIVE_RATE, help="Target false positive rate for the model.", show_default=True)
@click.option("--dynamic-negative-weight/--no-dynamic-negative-weight", default=True, is_flag=True, help="Dynamically adjust the negative weight at each validation step.", show_default=True)
@click.option("--negative-weight", type=float, default=DEFAULT_NEGATIVE_WEIGHT, help="Negative weight for the loss function.", show_default=True)
@click.option("--training-full-default-dataset", "training_default_size", flag_value="full", help="Use the full precalculated default training set.", default=True, show_default=True)
@click.option("--training-large-default-dataset", "training_default_size", flag_value="large", help="Use the large precalculated default training set.", default=False, show_default=True)
@click.option("--training-medium-default-dataset", "training_default_size", flag_value="medium", help="Use the medium precalculated default training set.", default=False, show_default=True)
@click.option("--training-no-default-dataset", "training_default_size", flag_value="none", help="Do not use a precalculated default training set.", default=False, show_default=True)
@click.option("--training-dataset", type=click.Path(exists=True, dir_okay=False, file_okay=True), default=None, help="Use a custom precalculated training set.", show_default=True)
@click.option("--augment-phrase-prob", type=float, default=DEFAULT_AUGMENT_PHRASE_PROB, help="Probability of augmenting the phrase.", show_default=True)
@click.option("--augment-phrase-default-words/--augment-phrase-no-default-words", default=True, is_flag=True, help="Use the default words for augmentation.", show_default=True)
@click.option("--augment-phrase-word", type=str, default=None, multiple=True, help="Custom words to use for augmentation.", show_default=True)
@click.option("--augmentation-default-background-dataset/--augmentation-no-default-background-dataset", default=True, is_flag=True, help="Use the default background dataset for augmentation.", show_default=True)
@click.option("--augmentation-background-dataset", default=None, multiple=True, help="Use a custom background dataset for augmentation.", show_default=True)
@click.option("--augmentation-default-impulse-dataset/--augmentation-no-default-impulse-dataset", default=True, is_flag=True, help="Use the default impulse dataset for augmentation.", show_default=True)
@click.option("--augmentation-impulse-dataset", default=None, multiple=True, help="Use a custom impulse dataset for augmentation.", show_default=True)
@click.option("--augmentation-dataset-streaming/--augmentation-dataset-no-streaming", default=False, is_flag=True, help="Stream the augmentation datasets, instead of downloading first.", show_default=True)
@click.option("--augmentation-seven-band-prob", type=float, default=DEFAULT_AUGMENT_SEVEN_BAND_PROB, help="Probability of applying the seven band equalization augmentation.", show_default=True)
@click.option("--augmentation-seven-band-gain-db", type=float, default=DEFAULT_AUGMENT_SEVEN_BAND_GAIN_DB, help="Gain in decibels for the seven band equalization augmentation.", show_default=True)
@click.option("--augmentation-tanh-distortion-prob", type=float, default=DEFAULT_AUGMENT_TANH_DISTORTION_PROB, help="Probability of applying the tanh distortion augmentation.", show_default=True)
@click.option("--augmentation-tanh-distortion-min", type=float, default=DEFAULT_AUGMENT_TANH_MIN_DISTORTION, help="Minimum value for the tanh distortion augmentation.", show_default=True)
@click.option("--augmentation-tanh-distortion-max", type=float, default=DEFAULT_AUGMENT_TANH_MAX_DISTORTION, help="Maximum value for the tanh distortion augmentation.", show_default=True)
@click.option("--augmentation-pitch-shift-prob", type=float, default=DEFAULT_AUGMENT_PITCH_SHIFT_PROB, help="Probability of applying the pitch shift augmentation.", show_default=True)
@click.option("--augmentation-pitch-shift-semitones", type=int, default=DEFAULT_AUGMENT_PITCH_SHIFT_SEMITONES, help="Number of semitones to shift the pitch for the pitch shift augmentation.", show_default=True)
@click.option("--augmentation-band-stop-prob", type=float, default=DEFAULT_AUGMENT_BAND_STOP_PROB, help="Probability of applying the band stop filter augmentation.", show_default=True)
@click.option("--augmentation-colored-noise-prob", type=float, default=DEFAULT_AUGMENT_COLORED_NOISE_PROB, help="Probability of applying the colored noise augmentation.", show_default=True)
@click.option("--augmentation-colored-noise-min-snr-db", type=float, default=DEFAULT_AUGMENT_COLORED_NOISE_MIN_SNR_DB, help="Minimum signal-to-noise ratio for the colored noise augmentation.", show_default=True)
@click.option("--augmentation-colored-noise-max-snr-db", type=float, default=DEFAULT_AUGMENT_COLORED_NOISE_MAX_SNR_DB, help="Maximum signal-to-noise ratio for the colored noise augmentation.", show_default=True)
@click.option("--augmentation-colored-noise-min-f-decay", type=float, default=DEFAULT_AUGMENT_COLORED_NOISE_MIN_F_DECAY, help="Minimum frequency decay for the colored noise augmentation.", show_default=True)
@click.option("--augmentation-colored-noise-max-f-decay", type=float, default=DEFAULT_AUGMENT_COLORED_NOISE_MAX_F_DECAY, help="Maximum frequency decay for the colored noise augmentation.", show_default=True)
@click.option("--augmentation-background-noise-prob", type=float, default=DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB, help="Probability of applying the background noise augmentation.", show_default=True)
@click.option("--augmentation-background-noise-min-snr-db", type=float, default=DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB, help="Minimum signal-to-noise ratio for the background noise augmentation.", show_default=True)
@click.option("--augmentation-background-noise-max-snr-db", type=float, default=DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB, help="Maximum signal-to-noise ratio for the background noise augmentation.", show_default=True)
@click.option("--augmentation-gain-prob", type=float, default=DEFAULT_AUGMENT_GAIN_PROB, help="Probability of applying the gain augmentation.", show_default=True)
@click.option("--augmentation-reverb-prob", type=float, default=DEFAULT_AUGMENT_REVERB_PROB, help="Probability of applying the reverb augmentation.", show_default=True)
@click.option("--logging-steps", type=int, default=DEFAULT_LOGGING_STEPS, help="How often to log step details.", show_default=True)
@click.option("--validation-steps", type=int, default=DEFAULT_VALIDATION_STEPS, help="How often to validate the model.", show_default=True)
@click.option("--checkpoint-steps", type=int, default=DEFAULT_CHECKPOINT_STEPS, help="How often to save the model.", show_default=True)
@click.option("--positive-samples", type=int, default=DEFAULT_POSITIVE_SAMPLES, help="Number of positive samples to use for training.", show_default=True)
@click.option("--adversarial-samples", type=int, default=DEFAULT_ADVERSARIAL_SAMPLES, help="Number of adversarial samples to use for training.", show_default=True)
@click.option("--adversarial-phrases", type=int, default=DEFAULT_ADVERSARIAL_PHRASES, help="Number of adversarial phrases to use for training.", show_default=True)
@click.option("--adversarial-phrase-custom", type=str, default=None, multiple=True, help="Custom adversarial phrases to use for training.", show_default=True)
@click.option("--positive-batch-size", type=int, default=DEFAULT_POSITIVE_BATCH_SIZE, help="The number of positive samples in each training batch.", show_default=True)
@click.option("--negative-batch-size", type=int, default=DEFAULT_NEGATIVE_BATCH_SIZE, help="The number of negative samples in each training batch.", show_default=True)
@click.option("--adversarial-batch-size", type=int, default=DEFAULT_ADVERSARIAL_BATCH_SIZE, help="The number of adversarial samples in each training batch.", show_default=True)
@click.option("--num-batch-threads", type=int, default=DEFAULT_BATCH_THREADS, help="Batch threads (batches are sampled on the device here: accepted, unused).", show_default=True)
@click.option("--validation-positive-batch-size", type=int, default=DEFAULT_VALIDATION_POSITIVE_BATCH_SIZE, help="The number of positive samples in each validation batch.", show_default=True)
@click.option("--validation-negative-batch-size", type=int, default=DEFAULT_VALIDATION_NEGATIVE_BATCH_SIZE, help="The number of negative samples in each validation batch.", show_default=True)
@click.option("--validation-samples", type=int, default=DEFAULT_VALIDATION_SAMPLES, help="The number of samples to use for validation.", show_default=True)
@click.option("--validation-num-batch-threads", type=int, default=1, help="Validation batch threads (accepted, unused).", show_default=True)
@click.option("--validation-default-dataset/--validation-no-default-dataset", default=True, is_flag=True, help="Use the default validation dataset.", show_default=True)
@click.option("--validation-dataset", type=click.Path(exists=True, dir_okay=False, file_okay=True), default=None, help="Use a custom precalculated validation set.", show_default=True)
@click.option("--testing-positive-samples", type=int, default=DEFAULT_TESTING_POSITIVE_SAMPLES, help="The number of positive samples to use for testing.", show_default=True)
@click.option("--testing-adversarial-samples", type=int, default=DEFAULT_TESTING_ADVERSARIAL_SAMPLES, help="The number of adversarial samples to use for testing.", show_default=True)
@click.option("--testing-positive-batch-size", type=int, default=None, help="Positive samples per testing batch (default: the training size).", show_default=True)
@click.option("--testing-adversarial-batch-size", type=int, default=None, help="Adversarial samples per testing batch (default: the training size).", show_default=True)
@click.option("--testing-num-batch-threads", type=int, default=1, help="Testing batch threads (accepted, unused).", show_default=True)
@click.option("--resume/--no-resume", default=False, is_flag=True, help="Resume training from the last checkpoint.", show_default=True)
@click.option("--debug/--no-debug", default=False, is_flag=True, help="Enable debug logging.", show_default=True)
# MI355X-path additions (offline stand-ins and run control; not in the reference)
@click.option("--negative-samples", type=int, default=OFFLINE_NEGATIVE_SAMPLES, show_default=True,
              help="Synthetic negatives featurized when the hosted precalculated sets are not on disk.")
@click.option("--validation-negative-samples", type=int, default=OFFLINE_VALIDATION_NEGATIVE_SAMPLES, show_default=True,
              help="Synthetic validation negatives when the hosted validation set is not on disk.")
@click.option("--checkpoint-dir", type=str, default="./checkpoints", show_default=True)
@click.option("--seed", type=int, default=0, show_default=True)
def train(phrase: str, additional_phrase: List[str] = [], wandb_entity: Optional[str] = None,
          architecture: str = DEFAULT_ARCHITECTURE, use_half_layers: bool = DEFAULT_USE_HALF_LAYERS,
          use_gating: bool = DEFAULT_USE_GATING, layer_dim: int = DEFAULT_LAYER_DIM, num_layers: int = DEFAULT_LAYERS,
          num_heads: int = DEFAULT_HEADS, steps: int = DEFAULT_STEPS, stages: int = DEFAULT_STAGES,
          threshold: float = DEFAULT_ACTIVATION_THRESHOLD, learning_rate: float = DEFAULT_LEARNING_RATE,
          high_loss_threshold: float = DEFAULT_HIGH_LOSS_THRESHOLD,
          target_false_positive_rate: float = DEFAULT_TARGET_FALSE_POSITIVE_RATE,
          dynamic_negative_weight: bool = True, negative_weight: float = DEFAULT_NEGATIVE_WEIGHT,
          training_default_size: str = "full", training_dataset: Optional[str] = None,
          augment_phrase_prob: float = DEFAULT_AUGMENT_PHRASE_PROB, augment_phrase_default_words: bool = True,
          augment_phrase_word: List[str] = [], augmentation_default_background_dataset: bool = True,
          augmentation_background_dataset: List[str] = [], augmentation_default_impulse_dataset: bool = True,
          augmentation_impulse_dataset: List[str] = [], augmentation_dataset_streaming: bool = False,
          augmentation_seven_band_prob: float = DEFAULT_AUGMENT_SEVEN_BAND_PROB,
          augmentation_seven_band_gain_db: float = DEFAULT_AUGMENT_SEVEN_BAND_GAIN_DB,
          augmentation_tanh_distortion_prob: float = DEFAULT_AUGMENT_TANH_DISTORTION_PROB,
          augmentation_tanh_distortion_min: float = DEFAULT_AUGMENT_TANH_MIN_DISTORTION,
          augmentation_tanh_distortion_max: float = DEFAULT_AUGMENT_TANH_MAX_DISTORTION,
          augmentation_pitch_shift_prob: float = DEFAULT_AUGMENT_PITCH_SHIFT_PROB,
          augmentation_pitch_shift_semitones: int = DEFAULT_AUGMENT_PITCH_SHIFT_SEMITONES,
          augmentation_band_stop_prob: float = DEFAULT_AUGMENT_BAND_STOP_PROB,
          augmentation_colored_noise_prob: float = DEFAULT_AUGMENT_COLORED_NOISE_PROB,
          augmentation_colored_noise_min_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_SNR_DB,
          augmentation_colored_noise_max_snr_db: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_SNR_DB,
          augmentation_colored_noise_min_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MIN_F_DECAY,
          augmentation_colored_noise_max_f_decay: float = DEFAULT_AUGMENT_COLORED_NOISE_MAX_F_DECAY,
          augmentation_background_noise_prob: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_PROB,
          augmentation_background_noise_min_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MIN_SNR_DB,
          augmentation_background_noise_max_snr_db: float = DEFAULT_AUGMENT_BACKGROUND_NOISE_MAX_SNR_DB,
          augmentation_gain_prob: float = DEFAULT_AUGMENT_GAIN_PROB,
          augmentation_reverb_prob: float = DEFAULT_AUGMENT_REVERB_PROB,
          logging_steps: int = DEFAULT_LOGGING_STEPS, validation_steps: int = DEFAULT_VALIDATION_STEPS,
          checkpoint_steps: int = DEFAULT_CHECKPOINT_STEPS, positive_samples: int = DEFAULT_POSITIVE_SAMPLES,
          adversarial_samples: int = DEFAULT_ADVERSARIAL_SAMPLES, adversarial_phrases: int = DEFAULT_ADVERSARIAL_PHRASES,
          adversarial_phrase_custom: List[str] = [], positive_batch_size: int = DEFAULT_POSITIVE_BATCH_SIZE,
          negative_batch_size: int = DEFAULT_NEGATIVE_BATCH_SIZE,
          adversarial_batch_size: int = DEFAULT_ADVERSARIAL_BATCH_SIZE, num_batch_threads: int = DEFAULT_BATCH_THREADS,
          validation_positive_batch_size: int = DEFAULT_VALIDATION_POSITIVE_BATCH_SIZE,
          validation_negative_batch_size: int = DEFAULT_VALIDATION_NEGATIVE_BATCH_SIZE,
          validation_samples: int = DEFAULT_VALIDATION_SAMPLES, validation_num_batch_threads: int = 1,
          validation_default_dataset: bool = True, validation_dataset: Optional[str] = None,
          testing_positive_samples: int = DEFAULT_TESTING_POSITIVE_SAMPLES,
          testing_adversarial_samples: int = DEFAULT_TESTING_ADVERSARIAL_SAMPLES,
          testing_positive_batch_size: Optional[int] = None, testing_adversarial_batch_size: Optional[int] = None,
          testing_num_batch_threads: int = 1, resume: bool = False, debug: bool = False,
          negative_samples: int = OFFLINE_NEGATIVE_SAMPLES,
          validation_negative_samples: int = OFFLINE_VALIDATION_NEGATIVE_SAMPLES,
          checkpoint_dir: str = "./checkpoints", seed: int = 0) -> None:
    """Trains a wake word detection model (reference __main__.py:245-429):
    WakeWordTrainingDatasetIterator.all -> WakeWordTrainer(...)(...), with the
    featurization and every train step on the device."""
    import numpy as np
    from heybuddy import distributed as hd
    from heybuddy.dataset.training import WakeWordTrainingDatasetIterator
    from heybuddy.trainer import WakeWordTrainer
    from heybuddy.util import logger

    # flag groups sharing a destination (--perceptron / --transformer, --training-*-default-dataset):
    # click >= 8.2 gives such a group the LAST member's default ("False") when no flag is passed
    if architecture not in ("perceptron", "transformer"):
        architecture = DEFAULT_ARCHITECTURE
    if training_default_size not in ("full", "large", "medium", "none"):
        training_default_size = "full"
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1 and not torch.distributed.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    torch.manual_seed(seed)
    np.random.seed(seed)
    if wandb_entity:
        logger.warning("wandb logging is outside the MI355X hot path; ignored")

    phrase_augment_words: List[str] = []
    if augment_phrase_default_words:
        phrase_augment_words.extend(DEFAULT_AUGMENT_PHRASE_WORDS)
    phrase_augment_words.extend(augment_phrase_word or [])
    background: List[str] = []
    if augmentation_default_background_dataset:
        background.extend([DEFAULT_BACKGROUND_DATASET] if isinstance(DEFAULT_BACKGROUND_DATASET, str)
                          else DEFAULT_BACKGROUND_DATASET)
    background.extend(augmentation_background_dataset or [])
    impulse: List[str] = []
    if augmentation_default_impulse_dataset:
        impulse.extend([DEFAULT_IMPULSE_DATASET] if isinstance(DEFAULT_IMPULSE_DATASET, str)
                       else DEFAULT_IMPULSE_DATASET)
    impulse.extend(augmentation_impulse_dataset or [])

    training, validation, testing = WakeWordTrainingDatasetIterator.all(
        wake_phrase=phrase, additional_wake_phrases=list(additional_phrase or []),
        adversarial_per_batch=adversarial_batch_size, augment_background_dataset=background,
        augment_background_noise_max_snr_db=augmentation_background_noise_max_snr_db,
        augment_background_noise_min_snr_db=augmentation_background_noise_min_snr_db,
        augment_background_noise_prob=augmentation_background_noise_prob,
        augment_band_stop_prob=augmentation_band_stop_prob,
        augment_colored_noise_max_f_decay=augmentation_colored_noise_max_f_decay,
        augment_colored_noise_max_snr_db=augmentation_colored_noise_max_snr_db,
        augment_colored_noise_min_f_decay=augmentation_colored_noise_min_f_decay,
        augment_colored_noise_min_snr_db=augmentation_colored_noise_min_snr_db,
        augment_colored_noise_prob=augmentation_colored_noise_prob,
        augment_dataset_streaming=augmentation_dataset_streaming, augment_gain_prob=augmentation_gain_prob,
        augment_impulse_dataset=impulse, augment_pitch_shift_prob=augmentation_pitch_shift_prob,
        augment_pitch_shift_semitones=augmentation_pitch_shift_semitones,
        augment_reverb_prob=augmentation_reverb_prob, augment_seven_band_gain_db=augmentation_seven_band_gain_db,
        augment_seven_band_prob=augmentation_seven_band_prob,
        augment_tanh_distortion_prob=augmentation_tanh_distortion_prob,
        augment_tanh_max_distortion=augmentation_tanh_distortion_max,
        augment_tanh_min_distortion=augmentation_tanh_distortion_min,
        custom_adversarial_phrases=list(adversarial_phrase_custom or []), custom_training=training_dataset,
        large_training=training_default_size in ["full", "large"],
        medium_training=training_default_size in ["full", "medium"], negative_per_batch=negative_batch_size,
        num_adversarial_phrases=adversarial_phrases, num_adversarial_samples=adversarial_samples,
        num_batch_threads=num_batch_threads, num_positive_samples=positive_samples,
        phrase_augment_prob=augment_phrase_prob, phrase_augment_words=phrase_augment_words,
        positive_per_batch=positive_batch_size, testing_adversarial_per_batch=testing_adversarial_batch_size,
        testing_num_adversarial_samples=testing_adversarial_samples,
        testing_num_batch_threads=testing_num_batch_threads, testing_num_positive_samples=testing_positive_samples,
        testing_positive_per_batch=testing_positive_batch_size, validation_custom=validation_dataset,
        validation_include_precalculated=validation_default_dataset,
        validation_negative_batch_size=validation_negative_batch_size,
        validation_num_batch_threads=validation_num_batch_threads, validation_num_positive_samples=validation_samples,
        validation_positive_batch_size=validation_positive_batch_size,
        device_id=device.index, seed=seed, offline_negative_samples=negative_samples,
        offline_validation_negative_samples=validation_negative_samples)

    rank, world = hd.world()
    trainer = WakeWordTrainer(checkpoint_dir=checkpoint_dir, architecture=architecture,
                              use_half_layers=use_half_layers, use_gating=use_gating, layer_dim=layer_dim,
                              num_layers=num_layers, num_heads=num_heads, device=device)
    name = safe_name(phrase)
    if resume:
        trainer.resume(name)
    trainer(training=training, validation=validation, testing=testing, activation_threshold=threshold,
            checkpoint_steps=checkpoint_steps, dynamic_negative_weight=dynamic_negative_weight,
            high_loss_threshold=high_loss_threshold, learning_rate=learning_rate,
            max_negative_weight=negative_weight, name=name if rank == 0 else f"{name}_rank{rank}",
            num_stages=stages, num_steps=steps, target_false_positive_rate=target_false_positive_rate,
            validation_steps=validation_steps, logging_steps=logging_steps, wandb_entity=wandb_entity)
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
            # BERTTokenizer(length=L) (tokens.py:53-66): ids without [CLS] / [SEP]
            # (encode(text).ids[1:-1]), cut to L, padded with 0
            def tok(text):
                ids = list(t(text, add_special_tokens=False)["input_ids"])[:tokenizer_max_length]
                return ids + [0] * (tokenizer_max_length - len(ids))
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
