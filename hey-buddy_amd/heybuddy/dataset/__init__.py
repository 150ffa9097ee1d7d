"""Device-resident data path of the hot loop: clip placement and batch
augmentation, the feature generator, precalculated feature sets and the
training batch sampler."""
from heybuddy.dataset.augmented import AugmentedAudioGenerator, BatchAugmenter
from heybuddy.dataset.features import TrainingFeaturesGenerator
from heybuddy.dataset.precalculated import PrecalculatedDatasetIterator
from heybuddy.dataset.training import DevicePool, TrainingDatasetIterator, WakeWordTrainingDatasetIterator

__all__ = ["AugmentedAudioGenerator", "BatchAugmenter", "DevicePool", "PrecalculatedDatasetIterator",
           "TrainingDatasetIterator", "TrainingFeaturesGenerator", "WakeWordTrainingDatasetIterator"]
