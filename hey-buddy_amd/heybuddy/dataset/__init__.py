"""Device-resident data path of the hot loop: batch augmentation, the
training batch sampler, and the feature generator."""
from heybuddy.dataset.augmented import BatchAugmenter
from heybuddy.dataset.training import DevicePool, TrainingDatasetIterator, WakeWordTrainingDatasetIterator

__all__ = ["BatchAugmenter", "DevicePool", "TrainingDatasetIterator", "WakeWordTrainingDatasetIterator"]
