"""hey-buddy, MI355X-native hot path.

Drop-in for the featurizer (``heybuddy.embeddings``, ``heybuddy.spectrogram``),
the feature generator (``heybuddy.dataset.features``) and the wake-word
trainer (``heybuddy.trainer``, ``heybuddy train`` CLI) of
therealadityashankar/hey-buddy, with every hot op running as hand-written HIP
for gfx950 through libhbk.so (include/hbk.h).
"""
__version__ = "0.1.0"
