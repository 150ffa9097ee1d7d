"""CPU oracle for the hey-buddy hot path — TEST INFRASTRUCTURE ONLY.

This package is a plain numpy restatement of the reference algorithms
(therealadityashankar/hey-buddy, src/python/heybuddy/...) used as the parity
checker for the HIP kernels in ``hey-buddy_amd/``. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker / the timed CPU baseline — never as the product
path. The product (``heybuddy`` package) fails loudly when libhbk.so is missing
and never falls back to anything in here.

Pinning:
  * featurizer orchestration (frame / window index maps, batching, NaN
    replacement) — pinned bit-exactly against the reference's own
    ``SpeechEmbeddings`` run with index-encoding fakes (tests/golden/).
  * classifier forward / BCE filter / Adam / LR schedule / train_epoch —
    pinned against the reference's ``WakeWordMLPModel`` and
    ``WakeWordTrainer.train_epoch`` run on seeded inputs (tests/golden/).
  * mel graph and speech-embedding graph numerics — PARITY UNPINNED against
    the true ONNX graphs (not in the reference tree, network fetch only,
    spectrogram.py:20, embeddings.py:29); restated from their documented
    construction (torchaudio MelSpectrogram, H0 parameters) and a generic conv
    executor over runtime weights.
  * add_noise / reverberate — PARITY UNPINNED (torchaudio / speechbrain are
    not installed and hold no fixtures in the reference); restated from their
    published algorithms at the versions pinned in environment.yml.
"""
