"""Host-side helpers mirroring heybuddy.util of the reference (only what the
hot path needs: input normalisation and logging)."""
from heybuddy.util.audio_util import audio_to_bct_tensor, resample
from heybuddy.util.log_util import logger

__all__ = ["audio_to_bct_tensor", "logger", "resample"]
