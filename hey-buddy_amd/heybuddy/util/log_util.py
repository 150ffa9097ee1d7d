"""The ``heybuddy`` logger (reference: util/log_util.py:39)."""
import logging

logger = logging.getLogger("heybuddy")
if not logger.handlers:
    _h = logging.StreamHandler()
    _h.setFormatter(logging.Formatter("%(asctime)s [%(levelname)s] %(name)s: %(message)s"))
    logger.addHandler(_h)
    logger.setLevel(logging.INFO)
