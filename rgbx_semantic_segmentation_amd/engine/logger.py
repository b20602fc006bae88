"""Engine logger (reference: engine/logger.py) -- level from ENGINE_LOGGING_LEVEL, optional file."""
from __future__ import annotations

import logging
import os

_LEVEL = logging.getLevelName(os.getenv("ENGINE_LOGGING_LEVEL", "INFO").upper())


def get_logger(log_dir: str | None = None, log_file: str | None = None) -> logging.Logger:
    logger = logging.getLogger("cmx_engine")
    logger.setLevel(_LEVEL)
    if not logger.handlers:
        h = logging.StreamHandler()
        h.setFormatter(logging.Formatter("%(asctime)s %(message)s"))
        logger.addHandler(h)
        logger.propagate = False
    if log_file is not None:
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)
        fh = logging.FileHandler(log_file, mode="a")
        fh.setFormatter(logging.Formatter("[%(asctime)s %(lineno)d@%(filename)s:%(name)s] %(message)s"))
        logger.addHandler(fh)
    return logger
