"""Logging set-up shared by the worker and the rater.

The reference configures the *same* logger (literally named ``"__name__"``)
twice -- once in /root/reference/worker.py:202-217 and once in
/root/reference/rater.py:172-188 -- so every INFO line is printed twice.  We
keep the logger name and the stdout/stderr split (INFO/DEBUG -> stdout,
WARNING+ -> stderr) but attach the handlers exactly once.
"""
from __future__ import annotations

import logging
import sys

LOGGER_NAME = "__name__"


class InfoFilter(logging.Filter):
    """Pass only DEBUG/INFO records (the stdout half of the split)."""

    def filter(self, record: logging.LogRecord) -> bool:
        return record.levelno in (logging.DEBUG, logging.INFO)


def get_logger() -> logging.Logger:
    logger = logging.getLogger(LOGGER_NAME)
    if not getattr(logger, "_analyzer_amd_configured", False):
        logger.setLevel(logging.INFO)
        out = logging.StreamHandler(sys.stdout)
        out.setLevel(logging.INFO)
        out.addFilter(InfoFilter())
        err = logging.StreamHandler(sys.stderr)
        err.setLevel(logging.WARNING)
        logger.addHandler(out)
        logger.addHandler(err)
        logger._analyzer_amd_configured = True  # type: ignore[attr-defined]
    return logger
