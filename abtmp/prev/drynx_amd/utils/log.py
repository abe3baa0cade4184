"""Logging with onet-style verbosity levels (reference: onet ``log.Lvl1..5``,
``log.SetDebugVisible``; services log prefix ``[SERVICE] <drynx> Server``,
services/service.go:264-277).  ``DRYNX_DEBUG=<lvl>`` sets the visible level."""
from __future__ import annotations

import logging
import os
import sys

_LEVEL = int(os.environ.get("DRYNX_DEBUG", "1"))
_handler = logging.StreamHandler(sys.stderr)
_handler.setFormatter(logging.Formatter("%(asctime)s [%(name)s] %(levelname)s %(message)s", "%H:%M:%S"))


def get_logger(name: str) -> logging.Logger:
    lg = logging.getLogger(f"drynx.{name}")
    if not lg.handlers:
        lg.addHandler(_handler)
        lg.propagate = False
    lg.setLevel(logging.DEBUG if _LEVEL >= 3 else logging.INFO if _LEVEL >= 1 else logging.WARNING)
    return lg


def set_debug_visible(level: int):
    global _LEVEL
    _LEVEL = level
    for name, lg in logging.Logger.manager.loggerDict.items():
        if name.startswith("drynx.") and isinstance(lg, logging.Logger):
            lg.setLevel(logging.DEBUG if level >= 3 else logging.INFO if level >= 1 else logging.WARNING)
