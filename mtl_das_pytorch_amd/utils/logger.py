"""Console tee logger (reference utils.py:23-48), written incrementally.

The reference buffers the whole console transcript in memory and appends it to
``console output.log`` only when the run finishes (utils.py:223), so a crash loses the log.  This
version mirrors every write to the terminal and flushes it to the file immediately; ``save()`` is kept
for API compatibility.  Only rank 0 opens the file under data parallelism.
"""
from __future__ import annotations

import os
import sys


class Logger:
    def __init__(self, filename: str = "Default.log", path: str = "./", terminal=None, enabled: bool = True,
                 append: bool = True):
        """The log file is written incrementally (the reference keeps it in memory until the end and
        loses it on a crash); an elastic restart (``append``) continues the same file."""
        self.terminal = terminal if terminal is not None else sys.stdout
        self.filename = filename
        self.path = path
        self.log = ""
        self._fh = None
        if enabled:
            os.makedirs(path, exist_ok=True)
            self._fh = open(os.path.join(path, filename), "a" if append else "w", encoding="utf-8")

    def write(self, message: str):
        self.terminal.write(message)
        self.log += message
        if self._fh is not None:
            self._fh.write(message)
            self._fh.flush()

    def flush(self):
        self.terminal.flush()
        if self._fh is not None:
            self._fh.flush()

    def save(self):
        self.flush()

    def close(self):
        if self._fh is not None:
            self._fh.close()
            self._fh = None

    def isatty(self):
        return False


class tee_stdout:
    """Context manager installing a :class:`Logger` as ``sys.stdout``."""

    def __init__(self, logger: Logger):
        self.logger = logger
        self._old = None

    def __enter__(self):
        self._old = sys.stdout
        sys.stdout = self.logger
        return self.logger

    def __exit__(self, *exc):
        sys.stdout = self._old
        self.logger.close()
        return False
