"""matcha_hip — MI355X (gfx950) runtime for the Matcha-TTS synthesis hot path.

Importing this package does not touch the GPU or load the native library; the
library is loaded on first use (``matcha_hip._lib.lib()``).
"""
from ._lib import LIB_PATH, HipPathError, lib  # noqa: F401

__all__ = ["LIB_PATH", "HipPathError", "lib", "runtime", "synthetic"]


def __getattr__(name):
    if name in ("runtime", "synthetic"):
        import importlib
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
