"""Loads the native module (``mpit_amd/_mpit*.so``), building it in-tree if missing.

There is no Python fallback for any op: if the extension cannot be loaded the import
fails loudly, so a GPU run can never silently measure an eager/PyTorch path.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
import threading

_lock = threading.Lock()
_mod = None


def native():
    """Return the ``_mpit`` extension module (build it first if it is absent)."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        so = os.environ.get("MPIT_NATIVE_SO")
        if so:  # an explicitly built variant (e.g. the sanitizer builds of _build.py)
            spec = importlib.util.spec_from_file_location("mpit_amd._mpit", so)
            _mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_mod)
            sys.modules["mpit_amd._mpit"] = _mod
            return _mod
        try:
            _mod = importlib.import_module("mpit_amd._mpit")
        except ImportError:
            if os.environ.get("MPIT_NO_AUTOBUILD"):
                raise
            from . import _build

            _build.build()
            importlib.invalidate_caches()
            _mod = importlib.import_module("mpit_amd._mpit")
    return _mod


def native_path() -> str:
    return native().__file__
