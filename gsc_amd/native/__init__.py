"""Loader for the in-tree native extension (HIP kernels + host simulator path).

The extension is built by :func:`gsc_amd.native.build.build` (``__graft_entry__.build``).  Import
fails loudly when it is missing: there is no silent Python fallback for the device path.
"""
from __future__ import annotations

import importlib
import os

_mod = None


def load(auto_build: bool = None):
    """Return the ``gsc_amd._native`` module (building it first if allowed and missing)."""
    global _mod
    if _mod is not None:
        return _mod
    if auto_build is None:
        auto_build = os.environ.get("GSC_AUTO_BUILD", "1") == "1"
    so = os.environ.get("GSC_NATIVE_SO")
    if so:  # an alternative build of the same module (e.g. the host-sanitizer build, scripts/asan_check.sh)
        import importlib.util as ilu
        import sys
        spec = ilu.spec_from_file_location("gsc_amd._native", so)
        _mod = ilu.module_from_spec(spec)
        spec.loader.exec_module(_mod)
        sys.modules["gsc_amd._native"] = _mod
        return _mod
    try:
        _mod = importlib.import_module("gsc_amd._native")
    except ImportError:
        if not auto_build:
            raise ImportError("gsc_amd native extension not built: run `python -m gsc_amd.native.build` "
                              "(or __graft_entry__.build())") from None
        from .build import build
        build(verbose=False)
        _mod = importlib.import_module("gsc_amd._native")
    return _mod


def available() -> bool:
    try:
        load(auto_build=False)
        return True
    except ImportError:
        return False
