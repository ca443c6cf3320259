"""Loader for the in-tree native extension (``_native*.so``, built by ``make``).

The extension links ``build/lib/libbibfs.so`` (HIP kernels for gfx950 + RCCL).
There is no pure-Python fallback for the engines: if the extension is missing
the import fails loudly with the build command to run.
"""
from __future__ import annotations

import importlib
import os

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

try:
    native = importlib.import_module("bidirectional_bfs_amd._native")
except ImportError as exc:  # pragma: no cover - exercised only on a broken build
    raise ImportError(
        "bidirectional_bfs_amd native extension is not built; run `make -j8` in "
        f"{_REPO} (or python -c 'import __graft_entry__ as g; g.build()')"
    ) from exc

BibfsError = native.BibfsError

__all__ = ["native", "BibfsError", "repo_root", "tool_path"]


def repo_root() -> str:
    return _REPO


def tool_path(name: str) -> str:
    """Absolute path of a native CLI tool in build/bin (bibfs_serial, second_try, ...).

    ``BIBFS_BIN_DIR`` overrides the directory (e.g. ``build-asan/bin`` for the
    sanitizer build, ``make asan``)."""
    p = os.path.join(os.environ.get("BIBFS_BIN_DIR") or os.path.join(_REPO, "build", "bin"), name)
    if not os.path.exists(p):
        raise FileNotFoundError(f"{p} missing; run `make -j8` in {_REPO}")
    return p
