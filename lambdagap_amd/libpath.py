"""Locate (and if needed build) the native library ``lib_lambdagap.so``.

The library is built in-tree by the top-level ``Makefile`` (host C++ with
OpenMP + HIP kernels cross-compiled for gfx950), so the same file ships to a
GPU box with the source tree.
"""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

PACKAGE_DIR = Path(__file__).resolve().parent
REPO_ROOT = PACKAGE_DIR.parent
LIB_NAME = "lib_lambdagap.so"


def find_lib_path() -> str:
    """Return the path of the native library, building it if it is missing."""
    env = os.environ.get("LAMBDAGAP_LIB")
    candidates = [Path(env)] if env else []
    candidates.append(PACKAGE_DIR / "lib" / LIB_NAME)
    for c in candidates:
        if c.is_file():
            return str(c)
    if (REPO_ROOT / "Makefile").is_file() and os.environ.get("LAMBDAGAP_NO_AUTOBUILD") != "1":
        build_native()
        p = PACKAGE_DIR / "lib" / LIB_NAME
        if p.is_file():
            return str(p)
    raise FileNotFoundError(
        f"Cannot find {LIB_NAME}; run `make -j8` in {REPO_ROOT} (needs hipcc from ROCm)")


def cli_path() -> str:
    return str(PACKAGE_DIR / "lib" / "lambdagap")


def build_native(jobs: int | None = None, arch: str = "gfx950") -> None:
    """Compile the host library, HIP kernels and CLI with the repository Makefile."""
    jobs = jobs or min(16, os.cpu_count() or 4)
    cmd = ["make", f"-j{jobs}", f"ARCH={arch}"]
    subprocess.run(cmd, cwd=str(REPO_ROOT), check=True)
