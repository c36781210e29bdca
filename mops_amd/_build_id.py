"""Identity of the engine build (``mops_build_id`` in include/mops_traj.h).

A sha256 over everything that determines the machine code of
``libmops_traj.so``: the engine's sources and headers, the hipcc flags and the
ROCm release.  ``__graft_entry__.build_engine`` stamps it into the library at
compile time; ``_lib.load`` refuses a library whose stamp differs from the
sources next to it, so a stale binary (built from older sources, or by another
toolchain) never runs.  bench.py keys its PMC traffic records on the same id.
"""
from __future__ import annotations

import hashlib
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_PKG)
CSRC = os.path.join(_PKG, "csrc")
SOURCES = tuple(os.path.join(CSRC, f) for f in ("mops_engine.hip", "mops_api.cpp", "mops_io.cpp", "mops_netcdf.cpp"))
HEADERS = tuple(os.path.join(ROOT, "include", f) for f in ("mops_traj.h", "mops_io.h", "mops_netcdf.h",
                                                           os.path.join("mops", "MOPS.h")))
# bit-parity with the reference's x86-64 -O2 build: no FMA contraction
HIPCC_FLAGS = ("--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off")
MARKER = "mops-build-id:"


def rocm_version() -> str:
    try:
        with open("/opt/rocm/.info/version") as f:
            return f.read().strip()
    except OSError:
        return "unknown"


def build_id(extra_flags=()) -> str:
    """16 hex digits over sources, headers, flags and the ROCm release."""
    h = hashlib.sha256()
    for p in SOURCES + HEADERS:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(HIPCC_FLAGS + tuple(extra_flags)).encode())
    h.update(rocm_version().encode())
    return h.hexdigest()[:16]


def stamped_id(lib_path: str) -> str | None:
    """The id compiled into a library file (without loading it), or None."""
    try:
        with open(lib_path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(MARKER.encode())
    if i < 0:
        return None
    return data[i + len(MARKER):i + len(MARKER) + 16].decode(errors="replace")
