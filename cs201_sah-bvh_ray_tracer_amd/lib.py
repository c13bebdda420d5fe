"""Loader for libmirt.so (the HIP render path behind include/mirt.h).

The library is built in-tree (`make -C csrc`, or __graft_entry__.build()).
There is no fallback: if the shared object is missing or cannot be loaded,
every entry point raises.
"""
import ctypes as C
import os
import subprocess

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
# MIRT_LIB: another build of the same ABI (A/B measurements of kernel variants)
LIB_PATH = os.environ.get("MIRT_LIB") or os.path.join(HERE, "libmirt.so")
_lib = None


class MirtError(RuntimeError):
    pass


def build(jobs=8):
    """Compile libmirt.so for gfx950 (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "csrc"), f"-j{jobs}"], check=True)
    return LIB_PATH


def load():
    """The loaded library (raises MirtError if it is not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MirtError(f"{LIB_PATH} is not built: run __graft_entry__.build() or `make -C csrc`")
        L = C.CDLL(LIB_PATH)
        for name, res, args in abi.SIGNATURES:
            try:
                f = getattr(L, name)
            except AttributeError:
                if os.environ.get("MIRT_LIB"):
                    continue  # an older build under A/B: entry points it lacks stay unbound
                raise
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


def check(rc, what="mirt"):
    if rc < 0:
        msg = load().mirt_last_error().decode(errors="replace")
        raise MirtError(f"{what} failed ({rc}): {msg}")
    return rc
