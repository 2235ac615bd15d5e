"""ctypes loader for libfddm_hip.so (the C-ABI declared in include/fddm_hip.h).

The argument types are derived from the header itself, so the Python side and the C declarations
cannot drift apart. There is deliberately no fallback: importing the product path without the
compiled library raises, and every nonzero hipError_t becomes a RuntimeError.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FDDM_HIP_LIB", os.path.join(_HERE, "libfddm_hip.so"))
_HEADER_CANDIDATES = [
    os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "fddm_hip.h"),
    os.path.join(os.path.dirname(_HERE), "include", "fddm_hip.h"),
]


def header_path() -> str:
    for p in _HEADER_CANDIDATES:
        if os.path.exists(p):
            return p
    raise FileNotFoundError("include/fddm_hip.h not found next to the package")


def _ctype(t: str):
    t = t.strip()
    if "*" in t:
        return ctypes.c_void_p
    t = t.replace("const", "").strip()
    if t == "unsigned long long":
        return ctypes.c_uint64
    if t == "long":
        return ctypes.c_long
    if t in ("int",):
        return ctypes.c_int
    if t == "float":
        return ctypes.c_float
    if t == "double":
        return ctypes.c_double
    if t == "void":
        return None
    raise ValueError(f"unsupported C type {t!r}")


def parse_header(path: str | None = None) -> dict:
    """Return {name: (restype, [argtypes])} for every function declared in the header."""
    src = open(path or header_path()).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    decls = {}
    for m in re.finditer(r"(const\s+char\s*\*|int|long)\s+(fddm_\w+)\s*\(([^)]*)\)\s*;", src):
        ret, name, args = m.group(1), m.group(2), m.group(3).strip()
        restype = ctypes.c_char_p if "char" in ret else ctypes.c_long if ret == "long" else ctypes.c_int
        argtypes = []
        if args and args != "void":
            for a in args.split(","):
                a = a.strip()
                # drop the parameter name
                mm = re.match(r"(.*?)(\w+)$", a)
                argtypes.append(_ctype(mm.group(1)))
        decls[name] = (restype, argtypes)
    return decls


_lib = None
_decls = None


def lib():
    global _lib, _decls
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libfddm_hip.so not built ({LIB_PATH}); run `make -C fddm-asr_amd` or "
                              "__graft_entry__.build(). There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        _decls = parse_header()
        for name, (res, args) in _decls.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        # diagnostic A/B knob (tools/ab.sh): FDDM_ATTN_KERNELS = auto | v6 | nofused | fwd7 | fwd8 | relfwd5 (ops.ATTN_KERNELS)
        ak = os.environ.get("FDDM_ATTN_KERNELS")
        if ak:
            L.fddm_attn_set_kernels({"auto": 0, "v6": 1, "nofused": 2, "fwd7": 3, "fwd8": 4, "relfwd5": 5}[ak])
    return _lib


def declared_symbols():
    return sorted(parse_header().keys())


def call(name: str, *args):
    f = getattr(lib(), name)
    rc = f(*args)
    if rc != 0:
        msg = lib().fddm_error_string(rc)
        raise RuntimeError(f"{name} failed: hipError {rc} ({msg.decode() if msg else '?'})")
    return rc
