"""MI355X runtime for the FDDM-ASR train step: ctypes binding of libfddm_hip (C-ABI in
include/fddm_hip.h), autograd Functions, fused optimizer and data-parallel helpers."""
from . import _lib, ops, runtime  # noqa: F401
from .runtime import precision, set_precision, use_precision  # noqa: F401

_lib.lib()  # fail loudly at import if the HIP library is missing: there is no fallback path
