"""Access to the native timing tree (SPFFT_TIMING=1 or timing_enable())."""
from __future__ import annotations

import ctypes
import json

from ..ops._lib import lib


def timing_enable(on: bool = True, gpu_stages: bool = True) -> None:
    """Host timer scopes, plus (gpu_stages) hipEvent intervals of every GPU stage
    under gpu/<direction>/<stage>."""
    lib().spfft_amd_timing_enable((2 if gpu_stages else 1) if on else 0)


def timing_reset() -> None:
    lib().spfft_amd_timing_reset()


def _report(fn) -> str:
    need = ctypes.c_size_t()
    fn(None, 0, ctypes.byref(need))
    buf = ctypes.create_string_buffer(need.value)
    fn(buf, need.value, None)
    return buf.value.decode()


def timing_json() -> dict:
    return json.loads(_report(lib().spfft_amd_timing_json))


def timing_report() -> str:
    return _report(lib().spfft_amd_timing_print)
