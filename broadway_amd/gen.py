"""Seeded synthetic H.264 Baseline stream generator (Python binding).

Configs follow BASELINE.json ``configs`` / SURVEY.md §8d:
  0  640x368 (crop 360) plumbing stream, loop filter off (substitute for the
     missing Player/mozilla_story.mp4)
  1  1280x720 I-slices only
  2  1920x1088 (crop 1080) I+P, 1 I per 60, 4 slices, deblock idc 0/2
  3  same stream type as 2 (64 streams = seeds 100..163, 8 per GPU)
  4  3840x2160 I+P
"""
from __future__ import annotations

import ctypes as C

from . import _lib


def params(config: int, seed: int, **overrides) -> _lib.GenParams:
    p = _lib.GenParams()
    if _lib.gen().h264gen_preset(C.byref(p), int(config), int(seed)) != 0:
        raise ValueError(f"unknown config {config}")
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise KeyError(k)
        setattr(p, k, int(v))
    return p


def generate(config: int = 2, seed: int = 1, **overrides) -> bytes:
    """Return an Annex-B byte stream."""
    p = params(config, seed, **overrides)
    out = C.POINTER(C.c_uint8)()
    n = C.c_size_t()
    L = _lib.gen()
    if L.h264gen_generate(C.byref(p), C.byref(out), C.byref(n)) != 0:
        raise RuntimeError("stream generation failed")
    try:
        return C.string_at(out, n.value)
    finally:
        L.h264gen_free(out)


def cavlc_selftest(iters: int = 20000, seed: int = 1) -> int:
    """Round-trip random residual blocks through CAVLC encode/decode;
    returns the number of mismatches (0 expected)."""
    return _lib.gen().h264gen_cavlc_selftest(int(iters), int(seed))
