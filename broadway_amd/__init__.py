"""broadway_amd -- MI355X-native H.264 Baseline macroblock-reconstruction path
for the Broadway decoder API.

Layout:
  csrc/common  bit I/O, CAVLC, H.264 tables, neighbour / MV-prediction logic
  csrc/host    host parser (NAL, parameter sets, slice data -> MB records),
               DPB bookkeeping, H264SwDec*/broadway* C-ABI, record capture
  csrc/hip     HIP kernels for gfx950 (k_prep, k_wgpp, k_conceal, k_yuv2rgba, k_omx) and
               the engine
  csrc/gen     seeded synthetic Baseline stream generator
  decoder.py   Decoder.js-style API (decode(nal) -> onPictureDecoded)
  engine.py    batched multi-stream reconstruction (throughput path)
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
