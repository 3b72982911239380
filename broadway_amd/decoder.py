"""Host-side mirror of Broadway's JavaScript decoder API.

``Decoder(options).decode(nal, info)`` -> ``onPictureDecoded(buffer, width,
height, infos)`` with the semantics of templates/DecoderPost.js:55-285 on top
of the wasm glue of Decoder/src/Decoder.c:44-162:

* ``decode`` copies the input into the decoder's stream buffer (a 1 MiB heap
  buffer in the reference, DecoderPost.js:152/:283) and runs synchronously;
* ``onPictureDecoded`` receives the MB-aligned planar I420 picture
  (``width*height*3/2`` bytes, width/height multiples of 16, no cropping --
  H264SwDecApi.c:233-234) plus the ``infos`` collected since the last picture
  with ``startDecoding``/``finishDecoding`` stamps (DecoderPost.js:77-103);
* after a picture completes, the rest of the buffer is dropped
  (Decoder.c:122-134) and the DPB is never flushed (Decoder.c:140), so
  pictures held for display reordering are not emitted.

* ``rgb: true`` (DecoderPost.js:82-97): ``onPictureDecoded`` receives a new
  RGBA array (``width*height*4`` bytes) converted on the GPU with the
  reference converter's per-pixel arithmetic (yuv2rgbcalc, :514-560) --
  ``H264SwDecNextPictureRGBA`` instead of ``H264SwDecNextPicture``.

Unlike the reference module (a single global instance) every ``Decoder`` has
its own H264SwDec instance, so several streams can be decoded side by side.
Reconstruction always runs on the GPU through libh264mi.so; ``sliceMode``
(per-slice web workers) is not supported.
"""
from __future__ import annotations

import ctypes as C
import time
from typing import Callable, List, Optional

import numpy as np

from . import _lib

STREAM_BUFFER_SIZE = 1024 * 1024


def _now() -> float:
    return time.perf_counter() * 1000.0


class Decoder:
    def __init__(self, options: Optional[dict] = None):
        self.options = dict(options or {})
        if self.options.get("sliceMode"):
            raise NotImplementedError("sliceMode (per-slice workers) is not part of the MI355X path")
        self._rgb = bool(self.options.get("rgb"))
        self._L = _lib.mi()
        inst = C.c_void_p()
        ret = self._L.H264SwDecInit(C.byref(inst), 0)
        if ret != _lib.H264SWDEC_OK:
            raise RuntimeError(f"DECODER INITIALIZATION FAILED ({ret})")
        self._inst = inst
        self._buf = (C.c_uint8 * STREAM_BUFFER_SIZE)()
        self._info = _lib.H264SwDecInfo()
        self._pic = _lib.H264SwDecPicture()
        self.infoAr: List[dict] = []
        self.pic_decode_number = 1
        self.pic_display_number = 1
        self.onPictureDecoded: Callable = lambda buffer, width, height, infos: None
        self.onHeadersDecoded: Callable = lambda: None

    # DecoderPost.js:275-285 + Decoder.c:44-53
    def decode(self, typed_ar, par_info: Optional[dict] = None) -> None:
        data = bytes(typed_ar)
        if len(data) > STREAM_BUFFER_SIZE:
            raise ValueError("NAL larger than the 1 MiB stream buffer (DecoderPost.js:152)")
        if par_info is not None:
            self.infoAr.append(par_info)
            par_info["startDecoding"] = _now()
        C.memmove(self._buf, data, len(data))
        inp = _lib.H264SwDecInput()
        out = _lib.H264SwDecOutput()
        inp.pStream = C.cast(self._buf, C.POINTER(C.c_uint8))
        inp.dataLen = len(data)
        base = C.addressof(self._buf)
        while inp.dataLen > 0:
            self._decode_once(inp, out, base)

    # Decoder.c:100-162
    def _decode_once(self, inp, out, base) -> int:
        L = self._L
        inp.picId = self.pic_decode_number
        ret = L.H264SwDecDecode(self._inst, C.byref(inp), C.byref(out))

        def consumed() -> int:
            return C.cast(out.pStrmCurrPos, C.c_void_p).value - C.cast(inp.pStream, C.c_void_p).value

        if ret == _lib.H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY:
            if L.H264SwDecGetInfo(self._inst, C.byref(self._info)) != _lib.H264SWDEC_OK:
                return -1
            self.onHeadersDecoded()
            n = consumed()
            inp.dataLen -= n
            inp.pStream = out.pStrmCurrPos
        elif ret in (_lib.H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY, _lib.H264SWDEC_PIC_RDY):
            inp.dataLen = 0
            self.pic_decode_number += 1
            while True:
                if self._rgb:
                    w, h = self._info.picWidth, self._info.picHeight
                    rgba = np.empty(w * h * 4, dtype=np.uint8)
                    if L.H264SwDecNextPictureRGBA(self._inst, C.byref(self._pic), 0,
                                                  rgba.ctypes.data) != _lib.H264SWDEC_PIC_RDY:
                        break
                    self.pic_display_number += 1
                    self._emit(self._pic, rgba)
                else:
                    if L.H264SwDecNextPicture(self._inst, C.byref(self._pic), 0) != _lib.H264SWDEC_PIC_RDY:
                        break
                    self.pic_display_number += 1
                    self._emit(self._pic)
        elif ret in (_lib.H264SWDEC_STRM_PROCESSED, _lib.H264SWDEC_STRM_ERR):
            inp.dataLen = 0
        return ret

    def _emit(self, pic, rgba=None) -> None:
        w, h = self._info.picWidth, self._info.picHeight
        if rgba is not None:
            buf = rgba
        else:
            n = w * h * 3 // 2
            buf = np.ctypeslib.as_array(C.cast(pic.pOutputPicture, C.POINTER(C.c_uint8)), shape=(n,))
        infos = None
        if self.infoAr:
            infos = self.infoAr
            infos[0]["finishDecoding"] = _now()
        self.infoAr = []
        self.onPictureDecoded(buf, w, h, infos)

    def info(self) -> _lib.H264SwDecInfo:
        return self._info

    def close(self) -> None:
        if self._inst:
            self._L.H264SwDecRelease(self._inst)
            self._inst = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def split_annexb(stream: bytes) -> List[bytes]:
    """Split an Annex-B stream into NAL units (with their start codes), the
    way Player/mp4.js feeds one NAL per decode() call."""
    out = []
    i, n = 0, len(stream)
    starts = []
    while i + 3 <= n:
        if stream[i] == 0 and stream[i + 1] == 0 and stream[i + 2] == 1:
            s = i - 1 if i > 0 and stream[i - 1] == 0 else i
            starts.append(s)
            i += 3
        else:
            i += 1
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else n
        out.append(stream[s:e])
    return out
