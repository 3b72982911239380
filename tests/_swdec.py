"""DecTestBench-style driver of the product H264SwDec* C-ABI (ctypes): feed
the whole Annex-B buffer, drain NextPicture after every PIC_RDY, flush at end
of stream (reference DecTestBench.c:218-416 call protocol: picId counts
decoded pictures from 1; STRM_PROCESSED / STRM_ERR end a byte-stream run)."""
import ctypes as C

from broadway_amd import _lib


def swdec_decode(stream: bytes, no_reorder: bool = False, info: bool = False):
    """Returns (frames, error_returns) [+ per output picture (picId,
    isIdrPicture, nbrOfErrMBs) if info]."""
    L = _lib.mi()
    inst = C.c_void_p()
    assert L.H264SwDecInit(C.byref(inst), int(no_reorder)) == _lib.H264SWDEC_OK
    buf = (C.c_uint8 * len(stream)).from_buffer_copy(stream)
    inp, out = _lib.H264SwDecInput(), _lib.H264SwDecOutput()
    pic, dinfo = _lib.H264SwDecPicture(), _lib.H264SwDecInfo()
    inp.pStream = C.cast(buf, C.POINTER(C.c_uint8))
    inp.dataLen = len(stream)
    inp.intraConcealmentMethod = 0
    frames, pics, size, errors = [], [], 0, 0

    def drain(flush):
        while L.H264SwDecNextPicture(inst, C.byref(pic), flush) == _lib.H264SWDEC_PIC_RDY:
            frames.append(C.string_at(C.cast(pic.pOutputPicture, C.c_void_p), size))
            pics.append((pic.picId, pic.isIdrPicture, pic.nbrOfErrMBs))

    def advance():
        consumed = C.cast(out.pStrmCurrPos, C.c_void_p).value - C.cast(inp.pStream, C.c_void_p).value
        inp.dataLen -= consumed
        inp.pStream = C.cast(C.c_void_p(C.cast(inp.pStream, C.c_void_p).value + consumed), C.POINTER(C.c_uint8))

    pic_id = 1
    while inp.dataLen > 0:
        inp.picId = pic_id
        ret = L.H264SwDecDecode(inst, C.byref(inp), C.byref(out))
        if ret == _lib.H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY:
            assert L.H264SwDecGetInfo(inst, C.byref(dinfo)) == _lib.H264SWDEC_OK
            size = dinfo.picWidth * dinfo.picHeight * 3 // 2
            advance()
        elif ret in (_lib.H264SWDEC_PIC_RDY, _lib.H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY):
            if ret == _lib.H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY:
                advance()
            else:
                inp.dataLen = 0
            pic_id += 1
            drain(0)
        elif ret in (_lib.H264SWDEC_STRM_PROCESSED, _lib.H264SWDEC_STRM_ERR):
            errors += ret == _lib.H264SWDEC_STRM_ERR
            inp.dataLen = 0
        else:
            errors += 1
            break
    drain(1)
    L.H264SwDecRelease(inst)
    return (frames, errors, pics) if info else (frames, errors)


def _nal_starts(b: bytes):
    i, out = 0, []
    while True:
        i = b.find(b"\0\0\1", i)
        if i < 0:
            break
        out.append(i - 1 if i > 0 and b[i - 1] == 0 else i)
        i += 3
    return out


def softavc_decode(stream: bytes, method: int = 1):
    """The SoftAVC OMX component's protocol over the product H264SwDec* C-ABI
    (Decoder/SoftAVC.cpp:289-400): one NAL unit (start code included) per
    input buffer, picId incremented per buffer, intraConcealmentMethod =
    `method` (SoftAVC.cpp:335 sets 1), the buffer re-fed while the decoder
    returns *_BUFF_NOT_EMPTY, NextPicture(…, 0) drained after every buffer
    once headers are decoded, NextPicture(…, 1) at end of stream.  Returns
    (frames, [(picId, isIdrPicture, nbrOfErrMBs)])."""
    L = _lib.mi()
    inst = C.c_void_p()
    assert L.H264SwDecInit(C.byref(inst), 0) == _lib.H264SWDEC_OK
    buf = (C.c_uint8 * len(stream)).from_buffer_copy(stream)
    base = C.addressof(buf)
    inp, out = _lib.H264SwDecInput(), _lib.H264SwDecOutput()
    pic, dinfo = _lib.H264SwDecPicture(), _lib.H264SwDecInfo()
    frames, pics = [], []
    size = 0
    starts = _nal_starts(stream) + [len(stream)]

    def drain(flush):
        while L.H264SwDecNextPicture(inst, C.byref(pic), flush) == _lib.H264SWDEC_PIC_RDY:
            frames.append(C.string_at(C.cast(pic.pOutputPicture, C.c_void_p), size))
            pics.append((pic.picId, pic.isIdrPicture, pic.nbrOfErrMBs))

    pic_id = 0
    for a, b in zip(starts, starts[1:]):
        pic_id += 1
        inp.pStream = C.cast(C.c_void_p(base + a), C.POINTER(C.c_uint8))
        inp.dataLen = b - a
        inp.picId = pic_id
        inp.intraConcealmentMethod = method
        while inp.dataLen > 0:
            ret = L.H264SwDecDecode(inst, C.byref(inp), C.byref(out))
            if ret in (_lib.H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY, _lib.H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY):
                cur = C.cast(out.pStrmCurrPos, C.c_void_p).value
                inp.dataLen -= cur - C.cast(inp.pStream, C.c_void_p).value
                inp.pStream = C.cast(C.c_void_p(cur), C.POINTER(C.c_uint8))
                if ret == _lib.H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY:
                    assert L.H264SwDecGetInfo(inst, C.byref(dinfo)) == _lib.H264SWDEC_OK
                    size = dinfo.picWidth * dinfo.picHeight * 3 // 2
            else:
                inp.dataLen = 0
        if size:
            drain(0)
    if size:
        drain(1)
    L.H264SwDecRelease(inst)
    return frames, pics
