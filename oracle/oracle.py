"""ORACLE -- TEST INFRASTRUCTURE ONLY (checker / CPU baseline, never product).

Python binding of oracle/_build/liboracle.so: the plain-C restatement of the
reference reconstruction (oracle/recon_cpu.c) driven by the product host
parser, plus the reference decoder binary oracle/_ref/refdec (built here from
/root/reference by oracle/Makefile.ref, used to make golden fixtures).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import subprocess
import tempfile
from typing import List, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
REFDEC = os.path.join(HERE, "_ref", "refdec")
REFDEC_SOFTAVC = os.path.join(HERE, "_ref", "refdec_softavc")

_L = None


def make(*targets: str) -> None:
    """make in oracle/ under a file lock: concurrent test processes (pytest
    -n) must not rebuild the same outputs at once.  Brings liboracle.so up to
    date with the product host sources it is built from."""
    import fcntl
    os.makedirs(os.path.join(HERE, "_build"), exist_ok=True)
    with open(os.path.join(HERE, "_build", ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.check_call(["make", "-s", "-C", HERE] + list(targets))


def lib() -> C.CDLL:
    global _L
    if _L is None:
        if os.path.isdir(os.path.join(HERE, "..", "broadway_amd", "csrc")):
            make()
        L = C.CDLL(LIB)
        L.oracle_decode_stream.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.POINTER(C.c_double)]
        L.oracle_decode_stream.restype = C.c_void_p
        L.oracle_decode_stream_nals.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.POINTER(C.c_double)]
        L.oracle_decode_stream_nals.restype = C.c_void_p
        L.oracle_result_info.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                         C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_size_t)]
        L.oracle_result_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.oracle_result_free.argtypes = [C.c_void_p]
        L.oracle_result_pics.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.oracle_result_pics.restype = C.c_int
        L.oracle_replay_create.argtypes = [C.c_int, C.c_int, C.c_int]
        L.oracle_replay_create.restype = C.c_void_p
        L.oracle_replay_picture.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
        L.oracle_replay_picture.restype = C.c_int
        L.oracle_replay_frame.argtypes = [C.c_void_p, C.c_int]
        L.oracle_replay_frame.restype = C.c_void_p
        L.oracle_replay_free.argtypes = [C.c_void_p]
        L.oracle_yuv2rgba.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        L.oracle_yuv2rgba.restype = None
        _L = L
    return _L


def decode(stream: bytes, no_reorder: bool = False, info: bool = False, softavc: int = -1):
    """Decode a whole Annex-B stream on the CPU (DecTestBench semantics incl.
    the end-of-stream flush; softavc >= 0: the SoftAVC protocol -- one NAL
    per input buffer, intraConcealmentMethod = softavc).  Returns (frames,
    errors, width, height, seconds) [+ per output picture (pic_id, is_idr,
    nbrOfErrMBs) if info]."""
    L = lib()
    buf = C.create_string_buffer(stream, len(stream))
    secs = C.c_double()
    if softavc >= 0:
        res = L.oracle_decode_stream_nals(C.cast(buf, C.c_void_p), len(stream), int(softavc), C.byref(secs))
    else:
        res = L.oracle_decode_stream(C.cast(buf, C.c_void_p), len(stream), int(no_reorder), C.byref(secs))
    n, e, w, h, nb = C.c_int(), C.c_int(), C.c_int(), C.c_int(), C.c_size_t()
    L.oracle_result_info(res, C.byref(n), C.byref(e), C.byref(w), C.byref(h), C.byref(nb))
    data = np.empty(nb.value, dtype=np.uint8)
    L.oracle_result_copy(res, data.ctypes.data, nb.value)
    pics = np.zeros(3 * max(n.value, 1), dtype=np.int32)
    L.oracle_result_pics(res, pics.ctypes.data, int(pics.size))
    L.oracle_result_free(res)
    fb = w.value * h.value * 3 // 2
    frames = [data[i * fb:(i + 1) * fb].tobytes() for i in range(n.value)] if fb else []
    if info:
        return frames, e.value, w.value, h.value, secs.value, [tuple(int(x) for x in pics[3 * i:3 * i + 3])
                                                               for i in range(n.value)]
    return frames, e.value, w.value, h.value, secs.value


class Replay:
    """CPU reconstruction of captured MB-record pictures into frame slots."""

    def __init__(self, w_mbs: int, h_mbs: int, nslots: int):
        self.w, self.h, self.nslots = w_mbs, h_mbs, nslots
        self._c = lib().oracle_replay_create(w_mbs, h_mbs, nslots)

    def picture(self, rec_addr: int, coef_addr: int, cur_slot: int) -> int:
        return lib().oracle_replay_picture(self._c, rec_addr, coef_addr, self.w, self.h, cur_slot)

    def frame(self, slot: int) -> bytes:
        p = lib().oracle_replay_frame(self._c, slot)
        return C.string_at(p, self.w * self.h * 384)

    def __del__(self):
        try:
            lib().oracle_replay_free(self._c)
        except Exception:
            pass


def md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


def refdec_frames(stream: bytes, no_reorder: bool = False, info: bool = False):
    """Decode with the reference C decoder (only in the build container).
    info=True: also return one (pic_id, is_idr, concealed MBs) per output
    picture, parsed from DecTestBench's "PIC n, type T[, decoded pic k]
    [, concealed c]" lines (DecTestBench.c:313-323, 377-385)."""
    if not os.path.exists(REFDEC):
        raise FileNotFoundError(REFDEC)
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "in.h264")
        yuv = os.path.join(td, "out.yuv")
        with open(src, "wb") as f:
            f.write(stream)
        args = [REFDEC, "-O" + yuv] + (["-R"] if no_reorder else []) + [src]
        out = subprocess.run(args, capture_output=True, text=True)
        w = h = None
        pics = []
        for line in out.stdout.splitlines():
            if line.startswith("Width"):
                parts = line.split()
                w, h = int(parts[1]), int(parts[3])
            elif line.startswith("PIC "):
                f = [x.strip() for x in line.split(",")]
                n = int(f[0].split()[1])
                pid, conc = n, 0
                for x in f[2:]:
                    if x.startswith("decoded pic"):
                        pid = int(x.split()[2])
                    elif x.startswith("concealed"):
                        conc = int(x.split()[1])
                pics.append((pid, int(f[1] == "type IDR"), conc))
        data = open(yuv, "rb").read() if os.path.exists(yuv) else b""
    fb = w * h * 3 // 2 if w else 0
    frames = [data[i:i + fb] for i in range(0, len(data), fb)] if fb else []
    return (frames, pics) if info else frames


def refdec_softavc_frames(stream: bytes, method: int = 1):
    """The reference decoder driven like SoftAVC (oracle/softavc_bench.c,
    build container only): (frames, [(picId, isIdr, nbrOfErrMBs)])."""
    if not os.path.exists(REFDEC_SOFTAVC):
        raise FileNotFoundError(REFDEC_SOFTAVC)
    with tempfile.TemporaryDirectory() as td:
        src, yuv = os.path.join(td, "in.h264"), os.path.join(td, "out.yuv")
        with open(src, "wb") as f:
            f.write(stream)
        out = subprocess.run([REFDEC_SOFTAVC, f"-M{method}", src, yuv], capture_output=True, text=True, check=True)
        w = h = 0
        pics = []
        for line in out.stdout.splitlines():
            f = line.split()
            if f[0] == "SIZE":
                w, h = int(f[1]), int(f[2])
            elif f[0] == "PIC":
                pics.append((int(f[1]), int(f[2]), int(f[3])))
        data = open(yuv, "rb").read()
    fb = w * h * 3 // 2
    frames = [data[i:i + fb] for i in range(0, len(data), fb)] if fb else []
    return frames, pics


def yuv2rgba(i420, width: int, height: int) -> bytes:
    """Decoder.js `rgb: true` conversion of one MB-aligned I420 picture
    (oracle_yuv2rgba, restating DecoderPost.js:420-560): width*height*4 bytes RGBA."""
    src = np.ascontiguousarray(np.frombuffer(bytes(i420), dtype=np.uint8))
    assert src.size == width * height * 3 // 2
    out = np.empty(width * height * 4, dtype=np.uint8)
    lib().oracle_yuv2rgba(src.ctypes.data, width, height, out.ctypes.data)
    return out.tobytes()
