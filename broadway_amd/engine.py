"""Batched multi-stream reconstruction on one MI355X (the throughput path).

``Capture`` runs the product host parser over a whole stream and keeps each
picture's MB-record batch (include/h264mi_records.h).  ``Engine`` owns the
HBM frame slots of S streams and reconstructs one picture of each stream per
launch pair (k_prep: deblocking records + residuals; k_wgpp: MC, intra and the
deblocking row chain).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Sequence

import numpy as np

from . import _lib

MBREC_BYTES = 96
PICDESC_BYTES = 32


@dataclass
class CapturedPicture:
    rec: int            # host address of w*h MbRec
    coef: int           # host address of ncoef coefficient blocks
    ncoef: int
    cur_slot: int
    alg_ref_bytes: int
    n_inter: int
    n_intra: int
    n_coded: int
    ref_line_bytes: int = 0     # distinct 128-B reference lines the MC windows touch, x 128


class Capture:
    def __init__(self, stream: bytes, no_reorder: bool = False):
        self._L = _lib.mi()
        self._buf = C.create_string_buffer(stream, len(stream))
        self._h = self._L.h264mi_capture_stream(C.cast(self._buf, C.c_void_p), len(stream), int(no_reorder))
        if not self._h:
            raise RuntimeError("capture failed")
        w, h, ns, npics, err = (C.c_int() for _ in range(5))
        self._L.h264mi_capture_info(self._h, C.byref(w), C.byref(h), C.byref(ns), C.byref(npics), C.byref(err))
        self.w_mbs, self.h_mbs, self.nslots = w.value, h.value, ns.value
        self.npics, self.errors = npics.value, err.value
        self.pictures: List[CapturedPicture] = [self._picture(i) for i in range(self.npics)]

    def _picture(self, i: int) -> CapturedPicture:
        rec, coef = C.c_void_p(), C.c_void_p()
        nc, slot = C.c_uint32(), C.c_int()
        alg = C.c_uint64()
        self._L.h264mi_capture_picture(self._h, i, C.byref(rec), C.byref(coef), C.byref(nc), C.byref(slot),
                                       C.byref(alg))
        a, b, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
        self._L.h264mi_capture_stats(self._h, i, C.byref(a), C.byref(b), C.byref(c))
        lb = C.c_uint64()
        self._L.h264mi_capture_ref_lines(self._h, i, C.byref(lb))
        return CapturedPicture(rec.value or 0, coef.value or 0, nc.value, slot.value, alg.value,
                               a.value, b.value, c.value, lb.value)

    def records_bytes(self, i: int) -> bytes:
        p = self.pictures[i]
        return C.string_at(p.rec, self.w_mbs * self.h_mbs * MBREC_BYTES)

    def coef_bytes(self, i: int) -> bytes:
        p = self.pictures[i]
        return C.string_at(p.coef, p.ncoef * 32) if p.ncoef else b""

    def close(self):
        if self._h:
            self._L.h264mi_capture_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Engine:
    def __init__(self, w_mbs: int, h_mbs: int, nstreams: int, nslots: int, device: int = 0):
        self._L = _lib.mi()
        self.w_mbs, self.h_mbs, self.nstreams, self.nslots = w_mbs, h_mbs, nstreams, nslots
        self._h = self._L.h264mi_engine_create(device, w_mbs, h_mbs, nstreams, nslots)
        if not self._h:
            raise RuntimeError("h264mi_engine_create failed (no HIP device?)")
        self.frame_bytes = self._L.h264mi_engine_frame_bytes(self._h)       # packed I420 (read's output)
        if hasattr(self._L, "h264mi_engine_slot_bytes"):
            self.slot_bytes = self._L.h264mi_engine_slot_bytes(self._h)     # device slot stride
            self.chroma_pitch = self._L.h264mi_engine_chroma_pitch(self._h) # H264MI_CPITCH
        else:                                                               # an older tree's A/B build: packed slots
            self.slot_bytes, self.chroma_pitch = self.frame_bytes, w_mbs * 8

    def decode(self, streams: Sequence[int], pics: Sequence[CapturedPicture]) -> None:
        n = len(pics)
        st = (C.c_int * n)(*streams)
        sl = (C.c_int * n)(*[p.cur_slot for p in pics])
        recs = (C.c_void_p * n)(*[p.rec for p in pics])
        coefs = (C.c_void_p * n)(*[p.coef for p in pics])
        nc = (C.c_uint32 * n)(*[p.ncoef for p in pics])
        if self._L.h264mi_engine_decode(self._h, n, st, sl, recs, coefs, nc) != 0:
            raise RuntimeError("h264mi_engine_decode failed")

    def decode_device(self, npics: int, d_recs: int, d_coef: int, d_pics: int) -> None:
        if self._L.h264mi_engine_decode_device(self._h, npics, d_recs, d_coef, d_pics) != 0:
            raise RuntimeError("h264mi_engine_decode_device failed")

    def decode_device_next(self, npics: int, d_recs: int, d_coef: int, d_pics: int,
                           n_recs: int, n_coef: int, n_pics: int) -> None:
        """decode_device, naming the next batch: its k_prep runs in this
        launch's tail."""
        if self._L.h264mi_engine_decode_device_next(self._h, npics, d_recs, d_coef, d_pics,
                                                    n_recs, n_coef, n_pics) != 0:
            raise RuntimeError("h264mi_engine_decode_device_next failed")

    def hint_deps(self, mode: int) -> None:
        """Dependency mode of the next frame-pipelined launch: 1 whole MB
        rows, 2 (MB row, MB column) cells, 0 the engine's default."""
        if not hasattr(self._L, "h264mi_engine_hint_deps"):     # an older tree's A/B build
            return
        if self._L.h264mi_engine_hint_deps(self._h, int(mode)) != 0:
            raise RuntimeError("h264mi_engine_hint_deps failed")

    def last_deps(self) -> int:
        if not hasattr(self._L, "h264mi_engine_last_deps"):
            return -1
        return int(self._L.h264mi_engine_last_deps(self._h))

    def last_mc_waves(self) -> int:
        """MC waves per row workgroup of the last launch (-1: an older build)."""
        if not hasattr(self._L, "h264mi_engine_last_mc_waves"):
            return -1
        return int(self._L.h264mi_engine_last_mc_waves(self._h))

    def hint_intra(self, intra_heavy: bool) -> None:
        """Shape hint for the next device-resident launch: does some picture
        have more than half its MBs intra (include/h264mi.h)."""
        if self._L.h264mi_engine_hint_intra(self._h, int(bool(intra_heavy))) != 0:
            raise RuntimeError("h264mi_engine_hint_intra failed")

    def set_steps(self, steps: int) -> None:
        """Pictures per stream per launch for decode_device_steps (1..2)."""
        if self._L.h264mi_engine_set_steps(self._h, steps) != 0:
            raise RuntimeError("h264mi_engine_set_steps failed")

    def decode_device_steps(self, S: int, P: int, d_recs: int, d_coef: int, d_pics: int,
                            n_recs: int = 0, n_coef: int = 0, n_pics: int = 0) -> None:
        """P consecutive pictures of each of S streams in one launch
        (descriptors step-major, rec_base relative to d_recs); the next
        batch's k_prep in this launch's tail when n_recs is given."""
        if self._L.h264mi_engine_decode_device_steps(self._h, S, P, d_recs, d_coef, d_pics,
                                                     n_recs or None, n_coef or None, n_pics or None) != 0:
            raise RuntimeError("h264mi_engine_decode_device_steps failed")

    def decode_device_steps_next(self, S: int, P: int, d_recs: int, d_coef: int, d_pics: int,
                                 n_recs: int, n_coef: int, n_pics: int, next_P: int) -> bool:
        """decode_device_steps with the next batch's step count when it
        differs (its k_prep over S * next_P pictures in this launch's tail).
        False: the library predates it (nothing launched)."""
        if not hasattr(self._L, "h264mi_engine_decode_device_steps_next"):
            return False
        if self._L.h264mi_engine_decode_device_steps_next(self._h, S, P, d_recs, d_coef, d_pics,
                                                          n_recs, n_coef, n_pics, next_P) != 0:
            raise RuntimeError("h264mi_engine_decode_device_steps_next failed")
        return True

    def read(self, stream: int, slot: int) -> np.ndarray:
        out = np.empty(self.frame_bytes, dtype=np.uint8)
        if self._L.h264mi_engine_read(self._h, stream, slot, out.ctypes.data) != 0:
            raise RuntimeError("h264mi_engine_read failed")
        return out

    def read_rgba(self, stream: int, slot: int) -> np.ndarray:
        """The slot converted to RGBA on the GPU (Decoder.js `rgb: true`)."""
        out = np.empty(self.frame_bytes // 3 * 8, dtype=np.uint8)       # w*h*1.5 -> w*h*4
        if self._L.h264mi_engine_read_rgba(self._h, stream, slot, out.ctypes.data) != 0:
            raise RuntimeError("h264mi_engine_read_rgba failed")
        return out

    @property
    def device(self) -> int:
        return int(self._L.h264mi_engine_device(self._h))

    def alloc(self, nbytes: int) -> int:
        """Device memory on the engine's GPU (whatever the caller's current
        HIP device is)."""
        p = self._L.h264mi_engine_alloc(self._h, int(nbytes))
        if not p:
            raise RuntimeError(f"h264mi_engine_alloc({nbytes}) failed on device {self.device}")
        return int(p)

    def free(self, p: int) -> None:
        self._L.h264mi_engine_free(self._h, p)

    def upload(self, dst: int, src, nbytes: int) -> None:
        """H2D into memory of this engine's GPU (refused for another GPU's)."""
        if self._L.h264mi_engine_copy_h2d(self._h, dst, src, int(nbytes)) != 0:
            raise RuntimeError("h264mi_engine_copy_h2d failed (destination not on the engine's device?)")

    def pointer_device(self, p: int) -> int:
        return int(self._L.h264mi_pointer_device(p))

    def frame_ptr(self, stream: int, slot: int) -> int:
        """Device address of a frame slot (I420, chroma rows chroma_pitch
        bytes apart; slots slot_bytes apart)."""
        return int(self._L.h264mi_engine_frame_ptr(self._h, stream, slot))

    def sync(self) -> None:
        if self._L.h264mi_engine_sync(self._h) != 0:
            raise RuntimeError("h264mi_engine_sync failed")

    def kernel_name(self) -> str:
        """Reconstruction kernel of the last batch (diagnostics)."""
        return self._L.h264mi_engine_kernel(self._h).decode()

    def errors(self) -> int:
        return int(self._L.h264mi_engine_errors(self._h))

    def error_bits(self) -> int:
        """OR of the device flags of the pictures synced since the last call."""
        return int(self._L.h264mi_engine_error_bits(self._h))

    def rows_per_workgroup(self, npics: int) -> int:
        """MB rows per k_wgpp workgroup for a batch of npics pictures."""
        return int(self._L.h264mi_engine_rows_per_workgroup(self._h, npics))

    def last_timing_us(self):
        v = (C.c_float * 2)()
        if self._L.h264mi_engine_last_timing(self._h, v) != 0:
            return None
        return float(v[0]), float(v[1])

    def set_timing(self, max_batches: int, stride: int = 1) -> None:
        """HIP-event timing of up to max_batches launches, every stride-th one."""
        if self._L.h264mi_engine_set_timing(self._h, int(max_batches)) != 0:
            raise RuntimeError("h264mi_engine_set_timing failed")
        if self._L.h264mi_engine_set_timing_stride(self._h, int(stride)) != 0:
            raise RuntimeError("h264mi_engine_set_timing_stride failed")

    def timing_list(self, cap: int = 4096):
        """k_wgpp duration (us) of every recorded launch, in order."""
        if not hasattr(self._L, "h264mi_engine_timing_list"):
            return None
        v = (C.c_double * cap)()
        n = self._L.h264mi_engine_timing_list(self._h, v, int(cap))
        if n < 0:
            return None
        return [float(v[i]) for i in range(n)]

    def timing_report(self):
        a, b, n = C.c_double(), C.c_double(), C.c_int()
        if self._L.h264mi_engine_timing_report(self._h, C.byref(a), C.byref(b), C.byref(n)) != 0:
            return None
        return a.value, b.value, n.value

    def close(self):
        if self._h:
            self._L.h264mi_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
