"""ctypes bindings to the in-tree native libraries.

libh264mi.so  -- product: host parser + HIP reconstruction engine + C-ABI
                 (include/h264mi.h).  No CPU reconstruction exists in it.
libh264gen.so -- seeded synthetic Baseline stream generator (test/bench input).

The libraries are built by ``__graft_entry__.build()`` (or ``make -C
broadway_amd/csrc``) into ``broadway_amd/lib``.  Loading fails loudly when a
library is missing: there is no fallback path.
"""
from __future__ import annotations

import ctypes as C
import os

# H264MI_LIB_DIR: load another build of the same libraries (A/B timing of
# kernel variants in one process tree; tools/ab.sh)
LIB_DIR = os.environ.get("H264MI_LIB_DIR") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")


class NativeLibraryMissing(RuntimeError):
    pass


def _load(name: str) -> C.CDLL:
    path = os.path.join(LIB_DIR, name)
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f"{path} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
    return C.CDLL(path, mode=C.RTLD_GLOBAL)


_mi = None
_gen = None


# ---------------------------------------------------------------- structs ---
class H264SwDecInput(C.Structure):
    _fields_ = [("pStream", C.POINTER(C.c_uint8)), ("dataLen", C.c_uint32),
                ("picId", C.c_uint32), ("intraConcealmentMethod", C.c_uint32)]


class H264SwDecOutput(C.Structure):
    _fields_ = [("pStrmCurrPos", C.POINTER(C.c_uint8))]


class H264SwDecPicture(C.Structure):
    _fields_ = [("pOutputPicture", C.POINTER(C.c_uint32)), ("picId", C.c_uint32),
                ("isIdrPicture", C.c_uint32), ("nbrOfErrMBs", C.c_uint32)]


class CropParams(C.Structure):
    _fields_ = [("cropLeftOffset", C.c_uint32), ("cropOutWidth", C.c_uint32),
                ("cropTopOffset", C.c_uint32), ("cropOutHeight", C.c_uint32)]


class H264SwDecInfo(C.Structure):
    _fields_ = [("profile", C.c_uint32), ("picWidth", C.c_uint32), ("picHeight", C.c_uint32),
                ("videoRange", C.c_uint32), ("matrixCoefficients", C.c_uint32),
                ("parWidth", C.c_uint32), ("parHeight", C.c_uint32),
                ("croppingFlag", C.c_uint32), ("cropParams", CropParams)]


class H264SwDecApiVersion(C.Structure):
    _fields_ = [("major", C.c_uint32), ("minor", C.c_uint32)]


class GenParams(C.Structure):
    _fields_ = [(n, C.c_int) for n in (
        "w_mbs", "h_mbs", "crop_right", "crop_bottom", "nframes", "gop", "slices",
        "pm_skip", "pm_16x16", "pm_16x8", "pm_8x16", "pm_8x8", "pm_intra", "p8x8_ref0_pct",
        "im_i4", "im_i16", "im_pcm", "i4_rem_pct", "qp_min", "qp_max", "qp_delta",
        "dbf_idc1_pct", "dbf_idc2_pct", "dbf_off", "num_ref_frames", "cip", "chroma_qp_offset",
        "poc_type", "coef_pct", "level_tail_pct", "mv_jitter", "offpic_pct",
        "log2_max_frame_num", "poc_swap",
        "err_range_pct", "drop_slice_pct", "trunc_slice_pct", "drop_pic_pct", "gaps_allowed",
        "nonref_pct", "ref_mod_pct", "mmco_pct", "lt_idr_pct")] + [("seed", C.c_uint64)]


HEADERS_CB = C.CFUNCTYPE(None, C.c_void_p)
PICTURE_CB = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_uint8), C.c_uint32, C.c_uint32)

H264SWDEC_OK = 0
H264SWDEC_STRM_PROCESSED = 1
H264SWDEC_PIC_RDY = 2
H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY = 3
H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY = 4
H264SWDEC_PARAM_ERR = -1
H264SWDEC_STRM_ERR = -2
H264SWDEC_NOT_INITIALIZED = -3
H264SWDEC_MEMFAIL = -4
H264SWDEC_INITFAIL = -5
H264SWDEC_HDRS_NOT_RDY = -6


def mi() -> C.CDLL:
    """libh264mi.so with prototypes set.

    PyTorch-ROCm ships its own libamdhip64.so (same SONAME libamdhip64.so.7 as
    /opt/rocm's).  If torch is importable it is imported first so that
    libh264mi.so binds to that already-loaded runtime and the process holds a
    single HIP runtime (torch.cuda.synchronize() then sees our stream work)."""
    global _mi
    if _mi is not None:
        return _mi
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = _load("libh264mi.so")
    vp, i32, u32, sz = C.c_void_p, C.c_int, C.c_uint32, C.c_size_t
    L.H264SwDecInit.argtypes = [C.POINTER(vp), u32]
    L.H264SwDecInit.restype = i32
    L.H264SwDecDecode.argtypes = [vp, C.POINTER(H264SwDecInput), C.POINTER(H264SwDecOutput)]
    L.H264SwDecDecode.restype = i32
    L.H264SwDecNextPicture.argtypes = [vp, C.POINTER(H264SwDecPicture), u32]
    L.H264SwDecNextPicture.restype = i32
    L.H264SwDecGetInfo.argtypes = [vp, C.POINTER(H264SwDecInfo)]
    L.H264SwDecGetInfo.restype = i32
    L.H264SwDecRelease.argtypes = [vp]
    L.H264SwDecRelease.restype = None
    L.H264SwDecGetAPIVersion.argtypes = []
    L.H264SwDecGetAPIVersion.restype = H264SwDecApiVersion
    L.broadwaySetCallbacks.argtypes = [HEADERS_CB, PICTURE_CB, vp]
    L.broadwaySetCallbacks.restype = None
    L.broadwayInit.restype = u32
    L.broadwayCreateStream.argtypes = [u32]
    L.broadwayCreateStream.restype = C.POINTER(C.c_uint8)
    L.broadwayPlayStream.argtypes = [u32]
    L.broadwayPlayStream.restype = None
    L.broadwayExit.restype = None
    L.broadwayGetMajorVersion.restype = u32
    L.broadwayGetMinorVersion.restype = u32
    L.h264mi_engine_create.argtypes = [i32, i32, i32, i32, i32]
    L.h264mi_engine_create.restype = vp
    L.h264mi_engine_destroy.argtypes = [vp]
    L.h264mi_engine_destroy.restype = None
    L.h264mi_engine_decode.argtypes = [vp, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(vp),
                                       C.POINTER(vp), C.POINTER(u32)]
    L.h264mi_engine_decode.restype = i32
    L.h264mi_engine_decode_device.argtypes = [vp, i32, vp, vp, vp]
    L.h264mi_engine_decode_device.restype = i32
    L.h264mi_engine_hint_intra.argtypes = [vp, i32]
    L.h264mi_engine_hint_intra.restype = i32
    if hasattr(L, "h264mi_engine_hint_deps"):
        L.h264mi_engine_hint_deps.argtypes = [vp, i32]
        L.h264mi_engine_hint_deps.restype = i32
        L.h264mi_engine_last_deps.argtypes = [vp]
        L.h264mi_engine_last_deps.restype = i32
    if hasattr(L, "h264mi_engine_last_mc_waves"):
        L.h264mi_engine_last_mc_waves.argtypes = [vp]
        L.h264mi_engine_last_mc_waves.restype = i32
    L.h264mi_engine_decode_device_next.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp]
    L.h264mi_engine_decode_device_next.restype = i32
    L.h264mi_engine_decode_device_steps.argtypes = [vp, i32, i32, vp, vp, vp, vp, vp, vp]
    L.h264mi_engine_decode_device_steps.restype = i32
    if hasattr(L, "h264mi_engine_decode_device_steps_next"):
        L.h264mi_engine_decode_device_steps_next.argtypes = [vp, i32, i32, vp, vp, vp, vp, vp, vp, i32]
        L.h264mi_engine_decode_device_steps_next.restype = i32
    L.h264mi_engine_set_steps.argtypes = [vp, i32]
    L.h264mi_engine_set_steps.restype = i32
    L.h264mi_set_share.argtypes = [i32]
    L.h264mi_set_share.restype = i32
    L.h264mi_share_stats.argtypes = [i32, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]
    L.h264mi_share_stats.restype = i32
    L.h264mi_engine_pool_stats.argtypes = [C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]
    L.h264mi_engine_pool_stats.restype = None
    L.h264mi_engine_read.argtypes = [vp, i32, i32, vp]
    L.h264mi_engine_read.restype = i32
    L.h264mi_engine_read_rgba.argtypes = [vp, i32, i32, vp]
    L.h264mi_engine_read_rgba.restype = i32
    L.h264mi_yuv2rgba_device.argtypes = [vp, vp, i32, i32, i32, C.c_size_t, C.c_size_t, vp]
    L.h264mi_yuv2rgba_device.restype = i32
    if hasattr(L, "h264mi_yuv2rgba_device_pitch"):      # (absent from A/B builds of older trees)
        L.h264mi_yuv2rgba_device_pitch.argtypes = [vp, vp, i32, i32, i32, i32, C.c_size_t, C.c_size_t, vp]
        L.h264mi_yuv2rgba_device_pitch.restype = i32
    L.H264SwDecNextPictureRGBA.argtypes = [vp, C.POINTER(H264SwDecPicture), u32, vp]
    L.H264SwDecNextPictureRGBA.restype = i32
    L.h264mi_engine_sync.argtypes = [vp]
    L.h264mi_engine_sync.restype = i32
    L.h264mi_engine_kernel.argtypes = [vp]
    L.h264mi_engine_kernel.restype = C.c_char_p
    L.h264mi_engine_errors.argtypes = [vp]
    L.h264mi_engine_errors.restype = u32
    L.h264mi_engine_rows_per_workgroup.argtypes = [vp, C.c_int]
    L.h264mi_engine_rows_per_workgroup.restype = C.c_int
    L.h264mi_engine_last_timing.argtypes = [vp, C.POINTER(C.c_float)]
    L.h264mi_engine_last_timing.restype = i32
    L.h264mi_engine_set_timing.argtypes = [vp, i32]
    L.h264mi_engine_set_timing.restype = i32
    L.h264mi_engine_set_timing_stride.argtypes = [vp, i32]
    L.h264mi_engine_set_timing_stride.restype = i32
    L.h264mi_engine_timing_report.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(i32)]
    L.h264mi_engine_timing_report.restype = i32
    # (round-4 additions; absent from older builds loaded for A/B timing)
    if hasattr(L, "h264mi_engine_error_bits"):
        L.h264mi_engine_error_bits.argtypes = [vp]
        L.h264mi_engine_error_bits.restype = C.c_uint32
    if hasattr(L, "h264mi_engine_timing_list"):
        L.h264mi_engine_timing_list.argtypes = [vp, C.POINTER(C.c_double), i32]
        L.h264mi_engine_timing_list.restype = i32
    L.h264mi_engine_profile.argtypes = [vp, i32, C.POINTER(C.c_uint64), sz]
    L.h264mi_engine_profile.restype = i32
    L.h264mi_engine_frame_ptr.argtypes = [vp, i32, i32]
    L.h264mi_engine_frame_ptr.restype = vp
    L.h264mi_engine_frame_bytes.argtypes = [vp]
    L.h264mi_engine_frame_bytes.restype = sz
    if hasattr(L, "h264mi_engine_slot_bytes"):
        L.h264mi_engine_slot_bytes.argtypes = [vp]
        L.h264mi_engine_slot_bytes.restype = sz
        L.h264mi_engine_chroma_pitch.argtypes = [vp]
        L.h264mi_engine_chroma_pitch.restype = i32
    L.h264mi_capture_stream.argtypes = [vp, sz, i32]
    L.h264mi_capture_stream.restype = vp
    L.h264mi_capture_info.argtypes = [vp] + [C.POINTER(i32)] * 5
    L.h264mi_capture_info.restype = i32
    L.h264mi_capture_picture.argtypes = [vp, i32, C.POINTER(vp), C.POINTER(vp), C.POINTER(u32),
                                         C.POINTER(i32), C.POINTER(C.c_uint64)]
    L.h264mi_capture_picture.restype = i32
    L.h264mi_capture_stats.argtypes = [vp, i32, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)]
    L.h264mi_capture_stats.restype = i32
    L.h264mi_capture_ref_lines.argtypes = [vp, i32, C.POINTER(C.c_uint64)]
    L.h264mi_capture_ref_lines.restype = i32
    L.h264mi_capture_free.argtypes = [vp]
    L.h264mi_capture_free.restype = None
    L.h264mi_device_alloc.argtypes = [sz]
    L.h264mi_device_alloc.restype = vp
    L.h264mi_device_free.argtypes = [vp]
    L.h264mi_device_free.restype = i32
    L.h264mi_copy_h2d.argtypes = [vp, vp, sz]
    L.h264mi_copy_h2d.restype = i32
    L.h264mi_engine_device.argtypes = [vp]
    L.h264mi_engine_device.restype = i32
    L.h264mi_engine_alloc.argtypes = [vp, sz]
    L.h264mi_engine_alloc.restype = vp
    L.h264mi_engine_free.argtypes = [vp, vp]
    L.h264mi_engine_free.restype = i32
    L.h264mi_engine_copy_h2d.argtypes = [vp, vp, vp, sz]
    L.h264mi_engine_copy_h2d.restype = i32
    L.h264mi_pointer_device.argtypes = [vp]
    L.h264mi_pointer_device.restype = i32
    _mi = L
    return L


def gen() -> C.CDLL:
    global _gen
    if _gen is not None:
        return _gen
    L = _load("libh264gen.so")
    L.h264gen_default_params.argtypes = [C.POINTER(GenParams), C.c_int, C.c_int]
    L.h264gen_default_params.restype = None
    L.h264gen_preset.argtypes = [C.POINTER(GenParams), C.c_int, C.c_uint64]
    L.h264gen_preset.restype = C.c_int
    L.h264gen_generate.argtypes = [C.POINTER(GenParams), C.POINTER(C.POINTER(C.c_uint8)),
                                   C.POINTER(C.c_size_t)]
    L.h264gen_generate.restype = C.c_int
    L.h264gen_free.argtypes = [C.c_void_p]
    L.h264gen_free.restype = None
    L.h264gen_cavlc_selftest.argtypes = [C.c_int, C.c_uint64]
    L.h264gen_cavlc_selftest.restype = C.c_int
    _gen = L
    return L
