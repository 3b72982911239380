"""The C-ABI library loads and exports every function include/*.h declares
(no compute calls: this runs without a GPU)."""
import ctypes as C
import os
import re

from broadway_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if not fn.endswith(".h"):
            continue
        src = open(os.path.join(ROOT, "include", fn)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        src = re.sub(r"#[^\n]*", "", src)
        for m in re.finditer(r"\b([A-Za-z_]\w*)\s*\(([^;{}()]*)\)\s*;", src):
            name = m.group(1)
            if name in ("if", "while", "for", "return", "sizeof"):
                continue
            # skip function-pointer typedef members: "(*name)(...)"
            names.add(name)
    return names


def test_header_declares_the_reference_api():
    names = declared_functions()
    for n in ("H264SwDecInit", "H264SwDecDecode", "H264SwDecNextPicture", "H264SwDecGetInfo",
              "H264SwDecRelease", "H264SwDecGetAPIVersion", "broadwayInit", "broadwayCreateStream",
              "broadwayPlayStream", "broadwayExit", "broadwayGetMajorVersion", "broadwayGetMinorVersion"):
        assert n in names, n


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(os.path.join(_lib.LIB_DIR, "libh264mi.so"))
    missing = [n for n in sorted(declared_functions()) if not hasattr(lib, n)]
    assert not missing, missing


def test_api_version_without_device():
    L = _lib.mi()
    v = L.H264SwDecGetAPIVersion()
    assert (v.major, v.minor) == (2, 3)          # H264SwDecApi.c:52-53


def test_init_rejects_null_instance():
    L = _lib.mi()
    assert L.H264SwDecInit(None, 0) == _lib.H264SWDEC_PARAM_ERR
