"""Drop-in boundary at link level: the reference's own C callers of the
H264SwDec API (Decoder/src/DecTestBench.c, TestBenchMultipleInstance.c)
compile UNCHANGED against include/ (H264SwDecApi.h -> h264mi.h) and link
against libh264mi.so, and an application's H264SwDecMalloc / H264SwDecFree
hooks (inc/H264SwDecApi.h:160-173) are the ones the library calls.

Build container only for the reference callers (their sources are read from
/root/reference, nothing is copied); the hook probe is the repo's own C."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
LIB = os.path.join(ROOT, "broadway_amd", "lib")
REF_SRC = "/root/reference/Decoder/src"


def _link(src, out):
    subprocess.check_call(["gcc", "-O1", "-Wall", "-I", INC, src, "-o", out, "-L", LIB, "-lh264mi",
                           f"-Wl,-rpath,{LIB}"])


def _dynsyms(exe):
    out = subprocess.check_output(["nm", "-D", "--defined-only", exe], text=True)
    return {l.split()[-1] for l in out.splitlines() if l.strip()}


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference sources absent (GPU box)")
@pytest.mark.parametrize("caller", ["DecTestBench.c", "TestBenchMultipleInstance.c"])
def test_reference_caller_compiles_and_links_unchanged(caller, tmp_path):
    exe = str(tmp_path / caller[:-2])
    _link(os.path.join(REF_SRC, caller), exe)
    # the caller's hook definitions are exported, so they interpose the library's defaults
    assert {"H264SwDecMalloc", "H264SwDecFree", "H264SwDecMemcpy", "H264SwDecMemset",
            "H264SwDecTrace"} <= _dynsyms(exe)
    undef = subprocess.check_output(["nm", "-D", "--undefined-only", exe], text=True)
    used = {l.split()[-1] for l in undef.splitlines() if "H264SwDec" in l}
    assert used <= {"H264SwDecInit", "H264SwDecDecode", "H264SwDecNextPicture", "H264SwDecGetInfo",
                    "H264SwDecRelease", "H264SwDecGetAPIVersion"}
    assert "H264SwDecDecode" in used


def test_application_hooks_allocate_the_instance(tmp_path):
    exe = str(tmp_path / "hooks_probe")
    _link(os.path.join(ROOT, "tests", "c", "hooks_probe.c"), exe)
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr
    n_malloc, n_free, ret = map(int, out.stdout.split())
    assert n_malloc == 1 and n_free == 1          # the instance, through the application's hooks
    assert ret in (0, -4)                         # OK with a GPU, MEMFAIL (no HIP device) without
