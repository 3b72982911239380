"""bindings/node: the N-API addon behind Broadway's JS Decoder API."""
import json
import os
import shutil
import subprocess
import tempfile

import pytest

from _golden import cases, stream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ADDON = os.path.join(ROOT, "broadway_amd", "lib", "broadway.node")
NODE = shutil.which("node")
need_node = pytest.mark.skipif(not (NODE and os.path.exists(ADDON)), reason="node / addon not available")


@need_node
def test_addon_loads_and_reports_api_version():
    r = subprocess.run([NODE, "-e", "console.log(JSON.stringify(require(process.argv[1]).version))",
                        os.path.join(ROOT, "bindings", "node", "Decoder.js")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1]) == [2, 3]


@need_node
@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="checks the no-GPU failure mode")
def test_decoder_fails_loudly_without_gpu():
    """No CPU fallback: constructing a Decoder without a HIP device throws."""
    r = subprocess.run([NODE, "-e", "var D=require(process.argv[1]); new D({});",
                        os.path.join(ROOT, "bindings", "node", "Decoder.js")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "INITIALIZATION FAILED" in r.stderr


@need_node
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["small_ip_8x6_2sl", "cfg1_plumbing_640x368"])
def test_node_decoder_vs_reference(name):
    c = cases()[name]
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "s.h264")
        open(p, "wb").write(stream(c))
        r = subprocess.run([NODE, os.path.join(ROOT, "tests", "node", "decode_md5.js"), p],
                           capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert (out["width"], out["height"]) == (c["width"], c["height"])
    assert out["frames"] == c["frames"]
    assert out["infos"] == len(c["frames"]) or out["infos"] > 0


@need_node
@pytest.mark.gpu
def test_node_decoder_rgb_option():
    """new Decoder({rgb: true}): RGBA pictures, each the conversion of the
    reference's I420 picture (DecoderPost.js yuv2rgbcalc, oracle restatement)."""
    import hashlib
    import oracle as O
    c = cases()["small_ip_8x6_2sl"]
    s = stream(c)
    frames, _, w, h, _ = O.decode(s)
    assert [hashlib.md5(f).hexdigest() for f in frames] == c["frames"]
    want = [hashlib.md5(O.yuv2rgba(f, w, h)).hexdigest() for f in frames]
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "s.h264")
        open(p, "wb").write(s)
        r = subprocess.run([NODE, os.path.join(ROOT, "tests", "node", "decode_md5.js"), p, "rgb"],
                           capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert (out["width"], out["height"]) == (w, h)
    assert out["frames"] == want
