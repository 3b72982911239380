"""SoftAVC drop-in (Decoder/SoftAVC.cpp): its protocol -- one NAL unit per
H264SwDecDecode input buffer, picId per buffer -- and its
intraConcealmentMethod = 1 (SoftAVC.cpp:335), under which a picture whose
slices all fail is concealed by copying the first available reference
picture, I pictures included, instead of painting it grey
(h264bsd_conceal.c:149-159, 177-181).  Pinned by tests/golden/softavc.json:
the reference decoder driven the same way (oracle/softavc_bench.c,
tests/golden/make_golden_softavc.py), frame MD5s and (picId, isIdr,
nbrOfErrMBs) per output picture, for method 1 and for method 0 as the
control.  CPU: the oracle (product parser + CPU reconstruction) against the
fixtures; GPU: the product C-ABI (HIP reconstruction) against them."""
import hashlib
import json
import os

import pytest

import oracle as O
from _swdec import softavc_decode
from broadway_amd import gen

FIX = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "softavc.json")))["cases"]


def _stream(c):
    s = gen.generate(c["config"], c["seed"], **c["overrides"])
    assert hashlib.sha256(s).hexdigest() == c["stream_sha256"], "generator drift"
    return s


def _md5s(frames):
    return [hashlib.md5(f).hexdigest() for f in frames]


def test_fixtures_exercise_method_1():
    """At least three streams where method 1 changes the output (whole
    pictures lost, I pictures among them)."""
    sens = [n for n, c in FIX.items() if c["method_sensitive"]]
    assert len(sens) >= 3
    nmbs = lambda c: (c["overrides"].get("w_mbs", 80) * c["overrides"].get("h_mbs", 45))  # noqa: E731
    assert any(p[1] == 1 and p[2] == nmbs(FIX[n]) for n in sens for p in FIX[n]["method1"]["pics"])


@pytest.mark.parametrize("method", [1, 0])
@pytest.mark.parametrize("name", sorted(FIX))
def test_oracle_softavc_vs_reference(name, method):
    c = FIX[name]
    frames, _, _, _, _, pics = O.decode(_stream(c), info=True, softavc=method)
    assert _md5s(frames) == c[f"method{method}"]["frames"]
    assert [list(p) for p in pics] == c[f"method{method}"]["pics"]


@pytest.mark.gpu
@pytest.mark.parametrize("method", [1, 0])
@pytest.mark.parametrize("name", sorted(FIX))
def test_swdec_softavc_protocol_vs_reference(name, method):
    """Through H264SwDec* on the GPU with SoftAVC's call pattern."""
    c = FIX[name]
    frames, pics = softavc_decode(_stream(c), method)
    assert _md5s(frames) == c[f"method{method}"]["frames"]
    assert [list(p) for p in pics] == c[f"method{method}"]["pics"]
