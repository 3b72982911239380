"""Access to the committed reference-decoder fixtures (tests/golden/golden.json)."""
import hashlib
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.json")


def cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


def stream(case):
    """Regenerate a fixture's stream and check it is byte-identical to the one
    the reference decoded when the fixture was made."""
    from broadway_amd import gen
    s = gen.generate(case["config"], case["seed"], **case["overrides"])
    assert hashlib.sha256(s).hexdigest() == case["stream_sha256"], "generator drift"
    if case.get("patch"):          # byte patches recorded with the fixture
        b = bytearray(s)
        for off, hexb in case["patch"]:
            v = bytes.fromhex(hexb)
            b[off:off + len(v)] = v
        s = bytes(b)
    return s


def md5s(frames):
    return [hashlib.md5(f).hexdigest() for f in frames]
