"""CPU oracle (oracle/recon_cpu.c + the product host parser) against the
reference decoder's per-frame MD5s (tests/golden/golden.json).  This pins
the oracle that the GPU parity tests then trust."""
import pytest

import oracle as O
from _golden import cases, md5s, stream

CASES = cases()
FAST = [n for n in CASES if not n.startswith("bench_")] + ["bench_1080p_s100", "bench_1080p_s105"]


@pytest.mark.parametrize("name", FAST)
def test_oracle_matches_reference(name):
    c = CASES[name]
    frames, errs, w, h, _ = O.decode(stream(c), no_reorder=c["no_reorder"])
    assert errs == 0
    assert (w, h) == (c["width"], c["height"])
    assert md5s(frames) == c["frames"]


def test_fixture_inventory():
    # every SURVEY §8d config is pinned, and the bench streams cover 60 frames
    names = set(CASES)
    assert {"cfg1_plumbing_640x368", "cfg2_720p_ionly_s1", "cfg5_2160p_s200"} <= names
    assert all(len(CASES[f"bench_1080p_s{s}"]["frames"]) == 60 for s in range(100, 108))
