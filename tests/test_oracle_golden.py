"""CPU oracle (oracle/recon_cpu.c + the product host parser) against the
reference decoder's per-frame MD5s (tests/golden/golden.json).  This pins
the oracle that the GPU parity tests then trust."""
import pytest

import oracle as O
from _golden import cases, md5s, stream

CASES = cases()
FAST = [n for n in CASES if not n.startswith(("bench_", "leg_"))] + ["bench_1080p_s100", "bench_1080p_s105",
                                                                     "leg_cfg2_720p_s1", "bench_1080p_offpic0_s100"]


@pytest.mark.parametrize("name", FAST)
def test_oracle_matches_reference(name):
    c = CASES[name]
    frames, errs, w, h, _, pics = O.decode(stream(c), no_reorder=c["no_reorder"], info=True)
    assert (w, h) == (c["width"], c["height"])
    assert md5s(frames) == c["frames"]
    if "pics" in c:
        # damaged stream: same pictures, ids, IDR flags and concealed-MB
        # counts (nbrOfErrMBs) as the reference decoder printed
        assert [list(p) for p in pics] == c["pics"]
    else:
        assert errs == 0


def test_error_fixtures_exercise_concealment():
    """The damaged-stream fixtures cover P-copy and neighbour (intra)
    concealment, whole lost pictures and the I-slice un-marking quirk."""
    err = {n: c for n, c in CASES.items() if "pics" in c}
    assert len(err) >= 8
    assert any(p[2] == c["width"] * c["height"] // 256 for c in err.values() for p in c["pics"])
    assert sum(sum(p[2] for p in c["pics"]) > 0 for c in err.values()) >= 8


def test_fixture_inventory():
    # every SURVEY §8d config is pinned, and the bench streams cover 60 frames
    names = set(CASES)
    assert {"cfg1_plumbing_640x368", "cfg2_720p_ionly_s1", "cfg5_2160p_s200"} <= names
    assert all(len(CASES[f"bench_1080p_s{s}"]["frames"]) == 60 for s in range(100, 108))
    # the loop-filter-off encode of the same streams (bench leg cfg3_no_loop_filter)
    assert all(len(CASES[f"bench_1080p_noloop_s{s}"]["frames"]) == 60 and
               CASES[f"bench_1080p_noloop_s{s}"]["overrides"].get("dbf_idc1_pct") == 100 for s in range(100, 108))
