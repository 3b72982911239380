"""Host-side logic that needs no GPU: CAVLC tables, the MB-record capture of
the product parser, picture slots / output order, Annex-B splitting."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from _golden import cases, md5s, stream
from broadway_amd import gen
from broadway_amd.decoder import split_annexb
from broadway_amd.engine import MBREC_BYTES, Capture

CASES = cases()

REC_DT = np.dtype([("type", "u1"), ("qp", "u1"), ("qpc", "u1"), ("avail", "u1"), ("pred", "u1"),
                   ("dbf", "u1"), ("offA", "i1"), ("offB", "i1"), ("cbits", "<u4"), ("coef", "<u4"),
                   ("i4", "u1", 8), ("ref", "u1", 4), ("mv", "<i2", 32), ("slice", "<u2"), ("rsv", "<u2")])


def test_record_layout():
    assert REC_DT.itemsize == MBREC_BYTES == 96


def test_cavlc_roundtrip():
    # encode/decode random residual blocks through tables 9-5/9-7/9-8/9-9a/9-10
    assert gen.cavlc_selftest(20000, 7) == 0


@pytest.mark.parametrize("name", ["small_ip_8x6_2sl", "small_ip_13x7_qpoff", "cfg2_720p_ionly_s1"])
def test_capture_replay_matches_reference(name):
    """Record batches captured by the product parser, reconstructed by the CPU
    oracle slot by slot, reproduce the reference decoder's frames (decode
    order == output order for POC type 2)."""
    c = CASES[name]
    cap = Capture(stream(c))
    assert cap.errors == 0 and cap.npics == len(c["frames"])
    rep = O.Replay(cap.w_mbs, cap.h_mbs, cap.nslots)
    got = []
    for p in cap.pictures:
        assert 0 <= p.cur_slot < cap.nslots
        assert rep.picture(p.rec, p.coef, p.cur_slot) == 0
        got.append(rep.frame(p.cur_slot))
    assert md5s(got) == c["frames"]


def test_capture_records_sane():
    c = CASES["small_ip_11x9_cip"]
    cap = Capture(stream(c))
    for i, p in enumerate(cap.pictures):
        r = np.frombuffer(cap.records_bytes(i), dtype=REC_DT)
        assert r.shape[0] == cap.w_mbs * cap.h_mbs
        assert np.all(r["type"] <= 4)
        assert np.all(r["qp"] <= 51) and np.all(r["qpc"] <= 51)
        # coefficient blocks referenced by records stay inside the batch
        coded = r["cbits"] != 0
        if coded.any():
            assert int(r["coef"][coded].max()) < max(p.ncoef, 1)
        # neighbour availability never points outside the picture
        col = np.arange(r.shape[0]) % cap.w_mbs
        row = np.arange(r.shape[0]) // cap.w_mbs
        assert not np.any((r["avail"] & 1) & (col == 0))
        assert not np.any((r["avail"] & 2) & (row == 0))
        assert p.n_inter + p.n_intra == r.shape[0]


def test_split_annexb_roundtrip():
    s = stream(CASES["small_plumb_9x5"])
    nals = split_annexb(s)
    assert len(nals) >= 2 + 6                      # SPS, PPS, one slice per frame at least
    # each unit keeps its start code (one NAL per decode() call, as mp4.js feeds it)
    assert all(n.startswith(b"\0\0\0\1") or n.startswith(b"\0\0\1") for n in nals)
    types = [n[n.index(b"\1") + 1] & 31 for n in nals]
    assert types[0] == 7 and types[1] == 8 and 5 in types
    assert b"".join(nals) == s


def test_oracle_no_reorder_changes_order_only():
    a = CASES["poc0_reorder"]["frames"]
    b = CASES["poc0_noreorder"]["frames"]
    assert sorted(a) == sorted(b) and a != b
