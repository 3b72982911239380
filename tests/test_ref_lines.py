"""h264mi_capture_ref_lines (bench.py's roofline.ref_line_bytes_per_launch):
the distinct 128-B reference lines k_wgpp's MC windows touch, restated here
from the records with numpy -- mc_issue's window geometry (recon_kernels.hip):
luma 9 rows x 12 B per 4x4 block from (x0 & ~3) clamped to [0, W16 - 12],
chroma 3 rows x 8 B per 2x2 block and component from (x0 & ~3) clamped to
[0, CW - 8], rows clamped to the plane, chroma rows H264MI_CPITCH apart.  Host C only: runs without a GPU."""
import numpy as np
import pytest

from broadway_amd import engine, gen

REC = np.dtype([("type", "u1"), ("qp", "u1"), ("qpc", "u1"), ("avail", "u1"), ("pred", "u1"), ("dbf", "u1"),
                ("offA", "i1"), ("offB", "i1"), ("cbits", "<u4"), ("coef", "<u4"), ("i4", "u1", 8),
                ("ref", "u1", 4), ("mv", "<i2", (16, 2)), ("slice", "<u2"), ("refidx", "<u2")])
assert REC.itemsize == engine.MBREC_BYTES


def lines_numpy(rec, w, h):
    W16, H16 = w * 16, h * 16
    CW, CH = W16 // 2, H16 // 2
    CP = (CW + 127) & ~127                      # H264MI_CPITCH: chroma rows padded to 128 B
    seen = set()
    b = np.arange(16)
    bx = ((b >> 2) & 1) * 2 + (b & 1)
    by = ((b >> 3) & 1) * 2 + ((b >> 1) & 1)
    for i in range(w * h):
        r = rec[i]
        if r["type"] not in (0, 1):          # MBT_INTER, MBT_SKIP
            continue
        mbx, mby = i % w, i // w
        slot = r["ref"][b >> 2].astype(np.int64)
        mvx, mvy = r["mv"][:, 0].astype(np.int64), r["mv"][:, 1].astype(np.int64)
        ax = np.clip((mbx * 16 + bx * 4 + (mvx >> 2) - 2) & ~3, 0, W16 - 12)
        y0 = mby * 16 + by * 4 + (mvy >> 2) - 2
        for k in range(9):
            y = np.clip(y0 + k, 0, H16 - 1)
            for o in (0, 11):
                seen.update(zip(slot.tolist(), ((y * W16 + ax + o) // 128).tolist()))
        cax = np.clip((mbx * 8 + bx * 2 + (mvx >> 3)) & ~3, 0, CW - 8)
        cy0 = mby * 8 + by * 2 + (mvy >> 3)
        for comp in range(2):
            for k in range(3):
                y = np.clip(cy0 + k, 0, CH - 1)
                base = W16 * H16 + comp * CP * CH
                for o in (0, 7):
                    seen.update(zip(slot.tolist(), ((base + y * CP + cax + o) // 128).tolist()))
    return 128 * len(seen)


@pytest.mark.parametrize("over", [dict(w_mbs=12, h_mbs=8, nframes=4),
                                  dict(w_mbs=9, h_mbs=5, nframes=4, offpic_pct=25, mv_jitter=64),
                                  dict(w_mbs=3, h_mbs=2, nframes=3, offpic_pct=50)])
def test_ref_lines_match_numpy_restatement(over):
    cap = engine.Capture(gen.generate(2, 7, **over))
    assert cap.errors == 0
    n_inter = 0
    for i, p in enumerate(cap.pictures):
        rec = np.frombuffer(cap.records_bytes(i), dtype=REC)
        assert p.ref_line_bytes == lines_numpy(rec, cap.w_mbs, cap.h_mbs), f"picture {i}"
        n_inter += p.n_inter
    assert n_inter > 0
    # an I picture reads no reference
    assert cap.pictures[0].ref_line_bytes == 0
