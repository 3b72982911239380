#!/usr/bin/env python3
"""Generate tests/golden/golden.json: per-frame MD5s of the REFERENCE decoder.

Runs only in the build container, where oracle/_ref/refdec is built from the
reference C sources (oracle/Makefile.ref; SURVEY.md §8c: the reference ships
no test vectors, so parity is pinned by running it on identical input here).
Every stream comes from the in-tree seeded generator; the fixture records the
generator parameters, the stream's SHA-256 (so generator drift is detected)
and the MD5 of every output frame (full MB-aligned I420 buffer, the
DecTestBench -O output).  Nothing from the reference itself is stored.

    python tests/golden/make_golden.py          # rewrites golden.json
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# name -> (config, seed, overrides, no_reorder)
CASES = {
    # GPU parity cases (tests/test_gpu_parity.py SMALL)
    "small_i_6x5": (1, 1, dict(nframes=3, w_mbs=6, h_mbs=5), False),
    "small_ip_8x6_2sl": (2, 11, dict(nframes=8, w_mbs=8, h_mbs=6, crop_bottom=0, slices=2, gop=6), False),
    "small_ip_11x9_cip": (2, 21, dict(nframes=8, w_mbs=11, h_mbs=9, crop_bottom=0, slices=3, cip=1, gop=4), False),
    "small_ip_13x7_qpoff": (2, 33, dict(nframes=10, w_mbs=13, h_mbs=7, crop_bottom=0, slices=4, gop=5,
                                        chroma_qp_offset=-7, num_ref_frames=3, dbf_idc1_pct=10,
                                        dbf_idc2_pct=30, level_tail_pct=20), False),
    "small_plumb_9x5": (0, 3, dict(nframes=6, w_mbs=9, h_mbs=5, crop_bottom=0), False),
    # POC type 0 (output reordering through the DPB), with and without reordering
    "poc0_reorder": (2, 41, dict(nframes=12, w_mbs=10, h_mbs=6, crop_bottom=0, poc_type=0, gop=6,
                                 num_ref_frames=2, poc_swap=1), False),
    "poc0_noreorder": (2, 41, dict(nframes=12, w_mbs=10, h_mbs=6, crop_bottom=0, poc_type=0, gop=6,
                                   num_ref_frames=2, poc_swap=1), True),
    "poc0_inorder": (2, 42, dict(nframes=9, w_mbs=7, h_mbs=5, crop_bottom=0, poc_type=0, gop=4), False),
    # SURVEY §8d configs
    "cfg1_plumbing_640x368": (0, 1, dict(nframes=30), False),
    "cfg2_720p_ionly_s1": (1, 1, dict(nframes=4), False),
    "cfg2_720p_ionly_idc1_s2": (1, 2, dict(nframes=3, dbf_idc1_pct=100), False),
    "cfg5_2160p_s200": (4, 200, dict(nframes=4), False),
}
# Damaged streams (generator knobs err_range_pct / drop_* /
# trunc_slice_pct / gaps_allowed): residuals out of range, lost and truncated
# slices, lost pictures -> the reference's slice un-marking and concealment.
# Their fixtures also hold every output picture's (picId, isIdr, nbrOfErrMBs)
# as DecTestBench prints it.
_B = dict(nframes=12, w_mbs=11, h_mbs=9, crop_bottom=0, slices=3, gop=6)
ERR_CASES = {
    # I slices: includes an error on a slice's second MB, which the
    # reference's un-marking does not reach (slice_data.c:322-338)
    "err_range_i_9x6": (1, 2, dict(nframes=4, w_mbs=9, h_mbs=6, slices=4, err_range_pct=60), False),
    "err_range_p_11x9": (2, 6, dict(_B, err_range_pct=60), False),
    "err_drop_slice_11x9": (2, 7, dict(_B, drop_slice_pct=25), False),
    "err_trunc_slice_11x9": (2, 8, dict(_B, trunc_slice_pct=25), False),
    "err_drop_pic_gaps_11x9": (2, 10, dict(_B, drop_pic_pct=20, gaps_allowed=1), False),
    # POC type 0 reordering + truncation inside slice headers (the access-unit
    # boundary check fails part-way, storage.c:632-776)
    "err_mixed_poc0_9x2": (2, 5822, dict(nframes=12, w_mbs=9, h_mbs=2, slices=4, crop_bottom=0, gop=7,
                                         num_ref_frames=2, poc_type=0, dbf_idc2_pct=60, poc_swap=1,
                                         err_range_pct=10, trunc_slice_pct=30, drop_pic_pct=10), False),
    "err_720p_ionly_conceal": (1, 3, dict(nframes=3, drop_slice_pct=30, trunc_slice_pct=30), False),
    "err_1080p_mixed": (3, 300, dict(nframes=8, err_range_pct=20, drop_slice_pct=10, trunc_slice_pct=10), False),
    # 00 00 02 inside a slice NAL without any 00 00 03 (patched in, see
    # find_patch): no emulation check, the slice fails to parse instead
    "err_000002_no_epb": (1, 12, dict(nframes=3, w_mbs=12, h_mbs=6, slices=1), False),
}
PATCHED = {"err_000002_no_epb"}
CASES.update(ERR_CASES)
# Reference-picture management (generator knobs ref_mod_pct / mmco_pct /
# lt_idr_pct / nonref_pct): RefPicList0 modification incl. two indices naming
# one picture (bS compares pictures, deblocking.c:348, 402), MMCO 1-6,
# long-term pictures, non-reference pictures, gaps (dpb.c:224-1350).
REF_CASES = {
    "ref_mod_alias_12x8": (2, 3, dict(nframes=10, w_mbs=12, h_mbs=8, crop_bottom=0, slices=2, gop=10,
                                      num_ref_frames=4, ref_mod_pct=90, mv_jitter=2), False),
    "ref_mmco_lt_12x8": (2, 22, dict(nframes=30, w_mbs=12, h_mbs=8, crop_bottom=0, slices=2, gop=15,
                                     num_ref_frames=4, log2_max_frame_num=4, mmco_pct=60, lt_idr_pct=100,
                                     ref_mod_pct=40), False),
    "ref_mmco_poc0_reorder": (2, 22, dict(nframes=24, w_mbs=10, h_mbs=6, crop_bottom=0, slices=2, gop=12,
                                          num_ref_frames=3, poc_type=0, poc_swap=1, mmco_pct=50,
                                          nonref_pct=30, lt_idr_pct=50, ref_mod_pct=40), False),
    "ref_nonref_gaps_poc0": (2, 23, dict(nframes=24, w_mbs=10, h_mbs=6, crop_bottom=0, slices=2, gop=12,
                                         num_ref_frames=3, poc_type=0, poc_swap=1, nonref_pct=40,
                                         drop_pic_pct=20, gaps_allowed=1), False),
    "ref_all_1080p": (3, 400, dict(nframes=16, ref_mod_pct=50, mmco_pct=40, lt_idr_pct=50, nonref_pct=20), False),
}
CASES.update(REF_CASES)
# Degenerate picture shapes (one MB, one MB row, one MB column, thin strips):
# every neighbour-availability, ring, row-hand-off and edge-clamp corner of
# the row workgroups, with heavy off-picture MVs, intra-heavy P pictures,
# constrained intra and one slice per MB
_E = dict(nframes=8, crop_bottom=0, gop=5, offpic_pct=25, mv_jitter=8)
EDGE_CASES = {
    "edge_1x1_i": (1, 901, dict(_E, w_mbs=1, h_mbs=1, slices=1, im_pcm=20), False),
    "edge_1x1_ip": (2, 902, dict(_E, w_mbs=1, h_mbs=1, slices=1), False),
    "edge_1x9_ip": (2, 903, dict(_E, w_mbs=1, h_mbs=9, slices=3, pm_intra=30), False),
    "edge_9x1_ip": (2, 904, dict(_E, w_mbs=9, h_mbs=1, slices=2, dbf_idc2_pct=50), False),
    "edge_2x2_ip_mbslices": (2, 905, dict(_E, w_mbs=2, h_mbs=2, slices=4, cip=1, pm_intra=40), False),
    "edge_2x13_ip": (2, 906, dict(_E, w_mbs=2, h_mbs=13, slices=2, num_ref_frames=4), False),
    "edge_17x2_ip": (2, 907, dict(_E, w_mbs=17, h_mbs=2, slices=3, chroma_qp_offset=9), False),
    "edge_31x1_i": (1, 908, dict(_E, w_mbs=31, h_mbs=1, slices=1), False),
    "edge_3x23_ip_idc1": (2, 909, dict(_E, w_mbs=3, h_mbs=23, slices=2, dbf_idc1_pct=40), False),
}
CASES.update(EDGE_CASES)
# bench.py config legs: 24 pictures each
for s in (1, 2, 3, 4):
    CASES[f"leg_cfg2_720p_s{s}"] = (1, s, dict(nframes=24), False)
CASES["leg_cfg5_2160p_s100"] = (4, 100, dict(nframes=24), False)
# bench.py streams: config 3, 60 frames (4 warmup + 56 timed).  configs[3]
# (64 streams, 8 per GPU) uses seeds 100..163: rank r of bench.py --gpus N owns
# seeds 100 + 8r .. 100 + 8r + 7 (tests/test_gpu_parity.py decodes each shard)
for s in range(100, 164):
    CASES[f"bench_1080p_s{s}"] = (3, s, dict(nframes=60), False)
# bench.py leg `cfg3_realistic_motion`: rank 0's streams without off-picture
# motion (the generator's offpic_pct = 0), where frame-pipelined launches
# wait on (MB row, MB column) cells
for s in range(100, 108):
    CASES[f"bench_1080p_offpic0_s{s}"] = (3, s, dict(nframes=60, offpic_pct=0), False)
# bench.py leg `cfg3_no_loop_filter`: rank 0's streams with the loop filter
# off in every slice (disable_deblocking_filter_idc 1) -- the reference's own
# recommended encode (README.markdown:32-35, `-flags -loop`), where no MB row
# waits on the row above
for s in range(100, 108):
    CASES[f"bench_1080p_noloop_s{s}"] = (3, s, dict(nframes=60, dbf_idc1_pct=100), False)


def find_patch(stream: bytes):
    """A byte patch that puts 00 00 02 inside a slice NAL that has no
    emulation-prevention byte: the reference then skips the emulation check
    (byte_stream.c:142-145, 193) and parses the bytes as slice data."""
    starts = [i for i in range(len(stream) - 3) if stream[i:i + 4] == b"\0\0\0\1"] + [len(stream)]
    for a, b in zip(starts, starts[1:]):
        nal = stream[a + 4:b]
        if (nal[0] & 31) in (1, 5) and b"\0\0\3" not in nal and len(nal) > 200:
            return [[a + 4 + len(nal) * 3 // 4, "000002"]]
    raise RuntimeError("no candidate NAL")


def apply_patch(stream: bytes, patch) -> bytes:
    s = bytearray(stream)
    for off, hexb in patch or []:
        b = bytes.fromhex(hexb)
        s[off:off + len(b)] = b
    return bytes(s)


def one_case(item):
    """Generate one case's stream and decode it with the reference build."""
    from broadway_amd import gen
    import oracle as O

    name, (cfg, seed, ov, nr) = item
    stream = gen.generate(cfg, seed, **ov)
    base_sha = hashlib.sha256(stream).hexdigest()
    patch = find_patch(stream) if name in PATCHED else None
    stream = apply_patch(stream, patch)
    frames, pics = O.refdec_frames(stream, no_reorder=nr, info=True)
    p = gen.params(cfg, seed, **ov)
    w, h = p.w_mbs * 16, p.h_mbs * 16
    assert frames and all(len(f) == w * h * 3 // 2 for f in frames), name
    out = {
        "config": cfg, "seed": seed, "overrides": ov, "no_reorder": nr,
        "stream_bytes": len(stream), "stream_sha256": base_sha,
        "width": w, "height": h,
        "frames": [hashlib.md5(f).hexdigest() for f in frames],
    }
    if patch:
        out["patch"] = patch
    if name in ERR_CASES or name in REF_CASES:
        out["pics"] = [list(x) for x in pics]
    return name, out


def main():
    """--missing: keep the committed cases, add only the absent ones."""
    import concurrent.futures as cf

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    out = {"generator": "broadway_amd.gen (libh264gen.so)",
           "decoder": "reference C (Decoder/src, make.py file list + DecTestBench.c), gcc -O2",
           "frame_md5": "MD5 of each output frame: full MB-aligned I420 (w*h*3/2 bytes), output order",
           "cases": {}}
    old = {}
    if "--missing" in sys.argv and os.path.exists(path):
        old = json.load(open(path))["cases"]
    todo = [(n, c) for n, c in CASES.items() if n not in old]
    with cf.ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        done = dict(ex.map(one_case, todo))
    for name in CASES:
        out["cases"][name] = old[name] if name in old else done[name]
        if name in done:
            print(f"{name}: {len(done[name]['frames'])} frames {done[name]['width']}x{done[name]['height']}",
                  flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
