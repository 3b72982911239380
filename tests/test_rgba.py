"""`rgb: true` output: I420 -> RGBA with the reference
converter's per-pixel arithmetic (DecoderPost.js yuv2rgbcalc, :514-560).

Pinned by tests/golden/rgba_golden.json, made by running the reference's own
yuv2rgbcalc under node over all 2^24 (y, u, v) inputs
(tests/golden/make_rgba_golden.js).  One frame here enumerates every input
(each 2x2 block one (u, v) and four y), so the table MD5 checks a whole
conversion exhaustively: the CPU oracle on CPU, the HIP kernel on the GPU.

The fixture also records that the reference's asm.js driver (doit) does NOT
reproduce its own per-pixel function on a 1080p frame (its result cache is
indexed by byte address and can overlap the input, see the generator's
header); that cache-history-dependent output is not reproduced."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import oracle as O
from _golden import cases, stream
from broadway_amd.decoder import Decoder, split_annexb

GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rgba_golden.json")))
W = H = 4096          # 4,194,304 2x2 blocks = 65,536 (u, v) x 64 groups of 4 y


def all_inputs_frame():
    """I420 W x H frame whose pixels take every (y, u, v) exactly once:
    block k (raster over the 2048 x 2048 chroma grid) has u = k & 255,
    v = (k >> 8) & 255 and y = 4 (k >> 16) + {0, 1, 2, 3} for its pixels
    (0,0), (0,1), (1,0), (1,1)."""
    k = np.arange((W // 2) * (H // 2), dtype=np.int64).reshape(H // 2, W // 2)
    g = (k >> 16) * 4
    y = np.empty((H, W), dtype=np.uint8)
    y[0::2, 0::2] = g
    y[0::2, 1::2] = g + 1
    y[1::2, 0::2] = g + 2
    y[1::2, 1::2] = g + 3
    u = (k & 255).astype(np.uint8)
    v = ((k >> 8) & 255).astype(np.uint8)
    return np.concatenate([y.ravel(), u.ravel(), v.ravel()]), y, u, v


def table_md5(rgba, y, u, v):
    """Reorder a converted all-inputs frame into the fixture's table order
    (index (y << 16) | (u << 8) | v, one uint32 RGBA word each) and hash it."""
    words = np.frombuffer(rgba, dtype=np.uint32).reshape(H, W)
    uu = np.repeat(np.repeat(u, 2, axis=0), 2, axis=1).astype(np.int64)
    vv = np.repeat(np.repeat(v, 2, axis=0), 2, axis=1).astype(np.int64)
    idx = (y.astype(np.int64) << 16) | (uu << 8) | vv
    table = np.zeros(1 << 24, dtype=np.uint32)
    table[idx.ravel()] = words.ravel()
    return hashlib.md5(table.tobytes()).hexdigest(), table


def test_oracle_matches_reference_yuv2rgbcalc_table():
    frame, y, u, v = all_inputs_frame()
    rgba = O.yuv2rgba(frame.tobytes(), W, H)
    md5, table = table_md5(rgba, y, u, v)
    assert md5 == GOLD["table_md5"]
    for key, word in GOLD["table_samples"].items():
        yy, uu, vv = map(int, key.split(","))
        assert table[(yy << 16) | (uu << 8) | vv] == int(word, 16)


def test_fixture_records_reference_driver_divergence():
    d = GOLD["doit_1920x1088"]
    assert d["pixels"] == 1920 * 1088 and 0 < d["differ_from_table"] < d["pixels"]


@pytest.mark.gpu
def test_hip_kernel_matches_reference_table():
    import torch
    from broadway_amd import _lib
    L = _lib.mi()
    frame, y, u, v = all_inputs_frame()
    d_in = torch.from_numpy(frame).to("cuda")
    d_out = torch.empty(W * H * 4, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    assert L.h264mi_yuv2rgba_device(d_in.data_ptr(), d_out.data_ptr(), W, H, 1, 0, 0, st.cuda_stream) == 0
    torch.cuda.synchronize()
    md5, _ = table_md5(d_out.cpu().numpy().tobytes(), y, u, v)
    assert md5 == GOLD["table_md5"]


@pytest.mark.gpu
def test_hip_kernel_batched_pictures_vs_oracle():
    """npics > 1 with padded strides, 1080p-sized pictures (MB-aligned)."""
    import torch
    from broadway_amd import _lib
    L = _lib.mi()
    w, h, n = 1920, 1088, 3
    rng = np.random.default_rng(7)
    pics = [rng.integers(0, 256, w * h * 3 // 2, dtype=np.uint8) for _ in range(n)]
    in_stride, out_stride = w * h * 3 // 2 + 4096, w * h * 4 + 8192
    host_in = np.zeros(in_stride * n, dtype=np.uint8)
    for k, p in enumerate(pics):
        host_in[k * in_stride:k * in_stride + p.size] = p
    d_in = torch.from_numpy(host_in).to("cuda")
    d_out = torch.zeros(out_stride * n, dtype=torch.uint8, device="cuda")
    assert L.h264mi_yuv2rgba_device(d_in.data_ptr(), d_out.data_ptr(), w, h, n, in_stride, out_stride,
                                    torch.cuda.current_stream().cuda_stream) == 0
    out = d_out.cpu().numpy()
    for k, p in enumerate(pics):
        assert out[k * out_stride:k * out_stride + w * h * 4].tobytes() == O.yuv2rgba(p.tobytes(), w, h)
        assert not out[k * out_stride + w * h * 4:(k + 1) * out_stride].any()     # nothing written past a picture


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["small_ip_8x6_2sl", "cfg1_plumbing_640x368"])
def test_decoder_js_rgb_option_vs_reference(name):
    """Decoder({rgb: true}): every emitted picture is the RGBA conversion of
    the reference decoder's I420 output for that picture (golden MD5s)."""
    c = cases()[name]
    s = stream(c)
    yuv, rgb, dims = [], [], []
    for opts, sink in (({}, yuv), ({"rgb": True}, rgb)):
        dec = Decoder(opts)
        dec.onPictureDecoded = lambda buf, w, h, infos, sink=sink: (sink.append(bytes(buf)), dims.append((w, h)))
        for nal in split_annexb(s):
            dec.decode(nal)
        dec.close()
    assert len(rgb) == len(yuv) > 0
    w, h = dims[0]
    for f_yuv, f_rgb in zip(yuv, rgb):
        assert hashlib.md5(f_yuv).hexdigest() in c["frames"]
        assert len(f_rgb) == w * h * 4
        assert f_rgb == O.yuv2rgba(f_yuv, w, h)
