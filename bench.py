#!/usr/bin/env python3
"""Throughput benchmark: bit-exact 1080p H.264 Baseline reconstruction on MI355X.

Workload (BASELINE.json metric "1080p Baseline frames/s per GPU"; configs[3]:
64 concurrent 1080p streams sharded 8 per GPU): every rank owns 8 independent
synthetic 1080p I+P streams (seeds 100 + 8*rank .. +7, generated here by the
seeded Baseline generator -- there is no network for real media).  Each
stream is parsed once on the host into MB-record batches (the product parser,
libh264mi.so) and the batches are uploaded to HBM before timing, so the timed
region is the reconstruction hot path only (kernel-only fps).

A *step* = one picture of each of the rank's 8 streams reconstructed on the
GPU: k_inter (residual + motion compensation for all inter MBs of the 8
pictures) followed by the k_wave anti-diagonal sweep (intra + deblocking).
Steps follow decoding order, so the W warmup steps decode the first W
pictures and the K timed steps the next K.

Multi-GPU: one process per GPU (torch.distributed.run), streams partitioned
across ranks with no data-path collective -> "scaling": "weak";
the only communication is the barrier and the max-over-ranks of the timing.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import ctypes as C
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MBREC = 96


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=56)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--streams", type=int, default=8, help="streams per GPU (configs[3]: 8)")
    ap.add_argument("--config", type=int, default=3, help="generator preset (3 = 1080p I+P)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    return ap.parse_args()


def dist_setup(gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return torch, (dist if world > 1 else None), rank, local, world


def prepare(config, seeds, nframes):
    """generate + host-parse every stream (threads: ctypes releases the GIL)"""
    from broadway_amd import gen
    from broadway_amd.engine import Capture

    def one(seed):
        s = gen.generate(config, seed, nframes=nframes)
        return s, Capture(s)

    with cf.ThreadPoolExecutor(max_workers=min(len(seeds), 8)) as ex:
        res = list(ex.map(one, seeds))
    return [r[0] for r in res], [r[1] for r in res]


def upload(L, caps, nsteps):
    """Lay out all record batches / coefficients / picture descriptors in HBM.
    Step k's batch = picture k of every stream, records contiguous."""
    S = len(caps)
    w, h = caps[0].w_mbs, caps[0].h_mbs
    nmbs = w * h
    nslots = max(c.nslots for c in caps)
    rec_bytes = nmbs * MBREC
    recs = bytearray(nsteps * S * rec_bytes)
    coef_parts = []
    pics = np.zeros((nsteps * S, 8), dtype=np.uint32)
    cbase = 0
    for k in range(nsteps):
        for s, c in enumerate(caps):
            p = c.pictures[k]
            off = (k * S + s) * rec_bytes
            recs[off:off + rec_bytes] = C.string_at(p.rec, rec_bytes)
            if p.ncoef:
                coef_parts.append(C.string_at(p.coef, p.ncoef * 32))
            pics[k * S + s] = (s * nmbs, s * nslots, p.cur_slot, 0, cbase, 0, 0, 0)
            cbase += p.ncoef
    coefs = b"".join(coef_parts) + b"\0" * 64
    d_recs = L.h264mi_device_alloc(len(recs))
    d_coef = L.h264mi_device_alloc(len(coefs))
    d_pics = L.h264mi_device_alloc(pics.nbytes)
    if not (d_recs and d_coef and d_pics):
        raise RuntimeError("device allocation failed")
    rb = (C.c_char * len(recs)).from_buffer(recs)
    assert L.h264mi_copy_h2d(d_recs, rb, len(recs)) == 0
    assert L.h264mi_copy_h2d(d_coef, coefs, len(coefs)) == 0
    assert L.h264mi_copy_h2d(d_pics, pics.ctypes.data, pics.nbytes) == 0
    return d_recs, d_coef, d_pics, rec_bytes * S, nslots, len(recs) + len(coefs)


def inter_alg_bytes(caps, lo, hi):
    """Algorithmic bytes of k_inter for pictures [lo, hi) of every stream:
    MC reference footprint (SURVEY §8d R_alg luma+chroma term), the
    coefficient blocks and records of inter MBs, and the 384-B write of every
    inter MB."""
    dt = np.dtype([("type", "u1"), ("qp", "u1"), ("qpc", "u1"), ("avail", "u1"), ("pred", "u1"),
                   ("dbf", "u1"), ("offA", "i1"), ("offB", "i1"), ("cbits", "<u4"), ("coef", "<u4"),
                   ("i4", "u1", 8), ("ref", "u1", 4), ("mv", "<i2", 32), ("slice", "<u2"), ("rsv", "<u2")])
    assert dt.itemsize == MBREC
    total = 0
    n_inter = 0
    for c in caps:
        nmbs = c.w_mbs * c.h_mbs
        for k in range(lo, hi):
            p = c.pictures[k]
            r = np.frombuffer(C.string_at(p.rec, nmbs * MBREC), dtype=dt)
            inter = r["type"] <= 1
            cb = r["cbits"][inter]
            nblk = int(np.unpackbits(cb.view(np.uint8)).sum())
            ni = int(inter.sum())
            total += p.alg_ref_bytes + 32 * nblk + (MBREC + 384) * ni
            n_inter += ni
    return total, n_inter


def cpu_baseline(streams, nframes):
    """Reference C decoder (oracle/_ref/refdec, built from /root/reference
    sources) when present, else the CPU oracle restatement; one decoder
    process per stream, all streams in parallel."""
    refdec = os.path.join(ROOT, "oracle", "_ref", "refdec")
    ncores = min(len(streams), os.cpu_count() or 1, 16)
    td = tempfile.mkdtemp(prefix="h264bench")
    try:
        paths = []
        for i, s in enumerate(streams):
            pth = os.path.join(td, f"s{i}.h264")
            with open(pth, "wb") as f:
                f.write(s)
            paths.append(pth)
        if os.path.exists(refdec):
            kind = "reference"
            cmd = lambda p: [refdec, "-Onone", p]  # noqa: E731
        else:
            kind = "port"
            exe = os.path.join(ROOT, "oracle", "_build", "oracle_dec")
            cmd = lambda p: [exe, "-Onone", p]  # noqa: E731
        t0 = time.perf_counter()
        t_single = None
        for batch_start in range(0, len(paths), ncores):
            procs = [subprocess.Popen(cmd(p), stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
                     for p in paths[batch_start:batch_start + ncores]]
            for pr in procs:
                pr.wait()
        t1 = time.perf_counter()
        # single-core rate on one stream
        ts = time.perf_counter()
        subprocess.run(cmd(paths[0]), stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        t_single = time.perf_counter() - ts
        frames = nframes * len(paths)
        return {"value": round(frames / (t1 - t0), 2), "unit": "frames/s", "cores": ncores, "kind": kind,
                "sample": f"{len(paths)} x {nframes}-frame 1080p streams, one decoder process per stream "
                          f"on {ncores} host cores ({frames} frames, {t1 - t0:.1f}s); single core "
                          f"{nframes / t_single:.1f} fps"}
    finally:
        shutil.rmtree(td, ignore_errors=True)


def verify(eng, caps, streams, n_decoded):
    """Bit-exactness spot check: every slot still holding one of the last
    decoded pictures of stream 0 vs the CPU oracle's frame of that picture."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    c = caps[0]
    rep = O.Replay(c.w_mbs, c.h_mbs, c.nslots)
    for k in range(n_decoded):
        p = c.pictures[k]
        rep.picture(p.rec, p.coef, p.cur_slot)
    last = {}
    for k in range(n_decoded):
        last[c.pictures[k].cur_slot] = k
    ok = True
    for slot, k in last.items():
        if eng.read(0, slot).tobytes() != rep.frame(slot):
            ok = False
    return ok, len(last)


def main():
    a = parse_args()
    torch, dist, rank, local, world = dist_setup(a.gpus)
    from broadway_amd import _lib
    from broadway_amd.engine import Engine
    L = _lib.mi()

    S = a.streams
    seeds = [100 + rank * S + i for i in range(S)]
    nframes = a.warmup + a.steps
    t_prep = time.perf_counter()
    streams, caps = prepare(a.config, seeds, nframes)
    assert all(c.errors == 0 and c.npics >= nframes for c in caps), "stream preparation failed"
    w, h = caps[0].w_mbs, caps[0].h_mbs
    d_recs, d_coef, d_pics, step_rec_bytes, nslots, resident = upload(L, caps, nframes)
    t_prep = time.perf_counter() - t_prep

    eng = Engine(w, h, S, nslots, device=local)
    torch.cuda.set_device(local)

    def step(k):
        eng.decode_device(S, d_recs + k * step_rec_bytes, d_coef, d_pics + k * S * 32)

    for k in range(a.warmup):
        step(k)
    eng.sync()
    torch.cuda.synchronize()
    eng.set_timing(a.steps)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.warmup, a.warmup + a.steps):
        step(k)
    eng.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    dt = t1 - t0
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    inter_us, wave_us, nb = eng.timing_report()
    errors = eng.errors()

    frames_total = S * a.steps * world
    fps = frames_total / dt
    alg, n_inter = inter_alg_bytes(caps, a.warmup, a.warmup + a.steps)
    per_launch_bytes = alg / a.steps
    per_launch_us = inter_us / max(nb, 1)
    achieved = per_launch_bytes / (per_launch_us * 1e-6) / 1e9 if per_launch_us > 0 else 0.0
    # whole-frame read roofline of SURVEY §8d: R_alg = MC footprint + coefficients + records
    r_alg = 0
    for c in caps:
        for k in range(a.warmup, a.warmup + a.steps):
            p = c.pictures[k]
            r_alg += p.alg_ref_bytes + 32 * p.n_coded + MBREC * c.w_mbs * c.h_mbs
    frame_read_gbs = r_alg * world / dt / 1e9

    ok = None
    n_checked = 0
    if not a.no_verify and rank == 0:
        ok, n_checked = verify(eng, caps, streams, nframes)

    cpu = None
    if rank == 0 and not a.no_cpu_baseline:
        cpu = cpu_baseline(streams, nframes)

    if rank == 0:
        line = {
            "metric": "1080p Baseline frames/s per GPU; bit-exact YUV; % HBM-read roofline",
            "value": round(fps, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded H.264 Baseline generator; records pre-parsed on host, resident in HBM)",
            "config": {"workload": "configs[3]: 1080p (1920x1088, crop 1080) Baseline I+P, 1 I per 60, "
                                   "4 slices/picture, deblock idc 0/2",
                       "streams_per_gpu": S, "total_streams": S * world,
                       "frames_per_stream_timed": a.steps, "seeds": f"100..{100 + S * world - 1}",
                       "parallelism": f"streams sharded {S}/GPU, no collective"},
            "roofline": {"kernel": "k_inter", "bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None,
                         "alg_bytes_per_launch": int(per_launch_bytes),
                         "avg_launch_us": round(per_launch_us, 2)},
            "kernel_time_us_per_step": {"k_inter": round(inter_us / max(nb, 1), 2),
                                        "k_wave_sweep": round(wave_us / max(nb, 1), 2)},
            "frame_read_roofline": {"R_alg_GBs": round(frame_read_gbs, 2),
                                    "frac": round(frame_read_gbs / HBM_PEAK_GBS, 5)},
            "cpu_baseline": cpu,
            "bitexact_check": {"ok": ok, "frames_checked": n_checked, "residual_range_errors": errors},
            "prep_seconds": round(t_prep, 1),
            "hbm_resident_input_MB": round(resident / 1e6, 1),
        }
        print(json.dumps(line))
    eng.close()
    for p in (d_recs, d_coef, d_pics):
        L.h264mi_device_free(p)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
