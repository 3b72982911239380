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
GPU by one k_wgpp launch:
  row workgroups   one per (picture, MB row): three MC waves (6-tap luma /
                   bilinear chroma MC, intra prediction, clip-add) feed an
                   LDS ring, two ping-pong row waves run the in-loop
                   deblocking chain; rows hand off through tagged-granule
                   mailboxes;
  tail workgroups  k_prep of step t+1 (every MB in parallel: deblocking
                   record and residual -- dequant + inverse transforms; it
                   reads no reconstructed sample); they come after every row
                   workgroup in dispatch order, so they run on the CUs that
                   drained rows free (tools/prep_at.sh: waiting for 20-70 %
                   of the rows on top of that is 1-6 % slower).
The first step's k_prep is its own launch.
Steps follow decoding order, so the W warmup steps decode the first W
pictures and the K timed steps the next K.

Bit-exactness: after the timed loop an untimed pass decodes the same W + K
steps again and compares EVERY picture of every stream of every rank with the
reference decoder's per-frame MD5s (tests/golden/golden.json, made by running
the reference C on the same generated streams, seeds 100..163).

Multi-GPU: one process per GPU, streams partitioned across ranks with no
data-path collective -> "scaling": "weak"; the only
communication is the barrier, the max-over-ranks of the timing and the sum of
the verification counts (gloo, host scalars).  `--gpus N` without a
torch.distributed environment starts the N ranks itself (torch.distributed.run,
before this process touches the GPU).  `--dry-run` runs the sharding, host
parse, step loop and reductions without any device call (CPU tests).

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
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MBREC = 96
MAX_E2E_PROCS = 8          # end-to-end leg: decoder processes (the box allows 16 GPU processes)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=56)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--streams", type=int, default=8, help="streams per GPU (configs[3]: 8)")
    ap.add_argument("--config", type=int, default=3, help="generator preset (3 = 1080p I+P)")
    ap.add_argument("--gen", default="", help="generator overrides k=v,... (experiments; default: preset)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (host parse + GPU + D2H) leg")
    ap.add_argument("--no-rgba", action="store_true", help="skip the RGBA output leg")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the SURVEY §8d config 2 (720p I-only) / config 5 (2160p) legs")
    ap.add_argument("--pipe", type=int, default=int(os.environ.get("BENCH_PIPE", "1")),
                    help="steps per launch (1 or 2): with 2, a launch reconstructs two consecutive pictures of "
                         "every stream and the second's rows start as the reference rows they read are final")
    ap.add_argument("--dry-run", action="store_true",
                    help="no device calls: sharding, host parse, step loop and reductions only (CPU tests)")
    return ap.parse_args(argv)


def shard_seeds(rank: int, streams_per_gpu: int):
    """Stream seeds of one rank: streams partition across ranks, no overlap."""
    return [100 + rank * streams_per_gpu + i for i in range(streams_per_gpu)]


def reduce_over_ranks(dist, torch, value: float, op: str = "max") -> float:
    if dist is None:
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def max_over_ranks(dist, torch, value: float) -> float:
    return reduce_over_ranks(dist, torch, value, "max")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(gpus: int, argv) -> int:
    """--gpus N outside torch.distributed: start N ranks (one per GPU) with
    torch.distributed.run as a child process (this process has not touched
    the GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dist_setup(gpus: int):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    # BENCH_ONE_DEVICE=1: every rank on device 0 -- a rehearsal of the N-rank
    # path (sharding, barriers, max-over-ranks timing, verification sums) on
    # a one-GPU box; the value is then NOT a multi-GPU throughput
    if os.environ.get("BENCH_ONE_DEVICE") == "1":
        local = 0
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}")
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return torch, (dist if world > 1 else None), rank, local, world


def prepare(config, seeds, nframes, overrides=None):
    """generate + host-parse every stream (threads: ctypes releases the GIL)"""
    from broadway_amd import gen
    from broadway_amd.engine import Capture

    def one(seed):
        s = gen.generate(config, seed, nframes=nframes, **(overrides or {}))
        return s, Capture(s)

    with cf.ThreadPoolExecutor(max_workers=min(len(seeds), 8)) as ex:
        res = list(ex.map(one, seeds))
    return [r[0] for r in res], [r[1] for r in res]


def pack(caps, npics):
    """Host image of every record batch / coefficient block / picture
    descriptor of pictures [0, npics) of every stream.  Step k's records are
    contiguous, picture-major (stream s at k*S + s); PicDesc.rec_base is
    relative to the step's records, coef_base to the whole coefficient pool."""
    S = len(caps)
    nmbs = caps[0].w_mbs * caps[0].h_mbs
    nslots = max(c.nslots for c in caps)
    rec_bytes = nmbs * MBREC
    recs = bytearray(npics * S * rec_bytes)
    coef_parts = []
    pics = np.zeros((npics * S, 8), dtype=np.uint32)
    cbase = 0
    for j in range(npics):
        for s, c in enumerate(caps):
            p = c.pictures[j]
            off = (j * S + s) * rec_bytes
            recs[off:off + rec_bytes] = C.string_at(p.rec, rec_bytes)
            if p.ncoef:
                coef_parts.append(C.string_at(p.coef, p.ncoef * 32))
            pics[j * S + s] = (s * nmbs, s * nslots, p.cur_slot, 0, cbase, 0, 0, 0)
            cbase += p.ncoef
    coefs = b"".join(coef_parts) + b"\0" * 64
    return recs, coefs, pics, rec_bytes * S, nslots


def upload(L, caps, npics, packed=None):
    """pack() into HBM; returns (d_recs, d_coef, d_pics, step_rec_bytes,
    nslots, resident bytes)."""
    recs, coefs, pics, step_rec_bytes, nslots = packed or pack(caps, npics)
    d_recs = L.h264mi_device_alloc(len(recs))
    d_coef = L.h264mi_device_alloc(len(coefs))
    d_pics = L.h264mi_device_alloc(pics.nbytes)
    if not (d_recs and d_coef and d_pics):
        raise RuntimeError("device allocation failed")
    rb = (C.c_char * len(recs)).from_buffer(recs)
    assert L.h264mi_copy_h2d(d_recs, rb, len(recs)) == 0
    assert L.h264mi_copy_h2d(d_coef, coefs, len(coefs)) == 0
    assert L.h264mi_copy_h2d(d_pics, pics.ctypes.data, pics.nbytes) == 0
    return d_recs, d_coef, d_pics, step_rec_bytes, nslots, len(recs) + len(coefs)


def slots_read(recs, nmbs, i):
    """DPB slots the inter MBs of packed picture i read (MbRec.ref, bytes
    24..27 of each 96-B record; MBT_INTER = 0, MBT_SKIP = 1)."""
    r = np.frombuffer(recs, dtype=np.uint8, count=nmbs * MBREC, offset=i * nmbs * MBREC).reshape(nmbs, MBREC)
    inter = r[:, 0] <= 1
    return set(np.unique(r[inter, 24:28]).tolist())


def rename_slots(recs, pics, S, nmbs, nslots):
    """Physical frame slots for frame-pipelined launches: the host parser's
    DPB slot d of a stream maps to one of nslots + 1 physical slots, and a
    picture decoded into d gets the physical slot released longest ago --
    never the one d held before (which the previous picture may still be
    reading, e.g. the reference the sliding window just dropped).  The
    mapping is a bijection at every picture, so the records' reference-slot
    comparisons (bS) are unchanged; MbRec.ref and PicDesc cur_slot /
    frame_base are rewritten in place.  Returns the physical slot count."""
    nphys = nslots + 1
    n = len(pics) // S
    arr = np.frombuffer(recs, dtype=np.uint8).reshape(-1, MBREC)
    for s in range(S):
        cur = {}                              # DPB slot -> physical slot
        free = list(range(nphys))             # released order, oldest first
        for k in range(n):
            i = k * S + s
            lut = np.arange(256, dtype=np.uint8)
            for d, ph in cur.items():
                lut[d] = ph
            r = arr[i * nmbs:(i + 1) * nmbs]
            inter = r[:, 0] <= 1
            r[inter, 24:28] = lut[r[inter, 24:28]]
            d = int(pics[i][2])
            old = cur.get(d)
            ph = next(x for x in free if x != old)
            free.remove(ph)
            if old is not None:
                free.append(old)
            cur[d] = ph
            pics[i][1] = s * nphys
            pics[i][2] = ph
    return nphys


def schedule(recs, pics, S, nmbs, warmup, steps, P):
    """Launches as (first step, steps in it).  P = 2 pairs steps (2i, 2i+1)
    when, for every stream, the pair's pictures write different slots and
    the first does not read the slot the second writes (the engine's
    frame-pipelined batch contract); otherwise, or when warmup / steps are
    odd, every launch is one step."""
    n = warmup + steps
    if P > 1 and warmup % P == 0 and steps % P == 0:
        ok = True
        for k0 in range(0, n, P):
            for s in range(S):
                a, b = k0 * S + s, (k0 + 1) * S + s
                if pics[a][2] == pics[b][2] or pics[b][2] in slots_read(recs, nmbs, a):
                    ok = False
        if ok:
            return [(k, P) for k in range(0, n, P)]
    return [(k, 1) for k in range(n)]


def pack_steps(pics, S, nmbs, P):
    """PicDesc array for P-step launches: picture j * S + s of the launch at
    step k0 has rec_base relative to step k0's records."""
    out = pics.copy()
    for i in range(len(pics)):
        k, s = divmod(i, S)
        out[i][0] = ((k % P) * S + s) * nmbs
    return out


def golden_frames(config, seed, overrides):
    """The reference decoder's per-frame MD5s of generator stream (config,
    seed) when a fixture covers it (overrides other than nframes: none)."""
    if overrides:
        return None
    gold = os.path.join(ROOT, "tests", "golden", "golden.json")
    if not os.path.exists(gold):
        return None
    best = None
    for c in json.load(open(gold))["cases"].values():
        if c["config"] == config and c["seed"] == seed and set(c["overrides"]) <= {"nframes"} \
                and not c["no_reorder"] and (best is None or len(c["frames"]) > len(best)):
            best = c["frames"]
    return best


def cpu_baseline(streams, nframes, reps=10):
    """Reference C decoder (oracle/_ref/refdec, built from /root/reference
    sources by oracle/Makefile.ref) when present, else the CPU oracle
    restatement.  One decoder process per stream, all streams in parallel
    (one host core each), each stream decoded `reps` times back to back:
    a bounded sample of about 10 s of CPU work."""
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

        def run(pth):
            for _ in range(reps):
                subprocess.run(cmd(pth), stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True)

        ts = time.perf_counter()
        subprocess.run(cmd(paths[0]), stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True)
        t_single = time.perf_counter() - ts
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(max_workers=ncores) as ex:
            list(ex.map(run, paths[:ncores]))
        t1 = time.perf_counter()
        frames = nframes * ncores * reps
        try:
            cpu_model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
        except (OSError, StopIteration):
            cpu_model = "unknown"
        return {"value": round(frames / (t1 - t0), 2), "unit": "frames/s", "cores": ncores, "kind": kind,
                "sample": f"{ncores} x {nframes}-frame 1080p streams x {reps} passes, one decoder process per "
                          f"stream on {ncores} host cores ({frames} frames, {t1 - t0:.1f} s, {cpu_model}); "
                          f"single core {nframes / t_single:.1f} fps"}
    finally:
        shutil.rmtree(td, ignore_errors=True)


def rgba_leg(torch, L, eng, S, w_mbs, h_mbs, reps=50):
    """Decoder.js `rgb: true` output: the I420 -> RGBA
    kernel (k_yuv2rgba, color.hip) over one reconstructed picture of each
    stream (frame slot 0, resident in HBM), one launch per step, timed with
    HIP events on the launch stream.  An HBM-bound elementwise kernel: 1.5 B
    read + 4 B written per pixel are its algorithmic bytes."""
    width, height = w_mbs * 16, h_mbs * 16
    out = torch.empty(S * width * height * 4, dtype=torch.uint8, device="cuda")
    base = eng.frame_ptr(0, 0)
    stride = eng.frame_ptr(1, 0) - base if S > 1 else 0
    st = torch.cuda.current_stream()
    launch = lambda: L.h264mi_yuv2rgba_device(base, out.data_ptr(), width, height, S, stride, width * height * 4,
                                              st.cuda_stream)
    for _ in range(5):
        assert launch() == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        launch()
    e1.record(st)
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    alg = S * width * height * (1.5 + 4)
    gbs = alg / (us * 1e-6) / 1e9
    del out
    return {"kernel": "k_yuv2rgba", "pictures_per_launch": S, "avg_launch_us": round(us, 2),
            "frames_per_s": round(S / (us * 1e-6), 1), "alg_bytes_per_launch": int(alg),
            "achieved_GBs": round(gbs, 1), "peak": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4),
            "semantics": "per pixel DecoderPost.js yuv2rgbcalc (:514-560), RGBA bytes",
            "note": "repeated launches over the same pictures: the I420 input stays in the 256 MB "
                    "MALL, the RGBA output is written with non-temporal stores"}


def end_to_end(streams, nframes, reps=3):
    """End-to-end decode through the product C-ABI: one
    broadway_amd/lib/h264mi_dec process per stream (at most MAX_E2E_PROCS),
    all in parallel (one host thread each), each decoding its stream `reps`
    times -- host CAVLC parse, H2D of the MB records, k_prep + k_wgpp, D2H of
    every output picture.  Rate = all pictures / the slowest process's decode
    time (HIP start-up of each process excluded; it is paid before its timed
    loop)."""
    exe = os.path.join(ROOT, "broadway_amd", "lib", "h264mi_dec")
    if not os.path.exists(exe):
        return None
    streams = streams[:MAX_E2E_PROCS]
    # a thread waiting for the GPU sleeps instead of spinning: the host cores
    # are the bound on this path (tools/e2e_env_sweep.sh: 1.89k -> 2.08k fps)
    env = dict(os.environ)
    env.setdefault("H264MI_BLOCKING_SYNC", "1")
    td = tempfile.mkdtemp(prefix="h264e2e")
    try:
        procs = []
        for i, s in enumerate(streams):
            pth = os.path.join(td, f"s{i}.h264")
            with open(pth, "wb") as f:
                f.write(s)
            procs.append(subprocess.Popen([exe, "-Onone", f"-r{reps}", "-T", pth], stdout=subprocess.PIPE,
                                          stderr=subprocess.PIPE, text=True, env=env))
        secs, pics, parts, cpu_s = [], 0, {}, 0.0
        for pr in procs:
            o, e = pr.communicate(timeout=600)
            if pr.returncode != 0:
                raise RuntimeError(f"h264mi_dec failed: {e.strip()[-300:]}")
            for line in o.splitlines():
                f = line.split()
                if not f:
                    continue
                if f[0] == "pictures":
                    pics += int(f[1])
                elif f[0] == "decode_seconds":
                    secs.append(float(f[1]))
                elif f[0].startswith("t_") and len(f) > 1:
                    parts[f[0]] = parts.get(f[0], 0.0) + float(f[1])
                elif f[0] == "cpu_seconds":
                    cpu_s += float(f[1])
        t = max(secs)
        res = {"value": round(pics / t, 2), "unit": "frames/s", "host_threads": len(streams),
               "sample": f"{len(streams)} x {nframes}-frame 1080p streams x {reps} passes, one h264mi_dec process "
                         f"(H264SwDec* C-ABI) per stream: host parse + H2D + kernels + D2H of every picture; "
                         f"{pics} frames in {t:.2f} s"}
        if parts and pics:
            # per picture inside one decoder process (H264SwDecGetTiming):
            # host parse / record upload + launch / wait for the GPU / D2H copy
            res["per_picture_ms"] = {k[2:]: round(v * 1e3 / pics, 3) for k, v in sorted(parts.items())}
            res["parse_threads_per_process"] = 1 + int(os.environ.get("H264MI_PARSE_THREADS", "3"))
            res["host_sync"] = "blocking" if env["H264MI_BLOCKING_SYNC"] == "1" else "spin"
            # host CPU time (all threads of all processes) per picture, and the
            # cores that keeps busy at the measured rate
            res["host_cpu_ms_per_picture"] = round(cpu_s * 1e3 / pics, 3)
            res["host_cores_busy"] = round(cpu_s / t, 2)
        # the same streams in ONE process, one thread (H264SwDec instance) per
        # stream, sharing one batched engine (h264mi_set_share, -S)
        paths = [os.path.join(td, f"s{i}.h264") for i in range(len(streams))]
        o = subprocess.run([exe, "-Onone", f"-r{reps}", "-T", f"-S{len(streams)}"] + paths, capture_output=True,
                           text=True, timeout=600, env=env)
        if o.returncode == 0:
            d = {}
            for line in o.stdout.splitlines():
                f = line.split()
                if len(f) >= 2:
                    try:
                        d[f[0]] = float(f[1])
                    except ValueError:
                        pass
            if d.get("pictures") and d.get("decode_seconds"):
                res["one_process_shared_engine"] = {
                    "value": round(d["pictures"] / d["decode_seconds"], 2), "unit": "frames/s",
                    "threads": len(streams),
                    "pictures_per_launch": round(d.get("share_pictures", 0) / max(d.get("share_batches", 1), 1), 2),
                    "host_cpu_ms_per_picture": round(d.get("cpu_seconds", 0) * 1e3 / d["pictures"], 3)}
        return res
    finally:
        shutil.rmtree(td, ignore_errors=True)


def verify_all(eng, launch, sched, caps, seeds, config, overrides, cur_slots=None):
    """Untimed verification pass: run every launch of the schedule again and
    compare every picture of every stream with the reference decoder's MD5s
    (POC type 2: output order == decode order, frame k = picture k) right
    after its launch (the pictures of one launch write distinct slots).
    Returns (ok, frames checked, frames without a fixture)."""
    refs = [golden_frames(config, sd, overrides) for sd in seeds]
    ok, n, missing = True, 0, 0
    for i, (k0, P) in enumerate(sched):
        launch(i)
        eng.sync()
        for k in range(k0, k0 + P):
            for s, c in enumerate(caps):
                ref = refs[s]
                if ref is None or k >= len(ref):
                    missing += 1
                    continue
                slot = c.pictures[k].cur_slot if cur_slots is None else int(cur_slots[k][s])
                got = hashlib.md5(eng.read(s, slot).tobytes()).hexdigest()
                n += 1
                if got != ref[k]:
                    ok = False
    return ok, n, missing


def load_traffic():
    """HBM bytes per step from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.py -> profiles/traffic.json), or None."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p))
    except ValueError:
        return None


class _DryEngine:
    """--dry-run stand-in for broadway_amd.engine.Engine: no device calls."""

    def __init__(self, *a, **k):
        self.launches = 0

    def decode_device(self, *a):
        self.launches += 1

    def decode_device_next(self, *a):
        self.launches += 1

    def decode_device_steps(self, *a):
        self.launches += 1

    def set_steps(self, *a):
        pass

    def sync(self):
        pass

    def set_timing(self, *a, **k):
        pass

    def timing_report(self):
        return 0.0, 0.0, 0

    def errors(self):
        return 0

    def kernel_name(self):
        return "dry-run"

    def close(self):
        pass


class DeviceRun:
    """The bench's device-resident path for one rank: records, coefficient
    blocks and descriptors of pictures [0, warmup + steps) of every stream in
    HBM, an engine for the S streams, and the launch schedule (P steps per
    launch when the streams allow it, physical slots renamed for it; the next
    launch's k_prep in each launch's tail).  dry: no device calls."""

    def __init__(self, L, caps, warmup, steps, pipe, device=0, dry=False):
        self.L, self.S = L, len(caps)
        S, nframes = self.S, warmup + steps
        w, h = caps[0].w_mbs, caps[0].h_mbs
        nmbs = w * h
        packed = pack(caps, nframes)
        recs_h, _, pics_h, self.srb, nslots = packed
        if pipe > 1:
            nslots = rename_slots(recs_h, pics_h, S, nmbs, nslots)
            packed = packed[:4] + (nslots,)
        self.sched = schedule(recs_h, pics_h, S, nmbs, warmup, steps, pipe)
        self.P = self.sched[0][1]
        self.cur_slots = pics_h[:, 2].reshape(nframes, S).copy()
        self.bufs = []
        if dry:
            self.d_recs = self.d_coef = self.pics_base = 0
            self.resident = 0
            self.eng = _DryEngine()
            return
        from broadway_amd.engine import Engine
        self.d_recs, self.d_coef, d_pics, _, nslots, self.resident = upload(L, caps, nframes, packed)
        self.bufs = [self.d_recs, self.d_coef, d_pics]
        self.pics_base = d_pics
        if self.P > 1:
            ps = pack_steps(pics_h, S, nmbs, self.P)
            d = L.h264mi_device_alloc(ps.nbytes)
            assert d and L.h264mi_copy_h2d(d, ps.ctypes.data, ps.nbytes) == 0
            self.bufs.append(d)
            self.pics_base = d
        self.eng = Engine(w, h, S, nslots, device=device)
        if self.P > 1:
            self.eng.set_steps(self.P)

    def launch(self, i):
        """Launch i of the schedule: P steps; the next launch's k_prep runs
        in its tail workgroups."""
        S, srb = self.S, self.srb
        k0, p = self.sched[i]
        args = (self.d_recs + k0 * srb, self.d_coef, self.pics_base + k0 * S * 32)
        if i + 1 < len(self.sched):
            k1 = self.sched[i + 1][0]
            self.eng.decode_device_steps(S, p, *args, self.d_recs + k1 * srb, self.d_coef,
                                         self.pics_base + k1 * S * 32)
        else:
            self.eng.decode_device_steps(S, p, *args)

    def close_engine(self):
        if self.eng is not None:
            self.eng.close()
            self.eng = None

    def free(self):
        self.close_engine()
        for p in self.bufs:
            self.L.h264mi_device_free(p)
        self.bufs = []


def run_leg(L, torch, config, seeds, steps, warmup, mc_waves=3, rpw=0):
    """One single-GPU measurement of another SURVEY §8d config with the same
    step structure (records resident in HBM, one k_wgpp launch per step,
    HIP events on every launch) and the same untimed verification against
    the reference MD5s.  Returns a dict for the bench line."""
    from broadway_amd.engine import Engine
    nframes = warmup + steps
    streams, caps = prepare(config, seeds, nframes)
    assert all(c.errors == 0 and c.npics >= nframes for c in caps), "leg stream preparation failed"
    S = len(caps)
    w, h = caps[0].w_mbs, caps[0].h_mbs
    d_recs, d_coef, d_pics, srb, nslots, _ = upload(L, caps, nframes)
    # both knobs are read once, when the engine is created
    os.environ["H264MI_MC_WAVES"] = str(mc_waves)
    if rpw:
        os.environ["H264MI_RPW"] = str(rpw)
    try:
        eng = Engine(w, h, S, nslots, device=torch.cuda.current_device())
    finally:
        os.environ.pop("H264MI_MC_WAVES", None)
        os.environ.pop("H264MI_RPW", None)
    try:
        def step(k):
            if k + 1 < nframes:
                eng.decode_device_next(S, d_recs + k * srb, d_coef, d_pics + k * S * 32,
                                       d_recs + (k + 1) * srb, d_coef, d_pics + (k + 1) * S * 32)
            else:
                eng.decode_device(S, d_recs + k * srb, d_coef, d_pics + k * S * 32)
        for k in range(warmup):
            step(k)
        eng.sync()
        eng.set_timing(steps, stride=1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(warmup, nframes):
            step(k)
        eng.sync()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        _, us, nb = eng.timing_report()
        launch_us = us / max(nb, 1)
        r_alg = sum(c.pictures[k].alg_ref_bytes + 32 * c.pictures[k].n_coded + MBREC * w * h
                    for c in caps for k in range(warmup, nframes)) / steps
        ok, n, missing = verify_all(eng, step, [(k, 1) for k in range(nframes)], caps, seeds, config, {})
        gbs = r_alg / (launch_us * 1e-6) / 1e9 if launch_us > 0 else 0.0
        return {"size": f"{w * 16}x{h * 16}", "streams": S, "seeds": seeds, "steps": steps,
                "mc_waves_per_row_workgroup": mc_waves,
                "rows_per_workgroup": eng.rows_per_workgroup(S),
                "frames_per_s": round(S * steps / dt, 1), "avg_launch_us": round(launch_us, 2),
                "picture_latency_ms": round(launch_us / 1e3, 3),
                "alg_bytes_per_launch": int(r_alg), "achieved_GBs": round(gbs, 1),
                "frac_hbm": round(gbs / HBM_PEAK_GBS, 5),
                "bitexact": {"ok": ok, "frames_checked": n, "frames_without_fixture": missing},
                "device_errors": eng.errors()}
    finally:
        eng.close()
        for p in (d_recs, d_coef, d_pics):
            L.h264mi_device_free(p)


def config_legs(L, torch):
    """SURVEY §8d config 2 (1280x720 I-only, seeds 1..4: the dependency-bound
    intra wavefront -- frames/s, not a roofline) and config 5 (3840x2160, one
    stream, the config-3 mix) with the MC-wave count of the row workgroup
    swept (2 vs 3: the sizing choice of this design)."""
    return {
        "cfg2_720p_ionly_4streams": run_leg(L, torch, 1, [1, 2, 3, 4], 20, 4),
        "cfg2_720p_ionly_1stream": run_leg(L, torch, 1, [1], 20, 4),
        "cfg5_2160p_1stream": run_leg(L, torch, 4, [100], 20, 4),
        "cfg5_2160p_1stream_2mc": run_leg(L, torch, 4, [100], 20, 4, mc_waves=2),
        "cfg5_2160p_1stream_2rows": run_leg(L, torch, 4, [100], 20, 4, rpw=2),
        "cfg5_2160p_1stream_2mc_2rows": run_leg(L, torch, 4, [100], 20, 4, mc_waves=2, rpw=2),
    }


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse_args(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, argv))
    torch, dist, rank, local, world = dist_setup(a.gpus)
    from broadway_amd import _lib
    L = _lib.mi()

    S = a.streams
    seeds = shard_seeds(rank, S)
    nframes = a.warmup + a.steps
    t_prep = time.perf_counter()
    overrides = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.gen.split(",") if kv)
    streams, caps = prepare(a.config, seeds, nframes, overrides)
    assert all(c.errors == 0 and c.npics >= nframes for c in caps), "stream preparation failed"
    w, h = caps[0].w_mbs, caps[0].h_mbs
    run = DeviceRun(L, caps, a.warmup, a.steps, a.pipe, device=local, dry=a.dry_run)
    if not a.dry_run:
        torch.cuda.set_device(local)
    eng, sched, launch, P, resident = run.eng, run.sched, run.launch, run.P, run.resident
    t_prep = time.perf_counter() - t_prep
    sync = (lambda: None) if a.dry_run else torch.cuda.synchronize

    nwarm = sum(1 for k0, _ in sched if k0 < a.warmup)
    for i in range(nwarm):
        launch(i)
    eng.sync()
    sync()
    # HIP events around every 4th launch, carried by k_wgpp's own dispatch
    # packet (hipExtLaunchKernelGGL: no marker packets between launches); a
    # profiled dispatch still costs the stream a little, hence the stride
    eng.set_timing(a.steps, stride=int(os.environ.get("BENCH_TIMING_STRIDE", "4")))
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(nwarm, len(sched)):
        launch(i)
    eng.sync()
    sync()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    dt = max_over_ranks(dist, torch, t1 - t0)
    _, rows_us, nb = eng.timing_report()
    errors = eng.errors()

    frames_total = S * a.steps * world
    fps = frames_total / dt
    # roofline: R_alg per frame = MC reference footprint + coded
    # 4x4 blocks x 32 B + 96-B MB records; one step = one picture of each of
    # the S streams, reconstructed by one k_prep + k_wgpp launch pair
    r_alg = 0
    for c in caps:
        for k in range(a.warmup, a.warmup + a.steps):
            p = c.pictures[k]
            r_alg += p.alg_ref_bytes + 32 * p.n_coded + MBREC * c.w_mbs * c.h_mbs
    launch_bytes = r_alg / (len(sched) - nwarm)
    step_us = rows_us / max(nb, 1)
    achieved = launch_bytes / (step_us * 1e-6) / 1e9 if step_us > 0 else 0.0
    traffic = load_traffic()
    frame_read_gbs = r_alg * world / dt / 1e9

    ok, n_checked, n_missing = None, 0, 0
    if not a.no_verify and not a.dry_run:
        ok, n_checked, n_missing = verify_all(eng, launch, sched, caps, seeds, a.config, overrides, run.cur_slots)
    n_checked_all = int(reduce_over_ranks(dist, torch, n_checked, "sum"))
    n_missing_all = int(reduce_over_ranks(dist, torch, n_missing, "sum"))
    ok_all = None if ok is None else reduce_over_ranks(dist, torch, 0.0 if ok else 1.0, "max") == 0.0
    errors_all = int(reduce_over_ranks(dist, torch, errors, "sum"))
    rgba = rgba_leg(torch, L, eng, S, w, h) if rank == 0 and not a.dry_run and not a.no_rgba else None

    cpu = None
    if rank == 0 and not a.no_cpu_baseline and not a.dry_run:
        cpu = cpu_baseline(streams, nframes)
    run.close_engine()
    legs = None
    if rank == 0 and world == 1 and not a.no_legs and not a.dry_run:
        legs = config_legs(L, torch)
    e2e = None
    if rank == 0 and world == 1 and not a.no_e2e and not a.dry_run:
        e2e = end_to_end(streams, nframes)

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
                                   "4 slices/picture, deblock idc 0/2" if a.config == 3 and not overrides
                                   else f"generator preset {a.config} {overrides or ''}".strip(),
                       "streams_per_gpu": S, "total_streams": S * world,
                       "frames_per_stream_timed": a.steps,
                       "seeds": f"100..{100 + S * world - 1}",
                       "parallelism": f"streams sharded {S}/GPU over {world} rank(s), no collective; "
                                      f"{P} consecutive picture(s) of each stream per launch"},
            "roofline": {"kernel": f"k_wgpp (one launch = {P} step(s); k_prep of the next launch runs in its tail)",
                         # what limits the kernel: the MB-row deblocking dependency chain
                         # (SQ counters profiles/r19_sq_s8.json), not HBM;
                         # `frac` is still quoted against the HBM peak, the metric's axis
                         "bound": "latency",
                         "frac_axis": "hbm",
                         "limiter": "latency: the MB-row deblocking dependency chain (DESIGN.md §3), not HBM",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic.get("hbm_bytes_per_step") if traffic else None,
                         "alg_bytes_per_launch": int(launch_bytes),
                         "avg_launch_kernel_us": round(step_us, 2),
                         "aggregate_achieved_GBs": round(frame_read_gbs, 1),
                         "traffic_source": traffic.get("source") if traffic else None},
            "kernels": {"k_wgpp": {"avg_launch_us": round(step_us, 2), "pictures_per_launch": S * P,
                                   "steps_per_launch": P,
                                   "timed_launches": nb,
                                   "bound": "latency (MB-row deblocking dependency chain); MC waves overlap it"}},
            "wall_read_GBs": round(frame_read_gbs, 2),
            "cpu_baseline": cpu,
            "end_to_end": e2e,
            "rgba_output": rgba,
            "config_legs": legs,
            "bitexact_check": {"ok": ok_all, "frames_checked": n_checked_all,
                               "frames_expected": S * world * nframes, "frames_without_fixture": n_missing_all,
                               "method": "untimed re-decode of all warmup+timed steps, every picture of every "
                                         "stream of every rank vs reference-decoder MD5s",
                               "residual_range_errors": errors_all},
            "prep_seconds": round(t_prep, 1),
            **({"one_device_rehearsal": f"{world} ranks shared device 0 (BENCH_ONE_DEVICE=1): not a multi-GPU rate"}
               if os.environ.get("BENCH_ONE_DEVICE") == "1" else {}),
            "hbm_resident_input_MB": round(resident / 1e6, 1),
        }
        if a.dry_run:
            line["dry_run"] = {"launches": eng.launches, "seeds": seeds}
        print(json.dumps(line), flush=True)
    run.free()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
