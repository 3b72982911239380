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
DB_INNER = 64            # MbRec.avail: the MB filters its edges (include/h264mi_records.h)
MAX_E2E_PROCS = 8          # end-to-end leg: decoder processes (the box allows 16 GPU processes)
E2E_REPS = 21              # end-to-end leg: passes over each 60-picture stream (>= 3 s at ~400 frames/s per process)


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
    ap.add_argument("--pipe", type=int, default=int(os.environ.get("BENCH_PIPE", "3")),
                    help="steps per launch (1..4; default 3, profiles/r91_ab_pipe3.txt): with P > 1, a launch "
                         "reconstructs P consecutive pictures of every stream and a later picture's rows start as "
                         "the reference rows they read are final; the GOP phases put every IDR last in its launch")
    ap.add_argument("--aligned", action="store_true",
                    help="all streams' GOPs aligned, pictures W .. W+K-1 timed (no IDR in short windows); "
                         "default: GOP phases staggered over the streams")
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
    descriptor of pictures [0, npics) of every stream.  Picture k of stream s
    is record batch k*S + s; its PicDesc (row k*S + s) has rec_base relative
    to the whole record pool and coef_base to the whole coefficient pool, so
    a launch may take any picture of any stream (DeviceRun's plans)."""
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
            heavy = 4 if 2 * p.n_intra > nmbs else 0          # PicDesc.flags PD_INTRA_HEAVY
            # PD_NO_DEBLOCK: no record's avail byte (MbRec byte 3) has DB_INNER
            nodb = 0 if (np.frombuffer(recs, dtype=np.uint8, count=rec_bytes, offset=off)[3::MBREC] & DB_INNER).any() else 8
            pics[j * S + s] = ((j * S + s) * nmbs, s * nslots, p.cur_slot, heavy | nodb, cbase, 0, 0, 0)
            cbase += p.ncoef
    coefs = b"".join(coef_parts) + b"\0" * 64
    return recs, coefs, pics, rec_bytes * S, nslots


def upload(eng, packed):
    """pack() output into HBM of the engine's GPU (engine-scoped allocations:
    a rank's buffers live on its own device whatever the thread's current
    HIP device is); returns (d_recs, d_coef, resident bytes)."""
    recs, coefs = packed[0], packed[1]
    d_recs = eng.alloc(len(recs))
    d_coef = eng.alloc(len(coefs))
    rb = (C.c_char * len(recs)).from_buffer(recs)
    eng.upload(d_recs, rb, len(recs))
    eng.upload(d_coef, coefs, len(coefs))
    return d_recs, d_coef, len(recs) + len(coefs)


def slots_read(recs, nmbs, i):
    """DPB slots the inter MBs of packed picture i read (MbRec.ref, bytes
    24..27 of each 96-B record; MBT_INTER = 0, MBT_SKIP = 1)."""
    r = np.frombuffer(recs, dtype=np.uint8, count=nmbs * MBREC, offset=i * nmbs * MBREC).reshape(nmbs, MBREC)
    inter = r[:, 0] <= 1
    return set(np.unique(r[inter, 24:28]).tolist())


def rename_slots(recs, pics, S, nmbs, nslots, P=2):
    """Physical frame slots for frame-pipelined launches of P steps: the
    host parser's DPB slot d of a stream maps to one of nphys >= nslots +
    P - 1 physical slots, and a picture decoded into d gets the physical
    slot released longest ago -- P - 1 pictures ago at the latest, so none
    of the P - 1 pictures before it in its launch still reads it (e.g. the
    reference the sliding window just dropped) or writes it.  The streams
    are decoded cyclically (picture 0, an IDR, after the last), so the
    launches across the wrap must qualify too: nphys grows from nslots +
    P - 1 until they do (a sliding-window DPB assigns the slots round robin:
    configs[3]'s 60-picture GOP with 5 DPB slots takes 6 for P = 2, 10 for P
    = 3 and 4).  The mapping is a bijection at every picture, so the
    records' reference-slot comparisons (bS) are unchanged; MbRec.ref and
    PicDesc cur_slot / frame_base are rewritten in place.  Returns the
    physical slot count."""
    n = len(pics) // S
    arr = np.frombuffer(recs, dtype=np.uint8).reshape(-1, MBREC)
    refs = [[slots_read(recs, nmbs, k * S + s) for k in range(n)] for s in range(S)]

    def assign(s, nphys):
        cur, free = {}, list(range(nphys))    # DPB slot -> physical; released order, oldest first
        luts, phs = [], []
        for k in range(n):
            luts.append(dict(cur))
            d = int(pics[k * S + s][2])
            old = cur.get(d)
            ph = next(x for x in free if x != old)
            free.remove(ph)
            if old is not None:
                free.append(old)
            cur[d] = ph
            phs.append(ph)
        reads = [{luts[k].get(x, x) for x in refs[s][k]} for k in range(n)]
        ok = all(phs[(k + i) % n] != phs[(k + m) % n] and phs[(k + i) % n] not in reads[(k + m) % n]
                 for k in range(n) for i in range(1, P) for m in range(i))
        return ok, luts, phs

    for nphys in range(nslots + P - 1, nslots + P + 15):
        plan = [assign(s, nphys) for s in range(S)]
        if all(ok for ok, _, _ in plan):
            break
    for s, (_, luts, phs) in enumerate(plan):
        for k in range(n):
            i = k * S + s
            lut = np.arange(256, dtype=np.uint8)
            for d, ph in luts[k].items():
                lut[d] = ph
            r = arr[i * nmbs:(i + 1) * nmbs]
            inter = r[:, 0] <= 1
            r[inter, 24:28] = lut[r[inter, 24:28]]
            pics[i][1] = s * nphys
            pics[i][2] = phs[k]
    return nphys


def far_rows(recs, npics, w, h):
    """Per picture: the fraction of its MB rows holding an inter MB whose
    motion reaches far from it -- 2 or more MB rows down or 8 or more MB
    columns right (a window clamped to the bottom or right picture edge
    included).  In a frame-pipelined launch such an MB waits for its
    producer's last rows or a whole row, so (MB row, MB column) waits gain
    nothing over whole-row waits, which keep the later pictures' rows idle
    meanwhile (tools/dep_sim.py)."""
    r = np.frombuffer(recs, dtype=np.uint8).reshape(npics, h * w, MBREC)
    inter = r[:, :, 0] <= 1
    mv = r[:, :, 28:92].copy().view("<i2").reshape(npics, h * w, 16, 2)
    far = inter & (((mv[..., 1] >> 2) >= 32) | ((mv[..., 0] >> 2) >= 128)).any(axis=2)
    return far.reshape(npics, h, w).any(axis=2).mean(axis=1)


def schedule(recs, pics, S, nmbs, warmup, steps, P):
    """Launches as (first step, steps in it).  P > 1 groups steps (Pi ..
    Pi+P-1) when every group meets the engine's frame-pipelined batch
    contract (batch_ok); otherwise, or when warmup / steps are not multiples
    of P, every launch is one step."""
    n = warmup + steps
    if P > 1 and warmup % P == 0 and steps % P == 0:
        if all(batch_ok(recs, pics, S, nmbs, range(k0, k0 + P)) for k0 in range(0, n, P)):
            return [(k, P) for k in range(0, n, P)]
    return [(k, 1) for k in range(n)]


def batch_ok(recs, pics, S, nmbs, ks):
    """The engine's frame-pipelined batch contract for one launch of the
    pictures ks (in step order) of every stream: no picture writes the slot
    an earlier one of the launch writes or reads."""
    ks = list(ks)
    for s in range(S):
        for i, kb in enumerate(ks[1:], 1):
            b = kb * S + s
            for ka in ks[:i]:
                a = ka * S + s
                if pics[a][2] == pics[b][2] or pics[b][2] in slots_read(recs, nmbs, a):
                    return False
    return True


def golden_frames(config, seed, overrides):
    """The reference decoder's per-frame MD5s of generator stream (config,
    seed, overrides) when a fixture covers it (the fixture's overrides other
    than nframes equal to `overrides`; the longest such fixture)."""
    gold = os.path.join(ROOT, "tests", "golden", "golden.json")
    if not os.path.exists(gold):
        return None
    want = {k: v for k, v in (overrides or {}).items() if k != "nframes"}
    best = None
    for c in json.load(open(gold))["cases"].values():
        ov = {k: v for k, v in c["overrides"].items() if k != "nframes"}
        if c["config"] == config and c["seed"] == seed and ov == want \
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
    launch = lambda: L.h264mi_yuv2rgba_device_pitch(base, out.data_ptr(), width, height, eng.chroma_pitch, S, stride,
                                                    width * height * 4,
                                              st.cuda_stream)
    for _ in range(5):
        assert launch() == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        launch()
    e1.record(st)
    e1.synchronize()
    us_warm = e0.elapsed_time(e1) * 1e3 / reps
    # cold input: before each timed launch a 512 MB scratch write evicts the
    # I420 pictures from the 256 MB MALL (and the L2s), so the launch reads
    # them from HBM; HIP events bracket the launch alone
    scratch = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
    cold = []
    for _ in range(max(reps // 5, 5)):
        scratch.fill_(1)
        a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a0.record(st)
        launch()
        a1.record(st)
        cold.append((a0, a1))
    torch.cuda.synchronize()
    us = sum(x.elapsed_time(y) for x, y in cold) * 1e3 / len(cold)
    del scratch
    alg = S * width * height * (1.5 + 4)
    gbs = alg / (us * 1e-6) / 1e9
    gbs_warm = alg / (us_warm * 1e-6) / 1e9
    del out
    return {"kernel": "k_yuv2rgba", "pictures_per_launch": S, "avg_launch_us": round(us, 2),
            "frames_per_s": round(S / (us * 1e-6), 1), "alg_bytes_per_launch": int(alg),
            "achieved_GBs": round(gbs, 1), "peak": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4),
            "input": "cold: the I420 pictures evicted from the MALL before every timed launch (512 MB "
                     "scratch write), so both the 1.5 B/pixel read and the 4 B/pixel RGBA write are HBM bytes",
            "warm_mall": {"avg_launch_us": round(us_warm, 2), "achieved_GBs": round(gbs_warm, 1),
                          "note": "back-to-back launches over the same pictures: the I420 input is served from "
                                  "the 256 MB MALL, so this rate is not an HBM fraction"},
            "semantics": "per pixel DecoderPost.js yuv2rgbcalc (:514-560), RGBA bytes; output written with "
                         "non-temporal stores"}


def parse_cpulist(text: str):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]"""
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def format_cpulist(cpus) -> str:
    """[0, 1, 2, 3, 8] -> '0-3,8'"""
    cpus, parts, i = sorted(set(cpus)), [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        parts.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(parts)


def gpu_numa_node(torch, dev: int) -> int:
    """NUMA node of HIP device `dev`, from sysfs of its PCI function; -1 when
    unknown (no GPU, no sysfs entry)."""
    try:
        pr = torch.cuda.get_device_properties(dev)
        path = f"/sys/bus/pci/devices/{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0/numa_node"
        with open(path) as f:
            return int(f.read().strip())
    except (OSError, ValueError, AttributeError, RuntimeError, AssertionError):
        return -1


def node_cpus(node: int):
    """Host cores of NUMA node `node` (sysfs), or None."""
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            return parse_cpulist(f.read())
    except (OSError, ValueError):
        return None


def l3_groups(cpus):
    """`cpus` split by last-level cache (sysfs cache/index3 shared_cpu_list;
    an EPYC CCD): a decoder process whose threads share one L3 hands the
    speculative workers' records and coefficients to its calling thread
    without crossing the fabric.  Falls back to one group."""
    groups, seen = [], set()
    for c in sorted(cpus):
        if c in seen:
            continue
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
                g = sorted(set(parse_cpulist(f.read())) & set(cpus))
        except (OSError, ValueError):
            return [sorted(cpus)]
        seen.update(g)
        groups.append(g)
    return groups or [sorted(cpus)]


def process_cpus(cpus, nprocs):
    """Each end-to-end decoder process's core set: its own L3 domain when the
    share has at least one per process (round-robin over the domains), else
    the whole share."""
    groups = [g for g in l3_groups(cpus) if len(g) >= 2]
    if len(groups) >= nprocs:
        return [groups[i] for i in range(nprocs)]
    return [sorted(cpus)] * nprocs


def e2e_core_plan(local: int, numa, allowed):
    """Host cores for each local rank's end-to-end decoder processes
    (each GPU has its own host parse threads on a NUMA-local core
    set): rank j gets an equal, disjoint share of the cores it may use on its
    GPU's NUMA node (numa[j], -1 = unknown), split among the local ranks whose
    GPUs sit on that node; a node without usable cores falls back to an equal
    share of every allowed core.  Returns (this rank's cores, the plan of
    every local rank)."""
    allowed = sorted(set(allowed))
    plan = []
    for j, n in enumerate(numa):
        pool = None
        if n >= 0:
            nc = node_cpus(n)
            pool = sorted(set(nc) & set(allowed)) if nc else None
            peers = [k for k, m in enumerate(numa) if m == n]
        if not pool:
            pool, peers = allowed, list(range(len(numa)))
        k, m = peers.index(j), len(peers)
        share = len(pool) // m
        plan.append(pool[k * share:(k + 1) * share] if share else pool[k % len(pool):k % len(pool) + 1])
    return plan[local], plan


def end_to_end(streams, nframes, reps=E2E_REPS, device=0, cpus=None, max_procs=MAX_E2E_PROCS, release=None):
    """End-to-end decode through the product C-ABI: one
    broadway_amd/lib/h264mi_dec process per stream (at most MAX_E2E_PROCS),
    all in parallel (one host thread each), each decoding its stream `reps`
    times -- host CAVLC parse, H2D of the MB records, k_prep + k_wgpp, D2H of
    every output picture.  Rate = all pictures / the slowest process's decode
    time (HIP start-up of each process excluded; it is paid before its timed
    loop).  Start gate (h264mi_dec -G): every process reports ready after its
    warm-up and all are released at once; the rate divides all pictures by
    the union of the processes' decode windows (CLOCK_MONOTONIC, earliest
    start to latest end), so start-up skew cannot inflate it.  The processes
    decode on GPU `device` (H264MI_DEVICE) and, given `cpus`, run pinned to
    those host cores (h264mi_dec -A: the process and every thread it
    starts).  `release`, if given, is called once every local process is
    ready and before they are released (the ranks' barrier: all GPUs' decoder
    processes start together)."""
    from broadway_amd import _lib
    exe = os.path.join(_lib.LIB_DIR, "h264mi_dec")      # H264MI_LIB_DIR: an A/B build's
    if not os.path.exists(exe):
        return None
    streams = streams[:max_procs]
    # a thread waiting for the GPU sleeps instead of spinning: the host cores
    # are the bound on this path (tools/e2e_env_sweep.sh: 1.89k -> 2.08k fps)
    env = dict(os.environ)
    env.setdefault("H264MI_BLOCKING_SYNC", "1")
    # 8 decoder processes, each pinned to one L3 domain (process_cpus): the
    # calling thread plus 3 slice workers each -- with the workers on their
    # caller's L3, a fourth parse thread keeps the box's 16-core share busy
    # (profiles/r154_e2e_threads.txt: 15.6 vs 13.4 cores, 3.55k vs 3.09k
    # fps; r153: L3 pinning 3.51k fps at 4.13 ms vs 3.31k at 4.41 unpinned
    # within the NUMA share; round 3's r51 had 2 workers better unpinned)
    env.setdefault("H264MI_PARSE_THREADS", "3")
    env["H264MI_DEVICE"] = str(device)
    # each process on one L3 domain of the share (E2E_L3=0: the whole share)
    per_proc = process_cpus(cpus, len(streams[:max_procs])) if cpus and os.environ.get("E2E_L3", "1") == "1" \
        else [cpus] * len(streams[:max_procs])
    td = tempfile.mkdtemp(prefix="h264e2e")
    try:
        procs = []
        for i, s in enumerate(streams):
            pth = os.path.join(td, f"s{i}.h264")
            with open(pth, "wb") as f:
                f.write(s)
            pin = [f"-A{format_cpulist(per_proc[i])}"] if per_proc[i] else []
            procs.append(subprocess.Popen([exe, "-Onone", f"-r{reps}", "-T", "-G"] + pin + [pth], stdin=subprocess.PIPE,
                                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
        # start gate: wait until every process has warmed up, then release all.
        # The ranks' barrier (release) is reached on every path, a failed
        # warm-up included, so that no other rank waits in it forever
        failed = None
        for pr in procs:
            line = pr.stdout.readline()
            if line.strip() != "ready":
                failed = (pr, line)
                break
        if release is not None:
            release()
        if failed is not None:
            for pr in procs:
                if pr.poll() is None:
                    pr.kill()
            pr, line = failed
            pr.wait(timeout=60)
            raise RuntimeError(f"h264mi_dec not ready: {line!r} {pr.stderr.read().strip()[-300:]}")
        for pr in procs:
            pr.stdin.write("g")
            pr.stdin.flush()
        secs, pics, parts, cpu_s, sys_s, starts, ends = [], 0, {}, 0.0, 0.0, [], []
        threads = {}
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
                elif f[0] == "t_start_mono":
                    starts.append(float(f[1]))
                elif f[0] == "t_end_mono":
                    ends.append(float(f[1]))
                elif f[0].startswith("t_") and len(f) > 1:
                    parts[f[0]] = parts.get(f[0], 0.0) + float(f[1])
                elif f[0] == "cpu_seconds":
                    cpu_s += float(f[1])
                elif f[0] == "cpu_sys_seconds":
                    sys_s += float(f[1])
                elif f[0] in ("cpu_decode_threads_seconds", "cpu_spec_workers_seconds", "cpu_other_live_threads_seconds"):
                    threads[f[0]] = threads.get(f[0], 0.0) + float(f[1])
        # the union of the decode windows: all processes released together
        t = max(ends) - min(starts) if starts and ends else max(secs)
        res = {"value": round(pics / t, 2), "unit": "frames/s", "host_threads": len(streams),
               "pictures": pics, "seconds": round(t, 6), "device": device,
               "window": "union of the processes' decode windows after a common start gate",
               "start_skew_ms": round((max(starts) - min(starts)) * 1e3, 3) if starts else None,
               "t_start_mono": min(starts) if starts else None, "t_end_mono": max(ends) if ends else None,
               "longest_single_window_s": round(max(secs), 6),
               "host_cores_assigned": len(cpus) if cpus else None,
               "cpus": format_cpulist(cpus) if cpus else None,
               "per_process_cpus": [format_cpulist(x) for x in per_proc] if cpus else None,
               "sample": f"{len(streams)} x {nframes}-frame 1080p streams x {reps} passes, one h264mi_dec process "
                         f"(H264SwDec* C-ABI) per stream: host parse + H2D + kernels + D2H of every picture; "
                         f"{pics} frames in {t:.2f} s"}
        if parts and pics:
            # per picture inside one decoder process (H264SwDecGetTiming):
            # host parse / record upload + launch / wait for the GPU / D2H copy
            res["per_picture_ms"] = {k[2:]: round(v * 1e3 / pics, 3) for k, v in sorted(parts.items())}
            res["parse_threads_per_process"] = 1 + int(env["H264MI_PARSE_THREADS"])
            res["host_sync"] = "blocking" if env["H264MI_BLOCKING_SYNC"] == "1" else "spin"
            # host CPU time (all threads of all processes) per picture, and the
            # cores that keeps busy at the measured rate
            res["host_cpu_ms_per_picture"] = round(cpu_s * 1e3 / pics, 3)
            res["host_sys_ms_per_picture"] = round(sys_s * 1e3 / pics, 3)   # of which in the kernel (HIP ioctls, page pinning)
            res["host_cores_busy"] = round(cpu_s / t, 2)
            if threads:
                # where the host CPU goes (ms per picture): the calling
                # (decoding) threads -- parse, submit, waits -- the
                # speculative-parse workers, the other threads alive in the
                # process (HIP runtime), and what none of these covers
                dec = threads.get("cpu_decode_threads_seconds", 0.0)
                spec = threads.get("cpu_spec_workers_seconds", 0.0)
                oth = threads.get("cpu_other_live_threads_seconds", 0.0)
                res["host_cpu_by_thread_ms_per_picture"] = {
                    "decoding_threads": round(dec * 1e3 / pics, 3),
                    "spec_parse_workers": round(spec * 1e3 / pics, 3),
                    "hip_runtime_and_other_threads": round(oth * 1e3 / pics, 3),
                    "unattributed": round((cpu_s - dec - spec - oth) * 1e3 / pics, 3)}
        # the same streams in ONE process, one thread (H264SwDec instance) per
        # stream, sharing one batched engine (h264mi_set_share, -S)
        paths = [os.path.join(td, f"s{i}.h264") for i in range(len(streams))]
        o = subprocess.run([exe, "-Onone", f"-r{max(1, reps // 3)}", "-T", f"-S{len(streams)}"] + pin + paths,
                           capture_output=True,
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


def load_ubench():
    """Lone-wave chain costs from the committed micro-benchmark
    (tools/ubench/ubench_deblock.hip's JSON line -> profiles/ubench.json), or
    None."""
    p = os.path.join(ROOT, "profiles", "ubench.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def load_dep_floor(cfg, streams, steps, gen):
    """The data-dependent launch floor (tools/dep_sim.py with the lone-wave
    costs -> profiles/dep_floor.json) when this run's workload is the one it
    simulated, else None."""
    p = os.path.join(ROOT, "profiles", "dep_floor.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    wl = d.get("workload", {})
    if (wl.get("config"), wl.get("streams"), wl.get("steps_per_launch")) != (cfg, streams, steps) or gen or wl.get("gen_overrides"):
        return None
    return d


def latency_floor(w_mbs, h_mbs, steps, ub, launch_us, dep=None):
    """The row chain's latency floor, beside the HBM
    roofline: a picture cannot finish before its last row has run W MBs of
    lone-wave vertical + horizontal passes after H - 1 row-to-row hand-offs,
    each the patch edge plus one granule hop; a later picture of a
    frame-pipelined launch trails the earlier one by at least two row lags
    and one 128-B line of MB columns plus the store-progress lag (8 MBs).
    The floor is per launch (the S streams' pictures run side by side);
    `frac` = floor / the measured launch time."""
    if not ub:
        return None
    mb = ub["vh_us"]
    lag = ub["patch_us"] + min(ub["hop_same_xcd_us"], ub["hop_other_xcd_us"])
    pic = w_mbs * mb + (h_mbs - 1) * lag
    trail = 2 * lag + 8 * mb
    floor = pic + (steps - 1) * trail
    return {"model": "W x (V+H) + (H-1) x (patch + hop) per picture, + (P-1) x (2 row lags + 8 MB periods) "
                     "per frame-pipelined launch",
            "per_mb_vh_us": round(mb, 4), "row_lag_us": round(lag, 4),
            "picture_floor_us": round(pic, 2), "step_trail_us": round(trail, 2),
            "launch_floor_us": round(floor, 2), "steps_per_launch": steps,
            "measured_launch_us": round(launch_us, 2),
            "frac": round(floor / launch_us, 4) if launch_us else None,
            "source": ub.get("source", "profiles/ubench.json"),
            # the same lone-wave costs with this workload's own data
            # dependencies between the pictures of a launch (a later picture's
            # MBs wait for the reference rows their windows read)
            "data_dependent_launch_floor_us": dep["launch_us"]["row"] if dep else None,
            "data_dependent_frac": round(dep["launch_us"]["row"] / launch_us, 4) if dep and launch_us else None,
            "data_dependent_source": "profiles/dep_floor.json (tools/dep_sim.py, rows rule, lone-wave period and lag)"
            if dep else None}


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


GOP = 60                   # configs[3]: 1 I + 59 P per GOP; the bench streams are one GOP long


def gop_phases(S: int, gop: int = GOP, step: int = 1, offset: int = None, warmup: int = 0):
    """GOP phase of each stream: stream s is s*gop/S pictures into its GOP
    when the first warmup step starts, so the S streams' IDR pictures are
    spread evenly over the steps (independent streams that did not start
    together) and every window of `gop` steps reconstructs S I pictures out
    of S*gop -- the configs[3] mix of 1 I per 60 in every step window, not
    only in the one step that happens to hold picture 0.  step = P (frame-
    pipelined launches of P pictures per stream): phases are multiples of
    P plus `offset`.  The default, (1 - warmup) mod P (BENCH_IDR_FIRST=1:
    -warmup mod P), puts a stream's IDR last in its launch (launches start
    at warmup mod P): with P = 2 and an even warmup every pair is (odd k,
    k + 1) -- (picture gop-1, picture 0): pictures that do not depend on
    each other -- instead of the IDR first, whose successors in the same
    launch would wait on its whole deblocking chain."""
    if offset is None:
        first = os.environ.get("BENCH_IDR_FIRST") == "1"
        offset = 0 if step == 1 else ((0 if first else 1) - warmup) % step
    return [((s * gop) // S) // step * step + offset for s in range(S)]


def launch_plan(N: int, S: int, warmup: int, steps: int, phases=None, sched=None, P: int = 1):
    """Per launch, per step of the launch, the picture index of each stream;
    returns (launches, pre-roll launch count).

    phases None: launches follow `sched` ((first step, steps) pairs), stream
    s decodes picture k at step k.  Otherwise warmup step v (then timed step
    v - warmup) decodes picture (v + phases[s]) % N of stream s: a stream of
    N pictures starting with its IDR is decoded cyclically -- after picture
    N-1 comes picture 0 again, an IDR (no reference is read across it), so
    the pictures and MD5s are the stream's own -- P steps per launch.  An
    untimed pre-roll of max(phases) one-step launches first brings stream s
    to picture phases[s]: its pictures 0 .. phases[s]-1 in order, preceded
    by repeats of the IDR picture 0 (which reads no reference, so repeating
    it is idempotent)."""
    if phases is None:
        return [[[k] * S for k in range(k0, k0 + P)] for k0, P in sched], 0
    R = max(phases)
    pre = [[[max(0, u - R + ph) for ph in phases]] for u in range(R)]
    # P-step launches aligned to the timed window's start: warmup % P single
    # steps first, a shorter launch last when steps % P != 0
    main, v = [], 0
    while v < warmup + steps:
        n = 1 if v < warmup % P else min(P, warmup + steps - v)
        main.append([[(v + j + ph) % N for ph in phases] for j in range(n)])
        v += n
    return pre + main, R


def pairs_ok(recs, pics, S, nmbs, N, P, first=0):
    """The engine's frame-pipelined batch contract (batch_ok) for launches
    of P consecutive pictures k .. k+P-1 (k = first, first + P, ...,
    cyclically: with P = 2 the pair (N-1, 0) included) of every stream."""
    return all(batch_ok(recs, pics, S, nmbs, [(k + i) % N for i in range(P)]) for k in range(first, N, P))


class _DryEngine:
    """--dry-run stand-in for broadway_amd.engine.Engine: no device calls;
    allocations are fake addresses that remember the device they were asked
    for (the gloo test checks every rank's buffers name its own GPU)."""

    def __init__(self, w=0, h=0, S=0, nslots=0, device=0):
        self.launches = 0
        self.device = device
        self._next = 1 << 40
        self.alloc_dev = {}

    def alloc(self, n):
        p = self._next
        self._next += (int(n) + 4095) & ~4095
        self.alloc_dev[p] = self.device
        return p

    def free(self, p):
        self.alloc_dev.pop(p, None)

    def upload(self, *a):
        pass

    def pointer_device(self, p):
        return self.alloc_dev.get(p, -1)

    def hint_intra(self, *a):
        pass

    def decode_device_steps(self, *a):
        self.launches += 1

    def set_steps(self, *a):
        pass

    def decode_device_steps_next(self, *a):
        self.launches += 1
        return True

    def sync(self):
        pass

    def set_timing(self, *a, **k):
        pass

    def timing_report(self):
        return 0.0, 0.0, 0

    def timing_list(self, cap=4096):
        return []

    def errors(self):
        return 0

    def kernel_name(self):
        return "dry-run"

    def read(self, *a):
        return np.zeros(1, np.uint8)

    def close(self):
        pass


class DeviceRun:
    """The bench's device-resident path for one rank: the engine for its S
    streams on its own GPU (`device`), every picture's records, coefficient
    blocks and descriptors in that GPU's HBM (engine-scoped allocations,
    placement asserted per buffer), and a launch plan (launch_plan: GOP
    phases, or P steps per launch with physical slots renamed for P > 1; the
    next launch's k_prep runs in each launch's tail).  dry: no device calls."""

    def __init__(self, L, caps, warmup, steps, pipe=1, device=0, dry=False, phases=None):
        from broadway_amd.engine import Engine
        self.L, self.S, self.caps = L, len(caps), caps
        S = self.S
        w, h = caps[0].w_mbs, caps[0].h_mbs
        self.nmbs = nmbs = w * h
        self.N = N = min(c.npics for c in caps)
        self.device = device
        packed = pack(caps, N)
        recs_h, _, pics_h, _, nslots = packed
        self.sched = None
        if pipe > 1:
            nslots = rename_slots(recs_h, pics_h, S, nmbs, nslots, pipe)
        if phases is None:
            if warmup + steps > N:
                raise ValueError(f"{warmup}+{steps} steps but the streams hold {N} pictures")
            self.sched = schedule(recs_h, pics_h, S, nmbs, warmup, steps, pipe)
            self.P = self.sched[0][1]
        else:
            # frame-pipelined GOP plan: P-aligned phases, an even GOP, P-aligned
            # warmup / steps and every (k, k+1) pair within the batch contract
            # pairs (k, k + 1) start where the timed window does: k = warmup +
            # phase (mod 2) -- one parity for every stream, N even so that the
            # cyclic pair (N - 1, 0) keeps it
            par = (warmup + phases[0]) % pipe if pipe > 1 else 0
            ok = (pipe > 1 and N % pipe == 0 and all(ph % pipe == phases[0] % pipe for ph in phases) and
                  pairs_ok(recs_h, pics_h, S, nmbs, N, pipe, par))
            self.P = pipe if ok else 1
        self.nslots = nslots
        self.pics_h, self.recs_h = pics_h, recs_h
        self.slot_of = pics_h[:, 2].reshape(N, S).copy()
        self.is_i = [[c.pictures[k].n_inter == 0 for c in caps] for k in range(N)]
        # per picture k of stream s: rows with far-reaching motion (far_rows)
        self.far = far_rows(recs_h, N * S, w, h).reshape(N, S)
        # frame-pipelined launches' dependency mode: BENCH_DEP_MODE=rows|cols
        # forces one; by default whole rows when a later picture of the
        # launch has far-reaching motion in over a quarter of its rows
        self.dep_force = {"rows": 1, "cols": 2}.get(os.environ.get("BENCH_DEP_MODE", ""), 0)
        self.eng = _DryEngine(device=device) if dry else Engine(w, h, S, nslots, device=device)
        if self.P > 1:
            self.eng.set_steps(self.P)
        self.d_recs, self.d_coef, self.resident = upload(self.eng, packed)
        self.bufs = [self.d_recs, self.d_coef]
        self.d_desc = 0
        self.set_plan(warmup, steps, phases)

    def set_plan(self, warmup, steps, phases=None):
        """(Re)build the launch plan and its descriptor table in HBM (each
        launch's steps step-major, launches back to back)."""
        S, P = self.S, self.P
        self.warmup, self.steps, self.phases = warmup, steps, phases
        if phases is not None and P > 1 and not all(ph % P == phases[0] % P for ph in phases):
            raise ValueError(f"phases {phases}: not all of one parity")
        if phases is not None and P > 1 and not pairs_ok(self.recs_h, self.pics_h, S, self.nmbs, self.N, P,
                                                         (warmup + phases[0]) % P):
            raise ValueError(f"phases {phases}: a pair of consecutive pictures breaks the batch contract")
        self.launches, self.n_pre = launch_plan(self.N, S, warmup, steps, phases, self.sched, P)
        if self.sched:
            self.n_warm = self.n_pre + sum(1 for k0, _ in self.sched if k0 < warmup)
        else:
            # GOP plan, P > 1: a launch splits after every step holding an
            # IDR that is not its last -- in the same launch, the IDR's own
            # next picture waits on the IDR's deblocking chain, the launch's
            # longest (r72 A/B, P = 2: 809 us against 434 + 325 us split).
            # With the default phases an IDR is always a launch's last
            # picture, and nothing splits.
            main, warm, v = [], 0, 0
            for x in self.launches[self.n_pre:]:
                parts, cur = [], []
                for st in x:
                    cur.append(st)
                    if self.holds_idr([st]):
                        parts.append(cur)
                        cur = []
                if cur:
                    parts.append(cur)
                main += parts
                warm += len(parts) if v < warmup else 0
                v += len(x)
            self.launches = self.launches[:self.n_pre] + main
            self.n_warm = self.n_pre + warm
        self.desc_off = np.cumsum([0] + [len(x) * S * 32 for x in self.launches]).tolist()
        d = np.zeros((sum(len(x) for x in self.launches) * S, 8), dtype=np.uint32)
        row = 0
        for launch in self.launches:
            for step in launch:
                for s, k in enumerate(step):
                    d[row + s] = self.pics_h[k * S + s]
                row += S
        if self.d_desc:
            self.eng.free(self.d_desc)
            self.bufs.remove(self.d_desc)
        self.d_desc = self.eng.alloc(d.nbytes)
        self.bufs.append(self.d_desc)
        self.eng.upload(self.d_desc, d.ctypes.data, d.nbytes)

    def holds_idr(self, launch):
        """Does one of the launch's pictures read no reference (I picture)."""
        return any(self.is_i[k][s] for step in launch for s, k in enumerate(step))

    def placement(self):
        """Device of every HBM buffer of this run: [(name, device)]."""
        names = ["records", "coefficients", "descriptors"]
        return [(n, self.eng.pointer_device(p)) for n, p in zip(names, self.bufs)]

    def launch(self, i):
        """Launch i of the plan: its steps (1 or P) of the S streams; the next
        launch's k_prep runs in this one's tail workgroups (over the next
        launch's own step count)."""
        S = self.S
        P = len(self.launches[i])
        desc = self.d_desc + self.desc_off[i]
        # the launch's shape hint: does it hold an intra-heavy picture
        self.eng.hint_intra(any(2 * self.caps[s].pictures[k].n_intra > self.nmbs
                                for step in self.launches[i] for s, k in enumerate(step)))
        if P > 1 and hasattr(self.eng, "hint_deps"):
            self.eng.hint_deps(self.dep_mode(i))
        if i + 1 < len(self.launches):
            nd, nP = self.d_desc + self.desc_off[i + 1], len(self.launches[i + 1])
            if nP == P:
                self.eng.decode_device_steps(S, P, self.d_recs, self.d_coef, desc, self.d_recs, self.d_coef, nd)
            elif not self.eng.decode_device_steps_next(S, P, self.d_recs, self.d_coef, desc,
                                                       self.d_recs, self.d_coef, nd, nP):
                self.eng.decode_device_steps(S, P, self.d_recs, self.d_coef, desc)
        else:
            self.eng.decode_device_steps(S, P, self.d_recs, self.d_coef, desc)

    def dep_mode(self, i):
        """Dependency mode of launch i (1 whole rows, 2 (row, column) cells)."""
        if self.dep_force:
            return self.dep_force
        far = max((self.far[k][s] for step in self.launches[i][1:] for s, k in enumerate(step)), default=0.0)
        return 1 if far > 0.25 else 2

    def timed_pictures(self):
        """(stream, picture) of every picture the timed launches decode."""
        return [(s, k) for launch in self.launches[self.n_warm:] for step in launch for s, k in enumerate(step)]

    def verify(self, refs):
        """Untimed re-run of the whole plan, every picture compared with the
        reference decoder's MD5 (refs[s][k]; POC type 2: output order ==
        decode order) right after its launch (the pictures of one launch
        write distinct slots).  Pre-roll repeats of the IDR are checked once.
        Returns (ok, frames checked in warmup + timed, frames without a
        fixture, pre-roll frames checked)."""
        ok, n, missing, n_pre = True, 0, 0, 0
        last = [None] * self.S
        for i, launch in enumerate(self.launches):
            self.launch(i)
            self.eng.sync()
            for step in launch:
                for s, k in enumerate(step):
                    pre = i < self.n_pre
                    if pre and last[s] == k:
                        continue
                    last[s] = k
                    if refs[s] is None or k >= len(refs[s]):
                        missing += 0 if pre else 1
                        continue
                    got = hashlib.md5(self.eng.read(s, int(self.slot_of[k][s])).tobytes()).hexdigest()
                    if pre:
                        n_pre += 1
                    else:
                        n += 1
                    ok &= got == refs[s][k]
        return ok, n, missing, n_pre

    def check_resident(self, refs):
        """After the plan ran: every frame slot still holds the last picture
        the plan decoded into it -- compare those (the timed launches' own
        output, not a re-run) with the reference MD5s.  Returns (ok, n)."""
        last = {}
        for launch in self.launches:
            for step in launch:
                for s, k in enumerate(step):
                    last[(s, int(self.slot_of[k][s]))] = k
        ok, n = True, 0
        for (s, slot), k in sorted(last.items()):
            if refs[s] is None or k >= len(refs[s]):
                continue
            ok &= hashlib.md5(self.eng.read(s, slot).tobytes()).hexdigest() == refs[s][k]
            n += 1
        return ok, n

    def close_engine(self):
        if self.eng is not None:
            for p in self.bufs:
                self.eng.free(p)
            self.bufs = []
            self.eng.close()
            self.eng = None

    def free(self):
        self.close_engine()


def timed_run(run, dist, torch, sync, stride=1):
    """Pre-roll + warmup launches untimed, then the timed launches bracketed
    by a barrier and device syncs; HIP events on every stride-th timed
    launch (default: every one), carried by k_wgpp's own dispatch packet.
    Returns (wall seconds max over ranks, avg k_wgpp us of the sampled
    launches, sampled launch indices, per-launch us of those launches)."""
    for i in range(run.n_warm):
        run.launch(i)
    run.eng.sync()
    sync()
    ntimed = len(run.launches) - run.n_warm
    run.eng.set_timing(ntimed, stride=stride)
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(run.n_warm, len(run.launches)):
        run.launch(i)
    run.eng.sync()
    sync()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    dt = max_over_ranks(dist, torch, t1 - t0)
    per = run.eng.timing_list(ntimed) or []
    _, us, nb = run.eng.timing_report()
    sampled = [run.n_warm + j for j in range(0, ntimed, stride)][:nb]
    return dt, us / max(nb, 1), sampled, per


def launch_split(run, sampled, per):
    """Sampled launches split by whether one of their pictures is an IDR
    (I picture): {"i": (n, avg us, avg us per step), "p": (...)}."""
    out = {}
    for key, want in (("i", True), ("p", False)):
        v = [(u, len(run.launches[i])) for i, u in zip(sampled, per) if run.holds_idr(run.launches[i]) == want]
        us = sum(u for u, _ in v)
        out[key] = (len(v), round(us / len(v), 2) if v else None,
                    round(us / sum(n for _, n in v), 2) if v else None)
    return out


def alg_bytes(run, launch_ids):
    """SURVEY §8d R_alg of the listed launches: MC reference footprint +
    32 B per coded 4x4 block + 96-B MB record, per picture."""
    tot = 0
    for i in launch_ids:
        for step in run.launches[i]:
            for s, k in enumerate(step):
                p = run.caps[s].pictures[k]
                tot += p.alg_ref_bytes + 32 * p.n_coded + MBREC * run.nmbs
    return tot


def ref_line_bytes(run, launch_ids):
    """The listed launches' reference footprint in whole 128-B lines (per
    picture: distinct lines of each reference slot its MC windows touch,
    h264mi_capture_ref_lines): the line-granular, compulsory part of the
    reference reads, beside R_alg's bytes used.  With 4 reference frames per
    stream it is close to 4 whole frames per picture."""
    tot = 0
    for i in launch_ids:
        for step in run.launches[i]:
            for s, k in enumerate(step):
                tot += run.caps[s].pictures[k].ref_line_bytes
    return tot


def run_leg(L, torch, config, seeds, steps, warmup, mc_waves=3, rpw=0, overrides=None, pipe=1, dep=""):
    """One single-GPU measurement of another SURVEY §8d config with the same
    step structure (records resident in HBM, one k_wgpp launch per step --
    `pipe` > 1: that many aligned steps per launch, dependency mode `dep`
    forced or per launch by far_rows -- HIP events on every launch) and the
    same untimed verification against the reference MD5s.  Returns a dict
    for the bench line."""
    nframes = warmup + steps
    streams, caps = prepare(config, seeds, nframes, overrides)
    assert all(c.errors == 0 and c.npics >= nframes for c in caps), "leg stream preparation failed"
    S = len(caps)
    w, h = caps[0].w_mbs, caps[0].h_mbs
    # both knobs are read once, when the engine is created; mc_waves 0: the
    # engine's own per-launch choice (engine.hip launch_nmc)
    if pipe == 1 and mc_waves:
        os.environ["H264MI_MC_WAVES"] = str(mc_waves)
    if rpw:
        os.environ["H264MI_RPW"] = str(rpw)
    saved_dep = os.environ.get("BENCH_DEP_MODE")
    if dep:
        os.environ["BENCH_DEP_MODE"] = dep
    try:
        run = DeviceRun(L, caps, warmup, steps, pipe, device=torch.cuda.current_device())
    finally:
        os.environ.pop("H264MI_MC_WAVES", None)
        os.environ.pop("H264MI_RPW", None)
        if dep:
            if saved_dep is None:
                os.environ.pop("BENCH_DEP_MODE", None)
            else:
                os.environ["BENCH_DEP_MODE"] = saved_dep
    try:
        dt, launch_us, sampled, _ = timed_run(run, None, torch, torch.cuda.synchronize, 1)
        modes = sorted({run.dep_mode(i) for i in range(run.n_warm, len(run.launches)) if len(run.launches[i]) > 1})
        r_alg = alg_bytes(run, sampled) / max(len(sampled), 1)
        refs = [golden_frames(config, sd, overrides or {}) for sd in seeds]
        ok, n, missing, _ = run.verify(refs)
        gbs = r_alg / (launch_us * 1e-6) / 1e9 if launch_us > 0 else 0.0
        per_step = launch_us * len(sampled) / max(1, sum(len(run.launches[i]) for i in sampled))
        return {"size": f"{w * 16}x{h * 16}", "streams": S, "seeds": seeds, "steps": steps,
                **({"generator_overrides": overrides} if overrides else {}),
                **({"steps_per_launch": run.P, "avg_kernel_us_per_step": round(per_step, 2),
                    "dependency_modes": [{1: "rows", 2: "cols"}[m] for m in modes]} if pipe > 1 else {}),
                "mc_waves_per_row_workgroup": run.eng.last_mc_waves() if hasattr(run.eng, "last_mc_waves") else mc_waves,
                "rows_per_workgroup": run.eng.rows_per_workgroup(S),
                "frames_per_s": round(S * steps / dt, 1), "avg_launch_us": round(launch_us, 2),
                "picture_latency_ms": round(launch_us / 1e3, 3),
                "alg_bytes_per_launch": int(r_alg), "achieved_GBs": round(gbs, 1),
                "frac_hbm": round(gbs / HBM_PEAK_GBS, 5),
                "bitexact": {"ok": ok, "frames_checked": n, "frames_without_fixture": missing},
                "device_errors": run.eng.errors()}
    finally:
        run.free()


def config_legs(L, torch):
    """SURVEY §8d config 2 (1280x720 I-only, seeds 1..4: the dependency-bound
    intra wavefront -- frames/s, not a roofline) and config 5 (3840x2160, one
    stream, the config-3 mix) with the MC-wave count of the row workgroup
    swept (2 vs 3: the sizing choice of this design)."""
    return {
        "cfg2_720p_ionly_4streams": run_leg(L, torch, 1, [1, 2, 3, 4], 20, 4, mc_waves=0),
        "cfg2_720p_ionly_1stream": run_leg(L, torch, 1, [1], 20, 4, mc_waves=0),
        "cfg5_2160p_1stream": run_leg(L, torch, 4, [100], 20, 4),
        "cfg5_2160p_1stream_2mc": run_leg(L, torch, 4, [100], 20, 4, mc_waves=2),
        "cfg5_2160p_1stream_2rows": run_leg(L, torch, 4, [100], 20, 4, rpw=2),
        "cfg5_2160p_1stream_2mc_2rows": run_leg(L, torch, 4, [100], 20, 4, mc_waves=2, rpw=2),
        # the single 4K stream with three consecutive pictures per launch
        "cfg5_2160p_1stream_pipe3": run_leg(L, torch, 4, [100], 21, 3, pipe=3),
        # configs[3]'s rank-0 streams without off-picture motion: frame-pipelined
        # launches on (MB row, MB column) waits (chosen per launch), and forced
        # to whole rows beside it
        "cfg3_realistic_motion_8streams": run_leg(L, torch, 3, list(range(100, 108)), 54, 3,
                                                  overrides={"offpic_pct": 0}, pipe=3),
        "cfg3_realistic_motion_8streams_rows": run_leg(L, torch, 3, list(range(100, 108)), 54, 3,
                                                       overrides={"offpic_pct": 0}, pipe=3, dep="rows"),
        # the same streams encoded the way the reference recommends, loop
        # filter off in every slice (README.markdown:32-35, `-flags -loop`;
        # disable_deblocking_filter_idc 1): no MB row waits on the row above
        # (DESIGN.md §3.2), only on the MC of its own MBs and intra neighbours
        "cfg3_no_loop_filter_8streams": run_leg(L, torch, 3, list(range(100, 108)), 54, 3,
                                                overrides={"dbf_idc1_pct": 100}, pipe=3),
        "cfg3_no_loop_filter_8streams_pipe1": run_leg(L, torch, 3, list(range(100, 108)), 56, 4,
                                                      overrides={"dbf_idc1_pct": 100}, pipe=1, mc_waves=2),
    }


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse_args(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, argv))
    torch, dist, rank, local, world = dist_setup(a.gpus)
    if not a.dry_run:
        # the rank's GPU is the current device from here on (torch and the
        # HIP runtime libh264mi.so shares with it); the engine and every
        # buffer of the run are bound to it explicitly as well
        torch.cuda.set_device(local)
    from broadway_amd import _lib
    L = _lib.mi()

    S = a.streams
    seeds = shard_seeds(rank, S)
    overrides = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.gen.split(",") if kv)
    # GOP phases (the default): every stream is one 60-picture GOP decoded
    # cyclically, IDRs staggered over the steps; --aligned / --pipe 2: the
    # round-2 layout (pictures W .. W+K-1 of every stream, decode order)
    staggered = not a.aligned
    nframes = GOP if staggered and not overrides else max(GOP, a.warmup + a.steps)
    t_prep = time.perf_counter()
    streams, caps = prepare(a.config, seeds, nframes, overrides)
    assert all(c.errors == 0 and c.npics >= min(nframes, GOP) for c in caps), "stream preparation failed"
    w, h = caps[0].w_mbs, caps[0].h_mbs
    # phases for P-step launches: launches start at the timed window's first
    # step, and an IDR is its launch's last picture (BENCH_IDR_FIRST=1: the
    # first, such launches split)
    pstep = a.pipe if a.pipe > 1 else 1
    phases = gop_phases(S, min(c.npics for c in caps), pstep, warmup=a.warmup) if staggered else None
    run = DeviceRun(L, caps, a.warmup, a.steps, a.pipe, device=local, dry=a.dry_run, phases=phases)
    placement = run.placement()
    assert all(d == local for _, d in placement), f"rank {rank}: buffers not on device {local}: {placement}"
    eng, P, resident = run.eng, run.P, run.resident
    t_prep = time.perf_counter() - t_prep
    sync = (lambda: None) if a.dry_run else torch.cuda.synchronize
    # HIP events on every timed launch by default: they ride k_wgpp's own
    # dispatch packet (no extra launch or sync), and every launch -- those
    # holding an IDR included -- enters the roofline's kernel time
    stride = int(os.environ.get("BENCH_TIMING_STRIDE", "1"))

    dt, step_us, sampled, per_launch = timed_run(run, dist, torch, sync, stride)
    split = launch_split(run, sampled, per_launch) if per_launch else None
    launches_timed = len(run.launches) - run.n_warm
    errors = eng.errors()
    timed = run.timed_pictures()
    n_i = sum(1 for s, k in timed if run.is_i[k][s])
    refs = [golden_frames(a.config, sd, overrides) for sd in seeds]
    res_ok, res_n = (None, 0) if a.dry_run or a.no_verify else run.check_resident(refs)

    frames_total = S * a.steps * world
    fps = frames_total / dt
    # roofline: R_alg of the launches the HIP events sampled
    # (per picture: MC reference footprint + coded 4x4 blocks x 32 B + 96-B
    # MB records) / their average k_wgpp duration
    launch_bytes = alg_bytes(run, sampled) / max(len(sampled), 1)
    launch_ref_lines = ref_line_bytes(run, sampled) / max(len(sampled), 1)
    achieved = launch_bytes / (step_us * 1e-6) / 1e9 if step_us > 0 else 0.0
    # the committed PMC passes measured the default workload (configs[3], 8 streams, this
    # pipe depth): another config or stream count reports traffic null, never that one's
    traffic = load_traffic() if (a.config == 3 and a.streams == 8 and not a.gen and not a.aligned) else None
    frame_read_gbs = alg_bytes(run, range(run.n_warm, len(run.launches))) * world / dt / 1e9

    # the same streams with aligned GOPs, timed window P pictures only (the
    # round-2 headline's mix), beside the configs[3] mix -- not instead
    p_only = None
    if staggered:
        # pictures P+W .. P+W+kp-1: no IDR (P = steps per launch)
        kp = max(P, min(a.steps, run.N - P - a.warmup) // P * P)
        run.set_plan(a.warmup, kp, [P] * S)
        dt_p, us_p, _, _ = timed_run(run, dist, torch, sync, stride)
        tp = run.timed_pictures()
        p_only = {"value": round(S * kp * world / dt_p, 2), "unit": "frames/s", "steps": kp,
                  "avg_launch_kernel_us": round(us_p, 2),
                  "i_pictures_timed": sum(1 for s, k in tp if run.is_i[k][s]),
                  "window": f"pictures {P + a.warmup}..{P + a.warmup + kp - 1} of every stream (GOPs aligned, no IDR)"}
        run.set_plan(a.warmup, a.steps, phases)

    ok, n_checked, n_missing, n_pre = None, 0, 0, 0
    if not a.no_verify and not a.dry_run:
        ok, n_checked, n_missing, n_pre = run.verify(refs)
        ok = ok and res_ok
    n_checked_all = int(reduce_over_ranks(dist, torch, n_checked, "sum"))
    n_missing_all = int(reduce_over_ranks(dist, torch, n_missing, "sum"))
    res_n_all = int(reduce_over_ranks(dist, torch, res_n, "sum"))
    n_i_all = int(reduce_over_ranks(dist, torch, n_i, "sum"))
    ok_all = None if ok is None else reduce_over_ranks(dist, torch, 0.0 if ok else 1.0, "max") == 0.0
    errors_all = int(reduce_over_ranks(dist, torch, errors, "sum"))
    if dist:
        allp = [None] * world
        dist.all_gather_object(allp, {"rank": rank, "device": local, "buffers": placement})
    else:
        allp = [{"rank": rank, "device": local, "buffers": placement}]
    rgba = rgba_leg(torch, L, eng, S, w, h) if rank == 0 and not a.dry_run and not a.no_rgba else None

    cpu = None
    if rank == 0 and not a.no_cpu_baseline and not a.dry_run:
        cpu = cpu_baseline(streams, nframes)
    run.close_engine()
    legs = None
    if rank == 0 and world == 1 and not a.no_legs and not a.dry_run:
        legs = config_legs(L, torch)
    # end-to-end drop-in path on every rank: its own h264mi_dec processes on
    # its own GPU, pinned to a disjoint, NUMA-local host-core share
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    # the rank's own index among the local ranks: under BENCH_ONE_DEVICE every
    # rank's GPU is device 0 (local = 0), but each still takes its own
    # disjoint share of that device's NUMA-local cores
    core_idx = int(os.environ.get("LOCAL_RANK", str(rank)))
    one_dev = os.environ.get("BENCH_ONE_DEVICE") == "1"
    numa = [-1 if a.dry_run else gpu_numa_node(torch, 0 if one_dev else j) for j in range(local_world)]
    my_cpus, _ = e2e_core_plan(core_idx, numa, os.sched_getaffinity(0))
    e2e_plan = {"rank": rank, "device": local, "numa_node": numa[core_idx] if core_idx < len(numa) else -1,
                "cpus": format_cpulist(my_cpus), "host_cores": len(my_cpus)}
    e2e = None
    if not a.no_e2e and not a.dry_run:
        if dist:
            dist.barrier()
        # pinned at N = 1 too: the GPU's NUMA-local cores (tools/e2e_only.py
        # E2E_PIN A/B, profiles/r80_e2e_pin.txt: 4.53-4.68 vs 4.97-5.70 ms of
        # host CPU per picture, and steadier)
        # one-device rehearsal (BENCH_ONE_DEVICE=1): every rank's processes
        # share one GPU, which admits 16 GPU processes -- the ranks, their
        # decoder processes and each rank's one-process shared-engine run
        # (ranks finish at different times) stay within that
        procs = MAX_E2E_PROCS if os.environ.get("BENCH_ONE_DEVICE") != "1" or world == 1 \
            else max(1, (16 - 2 * world) // world - 1)
        e2e = end_to_end(streams, nframes, device=local, cpus=my_cpus if my_cpus else None, max_procs=procs,
                         release=dist.barrier if dist else None)
    if dist:
        plans, e2es = [None] * world, [None] * world
        dist.all_gather_object(plans, e2e_plan)
        dist.all_gather_object(e2es, e2e)
        if e2e is not None and all(x is not None for x in e2es):
            # all ranks' processes released together (the barrier in the
            # start gate): every rank's pictures over the union of all windows
            # (CLOCK_MONOTONIC is one clock on the host)
            # (a rank whose processes reported no window: its longest single window)
            if all(x.get("t_start_mono") is not None and x.get("t_end_mono") is not None for x in e2es):
                span = max(x["t_end_mono"] for x in e2es) - min(x["t_start_mono"] for x in e2es)
            else:
                span = max(x["seconds"] for x in e2es)
            e2e = {"value": round(sum(x["pictures"] for x in e2es) / span, 2),
                   "seconds": round(span, 6), "window": "union of every rank's decode windows, common start gate",
                   "unit": "frames/s", "n_gpus": world,
                   "host_cores_total": sum(x["host_cores_assigned"] or 0 for x in e2es),
                   "host_cpu_ms_per_picture": round(sum(x.get("host_cpu_ms_per_picture", 0) * x["pictures"] for x in e2es)
                                                    / max(sum(x["pictures"] for x in e2es), 1), 3),
                   "per_rank": e2es}
    else:
        plans = [e2e_plan]

    if rank == 0:
        mix = (f"IDRs staggered: stream s enters the timed window {phases} pictures into its GOP "
               f"(s*{run.N}/{S}, rounded down to whole launches; pre-roll + warmup untimed), "
               f"1 I per {run.N} in every {run.N}-step window"
               if staggered else "decode order from picture 0 (aligned GOPs)")
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
                       "gop_mix": mix,
                       "i_pictures_timed": n_i_all,
                       "i_share_timed": round(n_i_all / max(frames_total, 1), 5),
                       "parallelism": f"streams sharded {S}/GPU over {world} rank(s), no collective; "
                                      f"{P} consecutive picture(s) of each stream per launch"},
            "roofline": {"kernel": f"k_wgpp (one launch = {P} step(s)" + (", every IDR the last picture of its launch" if P > 1 and phases else "") +
                                   "; k_prep of the next launch runs in its tail)",
                         # what limits the kernel: the MB-row deblocking dependency chain
                         # (DESIGN.md §3), not HBM; `frac` is still quoted against the HBM
                         # peak, the metric's axis
                         "bound": "latency",
                         "frac_axis": "hbm",
                         "limiter": "latency: the MB-row deblocking dependency chain (DESIGN.md §3), not HBM",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         # per timed launch, the unit of `achieved` (launches of 1 .. P steps)
                         "traffic": traffic.get("hbm_bytes_per_timed_launch")
                         if traffic else None,
                         "traffic_per_step": traffic.get("hbm_bytes_per_timed_step")
                         if traffic else None,
                         "alg_bytes_per_launch": int(launch_bytes),
                         # reference reads at 128-B line granularity (compulsory for these
                         # windows; R_alg counts only the bytes used) and the PMC traffic by
                         # request size (tools/pmc_bytes.sh), DESIGN.md §3.3
                         "ref_line_bytes_per_launch": int(launch_ref_lines),
                         "traffic_by_request_size": (traffic.get("request_size_accounting") or {}).get(
                             "dram_bytes_per_step") if traffic else None,
                         # over the whole timed window (every launch by default),
                         # with the launches holding an IDR and the P-only ones apart
                         "avg_launch_kernel_us": round(step_us, 2),
                         "avg_kernel_us_per_step": round(sum(per_launch) / max(1, sum(
                             len(run.launches[i]) for i in sampled[:len(per_launch)])), 2) if per_launch else None,
                         "timed_launches_sampled": len(sampled),
                         "sampling_stride": stride,
                         "launches_with_idr": {"n": split["i"][0], "avg_launch_kernel_us": split["i"][1],
                                               "avg_us_per_step": split["i"][2]} if split else None,
                         "launches_p_only": {"n": split["p"][0], "avg_launch_kernel_us": split["p"][1],
                                             "avg_us_per_step": split["p"][2]} if split else None,
                         "aggregate_achieved_GBs": round(frame_read_gbs, 1),
                         "traffic_source": traffic.get("source") if traffic else None,
                         # the bound this kernel actually has: the row chain's latency
                         "latency": latency_floor(w, h, P, load_ubench(),
                                                  (split["p"][1] if split and split["p"][0] else step_us),
                                                  load_dep_floor(a.config, a.streams, P, a.gen))},
            "kernels": {"k_wgpp": {"avg_launch_us": round(step_us, 2),
                                   "pictures_per_launch": round(S * a.steps / max(launches_timed, 1), 2),
                                   "steps_per_launch": P,
                                   "avg_steps_per_timed_launch": round(a.steps / max(launches_timed, 1), 3),
                                   "timed_launches": launches_timed,
                                   # this run's k_wgpp dispatch indices (0-based, in
                                   # rocprofv3 kernel-trace order): the timed window and
                                   # the launches the HIP events sampled
                                   "trace_window": [run.n_warm, len(run.launches)],
                                   "trace_steps": [len(run.launches[i]) for i in range(run.n_warm, len(run.launches))],
                                   "trace_sampled": sampled if len(sampled) != launches_timed else "all",
                                   "bound": "latency (MB-row deblocking dependency chain); MC waves overlap it"}},
            "p_only": p_only,
            "wall_read_GBs": round(frame_read_gbs, 2),
            "cpu_baseline": cpu,
            "end_to_end": e2e,
            "end_to_end_plan": plans,
            "rgba_output": rgba,
            "config_legs": legs,
            "bitexact_check": {"ok": ok_all, "frames_checked": n_checked_all,
                               "frames_expected": S * world * (a.warmup + a.steps),
                               "frames_without_fixture": n_missing_all,
                               "timed_run_resident_frames_checked": res_n_all,
                               "preroll_frames_checked": n_pre,
                               "method": "(1) after the timed loop, every frame slot's last picture -- the timed "
                                         "launches' own output -- vs reference-decoder MD5s; (2) untimed re-run "
                                         "of the whole plan, every warmup + timed picture of every stream of "
                                         "every rank vs the MD5s right after its launch",
                               "residual_range_errors": errors_all},
            "device_placement": allp,
            "prep_seconds": round(t_prep, 1),
            **({"one_device_rehearsal": f"{world} ranks shared device 0 (BENCH_ONE_DEVICE=1): not a multi-GPU rate"}
               if os.environ.get("BENCH_ONE_DEVICE") == "1" else {}),
            "hbm_resident_input_MB": round(resident / 1e6, 1),
        }
        if a.dry_run:
            line["dry_run"] = {"launches": eng.launches, "seeds": seeds, "preroll_launches": run.n_pre}
        print(json.dumps(line), flush=True)
    run.free()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
