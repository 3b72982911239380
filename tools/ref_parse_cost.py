"""Host parse cost bar: where the reference decoder spends its CPU per 1080p
picture, split by what the product keeps on the host (bitstream / CAVLC / MB
layer parse, MV prediction) and what it moves to the GPU (MC, intra, IDCT,
deblocking, output), beside the product's own host parse on the same streams
(tools/ubench/parse_null.c: decoder core over a backend that does nothing).

Test/measurement infrastructure: runs oracle/_ref/refdec (the reference's
sources compiled by oracle/Makefile.ref) and its gprof build refdec_pg
(`make -C oracle -f Makefile.ref prof`); functions are attributed to their
source file through the binary's own debug line table (nm -l), nothing under
/root/reference is read.

    python tools/ref_parse_cost.py [--streams 4] [--frames 60]
"""
import argparse
import glob
import os
import resource
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REF = os.path.join(ROOT, "oracle", "_ref")
CSRC = os.path.join(ROOT, "broadway_amd", "csrc")

# reference source file -> side (h264bsd_*.c); macroblock_layer.c is split by
# function: h264bsdDecodeMacroblock (+ its residual processing) reconstructs
PARSE_FILES = ("byte_stream", "stream", "vlc", "cavlc", "slice_data", "slice_header", "nal_unit",
               "seq_param_set", "pic_param_set", "neighbour", "pic_order_cnt", "vui", "slice_group_map",
               "macroblock_layer", "util")
MV_FILES = ("inter_prediction",)
RECON_FILES = ("transform", "intra_prediction", "reconstruct", "deblocking", "image", "conceal")
RECON_FUNCS = ("h264bsdDecodeMacroblock", "ProcessResidual", "ProcessIntra4x4Residual",
               "ProcessChromaResidual", "ProcessIntra16x16Residual", "h264bsdProcessBlock",
               "h264bsdProcessLumaDc", "h264bsdProcessChromaDc")
# product host sources (parse_null's decoder core)
OUR_SRCS = ["common/bits.c", "common/cavlc.c", "common/mbctx.c", "common/resid.c", "common/tables.c",
            "host/conceal.c", "host/decoder.c", "host/dpb.c", "host/slicedata.c", "host/specparse.c",
            "host/syntax.c"]


def streams(n, frames):
    import bench
    s, _ = bench.prepare(3, bench.shard_seeds(0, n), frames)
    return s


def func_files(binary):
    """function name -> source file stem, from the binary's debug info."""
    out = subprocess.run(["nm", "--line-numbers", binary], capture_output=True, text=True, check=True).stdout
    m = {}
    for line in out.splitlines():
        parts = line.split()
        if len(parts) >= 4 and parts[1] in "tTwW":
            stem = os.path.basename(parts[3].split(":")[0])
            m[parts[2]] = stem[:-2] if stem.endswith(".c") else stem
    return m


def flat(binary, gmon):
    """(self seconds, function) of gprof's flat profile."""
    out = subprocess.run(["gprof", "-b", "-p", binary, gmon], capture_output=True, text=True, check=True).stdout
    rows = []
    for line in out.splitlines():
        p = line.split()
        if len(p) >= 4 and p[0].replace(".", "").isdigit() and p[1].replace(".", "").isdigit():
            try:
                rows.append((float(p[2]), p[-1]))
            except ValueError:
                pass
    return rows


def side_ref(fn, stem):
    s = stem.replace("h264bsd_", "")
    if fn in RECON_FUNCS or s in RECON_FILES:
        return "recon"
    if s in MV_FILES:
        return "mv_pred" if fn != "h264bsdInterPrediction" else "mv_pred+mc_dispatch"
    if s in PARSE_FILES:
        return "parse"
    return "other"


def gprof_run(binary, paths, args, tmp, env=None, post=()):
    for g in glob.glob(os.path.join(tmp, "gmon*")):
        os.remove(g)
    e = dict(os.environ, GMON_OUT_PREFIX=os.path.join(tmp, "gmon"), **(env or {}))
    for p in paths:
        subprocess.run([binary] + args + [p] + list(post), stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                       check=True, cwd=tmp, env=e)
    files = sorted(glob.glob(os.path.join(tmp, "gmon.*")))
    subprocess.run(["gprof", "-s", binary] + files, check=True, cwd=tmp, capture_output=True)
    return flat(binary, os.path.join(tmp, "gmon.sum"))


def cpu_time(cmd, env=None):
    r0 = resource.getrusage(resource.RUSAGE_CHILDREN)
    t0 = time.perf_counter()
    subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, check=True, env=env)
    r1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    return time.perf_counter() - t0, (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)


def build_ours(tmp, pg):
    exe = os.path.join(tmp, "parse_null_pg" if pg else "parse_null")
    srcs = [os.path.join(CSRC, s) for s in OUR_SRCS]
    cmd = ["gcc", "-O3", "-march=x86-64-v3", "-std=gnu11", "-w", "-I" + CSRC] + (["-pg", "-g"] if pg else []) + \
          [os.path.join(ROOT, "tools", "ubench", "parse_null.c")] + srcs + ["-lpthread", "-o", exe]
    subprocess.run(cmd, check=True)
    return exe


def report(title, rows, classify, pics, scale):
    tot = sum(t for t, _ in rows) or 1e-9
    by = {}
    for t, fn in rows:
        by[classify(fn)] = by.get(classify(fn), 0.0) + t
    print(f"\n{title}: {tot:.2f} s sampled over {pics} pictures; ms/picture scaled to the un-instrumented "
          f"build's CPU ({scale * 1e3 / pics:.2f} ms/picture)")
    for k, v in sorted(by.items(), key=lambda kv: -kv[1]):
        print(f"  {k:22s} {100 * v / tot:5.1f} %   {scale * 1e3 / pics * v / tot:6.2f} ms/picture")
    print("  top functions:")
    for t, fn in sorted(rows, reverse=True)[:14]:
        print(f"    {100 * t / tot:5.1f} %  {fn}  [{classify(fn)}]")
    return by, tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--frames", type=int, default=60)
    a = ap.parse_args()
    for b in ("refdec", "refdec_pg"):
        if not os.path.exists(os.path.join(REF, b)):
            sys.exit(f"oracle/_ref/{b} missing: make -C oracle -f Makefile.ref all prof")
    with tempfile.TemporaryDirectory() as tmp:
        paths = []
        for i, s in enumerate(streams(a.streams, a.frames)):
            p = os.path.join(tmp, f"s{i}.h264")
            with open(p, "wb") as f:
                f.write(s)
            paths.append(p)
        pics = a.streams * a.frames
        print(f"configs[3] streams: {a.streams} x {a.frames} pictures 1080p (seeds 100..), one process at a time")

        # reference: plain build for the CPU per picture, gprof build for the split
        wall = cpu = 0.0
        for p in paths:
            w, c = cpu_time([os.path.join(REF, "refdec"), "-Onone", p])
            wall, cpu = wall + w, cpu + c
        print(f"reference decoder (refdec -Onone, gcc -O2): {1e3 * cpu / pics:.2f} ms CPU/picture "
              f"({pics / wall:.1f} fps single core)")
        rmap = func_files(os.path.join(REF, "refdec_pg"))
        rows = gprof_run(os.path.join(REF, "refdec_pg"), paths, ["-Onone"], tmp)
        by, tot = report("reference, gprof split", rows, lambda fn: side_ref(fn, rmap.get(fn, "?")), pics, cpu)
        host = sum(v for k, v in by.items() if k != "recon")
        print(f"  => reference host-side work (everything but recon): {1e3 * cpu / pics * host / tot:.2f} ms/picture")

        # ours: sequential parse (no slice workers), and its gprof split
        ours = build_ours(tmp, False)
        env = dict(os.environ, H264MI_PARSE_THREADS="0", H264MI_PARSE_HELP="0")
        wall = cpu = 0.0
        for p in paths:
            w, c = cpu_time([ours, p, "1"], env)
            wall, cpu = wall + w, cpu + c
        print(f"\nproduct host parse (parse_null, H264MI_PARSE_THREADS=0, gcc -O3 x86-64-v3): "
              f"{1e3 * cpu / pics:.2f} ms CPU/picture")
        ours_pg = build_ours(tmp, True)
        omap = func_files(ours_pg)
        rows = gprof_run(ours_pg, paths, [], tmp, {"H264MI_PARSE_THREADS": "0", "H264MI_PARSE_HELP": "0"}, post=["5"])   # 5 passes: samples
        report("product host parse, gprof split by file", rows, lambda fn: omap.get(fn, "?"), pics, cpu)


if __name__ == "__main__":
    main()
