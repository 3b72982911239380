"""End-to-end through H264SwDec* (h264mi_dec), three process models over the
same 8 x 60-frame 1080p streams (configs[3] seeds 100..107), each stream
decoded 3 times:  8 processes (bench.end_to_end's model), 1 process x 8
threads with private engines, 1 process x 8 threads sharing one 8-lane
engine (-S8).  GPU box: python tools/e2e_share.py"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

EXE = os.path.join(ROOT, "broadway_amd", "lib", "h264mi_dec")


def parse(out):
    r = {}
    for line in out.splitlines():
        f = line.split()
        if len(f) >= 2:
            try:
                r[f[0]] = float(f[1])
            except ValueError:
                pass
    return r


def main():
    streams, _ = bench.prepare(3, [100 + i for i in range(8)], 60)
    td = tempfile.mkdtemp(prefix="e2eshare")
    paths = []
    for i, s in enumerate(streams):
        p = os.path.join(td, f"s{i}.h264")
        open(p, "wb").write(s)
        paths.append(p)
    res = {}
    # 8 processes, one stream each
    procs = [subprocess.Popen([EXE, "-Onone", "-r3", "-T", p], stdout=subprocess.PIPE, text=True) for p in paths]
    outs = [parse(pr.communicate(timeout=300)[0]) for pr in procs]
    t = max(o["decode_seconds"] for o in outs)
    pics = sum(o["pictures"] for o in outs)
    res["8proc"] = {"fps": round(pics / t, 1), "cpu_s": round(sum(o["cpu_seconds"] for o in outs), 2)}
    for name, extra in (("1proc_8thr_private", []), ("1proc_8thr_shared", ["-S8"])):
        o = subprocess.run([EXE, "-Onone", "-r3", "-T"] + extra + paths, capture_output=True, text=True, timeout=300)
        if o.returncode:
            print(name, "failed", o.stderr[-500:])
            continue
        d = parse(o.stdout)
        res[name] = {"fps": round(d["pictures"] / d["decode_seconds"], 1), "cpu_s": round(d["cpu_seconds"], 2),
                     "per_picture_ms": {k[2:]: round(d[k] * 1e3 / d["pictures"], 3) for k in d if k.startswith("t_")}}
        if "share_batches" in d:
            res[name]["pictures_per_launch"] = round(d["share_pictures"] / max(d["share_batches"], 1), 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
