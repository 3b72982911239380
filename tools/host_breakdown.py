"""Host CPU per 1080p picture of the drop-in path, layer by layer (verdict r03
#4): the decoder core over a backend that does nothing (parse_null), then
h264mi_dec through the H264SwDec* C-ABI with the HIP backend, one process and
then 8 concurrent processes (bench.py end_to_end), with and without slice
workers.  The differences are what each layer adds on top of the parse.

    python tools/host_breakdown.py [--frames 60] [--reps 3]
"""
import argparse
import os
import resource
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from ref_parse_cost import build_ours, streams  # noqa: E402


def run(cmd, env):
    r0 = resource.getrusage(resource.RUSAGE_CHILDREN)
    t0 = time.perf_counter()
    o = subprocess.run(cmd, capture_output=True, text=True, check=True, env=env)
    r1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    return o.stdout, time.perf_counter() - t0, (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)


def fields(out):
    d = {}
    for line in out.splitlines():
        f = line.split()
        if len(f) >= 2:
            try:
                d[f[0]] = float(f[1])
            except ValueError:
                pass
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    exe = os.path.join(ROOT, "broadway_amd", "lib", "h264mi_dec")
    with tempfile.TemporaryDirectory() as tmp:
        paths = []
        for i, s in enumerate(streams(8, a.frames)):
            p = os.path.join(tmp, f"s{i}.h264")
            with open(p, "wb") as f:
                f.write(s)
            paths.append(p)
        pn = build_ours(tmp, False)
        print(f"configs[3] 1080p streams, {a.frames} pictures, {a.reps} passes; ms of host CPU per picture "
              f"(all threads, user + sys)")
        for th in ("0", "2", "3"):
            env = dict(os.environ, H264MI_PARSE_THREADS=th, H264MI_PARSE_HELP="0")
            out, w, c = run([pn, paths[0], str(a.reps)], env)
            n = a.frames * a.reps
            print(f"parse_null  workers {th}: cpu {1e3 * c / n:6.3f}  wall {1e3 * w / n:6.3f}   | {out.strip()}")
        combos = [("0", "0"), ("0", "1"), ("1", "1"), ("2", "0"), ("2", "1")]   # (workers, caller parses ahead)
        for th, hp in combos:
            env = dict(os.environ, H264MI_PARSE_THREADS=th, H264MI_PARSE_HELP=hp, H264MI_BLOCKING_SYNC="1")
            out, w, _ = run([exe, "-Onone", f"-r{a.reps}", "-T", paths[0]], env)
            d = fields(out)
            n = d["pictures"]
            print(f"h264mi_dec 1 process, workers {th} help {hp}: cpu {1e3 * d['cpu_seconds'] / n:6.3f} "
                  f"(decode thread {1e3 * d.get('cpu_decode_threads_seconds', 0) / n:6.3f}) "
                  f"(sys {1e3 * d['cpu_sys_seconds'] / n:5.3f})  fps {n / d['decode_seconds']:8.1f}  per picture in the calling "
                  f"thread: parse {1e3 * d['t_parse'] / n:5.3f} submit {1e3 * d['t_submit'] / n:5.3f} "
                  f"wait {1e3 * d['t_wait'] / n:5.3f} copy {1e3 * d['t_copy'] / n:5.3f}")
        for th, hp in combos:
            env = dict(os.environ, H264MI_PARSE_THREADS=th, H264MI_PARSE_HELP=hp, H264MI_BLOCKING_SYNC="1")
            procs = [subprocess.Popen([exe, "-Onone", f"-r{a.reps}", "-T", p], stdout=subprocess.PIPE, text=True,
                                      env=env) for p in paths]
            outs = [fields(pr.communicate()[0]) for pr in procs]
            n = sum(d["pictures"] for d in outs)
            cpu = sum(d["cpu_seconds"] for d in outs)
            t = max(d["decode_seconds"] for d in outs)
            dthr = sum(d.get("cpu_decode_threads_seconds", 0) for d in outs)
            print(f"h264mi_dec 8 processes, workers {th} help {hp}: cpu {1e3 * cpu / n:6.3f} (decode threads {1e3 * dthr / n:6.3f})"
                  f"  fps {n / t:8.1f}  "
                  f"parse {1e3 * sum(d['t_parse'] for d in outs) / n:5.3f} "
                  f"wait {1e3 * sum(d['t_wait'] for d in outs) / n:5.3f} "
                  f"copy {1e3 * sum(d['t_copy'] for d in outs) / n:5.3f}")


if __name__ == "__main__":
    main()
