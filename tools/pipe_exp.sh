set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
run() {
  timeout -k 10 300 env $1 python bench.py --no-cpu-baseline $2 > gpurun_out/pe.log 2>&1 || { tail -20 gpurun_out/pe.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/pe.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['roofline']['achieved'], d['kernels'], d['bitexact_check'])" "$1 $2"
}
run "X=1" ""
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/px/f -o b -- python3 bench.py --no-cpu-baseline --no-verify --steps 8 > /dev/null 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/px/w -o b -- python3 bench.py --no-cpu-baseline --no-verify --steps 8 > /dev/null 2>&1
