set -o pipefail
mkdir -p gpurun_out/e1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e1/t.log 2>&1 || { tail -30 gpurun_out/e1/t.log; exit 1; }
tail -2 gpurun_out/e1/t.log
for P in 1 2 3 4; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --pipeline $P > gpurun_out/e1/b$P.log 2>&1 || { tail -20 gpurun_out/e1/b$P.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/e1/b$P.log').read().strip().splitlines()[-1]);print('P=$P', d['value'], d['roofline']['achieved'], d['kernels'], d['bitexact_check'])"
done
