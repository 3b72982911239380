set -o pipefail
mkdir -p gpurun_out/r33
export TMPDIR=/tmp
ROUNDS=2 bash tools/ab_verify.sh base2 mcprio1 > gpurun_out/r33/ab.txt 2>&1 || { cat gpurun_out/r33/ab.txt; exit 1; }
cat gpurun_out/r33/ab.txt
