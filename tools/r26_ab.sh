set -o pipefail
mkdir -p gpurun_out/r26
export TMPDIR=/tmp
ROUNDS=2 bash tools/ab_verify.sh base late_release > gpurun_out/r26/ab.txt 2>&1 || { cat gpurun_out/r26/ab.txt; exit 1; }
cat gpurun_out/r26/ab.txt
