set -o pipefail
mkdir -p gpurun_out/r31
export TMPDIR=/tmp
ROUNDS=2 bash tools/ab_verify.sh base tail5 > gpurun_out/r31/ab.txt 2>&1 || { cat gpurun_out/r31/ab.txt; exit 1; }
cat gpurun_out/r31/ab.txt
