set -o pipefail
mkdir -p gpurun_out/r28
export TMPDIR=/tmp
ROUNDS=2 bash tools/ab_env.sh "H264MI_PREP_MC=0" "H264MI_PREP_MC=1" > gpurun_out/r28/ab.txt 2>&1 || { cat gpurun_out/r28/ab.txt; exit 1; }
cat gpurun_out/r28/ab.txt
