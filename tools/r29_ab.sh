set -o pipefail
mkdir -p gpurun_out/r29
export TMPDIR=/tmp
ROUNDS=2 bash tools/ab_env.sh "H264MI_PREP_WGS=2048" "H264MI_PREP_WGS=4096" "H264MI_PREP_WGS=8192" > gpurun_out/r29/ab2.txt 2>&1 || { cat gpurun_out/r29/ab2.txt; exit 1; }
cat gpurun_out/r29/ab2.txt
