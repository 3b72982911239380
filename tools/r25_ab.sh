set -o pipefail
mkdir -p gpurun_out/r25
export TMPDIR=/tmp
ROUNDS=2 bash tools/ab_verify.sh base lead3 lead6 > gpurun_out/r25/ab.txt 2>&1 || { cat gpurun_out/r25/ab.txt; exit 1; }
cat gpurun_out/r25/ab.txt
timeout -k 10 200 python tools/prof_chain.py > gpurun_out/r25/chain_s8.log 2>&1 || { tail -20 gpurun_out/r25/chain_s8.log; exit 1; }
tail -14 gpurun_out/r25/chain_s8.log
