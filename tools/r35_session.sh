set -o pipefail
mkdir -p gpurun_out/r35
timeout -k 10 200 python tools/prof_chain.py > gpurun_out/r35/chain_s8.log 2>&1 || { tail -20 gpurun_out/r35/chain_s8.log; exit 1; }
PROF_PIC=0 timeout -k 10 200 python tools/prof_chain.py > gpurun_out/r35/chain_i_s8.log 2>&1 || { tail -20 gpurun_out/r35/chain_i_s8.log; exit 1; }
PROF_CONFIG=1 PROF_PIC=0 PROF_S=4 timeout -k 10 200 python tools/prof_chain.py > gpurun_out/r35/chain_cfg2.log 2>&1 || { tail -20 gpurun_out/r35/chain_cfg2.log; exit 1; }
bash tools/sq_roles.sh r35_sqroles && bash tools/cfg5_profile.sh r35_cfg5
