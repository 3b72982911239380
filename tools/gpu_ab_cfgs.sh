#!/bin/bash
# A/B of (build, env) specs over the bench's configs: the GOP mix (configs[3]),
# 720p I-only (configs[1] x 4 streams) and one 2160p stream (configs[4]).
#   ROUNDS=1 bash tools/gpu_ab_cfgs.sh "cur:" "cur:H264MI_MC_WAVES=2"
set -o pipefail
ROUNDS=${ROUNDS:-1} bash tools/ab_env.sh "$@" || exit 1
BENCH_ARGS="--config 1 --streams 4 --steps 20 --warmup 4" ROUNDS=1 bash tools/ab_env.sh "$@" || exit 1
BENCH_ARGS="--config 4 --streams 1 --steps 20 --warmup 4" ROUNDS=1 bash tools/ab_env.sh "$@"
