#!/bin/bash
# One GPU session's evidence for profiles/: rocprofv3 kernel stats of the bench command, a
# FETCH_SIZE pass (HBM traffic per tier-1a launch -> profiles/pmc_c3.json), then the bench line.
# usage (on the GPU box, from the repo root): tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:-run}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-dropin > $OUT/stats_bench.json 2> $OUT/stats_bench.err || { echo "stats pass failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-dropin --steps 5 --warmup 1 > $OUT/fetch_bench.json 2> $OUT/fetch_bench.err || { echo "fetch pass failed"; exit 1; }
python3 tools/pmc_traffic.py $OUT/fetch c3 k_wave_lean || exit 1
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
cat $OUT/bench.json
