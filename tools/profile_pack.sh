#!/bin/bash
# Runs tools/profile_round.sh and tools/pmc_sq.sh under one tag on the GPU box, then keeps only the
# summaries gpurun copies back (its merge is capped at 64 MiB): kernel stats, the call timeline,
# the FETCH_SIZE counters, the SQ summary, the bench line.
# usage (GPU box, repo root): tools/profile_pack.sh <tag>
set -o pipefail
TAG=$1
tools/profile_round.sh $TAG > gpurun_out/pr_$TAG.log 2>&1 || { tail -5 gpurun_out/pr_$TAG.log; exit 1; }
python3 tools/timeline.py gpurun_out/prof_$TAG/stats > gpurun_out/prof_$TAG/timeline.txt || exit 1
tools/pmc_sq.sh $TAG > gpurun_out/sq_$TAG.log 2>&1 || { tail -5 gpurun_out/sq_$TAG.log; exit 1; }
mkdir -p gpurun_out/keep_$TAG
cp gpurun_out/prof_$TAG/stats/run_kernel_stats.csv gpurun_out/prof_$TAG/timeline.txt gpurun_out/prof_$TAG/bench.json \
   gpurun_out/pmc_$TAG/summary.txt gpurun_out/keep_$TAG/
cp gpurun_out/prof_$TAG/fetch/run_counter_collection.csv gpurun_out/keep_$TAG/fetch_counter_collection.csv
cp profiles/pmc_c3.json gpurun_out/keep_$TAG/pmc_c3.json
rm -rf gpurun_out/prof_$TAG gpurun_out/pmc_$TAG
ls -la gpurun_out/keep_$TAG
