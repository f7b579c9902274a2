#!/bin/bash
# One GPU session's roofline evidence for profiles/ (one config, default c3):
#   1. rocprofv3 kernel stats of the bench command (per-kernel durations, batches pipelined);
#   2. a FETCH_SIZE pass (HBM bytes per call);
#   3. an SQ counter pass (dispatches serialised: the main k_wave_lean launch's own duration);
#   4. tools/pmc_traffic.py -> profiles/pmc_<cfg>.json with both, stamped with the library profiled
#      (bench.py reports roofline.traffic / traffic_source / serialised from it);
#   5. the bench line itself.
# usage (on the GPU box, from the repo root): tools/profile_round.sh <tag> [cfg]
set -o pipefail
TAG=${1:-run}
CFG=${2:-c3}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 bench.py --config $CFG --no-cpu-baseline --no-dropin > $OUT/stats_bench.json 2> $OUT/stats_bench.err || { echo "stats pass failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
    python3 bench.py --config $CFG --no-cpu-baseline --no-dropin --steps 5 --warmup 1 > $OUT/fetch_bench.json 2> $OUT/fetch_bench.err || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- \
    python3 bench.py --config $CFG --no-cpu-baseline --no-dropin --steps 5 --warmup 1 > $OUT/sq_bench.json 2> $OUT/sq_bench.err || { echo "sq pass failed"; exit 1; }
LIBV=$(python3 -c "import json; print(json.load(open('$OUT/fetch_bench.json'))['detail']['library'])") || exit 1
python3 tools/pmc_traffic.py $OUT/fetch $CFG --sq $OUT/sq --library "$LIBV" || exit 1
timeout -k 10 400 python3 bench.py --config $CFG > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
cat $OUT/bench.json
