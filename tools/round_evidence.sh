#!/bin/bash
# A session's evidence on the current tree, in one GPU call (on the box, from the repo root):
#   1. the GPU test suite and smoke();
#   2. bench lines of every config (C3 with the drop-in and CPU-baseline legs);
#   3. tools/profile_round.sh on C3 (kernel stats, FETCH pass, SQ pass -> profiles/pmc_c3.json).
# Every step has its own time limit and the script stops at the first failure.
# usage: tools/round_evidence.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:?tag}
O=gpurun_out/ev_$TAG
mkdir -p $O
if [ "$2" != skip-tests ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || { echo "gpu tests failed"; tail -20 $O/gputest.txt; exit 1; }
  tail -1 $O/gputest.txt
  timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
fi
timeout -k 10 400 python3 bench.py > $O/c3_bench.json 2> $O/c3_bench.err || { echo "c3 bench failed"; tail -5 $O/c3_bench.err; exit 1; }
timeout -k 10 300 python3 bench.py --config c2 > $O/c2_bench.json 2> $O/c2_bench.err || { echo "c2 bench failed"; exit 1; }
timeout -k 10 400 python3 bench.py --config c5 --no-cpu-baseline --no-dropin --steps 20 > $O/c5_bench.json 2> $O/c5_bench.err || { echo "c5 bench failed"; exit 1; }
timeout -k 10 500 python3 bench.py --config c4 --no-cpu-baseline --no-dropin --steps 12 --warmup 4 > $O/c4_bench.json 2> $O/c4_bench.err || { echo "c4 bench failed"; exit 1; }
for c in c3 c2 c5 c4; do
  python3 -c "import json; d=json.load(open('$O/${c}_bench.json')); print('$c', d['value'], d['unit'], d['ms_per_step'], 'ms/step frac', d['roofline']['frac'])"
done
tools/profile_round.sh $TAG c3 > $O/profile_round.txt 2>&1 || { echo "profile_round failed"; tail -5 $O/profile_round.txt; exit 1; }
tail -1 $O/profile_round.txt | cut -c1-300
