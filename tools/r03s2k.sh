# session 2k: tier-1b persistent grids capped at 256 / 1024 workgroups (NGS_T1B_GRID) vs one per
# wave slot (main, 3,072): C3 (hand-over lists of 0-1 queries) and C4 (448 hand-overs x 4 slices)
export TMPDIR=/tmp
bash tools/ab.sh "main g256 g1k" || exit 1
bash tools/ab.sh "main g256 g1k" --config c4 --steps 10 --warmup 8 || exit 1
