# session 2j (final tree, part 2): C3 kernel stats + FETCH + bench line (profile_round.sh), SQ counters
export TMPDIR=/tmp
bash tools/profile_round.sh r03s7 || exit 1
bash tools/pmc_sq.sh r03s7 || exit 1
