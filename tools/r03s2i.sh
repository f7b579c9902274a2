# session 2i (final tree, part 1): full GPU suite, smoke, C2 / C4 / C5 bench lines
export TMPDIR=/tmp
O=gpurun_out/s2i
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -20 $O/gputest.txt; exit 1; }
tail -1 $O/gputest.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
for c in c2 c4 c5; do
  timeout -k 10 400 python3 bench.py --config $c --no-dropin --steps 20 --warmup 10 > $O/$c.json 2> $O/$c.err || { tail -3 $O/$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], 'Mq/s', d['ms_per_step'], 'ms frac', d['roofline']['frac'], d['detail']['paths'])"
done
