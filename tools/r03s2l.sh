# session 2l: the final stamp's full GPU suite, smoke and C3 bench line
export TMPDIR=/tmp
O=gpurun_out/s2l
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1 || { tail -20 $O/gputest.txt; exit 1; }
tail -1 $O/gputest.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python3 bench.py > $O/c3.json 2> $O/c3.err || { tail -3 $O/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3.json')); print('c3', d['value'], 'Mq/s', d['ms_per_step'], 'ms frac', d['roofline']['frac'], d['detail']['library'])"
