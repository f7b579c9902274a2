# session 2e: C4 against the survivor slots per query (fixed with NGS_ECAP; default: grown from 4096)
export TMPDIR=/tmp
mkdir -p gpurun_out/s2e
show() { python3 -c "import json,sys; d=json.load(open('$1')); p=d['detail']['paths']; print('$1', d['value'], 'Mq/s', d['ms_per_step'], 'ms/step frac', d['roofline']['frac'], 'handovers', p['tier1b_handovers'], 'slot_full', p.get('slot_full'), 'slots', d['detail'].get('survivor_slots'))"; }
for v in 16384 32768 grow; do
  if [ $v = grow ]; then unset NGS_ECAP; else export NGS_ECAP=$v; fi
  timeout -k 10 400 python3 bench.py --config c4 --no-cpu-baseline --no-dropin --steps 10 --warmup 4 > gpurun_out/s2e/c4_$v.json 2> gpurun_out/s2e/c4_$v.err || { tail -3 gpurun_out/s2e/c4_$v.err; exit 1; }
  show gpurun_out/s2e/c4_$v.json
done
