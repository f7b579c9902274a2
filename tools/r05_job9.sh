set -o pipefail
export TMPDIR=/tmp
AB_PASSES=3 bash tools/ab.sh "main main+NGS_LEAN_PAD_LDS=1800 main+NGS_LEAN_PAD_LDS=3800 main+NGS_LEAN_PAD_LDS=7400 wps5" --steps 300 2>&1 | tee gpurun_out/r05_s9_ab_occ.txt
timeout -k 10 400 python bench.py > gpurun_out/r05_s9_c3_bench.json 2> gpurun_out/r05_s9_c3_bench.err || { tail -5 gpurun_out/r05_s9_c3_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_s9_c3_bench.json')); print('c3', d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:600]); print(d['cpu_baseline']); print(d['detail']['dropin'])"
