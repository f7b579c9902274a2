set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python3 bench.py --config c4 --no-cpu-baseline --no-dropin --steps 3 --warmup 3 > gpurun_out/r05_s25_c4.json 2> gpurun_out/r05_s25_c4.err || { tail -5 gpurun_out/r05_s25_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_s25_c4.json')); print(d['value'], d['ms_per_step'], d['detail']['paths'])"
head -20 gpurun_out/prof_c4/run_kernel_stats.csv | cut -c1-200
