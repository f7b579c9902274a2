set -o pipefail
export TMPDIR=/tmp
rocm-smi --showpower --showclocks --showtemp --showmaxpower > gpurun_out/r05_s17_smi_idle.txt 2>&1 || true
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-dropin --steps 20000 --warmup 10 > gpurun_out/r05_s17_bench.json 2> gpurun_out/r05_s17_bench.err &
BP=$!
sleep 22
for i in 1 2 3 4 5 6; do rocm-smi --showpower --showclocks --showtemp >> gpurun_out/r05_s17_smi_load.txt 2>&1 || true; sleep 1; done
wait $BP || { tail -5 gpurun_out/r05_s17_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_s17_bench.json')); print('c3', d['value'], d['ms_per_step'])"
grep -i "power\|sclk\|mclk\|temp" gpurun_out/r05_s17_smi_idle.txt | head -12
grep -i "power\|sclk\|temp" gpurun_out/r05_s17_smi_load.txt | head -30
