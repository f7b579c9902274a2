export TMPDIR=/tmp
mkdir -p gpurun_out/r03z
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03z/c2 -o run --output-format csv -- python3 bench.py --config c2 --no-cpu-baseline --no-dropin --depth 1 --steps 50 --warmup 5 > gpurun_out/r03z/c2.json 2> gpurun_out/r03z/c2.err || { tail -3 gpurun_out/r03z/c2.err; exit 1; }
python3 tools/timeline.py gpurun_out/r03z/c2 > gpurun_out/r03z/c2_timeline.txt && cat gpurun_out/r03z/c2_timeline.txt
cp gpurun_out/r03z/c2/run_kernel_stats.csv gpurun_out/r03z/c2_kernel_stats.csv
rm -rf gpurun_out/r03z/c2
