# session 2a: locality headroom on the current tree (bench / sorted / hot batches), C3 bench line
export TMPDIR=/tmp
mkdir -p gpurun_out/s2a
timeout -k 10 300 python3 -u tools/locality_probe.py > gpurun_out/s2a/locality.txt 2>&1 || { tail -5 gpurun_out/s2a/locality.txt; exit 1; }
cat gpurun_out/s2a/locality.txt
timeout -k 10 300 python3 bench.py --no-dropin --steps 100 --warmup 5 > gpurun_out/s2a/c3.json 2> gpurun_out/s2a/c3.err || { tail -3 gpurun_out/s2a/c3.err; exit 1; }
cat gpurun_out/s2a/c3.json
