"""score() latency on BASELINE configs[0]'s shape (bench.c1_latency) as a short standalone run
for rocprofv3 (--kernel-trace --memory-copy-trace --hip-runtime-trace): where the microseconds
of one call go. usage: python tools/latency_trace.py [calls]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    print(bench.c1_latency(0, n), flush=True)


if __name__ == "__main__":
    main()
