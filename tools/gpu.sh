#!/bin/bash
# Submit one command to the GPU box via gpurun; if the box failed before the command started
# ("status=transient", nothing ran, nothing charged), wait and submit it once more.
# usage: tools/gpu.sh <timeout-seconds> '<command>'
T=$1; shift
out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
if echo "$out" | grep -q "status=transient"; then
  echo "$out" | tail -2
  sleep 75
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
fi
echo "$out" | grep -v "^\[gpurun\] sending"
exit $rc
