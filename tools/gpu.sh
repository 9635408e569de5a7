#!/bin/bash
# Run one command on a GPU box through gpurun after clearing the logs it will write.
# Retries (up to 3 times, 60 s apart) ONLY when gpurun reports status=transient, i.e. the box was
# never prepared and nothing ran.  Usage: tools/gpu.sh TIMEOUT 'command' log1 [log2 ...]
set -u
limit=$1; shift
cmd=$1; shift
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for f in "$@"; do rm -f "gpurun_out/$f"; done
for attempt in $(seq ${GPU_TRIES:-3}); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$limit" -- "$cmd" 2>&1)
  rc=$?
  echo "$out" | grep -E "^\[gpurun\] (status|GPU-minutes)"
  if echo "$out" | grep -q "status=transient"; then
    sleep ${GPU_WAIT:-60}
    continue
  fi
  exit $rc
done
exit 3
