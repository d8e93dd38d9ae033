#!/bin/bash
# GPU-call driver: runs each argument as one step (each step carries its own `timeout -k`), in order; a step that
# fails its tests (exit 1) does not stop the rest, anything else (fault, abort, time limit) ends the call there.
mkdir -p gpurun_out
for step in "$@"; do
  echo "== $(date +%T) $step"
  bash -c "$step"
  rc=$?
  echo "== rc $rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
