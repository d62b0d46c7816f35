#!/bin/bash
# Runs GPU steps in order; stops at the first crash/timeout (rc not in 0/1).
# usage: gpurun_steps.sh "<timeout> <logname> <cmd...>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  t=${spec%% *}; rest=${spec#* }; log=${rest%% *}; cmd=${rest#* }
  echo "=== [$log] $cmd (limit ${t}s)"
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "=== [$log] rc=$rc"; tail -5 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: rc=$rc"; exit $rc; fi
done
