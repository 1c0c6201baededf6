#!/bin/bash
# Runs every tools/call_repro/build/repro_* (one GPU process each, seconds); summary in OUT (default
# gpurun_out/call_repro.log). A binary that fails to launch is reported, not retried.
R=$(cd "$(dirname "$0")/../.." && pwd)
OUT=${OUT:-$R/gpurun_out/call_repro.log}
mkdir -p "$(dirname "$OUT")"
cat "$R/tools/call_repro/build/flags.txt" > "$OUT"
for b in "$R"/tools/call_repro/build/repro_*; do
  t=$(basename "$b")
  timeout -k 5 60 "$b" "$R/data" "$t" >> "$OUT" 2>&1
  rc=$?
  if [ $rc -ge 2 ]; then echo "$t: exit $rc" >> "$OUT"; fi
  if [ $rc -ge 124 ]; then break; fi
done
echo done >> "$OUT"
