#!/bin/bash
# Copy the judged summaries of a tools/profile_round.sh run (gpurun_out/r) into profiles/$1.
set -eu
R=${1:?round dir, e.g. r03}
D=profiles/$R
mkdir -p $D
cp gpurun_out/r/*.json gpurun_out/r/*.jsonl gpurun_out/r/trace_summary_*.txt gpurun_out/r/session.log $D/ 2>/dev/null || true
for p in gpurun_out/r/prof_*/; do
  c=$(basename $p); c=${c#prof_}
  f=$(ls $p/*kernel_stats.csv $p/*/*kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] && cp "$f" $D/kernel_stats_$c.csv
done
for p in pmc_fetch pmc_write pmc_mfma pmc_sq; do
  f=$(ls gpurun_out/r/$p/*counter_collection.csv gpurun_out/r/$p/*/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && mkdir -p $D/pmc && cp "$f" $D/pmc/$p.csv
done
ls $D
