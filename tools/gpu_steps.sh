#!/bin/bash
# Run named GPU steps in one gpurun call; each step has its own time limit, output in
# gpurun_out/$OUTDIR/<name>.log; stops at the first failing step.
#   OUTDIR=b tools/gpu_steps.sh "name|seconds|command" ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-s}
mkdir -p $O
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  echo "== $name $(date +%T)" | tee -a $O/session.log
  timeout -k 10 "$t" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  tail -2 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc" | tee -a $O/session.log; exit $rc; fi
done
echo done | tee -a $O/session.log
