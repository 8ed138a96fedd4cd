#!/bin/bash
# stamps of the kH2 train passes vs the recomputing ones (libh2S: -DDXRL_H2_STAMPS=1), then PPO 4 x 4
# with vs without the stored layer-2 rows, interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for v in both none both none; do
  DXRL_LIB=ab/libh2S.so DXRL_FUSED_DIAG=8 VARIANT=$v timeout -k 10 120 python tools/h2_stamps.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/r06/h2_stamps.log || exit 1
done
for i in 1 2; do for f in "" "--recompute-h2"; do
  timeout -k 10 200 python bench.py --epochs 4 --minibatches 4 --steps 10 --warmup 2 --no-cpu-baseline --no-roofline $f > gpurun_out/r06/ppo.log 2>&1 || exit 2
  echo "ppo ${f:-reuse} $(grep '^{' gpurun_out/r06/ppo.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), d["ms_per_step"], d.get("phases_ms"))')" >> gpurun_out/r06/ppo_ab.log
done; done
cat gpurun_out/r06/ppo_ab.log
