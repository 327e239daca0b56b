#!/bin/bash
# round 3 (session 2): fp32 parity-mode tile variants (the runtime's pick vs forced C64 / C128 shapes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fp32v
export TMPDIR=/tmp PREC=fp32
for cfg in "pick:" "c64v0:BUGSEG_BNECK_VARIANT_C64=0" "c64v1:BUGSEG_BNECK_VARIANT_C64=1" "c128v0:BUGSEG_BNECK_VARIANT_C128=0" "pick2:"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  o=gpurun_out/fp32v/$name
  env $envs timeout -k 10 150 python scripts/batch_probe.py 32 > $o.probe 2>&1 || { echo "probe $name failed"; tail $o.probe; exit 1; }
  grep -E "forward|C64|C128" $o.probe | head -8
done
