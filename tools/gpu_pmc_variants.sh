#!/bin/bash
# PMC passes (tools/gpu_pmc.sh) per library variant: VARS="old base" CFG=ipv6x
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
LIB=$R/netsniff-ng_amd/libnsdissect.so
mkdir -p gpurun_out/pmcv
cp "$LIB" gpurun_out/pmcv/base.so
for v in $VARS; do
  if [ "$v" = base ]; then cp gpurun_out/pmcv/base.so "$LIB"; else cp "$R/variants/$v/libnsdissect.so" "$LIB"; fi
  rm -rf gpurun_out/pmc
  echo "== $v"
  bash tools/gpu_pmc.sh || { cp gpurun_out/pmcv/base.so "$LIB"; exit 1; }
  mv gpurun_out/pmc gpurun_out/pmcv/$v
done
cp gpurun_out/pmcv/base.so "$LIB"
rm -f gpurun_out/pmcv/base.so
exit 0
