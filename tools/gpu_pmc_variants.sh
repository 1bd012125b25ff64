#!/bin/bash
# PMC passes (tools/gpu_pmc.sh) per library variant: VARS="old base" CFG=ipv6x
# (bench.py loads the in-tree library: each variant is copied over it for its
# passes, and the product build is restored on any exit, a killed run included)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
LIB=$R/netsniff-ng_amd/libnsdissect.so
mkdir -p gpurun_out/pmcv
cp "$LIB" gpurun_out/pmcv/base.so
trap 'cp gpurun_out/pmcv/base.so "$LIB"' EXIT
for v in $VARS; do
  if [ "$v" = base ]; then cp gpurun_out/pmcv/base.so "$LIB"; else cp "$R/variants/$v/libnsdissect.so" "$LIB"; fi
  rm -rf gpurun_out/pmc
  echo "== $v"
  bash tools/gpu_pmc.sh || exit 1
  mv gpurun_out/pmc gpurun_out/pmcv/$v
done
exit 0
