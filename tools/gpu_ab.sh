#!/bin/bash
# One A/B session: the GPU test suite on the in-tree library (TESTS=1), then
# kernel times (tools/gpu_variants.sh) and PMC fetch / write bytes
# (tools/gpu_pmc_variants.sh) of library variants built with
# tools/build_variant.sh.  Each GPU step has its own time limit; a failure
# ends the script.  Outputs under gpurun_out/ (var/, pmcv/, ab/).
#   TESTS=1 PYTEST_K="device_parity or fuzz" VARS="prev base" CFGS=ipv6x,udp64 PMC_VARS="prev base" PMC_CFG=ipv6x
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/ab/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -n 3 gpurun_out/ab/pytest_gpu.log; [ $rc = 0 ] || exit $rc
fi
if [ -n "$VARS" ]; then
  VARS="$VARS" CFGS="${CFGS:-udp64,imix,ipv6x}" bash tools/gpu_variants.sh || exit 1
fi
if [ -n "$PMC_VARS" ]; then
  VARS="$PMC_VARS" CFG="${PMC_CFG:-ipv6x}" PASSES="${PASSES:-fetch write}" bash tools/gpu_pmc_variants.sh || exit 1
fi
exit 0
