#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over one bench config.
#   CFG=imix  PASSES="sq1 sq2 fetch"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(pwd)
O=$R/gpurun_out/pmc
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
declare -A G
G[sq1]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
G[sq2]="SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"
G[fetch]="FETCH_SIZE"
G[write]="WRITE_SIZE"
G[tcc]="TCC_HIT_sum TCC_MISS_sum"
G[req]="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
G[wreq]="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
for g in ${PASSES:-sq1 sq2}; do
  timeout -s KILL 120 rocprofv3 --pmc ${G[$g]} --kernel-trace -d "$O/${CFG}_$g" -o run --output-format csv -- python3 "$R/bench.py" --config ${CFG:-udp64} --steps 3 --warmup 1 --no-cpu --no-e2e --no-replay --no-legs --no-pmc --no-bpf > "$O/${CFG}_$g.log" 2>&1; rc=$?
  echo "pmc $g rc=$rc"; [ $rc = 0 ] || { tail -5 "$O/${CFG}_$g.log"; exit $rc; }
done
python3 "$R/tools/pmc_summary.py" "$O" "${CFG:-udp64}"
exit 0
