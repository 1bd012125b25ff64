cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
for cfg in udp64 imix ipv6x; do
timeout -k 10 600 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_$cfg.log 2>&1; rc=$?; echo "bench $cfg rc=$rc"; python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$cfg.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], 'Mpkt/s', d['roofline'] and d['roofline']['achieved'], 'GB/s', d['roofline'] and d['roofline']['kernel_ms'], 'ms')" || tail -5 gpurun_out/bench_$cfg.log; case $rc in 124|134|137|139) exit $rc;; esac
done
cd /tmp && export TMPDIR=/tmp
for cfg in imix ipv6x; do
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 5 --warmup 1 --no-cpu > "$R/gpurun_out/prof_$cfg.log" 2>&1; rc=$?; echo "prof $cfg rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
done
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace -d "$R/gpurun_out/sq1" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/sq1.log" 2>&1; rc=$?; echo "sq1 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES --kernel-trace -d "$R/gpurun_out/sq2" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/gpurun_out/sq2.log" 2>&1; rc=$?; echo "sq2 rc=$rc"; tail -3 "$R/gpurun_out/sq2.log"
