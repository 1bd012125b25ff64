cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
for cfg in udp64 imix ipv6x; do
timeout -k 10 600 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_$cfg.log 2>&1; rc=$?; echo "bench $cfg rc=$rc"; python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$cfg.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], 'Mpkt/s', d['roofline'] and d['roofline']['achieved'], 'GB/s', d['roofline'] and d['roofline']['kernel_ms'], 'ms')" || tail -5 gpurun_out/bench_$cfg.log; case $rc in 124|134|137|139) exit $rc;; esac
done
cd /tmp && export TMPDIR=/tmp
for cfg in udp64 imix ipv6x; do
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/prof_$cfg.log" 2>&1; rc=$?; echo "prof $cfg rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
grep -E 'dissect|Name' "$R/gpurun_out/prof_$cfg/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-160
done
