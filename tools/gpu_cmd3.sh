cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
for cfg in imix ipv6x; do
timeout -k 10 600 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_$cfg.log 2>&1; rc=$?; echo "bench $cfg rc=$rc"; tail -c 1200 gpurun_out/bench_$cfg.log; case $rc in 124|134|137|139) exit $rc;; esac
done
