set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 ; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log &&
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.log 2>&1 && tail -3 gpurun_out/bench1.log
