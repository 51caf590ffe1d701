set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/t1.log 2>&1 && echo TESTS_OK && \
timeout -k 10 400 python -u bench.py > gpurun_out/b1.log 2>gpurun_out/b1.err && echo BENCH_OK
