set -o pipefail
mkdir -p gpurun_out/seam
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "intra" > gpurun_out/intra2.log 2>&1 || { tail -20 gpurun_out/intra2.log; exit 1; }
tail -3 gpurun_out/intra2.log
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_i2.log 2>&1 || exit 1
tail -1 gpurun_out/bench_i2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['intra_first_pass'])"
HVX_SEAM_LOG_DIR=$(pwd)/gpurun_out/seam timeout -k 10 700 python -u -m pytest tests/test_hm_seam.py -m gpu -x -v --timeout-method thread --durations=0 > gpurun_out/seam_tests.log 2>&1
rc=$?; tail -12 gpurun_out/seam_tests.log; exit $rc
