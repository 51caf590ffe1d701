# Round-end evidence, part 2: the HM encoder seams (leaf seams, CTU seam, batched CTU seam); $1 = pytest -k expression
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_hm_seam.py -v --timeout 900 --timeout-method thread -m gpu -k "$1" \
  > gpurun_out/final_seams_$2.log 2>&1; rc=$?; tail -12 gpurun_out/final_seams_$2.log
exit $rc
