# round 4: the SSIM cost inside the HM engine's decision (RA, 4 QPs) vs the restatement, then smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 600 --timeout-method thread -m gpu -k "ssim_rdo and hm_ctu" \
  > gpurun_out/r04_ssim.log 2>&1; rc=$?; tail -8 gpurun_out/r04_ssim.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r04_smoke.log; exit $rc
