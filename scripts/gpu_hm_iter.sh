# one engine iteration: HM CTU parity, the headline step, the per-category profile
set -o pipefail
bash scripts/gpu_hm_quick.sh "$@" || exit $?
bash scripts/gpu_hm_prof.sh > /dev/null 2>&1; grep -E "bench step|TUF |COEF |C.walk|rdoq|xform|CTU " gpurun_out/hprof.log
