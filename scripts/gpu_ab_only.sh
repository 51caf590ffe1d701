# A/B of HM-engine variants only (no parity): the tree's libhvx.so first, then each variant
set -o pipefail
bash scripts/gpu_hm_ab.sh "$@"
