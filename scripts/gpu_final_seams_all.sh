# Round-end evidence, part 2 in one call: the compressCtu seams (per-CTU and batched), then the leaf seams
set -o pipefail
bash scripts/gpu_final_seams.sh cu_seam cu || exit $?
bash scripts/gpu_final_seams.sh hvx_seams leaf
