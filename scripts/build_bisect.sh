# -O2 opt-bisect variants of the HM engine (device passes 1..N only; the fault hunt of DESIGN.md §3
# "Build"): bash scripts/build_bisect.sh N1 N2 ... -> video_codecs_amd/_variants/libhvx_bN.so
R=$(cd "$(dirname "$0")/.." && pwd)
for n in "$@"; do
  echo "$n"
done | xargs -P ${JOBS:-4} -I{} env OPT=-O2 bash $R/scripts/build_variant.sh b{} -mllvm -opt-bisect-limit={}
