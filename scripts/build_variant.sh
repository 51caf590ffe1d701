# Build a libhvx.so variant of the HM engine with extra defines (A/B experiments on the GPU box).
# usage: bash scripts/build_variant.sh NAME [-DFOO ...]  -> video_codecs_amd/_variants/libhvx_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
C=$R/video_codecs_amd/csrc
mkdir -p $R/video_codecs_amd/_variants $C/_build
/opt/rocm/bin/hipcc --offload-arch=gfx950 ${OPT:--O1} -ffp-contract=off -fPIC -std=c++17 -DHM_WAVES_PER_EU=${WPE:-2} "$@" \
  -c -o $C/_build/hvx_hm_$N.o $C/hvx_hm.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/video_codecs_amd/_variants/libhvx_$N.so \
  $C/_build/hvx_lib.o $C/_build/hvx_hm_$N.o
