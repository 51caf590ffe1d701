STEPS=4 bash scripts/gpu_hm_ab.sh video_codecs_amd/_variants/libhvx_estmemo.so video_codecs_amd/_variants/libhvx_rq2.so video_codecs_amd/_variants/libhvx_estmemo.so video_codecs_amd/_variants/libhvx_rq2.so > gpurun_out/ab_rq2.txt 2>&1 || exit 1
for v in prof_norq prof_rq; do for c in ctu_ldp_rand.bin ctu_ldp_smooth.bin ctu_ra_q32.bin; do
HVX_LIB_PATH=$(pwd)/video_codecs_amd/_variants/libhvx_$v.so timeout -k 10 300 python -u -m tests.hm_profile 0 $c > gpurun_out/cprof_${v}_$c.log 2>&1 || exit 1
done; done
cat gpurun_out/ab_rq2.txt
grep -H -E "mismatches|CTU ticks per job|  TUF4|  TUF8|  TUF16|  TUF32|  CTU " gpurun_out/cprof_*.log
