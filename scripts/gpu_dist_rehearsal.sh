# Rehearsal of the multi-GPU bench path (closed segments per rank + the DPB gather + max-over-ranks
# timing) with two ranks on the one GPU of a gpurun box: gloo instead of RCCL (two ranks cannot share a
# device under RCCL), 8 segments per rank.  The 8-GPU run itself is the driver's.
set -o pipefail
mkdir -p gpurun_out
HVX_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 5 --segs 8 > gpurun_out/dist_rehearsal.log 2>&1
rc=$?
grep '^{' gpurun_out/dist_rehearsal.log | cut -c1-3000
exit $rc
