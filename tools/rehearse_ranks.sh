#!/bin/bash
# GPU box: rehearse bench.py's N > 1 flow (torch.distributed launch, barrier,
# per-rank feeds, max-over-ranks time, summed stats) with 2 and 4 ranks on the
# one GPU (DVC_BENCH_ONE_DEVICE=1: gloo instead of RCCL, which refuses two ranks
# on one device). The 8-GPU runs are the driver's.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ranks
for n in 2 4; do
  DVC_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 2 \
      --no-cpu-baseline > gpurun_out/ranks/n$n.out 2> gpurun_out/ranks/n$n.err
  # rank 0's JSON line (the other ranks' gloo connection notices share stdout)
  grep '^{' gpurun_out/ranks/n$n.out > gpurun_out/ranks/n$n.json
done
