#!/bin/bash
# N > 1 rehearsal on a one-GPU box: bench.py under torch.distributed.run with 2
# ranks sharing cuda:0 over gloo (HBK_BENCH_REHEARSE=1), configs 5, 4 and 2,
# plus the distributed GPU tests. Exercises sharding, the per-step gradient
# all-reduce between the two launches of a train step and the max-over-ranks
# timing; the numbers it prints are not measurements.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp HBK_BENCH_REHEARSE=1
mkdir -p gpurun_out
for C in ${CONFIGS:-5 4 2}; do
  echo "=== rehearse config $C (2 ranks on cuda:0, gloo)"
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29500 + C)) bench.py --gpus 2 --config $C --steps 2 --warmup 1 --no-cpu \
    > gpurun_out/rehearse_c$C.json 2> gpurun_out/rehearse_c$C.err || { tail -40 gpurun_out/rehearse_c$C.err; exit 1; }
  cut -c1-400 gpurun_out/rehearse_c$C.json
done
