# rehearsal of the driver's N>1 bench launch: 2 ranks on the box's one GPU over gloo
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 6 --warmup 2 \
  > gpurun_out/d2.json 2> gpurun_out/d2.err
echo rc=$?
