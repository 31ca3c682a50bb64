# two ranks on the box's one GPU (BLP_DEVICE=0): the N > 1 launch path of the driver's scaling run
set -o pipefail
cd $GRAFT_REPO_ROOT
BLP_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/r2.json 2> gpurun_out/r2.err || exit 1
