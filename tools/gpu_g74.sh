set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TTIPM_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 1 --warmup 1 > gpurun_out/g74_bench2.json 2> gpurun_out/g74_bench2.err && \
TTIPM_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 1 --warmup 0 --schedule shard > gpurun_out/g74_bench2s.json 2> gpurun_out/g74_bench2s.err
