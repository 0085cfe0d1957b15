set -o pipefail
mkdir -p gpurun_out
export WSC_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/n2.json 2>gpurun_out/n2.err || { tail -30 gpurun_out/n2.err; exit 1; }
tail -c 1500 gpurun_out/n2.json
