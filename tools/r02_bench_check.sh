cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > gpurun_out/r02_bench_full.json 2> gpurun_out/r02_bench_full.err || exit 1
BENCH_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r02_bench_ws2.json 2> gpurun_out/r02_bench_ws2.err || exit 1
