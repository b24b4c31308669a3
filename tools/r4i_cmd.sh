# round 4: the N > 1 bench path rehearsed on one GPU (2 gloo ranks sharing device 0), short run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r4i_bench2.json 2> gpurun_out/r4i_bench2.err; rc=$?
tail -c 1500 gpurun_out/r4i_bench2.json; tail -5 gpurun_out/r4i_bench2.err
exit $rc
