#!/usr/bin/env bash
# Rehearse bench.py's N > 1 flow with 2 ranks on ONE GPU (the only multi-rank setup a 1-GPU box
# allows): torch transport (gloo, host-staged halo), then the rccl transport, which RCCL rejects
# for two ranks on one device -> exercises bench's fallback path.
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -n 6 $OUT/$name.log; if [ $rc -ge 124 ]; then exit $rc; fi; }
run n2_torch python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --transport torch --devices-per-gpu 16 --steps 3 --warmup 1
run n2_rccl_fallback python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --devices-per-gpu 16 --steps 3 --warmup 1
