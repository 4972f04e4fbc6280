#!/usr/bin/env bash
# Rehearse bench.py's strong-scaling N > 1 flow on ONE GPU (all ranks share the card; the halo
# goes host-staged over gloo, so the values say nothing about xGMI): 4 and 8 ranks over the
# fixed 128-device population at a reduced bucket, devices partition (routed, relayed halo)
# plus the params and hybrid legs; then RCCL requested without fallback must exit non-zero.
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 $OUT/$name.log | cut -c1-1500; if [ $rc -ge 124 ]; then exit $rc; fi; }
run r02_n4_torch python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 4 --transport torch --params 1000000 --steps 3 --warmup 1
run r02_n8_torch python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 8 --transport torch --params 1000000 --steps 3 --warmup 1
run r02_n2_rccl_nofallback python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --params 1000000 --steps 3 --warmup 1
echo "== done"
