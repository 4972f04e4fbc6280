#!/usr/bin/env bash
# Round-2 session 3: bench.py's N > 1 flow rehearsed on ONE GPU after the watchdog change (4 and 8
# ranks, torch transport; RCCL without fallback must exit 3), then a rocprofv3 kernel-trace
# summary of the default N = 1 bench.
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 $OUT/$name.log | cut -c1-1500; if [ $rc -ge 124 ]; then exit $rc; fi; }
run s3_n4_torch 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 4 --transport torch --allow-fallback --params 1000000 --steps 3 --warmup 1
run s3_n8_torch 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 8 --transport torch --allow-fallback --params 1000000 --steps 3 --warmup 1
run s3_n2_rccl_nofallback 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --params 1000000 --steps 3 --warmup 1
run s3_rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_s3" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-live-traffic
echo "== done"
