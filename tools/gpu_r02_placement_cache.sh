#!/usr/bin/env bash
# Placement calibration: rejected candidates freed to the driver (then the settle loop) vs left in
# torch's caching allocator, alternating processes on one box.
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for r in 1 2; do
  for v in release keep; do
    extra=""; [ $v = release ] && extra="--placement-release"
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-live-traffic $extra > $OUT/pc_${v}_$r.log 2>&1 || exit 1
    echo "$v $r: $(grep '^{' $OUT/pc_${v}_$r.log | cut -c1-120)"
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider > $OUT/pc_pytest.log 2>&1 || exit 1
tail -1 $OUT/pc_pytest.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 8 --transport torch --params 1000000 --steps 3 --warmup 1 > $OUT/pc_n8.log 2>&1 || exit 1
grep '^{' $OUT/pc_n8.log | cut -c1-200
