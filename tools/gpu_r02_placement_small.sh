#!/usr/bin/env bash
# Placement calibration at one N = 8 rank's share of the bench population (16 devices x 25M,
# 1.6 GB stacks) on one GPU: plain allocation vs calibrated, alternating processes.
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python bench.py --devices 16 --steps 20 --warmup 3 --no-cpu-baseline --no-live-traffic --placement-candidates 1 > $OUT/ps16_plain_$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --devices 16 --steps 20 --warmup 3 --no-cpu-baseline --no-live-traffic > $OUT/ps16_placed_$r.log 2>&1 || exit 1
done
echo done
