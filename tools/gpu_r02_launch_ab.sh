#!/usr/bin/env bash
# bench.py with the library's default mix launch shape (2 workgroups per CU, 4 float4 per lane)
# against 1 workgroup per CU x 2 float4 per lane (CFA_BLOCKS_PER_CU / CFA_VEC_PER_LANE), alternating
# processes on one box; placement-calibrated stacks in both.
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-live-traffic > $OUT/la_default_$r.log 2>&1 || exit 1
  CFA_BLOCKS_PER_CU=1 CFA_VEC_PER_LANE=2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-live-traffic > $OUT/la_b1v2_$r.log 2>&1 || exit 1
  echo "$r: $(grep -h '^{' $OUT/la_default_$r.log | cut -c90-120) | $(grep -h '^{' $OUT/la_b1v2_$r.log | cut -c90-120)"
done
