#!/usr/bin/env bash
# Round-2 session-3 closing evidence after the placement-calibrated stacks: whole GPU suite, smoke,
# the default bench line (CPU baselines, live PMC traffic), a rocprofv3 kernel-trace summary of the
# bench, and the N > 1 flow rehearsed with 4 and 8 ranks on this one GPU (gloo halo).
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "!! stop"; exit $rc; fi
}
step ${PFX:-fin}_pytest_gpu 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider
step ${PFX:-fin}_smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step ${PFX:-fin}_bench 500 python bench.py --steps 20 --warmup 5
step ${PFX:-fin}_rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${PFX:-fin}" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic
step ${PFX:-fin}_n4_torch 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 4 --transport torch --params 1000000 --steps 3 --warmup 1
step ${PFX:-fin}_n8_torch 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 8 --transport torch --params 1000000 --steps 3 --warmup 1
echo "== done"
