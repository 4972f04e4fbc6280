#!/usr/bin/env bash
# GPU-box session producing the round's evidence: GPU tests, smoke, bench (+e2e), rocprofv3
# kernel-trace stats of the bench command, and the two PMC passes (FETCH_SIZE / WRITE_SIZE).
# Each GPU step has its own time limit; a fault/abort/timeout ends the script (no more GPU work).
set -u
TAG=${1:-r01}
OUT=gpurun_out
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "!! stop"; exit $rc; fi
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -m pytest tests -m gpu -q
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 3 --e2e
BENCH="bench.py --steps 10 --warmup 2 --no-cpu-baseline"
step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 $BENCH
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_$TAG" -o fetch --output-format csv -- python3 $BENCH
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_$TAG" -o write --output-format csv -- python3 $BENCH
echo "== done"
