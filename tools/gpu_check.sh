#!/usr/bin/env bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel-trace profile.
# Each GPU step runs under its own time limit; a fault/abort/timeout (exit >= 124) ends the
# script immediately (no further GPU work). Test failures (exit 1) do not stop the later steps.
# Usage (from the repo root, on the box): bash tools/gpu_check.sh [tag]
set -u
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp

step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "!! $name ended with $rc: stopping GPU work"; exit $rc
  fi
  return 0
}

step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 3 --e2e
step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
echo "== done"
