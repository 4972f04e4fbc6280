#!/usr/bin/env bash
# Round-2 quick GPU session: population/transport GPU tests, smoke, the default bench line, and
# single-GPU emulations of one rank's work at N = 8 (params slice: P/8 per bucket for all 128
# devices; device block: 16 devices of the ring, compute only).
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "!! stop"; exit $rc; fi
}
step pytest_pop 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_population.py -m gpu
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 400 python bench.py --steps 20 --warmup 3
step emu_params8 200 python bench.py --steps 20 --warmup 3 --params 3125000 --no-cpu-baseline
step emu_devices8 200 python bench.py --steps 20 --warmup 3 --devices 16 --no-cpu-baseline
echo "== done"
