#!/usr/bin/env bash
# Round 3: the N > 1 bench flow rehearsed on ONE GPU (ranks share the card, halo over the gloo
# group: the line says "torch-gloo", "comparable": false). Case A exercises the halo / relay carve
# from placement-calibrated (>= 1 GiB) stacks at 2 ranks; case B the 8-rank relayed plan.
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  echo "== $name ($(date +%T))"
  timeout -k 10 300 "$@" > "$OUT/r03_rehearse_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '^{' "$OUT/r03_rehearse_$name.log" | cut -c1-300; tail -n 2 "$OUT/r03_rehearse_$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run n2_carve python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 \
  bench.py --gpus 2 --transport torch --devices 32 --params 17000000 --placement-candidates 2 --steps 3 --warmup 1 \
  --partition devices --no-extra-legs --no-weak-leg
run n8_relay python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29632 \
  bench.py --gpus 8 --transport torch --params 1000000 --steps 3 --warmup 1
echo "== done"
