#!/usr/bin/env bash
# Round 3: the N > 1 bench flow rehearsed on ONE GPU (ranks share the card).
#
#   bash tools/gpu_rehearse_r03.sh CASE [CASE ...]
#
# Cases:
#   n2_carve      2 ranks, devices partition, halo over the gloo group ("torch-gloo", not comparable),
#                 halo / relay carve from placement-calibrated (>= 1 GiB) stacks
#   n8_relay      8 ranks, torch transport: params headline + devices / hybrid2 / weak legs, relayed plan
#   n8_rccl       8 ranks, the default rccl transport, which RCCL refuses for ranks sharing one device:
#                 the params headline (no exchange) is still measured and printed, every leg that
#                 exchanges reports the transport error; exit status 0
#   n4_leg_budget 4 ranks, torch transport, --leg-seconds 1: the first exchanging leg runs out of its
#                 budget, rank 0 prints the line with the legs measured so far and that leg's error
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
# launch N PORT ARGS...: the argv of an N-rank bench run (timeout runs programs, not shell functions)
launch() { local n=$1 port=$2; shift 2
  L=(python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port "$port"
     bench.py --gpus "$n" "$@"); }
for c in "$@"; do
  case "$c" in
    n2_carve) launch 2 29631 --transport torch --devices 32 --params 17000000 --placement-candidates 2 \
                --steps 3 --warmup 1 --partition devices --no-extra-legs --no-weak-leg; run n2_carve "${L[@]}" ;;
    n8_relay) launch 8 29632 --transport torch --params 1000000 --steps 3 --warmup 1; run n8_relay "${L[@]}" ;;
    n8_rccl) launch 8 29633 --params 1000000 --steps 3 --warmup 1; run n8_rccl "${L[@]}" ;;
    n4_leg_budget) launch 4 29634 --transport torch --params 8000000 --steps 3 --warmup 1 \
                     --leg-seconds 1; run n4_leg_budget "${L[@]}" ;;
    *) echo "unknown case $c"; exit 2 ;;
  esac
done
echo "== done"
