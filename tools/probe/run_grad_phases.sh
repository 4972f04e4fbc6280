#!/usr/bin/env bash
# Build and run the gradient-kernel phase probe (GPU box): bash tools/probe/run_grad_phases.sh
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=${TMPDIR:-/tmp}/grad_phases
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I"$ROOT/include" \
    "$ROOT/tools/probe/grad_phases.hip" -o "$OUT"
"$OUT"
echo "-- LDS capped at 64 KiB (chunks):"
CFA_GRAD_LDS_CAP=65536 "$OUT"
echo "-- population form (config 3: 32 evaluations, batch split):"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I"$ROOT/include" \
    "$ROOT/tools/probe/grad_phases_pop.hip" -o "$OUT.pop"
"$OUT.pop"
