#!/bin/bash
# Runs bench.py once per "VAR=value ..." argument (each under its own time limit) and prints
# the ms/step of each: a tuning sweep over the kernels' env knobs.
#   bash tools/sweep_env.sh "PIO_CE_DH_WGS=256" "PIO_CE_DH_WGS=1024" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for cfg in "" "$@"; do
  out=$(env $cfg timeout -k 10 120 python bench.py --steps 50 --warmup 5 2>/dev/null) || { echo "FAILED: $cfg"; exit 1; }
  echo "$cfg -> $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["ms_per_step"], d["value"])')" | tee -a gpurun_out/sweep.log
done
