#!/bin/bash
# bench.py --config <cfg> once per "VAR=value ..." argument (first run: no override):
#   bash tools/sweep_cfg.sh <cfg> "PIO_X=1" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
cfgname=$1; shift
for cfg in "" "$@"; do
  out=$(env $cfg timeout -k 10 180 python bench.py --config "$cfgname" --steps 20 --warmup 5 2>/dev/null) || { echo "FAILED: $cfgname $cfg"; exit 1; }
  echo "$cfgname $cfg -> $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d["ms_per_step"], d["value"])')" | tee -a gpurun_out/sweep.log
done
