# Framework (non-pio) ops in a step, attributed to Python stacks (eager steps: the profiler does not
# see inside a replayed graph):  bash tools/gpu_stacks.sh <config>...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/stacks
for cfg in "$@"; do
  timeout -k 10 300 python bench.py --config $cfg --no-graph --steps 3 --warmup 2 --profile-steps 2 --profile-stacks 6 > gpurun_out/stacks/$cfg.json 2> gpurun_out/stacks/$cfg.log || { echo "stacks $cfg failed"; tail -20 gpurun_out/stacks/$cfg.log; exit 1; }
  grep -A7 -E "^aten\." gpurun_out/stacks/$cfg.log | head -90
done
