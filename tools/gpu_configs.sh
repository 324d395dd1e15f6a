# Bench + per-step kernel breakdown of several bench configs:  bash tools/gpu_configs.sh imagenet long_mlm ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in "$@"; do
  O=gpurun_out/cfg/$cfg
  mkdir -p $O
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench $cfg failed"; tail $O/bench.err; exit 1; }
  cat $O/bench.json
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --config $cfg --steps 6 --warmup 3 > $O/prof.log 2>&1 || { echo "prof $cfg failed"; tail $O/prof.log; exit 1; }
  python tools/step_breakdown.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > $O/breakdown.md
  head -24 $O/breakdown.md
done
echo done
