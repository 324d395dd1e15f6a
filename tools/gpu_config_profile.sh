# Per-step kernel breakdown of one bench config:  bash tools/gpu_config_profile.sh <config>
set -o pipefail
cfg=${1:-imagenet}
mkdir -p gpurun_out/cfg_$cfg
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 > gpurun_out/cfg_$cfg/bench.json 2> gpurun_out/cfg_$cfg/bench.err || { tail gpurun_out/cfg_$cfg/bench.err; exit 1; }
cat gpurun_out/cfg_$cfg/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cfg_$cfg/prof -o run -- python bench.py --config $cfg --steps 6 --warmup 3 > gpurun_out/cfg_$cfg/prof.log 2>&1 || { tail gpurun_out/cfg_$cfg/prof.log; exit 1; }
python tools/step_breakdown.py $(find gpurun_out/cfg_$cfg/prof -name "*kernel_trace.csv" | head -1) > gpurun_out/cfg_$cfg/breakdown.md
head -30 gpurun_out/cfg_$cfg/breakdown.md
