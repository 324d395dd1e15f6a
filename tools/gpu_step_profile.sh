# Headline step profile: bench (20 steps) + rocprofv3 kernel trace of a short bench run, reduced
# to a per-step kernel breakdown (tools/step_breakdown.py).
set -o pipefail
mkdir -p gpurun_out/step
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/step/bench.json 2> gpurun_out/step/bench.err || { tail gpurun_out/step/bench.err; exit 1; }
cat gpurun_out/step/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/step/prof -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/step/prof.log 2>&1 || { tail gpurun_out/step/prof.log; exit 1; }
python tools/step_breakdown.py $(find gpurun_out/step/prof -name "*kernel_trace.csv" | head -1) > gpurun_out/step/breakdown.md
head -40 gpurun_out/step/breakdown.md
