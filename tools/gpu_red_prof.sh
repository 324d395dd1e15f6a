# forced 1-rank reducer: kernel timelines of one step with per-bucket updates on / off; attn_bwd trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/redp
timeout -k 5 60 ./tools/trace/attn_bwd_trace > gpurun_out/redp/attn_bwd_trace.txt 2>&1 || { echo trace failed; cat gpurun_out/redp/attn_bwd_trace.txt; exit 1; }
cat gpurun_out/redp/attn_bwd_trace.txt
for bu in 0 1; do
  PERCEIVER_BUCKET_UPDATE=$bu PERCEIVER_BENCH_FORCE_REDUCER=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/redp/p$bu -o run -- python bench.py --steps 6 --warmup 3 > gpurun_out/redp/prof_$bu.log 2>&1 || { echo "prof $bu failed"; tail -20 gpurun_out/redp/prof_$bu.log; exit 1; }
  python tools/step_timeline.py $(find gpurun_out/redp/p$bu -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > gpurun_out/redp/timeline_$bu.txt
  echo "== bucket_update=$bu"; tail -40 gpurun_out/redp/timeline_$bu.txt
done
