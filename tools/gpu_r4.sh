# round-4 iteration: correctness of the touched kernels first, then bench + step profile, traces,
# forced-reducer timelines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_fuzz_gpu.py tests/test_model_gpu.py -q -k "not lartpc" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4/test.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4/test.log | tail -30
[ $rc -le 1 ] || { echo "test run aborted rc=$rc"; tail -30 gpurun_out/r4/test.log; exit $rc; }
tail -2 gpurun_out/r4/test.log
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/r4/mlm.json 2>gpurun_out/r4/mlm.err || { echo "bench failed"; tail -20 gpurun_out/r4/mlm.err; exit 1; }
cat gpurun_out/r4/mlm.json
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4/prof -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/r4/prof.log 2>&1 || { tail gpurun_out/r4/prof.log; exit 1; }
python tools/step_breakdown.py $(find gpurun_out/r4/prof -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > gpurun_out/r4/breakdown.md
head -45 gpurun_out/r4/breakdown.md
timeout -k 5 60 ./tools/trace/attn_bwd_trace > gpurun_out/r4/attn_bwd_trace.txt 2>&1 || { echo trace failed; cat gpurun_out/r4/attn_bwd_trace.txt; exit 1; }
cat gpurun_out/r4/attn_bwd_trace.txt
for bu in 0 1; do
  PERCEIVER_BUCKET_UPDATE=$bu PERCEIVER_BENCH_FORCE_REDUCER=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4/red$bu -o run -- python bench.py --steps 6 --warmup 3 > gpurun_out/r4/red_$bu.log 2>&1 || { echo "prof $bu failed"; tail -20 gpurun_out/r4/red_$bu.log; exit 1; }
  python tools/step_timeline.py $(find gpurun_out/r4/red$bu -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > gpurun_out/r4/timeline_$bu.txt
done
echo done
