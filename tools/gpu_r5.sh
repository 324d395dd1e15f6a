# round-5 iteration: the persistent-block tests first, then the model tests, bench A/B
# (PERCEIVER_PERSIST=0/1) and a step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest tests/test_persist_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5/persist.log 2>&1; rc=$?
tail -15 gpurun_out/r5/persist.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$R5_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $R5_TESTS -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5/tests.log 2>&1; rc=$?
  tail -5 gpurun_out/r5/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for ps in 0 1; do
  PERCEIVER_PERSIST=$ps timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/r5/mlm_p$ps.json 2>gpurun_out/r5/mlm_p$ps.err || { echo "bench failed"; tail -20 gpurun_out/r5/mlm_p$ps.err; exit 1; }
  cat gpurun_out/r5/mlm_p$ps.json
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/prof -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/r5/prof.log 2>&1 || { tail gpurun_out/r5/prof.log; exit 1; }
python tools/step_breakdown.py $(find gpurun_out/r5/prof -name "*kernel_trace.csv" | head -1) > gpurun_out/r5/breakdown.md
head -40 gpurun_out/r5/breakdown.md
