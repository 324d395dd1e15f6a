# CE head: kernel test, model tests, bench and a step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ce
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -k "cross_entropy or mlm_fused or headline or classifier or deterministic" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ce/test.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ce/test.log; exit 1; }
tail -2 gpurun_out/ce/test.log
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/ce/mlm.json 2>gpurun_out/ce/mlm.err || { echo "bench failed"; tail -20 gpurun_out/ce/mlm.err; exit 1; }
cat gpurun_out/ce/mlm.json
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ce/prof -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/ce/prof.log 2>&1 || { tail gpurun_out/ce/prof.log; exit 1; }
python tools/step_breakdown.py $(find gpurun_out/ce/prof -name "*kernel_trace.csv" | head -1) > gpurun_out/ce/breakdown.md
head -45 gpurun_out/ce/breakdown.md
