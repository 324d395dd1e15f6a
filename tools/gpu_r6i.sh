# LN-linear backward: per-operand vector loads (odd Kin) + the dXn tile aliased over the chunk-loop
# buffers (LArTPC's 160-channel variant: 100 -> 57 KB, two workgroups per CU): microbench, the
# LN-linear / split-PE / model GPU tests, then lartpc / mlm256 / imagenet bench + step tables
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6i
timeout -k 10 240 python -u tools/lartpc_kv_bench.py > gpurun_out/r6i/kv.log 2>&1 || { tail -20 gpurun_out/r6i/kv.log; exit 1; }
cat gpurun_out/r6i/kv.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu > gpurun_out/r6i/tests.log 2>&1 || { tail -30 gpurun_out/r6i/tests.log; exit 1; }
tail -3 gpurun_out/r6i/tests.log
bash tools/gpu_configs.sh lartpc mlm256 imagenet || exit 3
