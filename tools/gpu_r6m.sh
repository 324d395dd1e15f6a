# 64-latent persistent forward with the LDS-resident QKV hand-off (LOCAL): persist + model tests,
# mlm64 / seq_clf_ft bench + step tables
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6m
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_persist_gpu.py tests/test_model_gpu.py tests/test_trainer_gpu.py -m gpu -k "persist or mlm or dropout or deterministic or chain_fused or graph" > gpurun_out/r6m/tests.log 2>&1 || { tail -40 gpurun_out/r6m/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6m/tests.log | tail -3
bash tools/gpu_configs.sh mlm64 seq_clf_ft || exit 3
