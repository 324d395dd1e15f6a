# persistent 64-latent block backward (chain_block_bwd): kernel test vs step launches, model tests,
# mlm64 / seq_clf_ft bench + step tables
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6n
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_attn_bwd_selfattn_gpu.py -m gpu -k "block_boundary" > gpurun_out/r6n/ktest.log 2>&1 || { tail -40 gpurun_out/r6n/ktest.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6n/ktest.log | tail -2
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_trainer_gpu.py -m gpu -k "mlm or dropout or deterministic or chain_fused or graph or trainer" > gpurun_out/r6n/tests.log 2>&1 || { tail -40 gpurun_out/r6n/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6n/tests.log | tail -2
bash tools/gpu_configs.sh mlm64 seq_clf_ft || exit 3
