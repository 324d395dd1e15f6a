# the boundary kernel with the layer below's attention backward fused in (N = 64 latents):
# kernel + model tests, then mlm64 / seq_clf_ft / mlm256 bench + step tables
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6k
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attn_bwd_selfattn_gpu.py tests/test_model_gpu.py -m gpu -k "fused_attention or chain_fused or mlm or dropout or deterministic or bf16_dqkv or selfattn or two_wave or classifier or graph" > gpurun_out/r6k/tests.log 2>&1 || { tail -40 gpurun_out/r6k/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6k/tests.log | tail -3
bash tools/gpu_configs.sh mlm64 seq_clf_ft || exit 3
