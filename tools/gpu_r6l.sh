# split-KV for one-wave-per-SIMD cross-attention forwards (seq_clf / seq_clf_ft): bench + tables
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_configs.sh seq_clf_ft seq_clf || exit 3
