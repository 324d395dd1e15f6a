# round-end re-run after the decode-attention backward: the GPU suite at the defaults, then the
# classifier configs' bench + step profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
bash tools/gpu_configs.sh imagenet mnist seq_clf || exit 1
