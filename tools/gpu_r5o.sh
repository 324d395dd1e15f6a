# the main configs, then the GPU suite (build without SLP vectorisation)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_configs.sh mlm256 imagenet mnist lartpc seq_clf || exit 1
bash tools/gpu_suite.sh || exit 1
