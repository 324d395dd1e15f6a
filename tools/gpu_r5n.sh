# GPU suite, then the image configs (staggered sample order of the PE attention backward)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
bash tools/gpu_configs.sh imagenet mnist || exit 1
