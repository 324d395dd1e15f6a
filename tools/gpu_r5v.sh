# GPU suite, then seq_clf_ft (dropout seeds staged per replay: no generator kernels) and the
# configs' step profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
BENCH_CFG=seq_clf_ft bash tools/gpu_env_ab.sh - - || exit 1
bash tools/gpu_configs.sh seq_clf_ft imagenet mnist || exit 1
