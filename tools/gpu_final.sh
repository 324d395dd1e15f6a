# round-end evidence: the GPU suite, then bench + per-step kernel breakdown of every bench config
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
bash tools/gpu_configs.sh mlm256 seq_clf seq_clf_ft imagenet mnist long_mlm lartpc || exit 1
