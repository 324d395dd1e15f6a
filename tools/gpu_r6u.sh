# round-6 end evidence (after the PE offset fold, split rule, dropout hash hoist and CE small-vocab pass 2): full GPU suite, smoke, every config's bench + step table
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 2
bash tools/gpu_configs.sh mlm256 mlm64 seq_clf seq_clf_ft imagenet mnist long_mlm lartpc || exit 3
