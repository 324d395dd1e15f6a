# GPU suite, then seq_clf_ft (one dropout seed pool per encoder pass) with its step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
bash tools/gpu_configs.sh seq_clf_ft || exit 1
grep -E "at::|Fill|distribution" gpurun_out/cfg/seq_clf_ft/breakdown.md || true
