# GPU suite, then configs (appended slab-job workgroups spread over every grid row)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
bash tools/gpu_configs.sh imagenet mnist mlm256 lartpc || exit 1
