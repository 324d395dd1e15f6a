# GPU suite, then A/B of the slab reduction carried by the bf16 attention backward
# (PIO_ATTN_SLAB=1, two workgroups per CU) against the next chain kernel carrying it, and a step
# profile of the headline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
bash tools/gpu_env_ab.sh - PIO_ATTN_SLAB=1 PIO_ATTN_SLAB=0 || exit 1
BENCH_CFG=seq_clf_ft bash tools/gpu_env_ab.sh - - || exit 1
bash tools/gpu_step_profile.sh || exit 1
