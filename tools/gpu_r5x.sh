# GPU suite, then the few-key decode attention kernels (PIO_ATTN_DECODE A/B on the classifier configs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PIO_ATTN_DECODE=1 bash tools/gpu_suite.sh || exit 1
BENCH_CFG=imagenet bash tools/gpu_env_ab.sh - PIO_ATTN_DECODE=1 PIO_ATTN_DECODE=0 || exit 1
BENCH_CFG=mnist bash tools/gpu_env_ab.sh - PIO_ATTN_DECODE=1 PIO_ATTN_DECODE=0 || exit 1
BENCH_CFG=seq_clf bash tools/gpu_env_ab.sh - PIO_ATTN_DECODE=1 PIO_ATTN_DECODE=0 || exit 1
PIO_ATTN_DECODE=1 bash tools/gpu_configs.sh imagenet || exit 1
