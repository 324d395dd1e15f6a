# GPU suite (decode attention forward + backward on), then the few-key decode attention kernels
# (PIO_ATTN_DECODE 2 = fwd + bwd, 1 = bwd only, 0 = off) on the image classifier configs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PIO_ATTN_DECODE=2 bash tools/gpu_suite.sh || exit 1
BENCH_CFG=imagenet bash tools/gpu_env_ab.sh - PIO_ATTN_DECODE=2 PIO_ATTN_DECODE=1 PIO_ATTN_DECODE=0 || exit 1
BENCH_CFG=mnist bash tools/gpu_env_ab.sh - PIO_ATTN_DECODE=2 PIO_ATTN_DECODE=1 PIO_ATTN_DECODE=0 || exit 1
PIO_ATTN_DECODE=2 bash tools/gpu_configs.sh mnist || exit 1
