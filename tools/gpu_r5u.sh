# GPU suite, then a decoder's K|V projection folded into the encoder's last per-sample block
# (PIO_SB_KV A/B on imagenet / mnist)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
BENCH_CFG=imagenet bash tools/gpu_env_ab.sh - PIO_SB_KV=1 PIO_SB_KV=0 || exit 1
BENCH_CFG=mnist bash tools/gpu_env_ab.sh - PIO_SB_KV=1 PIO_SB_KV=0 || exit 1
