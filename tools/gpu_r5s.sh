# GPU suite, then the next cross layer's query path folded into the per-sample blocks
# (PIO_SB_POST A/B on imagenet / mnist) and the image configs' step profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
BENCH_CFG=imagenet bash tools/gpu_env_ab.sh - PIO_SB_POST=1 PIO_SB_POST=0 || exit 1
BENCH_CFG=mnist bash tools/gpu_env_ab.sh - PIO_SB_POST=1 PIO_SB_POST=0 || exit 1
bash tools/gpu_configs.sh imagenet mnist lartpc || exit 1
