# GPU suite, then the PE projection weight gradients on a side stream (PIO_PE_SIDE A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
BENCH_CFG=imagenet bash tools/gpu_env_ab.sh - PIO_PE_SIDE=1 PIO_PE_SIDE=0 || exit 1
BENCH_CFG=mnist bash tools/gpu_env_ab.sh - PIO_PE_SIDE=1 PIO_PE_SIDE=0 || exit 1
