# GPU suite, then A/B of the appended slab-reduction width (PIO_SLAB_TARGET) on the headline,
# the MNIST step (dQ + PE reduction in one zero span), the forced-reducer exposure and a step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
bash tools/gpu_env_ab.sh - - PIO_SLAB_TARGET=256 PIO_SLAB_TARGET=192 || exit 1
BENCH_CFG=mnist bash tools/gpu_env_ab.sh - - || exit 1
bash tools/gpu_reducer.sh || exit 1
bash tools/gpu_step_profile.sh > /dev/null || exit 1
head -30 gpurun_out/step/breakdown.md
