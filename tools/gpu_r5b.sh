# round-5 checkpoint: the new kernels' GPU tests, then bench + per-step kernel breakdown of every
# config that changed this round, then the framework-op stacks of the LArTPC step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5b
timeout -k 10 400 python -u -m pytest tests/test_sample_block_gpu.py tests/test_persist_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5b/new_tests.log 2>&1; rc=$?
tail -14 gpurun_out/r5b/new_tests.log
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r5b/new_tests.log | head -30; exit $rc; }
bash tools/gpu_configs.sh ${R5B_CONFIGS:-mlm256 lartpc mnist imagenet seq_clf_ft} || exit 1
bash tools/gpu_stacks.sh lartpc
