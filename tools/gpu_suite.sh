# the whole GPU test suite (one process), then the framework-op stacks of the given configs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/suite
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -o console_output_style=count > gpurun_out/suite/gpu_tests.log 2>&1; rc=$?
tail -8 gpurun_out/suite/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "^(E |FAILED)" gpurun_out/suite/gpu_tests.log | head -30; exit $rc; }
[ $# -gt 0 ] && bash tools/gpu_stacks.sh "$@"
exit 0
