# focused GPU check: selected tests (-k pattern in $1), then repeated MLM bench + a kernel-trace profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ${1:+-k "$1"} > gpurun_out/tq.log 2>&1; rc=$?
tail -4 gpurun_out/tq.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/tq.log | head -20; exit $rc; fi
bash tools/gpu_bench_rep.sh
