# DDP GPU tests + a short bench (bucket updates on the captured path)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ddp
timeout -k 10 400 python -u -m pytest tests/test_ddp_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ddp/test.log 2>&1; rc=$?
tail -15 gpurun_out/ddp/test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ddp/bench.json 2> gpurun_out/ddp/bench.err || { tail gpurun_out/ddp/bench.err; exit 1; }
cat gpurun_out/ddp/bench.json
PERCEIVER_BENCH_FORCE_REDUCER=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ddp/bench_red.json 2> gpurun_out/ddp/bench_red.err || { tail gpurun_out/ddp/bench_red.err; exit 1; }
cat gpurun_out/ddp/bench_red.json
