# round 6: PE backward dQ-reduce balance (timing + tests), CE head 4-waves-per-SIMD A/B (ab_ce tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6e
timeout -k 10 120 python tools/pe_attn_bench.py --which both --iters 20 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "pe or factored" tests/test_model_gpu.py -k "image" > gpurun_out/r6e/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6e/tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/r6e/tests.log | head; exit $rc; }
(cd ab_ce && timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "ce or cross_entropy" tests/test_model_gpu.py -k "headline or mlm_fused" > $GRAFT_REPO_ROOT/gpurun_out/r6e/tests_ce.log 2>&1); rc=$?
tail -3 gpurun_out/r6e/tests_ce.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/r6e/tests_ce.log | head; exit $rc; }
b() {
  d=$1
  (cd $d && timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/r6e/b.json 2> $GRAFT_REPO_ROOT/gpurun_out/r6e/b.err) || { echo bench failed; tail gpurun_out/r6e/b.err; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/r6e/b.json').read().strip().splitlines()[-1]); print('$d', d['ms_per_step'], d['value'])"
}
for i in 1 2 3; do b .; b ab_ce; done
for d in . ab_ce; do
  O=$GRAFT_REPO_ROOT/gpurun_out/r6e/prof_$(basename $(cd $d && pwd))
  mkdir -p $O
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1) || { echo prof failed; tail $O/prof.log; exit 5; }
  python tools/step_breakdown.py $(find $O -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > $O/breakdown.md
  grep -E "ce2|one step" $O/breakdown.md
done
BENCH=1 bash tools/gpu_configs.sh imagenet mnist
