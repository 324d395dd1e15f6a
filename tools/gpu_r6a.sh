# round 6: query-halves attention backward — kernel tests, headline three-way, then bench A/B + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6a
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_attn_bwd_selfattn_gpu.py > gpurun_out/r6a/tests.log 2>&1; rc=$?
tail -15 gpurun_out/r6a/tests.log; [ $rc -eq 0 ] || exit $rc
PIO_ATTN_QH=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_model_gpu.py -k "headline or deterministic" > gpurun_out/r6a/tests_model.log 2>&1; rc=$?
tail -3 gpurun_out/r6a/tests_model.log; [ $rc -eq 0 ] || exit $rc
for e in PIO_ATTN_QH=0 PIO_ATTN_QH=1 PIO_ATTN_QH=0 PIO_ATTN_QH=1; do
  env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/r6a/b.json 2> gpurun_out/r6a/b.err || { echo bench failed; tail gpurun_out/r6a/b.err; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/r6a/b.json').read().strip().splitlines()[-1]); print('$e', d['ms_per_step'], d['value'])"
done
for e in PIO_ATTN_QH=1; do
  O=gpurun_out/r6a/prof_$e; mkdir -p $O
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 5; }
  python tools/step_breakdown.py $(find $O -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > $O/breakdown.md
  head -16 $O/breakdown.md
done
