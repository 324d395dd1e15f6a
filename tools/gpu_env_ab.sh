# A/B of environment settings on one box: the GPU tests selected by $1 (-k pattern, "" = all,
# "-" = none), then the bench config $BENCH_CFG (default mlm256) twice under each setting given
# as the remaining arguments ("-" = defaults).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
pat=$1; shift
cfg=${BENCH_CFG:-mlm256}
if [ "$pat" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${pat:+-k "$pat"} > gpurun_out/ab/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab/tests.log
  [ $rc -le 1 ] || exit $rc
  [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/ab/tests.log | head -20; }
fi
for e in "$@"; do
  [ "$e" = "-" ] && e="PIO_NOTHING=1"
  for i in 1 2; do
    env $e timeout -k 10 200 python bench.py --config $cfg --steps 30 --warmup 5 > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { echo bench failed; tail gpurun_out/ab/b.err; exit 4; }
    python -c "import json; d=json.loads(open('gpurun_out/ab/b.json').read().strip().splitlines()[-1]); print('$e', '$cfg', d['ms_per_step'], d['value'])"
  done
done
