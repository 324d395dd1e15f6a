# A/B helper: the GPU tests selected by $1 (-k pattern, "" = all), then the chain trace and the
# MLM bench under each environment setting given as the remaining arguments ("-" = defaults).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
pat=$1; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${pat:+-k "$pat"} > gpurun_out/ab/tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab/tests.log
[ $rc -le 1 ] || exit $rc
for e in "$@"; do
  [ "$e" = "-" ] && e="PIO_NOTHING=1"
  echo "== $e"
  env $e timeout -k 10 60 ./tools/trace/chain_trace 16384 > gpurun_out/ab/trace.txt 2>&1 || { echo trace failed; exit 3; }
  grep "us/launch" gpurun_out/ab/trace.txt
  for i in 1 2; do
    env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { echo bench failed; tail gpurun_out/ab/b.err; exit 4; }
    python -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print('bench', d['ms_per_step'], d['value'])"
  done
done
