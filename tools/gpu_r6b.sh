# round 6: the GPU suite, then the forced 1-rank reducer A/B (overlap × bucket_update) + no-reducer bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh || exit 1
mkdir -p gpurun_out/r6b
for i in 1 2; do
  for e in "--overlap on --bucket-update on" "--overlap off --bucket-update on" "--overlap on --bucket-update off" "--overlap off --bucket-update off"; do
    PERCEIVER_BENCH_FORCE_REDUCER=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 $e > gpurun_out/r6b/b.json 2> gpurun_out/r6b/b.err || { echo bench failed; tail gpurun_out/r6b/b.err; exit 4; }
    python -c "import json; d=json.loads(open('gpurun_out/r6b/b.json').read().strip().splitlines()[-1]); print('force-reducer $e', d['ms_per_step'], d['value'])"
  done
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/r6b/b.json 2> gpurun_out/r6b/b.err || exit 4
  python -c "import json; d=json.loads(open('gpurun_out/r6b/b.json').read().strip().splitlines()[-1]); print('no reducer', d['ms_per_step'], d['value'])"
done
