# per-sample block kernels: numerics first, then image-config benches A/B (PERCEIVER_SAMPLE_BLOCK=0/1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sb
timeout -k 10 300 python -u -m pytest tests/test_sample_block_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sb/test.log 2>&1; rc=$?
tail -12 gpurun_out/sb/test.log
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/sb/test.log | head -30; exit $rc; }
for cfg in mnist imagenet; do
  for f in 0 1; do
    PERCEIVER_SAMPLE_BLOCK=$f timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 > gpurun_out/sb/${cfg}_$f.json 2> gpurun_out/sb/${cfg}_$f.err || { echo "bench $cfg $f failed"; tail -20 gpurun_out/sb/${cfg}_$f.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/sb/${cfg}_$f.json'));print('$cfg sb=$f', d['value'], d['ms_per_step'], d.get('final_loss'))"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sb/prof -o run -- python bench.py --config mnist --steps 6 --warmup 3 > gpurun_out/sb/prof.log 2>&1 || { tail gpurun_out/sb/prof.log; exit 1; }
python tools/step_breakdown.py gpurun_out/sb/prof/run_kernel_trace.csv --marker adamw4 > gpurun_out/sb/mnist_step.md
head -30 gpurun_out/sb/mnist_step.md
