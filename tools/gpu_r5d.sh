# LArTPC A/B of the tall-wgrad K/V backward (PERCEIVER_KV_TALL_MIN) with its GPU model tests, then
# the image configs after the sample-block LDS-only barriers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/mlm.json 2> $O/mlm.err || { tail -20 $O/mlm.err; exit 1; }
python -c "import json;d=json.load(open('$O/mlm.json'));print('mlm256', d['value'], d['ms_per_step'], d.get('final_loss'))"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/mprof -o run -- python bench.py --steps 6 --warmup 3 > $O/mprof.log 2>&1 || { tail $O/mprof.log; exit 1; }
python tools/step_breakdown.py $(find $O/mprof -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > $O/mlm_step.md
head -12 $O/mlm_step.md
PERCEIVER_KV_TALL_MIN=16384 timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k lartpc -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/lartpc_tests.log 2>&1; rc=$?
tail -3 $O/lartpc_tests.log
[ $rc -eq 0 ] || { grep -E "^E " $O/lartpc_tests.log | head -20; exit $rc; }
for t in 131072 16384; do
  PERCEIVER_KV_TALL_MIN=$t timeout -k 10 200 python bench.py --config lartpc --steps 20 --warmup 5 > $O/lar_$t.json 2> $O/lar_$t.err || { tail -20 $O/lar_$t.err; exit 1; }
  python -c "import json;d=json.load(open('$O/lar_$t.json'));print('kv_tall_min=$t', d['value'], d['ms_per_step'], d.get('final_loss'))"
done
PERCEIVER_KV_TALL_MIN=16384 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/lprof -o run -- python bench.py --config lartpc --steps 6 --warmup 3 > $O/lprof.log 2>&1 || { tail $O/lprof.log; exit 1; }
python tools/step_breakdown.py $(find $O/lprof -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > $O/lartpc_step.md
head -24 $O/lartpc_step.md
bash tools/gpu_configs.sh mnist imagenet
