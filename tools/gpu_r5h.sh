# MLM headline A/B of the XCD-local slab reductions (PIO_SLAB_XCD) + step profile + the tests
# that check the reduced gradients bitwise / against fp32
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5h
mkdir -p $O
for x in 0 1; do
  PIO_SLAB_XCD=$x timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/mlm_x$x.json 2> $O/mlm_x$x.err || { tail -20 $O/mlm_x$x.err; exit 1; }
  python -c "import json;d=json.load(open('$O/mlm_x$x.json'));print('slab_xcd=$x', d['value'], d['ms_per_step'], d.get('final_loss'))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python tools/step_breakdown.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > $O/mlm_step.md
head -14 $O/mlm_step.md
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_sample_block_gpu.py -k "mlm or headline or graph_engine or image or sample_block or lartpc" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^(E |FAILED)" $O/tests.log | head -20; exit $rc; }
bash tools/gpu_configs.sh mnist imagenet lartpc
