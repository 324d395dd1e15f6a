# MLM headline A/B of the two-tile attention backward (PIO_ATTN_BWD_QR2) + step profile, then the
# attention / model GPU tests that cover it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
for q in 0 1; do
  PIO_ATTN_BWD_QR2=$q timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/mlm_q$q.json 2> $O/mlm_q$q.err || { tail -20 $O/mlm_q$q.err; exit 1; }
  python -c "import json;d=json.load(open('$O/mlm_q$q.json'));print('qr2=$q', d['value'], d['ms_per_step'], d.get('final_loss'))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python tools/step_breakdown.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > $O/mlm_step.md
head -16 $O/mlm_step.md
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_fuzz_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^(E |FAILED)" $O/tests.log | head -30; exit $rc; }
