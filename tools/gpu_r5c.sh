# CE head numerics, then the MLM step A/B of the side-stream slab reductions (PERCEIVER_SLAB_SIDE)
# with a kernel profile of each, then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "entropy or ce_ or index_add" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/ce_tests.log 2>&1; rc=$?
tail -3 $O/ce_tests.log
[ $rc -eq 0 ] || { grep -E "^E " $O/ce_tests.log | head -20; exit $rc; }
for s in 0 1; do
  PERCEIVER_SLAB_SIDE=$s timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/mlm_s$s.json 2> $O/mlm_s$s.err || { tail -20 $O/mlm_s$s.err; exit 1; }
  python -c "import json;d=json.load(open('$O/mlm_s$s.json'));print('slab_side=$s', d['value'], d['ms_per_step'], d.get('final_loss'))"
  PERCEIVER_SLAB_SIDE=$s timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof$s -o run -- python bench.py --steps 6 --warmup 3 > $O/prof$s.log 2>&1 || { tail $O/prof$s.log; exit 1; }
  python tools/step_breakdown.py $(find $O/prof$s -name "*kernel_trace.csv" | head -1) --marker stage_step_kernel > $O/mlm_step_s$s.md
  head -1 $O/mlm_step_s$s.md
  grep ce2 $O/mlm_step_s$s.md
done
bash tools/gpu_suite.sh
