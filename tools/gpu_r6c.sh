# round 6: tests of the changed paths, persist / per-layer / HEAD A/B on one box, configs + step tables
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_attn_bwd_selfattn_gpu.py tests/test_ddp_gpu.py tests/test_model_gpu.py \
  "tests/test_kernels_gpu.py::test_attention_dropout_matches_emulation" "tests/test_kernels_gpu.py::test_checked_build_flags_out_of_range_indices" \
  > gpurun_out/r6c/tests.log 2>&1; rc=$?
tail -4 gpurun_out/r6c/tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/r6c/tests.log | head -20; exit $rc; }
b() {  # dir env...
  d=$1; shift
  (cd $d && env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/r6c/b.json 2> $GRAFT_REPO_ROOT/gpurun_out/r6c/b.err) || { echo bench failed; tail gpurun_out/r6c/b.err; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/r6c/b.json').read().strip().splitlines()[-1]); print('$d $*', d['ms_per_step'], d['value'])"
}
for i in 1 2; do
  b ab_old PERCEIVER_PERSIST=1
  b ab_old PERCEIVER_PERSIST=0
  b . PIO_NOTHING=1
done
timeout -k 10 300 python bench.py --config mlm64 --backend reference --steps 5 --warmup 2 > gpurun_out/r6c/ref_mlm64.json 2> gpurun_out/r6c/ref.err || { tail gpurun_out/r6c/ref.err; exit 5; }
cat gpurun_out/r6c/ref_mlm64.json
bash tools/gpu_configs.sh mlm64 seq_clf_ft seq_clf long_mlm
