# round 6: persist restored + loud spin timeouts; fixed-order grad-norm partials; configs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6d
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_persist_gpu.py tests/test_trainer_gpu.py tests/test_lartpc.py \
  "tests/test_kernels_gpu.py" "tests/test_model_gpu.py::test_deterministic_mode_bitwise" \
  > gpurun_out/r6d/tests.log 2>&1; rc=$?
tail -4 gpurun_out/r6d/tests.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/r6d/tests.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/r6d/b.json 2> gpurun_out/r6d/b.err || { tail gpurun_out/r6d/b.err; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/r6d/b.json').read().strip().splitlines()[-1]); print('mlm256', d['ms_per_step'], d['value'])"
done
bash tools/gpu_configs.sh lartpc seq_clf mlm64
