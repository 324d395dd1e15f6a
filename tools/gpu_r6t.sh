# PE backward: fixed memory-op count per iteration (loop-head wait is a count, not a drain)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6t
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "pe or image or deterministic" > gpurun_out/r6t/tests.log 2>&1 || { tail -30 gpurun_out/r6t/tests.log; exit 1; }
tail -2 gpurun_out/r6t/tests.log
for rep in 1 2; do
  for t in new old; do
    d=.; [ $t = old ] && d=ab_old
    (cd $d && timeout -k 10 120 python tools/pe_attn_bench.py --which bwd --iters 50) | sed "s/^/$t /" | tee -a gpurun_out/r6t/ab.log || exit 2
    (cd $d && timeout -k 10 300 python bench.py --config imagenet --steps 40 --warmup 5) | python -c "import json,sys; print('$t imagenet', json.loads(sys.stdin.read())['ms_per_step'])" | tee -a gpurun_out/r6t/ab.log || exit 3
    (cd $d && timeout -k 10 300 python bench.py --config mnist --steps 40 --warmup 5) | python -c "import json,sys; print('$t mnist', json.loads(sys.stdin.read())['ms_per_step'])" | tee -a gpurun_out/r6t/ab.log || exit 4
  done
done
