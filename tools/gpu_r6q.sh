# PE forward with the softmax offset folded into the score MFMA: numerics, kernel time, ImageNet / MNIST step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6q
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pe" tests/test_model_gpu.py -k "pe or image" > gpurun_out/r6q/tests.log 2>&1 || { tail -30 gpurun_out/r6q/tests.log; exit 1; }
tail -3 gpurun_out/r6q/tests.log
timeout -k 10 120 python tools/pe_attn_bench.py --which fwd --iters 50 | tee gpurun_out/r6q/pe_fwd.log || exit 2
bash tools/gpu_configs.sh imagenet mnist || exit 3
