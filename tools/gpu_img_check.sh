cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "pe_grads or pe_gemm" tests/test_model_gpu.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t.log 2>&1; rc=$?; tail -5 gpurun_out/t.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config imagenet --steps 10 --warmup 3 > gpurun_out/img.log 2>&1 || exit $?
tail -1 gpurun_out/img.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_img -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --config imagenet --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_img.log 2>&1
