# sample-block numerics (kernel tests + the image model three-way tests), phase trace, image /
# LArTPC config benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_sample_block_gpu.py tests/test_model_gpu.py -k "sample_block or image or lartpc or deterministic" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^(E |FAILED)" $O/tests.log | head -20; exit $rc; }
timeout -k 5 60 ./tools/trace/sb_trace 128 > $O/trace.txt 2>&1 && timeout -k 5 60 ./tools/trace/sb_trace 32 >> $O/trace.txt 2>&1 || { cat $O/trace.txt; exit 1; }
grep -E "us/launch" $O/trace.txt
bash tools/gpu_configs.sh mnist imagenet lartpc
