# sample-block numerics, then the image / LArTPC configs' benches and step breakdowns
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sample_block_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/sb_tests.log 2>&1; rc=$?
tail -3 $O/sb_tests.log
[ $rc -eq 0 ] || { grep -E "^E " $O/sb_tests.log | head -20; exit $rc; }
bash tools/gpu_configs.sh mnist imagenet lartpc
