set -o pipefail
mkdir -p gpurun_out/pmc
cd $GRAFT_REPO_ROOT
timeout -k 5 60 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true
grep -oE "SQ_[A-Z0-9_]+" gpurun_out/pmc/avail.txt | sort -u > gpurun_out/pmc/sq_counters.txt || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o run -- python tools/chain_bench.py > gpurun_out/pmc/p1.log 2>&1 || echo "pmc1 failed"
wc -l gpurun_out/pmc/sq_counters.txt
