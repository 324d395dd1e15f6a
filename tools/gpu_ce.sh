# CE head: kernel tests, per-kernel timings, PMC passes (LDS conflicts, MFMA / VALU activity)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ce
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -k "cross_entropy or classifier or checked or mlm_fused or headline" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ce/test.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/ce/test.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/ce_bench.py > gpurun_out/ce/bench.log 2>&1 || { tail gpurun_out/ce/bench.log; exit 1; }
cat gpurun_out/ce/bench.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ce/kt -o run -- python tools/ce_bench.py --iters 10 > gpurun_out/ce/kt.log 2>&1 || { tail gpurun_out/ce/kt.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/ce/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1000:8.2f}")
PY
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/ce/pmc1 -o pmc -- python tools/ce_bench.py --iters 3 > gpurun_out/ce/pmc1.log 2>&1 || { tail gpurun_out/ce/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ce/pmc2 -o pmc -- python tools/ce_bench.py --iters 3 > gpurun_out/ce/pmc2.log 2>&1 || { tail gpurun_out/ce/pmc2.log; exit 1; }
python tools/pmc_summary.py gpurun_out/ce/pmc1 gpurun_out/ce/pmc2 --match ce > gpurun_out/ce/pmc_summary.txt 2>&1 || true
cat gpurun_out/ce/pmc_summary.txt
