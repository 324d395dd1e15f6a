# PMC passes over the MLM headline step (eager launches of the same kernels, --no-graph), one
# counter group per run, then the per-kernel summary (tools/pmc_summary.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_mlm
mkdir -p $O
CFG=${1:-mlm256}
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS --output-format csv -d $O/p1 -o pmc -- python bench.py --config $CFG --steps 2 --warmup 1 --no-graph > $O/p1.log 2>&1 || { echo "pmc pass 1 failed"; tail -20 $O/p1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o pmc -- python bench.py --config $CFG --steps 2 --warmup 1 --no-graph > $O/p2.log 2>&1 || { echo "pmc pass 2 failed"; tail -20 $O/p2.log; exit 1; }
python tools/pmc_summary.py $O/p1 $O/p2 --md > $O/summary_$CFG.md 2>&1
head -c 3000 $O/summary_$CFG.md
