# PMC passes over the factored PE forward (tools/pe_attn_bench.py --which fwd), one counter group
# per run; prints per-kernel sums
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/pmc_pef; mkdir -p $out
timeout -k 10 120 python tools/pe_attn_bench.py --which fwd --iters 20 > $out/bench.log 2>&1 || { tail $out/bench.log; exit 1; }
cat $out/bench.log
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o run -- python tools/pe_attn_bench.py --which fwd --iters 2 > $out/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $out/p$i.log; }
done
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/pmc_pef/p*/**/*counter_collection.csv', recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:40]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    for k, d in agg.items():
        if 'fwd_pe' in k:
            print(f.split('/')[2], k, {c: f"{v:.4g}" for c, v in d.items()})
PY
