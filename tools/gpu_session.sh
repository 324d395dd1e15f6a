#!/bin/bash
# Staged GPU session for gpurun: each GPU step has its own time limit; a step that faults,
# aborts, segfaults or times out ends the session (exit codes 124/134/137/139 or >128).
# Pytest failures (exit 1) are numerics findings and do not stop later steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() {  # run <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ] && [ $rc -ne 5 ]; then
    echo "stopping session after $name (rc=$rc)" | tee -a gpurun_out/session.log
    exit $rc
  fi
  return 0
}
# the in-tree .so (built on the CPU host) travels with the snapshot; "build" re-links it on the box
for step in "$@"; do
  case "$step" in
    build)    run build 900 python -m perceiver_io_amd.csrc.build ;;
    smoke)    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    kernels)  run kernels 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    kernels_all) run kernels_all 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    ref)      run bench_ref 600 python bench.py --backend reference --steps 5 --warmup 2 ;;
    ref32)    run bench_ref32 600 python bench.py --backend reference --dtype fp32 --steps 5 --warmup 2 ;;
    eager)    run bench_eager 600 python bench.py --no-graph --steps 10 --warmup 3 ;;
    bench)    run bench 600 python bench.py --steps 20 --warmup 5 ;;
    micro)    run micro 300 python tools/microbench.py ;;
    tiles)    run tiles 300 python tools/tile_latency.py ;;
    pmc_layer) run pmc_layer 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_layer -o pmc -- python tools/tile_latency.py pmc ;;
    pmc_layer2) run pmc_layer2 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/pmc_layer2 -o pmc -- python tools/tile_latency.py pmc ;;
    attn)     run attn 300 python tools/attn_scaling.py ;;
    pmc_attn) run pmc_attn 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc -o attn -- python tools/attn_scaling.py 64 ;;
    configs)  for c in seq_clf imagenet long_mlm mnist; do
                run "cfg_${c}" 600 python bench.py --config $c --steps 10 --warmup 3
              done ;;
    configs_ref) for c in mlm256 seq_clf imagenet long_mlm mnist; do
                run "cfgref_${c}" 900 python bench.py --config $c --backend reference --steps 5 --warmup 2
              done ;;
    prof_img) run prof_img 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_img -o run --output-format csv -- python bench.py --config imagenet --steps 3 --warmup 2 ;;
    prof_mnist) run prof_mnist 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mnist -o run --output-format csv -- python bench.py --config mnist --steps 3 --warmup 2 ;;
    ddp2)     run ddp2 600 env PERCEIVER_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 3 ;;
    trace)    for t in tools/trace/*_trace; do run "trace_$(basename $t)" 120 $t; done ;;
    pmc_trace) run pmc_trace 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_trace -o pmc -- tools/trace/attn_bwd_trace ;;
    bench_noslab) run bench_noslab 600 env PERCEIVER_WGRAD_SLAB=0 python bench.py --steps 20 --warmup 5 ;;
    prof_noslab) run prof_noslab 600 env PERCEIVER_WGRAD_SLAB=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_noslab -o run --output-format csv -- python bench.py --steps 5 --warmup 3 ;;
    prof)     run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 3 ;;
    lartpc)   run lartpc 600 python run.py --epochs 1 --events 8 --val-events 4 --size 512 --batch-size 4 --max-steps 2 --log-dir /tmp/lartpc_runs --ckpt-dir /tmp/lartpc_ckpt ;;
    lartpc_test) run lartpc_test 300 python -u -m pytest tests/test_components.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider ;;
    *) echo "unknown step $step" ;;
  esac
done
echo "session done"
