# sample-block weight-gradient rows per workgroup sweep (temporary A/B knob PIO_SBW_ROWS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rows in 256 512 1024; do
  echo "rows=$rows"
  for cfg in mnist imagenet; do
    PIO_SBW_ROWS=$rows timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 5 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'])" || exit 1
  done
done
