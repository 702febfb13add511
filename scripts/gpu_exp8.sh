cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/exp8
for v in ${FLAGS:-0 1 3 5 9 15 4}; do
  export OCM_GRAM8_NOLOAD=$v
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/exp8/t$v -o run --output-format csv -- python3 scripts/gram_once.py --reps 2 > gpurun_out/exp8/t$v.log 2>&1 || exit 7
  python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/exp8/t$v/run_kernel_stats.csv')))[:3]:
  if 'gram8' in r['Name']: print('flags=$v', r['Name'][:30], round(float(r['AverageNs'])/1e6,3))"
done
