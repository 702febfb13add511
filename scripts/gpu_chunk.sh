# Bench A/B of the Gram chunk size (partials volume vs parallelism).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 0 3072 1536 0 3072; do
  if [ $c = 0 ]; then unset OCM_GRAM_CHUNK; else export OCM_GRAM_CHUNK=$c; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-vae --steps 8 > gpurun_out/chunk_$c.log 2>&1 || { echo bench failed; exit 3; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/chunk_$c.log').read().strip().splitlines()[-1]); print('chunk $c', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
