set -u
# Round 6: where the GPU idles inside a timed step (headline 1M x 2048 and the
# 125k-row share): kernel traces → scripts/step_gaps.py.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06y}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_1m -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-vae --no-cv --no-prep --phase-steps 0 > $OUT/trace_1m.log 2>&1 || exit 1
python scripts/step_gaps.py $OUT/prof_1m/run_kernel_trace.csv --steps 2 > $OUT/gaps_1m.txt; cat $OUT/gaps_1m.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_125k -o run --output-format csv -- python3 bench.py --rows 125000 --steps 6 --warmup 1 --no-cpu --no-vae --no-cv --no-prep --phase-steps 0 > $OUT/trace_125k.log 2>&1 || exit 1
python scripts/step_gaps.py $OUT/prof_125k/run_kernel_trace.csv --steps 2 > $OUT/gaps_125k.txt; cat $OUT/gaps_125k.txt
rm -f $OUT/prof_*/*_kernel_trace.csv
