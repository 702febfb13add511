set -o pipefail
O=gpurun_out/r04z9
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
tail -2 $O/tests.log
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 300 python3 -u bench.py --rows 125000 --no-cpu --no-vae --no-cv --no-prep --steps 20 > $O/share125k.json 2>> $O/bench.err || exit 3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --no-cpu --steps 5 > $O/bench_prof.json 2> $O/bench_prof.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/vprof -o run --output-format csv -- python3 scripts/vae_step_trace.py 50 > $O/vrun.log 2>&1 || exit 5
python3 scripts/vae_step_trace.py --summarize $O/vprof/run_kernel_trace.csv 50 > $O/vae_trace.md
rm -f $O/prof/run_kernel_trace.csv $O/vprof/run_kernel_trace.csv
echo done
