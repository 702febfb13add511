# i8x3 Gram with 768-row scale blocks: parity tests (both variants), A/B, ablations.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_simca.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g8b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g8b_tests.log; [ $rc -eq 0 ] || exit $rc
OCM_GRAM8_VARIANT=shared timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k gram > gpurun_out/g8b_tests_s.log 2>&1
rc=$?; tail -3 gpurun_out/g8b_tests_s.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ablate_g8.py --variant direct --flags 0 > gpurun_out/abl.log 2>&1 || { echo "ablate failed"; tail -20 gpurun_out/abl.log; exit 3; }
grep -v amdgpu.ids gpurun_out/abl.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g8b -o run --output-format csv -- python3 scripts/gram_once.py --reps 3 > gpurun_out/g8b_trace.log 2>&1 || { echo "trace failed"; exit 4; }
echo done
