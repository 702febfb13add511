# k_gram8s (shared-LDS i8x3 Gram): parity tests under the variant, then A/B vs k_gram8d.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OCM_GRAM8_VARIANT=shared timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gram" > gpurun_out/g8s_tests.log 2>&1
rc=$?; tail -5 gpurun_out/g8s_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_gram.py --rounds 3 --variants ${VARIANTS:-i8x3d:128x32:4096,i8x3s:128x32:4096,i8x3s:128x32:9216} > gpurun_out/g8s_bench.log 2>&1 || { echo "bench_gram failed"; tail -20 gpurun_out/g8s_bench.log; exit 3; }
grep -v amdgpu.ids gpurun_out/g8s_bench.log
echo done
