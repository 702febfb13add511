cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gram" > gpurun_out/pytest_d.log 2>&1 || { tail -20 gpurun_out/pytest_d.log; exit 1; }
OCM_GRAM8_VARIANT=lds timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "i8" > gpurun_out/pytest_dd.log 2>&1 || { tail -20 gpurun_out/pytest_dd.log; exit 2; }
tail -1 gpurun_out/pytest_d.log; tail -1 gpurun_out/pytest_dd.log
FLAGS="0" bash scripts/gpu_exp8.sh
OCM_GRAM8_VARIANT=lds FLAGS="0" bash scripts/gpu_exp8.sh
