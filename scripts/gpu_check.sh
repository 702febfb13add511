cd $GRAFT_REPO_ROOT
rocminfo | grep -m2 gfx > gpurun_out/rocminfo.txt 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench.log 2>&1
  echo "bench rc=$?"
  tail -3 gpurun_out/bench.log
fi
