cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ablate_g8.py --variant ${VARIANTS:-shared,direct} --flags ${FLAGS:-0,1,2,4,8,9,12,6} > gpurun_out/abl.log 2>&1 || { echo "ablate failed"; tail -20 gpurun_out/abl.log; exit 3; }
grep -v amdgpu.ids gpurun_out/abl.log
