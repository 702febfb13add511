# Round profile: kernel-trace stats of the bench command + PMC passes for the
# two hot kernels (separate rocprofv3 invocations per counter group).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench_trace.log 2>&1 || exit 1
K="--kernel-include-regex k_gram|k_score"
A="bench.py --steps 2 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT/pmc1 -o p --output-format csv -- python3 $A > $OUT/pmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 $K --pmc FETCH_SIZE -d $OUT/pmc2 -o p --output-format csv -- python3 $A > $OUT/pmc2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 $K --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc3 -o p --output-format csv -- python3 $A > $OUT/pmc3.log 2>&1 || exit 4
echo done
