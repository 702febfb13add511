# Round profile: kernel trace of the bench + PMC passes (one counter group per pass) on
# the bench's dominant kernels.  Output: gpurun_out/profr/{trace,pmc1,pmc2,pmc3}.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/profr
mkdir -p $OUT
K="--kernel-include-regex k_gram8d|k_q8_quant|k_score_direct"
A="bench.py --steps 2 --warmup 1 --no-cpu --no-vae"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-vae > $OUT/trace.log 2>&1 || { echo trace failed; exit 1; }
timeout -s KILL 240 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT/pmc1 -o p --output-format csv -- python3 $A > $OUT/pmc1.log 2>&1 || { echo pmc1 failed; exit 2; }
timeout -s KILL 240 rocprofv3 $K --pmc FETCH_SIZE -d $OUT/pmc2 -o p --output-format csv -- python3 $A > $OUT/pmc2.log 2>&1 || { echo pmc2 failed; exit 3; }
timeout -s KILL 240 rocprofv3 $K --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc3 -o p --output-format csv -- python3 $A > $OUT/pmc3.log 2>&1 || { echo pmc3 failed; exit 4; }
echo done
