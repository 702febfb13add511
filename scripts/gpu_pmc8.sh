cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc8
mkdir -p $OUT
K="--kernel-include-regex k_gram8|k_q8_quant"
A="scripts/gram_once.py --reps 2"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $A > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc1 -o p --output-format csv -- python3 $A > $OUT/pmc1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 $K --pmc FETCH_SIZE -d $OUT/pmc2 -o p --output-format csv -- python3 $A > $OUT/pmc2.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 $K --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc3 -o p --output-format csv -- python3 $A > $OUT/pmc3.log 2>&1 || exit 4
echo done
