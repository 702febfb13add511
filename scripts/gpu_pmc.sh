cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K="--kernel-include-regex k_gram|k_score"
A="scripts/bench_gram.py --variants f32:8192 --rounds 1"
timeout -k 10 300 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d gpurun_out/pmc1 -o p --output-format csv -- python3 $A > gpurun_out/pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 $K --pmc FETCH_SIZE -d gpurun_out/pmc2 -o p --output-format csv -- python3 $A > gpurun_out/pmc2.log 2>&1 && \
timeout -k 10 300 rocprofv3 $K --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc3 -o p --output-format csv -- python3 $A > gpurun_out/pmc3.log 2>&1
echo "rc=$?"
ls gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3
hipcc --offload-arch=gfx950 -O3 scripts/ubench_mfma.hip -o /tmp/ub && timeout -k 10 120 /tmp/ub > gpurun_out/ubench.log 2>&1
cat gpurun_out/ubench.log
