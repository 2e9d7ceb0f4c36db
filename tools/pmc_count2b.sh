export TMPDIR=/tmp
run() { timeout -s KILL 90 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmc_$2 -o p -- python bench.py --steps 3 --warmup 1 --no-cpu --no-replay --profile-only > /dev/null 2>> gpurun_out/pmc.err; echo "pass $2 rc=$?" >> gpurun_out/pmc.err; }
rm -rf gpurun_out/pmc_*
run "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" 1 && \
run "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" 2 && \
run "FETCH_SIZE" 3 && run "WRITE_SIZE" 4
ls gpurun_out/pmc_*/ ; grep rc= gpurun_out/pmc.err
