export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
run() { timeout -s KILL 90 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmc_$2 -o p -- python bench.py --steps 3 --warmup 1 --no-cpu --games 1000000 --replay-steps 1 --profile-only > /dev/null 2>> gpurun_out/pmc.err; echo "pass $2 rc=$?" >> gpurun_out/pmc.err; }
run "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" 1 && \
run "FETCH_SIZE" 2 && run "WRITE_SIZE" 3 && \
run "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" 4
ls gpurun_out/pmc_*/
