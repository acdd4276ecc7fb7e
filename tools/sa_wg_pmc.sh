set -u
R="$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
   -d "$R/$OUT/sqa" -o run --output-format csv -- python3 "$R/tools/sa_wg_pmc.py" ) > $OUT/sqa.log 2>&1 || exit $?
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_BUSY_CYCLES \
   -d "$R/$OUT/sqb" -o run --output-format csv -- python3 "$R/tools/sa_wg_pmc.py" ) > $OUT/sqb.log 2>&1 || exit $?
python3 tools/pmc_sq_parse.py $OUT/sqa $OUT/sqa.json && python3 tools/pmc_sq_parse.py $OUT/sqb $OUT/sqb.json
