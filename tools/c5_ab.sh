set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_rccl_gpu.py "tests/test_configs_gpu.py::test_c5_giant_binned_equals_gather" tests/test_partition.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
for lib in ${LIBS:-ab/libmjx_base.so master-thesis-optimizing-initialization-in-graph-dynamics-from-ferromagnetism-to-opinion-consensus_amd/libmjx.so ab/libmjx_base.so master-thesis-optimizing-initialization-in-graph-dynamics-from-ferromagnetism-to-opinion-consensus_amd/libmjx.so}; do
  timeout -k 10 240 python -u tools/ab_lib.py $lib tools/giant_time.py 1e9 6 20 >> $OUT/c5_ab.log 2>&1 || exit $?
done
R="$GRAFT_REPO_ROOT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/c5prof" -o run --output-format csv -- python3 "$R/tools/giant_time.py" 1e9 6 20 ) > $OUT/c5prof.log 2>&1
