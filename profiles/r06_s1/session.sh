set -o pipefail
O=gpurun_out/r06_s1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multi.py "tests/test_gpu_parity.py::test_generic_sub_batches_eq" "tests/test_gpu_parity.py::test_fast_loop_top_exit_regression" "tests/test_gpu_parity.py::test_fast_fallback_parity" "tests/test_gpu_parity.py::test_fast_edge_cases" "tests/test_gpu_parity.py::test_fast_wave_fallback_edges" "tests/test_gpu_parity.py::test_generic_sub_batches" > $O/pytest_new.log 2>&1; echo pytest rc=$?
timeout -k 10 500 python -u tools/large_fuzz_probe.py $O/large_default.json $(seq 0 63) > $O/large_default.log 2>&1 && \
timeout -k 10 300 python -u tools/c5_exact_cost.py 1024 1 > $O/c5_cost_1024.log 2>&1 && \
timeout -k 10 600 python -u tools/c5_exact_cost.py 4096 1 > $O/c5_cost_4096.log 2>&1
echo rc=$?
tail -3 $O/*.log
