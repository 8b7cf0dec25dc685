set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_core.py -m gpu -x -q --timeout 120 --timeout-method thread -k "banded or reduce or dot or vadd or vmul" > gpurun_out/r4g_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/spmv_banded_lab.py 100000 401 200 100 200 10 1,8,9 > gpurun_out/r4g_banded.log 2>&1 &&
timeout -k 10 300 python -u bench.py --sections reduce --steps 20 --warmup 5 --no-ref > gpurun_out/r4g_reduce.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d gpurun_out/r4g_clock -o p -- python3 scripts/sgemm_clock_lab.py 40 > gpurun_out/r4g_clock.log 2>&1 &&
python3 scripts/clock_summary.py gpurun_out/r4g_clock/p_counter_collection.csv sgemm > gpurun_out/r4g_clock_summary.txt 2>&1
