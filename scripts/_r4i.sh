set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./bin_lab/valu_rate_lab > gpurun_out/r4i_valu_rate.log 2>&1 &&
timeout -k 10 200 python -u scripts/spmv_banded_lab.py 100000 401 200 100 200 10 1,8,9 > gpurun_out/r4i_banded.log 2>&1 &&
timeout -k 10 300 python -u scripts/stencil_rpw_lab.py 8 16384 8,4 48,56,64,67,72,80,90,96,110,120,128,133,140,160,192 > gpurun_out/r4i_rpw_t8.log 2>&1 &&
timeout -k 10 200 python -u scripts/stencil_rpw_lab.py 8 2048 4,8 10,12,14,16,18,20,22,24,28,32,40 > gpurun_out/r4i_rpw_t8_2048.log 2>&1 &&
timeout -k 10 200 python -u scripts/stencil_rpw_lab.py 6 2048 4 14,16,18,20,22,24,26,27,28,29,30,32,36,40,48 > gpurun_out/r4i_rpw_t6_2048.log 2>&1 &&
timeout -k 10 200 python -u scripts/stencil_rpw_lab.py 6 16384 8,4 48,64,67,80,96,133 > gpurun_out/r4i_rpw_t6.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "spmv or bench or stencil" > gpurun_out/r4i_tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/spmv_rank_lab.py 8 4 > gpurun_out/r4i_spmv_rank.log 2>&1
