set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "banded" > gpurun_out/r4e_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/spmv_banded_lab.py 100000 401 200 100 200 10 1,8 > gpurun_out/r4e_banded.log 2>&1 &&
bash scripts/pmc_banded.sh gpurun_out/r4e_banded_pmc > gpurun_out/r4e_pmc.log 2>&1 &&
timeout -k 10 300 python -u scripts/spmv_store_lab.py 20 > gpurun_out/r4e_store.log 2>&1 &&
timeout -k 10 300 bin_lab/stream_bw_lab > gpurun_out/r4e_stream_bw.log 2>&1
