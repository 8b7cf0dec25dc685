set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "spmv or bench" > gpurun_out/r4h_tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/spmv_rank_lab.py 8 4 > gpurun_out/r4h_spmv_rank.log 2>&1
