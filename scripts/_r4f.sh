set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/spmv_banded_lab.py 100000 401 200 100 200 10 1,8 > gpurun_out/r4f_banded.log 2>&1 &&
bash scripts/pmc_banded.sh gpurun_out/r4f_banded_pmc > gpurun_out/r4f_pmc.log 2>&1 &&
bash scripts/gpu_round_check.sh r4f
