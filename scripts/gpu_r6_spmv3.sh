# round 6: native exchange event scopes (0 / 1 / 2) in the N = 8 rank lab; raycast variant tests
set -o pipefail
mkdir -p gpurun_out/r6
for sc in 0 1 2; do
  PCMX_XCOMM_EVENT_SCOPE=$sc SPMV_LAB_KINDS=paired SPMV_LAB_RCCL=1 SPMV_LAB_FRAC=0.5 SPMV_LAB_N1=0 timeout -k 10 300 python -u scripts/spmv_host_lab.py 8 40 > gpurun_out/r6/spmv_native_scope$sc.txt 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread -k "raycast" > gpurun_out/r6/test_raycast.txt 2>&1
