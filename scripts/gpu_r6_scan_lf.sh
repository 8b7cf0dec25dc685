# round 6: parked scan with the next tile's loads issued before the scan (variant 5) against production (4)
set -o pipefail
mkdir -p gpurun_out/r6/scan
timeout -k 10 300 python -u -m pytest tests/test_gpu_core.py -x -q -k "scan" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/scan/test.txt 2>&1 && \
timeout -k 10 300 python -u scripts/scan_tune.py 1e9 4,7,8 4 > gpurun_out/r6/scan/lf_ab.txt 2>&1
