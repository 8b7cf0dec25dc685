# round 6: the deep-halo step's edge launch shape (two 30-row bands at T = 6, m = 5; production 4 columns x 2-row
# waves) swept for one N = 8 / N = 4 rank
set -o pipefail
mkdir -p gpurun_out/r6/stencil
for e in 0:0 4:2 4:3 4:4 4:6 4:10 8:2 8:4 4:2 0:0; do
  STENCIL_LAB_EDGE=$e STENCIL_LAB_WORLDS=8,4 STENCIL_LAB_DEEP=5 STENCIL_LAB_ONLY=full timeout -k 10 120 python -u scripts/stencil_rank_lab.py 6 >> gpurun_out/r6/stencil/edge_sweep.txt 2>&1 || exit 1
  echo "edge $e done" >> gpurun_out/r6/stencil/edge_sweep.txt
done
