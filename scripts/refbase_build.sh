#!/bin/bash
# Builds the REFERENCE's OpenCL program (the only reference GPU code an MI355X can run: OpenCL C kernels JIT-compiled
# at run time by the AMD OpenCL runtime) from its own sources, for the same-hardware baseline (profiles/r5_refbase/).
# The sources are copied from /root/reference into refbase/ (git-ignored: never part of this repo's history; gpurun
# ships the directory to the GPU box with the built binaries) and compiled unmodified, exactly as the reference's
# Makefile does (gcc -std=c99 bmp.c clutil.c raycast.c -lOpenCL -lm), plus:
#   refbase/raycast_ref    the reference program itself (its main)
#   refbase/raycast_timed  the same objects with the reference main renamed and scripts/refbase_driver.c as main
#                          (times grow_region_gpu / raycast_gpu, prints region voxels and image sum)
#   refbase/wg256/         the same, with ONE change: the region kernel's work-group size {8, 8, 8} (512 work-items:
#                          above the 256 an MI355X OpenCL device allows, so the reference's unchecked launch fails and
#                          its grow never runs) lowered to {8, 8, 4}, the nearest launch the device accepts — the
#                          reference grow on the same hardware, everything else as written
# Run on the box from refbase/ (the program reads region.cl / raycast.cl from the working directory).
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
SRC=/root/reference/6-opencl-region-growing
OUT="$ROOT/refbase"
mkdir -p "$OUT"
for f in bmp.c bmp.h clutil.c clutil.h raycast.c raycast.cl region.cl; do cp "$SRC/$f" "$OUT/$f"; done
cd "$OUT"
gcc -std=c99 bmp.c clutil.c raycast.c -lOpenCL -lm -o raycast_ref 2> build_warnings.txt || { cat build_warnings.txt; exit 1; }
gcc -std=c99 -c raycast.c -Dmain=refbase_main -o raycast_ref_nomain.o 2>> build_warnings.txt
gcc -std=c99 bmp.c clutil.c raycast_ref_nomain.o "$ROOT/scripts/refbase_driver.c" -lOpenCL -lm -o raycast_timed \
    2>> build_warnings.txt
mkdir -p wg256
for f in bmp.c bmp.h clutil.c clutil.h raycast.cl region.cl; do cp "$f" wg256/; done
sed 's/size_t local\[\] = { 8, 8, 8 };/size_t local[] = { 8, 8, 4 };/' raycast.c > wg256/raycast.c
grep -q 'size_t local\[\] = { 8, 8, 4 };' wg256/raycast.c
(cd wg256 && gcc -std=c99 -c raycast.c -Dmain=refbase_main -o raycast_nomain.o 2>> ../build_warnings.txt &&
 gcc -std=c99 bmp.c clutil.c raycast_nomain.o "$ROOT/scripts/refbase_driver.c" -lOpenCL -lm -o raycast_timed \
   2>> ../build_warnings.txt)
echo "built $OUT/raycast_ref $OUT/raycast_timed $OUT/wg256/raycast_timed"
