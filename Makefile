# Convenience targets (the build itself is parallel_c_programs_amd/_build.py: in-tree, gfx950 only).
# Run targets mirror the reference Makefiles' `run` rules with MI355X-native programs.
PY      ?= python3
P       ?= 4
IMAGE   ?= assets/pic1.bmp

.PHONY: all cpu hip torch bin clean test test-gpu bench sanitize \
        run-matrix run-mpi run-region run-spmv run-histogram run-raycast run-raycast-opencl run-vmul

all:
	$(PY) -m parallel_c_programs_amd._build
cpu hip torch bin:
	$(PY) -m parallel_c_programs_amd._build --only $@
clean:
	rm -rf build bin parallel_c_programs_amd/lib parallel_c_programs_amd/_C.so

test:
	$(PY) -m pytest tests -q -m "not gpu"
test-gpu:
	$(PY) -m pytest tests -q -m gpu
bench:
	$(PY) bench.py
sanitize:
	$(PY) -m parallel_c_programs_amd.sanitize

# ---- reference programs
run-matrix: all                      # 1-introduction/matrix.c
	bin/matrix_demo
run-mpi: all                         # 1-introduction/mpi.c (mpirun -n P mpi)
	bin/pcmx_launch -n $(P) bin/mpi_ring
run-region: all                      # 2-mpi-region-growing/Makefile: mpirun -n P region pic1.bmp
	bin/pcmx_launch -n $(P) bin/region $(IMAGE)
run-spmv: all                        # 3-serial-optimization/Makefile: ./spmv 100000 401 200 100 200 10
	bin/spmv 100000 401 200 100 200 10
run-histogram: all                   # 4-histogram-*/Makefile: serial / omp / pthreads on peppers.bmp
	bin/histogram_serial assets/peppers.bmp 1 && bin/histogram_omp assets/peppers.bmp 4 && \
	bin/histogram_pthreads assets/peppers.bmp 4
run-raycast: all                     # 5-cuda-region-growing/Makefile
	bin/raycast
run-raycast-opencl: all              # 6-opencl-region-growing/Makefile (IMAGE_DIM 64, naive grow, global caster)
	bin/raycast --image-dim 64 --global --naive
run-vmul: all                        # 6-opencl-region-growing/multiply_opencl.c
	bin/vmul
