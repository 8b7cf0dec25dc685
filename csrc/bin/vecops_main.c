/* bin/vecops [n] [n_threads] [reps] — north-star config 1: vector-add + dot product of 1e7 f32 on the host
 * with OpenMP (the host side of 6-opencl-region-growing/multiply_opencl.c:10-14, scaled up). Prints a human
 * line per op and one JSON line (GB/s). n_threads 0 = OpenMP default. */
#include <stdlib.h>
#include "pcmx_cpu.h"

int main(int argc, char** argv) {
    long long n = argc > 1 ? (long long)atof(argv[1]) : 10000000LL;
    int threads = argc > 2 ? atoi(argv[2]) : 0;
    int reps = argc > 3 ? atoi(argv[3]) : 20;
    if (n < 1 || reps < 1) return 2;
    return pcmx_vecops_demo(n, threads, reps) == 0 ? 0 : 1;
}
