/* bin/histogram_{serial,omp,pthreads} image n_threads — the three programs of
 * 4-histogram-equalization-openmp-pthreads (histogram_serial.c:11-42, histogram_omp.c, histogram_pthreads.c:70-93).
 * One source, three tools selected at compile time (-DPCMX_TOOL_HISTOGRAM_*). Writes ./out.bmp; same argv and
 * usage text as the reference. The serial tool accepts and ignores n_threads, as the reference does. */
#include <stdio.h>
#include <stdlib.h>
#include "pcmx_cpu.h"

#if defined(PCMX_TOOL_HISTOGRAM_OMP)
#define METHOD 1
#elif defined(PCMX_TOOL_HISTOGRAM_PTHREADS)
#define METHOD 2
#else
#define METHOD 0
#endif

int main(int argc, char** argv) {
    if (argc != 3) {
        printf("Useage: %s image n_threads\n", argv[0]);
        exit(-1);
    }
    int n_threads = atoi(argv[2]);
    if (n_threads < 1) n_threads = 1;
    return pcmx_histogram_demo(argv[1], n_threads, METHOD) == 0 ? 0 : 1;
}
