/* bin/matrix_demo [--compat] — the reference's 1-introduction/matrix.c program (main :117-225): builds the
 * 3x4, 4x4 and 5x5 matrices and exercises the whole matrix_t API, printing the same lines.
 * --compat reproduces bug B1's printed "is sparse" values. Large products go to the registered GEMM
 * backend (the MFMA SGEMM when libpcmx_hip registered itself; host blocked SGEMM otherwise). */
#include <string.h>
#include "pcmx_cpu.h"

int main(int argc, char** argv) {
    int compat = 0;
    for (int i = 1; i < argc; ++i)
        if (!strcmp(argv[i], "--compat")) compat = 1;
    return pcmx_matrix_demo(compat) == 0 ? 0 : 1;
}
