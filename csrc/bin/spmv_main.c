/* bin/spmv dim a b c d e — the reference's 3-serial-optimization/spmv.c program (main :331-367): builds the
 * 5-band CSR matrix, times the naive CSR product and the implicit-index banded product ("Time : %f s" each)
 * and prints compare()'s report. Same argv and usage text as the reference (spmv.c:333-336). */
#include <stdio.h>
#include <stdlib.h>
#include "pcmx_cpu.h"

int main(int argc, char** argv) {
    if (argc != 7) {
        printf("useage %s dim a b c d e\n", argv[0]);
        exit(-1);
    }
    int v[6];
    for (int i = 0; i < 6; ++i) v[i] = atoi(argv[i + 1]);
    return pcmx_spmv_demo(v[0], v[1], v[2], v[3], v[4], v[5]) == 0 ? 0 : 1;
}
