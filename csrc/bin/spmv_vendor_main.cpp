/* bin/spmv_vendor [n_rows] [nnz] [reps] [warmup] [row0 row1 [device]] — the vendor-library bar of the north-star SpMV config: the same
 * 1e8-nnz power-law CSR matrix (libpcmx_cpu generator, bit-identical to the bench's) times x on the GPU through
 * rocSPARSE's generic SpMV, analysis/preprocess done ONCE, only the compute stage timed, for every CSR algorithm
 * rocSPARSE offers. Timed like bench.py's own sections: `warmup` untimed calls, then `reps` back-to-back compute
 * calls between two HIP events, the mean per call. The result is checked against an fp64 host product. One JSON
 * line.
 * A standalone process linked against /opt/rocm's rocSPARSE + HIP (not torch's copies): bench.py runs it as a
 * child process after its own sections (torch's sparse CSR path re-analyses the matrix on every call, which is
 * why its own bar, torch_sparse_csr_gflops, reads ~6 GFLOP/s).
 * With row0 row1 (N > 1: one child per rank, each on its rank's GPU `device`): the product of rows [row0, row1) of
 * the same matrix (a rank's block, generated alone by pcmx_powerlaw_fill_rows) with the whole x — the rank's local
 * product with no exchange, which bench.py times on every rank at once and aggregates by the slowest rank. */
#include <hip/hip_runtime.h>
#include <rocsparse/rocsparse.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pcmx_cpu.h"

#define HCK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "spmv_vendor: %s at line %d: %s\n", #x, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)
#define RCK(x)                                                                              \
    do {                                                                                    \
        rocsparse_status s_ = (x);                                                          \
        if (s_ != rocsparse_status_success) {                                               \
            fprintf(stderr, "spmv_vendor: %s at line %d: status %d\n", #x, __LINE__, (int)s_); \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

int main(int argc, char** argv) {
    const int n = argc > 1 ? (int)atof(argv[1]) : 10000000;
    const long long target = argc > 2 ? (long long)atof(argv[2]) : 100000000LL;
    const int reps = std::max(1, argc > 3 ? atoi(argv[3]) : 10);
    const int warmup = std::max(0, argc > 4 ? atoi(argv[4]) : 3);
    std::vector<long long> rp64(n + 1);
    const long long nnz_all = pcmx_powerlaw_row_counts(n, target, 2.5, 1, rp64.data());
    const int row0 = argc > 6 ? atoi(argv[5]) : 0, row1 = argc > 6 ? atoi(argv[6]) : n;
    if (row0 < 0 || row1 > n || row0 >= row1) return 2;
    if (argc > 7) HCK(hipSetDevice(atoi(argv[7])));
    const int m = row1 - row0;                           // rows of this product (all n without a row range)
    const long long nnz = rp64[row1] - rp64[row0];
    std::vector<int> col(nnz), rp(m + 1);
    std::vector<float> val(nnz), x(n), y(m);
    std::vector<double> yref(m);
    if (nnz >= (1LL << 31)) return 2;
    if (row0 == 0 && row1 == n)
        pcmx_powerlaw_fill(n, n, rp64.data(), 1, col.data(), val.data());
    else
        pcmx_powerlaw_fill_rows(row0, row1, n, rp64.data(), 1, col.data(), val.data());
    for (int i = 0; i <= m; ++i) rp[i] = (int)(rp64[row0 + i] - rp64[row0]);
    unsigned s = 12345u;
    for (auto& v : x) {
        s = s * 1664525u + 1013904223u;
        v = (float)(s >> 8) * (1.f / 16777216.f);
    }

    for (int i = 0; i < m; ++i) {  // fp64 reference
        double acc = 0.0;
        for (int j = rp[i]; j < rp[i + 1]; ++j) acc += (double)val[j] * (double)x[col[j]];
        yref[i] = acc;
    }

    int *drp, *dcol;
    float *dval, *dx, *dy;
    HCK(hipMalloc(&drp, sizeof(int) * (m + 1)));
    HCK(hipMalloc(&dcol, sizeof(int) * nnz));
    HCK(hipMalloc(&dval, sizeof(float) * nnz));
    HCK(hipMalloc(&dx, sizeof(float) * n));
    HCK(hipMalloc(&dy, sizeof(float) * m));
    HCK(hipMemcpy(drp, rp.data(), sizeof(int) * (m + 1), hipMemcpyHostToDevice));
    HCK(hipMemcpy(dcol, col.data(), sizeof(int) * nnz, hipMemcpyHostToDevice));
    HCK(hipMemcpy(dval, val.data(), sizeof(float) * nnz, hipMemcpyHostToDevice));
    HCK(hipMemcpy(dx, x.data(), sizeof(float) * n, hipMemcpyHostToDevice));

    rocsparse_handle h;
    RCK(rocsparse_create_handle(&h));
    rocsparse_spmat_descr A;
    rocsparse_dnvec_descr vx, vy;
    RCK(rocsparse_create_csr_descr(&A, m, n, nnz, drp, dcol, dval, rocsparse_indextype_i32, rocsparse_indextype_i32,
                                   rocsparse_index_base_zero, rocsparse_datatype_f32_r));
    RCK(rocsparse_create_dnvec_descr(&vx, n, dx, rocsparse_datatype_f32_r));
    RCK(rocsparse_create_dnvec_descr(&vy, m, dy, rocsparse_datatype_f32_r));
    const float one = 1.f, zero = 0.f;
    hipEvent_t e0, e1;
    HCK(hipEventCreate(&e0));
    HCK(hipEventCreate(&e1));
    const struct {
        rocsparse_spmv_alg alg;
        const char* name;
    } algs[] = {{rocsparse_spmv_alg_csr_adaptive, "csr_adaptive"},
                {rocsparse_spmv_alg_csr_rowsplit, "csr_rowsplit"}};
    // csr_lrb is NOT run: on this 1e7-row power-law matrix (ROCm 7.2 rocSPARSE) its compute stage returned after
    // 4.6 us without writing y and the next launch reported an illegal memory access (a GPU fault inside the
    // library), so it is excluded; csr_nnzsplit never ran because of it (profiles/r3_spmv/rocsparse_vendor.txt).
    printf("{\"metric\": \"rocSPARSE SpMV (generic API, preprocess once), power-law CSR\", \"n_rows\": %d, \"nnz\": %lld"
           ", \"row0\": %d, \"row1\": %d, \"nnz_all\": %lld",
           n, nnz, row0, row1, nnz_all);
    double best = 0.0;
    for (const auto& a : algs) {
        size_t bytes = 0;
        rocsparse_status st = rocsparse_spmv(h, rocsparse_operation_none, &one, A, vx, &zero, vy, rocsparse_datatype_f32_r,
                                             a.alg, rocsparse_spmv_stage_buffer_size, &bytes, nullptr);
        if (st != rocsparse_status_success) {
            printf(", \"%s\": \"unsupported (status %d)\"", a.name, (int)st);
            continue;
        }
        void* buf = nullptr;
        HCK(hipMalloc(&buf, bytes ? bytes : 16));
        RCK(rocsparse_spmv(h, rocsparse_operation_none, &one, A, vx, &zero, vy, rocsparse_datatype_f32_r, a.alg,
                           rocsparse_spmv_stage_preprocess, &bytes, buf));
        for (int r = 0; r < warmup; ++r)
            RCK(rocsparse_spmv(h, rocsparse_operation_none, &one, A, vx, &zero, vy, rocsparse_datatype_f32_r, a.alg,
                               rocsparse_spmv_stage_compute, &bytes, buf));
        HCK(hipDeviceSynchronize());
        HCK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r)
            RCK(rocsparse_spmv(h, rocsparse_operation_none, &one, A, vx, &zero, vy, rocsparse_datatype_f32_r, a.alg,
                               rocsparse_spmv_stage_compute, &bytes, buf));
        HCK(hipEventRecord(e1));
        HCK(hipEventSynchronize(e1));
        float total_ms = 0;
        HCK(hipEventElapsedTime(&total_ms, e0, e1));
        const double ms = total_ms / reps;
        HCK(hipMemcpy(y.data(), dy, sizeof(float) * m, hipMemcpyDeviceToHost));
        double err = 0.0, scale = 1e-30;
        for (int i = 0; i < m; ++i) {
            err = std::max(err, std::fabs((double)y[i] - yref[i]));
            scale = std::max(scale, std::fabs(yref[i]));
        }
        const double gf = 2.0 * nnz / (ms * 1e-3) / 1e9;
        best = std::max(best, gf);
        printf(", \"%s_ms\": %.4f, \"%s_gflops\": %.2f, \"%s_max_rel_err\": %.3g", a.name, ms, a.name, gf, a.name,
               err / scale);
        HCK(hipFree(buf));
    }
    printf(", \"best_gflops\": %.2f}\n", best);
    rocsparse_destroy_spmat_descr(A);
    rocsparse_destroy_dnvec_descr(vx);
    rocsparse_destroy_dnvec_descr(vy);
    rocsparse_destroy_handle(h);
    return 0;
}
