// Device runtime utilities: device-info printer (replaces print_properties, ref 5-cuda-region-growing/
// raycast.cu:99-110, and printPlatformInfo/printDeviceInfo, ref 6-opencl-region-growing/clutil.c:63-122),
// error strings (clErrorStr, clutil.c:5-55) and the host-matrix GEMM backend that matrix_multiply()
// (libpcmx_cpu, ref 1-introduction/matrix.c:63-81) dispatches to for large products.
#include <stdio.h>
#include <stdlib.h>
#include "pcmx_common.h"
#include "pcmx_cpu.h"
#include "pcmx_hip.h"
#include <string.h>

extern "C" int pcmx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" const char* pcmx_error_string(int err) {
    switch (err) {
        case PCMX_ERR_ARG: return "pcmx: shape/alignment/argument precondition violated";
        case PCMX_ERR_NOT_CONVERGED: return "pcmx: not converged within max_launches (result incomplete)";
        case PCMX_ERR_TIMEOUT: return "pcmx: bounded wait timed out (result invalid)";
        case PCMX_ERR_COMM: return "pcmx: communication failed";
        case PCMX_ERR_ALLOC: return "pcmx: allocation failed";
        default: return err < 0 ? "pcmx: unknown error" : hipGetErrorString((hipError_t)err);
    }
}

extern "C" void pcmx_print_device_info(int device) {
    int count = pcmx_device_count();
    printf("Device count: %d\n", count);
    if (count == 0) return;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) {
        printf("hipGetDeviceProperties failed for device %d\n", device);
        return;
    }
    printf("Name: %s\n", p.name[0] ? p.name : p.gcnArchName);
    printf("Architecture: %s (compute capability %d.%d)\n", p.gcnArchName, p.major, p.minor);
    printf("Compute units: %d, wavefront size: %d\n", p.multiProcessorCount, p.warpSize);
    printf("LDS per workgroup: %zu KiB, max threads per workgroup: %d\n", p.sharedMemPerBlock / 1024,
           p.maxThreadsPerBlock);
    printf("L2 cache: %d KiB, global memory: %.1f GiB\n", p.l2CacheSize / 1024,
           (double)p.totalGlobalMem / (1024.0 * 1024.0 * 1024.0));
    printf("Clock: %d MHz, memory clock: %d MHz, bus width: %d bit\n", p.clockRate / 1000, p.memoryClockRate / 1000,
           p.memoryBusWidth);
    printf("\n\n");
}

// ---- host-array SGEMM for matrix_t: copy in, pad to the MFMA tile, run, copy out ---------------
static int round_up(int x, int m) { return (x + m - 1) / m * m; }

extern "C" int pcmx_sgemm_host_arrays(const float* a, const float* b, float* c, int m, int n, int k) {
    if (pcmx_device_count() == 0) return (int)hipErrorNoDevice;
    // PCMX_SGEMM_PRECISION=bf16x6: the fp32-accurate GEMM on the bf16 matrix cores (sgemm_x6.hip, 256x256 tiles,
    // K % 32); otherwise the padding of the kernel pcmx_sgemm_f32 will pick: 256x256 tiles and K % 64
    // (direct-register variant 17) when the problem fills the chip with 256-tiles, else 128x128 tiles
    const char* prec = getenv("PCMX_SGEMM_PRECISION");
    const bool x6 = prec && strcmp(prec, "bf16x6") == 0;
    const bool big = x6 || (long long)((m + 255) / 256) * ((n + 255) / 256) >= 192;
    const int mp = round_up(m, big ? 256 : 128), np = round_up(n, big ? 256 : 128),
              kp = round_up(k, big && !x6 ? 64 : 32);
    float *da = nullptr, *db = nullptr, *dc = nullptr;
    int rc = 0;
    if (hipMalloc(&da, sizeof(float) * (size_t)mp * kp) != hipSuccess || hipMalloc(&db, sizeof(float) * (size_t)kp * np) != hipSuccess ||
        hipMalloc(&dc, sizeof(float) * (size_t)mp * np) != hipSuccess) {
        rc = PCMX_ERR_ALLOC;
        goto done;
    }
    PCMX_HIP_CHECK(hipMemset(da, 0, sizeof(float) * (size_t)mp * kp));
    PCMX_HIP_CHECK(hipMemset(db, 0, sizeof(float) * (size_t)kp * np));
    PCMX_HIP_CHECK(hipMemcpy2D(da, sizeof(float) * kp, a, sizeof(float) * k, sizeof(float) * k, m, hipMemcpyHostToDevice));
    PCMX_HIP_CHECK(hipMemcpy2D(db, sizeof(float) * np, b, sizeof(float) * n, sizeof(float) * n, k, hipMemcpyHostToDevice));
    rc = x6 ? pcmx_sgemm_f32_x6(da, db, dc, mp, np, kp, kp, np, np, 1.0f, 0.0f, 0)
            : pcmx_sgemm_f32(da, db, dc, mp, np, kp, kp, np, np, 1.0f, 0.0f, 0);
    if (rc == 0) {
        PCMX_HIP_CHECK(hipMemcpy2D(c, sizeof(float) * n, dc, sizeof(float) * np, sizeof(float) * n, m, hipMemcpyDeviceToHost));
    }
done:
    if (da) (void)hipFree(da);
    if (db) (void)hipFree(db);
    if (dc) (void)hipFree(dc);
    return rc;
}

extern "C" void pcmx_register_gemm_backend(long long min_flops) {
    pcmx_set_gemm_backend(pcmx_sgemm_host_arrays, min_flops);
}
