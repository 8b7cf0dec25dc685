/* bin/vmul — the OpenCL vector-multiply demo (6-opencl-region-growing/multiply_opencl.c:16-85 with kernel
 * multiply_opencl.cl:1-4) as a HIP program: 1024 floats, a[i] = i + 1, b[i] = 1 / (i + 1), result = a * b on the
 * gfx950 vmul kernel; prints the device info, then "Host\tDevice" and the first 10 results ("%0.2f\t%0.2f").
 * Every HIP call is checked (the reference ignored most OpenCL return codes). */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pcmx_cpu.h"
#include "pcmx_hip.h"

#define CHECK(x)                                                                                         \
    do {                                                                                                 \
        int rc_ = (int)(x);                                                                              \
        if (rc_) {                                                                                       \
            fprintf(stderr, "%s:%d: %s failed: %s\n", __FILE__, __LINE__, #x, pcmx_error_string(rc_)); \
            exit(1);                                                                                     \
        }                                                                                                \
    } while (0)

int main() {
    constexpr int kSize = 1024;
    if (pcmx_device_count() <= 0) {
        fprintf(stderr, "vmul: no GPU visible\n");
        return 1;
    }
    pcmx_print_device_info(0);
    std::vector<float> a(kSize), b(kSize), host(kSize), dev(kSize);
    for (int i = 0; i < kSize; ++i) a[i] = (float)(i + 1), b[i] = 1.0f / (float)(i + 1);
    pcmx_vmul_host(a.data(), b.data(), host.data(), kSize);
    float *da = nullptr, *db = nullptr, *dr = nullptr;
    CHECK(hipMalloc(&da, kSize * sizeof(float)));
    CHECK(hipMalloc(&db, kSize * sizeof(float)));
    CHECK(hipMalloc(&dr, kSize * sizeof(float)));
    CHECK(hipMemcpy(da, a.data(), kSize * sizeof(float), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(db, b.data(), kSize * sizeof(float), hipMemcpyHostToDevice));
    CHECK(pcmx_vmul_f32(da, db, dr, kSize, nullptr));
    CHECK(hipMemcpy(dev.data(), dr, kSize * sizeof(float), hipMemcpyDeviceToHost));
    printf("Host\tDevice\n");
    for (int i = 0; i < 10; i++) printf("%0.2f\t%0.2f\n", host[i], dev[i]);
    CHECK(hipFree(da));
    CHECK(hipFree(db));
    CHECK(hipFree(dr));
    return 0;
}
