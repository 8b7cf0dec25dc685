/* bin/device_info — device introspection (replaces print_properties of 5-cuda-region-growing/raycast.cu:99-110
 * and printPlatformInfo/printDeviceInfo of 6-opencl-region-growing/clutil.c:63-122): device count, name,
 * gcnArchName (gfx950), CUs, LDS per CU, L2, HBM size and clocks of every visible MI355X. */
#include <cstdio>

#include "pcmx_hip.h"

int main() {
    const int n = pcmx_device_count();
    if (n <= 0) {
        printf("Number of devices: 0\n");
        return 1;
    }
    for (int d = 0; d < n; ++d) pcmx_print_device_info(d);
    return 0;
}
