// Cross-stream wait lab (round 6, SpMV exchange): what a compute stream pays to wait for work on another stream of the
// same GPU. Two one-block kernels K1 -> K2 on stream A stamp the GPU wall clock (wall_clock64, 100 MHz) at their end /
// start; the gap K2.start - K1.end is printed (median and min of 30 repeats) for:
//   none      K1, K2 back to back on A
//   event     hipStreamWaitEvent(A, e) between them, e recorded on stream B long before (already complete)
//   event_dev the same with an event created with hipEventReleaseToDevice
//   pending   e recorded on B after a kernel that ends while K1 runs (the wait resolves mid-K1)
//   value     hipStreamWaitValue32(A, flag >= k) with the flag written by hipStreamWriteValue32 on B long before
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/stream_wait_lab.hip -o bin_lab/stream_wait_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            return 1;                                                        \
        }                                                                    \
    } while (0)

__global__ void stamp_kernel(unsigned long long* out, int idx, unsigned spin_ticks) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();
    out[2 * idx] = t0;
    unsigned long long t = t0;
    while (t - t0 < spin_ticks) t = wall_clock64();  // bounded: 100 MHz ticks
    out[2 * idx + 1] = t;
}

int main() {
    unsigned long long* st;
    unsigned* flag;
    CK(hipMalloc(&st, 64 * sizeof(unsigned long long)));
    CK(hipMalloc(&flag, 64));
    CK(hipMemset(flag, 0, 64));
    hipStream_t A, B;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    hipEvent_t e, enf;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&enf, hipEventDisableTiming | hipEventReleaseToDevice));
    const unsigned k1_ticks = 2000;  // K1 runs 20 us
    const char* names[] = {"none", "event", "event_dev", "pending", "value"};
    unsigned long long host[4];
    for (int mode = 0; mode < 5; ++mode) {
        std::vector<double> gaps;
        for (int rep = 0; rep < 30; ++rep) {
            if (mode == 1 || mode == 2) {
                stamp_kernel<<<1, 64, 0, B>>>(st, 3, 10);
                CK(hipEventRecord(mode == 1 ? e : enf, B));
                CK(hipStreamSynchronize(B));
            }
            if (mode == 4) {
                CK(hipStreamWriteValue32(B, flag, (unsigned)rep + 1, 0));
                CK(hipStreamSynchronize(B));
            }
            stamp_kernel<<<1, 64, 0, A>>>(st, 0, k1_ticks);
            if (mode == 3) {  // B's kernel ends ~10 us into K1
                stamp_kernel<<<1, 64, 0, B>>>(st, 3, 1000);
                CK(hipEventRecord(e, B));
            }
            if (mode == 1 || mode == 3) CK(hipStreamWaitEvent(A, e, 0));
            if (mode == 2) CK(hipStreamWaitEvent(A, enf, 0));
            if (mode == 4) CK(hipStreamWaitValue32(A, flag, (unsigned)rep + 1, hipStreamWaitValueGte, 0xffffffffu));
            stamp_kernel<<<1, 64, 0, A>>>(st, 1, 10);
            CK(hipStreamSynchronize(A));
            CK(hipStreamSynchronize(B));
            CK(hipMemcpy(host, st, sizeof(host), hipMemcpyDeviceToHost));
            gaps.push_back((double)(host[2] - host[1]) * 0.01);  // ticks of 10 ns -> us
        }
        std::sort(gaps.begin(), gaps.end());
        printf("%-9s K1.end -> K2.start: median %7.2f us, min %7.2f us, max %7.2f us\n", names[mode], gaps[gaps.size() / 2],
               gaps.front(), gaps.back());
        fflush(stdout);
    }
    return 0;
}
