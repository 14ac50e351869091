// join_probe.hip -- the C3 window loop's fork/join pattern under event churn from another
// thread.  chunks_step (runtime.cpp) forks a caller stream R onto two device streams
// (hipEventRecord(fork, R); SA, SB wait on it), launches there, records j1 / j2 and makes
// R wait on them, destroying the three events at once; the window loop then waits on an
// event recorded on R, and the run ends with hipStreamSynchronize(R).  The C3 host-lane
// test saw the last windows' piece CRCs (SB) missing when the sums were read after that
// sync.  Here SB's kernel writes flag[k] after a short spin; after the final sync of R
// every flag must be set.  A second thread meanwhile creates, records and destroys events
// and launches short kernels on streams of its own (normal and high priority).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

__global__ void spin_set(uint64_t ticks, uint32_t* flag, uint32_t k) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) flag[k] = 1u;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    int rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    const uint64_t ms = (uint64_t)rate_khz;  // ticks a millisecond
    hipStream_t R, SA, SB;
    CK(hipStreamCreateWithFlags(&R, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&SA, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&SB, hipStreamNonBlocking));
    uint32_t *flag, *scratch;
    CK(hipMalloc(&flag, iters * 4));
    CK(hipMemset(flag, 0, iters * 4));
    CK(hipMalloc(&scratch, 4096 * 4));
    std::atomic<bool> stop{false};
    std::atomic<long> churn{0};
    std::thread other([&] {
        hipSetDevice(0);
        int least = 0, greatest = 0;
        hipDeviceGetStreamPriorityRange(&least, &greatest);
        hipStream_t o[4];
        for (int i = 0; i < 4; ++i)
            hipStreamCreateWithPriority(&o[i], hipStreamNonBlocking, (i & 1) ? greatest : 0);
        for (long n = 0; !stop.load(); ++n) {
            hipEvent_t e;
            hipEventCreateWithFlags(&e, hipEventDisableTiming);
            spin_set<<<1, 64, 0, o[n & 3]>>>(ms / 20, scratch, (uint32_t)(n & 4095));
            hipEventRecord(e, o[n & 3]);
            if (n % 7 == 0) hipStreamWaitEvent(o[(n + 1) & 3], e, 0);
            hipEventDestroy(e);
            if (n % 64 == 0) hipStreamSynchronize(o[n & 3]);
            churn.fetch_add(1);
        }
        for (int i = 0; i < 4; ++i) hipStreamSynchronize(o[i]), hipStreamDestroy(o[i]);
    });
    hipEvent_t evs[2];
    CK(hipEventCreateWithFlags(&evs[0], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&evs[1], hipEventDisableTiming));
    int early = 0;
    for (int k = 0; k < iters; ++k) {
        hipEvent_t fork, j1, j2;
        CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&j2, hipEventDisableTiming));
        CK(hipEventRecord(fork, R));
        CK(hipStreamWaitEvent(SA, fork, 0));
        CK(hipStreamWaitEvent(SB, fork, 0));
        spin_set<<<1, 64, 0, SA>>>(ms * 2, scratch + 4000, 0);  // the window's SHA launch
        spin_set<<<1, 64, 0, SB>>>(ms, flag, (uint32_t)k);      // its CRC launch
        CK(hipEventRecord(j1, SA));
        CK(hipEventRecord(j2, SB));
        CK(hipStreamWaitEvent(R, j1, 0));
        CK(hipStreamWaitEvent(R, j2, 0));
        CK(hipEventDestroy(fork));
        CK(hipEventDestroy(j1));
        CK(hipEventDestroy(j2));
        CK(hipEventRecord(evs[k & 1], R));
        if (k) CK(hipEventSynchronize(evs[(k - 1) & 1]));
        if (k) {  // window k-1 is done: its flag must be set
            uint32_t f = 0;
            CK(hipMemcpy(&f, flag + (k - 1), 4, hipMemcpyDeviceToHost));
            early += f == 0;
        }
    }
    CK(hipStreamSynchronize(R));
    std::vector<uint32_t> h(iters);
    CK(hipMemcpy(h.data(), flag, iters * 4, hipMemcpyDeviceToHost));
    stop = true;
    other.join();
    int missing = 0;
    for (int k = 0; k < iters; ++k) missing += h[k] == 0;
    printf("{\"iters\": %d, \"churn\": %ld, \"early_event_done\": %d, \"missing_after_sync\": %d, \"join_ok\": %s}\n", iters,
           churn.load(), early, missing, (early || missing) ? "false" : "true");
    return 0;
}
