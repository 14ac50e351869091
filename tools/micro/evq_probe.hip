// evq_probe.hip -- does hipEventQuery report an event recorded behind pending work as
// complete?  The upload() pinned slots and the DevCache scratch blocks are reused across
// streams once hipEventQuery(ev) == hipSuccess; the C3 host-lane GPU test saw piece sums
// XOR'd twice (a CRC pack overwritten before its copy ran), which would follow if it did.
//
//   S1  spin kernel on A, small pinned H2D on A, record e on A, query at once
//   S2  B waits on an event of A (after the spin), small pinned H2D on B, record e on B
//   S3  S2 with the query made from another host thread
//   S4  the upload() pattern: if the query says done, overwrite the pinned source; the
//       device copy must still hold the first contents
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

__global__ void spin(uint64_t ticks, uint32_t* out) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

static const char* qs(hipError_t e) { return e == hipSuccess ? "COMPLETE" : e == hipErrorNotReady ? "not-ready" : hipGetErrorString(e); }

int main() {
    int rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    const uint64_t ticks = (uint64_t)rate_khz * 300;  // 300 ms
    hipStream_t A, B, C;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking));
    uint32_t* flag;
    uint8_t *dev, *pin;
    CK(hipMalloc(&flag, 4));
    CK(hipMalloc(&dev, 256));
    CK(hipHostMalloc(reinterpret_cast<void**>(&pin), 256, hipHostMallocDefault));
    hipEvent_t ea, e;
    CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int bad = 0;
    for (int rep = 0; rep < 3; ++rep) {
        // S1
        memset(pin, 0x11, 256);
        spin<<<1, 64, 0, A>>>(ticks, flag);
        CK(hipMemcpyAsync(dev, pin, 200, hipMemcpyHostToDevice, A));
        CK(hipEventRecord(e, A));
        hipError_t q1 = hipEventQuery(e);
        CK(hipStreamSynchronize(A));
        // S2
        spin<<<1, 64, 0, A>>>(ticks, flag);
        CK(hipEventRecord(ea, A));
        CK(hipStreamWaitEvent(B, ea, 0));
        CK(hipMemcpyAsync(dev, pin, 200, hipMemcpyHostToDevice, B));
        CK(hipEventRecord(e, B));
        hipError_t q2 = hipEventQuery(e);
        CK(hipStreamSynchronize(B));
        // S3
        spin<<<1, 64, 0, A>>>(ticks, flag);
        CK(hipEventRecord(ea, A));
        CK(hipStreamWaitEvent(B, ea, 0));
        CK(hipMemcpyAsync(dev, pin, 200, hipMemcpyHostToDevice, B));
        CK(hipEventRecord(e, B));
        std::atomic<int> q3{-1};
        std::thread th([&] {
            hipSetDevice(0);
            spin<<<1, 64, 0, C>>>(1000, flag);  // other traffic from this thread
            q3 = (int)hipEventQuery(e);
        });
        th.join();
        CK(hipStreamSynchronize(B));
        CK(hipStreamSynchronize(C));
        // S4
        memset(pin, 0x22, 256);
        spin<<<1, 64, 0, A>>>(ticks, flag);
        CK(hipEventRecord(ea, A));
        CK(hipStreamWaitEvent(B, ea, 0));
        CK(hipMemcpyAsync(dev, pin, 200, hipMemcpyHostToDevice, B));
        CK(hipEventRecord(e, B));
        hipError_t q4 = hipEventQuery(e);
        if (q4 == hipSuccess) memset(pin, 0x33, 256);
        CK(hipStreamSynchronize(B));
        uint8_t back[200];
        CK(hipMemcpy(back, dev, 200, hipMemcpyDeviceToHost));
        int corrupt = 0;
        for (int i = 0; i < 200; ++i) corrupt += back[i] != 0x22;
        printf("{\"rep\": %d, \"S1\": \"%s\", \"S2\": \"%s\", \"S3\": \"%s\", \"S4\": \"%s\", \"S4_corrupt_bytes\": %d}\n", rep,
               qs(q1), qs(q2), qs((hipError_t)q3.load()), qs(q4), corrupt);
        bad += (q1 == hipSuccess) + (q2 == hipSuccess) + (q3.load() == (int)hipSuccess) + (q4 == hipSuccess) + (corrupt > 0);
    }
    printf("{\"query_ok\": %s}\n", bad ? "false" : "true");
    return 0;
}
