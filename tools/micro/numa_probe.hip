// numa_probe.hip -- does the NUMA node of the pinned staging buffer and of the copy
// threads matter for the host paths?  For the GPU's own node and the other node:
// pinned -> device (H2D) and device -> pinned (D2H) DMA rates, and the 16-thread
// pageable -> pinned memcpy of the end-to-end path.  The node of a pinned buffer is set by
// allocating it from a thread bound to that node's CPUs.
// Development tool; build: hipcc -O2 --offload-arch=gfx950 numa_probe.hip -o numa_probe -lpthread
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

// CPUs of NUMA node `node` from sysfs ("0-63,128-191").
static cpu_set_t node_cpus(int node) {
    cpu_set_t s;
    CPU_ZERO(&s);
    std::string path = "/sys/devices/system/node/node" + std::to_string(node) + "/cpulist";
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return s;
    char buf[4096] = {};
    if (!fgets(buf, sizeof buf, f)) buf[0] = 0;
    fclose(f);
    for (char* p = strtok(buf, ",\n"); p; p = strtok(nullptr, ",\n")) {
        int a = 0, b = 0;
        if (sscanf(p, "%d-%d", &a, &b) == 2)
            for (int c = a; c <= b; ++c) CPU_SET(c, &s);
        else if (sscanf(p, "%d", &a) == 1)
            CPU_SET(a, &s);
    }
    return s;
}

static int gpu_node() {
    char bus[64] = {};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, 0) != hipSuccess) return -1;
    for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
    std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
    FILE* f = fopen(path.c_str(), "r");
    int n = -1;
    if (f) {
        if (fscanf(f, "%d", &n) != 1) n = -1;
        fclose(f);
    }
    return n;
}

int main() {
    const size_t N = size_t(8) << 30, W = size_t(256) << 20;
    uint8_t* dev = nullptr;
    CK(hipMalloc((void**)&dev, N));
    CK(hipMemset(dev, 3, N));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int g = gpu_node();
    printf("{\"gpu_numa_node\": %d}\n", g);
    const int nodes[2] = {g < 0 ? 0 : g, g == 1 ? 0 : 1};
    uint8_t* src = (uint8_t*)aligned_alloc(4096, N);  // pageable source, first touched below
    for (int rep = 0; rep < 2; ++rep)
        for (int which = 0; which < 2; ++which) {
            const int node = nodes[which];
            cpu_set_t cs = node_cpus(node), all;
            sched_getaffinity(0, sizeof all, &all);
            sched_setaffinity(0, sizeof cs, &cs);
            uint8_t* pin = nullptr;
            CK(hipHostMalloc((void**)&pin, W, hipHostMallocDefault));
            memset(pin, 1, W);
            if (rep == 0 && which == 0) memset(src, 5, N);  // the pageable source lives on the GPU's node
            sched_setaffinity(0, sizeof all, &all);
            double t0 = now();
            for (size_t o = 0; o < N; o += W) CK(hipMemcpyAsync(dev + o, pin, W, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            const double h2d = N / (now() - t0) / 1e9;
            t0 = now();
            for (size_t o = 0; o < N; o += W) CK(hipMemcpyAsync(pin, dev + o, W, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            const double d2h = N / (now() - t0) / 1e9;
            double cp[2];
            for (int tn = 0; tn < 2; ++tn) {  // copy threads on the GPU's node, then anywhere
                t0 = now();
                for (size_t o = 0; o < N; o += W) {
                    std::vector<std::thread> th;
                    const size_t span = W / 16;
                    for (int i = 0; i < 16; ++i)
                        th.emplace_back([&, i] {
                            if (tn == 0) {
                                cpu_set_t c = node_cpus(nodes[0]);
                                sched_setaffinity(0, sizeof c, &c);
                            }
                            memcpy(pin + i * span, src + o + i * span, span);
                        });
                    for (auto& x : th) x.join();
                }
                cp[tn] = N / (now() - t0) / 1e9;
            }
            printf("{\"pinned_node\": %d, \"h2d_GBps\": %.2f, \"d2h_GBps\": %.2f, \"memcpy16_threads_on_gpu_node_GBps\": %.2f, "
                   "\"memcpy16_threads_anywhere_GBps\": %.2f}\n",
                   node, h2d, d2h, cp[0], cp[1]);
            fflush(stdout);
            CK(hipHostFree(pin));
        }
    return 0;
}
