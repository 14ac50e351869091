// gather.hip -- host-memory gather into HBM: the kernel reads page-locked
// host bytes (hipHostMalloc'd slots, krk_host_alloc blocks, or caller memory the library
// registered with hipHostRegister for the call) straight over PCIe and writes them into a
// device window, one launch for thousands of chunks.  It replaces, for the host-resident
// batches, the pageable -> pinned staging copy (a host-DRAM read AND write per byte, on
// host threads) followed by the DMA read: the bytes are read from host DRAM once, by the
// GPU.  Measured on MI355X (tools/micro/gather_probe.hip, profiles/r05/gather_probe.jsonl):
// 57.0 GB/s for 1,000 chunks of 512 KiB and 55.0 GB/s for 14,339 chunks of 36 KiB, against
// 54.7 GB/s for one pinned DMA of a 512 MiB window and 25.5 / 3.4 GB/s for per-chunk DMA
// of the same chunks.
//
// A tile is <= kGatherTile bytes of one chunk; a workgroup (4 waves) copies a tile as 16-byte
// words: lane i of a wave loads the source's 16-B-aligned word i, and when the source is not
// 16-B aligned takes word i+1 from lane i+1 (the wave's last lane loads it) and funnel-shifts
// the pair (v_alignbyte).  Only aligned words that hold at least one of the tile's bytes are
// read, so no load leaves the pages the chunk lies in.  The destination is 16-B aligned and
// has room up to the next multiple of 16 (the window's chunk placement).
#include "device_util.hpp"
#include "kernels.hpp"

namespace krk {

namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4u shfl_down1(v4u v) {
    v4u o;
    o.x = __shfl_down(v.x, 1, 64);
    o.y = __shfl_down(v.y, 1, 64);
    o.z = __shfl_down(v.z, 1, 64);
    o.w = __shfl_down(v.w, 1, 64);
    return o;
}

// bytes [4Q + S, 4Q + S + 16) of the 32-byte pair (a, b): dword k from dwords Q + k and
// Q + k + 1 (v_alignbyte by S bytes; S == 0 takes the dword as is)
template <int Q>
__device__ __forceinline__ v4u funnel_q(v4u a, v4u b, uint32_t S) {
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    v4u o;
    o.x = S ? __builtin_amdgcn_alignbyte(w[Q + 1], w[Q], S) : w[Q];
    o.y = S ? __builtin_amdgcn_alignbyte(w[Q + 2], w[Q + 1], S) : w[Q + 1];
    o.z = S ? __builtin_amdgcn_alignbyte(w[Q + 3], w[Q + 2], S) : w[Q + 2];
    o.w = S ? __builtin_amdgcn_alignbyte(w[Q + 4], w[Q + 3], S) : w[Q + 3];
    return o;
}
// bytes [r, r + 16) of the pair, r in 1..15 (uniform in the workgroup: one tile at a time)
__device__ __forceinline__ v4u funnel(v4u a, v4u b, uint32_t r) {
    switch (r >> 2) {
        case 0: return funnel_q<0>(a, b, r & 3);
        case 1: return funnel_q<1>(a, b, r & 3);
        case 2: return funnel_q<2>(a, b, r & 3);
        default: return funnel_q<3>(a, b, r & 3);
    }
}

constexpr int kGatherThreads = 256;
constexpr int kUnroll = 4;

__global__ void __launch_bounds__(kGatherThreads) gather_kernel(const GatherTile* __restrict__ tiles, uint32_t n_tiles) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        const GatherTile T = tiles[t];
        const uint32_t r = (uint32_t)(T.src & 15);
        const gptr<v4u> s = as_global<v4u>(T.src - r);  // the aligned words (global_load, not flat)
        v4u* __restrict__ d = reinterpret_cast<v4u*>(T.dst);
        const uint64_t out_words = (T.n + 15) / 16;
        const uint64_t in_words = (r + T.n + 15) / 16;  // aligned words holding tile bytes
        for (uint64_t base = (uint64_t)wave * 64 * kUnroll; base < out_words;
             base += (uint64_t)(kGatherThreads / 64) * 64 * kUnroll) {
            v4u v[kUnroll], nx[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint64_t i = base + (uint64_t)u * 64 + lane;
                v[u] = i < in_words ? __builtin_nontemporal_load(s + i) : v4u{0, 0, 0, 0};
                // the word after the wave's last: the last lane loads it itself
                const uint64_t j = base + (uint64_t)u * 64 + 64;
                nx[u] = (r && lane == 63 && j < in_words) ? __builtin_nontemporal_load(s + j) : v4u{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint64_t i = base + (uint64_t)u * 64 + lane;
                v4u o = v[u];
                if (r) {
                    const v4u up = shfl_down1(v[u]);
                    o = funnel(v[u], lane == 63 ? nx[u] : up, r);
                }
                if (i < out_words) d[i] = o;
            }
        }
    }
}

}  // namespace

hipError_t launch_gather(const GatherTile* tiles, uint32_t n_tiles, int cus, hipStream_t s) {
    if (!n_tiles) return hipSuccess;
    const hipError_t pre = launch_precheck();
    if (pre != hipSuccess) return pre;
    // one workgroup a CU is enough to keep the link busy (the probe: 256 / 1,024 / 4,096
    // workgroups within 2 %); more would only take CUs from the kernels beside it
    const uint32_t grid = std::min<uint32_t>(n_tiles, (uint32_t)std::max(64, cus));
    t_launch_plan = 0;
    t_launch_units = n_tiles;
    hipLaunchKernelGGL(gather_kernel, dim3(grid), dim3(kGatherThreads), 0, s, tiles, n_tiles);
    return hipGetLastError();
}

}  // namespace krk
