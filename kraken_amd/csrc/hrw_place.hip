// hrw_place.hip -- weighted rendezvous hashing for gfx950 (lib/hrw/rendezvous.go)
// and the hashring.Locations filter (lib/hashring/ring.go:96-118).
//
// Score(key, node) = -w / Log(UInt64ToFloat64(murmur3.New64(hexdecode(key) || label)))
// (rendezvous.go:151-172, 99-118).  One workgroup scores a tile of keys x all nodes
// (one thread per (key, node) pair, fp64 throughout, FP contraction off so every
// operation rounds exactly like Go's amd64 math.Log), keeps the scores in LDS and
// ranks each node by counting (descending score, ties -> lower node index).
#include "kernels.hpp"
#include "device_util.hpp"

namespace krk {

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return k;
}

// MurmurHash3_x64_128 h1, seed 0 (spaolacci/murmur3 New64, glide.lock:231-232) over
// the virtual message A[0..na) || B[0..nb).
__device__ uint64_t murmur3_h1_cat(const uint8_t* A, uint32_t na, const uint8_t* B, uint32_t nb) {
    const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    const uint32_t n = na + nb;
    auto at = [&](uint32_t i) -> uint64_t { return i < na ? A[i] : B[i - na]; };
    uint64_t h1 = 0, h2 = 0;
    const uint32_t nblk = n / 16;
    for (uint32_t b = 0; b < nblk; ++b) {
        uint64_t k1 = 0, k2 = 0;
#pragma unroll
        for (int q = 7; q >= 0; --q) {
            k1 = (k1 << 8) | at(16 * b + q);
            k2 = (k2 << 8) | at(16 * b + 8 + q);
        }
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint32_t t = 16 * nblk, r = n & 15;
    uint64_t k1 = 0, k2 = 0;
    for (int q = (int)r - 1; q >= 8; --q) k2 = (k2 << 8) | at(t + q);
    for (int q = (r < 8 ? (int)r : 8) - 1; q >= 0; --q) k1 = (k1 << 8) | at(t + q);
    if (r > 8) { k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; }
    if (r > 0) { k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1; }
    h1 ^= n; h2 ^= n;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    return h1 + h2;
}

// Go math.Log (src/math/log.go), operation for operation, no FMA.
__device__ double go_log(double x) {
#pragma clang fp contract(off)
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
                 L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
                 L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
                 L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                 L7 = 1.479819860511658591e-01;
    if (__builtin_isnan(x) || (__builtin_isinf(x) && x > 0)) return x;
    if (x < 0) return __builtin_nan("");
    if (x == 0) return -__builtin_inf();
    // Frexp (src/math/frexp.go): x = f1 * 2^ki, f1 in [0.5, 1)
    int ki = 0;
    if (__builtin_fabs(x) < 2.2250738585072014e-308) { x *= 4503599627370496.0; ki = -52; }
    uint64_t bits = (uint64_t)__double_as_longlong(x);
    ki += (int)((bits >> 52) & 0x7FF) - 1022;
    bits = (bits & ~(0x7FFULL << 52)) | (1022ULL << 52);
    double f1 = __longlong_as_double((long long)bits);
    if (f1 < 0.70710678118654752440084436210484904) { f1 *= 2; ki--; }
    const double f = f1 - 1;
    const double k = (double)ki;
    const double s = f / (2 + f);
    const double s2 = s * s;
    const double s4 = s2 * s2;
    const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
    const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
    const double R = t1 + t2;
    const double hfsq = 0.5 * f * f;
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

// hrw.UInt64ToFloat64 (rendezvous.go:99-118) of the murmur3 Sum h1 (its 8 big-endian
// bytes) with MaxHashValue = 8 x 0xFF: the low 53 bits; when they are all zero and a
// hasher is given (every production caller: rehash = true), murmur3 of the 8 Sum bytes
// once more; / 2^53, exact.
__device__ __forceinline__ double u64_to_f64(uint64_t h1, bool rehash) {
    const uint64_t m53 = (1ULL << 53) - 1;
    uint64_t val = h1 & m53;
    if (val == 0 && rehash) {  // rendezvous.go:111-116
        uint8_t be[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) be[i] = (uint8_t)(h1 >> (56 - 8 * i));
        val = murmur3_h1_cat(be, 8, be, 0) & m53;
    }
    return (double)val / 9007199254740992.0;
}

__device__ double hrw_score(const uint8_t* key, uint32_t klen, const uint8_t* label, uint32_t llen,
                            int64_t weight) {
#pragma clang fp contract(off)
    const double sc = u64_to_f64(murmur3_h1_cat(key, klen, label, llen), true);
    return -(double)weight / go_log(sc);
}

// UInt64ToFloat64 over n given Sum values (big-endian uint64 each): the same device
// function the scoring kernel runs, so the rehash branch -- reached by 2^-53 of the
// scored pairs -- is exercised with chosen inputs (rendezvous_test.go:59-98).
__global__ void u64_to_f64_kernel(const uint64_t* vals, uint64_t n, int rehash, double* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = u64_to_f64(vals[i], rehash != 0);
}

hipError_t launch_u64_to_f64(const uint64_t* vals, uint64_t n, int rehash, double* out, hipStream_t s) {
    if (!n) return hipSuccess;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL(u64_to_f64_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, vals, n, rehash, out);
    return hipGetLastError();
}

constexpr int kHrwBlock = 256;
constexpr uint32_t kHrwMaxNodes = 4096;

__global__ void __launch_bounds__(kHrwBlock) hrw_order_kernel(HrwArgs a, uint32_t kpb) {
    __shared__ double sc[kHrwMaxNodes];
    const uint32_t N = a.n_nodes;
    const uint64_t key0 = (uint64_t)blockIdx.x * kpb;
    const uint32_t pairs = kpb * N;
    for (uint32_t idx = threadIdx.x; idx < pairs; idx += kHrwBlock) {
        const uint32_t kl = idx / N, j = idx % N;
        const uint64_t key = key0 + kl;
        double v = 0;
        if (key < a.n_keys) {
            if (a.key_bad[key]) {
                v = __builtin_nan("");
            } else {
                const uint64_t ko = a.key_off[key], lo = a.label_off[j];
                v = hrw_score(a.keys + ko, (uint32_t)(a.key_off[key + 1] - ko), a.labels + lo,
                              (uint32_t)(a.label_off[j + 1] - lo), a.weights[j]);
            }
            if (a.scores) a.scores[key * N + j] = v;
        }
        sc[idx] = v;
    }
    __syncthreads();
    for (uint32_t idx = threadIdx.x; idx < pairs; idx += kHrwBlock) {
        const uint32_t kl = idx / N, j = idx % N;
        const uint64_t key = key0 + kl;
        if (key >= a.n_keys) continue;
        const double* row = sc + kl * N;
        const double s = row[j];
        const bool sn = __builtin_isnan(s);
        uint32_t rank = 0;
        for (uint32_t q = 0; q < N; ++q) {
            const double o = row[q];
            const bool eq = (o == s) || (sn && __builtin_isnan(o));
            rank += (o > s) || (eq && q < j);
        }
        if (rank < a.n_out) a.order[key * a.n_out + rank] = (int32_t)j;
        if (j == 0)
            for (uint32_t r = N; r < a.n_out; ++r) a.order[key * a.n_out + r] = -1;
    }
}

hipError_t launch_hrw_order(const HrwArgs& a, hipStream_t s) {
    if (a.n_keys == 0) return hipSuccess;
    if (a.n_nodes == 0 || a.n_nodes > kHrwMaxNodes) return hipErrorInvalidValue;
    const uint32_t kpb = a.n_nodes >= kHrwMaxNodes ? 1 : kHrwMaxNodes / a.n_nodes > 64 ? 64
                                                                                     : kHrwMaxNodes / a.n_nodes;
    const uint64_t grid = (a.n_keys + kpb - 1) / kpb;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL(hrw_order_kernel, dim3((uint32_t)grid), dim3(kHrwBlock), 0, s, a, kpb);
    return hipGetLastError();
}

// ring.Locations (ring.go:106-117) over full HRW orders.
__global__ void ring_filter_kernel(const int32_t* order, uint64_t n_rows, uint32_t N,
                                   const uint8_t* healthy, int32_t max_replica, uint32_t row_out,
                                   int32_t* locs, uint8_t* counts) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    const int32_t* o = order + r * N;
    int32_t* L = locs + r * row_out;
    bool any = false;
    for (uint32_t j = 0; j < N; ++j) any |= healthy[j] != 0;
    uint32_t k = 0;
    if (!any) {
        L[k++] = o[0];
    } else {
        for (uint32_t i = 0; i < N && (k == 0 || (int64_t)i < max_replica); ++i)
            if (healthy[o[i]] && k < row_out) L[k++] = o[i];
    }
    counts[r] = (uint8_t)k;
    for (uint32_t q = k; q < row_out; ++q) L[q] = -1;
}

hipError_t launch_ring_filter(const int32_t* order, uint64_t n_rows, uint32_t n_nodes,
                              const uint8_t* healthy, int32_t max_replica, uint32_t row_out,
                              int32_t* locs, uint8_t* counts, hipStream_t s) {
    if (!n_rows) return hipSuccess;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL(ring_filter_kernel, dim3((uint32_t)((n_rows + 255) / 256)), dim3(256), 0, s,
                       order, n_rows, n_nodes, healthy, max_replica, row_out, locs, counts);
    return hipGetLastError();
}

// Locations(d) depends on d only through ShardID = hex[:4] (core/digest.go:148-150),
// i.e. the first two digest bytes: gather the precomputed row.
// One thread per digest: its ShardID row of the owner table.  T = int32_t (-1 pad) or
// uint8_t (compact owner lists for rings of <= 255 nodes: 0xFF pad, a quarter of the
// bytes to write and to copy back to the host).
template <typename T>
__global__ void shard_gather_kernel(const uint8_t* digests32, uint64_t n, const int32_t* tl,
                                    const uint8_t* tc, uint32_t row_out, T* locs, uint8_t* counts) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t shard = (uint32_t)digests32[32 * i] << 8 | digests32[32 * i + 1];
    for (uint32_t q = 0; q < row_out; ++q) {
        const int32_t v = tl[(uint64_t)shard * row_out + q];
        locs[i * row_out + q] = sizeof(T) == 1 ? (T)(v < 0 ? 0xFF : v) : (T)v;
    }
    counts[i] = tc[shard];
}

template <typename T>
static hipError_t launch_gather(const uint8_t* digests32, uint64_t n, const int32_t* table_locs,
                                const uint8_t* table_counts, uint32_t row_out, T* locs, uint8_t* counts,
                                hipStream_t s) {
    if (!n) return hipSuccess;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL(shard_gather_kernel<T>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                       digests32, n, table_locs, table_counts, row_out, locs, counts);
    return hipGetLastError();
}

hipError_t launch_shard_gather(const uint8_t* digests32, uint64_t n, const int32_t* table_locs,
                               const uint8_t* table_counts, uint32_t row_out, int32_t* locs,
                               uint8_t* counts, hipStream_t s) {
    return launch_gather(digests32, n, table_locs, table_counts, row_out, locs, counts, s);
}

hipError_t launch_shard_gather_u8(const uint8_t* digests32, uint64_t n, const int32_t* table_locs,
                                  const uint8_t* table_counts, uint32_t row_out, uint8_t* locs,
                                  uint8_t* counts, hipStream_t s) {
    return launch_gather(digests32, n, table_locs, table_counts, row_out, locs, counts, s);
}

// One word a ShardID: owners in bytes 0..row_out-1 (0xFF for none), 0xFF up to byte 2,
// the count in byte 3.
__global__ void pack_owner_rows_kernel(const int32_t* tl, const uint8_t* tc, uint32_t row_out, uint32_t* packed) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 65536u) return;
    uint32_t w = 0x00FFFFFFu;
    for (uint32_t q = 0; q < row_out; ++q) {
        const int32_t v = tl[(uint64_t)i * row_out + q];
        w = (w & ~(0xFFu << (8 * q))) | ((uint32_t)(v < 0 ? 0xFF : v) << (8 * q));
    }
    packed[i] = (w & 0x00FFFFFFu) | ((uint32_t)tc[i] << 24);
}

hipError_t launch_pack_owner_rows(const int32_t* table_locs, const uint8_t* table_counts, uint32_t row_out,
                                  uint32_t* packed, hipStream_t s) {
    if (row_out < 1 || row_out > 3) return hipErrorInvalidValue;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL(pack_owner_rows_kernel, dim3(65536 / 256), dim3(256), 0, s, table_locs, table_counts, row_out,
                       packed);
    return hipGetLastError();
}

// 256 digests a wave.  Loads are wave-contiguous (load k of lane l: digest 64k + l, so one
// instruction reads 64 consecutive 32-byte records), the ShardID is bytes 0, 1 of the
// record (one 16-bit load, big-endian), its packed row comes from the L2-resident 256 KiB
// table, and the rows go through LDS so that each lane then holds four CONSECUTIVE digests'
// rows: 4 x R owner bytes = R word stores and the four counts = one word store, adjacent
// lanes writing adjacent words.  A ragged tail writes byte by byte.
template <int R>
__global__ void __launch_bounds__(256) shard_gather_packed_kernel(const uint8_t* digests32, uint64_t n,
                                                                  const uint32_t* packed, uint8_t* locs,
                                                                  uint8_t* counts) {
    __shared__ uint32_t rows[4 * 256];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t wbase = ((uint64_t)blockIdx.x * 4 + wv) * 256;
    uint32_t* x = rows + wv * 256;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t d = wbase + 64 * k + lane;
        uint32_t shard = 0;
        if (d < n) {
            const uint32_t v = *reinterpret_cast<const uint16_t*>(digests32 + 32 * d);
            shard = ((v & 0xFFu) << 8) | (v >> 8);
        }
        x[64 * k + lane] = packed[shard];
    }
    __syncthreads();  // every thread reaches it: no early exit above
    const uint64_t base = wbase + 4 * lane;
    if (base >= n) return;
    const uint32_t m = (uint32_t)(n - base < 4 ? n - base : 4);
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = x[4 * lane + k];
    if (m == 4) {
        uint32_t* lo = reinterpret_cast<uint32_t*>(locs + base * R);
        if constexpr (R == 3) {
            lo[0] = (w[0] & 0xFFFFFFu) | (w[1] << 24);
            lo[1] = ((w[1] >> 8) & 0xFFFFu) | ((w[2] & 0xFFFFu) << 16);
            lo[2] = ((w[2] >> 16) & 0xFFu) | ((w[3] & 0xFFFFFFu) << 8);
        } else if constexpr (R == 2) {
            lo[0] = (w[0] & 0xFFFFu) | ((w[1] & 0xFFFFu) << 16);
            lo[1] = (w[2] & 0xFFFFu) | ((w[3] & 0xFFFFu) << 16);
        } else {
            lo[0] = (w[0] & 0xFFu) | ((w[1] & 0xFFu) << 8) | ((w[2] & 0xFFu) << 16) | ((w[3] & 0xFFu) << 24);
        }
        *reinterpret_cast<uint32_t*>(counts + base) =
            (w[0] >> 24) | ((w[1] >> 24) << 8) | ((w[2] >> 24) << 16) | ((w[3] >> 24) << 24);
        return;
    }
    for (uint32_t k = 0; k < m; ++k) {
        for (int q = 0; q < R; ++q) locs[(base + k) * R + q] = (uint8_t)(w[k] >> (8 * q));
        counts[base + k] = (uint8_t)(w[k] >> 24);
    }
}

hipError_t launch_shard_gather_packed(const uint8_t* digests32, uint64_t n, const uint32_t* packed,
                                      uint32_t row_out, uint8_t* locs, uint8_t* counts, hipStream_t s) {
    if (!n) return hipSuccess;
    if (row_out < 1 || row_out > 3 || ((uintptr_t)digests32 & 1) || ((uintptr_t)locs & 3) || ((uintptr_t)counts & 3))
        return hipErrorInvalidValue;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    const dim3 grid((uint32_t)((n + 1023) / 1024)), block(256);  // 1,024 digests a workgroup
    if (row_out == 3)
        hipLaunchKernelGGL(shard_gather_packed_kernel<3>, grid, block, 0, s, digests32, n, packed, locs, counts);
    else if (row_out == 2)
        hipLaunchKernelGGL(shard_gather_packed_kernel<2>, grid, block, 0, s, digests32, n, packed, locs, counts);
    else
        hipLaunchKernelGGL(shard_gather_packed_kernel<1>, grid, block, 0, s, digests32, n, packed, locs, counts);
    return hipGetLastError();
}

}  // namespace krk
