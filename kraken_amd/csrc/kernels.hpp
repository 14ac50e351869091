// kernels.hpp -- device work descriptors and kernel launchers (implemented in *.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

namespace krk {

// What the last launcher on this thread launched, for the kernel timeline
// (krk_kernel_timeline): SHA-256 plan id (KRK_SHA_PLAN_*) and work units (streams for
// SHA-256, work items + runs for CRC).  Written by the launchers, read by timed().
inline thread_local int t_launch_plan = 0;
inline thread_local uint64_t t_launch_units = 0;

// Before a launch: an error already pending on this thread belongs to an earlier HIP call
// that nobody checked (the caller's own, or one outside the library).  It is reported, not
// cleared away: the launcher returns it without launching, and launch_error_text() says
// where it came from, so the entry point's message names it.  hipErrorNotReady is an event
// query's answer, not an error.
inline thread_local bool t_launch_pending = false;
inline hipError_t launch_precheck() {
    t_launch_pending = false;
    const hipError_t p = hipPeekAtLastError();
    if (p == hipSuccess) return hipSuccess;
    (void)hipGetLastError();
    if (p == hipErrorNotReady) return hipSuccess;
    t_launch_pending = true;
    return p;
}
inline const char* launch_error_text(hipError_t e) {
    static thread_local char buf[256];
    if (!t_launch_pending) return hipGetErrorString(e);
    snprintf(buf, sizeof buf, "HIP error pending from an earlier call on this thread: %s", hipGetErrorString(e));
    return buf;
}

// ---------------------------------------------------------------- CRC pieces
// One work item = a contiguous byte run inside ONE piece, processed by one wave.
// Its raw CRC is shifted to the piece end (mul = x^(8*(piece_end - item_end))) and
// XOR-ed into sums[out]; the piece's first item also carries the init/xorout term
// xr = shift(~0, piece_len) ^ ~0.  XOR is order-free, so items of one piece may run
// on any wave, XCD or launch.
struct alignas(16) CrcItem {
    uint64_t ptr;   // device address of the run
    uint32_t len;   // bytes, 1 .. kItemBytes
    uint32_t out;   // index into sums[]
    uint32_t mul;
    uint32_t xr;
    uint32_t pad[2];
};
static_assert(sizeof(CrcItem) == 32, "CrcItem layout");

constexpr uint32_t kSeg = 64;                // bytes per lane per wave step
constexpr uint32_t kStep = 64 * kSeg;        // bytes per wave step (4 KiB)
constexpr uint32_t kGap = kStep - kSeg;      // zero-gap between a lane's segments
constexpr uint32_t kItemBytes = 256 * 1024;  // max bytes per work item

// Global constant table layout (uint32 words).
constexpr int kTabT = 0;        // T0..T3 slicing tables, 1024 words
constexpr int kTabG = 1024;     // G0..G3 shift-by-kGap tables, 1024 words
constexpr int kTabLaneMul = 2048;  // 64 words: x^(8*(63-l)*kSeg)
constexpr int kTabX8Pow = 2112;    // 64 words: x^(8*2^k)
// Coalesced layout (variants 2, 3): wave step = 4 KiB loaded as four fully coalesced
// 1 KiB wave-instructions; lane l owns chain k = bytes [1024k + 16l, +16) of every
// step, so a chain's segments are kGapC = 4080 zero bytes apart.
constexpr uint32_t kGapC = kStep - 16;
constexpr int kTabGC = 2176;       // G0..G3 shift-by-kGapC tables, 1024 words
constexpr int kTabLaneMulC = 3200; // 256 words [k*64 + l]: x^(8*(kGapC - 1024k - 16l))
constexpr int kTabWords = 3456;

// A run of consecutive WHOLE pieces of one blob, expanded into work items on the
// device: a whole piece's items and their constants depend only on the piece
// length, so the host writes one run per blob range instead of one item per
// 256 KiB (C4: 81,920 items -> 1 run).  consts[cpat + j] is item j's piece-end
// shift, consts[cpat + ipp] the piece's init/xor-out term.
struct alignas(16) CrcRun {
    uint64_t ptr;        // device address of the run's first piece
    uint64_t plen;       // piece length
    uint32_t n_pieces;
    uint32_t out;        // sums index of the first piece
    uint32_t item_base;  // index of the run's first item in the launch
    uint32_t ipp;        // items per piece = ceil(plen / kItemBytes)
    uint32_t cpat;
    uint32_t pad[3];
};
static_assert(sizeof(CrcRun) == 48, "CrcRun layout");

// One CRC launch: items [0, run_items) come from the runs, [run_items,
// run_items + n_items) from the explicit item array.
struct CrcWork {
    const CrcRun* runs;
    const CrcItem* items;
    const uint32_t* consts;
    uint32_t n_runs;
    uint32_t run_items;
    uint32_t n_items;
    uint32_t pad;
    uint32_t* next;  // work-queue head (zeroed per launch): waves claim items by atomicAdd
};

struct CrcLaunchCfg {
    int cus;           // compute units
    int variant;       // crc32_pieces.hip launch_crc_items; default 7 (byte-addressable tables)
};

bool crc_variant_valid(int variant);
hipError_t launch_crc_items(const CrcWork& w, const uint32_t* tabs, uint32_t* sums, const CrcLaunchCfg& cfg,
                            hipStream_t s);

// Piece verification: ok[i] = (sums[i] == expected[i]).
hipError_t launch_crc_verify(const uint32_t* sums, const uint32_t* expected, uint8_t* ok,
                             uint32_t n, hipStream_t s);

// ---------------------------------------------------------------- SHA-256
// One job = one Merkle-Damgard stream, run by one lane.  Processes len bytes
// starting from midstate h (or from out_state + 8*out when kShaFromState); if
// kShaFinal, pads with total = prefix + len bytes and writes the big-endian digest
// to out_digest + 32*out, else writes the midstate (len must then be a multiple of
// 64) to out_state + 8*out.
constexpr uint32_t kShaFinal = 1;
constexpr uint32_t kShaFromState = 2;
struct alignas(16) ShaJob {
    uint64_t ptr;
    uint64_t len;
    uint64_t prefix;   // bytes absorbed before this job (for the length field)
    uint32_t out;
    uint32_t flags;
    uint32_t h[8];
};
static_assert(sizeof(ShaJob) == 64, "ShaJob layout");

// Digests computed elsewhere (host offload) into digests[32 * idx]: n records of a
// little-endian uint32 idx + 32 digest bytes.
hipError_t launch_digest_scatter(const uint8_t* rec, uint32_t n, uint8_t* digests, hipStream_t s);
hipError_t launch_sha256(const ShaJob* jobs, uint32_t n_jobs, uint8_t* out_digest,
                         uint32_t* out_state, hipStream_t s);
// Lanes per stream launch_sha256 uses for a batch of n_jobs streams (1 or 2).
int sha_lanes_for(uint32_t n_jobs);
int sha_plan_for(uint32_t n_jobs);  // KRK_SHA_PLAN_* the next launch of n_jobs streams uses
// One launch on a given plan whatever the process-wide setting (planner calibration).
hipError_t launch_sha256_plan(int plan, const ShaJob* jobs, uint32_t n_jobs, uint8_t* out_digest,
                              uint32_t* out_state, hipStream_t s);
// Process-wide launch plan (KRK_SHA_PLAN_* of kraken_hip.h; diagnostic plans >= 100
// only in the KRK_DIAG build).
bool sha_plan_valid(int plan);
void set_sha_plan(int plan);

// ---------------------------------------------------------------- host gather
// One tile of a host -> device gather (gather.hip): n <= kGatherTile bytes from src (a
// device-visible address of page-locked host memory: a hipHostMalloc'd or registered
// mapping; any alignment) to dst (device, 16-B aligned, room for n rounded up to 16).
constexpr uint64_t kGatherTile = 64 << 10;
struct alignas(32) GatherTile {
    uint64_t src;
    uint64_t dst;
    uint64_t n;
    uint64_t pad;
};
static_assert(sizeof(GatherTile) == 32, "GatherTile layout");
hipError_t launch_gather(const GatherTile* tiles, uint32_t n_tiles, int cus, hipStream_t s);

// ---------------------------------------------------------------- HRW
// Scores for (key, node) pairs and the per-key descending order.
struct HrwArgs {
    const uint8_t* keys;      // decoded key bytes
    const uint64_t* key_off;  // n_keys + 1
    uint64_t n_keys;
    const uint8_t* labels;
    const uint64_t* label_off;  // n_nodes + 1
    const int64_t* weights;
    uint32_t n_nodes;
    uint32_t n_out;
    const uint8_t* key_bad;   // n_keys flags: invalid hex -> NaN scores
    int32_t* order;           // n_keys * n_out
    double* scores;           // nullable: n_keys * n_nodes
};
hipError_t launch_hrw_order(const HrwArgs& a, hipStream_t s);
// hrw.UInt64ToFloat64 of n Sum values (as uint64) on the device.
hipError_t launch_u64_to_f64(const uint64_t* vals, uint64_t n, int rehash, double* out, hipStream_t s);

// Locations filter over full orders (n_out == n_nodes rows).
hipError_t launch_ring_filter(const int32_t* order, uint64_t n_rows, uint32_t n_nodes,
                              const uint8_t* healthy, int32_t max_replica, uint32_t row_out,
                              int32_t* locs, uint8_t* counts, hipStream_t s);
// Per-digest gather from the 65,536-row shard table.
hipError_t launch_shard_gather(const uint8_t* digests32, uint64_t n, const int32_t* table_locs,
                               const uint8_t* table_counts, uint32_t row_out, int32_t* locs,
                               uint8_t* counts, hipStream_t s);
hipError_t launch_shard_gather_u8(const uint8_t* digests32, uint64_t n, const int32_t* table_locs,
                                  const uint8_t* table_counts, uint32_t row_out, uint8_t* locs,
                                  uint8_t* counts, hipStream_t s);
// The owner table of a ring of <= 255 nodes with rows of <= 3 owners packed one word a
// ShardID (owner bytes 0-2, 0xFF padded; the count in byte 3), and the gather over it:
// wave-contiguous digest loads, one word load a row, rows regrouped through LDS so owner
// lists and counts go out as whole words.
// Needs digests32 2-byte aligned and locs / counts 4-byte aligned (the caller checks).
hipError_t launch_pack_owner_rows(const int32_t* table_locs, const uint8_t* table_counts, uint32_t row_out,
                                  uint32_t* packed, hipStream_t s);
hipError_t launch_shard_gather_packed(const uint8_t* digests32, uint64_t n, const uint32_t* packed,
                                      uint32_t row_out, uint8_t* locs, uint8_t* counts, hipStream_t s);

// ---------------------------------------------------------------- synthetic data
// One synthetic chunk: bytes [offset, offset + n) of the blob whose stream seed is `seed`.
struct SynthChunk {
    uint8_t* dst;
    uint64_t seed;
    uint64_t offset;
    uint64_t n;
};
hipError_t launch_synth_fill_chunks(const SynthChunk* chunks, uint32_t n_chunks, int variant, hipStream_t s);
// Shader clock probe: out[0] = shader cycles, out[1] = 100 MHz ticks of one spin.
hipError_t launch_clock_probe(uint32_t spins, uint64_t* out, hipStream_t s);
hipError_t launch_synth_fill(uint8_t* dst, uint64_t seed, uint64_t offset, uint64_t n,
                             int variant, hipStream_t s);

}  // namespace krk
