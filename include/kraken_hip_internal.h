/*
 * kraken_hip_internal.h -- benchmark, test and diagnostic entry points of
 * libkraken_hip.so.
 *
 * NOT part of the drop-in boundary: a cgo binder of the reference includes only
 * kraken_hip.h (INTEGRATION.md lists everything it binds).  These symbols stay
 * exported from the same library so that bench.py, tools/ and tests/ can reach
 * the kernels' timing, the planners' models and the window schedule; the same
 * conventions apply (KRK_OK or a negative KRK_E* code, krk_last_error()).
 */
#ifndef KRAKEN_HIP_INTERNAL_H
#define KRAKEN_HIP_INTERNAL_H

#include "kraken_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------ CPU budget
 * The per-process host CPU budget every host thread pool of the library is sized by
 * (offload, copy threads, CPU tokens, the AUTO Digester crossover), the node's CPUs it
 * was derived from (affinity capped by the cgroup v2 cpu.max quota) and where the number
 * came from: "KRK_HOST_CPUS" (explicit), "node/LOCAL_WORLD_SIZE" (one process per GPU
 * under a launcher: the ranks of a node share it; a launcher's OMP_NUM_THREADS=1 does not
 * shrink it), "OMP_NUM_THREADS" (a single process capped by it) or "node".  Read once. */
int krk_host_cpu_budget(int* cpus, int* node_cpus, char* source, uint32_t cap);

/* --------------------------------------------------------- CRC host split
 * The calling thread's last krk_piece_sums_host / krk_verify_pieces_host split in bytes
 * and the GPU share the next pinned batch of its device will use (0 while host-only wins,
 * -1 until learned; KRK_CRC_GPU_FRACTION forces it). */
int krk_crc_host_split(uint64_t* gpu_bytes, uint64_t* host_bytes, double* gpu_fraction);

/* Submission-engine counters of the calling thread's device: SHA launches and the
 * jobs they carried (jobs / batches = streams coalesced per launch), CRC launches and
 * requests, pinned staging bytes held by the slot pool. */
int krk_engine_stats(uint64_t* sha_batches, uint64_t* sha_jobs, uint64_t* crc_batches,
                     uint64_t* crc_requests, uint64_t* pinned_bytes);

/* ------------------------------------------------------- window schedule
 * The window schedule of the host-resident batch calls (and of kraken_amd/windowed.py's
 * larger-than-HBM device batches): every live blob advances by the same chunk (a multiple of
 * 64 bytes but each blob's last, about window_bytes / live a window); at most live_cap blobs
 * are live, admitted longest first; a finished blob's place goes to the next-longest.  _next
 * writes the next window's chunks (blob index, offset, length; admission order) and their
 * count to *n_out, 0 once every blob is done (KRK_ERANGE if cap is too small: the window
 * has *n_out <= live_cap chunks). */
typedef struct krk_window_sched krk_window_sched;
int krk_window_sched_new(const uint64_t* lengths, uint64_t n, uint64_t window_bytes, uint64_t live_cap,
                         krk_window_sched** out);
int krk_window_sched_next(krk_window_sched* s, uint32_t* blobs, uint64_t* offsets, uint64_t* lengths, uint64_t cap,
                          uint64_t* n_out);
/* Take blob `blob` out of the schedule (a host thread continues its chain: the windowed tail
 * handoff); *offset = the bytes the windows gave it (0 if it was still waiting).  A live
 * blob's place goes to the next waiting blob at the next window.  KRK_EINVAL if it is
 * neither live nor waiting. */
int krk_window_sched_drop(krk_window_sched* s, uint32_t blob, uint64_t* offset);
/* At most max_chunk bytes (>= 64) a chunk from the next window on: windows stay short once
 * few blobs are live. */
int krk_window_sched_set_chunk_cap(krk_window_sched* s, uint64_t max_chunk);
void krk_window_sched_free(krk_window_sched* s);
/* krk_metainfo_digest_chunks_dev_on with the piece CRCs queued on `stream` only after the
 * SHA-256 launch on sha_stream has ended (no CRC waiting for CUs at the head of a
 * high-priority queue while the SHA launch holds them: that keeps the dispatcher from every
 * normal-priority queue, device-to-host copies included).  The C3 tail handoff's window step. */
int krk_metainfo_digest_chunks_dev_after(const krk_chunk* chunks, uint64_t n, uint32_t* state_dev, uint32_t* sums_dev,
                                         uint8_t* digests_dev, void* stream, void* sha_stream);
/* The piece CRCs of device chunks without SHA-256 (XOR-accumulated into sums_dev like a
 * window's; several chunks of one blob allowed): the tails of chains a host thread hashes.
 * Asynchronous on `stream`. */
int krk_chunks_crc_dev(const krk_chunk* chunks, uint64_t n, uint32_t* sums_dev, void* stream);
/* The calling thread's cumulative seconds in krk_sha256_resume_dev_on_host waiting for its
 * device-to-host copies and hashing (krk_sha256_resume_host's hashing counts too). */
int krk_sha256_resume_stats(double* copy_wait_s, double* hash_s);
/* ... and in enqueueing its copies and waiting for the caller's stream. */
int krk_sha256_resume_stats2(double* issue_s, double* ready_s);
/* Page-locked host memory from the HIP runtime's own allocator (hipHostMalloc), which places
 * it on the NUMA node nearest the calling thread's device: targets of device-to-host copies
 * (krk_host_alloc's pages land on the allocating thread's node; 53 vs 56 GB/s measured,
 * tools/pinned_d2h_probe.py).  Freed by krk_host_free. */
int krk_host_alloc_dma(uint64_t bytes, void** out);
/* *done = 1 once event `ev` has completed, else 0 (no wait). */
int krk_event_query(void* ev, int* done);
/* An event whose krk_event_sync polls instead of sleeping: for waits of microseconds (a
 * generator launch), where a sleeping wait's wake-up costs milliseconds. */
int krk_event_create_polling(void** out);
/* Work queued on `stream` after the call waits for event `ev` (hipStreamWaitEvent). */
int krk_stream_wait_event(void* stream, void* ev);
/* Continue one SHA-256 chain on the calling thread from n device bytes at data_dev (after
 * the work queued on `stream`; NULL: the bytes are ready now, nothing is waited for): state8
 * holds the midstate after `absorbed` bytes (a multiple of 64) and is updated by a non-final
 * run (n whole blocks); final != 0 pads and writes the digest to digest32 instead (n any
 * length).  Read through pinned buffers (copies three ahead), x86 SHA extensions.
 * Synchronous. */
int krk_sha256_resume_dev_on_host(uint32_t* state8, uint64_t absorbed, const uint8_t* data_dev, uint64_t n,
                                  int final, uint8_t* digest32, void* stream);
/* The same continuation over n bytes already in host memory (a device-to-host copy the
 * caller queued and waited for): no device call. */
int krk_sha256_resume_host(uint32_t* state8, uint64_t absorbed, const uint8_t* data_host, uint64_t n, int final,
                           uint8_t* digest32);
/* The live-stream cap of the windows on the calling thread's device: 7/8 of the largest
 * stream count whose SHA-256 launch runs more than one lane a stream (14,336 on 256 CUs),
 * so each window's CRC launch has the CUs the SHA workgroups leave free.  KRK_LIVE_CAP
 * overrides it for the host-resident calls. */
int krk_window_stream_cap(uint64_t* cap);
/* The calling thread's last krk_metainfo_digest_host / _files call: the most live blobs in
 * one window, the windows, and the blobs the host offload took. */
int krk_windows_last_call(uint64_t* max_live, int* windows, uint64_t* host_blobs);
/* ... and how many of its windows went to the device straight from the caller's
 * page-locked blobs (krk_host_alloc memory, windows of <= 64 chunks: no pinned staging
 * copy, one DMA a chunk).  KRK_PINNED_DIRECT=0 stages them instead. */
int krk_windows_last_direct(int* direct_windows);
/* ... and how many of its windows the GPU gathered from the caller's page-locked memory
 * (gather.hip: one launch a window reading the pages over PCIe -- krk_host_alloc blobs in
 * wide windows, or pageable blobs the call registered with hipHostRegister; KRK_HOST_GATHER
 * 0 / 1 forces off / on), the caller bytes it registered and the helper threads' seconds
 * spent registering them. */
int krk_windows_last_gather(int* gather_windows, uint64_t* registered_bytes, double* register_seconds);
/* ... and how many of the caller ranges it registered for the gather were still registered
 * when its results were copied out (0: every host-buffer call releases them first; a copy
 * into a page the call holds registered is refused). */
int krk_windows_last_copyout(uint64_t* live_registered);
/* The calling thread's last device-resident SHA-256 batch (krk_sha256_dev,
 * krk_metainfo_digest_dev): chains whose tails host threads finished from the GPU's midstate
 * (the tail handoff of the host offload; 0 when whole blobs or nothing went to the host) and
 * the GPU's prefix bytes of those chains.  KRK_SHA_TAIL=0 turns tail handoff off. */
int krk_sha_last_tail(uint64_t* chains, uint64_t* gpu_prefix_bytes);
/* Tail handoff plan of the host offload for a device-resident batch (the rates
 * krk_planner_rates_get reports on this thread's device; nominal without one): chain
 * host_idx[k] runs its first start[k] bytes on the GPU, the rest on a host thread; *n_out
 * chains (host_idx / start sized n); *end_s the planned batch end, *gpu_s the GPU alone. */
int krk_sha_tail_plan(const uint64_t* lengths, uint64_t n, int threads, uint32_t* host_idx, uint64_t* start,
                      uint64_t* n_out, double* end_s, double* gpu_s);
/* ... and its window loop's wall seconds, split into waiting for a free staging window,
 * filling windows (staging copies or file reads) and enqueueing copies and kernels; for a
 * krk_metainfo_digest_files call, the page-cache resident share of its sampled files (below
 * 0.5 the batch is disk-bound: no host offload under AUTO, O_DIRECT reads unless
 * KRK_FILE_DIRECT says otherwise), else -1; and whether it read with O_DIRECT. */
int krk_windows_last_phases(double* loop_s, double* acquire_s, double* fill_s, double* enqueue_s,
                            double* resident, int* direct_reads);
/* The gather of host-buffer calls, process-wide: -1 AUTO (the default: page-locked blobs
 * gathered in wide windows, pageable ones staged -- measured faster), 0 off
 * (stage every window through the pinned host windows), 1 on (pageable blobs registered for
 * the call with hipHostRegister and gathered too).  KRK_HOST_GATHER sets the same at the
 * first call.  For A/B runs (bench.py). */
int krk_set_host_gather(int mode);

/* --------------------------------------- host crossover primitives (CPU)
 * The host side of the Digester / PieceHash crossovers, exported so the
 * tests can pin the library's own SHA-NI / PCLMUL code against zlib / hashlib:
 * sha256.Sum256 and crc32.Update(crc, IEEETable, p). */
int krk_host_sha256(const uint8_t* data, uint64_t n, uint8_t out32[32]);
int krk_host_crc32_update(uint32_t crc, const uint8_t* data, uint64_t n, uint32_t* out);

/* ----------------------------------------------------- synthetic blobs
 * Fills a device buffer with bytes [offset, offset+n) of synthetic blob
 * blob_idx (splitmix64 counter stream, variant 0 = uniform bytes, 1 = alnum;
 * spec in DESIGN.md).  Benchmark/test data generator. */
int krk_synth_fill_dev(uint8_t* dst_dev, uint64_t blob_idx, uint64_t offset, uint64_t n,
                       int variant, void* stream);
/* Batched form for window generation: chunk i fills chunks[i].data (device)
 * with bytes [offset, offset+length) of synthetic blob chunks[i].blob (the
 * other krk_chunk fields are ignored).  One launch. */
int krk_synth_fill_chunks_dev(const krk_chunk* chunks, uint64_t n, int variant, void* stream);

/* -------------------------------------------------------- device identity
 * PCI bus id of the calling thread's device ("0000:05:00.0"; cap >= 16): an N-rank run
 * reports every rank's, so a scaling line shows it ran on N distinct GPUs. */
int krk_device_pci_bus_id(char* out, uint32_t cap);
/* CUs of the calling thread's device. */
int krk_device_cus(int* out);

/* ---------------------------------------------------------- kernel timing
 * When enabled, every kernel launch is bracketed by hipEvents recorded on the stream
 * the kernel runs on; krk_kernel_stats returns the number of launches and their summed
 * device time (ms) since the last reset for kernel name "crc32_pieces", "sha256_multi",
 * "hrw_shard_table", "hrw_gather" or "synth_fill" (timed launches are synchronised
 * lazily). */
int krk_set_timing(int on);
/* Shader clock of the calling thread's device, measured by a one-wave probe kernel on
 * `stream` (NULL = the library's stream): s_memtime cycles over s_memrealtime (100 MHz)
 * ticks of a ~2 ms spin.  Launched while another kernel runs it reads the clock the chip
 * holds under that load (bench.py prices the SHA-256 issue ceiling with it). */
int krk_device_clock_mhz(void* stream, double* mhz);
int krk_kernel_stats(const char* kernel, uint64_t* launches, double* total_ms);
/* Every timed launch of `kernel` since the last reset, in the order the host issued
 * them: device, SHA-256 plan (KRK_SHA_PLAN_*; 0 for other kernels), work units
 * (streams for sha256_multi, work items + runs for crc32_pieces, else 0) and the
 * launch's start / end in ms after the device's first timed launch (hipEvents on the
 * launch's own stream, so launches on different streams of one device share the
 * clock).  Up to `cap` records to out (may be NULL), the total count to *n; the
 * library keeps the first 2^20 launches. */
typedef struct krk_launch_rec {
    int32_t device;
    int32_t plan;
    uint64_t units;
    double start_ms;
    double end_ms;
} krk_launch_rec;
int krk_kernel_timeline(const char* kernel, krk_launch_rec* out, uint64_t cap, uint64_t* n);
int krk_reset_kernel_stats(void);

/* ------------------------------------------------------- SHA-256 plans
 * Lanes per stream (1, 2 or 8) the library uses for a batch of n_streams streams on
 * the current device (more lanes a stream -- a shorter chain a block -- while the
 * batch leaves SIMDs idle); bench.py prices the per-stream issue ceiling of that plan. */
int krk_sha_lanes_per_stream(uint64_t n_streams, int* lanes);
/* The launch plan itself (KRK_SHA_PLAN_1LANE .. KRK_SHA_PLAN_8LANE_2PAIR below) for a
 * batch of n_streams streams on the current device under the current plan setting. */
int krk_sha_plan_for(uint64_t n_streams, int* plan);
/* SHA-256 launch plan, process-wide (default AUTO: eight lanes per stream while the
 * batch leaves SIMDs idle, then two lanes, then two producer/consumer pairs per
 * workgroup, then one lane).  Every plan is bit-exact; the knob exists for tests and
 * tuning.  The environment variable KRK_SHA_PLAN, read once at the first launch, sets
 * the same. */
#define KRK_SHA_PLAN_AUTO 0
#define KRK_SHA_PLAN_1LANE 1        /* one lane per stream, one pair per workgroup */
#define KRK_SHA_PLAN_2LANE 2        /* two lanes per stream, one pair per workgroup */
#define KRK_SHA_PLAN_1LANE_2PAIR 3  /* one lane, two pairs per 4-wave workgroup */
#define KRK_SHA_PLAN_2LANE_2PAIR 4  /* two lanes, two pairs per workgroup */
#define KRK_SHA_PLAN_8LANE 5        /* eight lanes per stream, one pair per workgroup */
#define KRK_SHA_PLAN_8LANE_2PAIR 6  /* eight lanes, two pairs per workgroup */
int krk_set_sha_plan(int plan);

/* ------------------------------------------------------------- planners
 * Override the planner rates process-wide (NULL restores the measured ones): tests
 * inject rates to move the crossovers. */
int krk_planner_rates_set(const krk_planner_rates* in);
/* The offload plan for `n` blob lengths on `threads` host threads with the planner rates
 * (krk_planner_rates_get; `cus` > 0 overrides their CU count), no device work: the
 * indices (longest first) to host_idx (room for n, may be NULL), their count to n_host,
 * and the modelled GPU / host seconds (may be NULL).
 * krk_sha_offload_plan plans a device-resident batch (krk_sha256_dev,
 * krk_metainfo_digest_dev); krk_host_offload_plan plans for `mode`
 * KRK_OFFLOAD_DEVICE (the same), KRK_OFFLOAD_HOST_SHA (krk_sha256_host),
 * KRK_OFFLOAD_HOST_WHOLE (krk_metainfo_digest_host) or KRK_OFFLOAD_HOST_FILES
 * (krk_metainfo_digest_files). */
#define KRK_OFFLOAD_DEVICE 0
#define KRK_OFFLOAD_HOST_SHA 1
#define KRK_OFFLOAD_HOST_WHOLE 2
#define KRK_OFFLOAD_HOST_FILES 3  /* krk_metainfo_digest_files: one read, SHA-256 + CRC per host blob */
int krk_sha_offload_plan(const uint64_t* lengths, uint64_t n, int threads, int cus, uint32_t* host_idx,
                         uint64_t* n_host, double* gpu_seconds, double* host_seconds);
int krk_host_offload_plan(const uint64_t* lengths, uint64_t n, int threads, int cus, int mode, uint32_t* host_idx,
                          uint64_t* n_host, double* gpu_seconds, double* host_seconds);
/* The AUTO Digester crossover: how many live digesters still run SHA-NI on their
 * callers' threads (krk_digester_new), derived from the planner rates and the CPU budget
 * unless KRK_DIGESTER_HOST_STREAMS / krk_set_digester_host_streams pins it. */
int krk_digester_host_streams(int64_t* n);

#ifdef __cplusplus
}
#endif
#endif /* KRAKEN_HIP_INTERNAL_H */
