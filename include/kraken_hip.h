/*
 * kraken_hip.h -- C ABI of the MI355X-native blob-metainfo hot path.
 *
 * The drop-in boundary.  Plain pointers and sizes only (no torch types); all
 * entry points are re-entrant and return KRK_OK (0) or a negative KRK_E*
 * code, with a thread-local message from krk_last_error().  The Go wrappers
 *  bind these through cgo and re-create the reference's exact
 * error strings.  Each entry point names the reference interface it replaces.
 *
 * Device work runs on the calling thread's current device (krk_set_device);
 * "stream" arguments are hipStream_t passed as void* (NULL = the library's
 * own per-device stream).  *_dev entry points take device pointers and do no
 * host<->device copies of bulk data; the host entry points stage through
 * library-owned hipHostMalloc buffers with double-buffered hipMemcpyAsync.
 */
#ifndef KRAKEN_HIP_H
#define KRAKEN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KRK_OK 0
#define KRK_EINVAL (-1)    /* bad argument; e.g. "piece length must be positive" */
#define KRK_EHIP (-2)      /* HIP runtime error (message has the hip error string) */
#define KRK_ENOMEM (-3)    /* host or device allocation failed */
#define KRK_ENODEV (-4)    /* no MI355X (gfx950) device visible */
#define KRK_ERANGE (-5)    /* output capacity too small */
#define KRK_EHEX (-6)      /* invalid hex key (hrw.Score returns NaN, rendezvous.go:154-157) */
#define KRK_EIO (-7)       /* file open/read failed (message has the path and errno text) */

/* ---------------------------------------------------------------- runtime */
const char* krk_version(void);
const char* krk_last_error(void);            /* thread-local, never NULL */
int krk_device_count(int* n);                /* gfx950 devices visible */
int krk_set_device(int dev);                 /* per calling thread */
/* Eager context creation (streams, CRC tables) for the devices in dev_mask (bit i =
 * device i; 0 = the calling thread's current device), so the first request on a
 * device does not pay it; otherwise contexts are created on first use.  KRK_ENODEV
 * if a masked device is absent or not gfx950.  (SURVEY.md 8(b) krk_init.) */
int krk_init(uint64_t dev_mask);
/* Free every device context: streams, tables, scratch, pinned upload slots and the
 * staging windows kept across host-path calls (up to 2 x 1 GiB pinned per device).
 * The caller guarantees no library call is in flight and every krk_digester /
 * krk_piece_stream / krk_stream handle is freed.  Later calls re-create contexts
 * lazily. */
int krk_shutdown(void);
int krk_synchronize(void);                   /* drain the library's streams on the current device */

/* ------------------------------------------------- CRC-32/IEEE piece sums
 * Replaces core.calcPieceSums (core/metainfo.go:158-179), the loop inside
 * core.NewMetaInfo (core/metainfo.go:55-79); PieceHash() = crc32.NewIEEE()
 * (core/piece_hash.go:22-24).  Pieces are [i*P, min((i+1)*P, L)), ceil(L/P)
 * sums, none for L == 0, no empty trailing piece. */

typedef struct krk_blob {
    const uint8_t* data;     /* device pointer (any alignment; 16 B is the fast path) */
    uint64_t length;         /* bytes */
    int64_t piece_length;    /* > 0, else KRK_EINVAL "piece length must be positive" */
    uint64_t sums_offset;    /* index of this blob's first sum in the sums array */
} krk_blob;

/* Number of piece sums for a blob: ceil(length / piece_length). */
uint64_t krk_num_pieces(uint64_t length, int64_t piece_length);

/* Device-resident batch: sums_dev (device, uint32) receives every blob's sums
 * at blobs[i].sums_offset.  Asynchronous on `stream`. */
int krk_piece_sums_dev(const krk_blob* blobs, uint64_t n_blobs, uint32_t* sums_dev, void* stream);

/* Host batch (end-to-end): blobs[i].data are HOST pointers; sums_host receives
 * the sums.  Streams bytes through pinned staging, overlapping H2D with the
 * kernel.  Synchronous.  This is the batch form of Generator.Generate's
 * NewMetaInfo call (lib/metainfogen/generator.go:41-58). */
int krk_piece_sums_host(const krk_blob* blobs, uint64_t n_blobs, uint32_t* sums_host);
/* krk_piece_sums_host and krk_verify_pieces_host split a batch, whole pieces at a time,
 * between host PCLMUL threads (the reference's own placement: one hash.Hash32 per piece,
 * lib/torrent/storage/agentstorage/torrent.go:182-193) and the GPU pass.  Pinned caller
 * bytes (krk_host_alloc) are DMA'd straight into the device windows and the GPU takes a
 * share learned from the previous calls' measured rates of both sides (first call: the
 * planner rates' model, at most 10 %) -- or none, when host-only calls measured faster
 * than split ones (after two split calls -- the first sets up the staging windows -- one
 * runs host-only to find out; every 16th call re-measures the other choice).  Pageable
 * bytes stay on the host (a staging copy per byte costs more than the GPU saves).
 * KRK_CRC_GPU_FRACTION forces the share. */

/* Piece sums of cache FILES: the batch form of Generator.Generate reading the
 * CAS cache file itself (lib/metainfogen/generator.go:41-58: GetCacheFileReader
 * -> NewMetaInfo).  Placement as krk_crc32_update (krk_set_crc_placement; AUTO =
 * the measured crossover, HOST without a device): HOST reads each file once in
 * 512 KiB preads on the host pool and CRCs each chunk in cache; GPU reads the
 * bytes (pread on a pool of host threads, or O_DIRECT when KRK_FILE_DIRECT=1 and
 * the filesystem allows it) straight into the pinned staging windows -- no
 * pageable copy -- and the windows feed the CRC kernel as in krk_piece_sums_host.
 * The call's bytes on each side are reported by
 * krk_crc_host_split (kraken_hip_internal.h).  length is the size
 * the caller stat-ed (Generate picks the piece length from it); a file shorter
 * than that is KRK_EIO "read blob: <path>: unexpected EOF".  Synchronous. */
typedef struct krk_file_blob {
    const char* path;
    uint64_t length;
    int64_t piece_length;    /* > 0 */
    uint64_t sums_offset;
} krk_file_blob;
int krk_piece_sums_files(const krk_file_blob* files, uint64_t n_files, uint32_t* sums_host);

/* Streaming form for NewMetaInfo(d, io.Reader, P): the cgo shim copies each Read() chunk in
 * with _update; _end returns the io.CopyN-loop results (core/metainfo.go:157-179).
 * Placement (KRK_PLACE_* below), fixed at _begin:
 *   KRK_PLACE_HOST  the caller's thread runs PCLMUL CRC-32 over each chunk in place (~17 GB/s
 *                   a core, the reference's own placement) -- no copy, no PCIe;
 *   KRK_PLACE_GPU   bytes go through the device's submission engine (pooled pinned slots;
 *                   the CRC requests of all concurrent streams and crc32_update calls share
 *                   launches); each slot's piece portions are hashed as independent
 *                   messages and folded into the piece sums on the host with the GF(2)
 *                   combine, so state crosses slot and piece boundaries;
 *   KRK_PLACE_AUTO  (krk_piece_stream_begin) the process setting (krk_set_crc_placement,
 *                   KRK_CRC_PLACEMENT), by default the crossover: HOST unless the host's CRC
 *                   capacity (the CPUs this process may use x one thread's measured PCLMUL
 *                   rate) is below what the host link could carry to the GPU (0.85 x the
 *                   measured pinned H2D rate) -- on MI355X hosts the host side carries
 *                   60-80 GB/s for one stream and > 100 GB/s for several against ~20 GB/s
 *                   through the engine; HOST when no gfx950 device is present.
 * HOST placement needs no device; GPU placement without one is KRK_ENODEV. */
typedef struct krk_piece_stream krk_piece_stream;
int krk_piece_stream_begin(int64_t piece_length, krk_piece_stream** out);
int krk_piece_stream_begin_on(int placement, int64_t piece_length, krk_piece_stream** out);
int krk_piece_stream_placement(const krk_piece_stream* s, int* placement);
int krk_piece_stream_update(krk_piece_stream* s, const uint8_t* host_buf, uint64_t n);
int krk_piece_stream_end(krk_piece_stream* s, uint32_t* sums_out, uint64_t cap,
                         uint64_t* n_sums, uint64_t* length);
void krk_piece_stream_free(krk_piece_stream* s);

/* crc32.Update(crc, IEEETable, p) for one buffer (hash.Hash32 Write path used by
 * agentstorage.Torrent.writePiece, lib/torrent/storage/agentstorage/torrent.go:175-199).
 * data is a HOST pointer.  AUTO (krk_crc32_update): calls of at most 64 KiB
 * (KRK_CRC_HOST_MAX) and every call while the crossover of krk_piece_stream_begin says HOST
 * run on the caller's thread (large ones shared with idle host-pool threads); the rest go
 * through the device's CRC queue, coalesced with the other pending requests of the device
 * into one launch.  krk_crc32_update_on forces a placement. */
int krk_crc32_update(uint32_t crc, const uint8_t* data, uint64_t n, uint32_t* out);
int krk_crc32_update_on(int placement, uint32_t crc, const uint8_t* data, uint64_t n, uint32_t* out);
/* What KRK_PLACE_AUTO means for new piece streams and crc32_update calls, process-wide:
 * KRK_PLACE_AUTO (default: the crossover), KRK_PLACE_HOST or KRK_PLACE_GPU. */
int krk_set_crc_placement(int placement);

/* Batch piece verification (the same kernel in verify mode): ok_out[i] = 1 iff
 * piece i of the blob matches expected[i].  data is a device pointer. */
int krk_verify_pieces_dev(const krk_blob* blob, const uint32_t* expected_host,
                          uint8_t* ok_out_host, void* stream);

/* Batched agent piece verification over HOST buffers: ok_out[i] = 1 iff
 * crc32(data[i][0:lengths[i]]) == expected[i] -- the h.Sum32() != GetPieceSum(pi)
 * check of agentstorage.Torrent.writePiece (lib/torrent/storage/agentstorage/
 * torrent.go:174-199, error "invalid piece sum"), for many received pieces (any
 * torrents, any lengths) in one pinned, pipelined GPU pass instead of one
 * hash.Hash32 per piece.  Synchronous. */
int krk_verify_pieces_host(const uint8_t* const* data, const uint64_t* lengths, const uint32_t* expected,
                           uint64_t n, uint8_t* ok_out);

/* ----------------------------------------------------- SHA-256 (Digester)
 * Replaces core.Digester (core/digester.go:28-72): crypto.SHA256 over the whole
 * blob.  One Merkle-Damgard stream per lane, many blobs per launch. */

/* Device-resident batch: data_dev[i] (device pointers, array itself on host),
 * lengths[i]; digests_dev receives n*32 bytes (device). Asynchronous. */
int krk_sha256_dev(const uint8_t* const* data_dev, const uint64_t* lengths, uint64_t n,
                   uint8_t* digests_dev, void* stream);

/* Device-resident batch hashed by host threads (x86 SHA extensions): up to `threads`
 * threads (<= 0: the CPUs this process may use) each read a blob out of device memory
 * through their own pinned double buffers, after the work queued on `stream` up to the
 * call; digests_host n*32 bytes.  Synchronous.  The host lane of a windowed batch
 * (kraken_amd/windowed.py): the longest chains of a larger-than-HBM batch hashed on the
 * host while the GPU windows run the rest. */
int krk_sha256_dev_on_host(const uint8_t* const* data_dev, const uint64_t* lengths, uint64_t n, int threads,
                           void* stream, uint8_t* digests_host);

/* Host batch: HOST data pointers; digests_host n*32 bytes.  Synchronous.  The window
 * schedule of krk_metainfo_digest_host without the piece CRCs (at most the window
 * stream cap of blobs live, admitted longest first; page-locked blobs DMA'd directly),
 * and the planner's blobs hashed in place on host threads under the default AUTO host
 * offload. */
int krk_sha256_host(const uint8_t* const* data_host, const uint64_t* lengths, uint64_t n,
                    uint8_t* digests_host);

/* Streaming Digester (core.NewDigester, digester.go:34): _write may be called any
 * number of times (io.Copy chunks); _sum does not reset (Digester.Digest(),
 * digester.go:41-48) so writing may continue afterwards.  One digester is
 * single-owner (like hash.Hash); different digesters may be used from different
 * threads at once.
 *
 * Placement, fixed at creation:
 *   KRK_PLACE_GPU   bytes go through the device's submission engine: the caller copies
 *                   them into pooled pinned slots (512 KiB, KRK_SLOT_KB) and every
 *                   pending slot of every GPU digester of the device is digested in
 *                   ONE multi-stream sha256_multi launch (a dispatcher thread batches
 *                   them).  A digester's midstate lives in an HBM row of the engine,
 *                   so its requests chain through the device in stream order and the
 *                   next launch is queued behind the running one (up to 8 requests
 *                   of a digester in flight; the kernel reads the pinned slots in
 *                   place).  Creation allocates nothing on the device.
 *   KRK_PLACE_HOST  SHA-NI on the caller's thread (host_meta.cpp): ~2 GB/s per stream
 *                   against ~59 MB/s for one GPU stream.
 *   KRK_PLACE_AUTO  (krk_digester_new) HOST while at most N digesters are live in the
 *                   process, GPU beyond.  N is the crossover computed from the calling
 *                   thread's device's planner rates: the fewest live GPU digesters whose
 *                   aggregate (live streams x the measured per-stream rate of the launch
 *                   plan they get, capped by what the engine's zero-copy slot reads carry:
 *                   0.58 x the measured pinned H2D rate) beats the host's (the process's CPU
 *                   budget x one thread's measured SHA-NI rate); never (all on the host) when
 *                   the host out-hashes that -- the case on MI355X boxes' 16-CPU shares
 *                   (measured: 32.7 GB/s at best on the GPU against 34-37 on the host).  KRK_DIGESTER_HOST_STREAMS or
 *                   krk_set_digester_host_streams pins N (-1 restores the default).
 * HOST placement needs no device; GPU placement without a gfx950 device is KRK_ENODEV and
 * AUTO without one is HOST (the product's own SHA-NI path, not the oracle). */
typedef struct krk_digester krk_digester;
#define KRK_PLACE_AUTO 0
#define KRK_PLACE_HOST 1
#define KRK_PLACE_GPU 2
int krk_digester_new(krk_digester** out);
int krk_digester_new_on(int placement, krk_digester** out);
int krk_digester_placement(const krk_digester* d, int* placement);
int krk_digester_write(krk_digester* d, const uint8_t* host_buf, uint64_t n);
int krk_digester_sum(krk_digester* d, uint8_t out32[32]);
void krk_digester_free(krk_digester* d);
int krk_set_digester_host_streams(int64_t n);

/* The slot pool's HARD cap on pinned staging bytes for the calling thread's device
 * (default KRK_SLOT_POOL_MB = 4096 MiB; at least one 16-slot chunk).  At the cap a
 * writer waits for a slot to come back (backpressure) instead of pinning more: slots
 * are held only by requests in flight, never by an idle digester or piece stream (their
 * partial data stays in their own host buffer).  Lowering the cap frees nothing already
 * pinned.  bytes == 0 only reads: *cap_out = the cap, *waits_out = how many times a
 * writer waited at it (either may be NULL). */
int krk_engine_set_pool_cap(uint64_t bytes, uint64_t* cap_out, uint64_t* waits_out);

/* ----------------------------------------- metainfo + digest (batch)
 * Both products for every blob in one call: the Digester SHA-256 of
 * uploader.verify (origin/blobserver/uploader.go:74-94) and the piece sums of
 * Generate (lib/metainfogen/generator.go:41-58).  The SHA and CRC kernels run
 * concurrently on two internal streams joined back into `stream`.  Device
 * pointers; asynchronous. */
int krk_metainfo_digest_dev(const krk_blob* blobs, uint64_t n_blobs, uint32_t* sums_dev,
                            uint8_t* digests_dev, void* stream);

/* Chunked (streaming) form on device data: each call advances every listed blob
 * by one chunk -- SHA-256 from the blob's midstate in state_dev (8 words per
 * blob slot, written back), CRC-32 of the chunk's byte range XOR-accumulated
 * into its pieces' sums (sums_dev must be zero before a blob's first chunk).
 * A blob's chunks are submitted in order, one per call; every chunk but the
 * last is a multiple of 64 bytes; the chunk that reaches blob_length writes
 * the digest to digests_dev[32*blob].  This is the multi-blob Digester.Write +
 * calcPieceSums step that end-to-end and larger-than-HBM batches (C3) run
 * window by window.  Asynchronous on `stream`. */
typedef struct krk_chunk {
    const uint8_t* data;     /* device pointer to the chunk's bytes */
    uint64_t offset;         /* chunk's first byte inside its blob */
    uint64_t length;         /* chunk bytes */
    uint64_t blob_length;    /* total blob length */
    int64_t piece_length;    /* > 0 */
    uint64_t sums_offset;    /* blob's first piece-sum slot */
    uint64_t blob;           /* blob slot for state_dev / digests_dev */
} krk_chunk;
int krk_metainfo_digest_chunks_dev(const krk_chunk* chunks, uint64_t n_chunks, uint32_t* state_dev,
                                   uint32_t* sums_dev, uint8_t* digests_dev, void* stream);
/* The same with the SHA-256 launch on `sha_stream` (NULL: the library's own), forked from
 * and joined back into `stream` like the default; with a sha_stream the piece CRCs run on
 * `stream` itself (no barrier of the step on the library's streams).  A caller that runs D2H copies beside
 * the windows (the C3 host lane, kraken_amd/windowed.py) passes a stream of another
 * priority (krk_stream_create_prio): streams of one priority share the device's few
 * hardware queues, and a copy queued behind a window's ~0.6 s SHA-256 launch on a shared
 * queue waits for it. */
int krk_metainfo_digest_chunks_dev_on(const krk_chunk* chunks, uint64_t n_chunks, uint32_t* state_dev,
                                      uint32_t* sums_dev, uint8_t* digests_dev, void* stream, void* sha_stream);

/* End-to-end form: blobs[i].data are HOST pointers (pageable or pinned).  Every
 * byte crosses PCIe once, window by window, and both kernels run on each window
 * (SHA-256 chained from per-blob midstates, CRC by byte range) while the next window
 * goes up.  How a window goes up: page-locked blobs (krk_host_alloc) by one DMA a chunk
 * (few wide chunks) or one gather launch that reads the caller's pages over PCIe, so each
 * byte is read from host memory once, by the GPU; pageable blobs are copied by host threads
 * into the library's pinned windows first (measured faster than registering the caller's
 * 4 KiB pages for the gather, which KRK_HOST_GATHER=1 still does).  Allocate receive buffers
 * with krk_host_alloc to get the one-read path.  sums_host indexed by blobs[i].sums_offset;
 * digests_host n_blobs*32 bytes.  Synchronous. */
int krk_metainfo_digest_host(const krk_blob* blobs, uint64_t n_blobs, uint32_t* sums_host,
                             uint8_t* digests_host);

/* The same from the CAS files themselves: the upload verify of uploader.verify
 * (origin/blobserver/uploader.go:74-94) or the cache-fill digest of CAStore.WriteCacheFile
 * (lib/store/ca_store.go:99-135) fused with the metainfo Generator.Generate computes from the
 * cache file (lib/metainfogen/generator.go:41-58): each file is read ONCE (pread on the host
 * pool into the pinned windows; O_DIRECT for a cold batch, below) and that read feeds both
 * the SHA-256 digest and the piece CRCs -- the reference reads it twice.  files[i].length is
 * the size the caller stat-ed; a shorter file is KRK_EIO "read blob: <path>: unexpected EOF",
 * an unopenable one KRK_EIO "open <path>: <errno text>".  Live blobs per window are also
 * capped by the file descriptors the process may still open (RLIMIT_NOFILE).  With the host
 * offload (KRK_OFFLOAD_AUTO) the planner's files are read, hashed and piece-summed on host
 * threads in one pass each -- unless a sample of the files (mmap + mincore, no reads) finds
 * them mostly outside the page cache: a disk-bound batch stays on the windows and is read
 * O_DIRECT through Linux AIO (one thread queues a window's chunks; KRK_FILE_DIRECT=1/0
 * forces O_DIRECT on/off).  KRK_FILE_READAHEAD_MB=N keeps each file hinted N MiB ahead of
 * its page-cache reads (POSIX_FADV_WILLNEED; off by default).  Synchronous. */
int krk_metainfo_digest_files(const krk_file_blob* files, uint64_t n_files, uint32_t* sums_host,
                              uint8_t* digests_host);

/* ------------------------------------------------------- multi-device
 * One process, several GPUs (the origin is one process,
 * origin/cmd/cmd.go:164).  The device set -- the devices of the last krk_init mask,
 * or krk_set_devices (a device may repeat: several workers on one GPU), default the
 * calling thread's device -- is where the *_multi calls run and where new Digesters
 * and piece streams are placed (round-robin).  A *_multi call splits its batch by
 * bytes (LPT: the longest blob to the least-loaded device), runs the single-device
 * entry point on every device from its own host thread and gathers the results
 * into the caller's arrays (same layout as the single-device call).  No collective:
 * blobs are independent.  Synchronous. */
int krk_set_devices(const int* devs, uint32_t n);
int krk_get_devices(int* devs, uint32_t cap, uint32_t* n);
int krk_metainfo_digest_host_multi(const krk_blob* blobs, uint64_t n_blobs, uint32_t* sums_host,
                                   uint8_t* digests_host);
int krk_piece_sums_host_multi(const krk_blob* blobs, uint64_t n_blobs, uint32_t* sums_host);
int krk_piece_sums_files_multi(const krk_file_blob* files, uint64_t n_files, uint32_t* sums_host);
int krk_metainfo_digest_files_multi(const krk_file_blob* files, uint64_t n_files, uint32_t* sums_host,
                                    uint8_t* digests_host);
int krk_sha256_host_multi(const uint8_t* const* data_host, const uint64_t* lengths, uint64_t n,
                          uint8_t* digests_host);

/* ---------------------------------------------------- InfoHash (host CPU)
 * info.Hash() (core/metainfo.go:37-44): SHA-1 over the bencoded
 * info{PieceLength, PieceSums, Name, Length}.  bencode_out may be NULL. */
int krk_info_hash(int64_t piece_length, const uint32_t* sums, uint64_t n_sums,
                  const char* name, uint64_t name_len, int64_t length, uint8_t out20[20]);
/* Batch form for many blobs (Generator.Generate over a batch, whole-CAS regen):
 * blob i has piece_lengths[i], sums[sums_off[i] .. sums_off[i] + n_sums[i]), name
 * names[name_off[i] .. name_off[i+1]), length lengths[i]; out20 receives 20*n bytes.
 * Spread over host threads.  names may be NULL when every name is empty. */
/* Generator.Generate over device-resident blobs (lib/metainfogen/generator.go:41-58 ->
 * core.NewMetaInfo, core/metainfo.go:53-79): every blob's piece sums (sums_dev, also
 * copied to sums_host at blobs[i].sums_offset) and its InfoHash (info_hash20, 20 B a
 * blob; names/name_off = the blobs' digest hex, the info Name).  The batch runs as up to
 * 8 groups of about equal bytes back to back on `stream`; each group's sums are copied
 * back and hashed on host threads while the later groups' kernels run.  Synchronous. */
int krk_metainfo_batch_dev(const krk_blob* blobs, uint64_t n_blobs, const char* names, const uint64_t* name_off,
                           uint32_t* sums_dev, uint32_t* sums_host, uint8_t* info_hash20, void* stream);
int krk_info_hash_batch(const int64_t* piece_lengths, const uint32_t* sums, const uint64_t* sums_off,
                        const uint64_t* n_sums, const char* names, const uint64_t* name_off,
                        const int64_t* lengths, uint64_t n, uint8_t* out20);
int krk_bencode_info(int64_t piece_length, const uint32_t* sums, uint64_t n_sums,
                     const char* name, uint64_t name_len, int64_t length,
                     uint8_t* out, uint64_t cap, uint64_t* written);

/* pieceLengthConfig.get (lib/metainfogen/config.go:71-80); thresholds ascending. */
int64_t krk_piece_length_for_size(const int64_t* thresholds, const int64_t* lengths,
                                  uint32_t n, int64_t size);

/* -------------------------------------------------------- HRW placement
 * Replaces hrw.RendezvousHash.GetOrderedNodes / RendezvousHashNode.Score
 * (lib/hrw/rendezvous.go:151-217) with murmur3.New64 + UInt64ToFloat64
 * (rendezvous.go:39,99-118), and hashring.ring.Locations (lib/hashring/ring.go:96-118).
 * Keys are hex strings (hex-decoded, then key||label is hashed).  Order is
 * descending score; exact ties go to the lower node index (the reference's
 * tie order is unspecified: Go map order, ring.go:151). */

typedef struct krk_nodes {
    const char* labels;          /* concatenated label bytes */
    const uint64_t* label_off;   /* n_nodes + 1 offsets into labels */
    const int64_t* weights;      /* n_nodes (ring nodes use 100, ring.go:28) */
    uint32_t n_nodes;
} krk_nodes;

/* keys: concatenated hex strings with key_off (n_keys+1).  order_out:
 * n_keys * n_out node indices (-1 padded when n_out > n_nodes); scores_out
 * (nullable): n_keys * n_nodes, in node order.  Returns KRK_EHEX if any key is
 * not valid hex (its row is then filled from NaN scores: node order). */
int krk_hrw_ordered(const char* keys, const uint64_t* key_off, uint64_t n_keys,
                    const krk_nodes* nodes, uint32_t n_out, int32_t* order_out,
                    double* scores_out);

/* hrw.UInt64ToFloat64 (rendezvous.go:99-118) with MaxHashValue = 8 x 0xFF (murmur3's
 * Sum size): sums8 holds n 8-byte big-endian hash Sums; out[i] = low 53 bits / 2^53,
 * where all-zero low bits are re-hashed once with murmur3.New64 when rehash != 0 (the
 * hasher argument; 0 = nil hasher).  Runs the scoring kernel's own device function. */
int krk_hrw_uint64_to_float64(const uint8_t* sums8, uint64_t n, int rehash, double* out);

/* ring.Locations for raw 32-byte sha256 digests (ShardID = first 2 bytes).
 * healthy: n_nodes flags.  locs_out: n * max(1, max_replica) node indices
 * (-1 padded); counts_out: n entries. */
int krk_ring_locations(const uint8_t* digests32, uint64_t n, const krk_nodes* nodes,
                       const uint8_t* healthy, int32_t max_replica,
                       int32_t* locs_out, uint8_t* counts_out);
/* The whole ring in one call: Locations(d) depends on d only through ShardID =
 * hex[:4] (core/digest.go:148-150), so the 65,536 possible owner lists are computed
 * once per membership or health change (ring.Refresh, lib/hashring/ring.go:141-165)
 * and Locations becomes a host lookup: row ((d[0] << 8) | d[1]) of locs_out
 * (65,536 x max(1, max_replica) node indices, -1 padded) with counts_out[row] valid
 * entries.  Same semantics as krk_ring_locations. */
int krk_ring_owner_table(const krk_nodes* nodes, const uint8_t* healthy, int32_t max_replica,
                         int32_t* locs_out, uint8_t* counts_out);
/* Device-resident form (digests in device memory).  The owner table of a membership
 * (labels, weights, healthy, max_replica) is built on its first call and kept (8
 * memberships a device, least recently used replaced), as the reference's Ring keeps its
 * hrw until Refresh; later calls only gather.  locs/counts: device memory, or page-locked
 * host memory (krk_host_alloc) that the gather writes over PCIe -- the owner lists are on
 * the host when the stream reaches the call's end, with no copy-back; any other pointer is
 * KRK_EINVAL. */
int krk_ring_locations_dev(const uint8_t* digests32_dev, uint64_t n, const krk_nodes* nodes,
                           const uint8_t* healthy, int32_t max_replica,
                           int32_t* locs_dev, uint8_t* counts_dev, void* stream);
/* Compact form for rings of <= 255 nodes (KRK_ERANGE beyond): owner indices as
 * uint8 (0xFF padded), a quarter of the bytes the caller copies back.  Same
 * ring.Locations semantics (lib/hashring/ring.go:91-118) as krk_ring_locations_dev. */
int krk_ring_locations_u8_dev(const uint8_t* digests32_dev, uint64_t n, const krk_nodes* nodes,
                              const uint8_t* healthy, int32_t max_replica,
                              uint8_t* locs_dev, uint8_t* counts_dev, void* stream);

/* ------------------------------------------------ device memory helpers
 * For callers (benchmarks, cgo) that do not own a device allocator. */
int krk_dev_alloc(uint64_t bytes, void** out);
int krk_dev_free(void* p);
/* Pinned (page-locked) host memory: what a cgo caller reads files / receives
 * pieces into so that the host entry points DMA it without a staging copy, and
 * where device results are gathered at full PCIe rate. */
int krk_host_alloc(uint64_t bytes, void** out);
int krk_host_free(void* p);
int krk_memcpy_h2d(void* dst_dev, const void* src_host, uint64_t n);
int krk_memcpy_d2h(void* dst_host, const void* src_dev, uint64_t n);
/* Queued on `stream` (NULL = the library's stream): dst_host should be pinned
 * (krk_host_alloc) for the copy to overlap the host. */
int krk_memcpy_d2h_async(void* dst_host, const void* src_dev, uint64_t n, void* stream);
int krk_stream_create(void** out);
/* A stream of the given priority: -1 high, 0 normal, 1 low (HIP's priority range).
 * Streams of another priority run on hardware queues of their own: a stream that holds
 * long kernels (a C3 window's SHA-256 launch runs ~0.6 s) is kept off the queues the
 * short work shares, which would otherwise wait behind it. */
int krk_stream_create_prio(int priority, void** out);
/* Waits for the stream's work, retires the library's state tied to it (events of upload
 * slots and scratch blocks last used on it), then destroys it.  Streams handed to the
 * library must be destroyed here, not with hipStreamDestroy. */
int krk_stream_destroy(void* s);
int krk_stream_sync(void* s);
/* Events (a window loop waits for ONE earlier window's kernels while the next
 * window's are already queued behind them on the same stream).  No timing; a thread in
 * krk_event_sync sleeps until the event completes rather than spinning a core. */
int krk_event_create(void** out);
int krk_event_record(void* ev, void* stream);
int krk_event_sync(void* ev);
int krk_event_destroy(void* ev);

/* Host offload of the longest SHA-256 chains, process-wide.  krk_sha256_dev and
 * krk_metainfo_digest_dev hand the longest blobs of a batch to host threads (x86 SHA
 * extensions, ~2 GB/s a thread against ~59 MB/s a GPU stream), which read them from device
 * memory through pinned double buffers while the GPU hashes the rest and every blob's piece
 * CRCs; the digests land in digests_dev as before.  How many go to the host minimises
 * max(GPU time, host time) at the planner's measured rates (krk_planner_rates_get) and is 0
 * unless that shortens the batch by 10 %: a single 1 GiB blob (C1) goes to the host.  When
 * whole blobs cannot shorten it -- 1,000 equal 100 MiB blobs (C2) each take the GPU ~1.8 s
 * wherever the others run -- every chain starts on the GPU and host threads take over the
 * tails of the longest ones from the GPU's midstate, each as soon as the GPU has reached its
 * planned split (tail handoff, when the model ends the batch 5 % sooner; KRK_SHA_TAIL=0
 * off): C2 1.42 s a batch against 1.77.  The call then returns after the host part is
 * hashed (the GPU part stays asynchronous on `stream`; with tail handoff, once the SHA-256
 * launch has ended too).  The host-buffer entry points work
 * on their offloaded blobs in place and never upload them: krk_sha256_host hashes them,
 * krk_metainfo_digest_host hashes them AND computes their piece sums (the SHA-256 pass and
 * the CRC pass of a blob are separate host tasks), so the bytes that cross the host link
 * shrink by theirs (the threshold there is 3 %).
 * threads: KRK_OFFLOAD_AUTO (-1, the default) = the process's host CPU budget (the node's
 * CPUs -- affinity capped by the cgroup quota -- divided among the LOCAL_WORLD_SIZE ranks of
 * a node, or KRK_HOST_CPUS) for device-resident batches and a quarter of them for
 * host-resident batches (whose staging windows need the rest as copy threads); 0 = off
 * (every chain on the GPU); n = up to n threads. */
#define KRK_OFFLOAD_AUTO (-1)
int krk_set_sha_host_offload(int threads);
int krk_sha_host_offload(int* threads);      /* the current setting */
/* The rates the planners use (the offload of the batch entry
 * points, the host/GPU split of the CRC-only host entry points), per device:
 * sha_stream_bps = one SHA-256 stream's rate at full residency under each AUTO tier
 * (eight lanes up to 16 x CUs streams, two lanes up to 64 x CUs, one lane beyond),
 * pinned D2H / H2D copy rates, one host thread's SHA-256, CRC-32 and memcpy rates.  Measured on
 * the calling thread's device at first use (~50 ms: each tier's launch plan timed on
 * 16 / 64 / 128 x CUs streams, a 64 MiB pinned copy each way); without a device the
 * nominal MI355X figures (source 0).  (kraken_hip_internal.h: krk_planner_rates_set
 * overrides them for tests, krk_host_offload_plan shows a plan without device work.) */
#define KRK_RATES_NOMINAL 0
#define KRK_RATES_MEASURED 1
#define KRK_RATES_SET 2
typedef struct krk_planner_rates {
    double sha_stream_bps[3];
    double d2h_bps, h2d_bps;
    double host_sha_bps, host_crc_bps, host_copy_bps;
    int32_t cus;
    int32_t source;
} krk_planner_rates;
int krk_planner_rates_get(krk_planner_rates* out);
/* Measure the calling thread's device's rates now (krk_init does it for its devices, so that
 * the measurement runs before the library has work of its own on them; otherwise the first
 * planner use measures).  Re-measure after a change of load the planners should see. */
int krk_planner_calibrate(void);

#ifdef __cplusplus
}
#endif
#endif /* KRAKEN_HIP_H */
