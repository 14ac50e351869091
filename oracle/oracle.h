/*
 * oracle.h -- CPU restatement of Kraken's blob-metainfo hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / the timed CPU baseline.  The product (kraken_amd, libkraken_hip)
 * never links, loads or calls it.
 *
 * Parity status: pinned.  Every primitive is checked against the reference's
 * own known-answer tests (InfoHash KAT core/metainfo_test.go:61-76,
 * sha256("test") core/digester_test.go:27-28, DigestEmptyTar core/digest.go:28,
 * GetPieceLength table core/metainfo_test.go:25-46, piece-length ranges
 * lib/metainfogen/config_test.go:23-38, the zero-rehash property
 * lib/hrw/rendezvous_test.go:59-98) and against independent implementations
 * (Python zlib.crc32 / hashlib) plus the published test vectors of the
 * un-vendored spaolacci/murmur3 @ 9f5d223c (glide.lock:231-232).
 * See tests/test_oracle_golden.py.
 */
#ifndef KRAKEN_ORACLE_H
#define KRAKEN_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- CRC-32/IEEE: core/piece_hash.go:22-24 (crc32.NewIEEE) ---- */
uint32_t orc_crc32_update(uint32_t crc, const uint8_t* p, uint64_t n);
/* PCLMULQDQ folding variant (what Go's amd64 crc32 uses for >=64 B); same result. */
uint32_t orc_crc32_update_clmul(uint32_t crc, const uint8_t* p, uint64_t n);
int orc_have_clmul(void);

/* ---- core.calcPieceSums: core/metainfo.go:158-179 ----
 * returns 0, or -1 for "piece length must be positive".
 * sums may be NULL to query the count.  *n_sums = ceil(len/piece_len). */
int orc_calc_piece_sums(const uint8_t* blob, uint64_t len, int64_t piece_len,
                        uint32_t* sums, uint64_t* n_sums, uint64_t* length);

/* ---- MetaInfo.GetPieceLength: core/metainfo.go:109-118 ---- */
int64_t orc_get_piece_length(int64_t length, int64_t piece_len, uint64_t n_pieces, int64_t i);

/* ---- SHA-256 (core.Digester, crypto/sha256), FIPS 180-4 ---- */
typedef struct { uint32_t h[8]; uint64_t nbytes; uint8_t buf[64]; uint32_t nbuf; } orc_sha256_ctx;
void orc_sha256_init(orc_sha256_ctx* c);
void orc_sha256_update(orc_sha256_ctx* c, const uint8_t* p, uint64_t n);
/* Sum without reset (Go hash.Hash.Sum semantics, digester.go:41-48). */
void orc_sha256_sum(const orc_sha256_ctx* c, uint8_t out[32]);
void orc_sha256(const uint8_t* p, uint64_t n, uint8_t out[32]);
/* SHA-NI variant used only by the CPU baseline; same result. */
void orc_sha256_shani(const uint8_t* p, uint64_t n, uint8_t out[32]);
int orc_have_shani(void);

/* ---- SHA-1 + bencode -> InfoHash: core/metainfo.go:37-44, core/infohash.go:42-49 ---- */
void orc_sha1(const uint8_t* p, uint64_t n, uint8_t out[20]);
/* bencode of info{PieceLength,PieceSums,Name,Length} (keys sorted: Length, Name,
 * PieceLength, PieceSums).  Returns bytes written (or needed if out==NULL). */
uint64_t orc_bencode_info(int64_t piece_len, const uint32_t* sums, uint64_t n_sums,
                          const char* name, uint64_t name_len, int64_t length,
                          uint8_t* out, uint64_t cap);
void orc_info_hash(int64_t piece_len, const uint32_t* sums, uint64_t n_sums,
                   const char* name, uint64_t name_len, int64_t length, uint8_t out[20]);

/* ---- murmur3 x64_128, h1 only (spaolacci murmur3.New64(), seed 0) ---- */
uint64_t orc_murmur3_h1(const uint8_t* p, uint64_t n, uint64_t seed);

/* ---- lib/hrw: rendezvous.go ---- */
double orc_go_log(double x);                      /* Go math.Log (src/math/log.go) */
double orc_uint64_to_float64(uint64_t h1, int rehash); /* rendezvous.go:99-118 */
/* Score(key) with key = hex string; returns NaN for invalid hex (rendezvous.go:154-157). */
double orc_hrw_score(const char* key_hex, uint64_t key_len, const char* label,
                     uint64_t label_len, int64_t weight);
/* GetOrderedNodes(key, n) (rendezvous.go:207-217): descending score; exact ties
 * broken by ascending node index (the reference leaves tie order unspecified). */
int orc_hrw_ordered(const char* key_hex, uint64_t key_len, const char* labels,
                    const uint64_t* label_off, const int64_t* weights, uint32_t n_nodes,
                    uint32_t n_out, int32_t* order_out, double* scores_out);
/* ring.Locations filtering (lib/hashring/ring.go:96-118) over a full order. */
uint32_t orc_ring_locations(const int32_t* order, uint32_t n_nodes, const uint8_t* healthy,
                            int32_t max_replica, int32_t* out);

/* Every ShardID's Locations: 65,536 rows of row_out owners (-1 padded) + counts. */
void orc_ring_owner_table(const char* labels, const uint64_t* label_off, const int64_t* weights,
                          uint32_t n_nodes, const uint8_t* healthy, int32_t max_replica, uint32_t row_out,
                          int32_t* locs, uint8_t* counts);

/* ---- lib/metainfogen/config.go:71-80 ---- */
int64_t orc_piece_length_for_size(const int64_t* thresholds, const int64_t* lengths,
                                  uint32_t n, int64_t size);

/* ---- synthetic content (shared spec with the device fill kernel) ---- */
uint64_t orc_blob_seed(uint64_t blob_idx);
/* bytes [off, off+n) of blob blob_idx; variant 0 = uniform bytes, 1 = alnum */
void orc_synth_fill(uint64_t blob_idx, uint64_t off, uint8_t* out, uint64_t n, int variant);

/* ---- CPU baseline: the reference's two-pass structure, one blob per thread ----
 * For each of n_blobs synthetic blobs (generated untimed): SHA-256 pass
 * (uploader.go:74-94) then CRC piece pass (metainfo.go:158-179), both streamed
 * in 32 KiB chunks; the job list visits every blob `repeats` times (bounded RAM,
 * longer sample).  passes: bit 0 SHA-256 pass, bit 1 CRC pass (0 = both).
 * Returns seconds of the timed section; outputs optional. */
double orc_baseline_run(const uint64_t* blob_idx, const uint64_t* lengths, uint64_t n_blobs,
                        int64_t piece_len, int n_threads, int fast, int passes, uint64_t repeats,
                        uint8_t* digests_out, uint32_t* sums_out, const uint64_t* sums_off);
/* Bounded-memory form (one buffer per thread; each blob materialised untimed just
 * before its passes): returns the SUMMED busy seconds of the threads, so the
 * sustained rate is bytes / (busy / n_threads).  Always the fast (SHA-NI/PCLMUL) path. */
/* Upload verify (passes & 1) and Generate (passes & 2) over files, the reference's way (32 KiB reads). */
double orc_baseline_files(const char* const* paths, const uint64_t* lengths, uint64_t n, int64_t piece_len,
                          int n_threads, int passes, uint32_t* sums_out, const uint64_t* sums_off,
                          uint8_t* digests_out);
double orc_baseline_run_lazy(const uint64_t* blob_idx, const uint64_t* lengths, uint64_t n_blobs,
                             int64_t piece_len, int n_threads, int passes, uint8_t* digests_out,
                             uint32_t* sums_out, const uint64_t* sums_off);
/* HRW baseline: GetOrderedNodes + Locations per digest on n_threads. */
double orc_baseline_hrw(const uint8_t* digests, uint64_t n, const char* labels,
                        const uint64_t* label_off, uint32_t n_nodes, const uint8_t* healthy,
                        int32_t max_replica, int n_threads, int32_t* locs_out, uint8_t* counts_out);

#ifdef __cplusplus
}
#endif
#endif
