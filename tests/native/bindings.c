/* bindings.c -- the C side of every cgo binding in INTEGRATION.md, compiled as C11 with
 * -Wall -Werror against include/kraken_hip.h and run on the GPU (tests/test_gpu_bindings.py).
 * No Go toolchain exists in this image, so the Go files there cannot be compiled; this
 * program makes exactly the C calls they make, with the same argument shapes (C-allocated
 * arrays, pinned receive buffers, the two-phase krk_piece_stream_end, a failing write that
 * must surface from crc32_update), and checks every result against the CPU oracle
 * (oracle/oracle.c, linked as the checker only: orc_sha256 / orc_crc32_update, pinned by
 * the reference's KATs and zlib / hashlib in tests/test_oracle_golden.py).  The binding
 * calls use include/kraken_hip.h only; kraken_hip_internal.h is included for one
 * test-side check (which windows went up straight from the caller's pages).
 *
 *   bindings <scratch dir>      exit 0 = every binding shape worked and agreed */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/kraken_hip.h"
#include "../../include/kraken_hip_internal.h" /* krk_windows_last_*: test-side check only */
#include "../../oracle/oracle.h"               /* the checker */

static int fails = 0;
#define CHECK(cond, ...)                                        \
    do {                                                        \
        if (!(cond)) {                                          \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                       \
            fprintf(stderr, " (%s)\n", krk_last_error());       \
            ++fails;                                            \
        }                                                       \
    } while (0)

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint8_t next_byte(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint8_t)rng;
}

static uint32_t host_crc(uint32_t c, const uint8_t* p, uint64_t n) { return orc_crc32_update(c, p, n); }

int main(int argc, char** argv) {
    const char* dir = argc > 1 ? argv[1] : "/tmp";
    /* core/krkgpu.go init(): contexts for every GPU, the defaults need no knob */
    int n = 0;
    CHECK(krk_device_count(&n) == KRK_OK && n > 0, "device count");
    if (n <= 0) return 1;
    CHECK(krk_init(((uint64_t)1 << n) - 1) == KRK_OK, "krk_init");
    int off = 0;
    CHECK(krk_sha_host_offload(&off) == KRK_OK && off == KRK_OFFLOAD_AUTO, "offload default %d", off);

    const uint64_t L = (9u << 20) + 12345, P = 4u << 20;
    uint8_t* blob = malloc(L);
    for (uint64_t i = 0; i < L; ++i) blob[i] = next_byte();

    /* core/metainfo_krkgpu.go calcPieceSums: 4 MiB reads, two-phase end */
    {
        krk_piece_stream* s = NULL;
        CHECK(krk_piece_stream_begin((int64_t)P, &s) == KRK_OK, "stream begin");
        for (uint64_t a = 0; a < L; a += 4u << 20) {
            const uint64_t m = L - a < (4u << 20) ? L - a : (4u << 20);
            CHECK(krk_piece_stream_update(s, blob + a, m) == KRK_OK, "stream update");
        }
        uint64_t ns = 0, total = 0;
        CHECK(krk_piece_stream_end(s, NULL, 0, &ns, &total) == KRK_OK && ns == 3 && total == L, "end (count)");
        uint32_t sums[3];
        CHECK(krk_piece_stream_end(s, sums, ns, &ns, &total) == KRK_OK, "end (sums)");
        for (uint64_t k = 0; k < 3; ++k) {
            const uint64_t m = L - k * P < P ? L - k * P : P;
            CHECK(sums[k] == host_crc(0, blob + k * P, m), "piece %llu", (unsigned long long)k);
        }
        krk_piece_stream_free(s);
        s = NULL;
        CHECK(krk_piece_stream_begin(0, &s) == KRK_EINVAL, "zero piece length");
        CHECK(strcmp(krk_last_error(), "piece length must be positive") == 0, "error text");
    }
    /* core/piece_hash_krkgpu.go gpuCRC.Write: every write folded at once; errors surface */
    {
        uint32_t crc = 0, out = 0;
        for (uint64_t a = 0; a < L; a += 1000003) {
            const uint64_t m = L - a < 1000003 ? L - a : 1000003;
            CHECK(krk_crc32_update(crc, blob + a, m, &out) == KRK_OK, "crc32_update");
            crc = out;
        }
        CHECK(crc == host_crc(0, blob, L), "PieceHash over writes");
        CHECK(krk_crc32_update(0, NULL, 5, &out) == KRK_EINVAL, "a bad write fails, no stale value");
    }
    /* agentstorage verifyPieces: pinned receive buffers */
    {
        enum { NP = 6 };
        void* pc[NP];
        const uint8_t* pp[NP];
        uint64_t lens[NP];
        uint32_t want[NP];
        uint8_t ok[NP];
        for (int i = 0; i < NP; ++i) {
            lens[i] = (uint64_t)(i + 1) * 700001;
            CHECK(krk_host_alloc(lens[i], &pc[i]) == KRK_OK, "host_alloc");
            memcpy(pc[i], blob + i * 1000, lens[i]);
            pp[i] = (const uint8_t*)pc[i];
            want[i] = host_crc(0, pp[i], lens[i]) ^ (i == 3 ? 1u : 0u); /* piece 3 corrupted */
        }
        CHECK(krk_verify_pieces_host(pp, lens, want, NP, ok) == KRK_OK, "verify_pieces_host");
        for (int i = 0; i < NP; ++i) CHECK(ok[i] == (i != 3), "verdict %d", i);
        for (int i = 0; i < NP; ++i) krk_host_free(pc[i]);
    }
    /* uploader.verify + Generate from files (verifyAndGenerate) and pieceSumsFiles */
    {
        enum { NF = 5 };
        char path[NF][512];
        krk_file_blob fb[NF];
        uint64_t sums_off = 0;
        const uint64_t flen[NF] = {0, 1, 4u << 20, (4u << 20) + 1, L};
        for (int i = 0; i < NF; ++i) {
            snprintf(path[i], sizeof path[i], "%s/bind_%d", dir, i);
            FILE* f = fopen(path[i], "wb");
            CHECK(f != NULL, "create %s", path[i]);
            if (!f) return 1;
            if (flen[i]) fwrite(blob, 1, flen[i], f);
            fclose(f);
            fb[i].path = path[i];
            fb[i].length = flen[i];
            fb[i].piece_length = (int64_t)P;
            fb[i].sums_offset = sums_off;
            sums_off += krk_num_pieces(flen[i], (int64_t)P);
        }
        uint32_t* all = calloc(sums_off + 1, 4);
        uint32_t* all2 = calloc(sums_off + 1, 4);
        uint8_t dg[NF * 32];
        CHECK(krk_metainfo_digest_files_multi(fb, NF, all, dg) == KRK_OK, "metainfo_digest_files_multi");
        CHECK(krk_piece_sums_files(fb, NF, all2) == KRK_OK, "piece_sums_files");
        for (int i = 0; i < NF; ++i) {
            uint8_t want[32];
            orc_sha256(blob, flen[i], want);
            CHECK(memcmp(dg + 32 * i, want, 32) == 0, "file digest %d", i);
            const uint64_t np = krk_num_pieces(flen[i], (int64_t)P);
            for (uint64_t k = 0; k < np; ++k) {
                const uint64_t m = flen[i] - k * P < P ? flen[i] - k * P : P;
                const uint32_t c = host_crc(0, blob + k * P, m);
                CHECK(all[fb[i].sums_offset + k] == c && all2[fb[i].sums_offset + k] == c, "file %d piece %llu", i,
                      (unsigned long long)k);
            }
        }
        fb[2].length += 7; /* the stat said more than the file holds */
        CHECK(krk_metainfo_digest_files(fb, NF, all, dg) == KRK_EIO, "short file");
        CHECK(strstr(krk_last_error(), "read blob: ") && strstr(krk_last_error(), "unexpected EOF"), "EOF text");
        free(all);
        free(all2);
    }
    /* Generate over pinned receive buffers: 48 page-locked blobs in windows of <= 64 chunks
     * go up straight from the caller's pages (one DMA a chunk, no staging copy) */
    {
        enum { NB = 48 };
        void* pc[NB];
        krk_blob bl[NB];
        uint64_t so = 0;
        for (int i = 0; i < NB; ++i) {
            const uint64_t len = (1u << 20) + (uint64_t)i * 4097;
            CHECK(krk_host_alloc(len, &pc[i]) == KRK_OK, "host_alloc");
            memcpy(pc[i], blob + i * 977, len);
            bl[i].data = (const uint8_t*)pc[i];
            bl[i].length = len;
            bl[i].piece_length = 1 << 20;
            bl[i].sums_offset = so;
            so += krk_num_pieces(len, 1 << 20);
        }
        uint32_t* sums = calloc(so, 4);
        uint8_t* dg = malloc(32 * NB);
        CHECK(krk_set_sha_host_offload(0) == KRK_OK, "offload off"); /* every blob through the windows */
        CHECK(krk_metainfo_digest_host(bl, NB, sums, dg) == KRK_OK, "metainfo_digest_host (pinned)");
        CHECK(krk_set_sha_host_offload(KRK_OFFLOAD_AUTO) == KRK_OK, "offload default");
        int windows = 0, direct = 0;
        CHECK(krk_windows_last_call(NULL, &windows, NULL) == KRK_OK && krk_windows_last_direct(&direct) == KRK_OK &&
                  windows >= 1 && direct == windows,
              "direct windows %d of %d", direct, windows);
        for (int i = 0; i < NB; ++i) {
            uint8_t want[32];
            orc_sha256(bl[i].data, bl[i].length, want);
            CHECK(memcmp(dg + 32 * i, want, 32) == 0, "pinned digest %d", i);
            CHECK(sums[bl[i].sums_offset] == host_crc(0, bl[i].data, 1 << 20), "pinned piece %d", i);
            CHECK(sums[bl[i].sums_offset + 1] == host_crc(0, bl[i].data + (1 << 20), bl[i].length - (1 << 20)) ||
                      bl[i].length == (1u << 20),
                  "pinned tail piece %d", i);
        }
        for (int i = 0; i < NB; ++i) krk_host_free(pc[i]);
        free(sums);
        free(dg);
    }
    /* core/digester_krkgpu.go: AUTO digester, io.Copy-sized writes, Digest() without reset */
    {
        krk_digester* d = NULL;
        CHECK(krk_digester_new(&d) == KRK_OK, "digester_new");
        CHECK(krk_digester_write(d, blob, 32768) == KRK_OK, "write");
        uint8_t a[32], b[32], w[32];
        CHECK(krk_digester_sum(d, a) == KRK_OK, "sum");
        orc_sha256(blob, 32768, w);
        CHECK(memcmp(a, w, 32) == 0, "digest");
        CHECK(krk_digester_write(d, blob + 32768, L - 32768) == KRK_OK, "write after Digest()");
        CHECK(krk_digester_sum(d, b) == KRK_OK, "sum 2");
        orc_sha256(blob, L, w);
        CHECK(memcmp(b, w, 32) == 0, "digest continues");
        krk_digester_free(d);
    }
    /* hashring buildOwnerTable: 65,536 owner lists in one call */
    {
        const char* labels = "origin-000.kraken.test:15002origin-001.kraken.test:15002origin-002.kraken.test:15002";
        const uint64_t loff[4] = {0, 28, 56, 84};
        const int64_t w[3] = {100, 100, 100};
        const uint8_t healthy[3] = {1, 1, 0};
        krk_nodes nodes = {labels, loff, w, 3};
        int32_t* locs = malloc(65536 * 2 * sizeof(int32_t));
        uint8_t* counts = malloc(65536);
        CHECK(krk_ring_owner_table(&nodes, healthy, 2, locs, counts) == KRK_OK, "owner table");
        for (int r = 0; r < 65536; r += 4099) {
            CHECK(counts[r] >= 1 && counts[r] <= 2, "row %d count", r);
            for (int k = 0; k < counts[r]; ++k) CHECK(locs[2 * r + k] != 2, "unhealthy node listed");
        }
        free(locs);
        free(counts);
    }
    free(blob);
    CHECK(krk_shutdown() == KRK_OK, "shutdown");
    printf("{\"bindings_ok\": %s, \"failures\": %d}\n", fails ? "false" : "true", fails);
    return fails ? 1 : 0;
}
