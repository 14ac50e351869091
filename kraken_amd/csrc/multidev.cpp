// multidev.cpp -- one process driving several GPUs.
//
// The reference's origin is ONE process with one metainfo generator
// (origin/cmd/cmd.go:164), fed by blobrefresh (lib/blobrefresh/refresher.go:116) and
// upload commits; through the C ABI it must be able to spread a batch over every GPU
// of the node.  The path shards by blob with no exchange step, so the multi-device
// entry points split a batch greedily by bytes (LPT: longest blob to the lightest
// device), run the single-device entry point on each device from its own host
// thread, and gather the per-blob results (piece sums, digests) into the caller's
// arrays on the host.  No collective, no peer traffic.
//
// The process's device set (krk_set_devices, or the devices of krk_init's mask)
// also spreads new Digesters / piece streams over the devices round-robin.  A device
// may appear more than once: two workers then share one GPU (their host copies and
// H2D overlap), which is also how the multi-device path is tested on a one-GPU box.
#include <queue>
#include <thread>

#include "runtime.hpp"

namespace krk {

namespace {
std::mutex g_set_mu;
std::vector<int> g_set;  // empty: the calling thread's device
std::atomic<uint32_t> g_rr{0};

std::vector<int> device_set() {
    std::lock_guard<std::mutex> g(g_set_mu);
    if (g_set.empty()) return {t_dev};
    return g_set;
}

// Blob indices per worker: LPT on bytes (ties in index order, so the split is deterministic).
std::vector<std::vector<uint64_t>> lpt(const std::vector<uint64_t>& bytes, size_t workers) {
    std::vector<uint64_t> order(bytes.size());
    for (uint64_t i = 0; i < order.size(); ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return bytes[a] > bytes[b]; });
    using Load = std::pair<uint64_t, size_t>;
    std::priority_queue<Load, std::vector<Load>, std::greater<Load>> heap;
    for (size_t w = 0; w < workers; ++w) heap.push({0, w});
    std::vector<std::vector<uint64_t>> out(workers);
    for (uint64_t i : order) {
        Load l = heap.top();
        heap.pop();
        out[l.second].push_back(i);
        heap.push({l.first + bytes[i], l.second});
    }
    for (auto& v : out) std::sort(v.begin(), v.end());
    return out;
}

// Run part(worker, indices) for every worker of the device set, each on its own host
// thread with that worker's device current; the first failure's status and message
// are returned on the calling thread.
template <class F>
int shard_run(const std::vector<uint64_t>& bytes, F&& part) {
    const std::vector<int> devs = device_set();
    const auto idx = lpt(bytes, devs.size());
    std::vector<int> rc(devs.size(), KRK_OK);
    std::vector<std::string> msg(devs.size());
    const int share = std::max(1, host_cpu_budget() / (int)std::max<size_t>(1, devs.size()));
    auto work = [&](size_t w) {
        if (idx[w].empty()) return;
        const int saved = t_dev, saved_share = t_host_share;
        t_dev = devs[w];
        t_host_share = share;  // this worker's share of the host threads
        rc[w] = part(w, idx[w]);
        if (rc[w]) msg[w] = t_err;
        t_dev = saved;
        t_host_share = saved_share;
    };
    std::vector<std::thread> th;
    for (size_t w = 1; w < devs.size(); ++w) th.emplace_back(work, w);
    work(0);
    for (auto& t : th) t.join();
    for (size_t w = 0; w < devs.size(); ++w)
        if (rc[w]) {
            t_err = msg[w];
            return rc[w];
        }
    return KRK_OK;
}

// A worker's blobs with their sums re-based into a private array (the single-device
// entry points copy whole sums spans back, which must not touch other workers' sums).
template <class B>
struct SubBatch {
    std::vector<B> blobs;
    std::vector<uint32_t> sums;
    std::vector<uint64_t> n_sums;
    SubBatch(const B* all, const std::vector<uint64_t>& idx) {
        uint64_t off = 0;
        for (uint64_t i : idx) {
            B b = all[i];
            b.sums_offset = off;
            const uint64_t np = krk_num_pieces(b.length, b.piece_length);
            n_sums.push_back(np);
            off += np;
            blobs.push_back(b);
        }
        sums.assign(std::max<uint64_t>(off, 1), 0);
    }
    void scatter(const B* all, const std::vector<uint64_t>& idx, uint32_t* sums_host) const {
        for (size_t k = 0; k < idx.size(); ++k)
            if (n_sums[k]) memcpy(sums_host + all[idx[k]].sums_offset, sums.data() + blobs[k].sums_offset, n_sums[k] * 4);
    }
};

template <class B>
int check_batch(const B* blobs, uint64_t n) {
    KRK_CHECK(n == 0 || blobs, KRK_EINVAL, "blobs is NULL");
    for (uint64_t i = 0; i < n; ++i)
        KRK_CHECK(blobs[i].piece_length > 0, KRK_EINVAL, "piece length must be positive");
    return KRK_OK;
}
}  // namespace

int place_device() {
    std::lock_guard<std::mutex> g(g_set_mu);
    if (g_set.empty()) return t_dev;
    return g_set[g_rr.fetch_add(1, std::memory_order_relaxed) % g_set.size()];
}

void set_device_set_from_mask(uint64_t mask) {
    std::vector<int> v;
    for (int i = 0; i < 64; ++i)
        if ((mask >> i) & 1) v.push_back(i);
    std::lock_guard<std::mutex> g(g_set_mu);
    g_set = v;
}

}  // namespace krk

using namespace krk;

extern "C" {

int krk_set_devices(const int* devs, uint32_t n) {
    KRK_CHECK(n == 0 || devs, KRK_EINVAL, "devs is NULL");
    KRK_CHECK(n <= 256, KRK_EINVAL, "more than 256 workers");
    const int saved = t_dev;
    for (uint32_t i = 0; i < n; ++i) {  // every listed device must be a usable gfx950 context
        int rc = KRK_OK;
        if (!device_id(devs[i], &rc)) {
            t_dev = saved;
            return rc;
        }
    }
    int rc = KRK_OK;
    device_id(saved, &rc);  // the calling thread's current device is unchanged
    std::lock_guard<std::mutex> g(g_set_mu);
    g_set.assign(devs, devs + n);
    return KRK_OK;
}

int krk_get_devices(int* devs, uint32_t cap, uint32_t* n) {
    KRK_CHECK(n, KRK_EINVAL, "n is NULL");
    const std::vector<int> v = device_set();
    *n = (uint32_t)v.size();
    KRK_CHECK(!devs || cap >= v.size(), KRK_ERANGE, "device set has %zu entries, capacity %u", v.size(), cap);
    if (devs) std::copy(v.begin(), v.end(), devs);
    return KRK_OK;
}

int krk_metainfo_digest_host_multi(const krk_blob* blobs, uint64_t n, uint32_t* sums_host, uint8_t* digests_host) {
    int r = check_batch(blobs, n);
    if (r || !n) return r;
    KRK_CHECK(digests_host, KRK_EINVAL, "digests_host is NULL");
    std::vector<uint64_t> bytes(n);
    bool any_sums = false;
    for (uint64_t i = 0; i < n; ++i) {
        bytes[i] = blobs[i].length;
        any_sums |= blobs[i].length > 0;
    }
    KRK_CHECK(!any_sums || sums_host, KRK_EINVAL, "sums_host is NULL");
    return shard_run(bytes, [&](size_t, const std::vector<uint64_t>& idx) {
        SubBatch<krk_blob> sb(blobs, idx);
        std::vector<uint8_t> dg(idx.size() * 32);
        int rc = krk_metainfo_digest_host(sb.blobs.data(), idx.size(), sb.sums.data(), dg.data());
        if (rc) return rc;
        sb.scatter(blobs, idx, sums_host);
        for (size_t k = 0; k < idx.size(); ++k) memcpy(digests_host + 32 * idx[k], dg.data() + 32 * k, 32);
        return KRK_OK;
    });
}

int krk_piece_sums_host_multi(const krk_blob* blobs, uint64_t n, uint32_t* sums_host) {
    int r = check_batch(blobs, n);
    if (r || !n) return r;
    std::vector<uint64_t> bytes(n);
    for (uint64_t i = 0; i < n; ++i) bytes[i] = blobs[i].length;
    KRK_CHECK(sums_host, KRK_EINVAL, "sums_host is NULL");
    return shard_run(bytes, [&](size_t, const std::vector<uint64_t>& idx) {
        SubBatch<krk_blob> sb(blobs, idx);
        int rc = krk_piece_sums_host(sb.blobs.data(), idx.size(), sb.sums.data());
        if (!rc) sb.scatter(blobs, idx, sums_host);
        return rc;
    });
}

int krk_piece_sums_files_multi(const krk_file_blob* files, uint64_t n, uint32_t* sums_host) {
    int r = check_batch(files, n);
    if (r || !n) return r;
    KRK_CHECK(sums_host, KRK_EINVAL, "sums_host is NULL");
    int prc = KRK_OK;  // host placement: one pass on the host pool, nothing to shard
    const int where = resolve_crc_placement(KRK_PLACE_AUTO, &prc);
    if (where < 0) return prc;
    if (where != KRK_PLACE_GPU) return krk_piece_sums_files(files, n, sums_host);
    std::vector<uint64_t> bytes(n);
    for (uint64_t i = 0; i < n; ++i) bytes[i] = files[i].length;
    return shard_run(bytes, [&](size_t, const std::vector<uint64_t>& idx) {
        SubBatch<krk_file_blob> sb(files, idx);
        int rc = krk_piece_sums_files(sb.blobs.data(), idx.size(), sb.sums.data());
        if (!rc) sb.scatter(files, idx, sums_host);
        return rc;
    });
}

int krk_metainfo_digest_files_multi(const krk_file_blob* files, uint64_t n, uint32_t* sums_host,
                                    uint8_t* digests_host) {
    int r = check_batch(files, n);
    if (r || !n) return r;
    KRK_CHECK(digests_host, KRK_EINVAL, "digests_host is NULL");
    std::vector<uint64_t> bytes(n);
    bool any_sums = false;
    for (uint64_t i = 0; i < n; ++i) {
        bytes[i] = files[i].length;
        any_sums |= files[i].length > 0;
    }
    KRK_CHECK(!any_sums || sums_host, KRK_EINVAL, "sums_host is NULL");
    return shard_run(bytes, [&](size_t, const std::vector<uint64_t>& idx) {
        SubBatch<krk_file_blob> sb(files, idx);
        std::vector<uint8_t> dg(idx.size() * 32);
        int rc = krk_metainfo_digest_files(sb.blobs.data(), idx.size(), sb.sums.data(), dg.data());
        if (rc) return rc;
        sb.scatter(files, idx, sums_host);
        for (size_t k = 0; k < idx.size(); ++k) memcpy(digests_host + 32 * idx[k], dg.data() + 32 * k, 32);
        return KRK_OK;
    });
}

int krk_sha256_host_multi(const uint8_t* const* data_host, const uint64_t* lengths, uint64_t n,
                          uint8_t* digests_host) {
    if (!n) return KRK_OK;
    KRK_CHECK(data_host && lengths && digests_host, KRK_EINVAL, "sha256_host_multi: null argument");
    std::vector<uint64_t> bytes(lengths, lengths + n);
    return shard_run(bytes, [&](size_t, const std::vector<uint64_t>& idx) {
        std::vector<const uint8_t*> d;
        std::vector<uint64_t> l;
        for (uint64_t i : idx) {
            d.push_back(data_host[i]);
            l.push_back(lengths[i]);
        }
        std::vector<uint8_t> dg(idx.size() * 32);
        int rc = krk_sha256_host(d.data(), l.data(), idx.size(), dg.data());
        if (rc) return rc;
        for (size_t k = 0; k < idx.size(); ++k) memcpy(digests_host + 32 * idx[k], dg.data() + 32 * k, 32);
        return KRK_OK;
    });
}

}  // extern "C"
