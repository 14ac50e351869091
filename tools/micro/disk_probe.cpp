// disk_probe.cpp -- how the GPU box's scratch disk reads cold files, for the files leg's
// read pattern (cold files).  No GPU.
//
//   disk_probe <dir> <GiB> [files_MiB]
//
// Writes <GiB> of distinct files of about files_MiB each (default 9) under <dir>, then for
// every pattern drops the page cache of every file (POSIX_FADV_DONTNEED) and times one pass:
//   whole     T threads, each takes the next file and reads it front to back in S-byte preads
//             (the bench's disk_read leg at T=16, S=8 MiB);
//   windows   the library's schedule: every file live, a "window" of W bytes holds one chunk of
//             W/live bytes of each, T threads split the window's chunks and all of them finish
//             before the next window starts (par_read's barrier);
//   windows+  the same with the next window's chunks handed to the kernel as WILLNEED on a
//             helper thread while this window is read;
//   stream    the same chunks, no barrier: T threads take chunks (window order) one by one.
// One JSON line per pattern.
#include <fcntl.h>
#include <linux/aio_abi.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <functional>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct File {
    std::string path;
    uint64_t len;
    int fd;
};

static void drop(std::vector<File>& fs) {
    for (auto& f : fs) {
        int fd = open(f.path.c_str(), O_RDONLY);
        if (fd < 0) continue;
        fdatasync(fd);
        posix_fadvise(fd, 0, 0, POSIX_FADV_DONTNEED);
        close(fd);
    }
}

static void open_all(std::vector<File>& fs) {
    for (auto& f : fs) f.fd = open(f.path.c_str(), O_RDONLY | O_CLOEXEC);
}
static void close_all(std::vector<File>& fs) {
    for (auto& f : fs) close(f.fd);
}

struct Chunk {
    int fd;
    uint64_t off, len;
};

static void run_threads(int T, const std::function<void(int)>& f) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(f, t);
    for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: disk_probe <dir> <GiB> [file_MiB]\n");
        return 2;
    }
    const std::string dir = argv[1];
    const uint64_t total = (uint64_t)(atof(argv[2]) * (1ull << 30));
    const uint64_t fmb = argc > 3 ? strtoull(argv[3], nullptr, 10) : 9;
    std::vector<File> fs;
    {
        std::vector<uint8_t> buf(fmb << 20);
        uint64_t x = 0x9E3779B97F4A7C15ull, got = 0;
        const double t0 = now();
        for (int i = 0; got < total; ++i) {
            const uint64_t len = ((fmb << 20) - (uint64_t)(i % 7) * 4096 * 37);
            for (size_t k = 0; k + 8 <= len; k += 8) {
                x ^= x << 13, x ^= x >> 7, x ^= x << 17;
                memcpy(&buf[k], &x, 8);
            }
            File f{dir + "/d" + std::to_string(i), len, -1};
            int fd = open(f.path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
            if (fd < 0) {
                perror("open");
                return 1;
            }
            for (uint64_t o = 0; o < len;) {
                ssize_t w = write(fd, buf.data() + o, len - o);
                if (w <= 0) {
                    perror("write");
                    return 1;
                }
                o += (uint64_t)w;
            }
            fsync(fd);
            close(fd);
            fs.push_back(f);
            got += len;
        }
        fprintf(stderr, "wrote %zu files, %.1f GiB in %.1f s\n", fs.size(), got / double(1ull << 30), now() - t0);
    }
    uint64_t bytes = 0;
    for (auto& f : fs) bytes += f.len;
    const uint64_t maxlen = fmb << 20;

    auto report = [&](const char* pat, int T, uint64_t S, double s, const char* extra) {
        printf("{\"pattern\": \"%s\", \"threads\": %d, \"request_KiB\": %llu, \"GBps\": %.3f, \"seconds\": %.3f%s}\n", pat,
               T, (unsigned long long)(S >> 10), bytes / s / 1e9, s, extra);
        fflush(stdout);
    };

    // whole-file sequential reads
    for (int T : {16, 32, 64})
        for (uint64_t S : {128ull << 10, 1ull << 20, 8ull << 20}) {
            drop(fs);
            std::atomic<size_t> next{0};
            const double t0 = now();
            run_threads(T, [&](int) {
                std::vector<uint8_t> b(S);
                for (size_t i; (i = next.fetch_add(1)) < fs.size();) {
                    int fd = open(fs[i].path.c_str(), O_RDONLY);
                    for (uint64_t o = 0; o < fs[i].len;) {
                        ssize_t r = pread(fd, b.data(), std::min<uint64_t>(S, fs[i].len - o), (off_t)o);
                        if (r <= 0) break;
                        o += (uint64_t)r;
                    }
                    close(fd);
                }
            });
            report("whole", T, S, now() - t0, "");
        }

    // the window schedule: every file live, one chunk of W/live bytes a file a window
    const uint64_t W = 512ull << 20;
    for (int mode = 0; mode < 3; ++mode)
        for (int T : {16, 32, 64}) {
            drop(fs);
            open_all(fs);
            const uint64_t c = std::max<uint64_t>(4096, W / fs.size() / 4096 * 4096);
            std::vector<std::vector<Chunk>> wins;
            for (uint64_t off = 0; off < maxlen; off += c) {
                std::vector<Chunk> w;
                for (auto& f : fs)
                    if (off < f.len) w.push_back({f.fd, off, std::min(c, f.len - off)});
                wins.push_back(std::move(w));
            }
            std::vector<uint8_t> win(W + (64ull << 20));
            const double t0 = now();
            if (mode == 2) {  // stream: no barrier
                std::vector<Chunk> all;
                for (auto& w : wins) all.insert(all.end(), w.begin(), w.end());
                std::atomic<size_t> next{0};
                run_threads(T, [&](int t) {
                    uint8_t* dst = win.data() + (uint64_t)t * (c + 4096) % W;
                    for (size_t i; (i = next.fetch_add(1)) < all.size();) {
                        const Chunk& k = all[i];
                        if (pread(k.fd, dst, k.len, (off_t)k.off) <= 0) break;
                    }
                });
            } else {
                for (size_t wi = 0; wi < wins.size(); ++wi) {
                    std::thread hint;
                    if (mode == 1 && wi + 1 < wins.size())
                        hint = std::thread([&, wi] {
                            for (const Chunk& k : wins[wi + 1])
                                posix_fadvise(k.fd, (off_t)k.off, (off_t)k.len, POSIX_FADV_WILLNEED);
                        });
                    const auto& w = wins[wi];
                    std::atomic<size_t> next{0};
                    run_threads(T, [&](int) {
                        for (size_t i; (i = next.fetch_add(1)) < w.size();) {
                            const Chunk& k = w[i];
                            if (pread(k.fd, win.data() + i * c % W, k.len, (off_t)k.off) <= 0) break;
                        }
                    });
                    if (hint.joinable()) hint.join();
                }
            }
            char extra[96];
            snprintf(extra, sizeof extra, ", \"live\": %zu, \"windows\": %zu", fs.size(), wins.size());
            report(mode == 0 ? "windows" : mode == 1 ? "windows+willneed_next" : "stream", T, c, now() - t0, extra);
            close_all(fs);
        }
    // the window schedule with the library's per-file readahead marks (staging.hpp par_read):
    // each file kept hinted R bytes past its reads, R bytes a WILLNEED
    for (uint64_t R : {2ull << 20, 8ull << 20})
        for (int barrier = 1; barrier >= 0; --barrier) {
            const int T = 16;
            drop(fs);
            open_all(fs);
            const uint64_t c = std::max<uint64_t>(4096, W / fs.size() / 4096 * 4096);
            std::vector<std::vector<size_t>> wins;  // file index per chunk
            for (uint64_t off = 0; off < maxlen; off += c) {
                std::vector<size_t> w;
                for (size_t i = 0; i < fs.size(); ++i)
                    if (off < fs[i].len) w.push_back(i);
                wins.push_back(std::move(w));
            }
            std::vector<uint64_t> mark(fs.size(), 0);
            std::vector<uint8_t> win(W + (64ull << 20));
            auto read_chunk = [&](size_t f, uint64_t off, uint8_t* dst) {
                const uint64_t len = std::min(c, fs[f].len - off);
                const uint64_t want = std::min(fs[f].len, off + len + R);
                while (mark[f] < want) {  // one thread a file a window: no race
                    const uint64_t to = std::min(fs[f].len, mark[f] + R);
                    posix_fadvise(fs[f].fd, (off_t)mark[f], (off_t)(to - mark[f]), POSIX_FADV_WILLNEED);
                    mark[f] = to;
                }
                return pread(fs[f].fd, dst, len, (off_t)off) > 0;
            };
            const double t0 = now();
            if (barrier) {
                for (size_t wi = 0; wi < wins.size(); ++wi) {
                    std::atomic<size_t> next{0};
                    run_threads(T, [&](int) {
                        for (size_t i; (i = next.fetch_add(1)) < wins[wi].size();)
                            if (!read_chunk(wins[wi][i], wi * c, win.data() + i * c % W)) break;
                    });
                }
            } else {
                std::vector<std::pair<size_t, uint64_t>> all;
                for (size_t wi = 0; wi < wins.size(); ++wi)
                    for (size_t f : wins[wi]) all.push_back({f, wi * c});
                std::atomic<size_t> next{0};
                run_threads(T, [&](int t) {
                    uint8_t* dst = win.data() + (uint64_t)t * (c + 4096) % W;
                    for (size_t i; (i = next.fetch_add(1)) < all.size();)
                        if (!read_chunk(all[i].first, all[i].second, dst)) break;
                });
            }
            char extra[128];
            snprintf(extra, sizeof extra, ", \"live\": %zu, \"windows\": %zu, \"readahead_MiB\": %llu", fs.size(),
                     wins.size(), (unsigned long long)(R >> 20));
            report(barrier ? "windows+readahead" : "stream+readahead", T, c, now() - t0, extra);
            close_all(fs);
        }
    // Linux AIO over O_DIRECT: one thread submits every chunk of a window (io_submit, up to
    // QD in flight) and reaps them (io_getevents) -- the disk sees a deep queue without a
    // thread per request.  The window barrier stays (the library's windows).
    for (int qd : {256, 1024, 4096}) {
        drop(fs);
        std::vector<int> dfd(fs.size());
        for (size_t i = 0; i < fs.size(); ++i) dfd[i] = open(fs[i].path.c_str(), O_RDONLY | O_DIRECT | O_CLOEXEC);
        const uint64_t c = std::max<uint64_t>(4096, W / fs.size() / 4096 * 4096);
        void* wbuf = nullptr;
        if (posix_memalign(&wbuf, 4096, W + (64ull << 20))) return 1;
        aio_context_t ctx = 0;
        if (syscall(SYS_io_setup, qd, &ctx) != 0) {
            perror("io_setup");
            return 1;
        }
        std::vector<iocb> cbs(qd);
        std::vector<iocb*> ptrs(qd);
        std::vector<io_event> ev(qd);
        uint64_t bad = 0;
        const double t0 = now();
        for (uint64_t off = 0; off < maxlen; off += c) {
            std::vector<std::pair<int, uint64_t>> todo;  // (file, len) of this window
            for (size_t i = 0; i < fs.size(); ++i)
                if (off < fs[i].len) todo.push_back({(int)i, std::min(c, fs[i].len - off)});
            size_t next = 0, inflight = 0;
            std::vector<int> free_slot;
            for (int q = 0; q < qd; ++q) free_slot.push_back(q);
            while (next < todo.size() || inflight) {
                int nsub = 0;
                while (next < todo.size() && !free_slot.empty()) {
                    const int q = free_slot.back();
                    free_slot.pop_back();
                    iocb& cb = cbs[q];
                    memset(&cb, 0, sizeof cb);
                    cb.aio_data = (uint64_t)q;
                    cb.aio_lio_opcode = IOCB_CMD_PREAD;
                    cb.aio_fildes = (uint32_t)dfd[todo[next].first];
                    cb.aio_buf = (uint64_t)((uint8_t*)wbuf + (next * c) % W);
                    cb.aio_nbytes = (todo[next].second + 4095) & ~4095ull;
                    cb.aio_offset = (int64_t)off;
                    ptrs[nsub++] = &cb;
                    ++next;
                }
                if (nsub) {
                    const long r = syscall(SYS_io_submit, ctx, nsub, ptrs.data());
                    if (r != nsub) {
                        perror("io_submit");
                        return 1;
                    }
                    inflight += (size_t)nsub;
                }
                const long got = syscall(SYS_io_getevents, ctx, 1, qd, ev.data(), nullptr);
                if (got < 0) {
                    perror("io_getevents");
                    return 1;
                }
                for (long e = 0; e < got; ++e) {
                    if (ev[e].res <= 0) ++bad;
                    free_slot.push_back((int)ev[e].data);
                }
                inflight -= (size_t)got;
            }
        }
        const double el = now() - t0;
        syscall(SYS_io_destroy, ctx);
        free(wbuf);
        for (int x : dfd) close(x);
        char extra[128];
        snprintf(extra, sizeof extra, ", \"live\": %zu, \"queue_depth\": %d, \"failed\": %llu", fs.size(), qd,
                 (unsigned long long)bad);
        report("aio_direct_windows", 1, c, el, extra);
    }
    for (auto& f : fs) unlink(f.path.c_str());
    return 0;
}
