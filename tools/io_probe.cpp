// io_probe.cpp -- host input-path measurements for config C5 (§8(f) rank 4):
// which way of moving a WAL file's bytes into HBM is fastest on the box.
//   pread      : T threads pread() into pinned (hipHostMalloc) or pageable memory
//   mmap+copy  : T threads memcpy from a MAP_SHARED mapping into pinned memory
//   mmap+reg   : hipHostRegister a window of the mapping, DMA it straight to HBM
//   odirect    : O_DIRECT pread (fails with EINVAL on tmpfs)
// Build: hipcc -O2 -std=c++17 tools/io_probe.cpp -o build/io_probe -pthread
// Usage: io_probe <file> <GiB> [tests...]   (creates/extends the file first)
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <functional>
#include <string>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define HIPCHECK(x)                                                                  \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            exit(3);                                                                 \
        }                                                                            \
    } while (0)

static void parallel(int T, uint64_t len, const std::function<void(uint64_t, uint64_t)>& f) {
    std::vector<std::thread> th;
    const uint64_t chunk = (len + T - 1) / T;
    for (int t = 0; t < T; ++t) {
        uint64_t o = t * chunk;
        if (o >= len) break;
        uint64_t n = std::min(chunk, len - o);
        th.emplace_back([&f, o, n] { f(o, n); });
    }
    for (auto& x : th) x.join();
}

static void make_file(const char* path, uint64_t size) {
    struct stat st;
    if (stat(path, &st) == 0 && (uint64_t)st.st_size == size) return;
    int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) { perror("open for write"); exit(2); }
    double t0 = now();
    parallel(16, size, [&](uint64_t o, uint64_t n) {
        std::vector<uint64_t> buf(1 << 17);
        for (uint64_t d = 0; d < n; d += 1 << 20) {
            uint64_t m = std::min<uint64_t>(1 << 20, n - d);
            for (size_t i = 0; i < buf.size(); ++i) buf[i] = (o + d) * 0x9E3779B97F4A7C15ull + i;
            if (pwrite(fd, buf.data(), m, o + d) != (ssize_t)m) { perror("pwrite"); exit(2); }
        }
    });
    close(fd);
    printf("{\"make_file_GiB_s\": %.2f}\n", size / 1073741824.0 / (now() - t0));
    fflush(stdout);
}

int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: io_probe file GiB [tests]\n"); return 1; }
    const char* path = argv[1];
    const uint64_t size = (uint64_t)(atof(argv[2]) * 1073741824.0);
    std::vector<std::string> tests;
    for (int i = 3; i < argc; ++i) tests.push_back(argv[i]);
    if (tests.empty()) tests = {"pread", "mmap", "reg", "odirect"};
    make_file(path, size);
    const uint64_t W = 64ull << 20;
    const int NB = 4;
    uint8_t* pin[NB];
    for (int i = 0; i < NB; ++i) HIPCHECK(hipHostMalloc((void**)&pin[i], W, hipHostMallocDefault));
    void* d;
    HIPCHECK(hipMalloc(&d, 2 * W));
    auto report = [&](const char* name, int T, double secs, const char* extra = "") {
        printf("{\"test\": \"%s\", \"threads\": %d, \"GiB\": %.1f, \"GiB_s\": %.2f%s}\n", name, T, size / 1073741824.0,
               size / 1073741824.0 / secs, extra);
        fflush(stdout);
    };
    for (auto& t : tests) {
        if (t == "pread") {
            int fd = open(path, O_RDONLY);
            std::vector<uint8_t> pageable(W);
            memset(pageable.data(), 1, W);
            for (int pinned = 1; pinned >= 0; --pinned)
                for (int T : {1, 4, 8, 16, 32}) {
                    double t0 = now();
                    for (uint64_t off = 0, k = 0; off < size; off += W, ++k) {
                        uint8_t* dst = pinned ? pin[k % NB] : pageable.data();
                        uint64_t len = std::min(W, size - off);
                        parallel(T, len, [&](uint64_t o, uint64_t n) {
                            uint64_t done = 0;
                            while (done < n) {
                                ssize_t r = pread(fd, dst + o + done, n - done, off + o + done);
                                if (r <= 0) { perror("pread"); exit(2); }
                                done += r;
                            }
                        });
                    }
                    report(pinned ? "pread_to_pinned" : "pread_to_pageable", T, now() - t0);
                }
            close(fd);
        } else if (t == "mmap") {
            int fd = open(path, O_RDONLY);
            for (int populate = 0; populate <= 1; ++populate) {
                double t0 = now();
                uint8_t* m = (uint8_t*)mmap(nullptr, size, PROT_READ, MAP_SHARED | (populate ? MAP_POPULATE : 0), fd, 0);
                if (m == MAP_FAILED) { perror("mmap"); exit(2); }
                madvise(m, size, MADV_SEQUENTIAL);
                double tm = now() - t0;
                for (int pass = 0; pass < 2; ++pass)
                    for (int T : {8, 16}) {
                        double t1 = now();
                        for (uint64_t off = 0, k = 0; off < size; off += W, ++k) {
                            uint64_t len = std::min(W, size - off);
                            parallel(T, len, [&](uint64_t o, uint64_t n) { memcpy(pin[k % NB] + o, m + off + o, n); });
                        }
                        char extra[96];
                        snprintf(extra, sizeof extra, ", \"populate\": %d, \"pass\": %d, \"mmap_s\": %.3f", populate, pass, tm);
                        report("mmap_memcpy_to_pinned", T, now() - t1, extra);
                    }
                munmap(m, size);
            }
            close(fd);
        } else if (t == "reg") {
            int fd = open(path, O_RDONLY);
            uint8_t* m = (uint8_t*)mmap(nullptr, size, PROT_READ, MAP_SHARED, fd, 0);
            if (m == MAP_FAILED) { perror("mmap"); exit(2); }
            hipStream_t s;
            HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            for (uint64_t RW : {64ull << 20, 256ull << 20, 1024ull << 20}) {
                double treg = 0, t0 = now();
                bool failed = false;
                for (uint64_t off = 0; off < size; off += RW) {
                    uint64_t len = std::min(RW, size - off);
                    double a = now();
                    hipError_t e = hipHostRegister(m + off, len, hipHostRegisterReadOnly | hipHostRegisterMapped);
                    if (e != hipSuccess) {
                        printf("{\"test\": \"mmap_register\", \"error\": \"%s\"}\n", hipGetErrorString(e));
                        failed = true;
                        break;
                    }
                    treg += now() - a;
                    for (uint64_t c = 0; c < len; c += W)
                        HIPCHECK(hipMemcpyAsync((uint8_t*)d + (c / W % 2) * W, m + off + c, std::min(W, len - c),
                                                hipMemcpyHostToDevice, s));
                    HIPCHECK(hipStreamSynchronize(s));
                    HIPCHECK(hipHostUnregister(m + off));
                }
                if (failed) break;
                char extra[96];
                snprintf(extra, sizeof extra, ", \"window_MiB\": %llu, \"register_s\": %.3f", (unsigned long long)(RW >> 20),
                         treg);
                report("mmap_register_dma", 1, now() - t0, extra);
            }
            munmap(m, size);
            close(fd);
        } else if (t == "odirect") {
            int fd = open(path, O_RDONLY | O_DIRECT);
            if (fd < 0) {
                printf("{\"test\": \"odirect\", \"error\": \"%s\"}\n", strerror(errno));
                continue;
            }
            for (int T : {4, 16}) {
                double t0 = now();
                bool bad = false;
                for (uint64_t off = 0, k = 0; off < size && !bad; off += W, ++k) {
                    uint64_t len = std::min(W, size - off);
                    parallel(T, len, [&](uint64_t o, uint64_t n) {
                        ssize_t r = pread(fd, pin[k % NB] + o, n, off + o);
                        if (r != (ssize_t)n) bad = true;
                    });
                }
                if (bad) {
                    printf("{\"test\": \"odirect\", \"error\": \"%s\"}\n", strerror(errno));
                    break;
                }
                report("odirect_pread_to_pinned", T, now() - t0);
            }
            close(fd);
        }
    }
    return 0;
}
