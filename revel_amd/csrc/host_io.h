// host_io.h -- host-side helpers shared by the replay paths (replay.cpp,
// shard.cpp): NUMA placement next to a GPU, parallel window fills and the
// release of consumed file-mapping ranges.
#pragma once
#include <ctype.h>
#include <hip/hip_runtime_api.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

namespace revel {

// NUMA placement: the pinned ring and the io threads go to the GPU's NUMA
// node (its PCI device's numa_node in sysfs), so the H2D DMA reads local
// memory and the fill threads write it locally -- on a two-socket host with a
// replay per GPU this keeps each GPU's traffic on its own socket.  The calling
// thread is bound to that node's CPUs (within the process's own affinity) for
// the replay; the io threads inherit the binding.  Unknown topology: no-op.
class NodeBinding {
   public:
    explicit NodeBinding(int device) {
        char bus[64] = {0};
        if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) return;
        for (char* c = bus; *c; ++c) *c = (char)tolower((unsigned char)*c);
        char path[160];
        snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
        const int node = read_int(path);
        if (node < 0) return;
        snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
        cpu_set_t want;
        if (!read_cpulist(path, &want)) return;
        if (sched_getaffinity(0, sizeof saved_, &saved_) != 0) return;
        CPU_AND(&want, &want, &saved_);
        if (CPU_COUNT(&want) == 0) return;
        active_ = sched_setaffinity(0, sizeof want, &want) == 0;
    }
    ~NodeBinding() {
        if (active_) (void)sched_setaffinity(0, sizeof saved_, &saved_);
    }
    NodeBinding(const NodeBinding&) = delete;
    NodeBinding& operator=(const NodeBinding&) = delete;

   private:
    static int read_int(const char* path) {
        FILE* f = fopen(path, "r");
        if (!f) return -1;
        int v = -1;
        if (fscanf(f, "%d", &v) != 1) v = -1;
        fclose(f);
        return v;
    }
    // "0-63,128-191"
    static bool read_cpulist(const char* path, cpu_set_t* set) {
        FILE* f = fopen(path, "r");
        if (!f) return false;
        char buf[1024] = {0};
        const bool got = fgets(buf, sizeof buf, f) != nullptr;
        fclose(f);
        if (!got) return false;
        CPU_ZERO(set);
        for (char* p = buf; *p && *p != '\n';) {
            char* e;
            long a = strtol(p, &e, 10);
            if (e == p) return false;
            long b = a;
            if (*e == '-') {
                p = e + 1;
                b = strtol(p, &e, 10);
                if (e == p) return false;
            }
            for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET((int)c, set);
            p = *e == ',' ? e + 1 : e;
        }
        return CPU_COUNT(set) > 0;
    }
    cpu_set_t saved_;
    bool active_ = false;
};

// Drop the page-table entries of the whole pages inside [p, p + n) of a
// read-only file mapping once a fill thread has copied them out (the pages
// stay in the page cache; a later access would fault them back in).  A window
// at a time, on the fill threads beside the PCIe-bound copy, instead of one
// munmap of the whole mapping at the end: for C5's 100 GiB file that final
// teardown took ~1.1 s of the call on the GPU box (~26 M PTEs), 32 of 51 GiB/s.
inline void release_mapped(const void* p, uint64_t n) {
    static const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
    const uintptr_t a = ((uintptr_t)p + pg - 1) & ~(pg - 1), b = ((uintptr_t)p + n) & ~(pg - 1);
    if (b > a) (void)::madvise(reinterpret_cast<void*>(a), b - a, MADV_DONTNEED);
}

// Fill dst[0..len) from the source with up to `threads` parallel workers.
template <typename F>
inline double parallel_fill(int threads, uint64_t len, F&& part) {
    auto t0 = std::chrono::steady_clock::now();
    // 64 KiB-aligned pieces (O_DIRECT needs page-aligned offsets and sizes)
    const uint64_t per = (len + threads - 1) / threads;
    const uint64_t chunk = std::max<uint64_t>(1 << 20, (per + 65535) / 65536 * 65536);
    std::vector<std::thread> pool;
    for (uint64_t off = 0; off < len; off += chunk) {
        const uint64_t n = std::min(chunk, len - off);
        if (off + n >= len) {
            part(off, n);  // the calling thread takes the last piece
        } else {
            pool.emplace_back([&part, off, n] { part(off, n); });
        }
    }
    for (auto& t : pool) t.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace revel
