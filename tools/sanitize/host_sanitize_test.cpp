// host_sanitize_test.cpp -- the host half of librevel_wal under
// AddressSanitizer + UndefinedBehaviorSanitizer (host code only; no GPU
// sanitizer exists on this pool).  Exercises every host-side C-ABI path:
// CRC, memory/posix files, the writer, the checksum=0 reader (host walk),
// initial_offset, framed-size layout, corruption, caller-implemented files
// (callbacks, short reads, release), the shard boundary walk + stitch, and
// the error returns of the GPU entry points without a device.  Built by tools/sanitize/Makefile;
// run by tests/test_sanitize.py.  Exit 0 = all checks passed, no reports.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "revel_wal.h"

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                         \
        }                                                                     \
    } while (0)

typedef std::vector<uint8_t> Bytes;

static Bytes write_image(const std::vector<Bytes>& recs, uint64_t boff) {
    revel_writable_file* f = revel_memory_writable_file_new();
    revel_log_writer* w = revel_log_writer_new(f, boff);
    for (const Bytes& r : recs) CHECK(revel_log_writer_add_record(w, r.data(), r.size()) == REVEL_OK);
    const uint8_t* p = nullptr;
    size_t n = 0;
    CHECK(revel_memory_writable_file_contents(f, &p, &n) == REVEL_OK);
    Bytes img(p, p + n);
    revel_log_writer_free(w);
    revel_writable_file_free(f);
    return img;
}

static std::vector<Bytes> read_all(const Bytes& img, uint64_t initial_offset, size_t window, int* err) {
    revel_sequential_file* s = revel_memory_sequential_file_new(img.data(), img.size());
    revel_log_reader* r = nullptr;
    std::vector<Bytes> out;
    *err = revel_log_reader_new(s, 0, initial_offset, nullptr, window, &r);
    if (*err) return out;
    for (;;) {
        const uint8_t* d = nullptr;
        size_t n = 0;
        int rc = revel_log_reader_read_record(r, &d, &n);
        if (rc != REVEL_OK) { *err = rc; continue; }  // the reader continues after an error
        if (!d) break;
        out.emplace_back(d, d + n);
    }
    revel_log_reader_free(r);
    return out;
}

// A caller's files behind the callback adapters (env.rs:40-57).
struct VecW {
    Bytes b;
    int flushes = 0, syncs = 0, closes = 0, released = 0;
    size_t fail_after = (size_t)-1;
};
static int vw_append(void* u, const uint8_t* d, size_t n) {
    auto* f = static_cast<VecW*>(u);
    if (f->b.size() + n > f->fail_after) return REVEL_IO_ERROR;
    f->b.insert(f->b.end(), d, d + n);
    return REVEL_OK;
}
static int vw_flush(void* u) { return ++static_cast<VecW*>(u)->flushes, REVEL_OK; }
static int vw_sync(void* u) { return ++static_cast<VecW*>(u)->syncs, REVEL_OK; }
static int vw_close(void* u) { return ++static_cast<VecW*>(u)->closes, 99; }  // out-of-range code -> IOError
static void vw_release(void* u) { ++static_cast<VecW*>(u)->released; }
struct VecR {
    const Bytes* b;
    size_t pos = 0, chunk = 1;
    int released = 0;
};
static int vr_read(void* u, uint8_t* p, size_t n, size_t* got) {
    auto* r = static_cast<VecR*>(u);
    size_t k = std::min(std::min(n, r->chunk), r->b->size() - std::min(r->pos, r->b->size()));
    if (k) memcpy(p, r->b->data() + r->pos, k);
    r->pos += k;
    *got = k;
    return REVEL_OK;
}
static void vr_release(void* u) { ++static_cast<VecR*>(u)->released; }

int main() {
    // ---- CRC known answers (crc.rs:50-76, RFC 3720 B.4) ----
    const char* digits = "123456789";
    CHECK(revel_crc32c_value((const uint8_t*)digits, 9) == 0xE3069283u);
    uint8_t buf[32];
    memset(buf, 0, 32);
    CHECK(revel_crc32c_value(buf, 32) == 0x8A9136AAu);
    memset(buf, 0xFF, 32);
    CHECK(revel_crc32c_value(buf, 32) == 0x62A8AB43u);
    for (int i = 0; i < 32; ++i) buf[i] = (uint8_t)i;
    CHECK(revel_crc32c_value(buf, 32) == 0x46DD794Eu);
    for (int i = 0; i < 32; ++i) buf[i] = (uint8_t)(31 - i);
    CHECK(revel_crc32c_value(buf, 32) == 0x113FDB5Cu);
    CHECK(revel_crc32c_value(nullptr, 0) == 0u);
    const char* hw = "hello world";
    CHECK(revel_crc32c_value((const uint8_t*)hw, 11) == revel_crc32c_extend('h', (const uint8_t*)hw + 1, 10));
    for (uint32_t c : {0u, 1u, 0xFFFFFFFFu, 0x12345678u}) CHECK(revel_crc32c_unmask(revel_crc32c_mask(c)) == c);

    // ---- writer + host-walk reader round trips ----
    std::mt19937_64 rng(7);
    for (uint64_t boff : {0ull, 1ull, 6ull, 7ull, 32760ull, 32761ull, 32767ull}) {
        std::vector<Bytes> recs;
        for (int i = 0; i < 60; ++i) {
            size_t len = (i % 7 == 0) ? 0 : rng() % (i % 5 == 0 ? 120000 : 3000);
            Bytes r(len);
            for (auto& b : r) b = (uint8_t)rng();
            recs.push_back(r);
        }
        Bytes img = write_image(recs, boff);
        std::vector<uint64_t> lens;
        for (auto& r : recs) lens.push_back(r.size());
        CHECK(revel_log_framed_size(lens.data(), lens.size(), boff) == img.size());
        if (boff == 0) {
            for (size_t window : {(size_t)32768, (size_t)65536, (size_t)1 << 20}) {
                int err = 0;
                std::vector<Bytes> got = read_all(img, 0, window, &err);
                CHECK(err == 0);
                CHECK(got == recs);
            }
            // initial_offset: records starting at or after it
            for (uint64_t off : {(uint64_t)1, (uint64_t)32768, (uint64_t)100000, (uint64_t)img.size()}) {
                int err = 0;
                std::vector<Bytes> got = read_all(img, off, 65536, &err);
                CHECK(got.size() <= recs.size());
                if (!got.empty()) CHECK(got.back() == recs.back());
            }
            // corruption: truncated tail and flipped length bytes must not crash
            Bytes cut(img.begin(), img.begin() + img.size() / 2 + 3);
            int err = 0;
            (void)read_all(cut, 0, 65536, &err);
            Bytes bad = img;
            for (size_t k = 4; k < bad.size(); k += 9973) bad[k] ^= 0x5A;
            (void)read_all(bad, 0, 65536, &err);
        }
    }

    // ---- posix files ----
    char path[] = "/tmp/revel_sanitize_XXXXXX";
    int fd = mkstemp(path);
    CHECK(fd >= 0);
    close(fd);
    revel_writable_file* pf = nullptr;
    CHECK(revel_posix_writable_file_new(path, &pf) == REVEL_OK);
    revel_log_writer* pw = revel_log_writer_new(pf, 0);
    Bytes big(200000, 0xAB);
    CHECK(revel_log_writer_add_record(pw, big.data(), big.size()) == REVEL_OK);
    CHECK(revel_log_writer_add_record(pw, (const uint8_t*)hw, 11) == REVEL_OK);
    CHECK(revel_writable_file_sync(pf) == REVEL_OK);
    CHECK(revel_writable_file_close(pf) == REVEL_OK);
    revel_log_writer_free(pw);
    revel_writable_file_free(pf);
    revel_sequential_file* ps = nullptr;
    CHECK(revel_posix_sequential_file_new(path, &ps) == REVEL_OK);
    revel_log_reader* pr = nullptr;
    CHECK(revel_log_reader_new(ps, 0, 0, nullptr, 0, &pr) == REVEL_OK);
    const uint8_t* d = nullptr;
    size_t n = 0;
    CHECK(revel_log_reader_read_record(pr, &d, &n) == REVEL_OK && n == big.size() && memcmp(d, big.data(), n) == 0);
    CHECK(revel_log_reader_read_record(pr, &d, &n) == REVEL_OK && n == 11 && memcmp(d, hw, 11) == 0);
    CHECK(revel_log_reader_read_record(pr, &d, &n) == REVEL_OK && d == nullptr && n == 0);
    revel_log_reader_free(pr);
    unlink(path);
    revel_sequential_file* missing = nullptr;
    CHECK(revel_posix_sequential_file_new("/nonexistent/revel.log", &missing) == REVEL_NOT_FOUND);

    // ---- memory sequential file semantics (relative skip) ----
    revel_sequential_file* ms = revel_memory_sequential_file_new((const uint8_t*)"0123456789", 10);
    uint8_t sc[16];
    size_t got = 0;
    CHECK(revel_sequential_file_read(ms, sc, 3, &got) == REVEL_OK && got == 3 && memcmp(sc, "012", 3) == 0);
    CHECK(revel_sequential_file_skip(ms, 2) == REVEL_OK);
    CHECK(revel_sequential_file_read(ms, sc, 16, &got) == REVEL_OK && got == 5 && memcmp(sc, "56789", 5) == 0);
    CHECK(revel_sequential_file_read(ms, sc, 16, &got) == REVEL_OK && got == 0);
    revel_sequential_file_free(ms);

    // ---- caller-implemented files ----
    {
        std::vector<Bytes> recs;
        for (int i = 0; i < 40; ++i) {
            Bytes r(rng() % 90000);
            for (auto& b : r) b = (uint8_t)rng();
            recs.push_back(r);
        }
        const Bytes want = write_image(recs, 0);
        VecW vw;
        revel_writable_file* cf = nullptr;
        CHECK(revel_writable_file_from_callbacks(&vw, vw_append, vw_flush, vw_close, vw_sync, vw_release, &cf) ==
              REVEL_OK);
        revel_log_writer* cw = revel_log_writer_new(cf, 0);
        for (const Bytes& r : recs) CHECK(revel_log_writer_add_record(cw, r.data(), r.size()) == REVEL_OK);
        CHECK(revel_writable_file_sync(cf) == REVEL_OK && vw.syncs == 1);
        CHECK(revel_writable_file_close(cf) == REVEL_IO_ERROR && vw.closes == 1);
        CHECK(vw.b == want && vw.flushes >= 40);
        revel_log_writer_free(cw);
        revel_writable_file_free(cf);
        CHECK(vw.released == 1);
        VecW full;
        full.fail_after = 1000;
        revel_writable_file* ff = nullptr;
        CHECK(revel_writable_file_from_callbacks(&full, vw_append, nullptr, nullptr, nullptr, nullptr, &ff) == REVEL_OK);
        revel_log_writer* fw = revel_log_writer_new(ff, 0);
        Bytes big2(5000, 1);
        CHECK(revel_log_writer_add_record(fw, big2.data(), big2.size()) == REVEL_IO_ERROR);
        revel_log_writer_free(fw);
        revel_writable_file_free(ff);
        CHECK(revel_writable_file_from_callbacks(&vw, nullptr, nullptr, nullptr, nullptr, nullptr, &ff) ==
              REVEL_INVALID_ARGUMENT);
        for (size_t chunk : {(size_t)1, (size_t)7, (size_t)4096, (size_t)1 << 30}) {
            VecR vr{&want, 0, chunk};
            revel_sequential_file* sf = nullptr;
            CHECK(revel_sequential_file_from_callbacks(&vr, vr_read, nullptr, vr_release, &sf) == REVEL_OK);
            revel_log_reader* cr = nullptr;
            CHECK(revel_log_reader_new(sf, 0, chunk == 7 ? 40000 : 0, nullptr, 65536, &cr) == REVEL_OK);
            size_t k = 0;
            for (;;) {
                const uint8_t* dd = nullptr;
                size_t nn = 0;
                if (revel_log_reader_read_record(cr, &dd, &nn) != REVEL_OK) continue;
                if (!dd) break;
                if (chunk != 7) CHECK(k < recs.size() && Bytes(dd, dd + nn) == recs[k]);
                ++k;
            }
            if (chunk != 7) CHECK(k == recs.size());
            revel_log_reader_free(cr);
            CHECK(vr.released == 1);
        }
    }

    // ---- shard boundaries + stitch (host walk) ----
    {
        std::vector<Bytes> recs;
        for (int i = 0; i < 50; ++i) {
            Bytes r(rng() % 150000);
            for (auto& b : r) b = (uint8_t)rng();
            recs.push_back(r);
        }
        Bytes img = write_image(recs, 0);
        img[img.size() / 3] ^= 0x11;  // some corruption (a header byte or payload)
        for (int nsh : {1, 2, 3, 7, 16}) {
            std::vector<uint64_t> offs(nsh + 1);
            CHECK(revel_wal_shard_ranges(img.size(), nsh, offs.data()) == REVEL_OK);
            std::vector<Bytes> blobs(nsh);
            std::vector<const uint8_t*> ptrs(nsh);
            std::vector<size_t> sizes(nsh);
            for (int k = 0; k < nsh; ++k) {
                size_t need = 0;
                CHECK(revel_wal_shard_boundary_host(img.data(), img.size(), offs[k], offs[k + 1] - offs[k],
                                                    REVEL_SHARD_READ, nullptr, 0, &need) == REVEL_OK);
                blobs[k].resize(need);
                CHECK(revel_wal_shard_boundary_host(img.data(), img.size(), offs[k], offs[k + 1] - offs[k],
                                                    REVEL_SHARD_READ, blobs[k].data(), need, &need) == REVEL_OK);
                ptrs[k] = blobs[k].data();
                sizes[k] = blobs[k].size();
            }
            revel_wal_stitch* st = nullptr;
            CHECK(revel_wal_stitch_new(ptrs.data(), sizes.data(), nsh, &st) == REVEL_OK);
            revel_wal_summary sum;
            CHECK(revel_wal_stitch_summary(st, &sum) == REVEL_OK);
            CHECK(sum.bytes == img.size());
            for (size_t i = 0; i < sum.stitched; ++i) {
                uint64_t fo = 0, nn = 0;
                const uint8_t* dd = nullptr;
                int before = -1;
                CHECK(revel_wal_stitch_record(st, i, &fo, &dd, &nn, &before) == REVEL_OK);
                CHECK(before > 0 && before < nsh && (dd != nullptr || nn == 0));
            }
            revel_wal_stitch_free(st);
            // truncated blobs are rejected, not read past
            if (nsh > 1) {
                sizes[1] -= 1;
                CHECK(revel_wal_stitch_new(ptrs.data(), sizes.data(), nsh, &st) == REVEL_INVALID_ARGUMENT);
            }
        }
    }

    // ---- GPU entry points fail loudly without a device; null arguments ----
    int count = -1;
    CHECK(revel_gpu_device_count(&count) == REVEL_OK);
    if (count == 0) {
        revel_gpu_context* ctx = nullptr;
        CHECK(revel_gpu_context_new(0, &ctx) == REVEL_NOT_SUPPORT);
        revel_sequential_file* s2 = revel_memory_sequential_file_new((const uint8_t*)"x", 1);
        revel_log_reader* r2 = nullptr;
        CHECK(revel_log_reader_new(s2, 1, 0, nullptr, 0, &r2) == REVEL_NOT_SUPPORT);
    }
    revel_replay_stats st;
    CHECK(revel_gpu_replay_memory(nullptr, nullptr, 0, 0, 0, 0, 0, 0, &st) != REVEL_OK);
    CHECK(revel_gpu_replay_file(nullptr, nullptr, 0, 0, 0, 0, 0, 0, &st) != REVEL_OK);
    uint64_t ne = 0;
    CHECK(revel_gpu_decode_batches(nullptr, nullptr, 0, nullptr, 0, nullptr, nullptr, 0, &ne, nullptr) != REVEL_OK);
    uint64_t nl = 0, pb = 0;
    CHECK(revel_gpu_reassemble(nullptr, nullptr, 0, 0, nullptr, 0, 1, nullptr, nullptr, &nl, &pb, nullptr) != REVEL_OK);
    CHECK(revel_last_error() != nullptr);
    CHECK(revel_log_writer_block_offset(nullptr) == 0);

    if (g_fail) {
        fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    printf("host sanitize test: all checks passed\n");
    return 0;
}
