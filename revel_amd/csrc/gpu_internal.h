// gpu_internal.h -- internal interface between the C-ABI layer and the
// gfx950 kernels (k_blocks.hip, k_records.hip, k_reasm.hip, batch.hip).  Not
// installed; see include/revel_wal.h.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <mutex>
#include <vector>

#include "revel_wal.h"

struct revel_gpu_context;

namespace revel {

// One physical record (or a zero trailer) of a batch append, laid out on the
// host by frame_layout() exactly as log_writer.rs:58-97 would.
constexpr uint32_t kTrailer = 0xFFu;
struct FragDesc {
    uint64_t dst;  // image offset of the 7-byte header (or of the trailer)
    uint64_t src;  // payload offset
    uint32_t len;  // payload length (trailer length for kTrailer)
    uint32_t type;  // record type, or kTrailer
};

struct DeviceInfo {
    int device = 0;
    int num_cu = 256;
};

// k_full_blocks4: interleaved word streams, load ring (k_blocks.hip).
hipError_t crc_full_blocks(const DeviceInfo& di, const void* d_blocks, uint64_t n, uint32_t* d_masked, uint8_t* d_ok,
                           hipStream_t st);
hipError_t frame_full_blocks(const DeviceInfo& di, void* d_blocks, uint64_t n, hipStream_t st);
hipError_t synth_full_blocks(const DeviceInfo& di, void* d_blocks, uint64_t n, uint64_t seed, uint64_t first,
                             hipStream_t st);
// d_hlist (nullable): kListStride u64 per block for verify: the 7 header
// bytes of each of the block's first kListCap records, then the in-block
// offset of record kListCap when there are more (verify lists the rest into
// its result slots, k_list_overflow).  kListCap covers db_bench-shaped logs
// (~240 records of ~140 B per block) in the count pass's one walk.
// kListPerBlock = records per list batch (one per lane) and the density
// threshold: blocks with more go to k_verify_records_dense.
constexpr uint32_t kListPerBlock = 64;
constexpr uint32_t kListCap = 256;
// kListCap entries + the resume offset, padded to 2 176 B = 17 lines of 128 B:
// every list starts on a line (the count pass writes them in whole lines)
constexpr uint32_t kListStride = 272;
static_assert(kListStride >= kListCap + 1, "a block's list holds kListCap entries and the resume offset");
hipError_t count_records(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint32_t* d_counts,
                         uint64_t* d_hlist, hipStream_t st, uint32_t* d_wsums = nullptr);
// With d_wsums (count_wave_sums(nblocks) u32), the count pass also leaves the
// records per 64 blocks.
uint64_t count_wave_sums(uint64_t nblocks);
// The verify kernel's list of qualifying blocks: kBlockListAux u32 (the list
// length, the number of dense blocks, the number of blocks with more than
// kListCap records, one row of kOrderRow counts per workgroup of the ordering
// kernels: blocks with 1..kListPerBlock records, dense ones, ones past kListCap),
// then nblocks u32.
constexpr uint32_t kOrderMaxWG = 256;
constexpr uint32_t kOrderRow = kListPerBlock + 2;
constexpr uint32_t kBlockListAux = 3 + kOrderMaxWG * kOrderRow;
// The production count pass (revel_gpu_count_records / _count_scan_records):
// counts, header lists and records per 64 blocks (d_wsums) as count_records,
// plus the block order's bucket rows in aux (kBlockListAux + nblocks u32).
// scan_order then turns them into the exclusive scan of the counts (d_first)
// and the verify kernel's block list in aux: together with the count pass,
// two launches for what count -> scan -> order histogram -> order scatter did in four.
hipError_t count_hist(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint32_t* d_counts,
                      uint64_t* d_hlist, uint32_t* d_wsums, uint32_t* d_aux, hipStream_t st);
hipError_t scan_order(const DeviceInfo& di, uint64_t nbytes, const uint32_t* d_counts, const uint32_t* d_wsums,
                      uint32_t* d_first, uint32_t* d_aux, hipStream_t st);
// The block list of verify inside a header-list buffer (after the lists).
uint32_t* block_list_of(uint64_t* d_hlist, uint64_t nblocks);
// u64 words of a header-list buffer for nblocks: the lists, then the block list.
uint64_t hlist_words(uint64_t nblocks);
// d_tile_scratch: scan_scratch_words(n) u32 of device scratch.
hipError_t exclusive_scan_u32(const DeviceInfo& di, const uint32_t* d_in, uint32_t* d_out, uint64_t n,
                              uint32_t* d_tile_scratch, hipStream_t st);
uint64_t scan_scratch_words(uint64_t n);
hipError_t exclusive_scan_u64(const DeviceInfo& di, const uint64_t* d_in, uint64_t* d_out, uint64_t n,
                              uint64_t* d_tile_scratch, hipStream_t st);
hipError_t reasm_classify(const DeviceInfo& di, const revel_record_result* d_phys, uint64_t n, uint64_t image_end,
                          int checksum, uint32_t* d_flag, uint64_t* d_len, uint32_t* d_end, hipStream_t st);
hipError_t reasm_emit(const DeviceInfo& di, const revel_record_result* d_phys, uint64_t n, uint64_t image_end,
                      int checksum, const uint32_t* d_flag, const uint32_t* d_idx, const uint64_t* d_off,
                      const uint32_t* d_end, revel_logical_record* d_out, uint64_t* d_frag_dst, hipStream_t st);
// *d_ok (zeroed by the caller) += events with status REVEL_LOGICAL_OK.
hipError_t count_ok_events(const DeviceInfo& di, const revel_logical_record* d_ev, uint64_t n, uint64_t* d_ok,
                           hipStream_t st);
hipError_t reasm_gather(const DeviceInfo& di, const void* d_image, uint64_t image_base,
                        const revel_record_result* d_phys, uint64_t n, const uint64_t* d_frag_dst, void* d_payload,
                        hipStream_t st);
// C3 verify paths (test hook): 0 = production, 1 = v3 walking the headers
// itself, 2 = v3 with the count pass's header lists.  Other values:
// hipErrorInvalidValue.  The experiment arms are in tools/experiments.
hipError_t verify_records_path(const DeviceInfo& di, int path, const void* d_image, uint64_t nbytes,
                               uint64_t base_offset, const uint32_t* d_first, revel_record_result* d_out,
                               const uint64_t* d_hlist, const uint32_t* d_counts, hipStream_t st,
                               bool list_ready = false);
// list_ready: the count pass was count_hist + scan_order for this image, so
// the block list in d_hlist's buffer is built (no ordering launches here).
hipError_t verify_records(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint64_t base_offset,
                          const uint32_t* d_first, revel_record_result* d_out, const uint64_t* d_hlist,
                          const uint32_t* d_counts, hipStream_t st, bool list_ready = false);

// Physical records of an image whose u32 result index could wrap: a block
// holds at most 32768 / 7 = 4681 records, so only images of more than
// kNoWrapBlocks blocks (~28 GiB) can reach 2^32.  total_records sums the
// counts in 64 bits (d_total: one device u64 of scratch) and synchronises st.
constexpr uint64_t kMaxRecordsPerBlock = REVEL_BLOCK_SIZE / REVEL_HEADER_SIZE;
constexpr uint64_t kNoWrapBlocks = 0xFFFFFFFFull / kMaxRecordsPerBlock;
hipError_t total_records(const DeviceInfo& di, const uint32_t* d_counts, uint64_t nblocks,
                         unsigned long long* d_total, uint64_t* total, hipStream_t st);

hipError_t summarize_records(const DeviceInfo& di, const revel_record_result* d_res, const uint32_t* d_first,
                             const uint32_t* d_counts, uint64_t nblocks, uint64_t* d_summary, hipStream_t st);
hipError_t summarize_blocks(const DeviceInfo& di, const uint8_t* d_ok, uint64_t nblocks, uint64_t base_offset,
                            uint64_t* d_summary, hipStream_t st);

// d_counts / d_first / d_xlist (all or none): per virtual block (image byte 0
// at in-block offset lead) the number of records and the fragment index of
// its first record, and one u64 header-list entry per fragment (written by
// the scatter); with them the CRC pass reads its header lists instead of
// walking the headers of every block.  d_blist: kBlockListAux + nblocks u32 of
// scratch for the CRC pass's block list.
hipError_t frame_records(const DeviceInfo& di, const void* d_payloads, const FragDesc* d_frags, uint64_t nfrags,
                         void* d_image, uint64_t image_len, uint32_t lead, hipStream_t st,
                         const uint32_t* d_counts = nullptr, const uint32_t* d_first = nullptr,
                         uint64_t* d_xlist = nullptr, uint32_t* d_blist = nullptr);

hipError_t batch_count(const DeviceInfo& di, const void* d_payload, uint64_t payload_bytes,
                       const revel_logical_record* d_logical, uint64_t n, revel_batch_info* d_info, uint64_t* d_nent,
                       hipStream_t st);
hipError_t batch_emit(const DeviceInfo& di, const void* d_payload, uint64_t payload_bytes,
                      const revel_logical_record* d_logical, uint64_t n, const uint64_t* d_first,
                      revel_batch_info* d_info, revel_batch_entry* d_entries, uint64_t cap, hipStream_t st);

// Grow-only device scratch owned by a revel_gpu_context.  The C-ABI calls
// that use it (decode_batches, reassemble, append framing) synchronise their
// stream before returning, so one call's scratch is free for the next; a call
// that fails synchronises too before it returns.
struct ScratchArena {
    void* base = nullptr;
    uint64_t bytes = 0;
    uint64_t want = 0;  // largest total a call asked for: the next call grows to it
};

// A call's scratch: carved out of the context's arena (no hipMalloc on the
// steady path -- per-call hipMalloc/hipFree of tens of MB cost more than the
// decode kernels); what does not fit is hipMalloc'd and freed on return, and
// the arena grows to the whole request at the next call.
struct DeviceScratch {
    ScratchArena* arena;
    uint64_t used = 0;
    void* ptrs[16] = {};
    int n = 0;
    explicit DeviceScratch(ScratchArena* a = nullptr) : arena(a) {
        if (arena && arena->want > arena->bytes) {
            if (arena->base) (void)hipFree(arena->base);
            arena->base = nullptr;
            arena->bytes = 0;
            if (hipMalloc(&arena->base, arena->want) == hipSuccess) arena->bytes = arena->want;
            else arena->base = nullptr;
        }
    }
    ~DeviceScratch() {
        for (int i = 0; i < n; ++i) (void)hipFree(ptrs[i]);
        if (arena && used > arena->want) arena->want = used;
    }
    template <typename T>
    hipError_t get(T** p, uint64_t count) {
        const uint64_t bytes = ((count ? count : 1) * sizeof(T) + 255) & ~uint64_t(255);
        const uint64_t at = used;
        used += bytes;
        if (arena && arena->base && used <= arena->bytes) {
            *p = reinterpret_cast<T*>(static_cast<uint8_t*>(arena->base) + at);
            return hipSuccess;
        }
        void* q = nullptr;
        if (n == 16) return hipErrorOutOfMemory;
        hipError_t e = hipMalloc(&q, bytes);
        if (e == hipSuccess) ptrs[n++] = q;
        *p = static_cast<T*>(q);
        return e;
    }
};

// Device reassembly of d_phys's events (revel_gpu_reassemble with the torn-
// tail rule at image_end); synchronises st.
hipError_t reassemble_events(revel_gpu_context* ctx, const void* d_image, uint64_t image_base, uint64_t image_end,
                             const revel_record_result* d_phys, uint64_t n, int checksum, revel_logical_record* d_out,
                             void* d_payload, uint64_t* nlogical, uint64_t* payload_bytes, hipStream_t st);

// Host header walk without CRC (a Reader with checksum == false): every
// physical record of img[0, n) (whole blocks from file offset base), statuses
// as the device walk's other than BAD_CHECKSUM (computed_crc = 0).
void host_walk(const uint8_t* img, size_t n, uint64_t base, std::vector<revel_record_result>& out);

// Set the thread-local error string; returns code.
int set_error(int code, const char* fmt, ...);

// Binds `device` on the calling thread for the lifetime of the guard and
// restores the thread's previous current device afterwards, so a C-ABI call
// never moves the caller's later HIP (or torch) work to another GPU.
class DeviceGuard {
   public:
    explicit DeviceGuard(int device) : want_(device) {
        if (hipGetDevice(&prev_) != hipSuccess) {
            (void)hipGetLastError();
            prev_ = -1;
        }
        err_ = prev_ == device ? hipSuccess : hipSetDevice(device);
    }
    ~DeviceGuard() {
        if (err_ == hipSuccess && prev_ >= 0 && prev_ != want_) (void)hipSetDevice(prev_);
    }
    hipError_t err() const { return err_; }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;

   private:
    int want_;
    int prev_ = -1;
    hipError_t err_ = hipSuccess;
};

// Frees the context's cached shard-load ring (device bound by the caller).
void free_shard_ring(revel_gpu_context* ctx);
// Releases the context's resources now (no readers left).  Internal: the
// public revel_gpu_context_free defers to the last reader.
void destroy_context(revel_gpu_context* ctx);
// Reader lifetime bookkeeping: a reader pins its context; the context is
// destroyed by whichever comes last, revel_gpu_context_free or the release
// of its last reader.
void context_pin(revel_gpu_context* ctx);
void context_unpin(revel_gpu_context* ctx);
// The calling thread's default context on its current HIP device (created on
// first use, owned by the thread; released at thread exit).  NOT_SUPPORT when
// the current device is not gfx950.
int default_context(revel_gpu_context** out);

}  // namespace revel

struct revel_gpu_context {
    revel::DeviceInfo di;
    hipStream_t stream = nullptr;
    // Header lists written by revel_gpu_count_records for the image it last
    // counted (single-threaded handle, so count -> scan -> verify on the same
    // context reuses them; any other image makes verify walk headers itself).
    uint64_t* hlist = nullptr;
    uint64_t hlist_cap_blocks = 0;
    const void* hlist_image = nullptr;
    uint64_t hlist_nbytes = 0;
    const uint32_t* hlist_counts = nullptr;
    bool hlist_list_ready = false;  // the count pass also built verify's block list (count_scan_records)
    // 16 B of device scratch: the record-index guard's u64 sum (words 2..3);
    // the experiment library (tools/experiments) also keeps a counter in word 0
    uint32_t* small_scratch = nullptr;
    uint32_t* scan_scratch = nullptr;  // tile sums of revel_gpu_exclusive_scan_u32
    uint64_t scan_scratch_cap = 0;
    // per-64-block record sums of the last count pass (revel_gpu_count_records),
    // consumed by the next revel_gpu_exclusive_scan_u32 of exactly those counts
    uint32_t* wsums = nullptr;
    uint64_t wsums_cap = 0;
    revel::ScratchArena arena;  // per-call scratch of decode_batches / reassemble / append framing
    // Window buffers of the last revel_log_reader freed on this context, parked
    // for the next reader with the same window (host_log.cpp): a reader per log
    // file no longer pays a pinned + device allocation of the window each time.
    struct ParkedReader {
        size_t window = 0;
        uint8_t* h_win = nullptr;  // pinned
        void* d_win = nullptr;
        uint32_t* d_counts = nullptr;
        uint32_t* d_first = nullptr;
        revel_record_result* d_out = nullptr;
        size_t d_out_cap = 0;
    } parked_reader;
    // Pinned load ring (windows + copy stream + events) of the last
    // revel_gpu_wal_shard_load on this context, kept for the next load with
    // the same window; freed with the context or by revel_gpu_context_trim.
    struct ShardRing {
        static constexpr int kSlots = 3;
        size_t window = 0;
        hipStream_t copy = nullptr;
        uint8_t* h[kSlots] = {};
        hipEvent_t e0[kSlots] = {}, e1[kSlots] = {};
    } shard_ring;
    // Lifetime: live readers pin the context; revel_gpu_context_free with
    // readers still alive only marks it, and the last reader's release
    // destroys it (revel_wal.h, "GPU context").
    std::mutex life_mu;
    int readers = 0;
    bool free_requested = false;
};
