// ss_counter.hip — ShortSeqCounter on the GPU: fused encode -> open-addressing hash table in HBM
// with atomic counts and first-occurrence indices (counter.pyx:41-54 semantics).
//
// Table: C = 2^k slots of 16 B (array of structs, one dwordx4 per slot) plus one sentinel slot:
//   key    u64 packed word; EMPTY = ~0.  Claimed once by atomicCAS EMPTY -> key, never changed.
//   ncount u32 = ~count (so a single 0xFF memset resets key, count and first together);
//          incremented with atomicAdd(-1).
//   first  u32 atomicMin of the global read index (0xFFFFFFFF = unset).
// A handle therefore counts reads with global indices below 2^32 - 1 (the 1B-read C5 job uses
// 0..1e9); an index past that raises overflow bit 3 (ss_counter_overflow) and the insert is
// refused up front when base_index + n says so.
// One slot = one dwordx4: the probe load, the count atomic and the first-index check touch the same
// 16 B, and a fresh slice is written back as one dwordx4 store per slot.
// The packed word ~0 ("G" * 32) collides with EMPTY and lives in the sentinel slot C.
// Every key of one handle has the same length L <= 32 (the host groups a mixed batch by length, so
// the dict key (length, packed) of short_seq_64.pyx:41-44 is (handle, word) here).
//
// Probing: Fibonacci hash of the key -> top k bits, linear probing.  A plain (possibly L1-stale)
// load of a key can only be stale as EMPTY (keys never change once claimed); the CAS then returns
// the true value, so no acquire fence is needed (MI355X_MICROARCH.md §visibility).
#include "ss_device.h"
#include "ss_internal.h"

using namespace ssd;

namespace {
struct alignas(16) Slot {
    unsigned long long key;
    uint32_t ncount;
    uint32_t first;
};
static_assert(sizeof(Slot) == 16, "one slot = one dwordx4");
constexpr uint32_t kNoFirst = 0xFFFFFFFFu;     // first index of an unused slot
constexpr uint64_t kMaxIndex = 0xFFFFFFFEull;  // largest global read index a slot can hold
constexpr unsigned long long kOvfTable = 1ull, kOvfExtract = 2ull, kOvfField = 4ull, kOvfIndex = 8ull;
constexpr int kThreads = 256;
constexpr uint32_t kMaxParts = 64;         // owners (GPUs) a table can be partitioned for
constexpr uint32_t kExtractBlocks = 4096;  // extract passes: fixed grid, contiguous slot ranges
constexpr uint32_t kExtractT = 64;         // ONE wave per extract block: slot order is output order
constexpr uint32_t kSliceLogMax = 11;                 // region slice: 2048 slots (one LDS-resident aggregation)
constexpr uint32_t kMwSliceLog = 11;                  // multi-word tables: the k_mw_aggregate LDS bound
constexpr uint32_t kPartBlocks = 1024;      // partition passes: fixed grid, contiguous read ranges
constexpr uint32_t kMaxRegions = 32768;    // per-block region histogram in LDS (128 KB)
}  // namespace

constexpr int32_t kWordKeys = -2;

struct ss_counter {
    uint64_t cap = 0;
    uint32_t log2cap = 0;
    uint32_t slice_log = 0;                // table = 2^(log2cap - slice_log) regions of 2^slice_log slots
    int32_t L = -1;                        // length of every key in this handle (-1: not fixed yet,
                                           // kWordKeys: packed multi-word keys, ss_counter_set_words)
    uint32_t W = 1;                        // words per key: 1 (L <= 32) or ceil(L/32) (multi-word keys)
    Slot* slots = nullptr;                 // [cap + 1]; multi-word: slot.key = 64-bit fingerprint
    uint64_t* keywords = nullptr;          // multi-word keys: [cap * W] the key words of slot s
    uint64_t* ws_words = nullptr;          // multi-word insert workspace: [ws_words_cap] packed reads
    uint64_t ws_words_cap = 0;             // words allocated at ws_words
    uint32_t keywords_W = 0;               // W the keywords array was allocated for
    unsigned long long* work = nullptr;    // [0]: overflow flags, [1..]: per-(part, block) counts
    // partitioned-insert workspace (ss_counter_reserve)
    uint64_t ws_reads = 0;
    uint64_t* ws_keys = nullptr;           // [ws_reads] packed key of read i; later bucketed by region
    uint64_t* ws_akey = nullptr;           // [ws_reads] keys bucketed by coarse bin
    uint32_t* ws_aidx = nullptr;           // [ws_reads] batch-local read index, same order
    uint32_t* ws_acnt = nullptr;           // weighted records' counts, coarse order (same size as ws_aidx)
    uint8_t* ws_areg = nullptr;            // region-in-bin byte per coarse record (same size as ws_aidx)
    uint32_t* ws_bidx = nullptr;           // [ws_reads] batch-local read index, region order
    uint32_t* ws_bcnt = nullptr;           // [ws_reads] weighted records' counts, region order
    uint4* ws_spill = nullptr;             // [ws_reads] records past a full sub-bin
    uint32_t* ws_hist = nullptr;           // [kPartBlocks * regions] per-(block, bin) counts -> offsets
    uint32_t* ws_rstart = nullptr;         // [regions + 1] region start in the bucket arrays
    uint32_t* ws_order = nullptr;          // [3 kNFill] sub-bins by descending fill, slab bases, slab sizes (k_pf_order)
    uint32_t* ws_segend = nullptr;         // [regions x kFinePerBin] end of each (sub-bin, region) fine segment
    uint32_t* ws_tot = nullptr;            // [regions + 1] scratch (bin totals / coarse starts)
    // optimistic coarse partition (k_pf_coarse): ws_akey / ws_aidx hold 128 bins of ws_cap1 slots
    uint64_t ws_cap1 = 0;
    uint64_t ws_slab = 0;                  // 1 = fine-scatter slabs per (sub-bin, region), 0 = counted cursors
    uint64_t ws_brecs = 0;                 // fine-record slots (ws_keys / ws_bidx / ws_bcnt)
    uint32_t* ws_fill = nullptr;           // sub-bin fill counters + the spill counter, kFillStride apart
    // per-region occupancy (used slots of each slice), written by the single-word aggregate (and
    // kept by the spill insert); lets ss_counter_pack_ranges skip its counting pass.
    // occ_src: 0 = stale, 1 = valid
    uint32_t* occ = nullptr;               // [R]
    void* aux = nullptr;                   // scratch of the fold / merge passes, kept between calls
    size_t aux_bytes = 0;                  // (stream-ordered allocations were released to the OS at
                                           // every sync: ~0.4 ms of unmap / remap per f2 chunk)
    unsigned long long* roff = nullptr;    // [R + 2] pack scratch: region offsets, sentinel position
    uint64_t occ_R = 0;
    int occ_src = 0;
    // ss_counter_reset is lazy for the slot array: the next partitioned single-word insert's
    // aggregate writes whole slices instead (fresh mode); any other access memsets first
    bool reset_pending = false;
    // per-pass timing of the optimistic partitioned insert (ss_counter_set_timing): a ring of event
    // sets, one per insert, folded into the sums when read back (or when the ring wraps)
    static constexpr uint32_t kTimerRing = 64, kPassEvents = 6;
    hipEvent_t* tev = nullptr;             // [kTimerRing * kPassEvents] or null (timing off)
    uint32_t thead = 0, tpend = 0;         // next set, sets recorded and not yet folded
    double tsum[kPassEvents - 1] = {};
    uint64_t tn = 0;
    // u64 counts: a slot's u32 count is its low part; wide[s] (allocated on first need,
    // zeroed when it goes live) holds the rest.  Inserts add at most one per read, so before the reads
    // inserted since the last spill could pass spill_at, every slot's count moves into wide
    // (k_spill_wide) and the slot restarts at 0 (the sentinel keeps 1); merges carry into wide as they
    // add.  Nothing reads wide while it is not live (tbl_of passes null), so the C5 insert is unchanged.
    uint64_t* wide = nullptr;              // [cap + 1]
    bool wide_live = false;
    uint64_t since = 0;                    // reads inserted since the last reset / spill (kSinceUnknown after a merge)
    uint64_t spill_at = 0xFFFFFFFFull;     // ss_counter_set_spill_limit (a test hook lowers it)
};

namespace {

struct Tbl {
    Slot* slots;
    uint64_t* wide;       // [cap + 1] high parts of the counts, or null (ss_counter::wide)
    uint64_t* keywords;   // multi-word keys only
    uint32_t* occ;        // [R] used slots per region (written by the single-word aggregate) or null
    uint32_t W;
    unsigned long long* overflow;
    uint64_t mask;        // cap - 1
    uint64_t slice_mask;  // slots per region - 1
    uint32_t shift;       // 64 - log2(cap)
    uint32_t slice_log;
};

__device__ __forceinline__ uint64_t slot_hash(uint64_t key, uint32_t shift) {
    return (key * 0x9E3779B97F4A7C15ull) >> shift;
}

// Owner partition for the multi-GPU merge (independent of the table's hash bits).
// Mirrored on the host by shortseq_amd/dist.py owner_of_np.
__host__ __device__ __forceinline__ uint32_t owner_of(uint64_t key, uint32_t nparts) {
    return (uint32_t)((splitmix64(key) >> 32) % nparts);
}

// Slot addressing: t = top log2(cap) bits of the Fibonacci hash = (region | offset); linear
// probing stays inside the region's slice, so a region is a self-contained sub-table that one
// workgroup can own (the partitioned insert below); with one region this is plain linear probing.
__device__ __forceinline__ uint64_t slot_top(const Tbl& t, uint64_t key) {
    return t.shift >= 64 ? 0 : slot_hash(key, t.shift);
}

// Insert / count `cnt` copies of `key` first seen at global read index `idx`.  Returns true when this
// call claimed a new slot (the spill pass keeps the region occupancy current with it).
__device__ __forceinline__ void count_add_wide(const Tbl& t, uint64_t s, uint32_t old_count, uint32_t lo, uint64_t hi);
__device__ __forceinline__ bool tbl_add(const Tbl& t, uint64_t key, uint64_t cnt64, unsigned long long idx) {
    const uint32_t cnt = (uint32_t)cnt64;
    bool claimed = false;
    uint64_t s;
    if (key == kEmpty) {
        s = t.mask + 1;  // sentinel slot
    } else {
        const uint64_t top = slot_top(t, key);
        const uint64_t base = top & ~t.slice_mask;
        uint64_t off = top & t.slice_mask;
        uint64_t probes = 0;
        for (;;) {
            const uint64_t h = base + off;
            const unsigned long long cur = t.slots[h].key;
            if (cur == key) {
                s = h;
                break;
            }
            if (cur == kEmpty) {
                const unsigned long long prev = atomicCAS(&t.slots[h].key, (unsigned long long)kEmpty,
                                                          (unsigned long long)key);
                if (prev == kEmpty || prev == key) {
                    claimed = prev == kEmpty;
                    s = h;
                    break;
                }
            }
            off = (off + 1) & t.slice_mask;
            if (++probes > t.slice_mask) {
                atomicOr(t.overflow, kOvfTable);
                return false;
            }
        }
    }
    if (idx > kMaxIndex) {
        atomicOr(t.overflow, kOvfIndex);
        idx = kMaxIndex;
    }
    Slot* sl = &t.slots[s];
    const uint32_t old = atomicAdd(&sl->ncount, 0u - cnt);
    count_add_wide(t, s, ~old, cnt, cnt64 & ~0xFFFFFFFFull);
    if (sl->first > (uint32_t)idx) atomicMin(&sl->first, (uint32_t)idx);
    return claimed;
}

// The part of a count add the slot's u32 cannot hold (hi: the added count's high part; the carry out
// of old_count + lo) goes to wide[s]; without a live wide array such an add flags kOvfField.
__device__ __forceinline__ void count_add_wide(const Tbl& t, uint64_t s, uint32_t old_count, uint32_t lo, uint64_t hi) {
    const uint64_t extra = hi + ((((uint64_t)old_count + lo) >> 32) << 32);
    if (!extra) return;
    if (t.wide)
        atomicAdd((unsigned long long*)&t.wide[s], (unsigned long long)extra);
    else
        atomicOr(t.overflow, kOvfField);
}

// Fast path, L in {16, 32}, 16-B aligned rows: two lanes per read (lane pair = one packed word,
// same chunk encoder as k_encode_g16), the even lane inserts.
template <int U>
__global__ __launch_bounds__(kThreads) void k_count_g16(Tbl t, const uint4* __restrict__ in,
                                                        uint64_t stride16, uint64_t n, uint32_t cpr,
                                                        uint64_t base_index, unsigned long long* first_bad,
                                                        const uint32_t* only_if = nullptr) {
    if (only_if && *only_if == 0u) return;   // fallback launch of the optimistic partition: idle
    // grid-stride over block tiles (uniform trip count: the lane-pair exchanges need whole waves)
    for (uint64_t tb = (uint64_t)blockIdx.x * (U * kThreads); tb < 2 * n; tb += (uint64_t)gridDim.x * (U * kThreads)) {
    const uint64_t base = tb + threadIdx.x;
    uint4 x[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t g = base + (uint64_t)j * kThreads;
        const uint64_t r = g >> 1;
        const uint32_t k = (uint32_t)g & 1u;
        x[j] = (r < n && k < cpr) ? ld_stream(&in[r * stride16 + k])
                                  : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t g = base + (uint64_t)j * kThreads;
        const uint64_t r = g >> 1;
        const uint32_t k = (uint32_t)g & 1u;
        Enc32 e = encode16(x[j].x, x[j].y, x[j].z, x[j].w, true);   // L <= 32: table path
        const uint32_t cin = swap_pair(e.cout);
        const uint32_t v = e.v | (k ? cin : 0u);
        const uint32_t hi = swap_pair(v);
        const uint32_t bad_pair = e.bad | swap_pair(e.bad);
        const bool live = r < n && k == 0;
        report_bad(live && bad_pair != 0u, r, first_bad);
        if (live && bad_pair == 0u) tbl_add(t, (uint64_t)v | ((uint64_t)hi << 32), 1u, base_index + r);
    }
    }
}

__device__ __forceinline__ uint64_t load_word_general(const uint8_t* p, uint32_t nb, uint32_t& bad);

// General path (any L <= 32, any stride): one lane per read.
__global__ __launch_bounds__(kThreads) void k_count_gen(Tbl t, const uint8_t* in, uint64_t stride,
                                                        uint64_t n, uint32_t L, uint64_t base_index,
                                                        unsigned long long* first_bad) {
    for (uint64_t r = (uint64_t)blockIdx.x * kThreads + threadIdx.x; r < n; r += (uint64_t)gridDim.x * kThreads) {
        uint32_t bad = 0;
        const uint64_t key = load_word_general(in + r * stride, L, bad);
        if (bad) {
            atomicMin(first_bad, (unsigned long long)r);
            continue;
        }
        tbl_add(t, key, 1u, base_index + r);
    }
}

__device__ __forceinline__ uint64_t load_word_general(const uint8_t* p, uint32_t nb, uint32_t& bad) {
    if (nb == 0) return 0;
    const uintptr_t addr = (uintptr_t)p;
    const uint32_t* d = (const uint32_t*)(addr & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(addr & 3);
    const uint32_t nd = (sh + nb + 3u) >> 2;
    uint32_t dw[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) dw[i] = ((uint32_t)i < nd) ? d[i] : 0x41414141u;
    uint32_t xw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t v = __builtin_amdgcn_alignbyte(dw[i + 1], dw[i], sh);
        const int m = (int)nb - 4 * i;
        if (m <= 0) {
            v = 0x41414141u;
        } else if (m < 4) {
            const uint32_t keep = (1u << (8 * m)) - 1u;
            v = (v & keep) | (0x41414141u & ~keep);
        }
        xw[i] = v;
    }
    Enc32 lo = encode16(xw[0], xw[1], xw[2], xw[3], true);
    Enc32 hi = encode16(xw[4], xw[5], xw[6], xw[7], true);
    bad |= lo.bad | hi.bad;
    return (uint64_t)lo.v | ((uint64_t)(hi.v | lo.cout) << 32);
}

__global__ __launch_bounds__(kThreads) void k_merge(Tbl t, const uint64_t* keys, const uint64_t* counts,
                                                    const uint64_t* first, uint64_t m) {
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < m; i += (uint64_t)gridDim.x * kThreads)
    {
        tbl_add(t, keys[i], counts[i], first[i]);   // (a count past 2^32 carries into wide)
    }
}

__device__ __forceinline__ bool slot_used(const Tbl& t, uint64_t s, uint64_t& key) {
    const Slot& sl = t.slots[s];
    if (s <= t.mask) {
        key = sl.key;
        return key != kEmpty;
    }
    key = kEmpty;
    return sl.ncount != 0xFFFFFFFFu;   // sentinel slot: used iff its count is nonzero
}

__global__ __launch_bounds__(kThreads) void k_size(Tbl t, unsigned long long* out) {
    __shared__ unsigned int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    unsigned int local = 0;
    for (uint64_t s = (uint64_t)blockIdx.x * kThreads + threadIdx.x; s <= t.mask + 1; s += (uint64_t)gridDim.x * kThreads) {
        uint64_t key;
        local += slot_used(t, s, key) ? 1u : 0u;
    }
    atomicAdd(&cnt, local);
    __syncthreads();
    if (threadIdx.x == 0 && cnt) atomicAdd(out, (unsigned long long)cnt);
}

// Wave-aggregated "reserve `mine` positions of part p0" helper: for every distinct part present in
// the wave (peeled with readfirstlane + ballot), ONE lane adds the wave's count to an LDS counter.
// Returns this lane's position (base + rank) for its part, or 0 for lanes with !used.
__device__ __forceinline__ unsigned long long wave_reserve(bool used, uint32_t part, unsigned long long* lds_ctr) {
    uint64_t pending = __ballot(used);
    unsigned long long pos = 0;
    const int lane = (int)(threadIdx.x & 63);
    while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const uint32_t p0 = (uint32_t)__shfl((int)part, leader);
        const uint64_t mine = __ballot(used && part == p0);
        const uint32_t rank = __popcll(mine & ((1ull << lane) - 1ull));
        unsigned long long base = 0;
        if (lane == leader) base = atomicAdd(&lds_ctr[p0], (unsigned long long)__popcll(mine));
        base = __shfl(base, leader);
        if (used && part == p0) pos = base + rank;
        pending &= ~mine;
    }
    return pos;
}

// Owner part of an occupied slot.  Hash owners (ranges = false): owner_of(key) — any table
// geometry.  Region-range owners (ranges = true, the multi-GPU counter): part p owns the table
// regions [p R / n, (p + 1) R / n) — slot s sits in region s >> slice_log; the sentinel slot (key
// ~0) belongs to the owner of region_of(~0).  Extracted in slot order, each part's entries are
// then sorted by region, which ss_counter_merge_runs relies on.
__device__ __forceinline__ uint32_t part_of(const Tbl& t, uint64_t s, uint64_t key, uint32_t nparts, bool ranges) {
    if (!ranges) return owner_of(key, nparts);
    const uint64_t R = (t.mask + 1) >> t.slice_log;
    const uint64_t region = s <= t.mask ? (s >> t.slice_log) : (slot_top(t, kEmpty) >> t.slice_log);
    return (uint32_t)(region * nparts / R);
}

// Extract pass 1: block b (one wave) counts the used slots of its contiguous range per part ->
// bc[p*B + b].  Pass 3 walks the same range in the same order, so within a part the output is in
// slot order (blocks in block order, a wave's lanes in lane order).
__global__ __launch_bounds__(kExtractT) void k_part_count(Tbl t, uint32_t nparts, unsigned long long* bc, bool ranges) {
    __shared__ unsigned long long hist[kMaxParts];
    for (uint32_t p = threadIdx.x; p < nparts; p += kExtractT) hist[p] = 0;
    __syncthreads();
    const uint64_t nslots = t.mask + 2;
    const uint64_t per = (nslots + kExtractBlocks - 1) / kExtractBlocks;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = min(nslots, lo + per);
    for (uint64_t s0 = lo; s0 < hi; s0 += kExtractT) {
        const uint64_t s = s0 + threadIdx.x;
        uint64_t key = kEmpty;
        const bool used = s < hi && slot_used(t, s, key);
        wave_reserve(used, used ? part_of(t, s, key, nparts, ranges) : 0u, hist);
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < nparts; p += kExtractT) bc[(uint64_t)p * kExtractBlocks + blockIdx.x] = hist[p];
}

// Extract pass 2 (one block of 1024): exclusive scan of bc in (part, block) order = each block's
// start offset in its part's region; part totals -> part_counts.
__global__ __launch_bounds__(1024) void k_part_offsets(uint32_t nparts, unsigned long long* bc,
                                                        unsigned long long* part_counts) {
    __shared__ unsigned long long sums[1024];
    const uint32_t total = nparts * kExtractBlocks;
    const uint32_t seg = (total + 1023) / 1024;
    const uint32_t lo = threadIdx.x * seg, hi = min(total, lo + seg);
    unsigned long long local = 0;
    for (uint32_t i = lo; i < hi; ++i) local += bc[i];
    sums[threadIdx.x] = local;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const unsigned long long v = threadIdx.x >= off ? sums[threadIdx.x - off] : 0ull;
        __syncthreads();
        sums[threadIdx.x] += v;
        __syncthreads();
    }
    unsigned long long run = sums[threadIdx.x] - local;   // exclusive prefix of this segment
    for (uint32_t i = lo; i < hi; ++i) {
        const unsigned long long c = bc[i];
        bc[i] = run;
        run += c;
    }
    __syncthreads();
    // part totals: part p spans bc[p*B .. (p+1)*B); total = next region start - this start
    for (uint32_t p = threadIdx.x; p < nparts; p += 1024) {
        const unsigned long long start = bc[(uint64_t)p * kExtractBlocks];
        const unsigned long long end = (p + 1 < nparts) ? bc[(uint64_t)(p + 1) * kExtractBlocks] : sums[1023];
        part_counts[p] = end - start;
    }
}

// Extract pass 3: same ranges as pass 1; LDS cursors start at the block's offsets, so every slot's
// position is reserved without any global atomic.
__global__ __launch_bounds__(kExtractT) void k_part_scatter(Tbl t, uint32_t nparts, int32_t L,
                                                           const unsigned long long* bc, uint64_t* okeys,
                                                           uint32_t* olens, uint64_t* ocounts, uint64_t* ofirst,
                                                           uint64_t cap_out, unsigned long long* overflow,
                                                           uint64_t* owords, bool ranges) {
    __shared__ unsigned long long cursor[kMaxParts];
    for (uint32_t p = threadIdx.x; p < nparts; p += kExtractT) cursor[p] = bc[(uint64_t)p * kExtractBlocks + blockIdx.x];
    __syncthreads();
    const uint64_t nslots = t.mask + 2;
    const uint64_t per = (nslots + kExtractBlocks - 1) / kExtractBlocks;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = min(nslots, lo + per);
    for (uint64_t s0 = lo; s0 < hi; s0 += kExtractT) {
        const uint64_t s = s0 + threadIdx.x;
        uint64_t key = kEmpty;
        const bool used = s < hi && slot_used(t, s, key);
        const unsigned long long pos = wave_reserve(used, used ? part_of(t, s, key, nparts, ranges) : 0u, cursor);
        if (!used) continue;
        if (pos >= cap_out) {
            atomicOr(overflow, kOvfExtract);
            continue;
        }
        const Slot& sl = t.slots[s];
        if (owords) {   // key words (multi-word: okeys gets the fingerprint; one word: the key)
            if (t.W == 1) {
                owords[pos] = key;
            } else {
                const uint64_t* kw = t.keywords + s * t.W;
                for (uint32_t q = 0; q < t.W; ++q) owords[pos * t.W + q] = kw[q];
            }
        }
        okeys[pos] = key;
        olens[pos] = (uint32_t)L;
        ocounts[pos] = (uint64_t)(uint32_t)~sl.ncount + (t.wide ? t.wide[s] : 0ull);
        ofirst[pos] = sl.first;
    }
}

// ------------------------------------------------------------------------------------------------
// Partitioned insert (the C5 hot path).  Per-read global atomics on a 1-GB table are memory-side
// atomic-bound; instead every table region (slice of 2^slice_log slots) is aggregated by ONE
// workgroup in LDS and merged into its slice with plain loads/stores.
//   L 16 / 32, aligned rows, > 128 regions (the C5 case): the optimistic coarse partition below
//     (k_pf_coarse: encode + coarse scatter with per-(tile, bin) atomic reservations; k_pf_count,
//     k_pf_tot / k_pc_scan / k_pf_offsets, k_pf_scatter: fine pass by coarse bin).
//   Otherwise the exact passes:
//     P1 k_pc_keys (or ss_encode_fixed + k_pc_hist for other L) -> keys[i], per-block coarse histogram
//     P2 scan      per-(block, bin) write offsets (k_pc_tot / k_pc_scan / k_pc_offsets)
//     P3 k_pc_scatter_lds by coarse bin, then k_pc_count + scan + k_pc_scatter_lds by region
//        (<= 256 regions per coarse bin) -- a 2-pass radix partition; every pass gives block b the
//        same contiguous input range, so offsets are exact.
//   P4 k_pc_aggregate_slice: one workgroup per region folds its bucket straight into an LDS copy of
//      the region's slice (the slice is the hash table: probe, LDS CAS for a new key, LDS add / min),
//      then writes the touched slots back; nobody else touches the slice.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kCoarseBits = 7;    // 128 coarse bins for the first partition pass

// Weighted partition record: read index | kWeighted means the record stands for several copies of
// its key (deduplicated inside one coarse tile); its count sits in the parallel count array (acnt
// in coarse order, bcnt in region order).  Batch-local indices are < 2^31 (ss_counter_reserve).
constexpr uint32_t kWeighted = 0x80000000u;

// Partition record: key and read index in one 12-B dwordx3, for the coarse and the fine records
// (the region bytes and the sparse counts stay apart).  Against two streams (u64 keys + u32
// indices): the scatter 2.54 -> 2.21-2.37 ms at its end, the insert -0.01 to -0.14 ms uniform 2^24
// over 3 same-box rounds; a 16-B record with the count inside measured no better.
struct __attribute__((packed, aligned(4))) Rec12 {
    uint32_t klo, khi, idx;
};
// fine-pass slabs instead of counted cursors (ss_counter_reserve decides per reservation): a slab
// holds 2 x its region's mean share of the sub-bin + kSlabPad records, rounded up to 16
constexpr uint64_t kSlabMinMean = 256;
constexpr uint32_t kSlabPad = 256;
// slab size of a sub-bin holding f coarse records over nb regions.  The fine scatter's heavy-region
// dedup keeps a region at <= 2 x the mean records per tile unless it holds that many distinct keys,
// so 2 x (f / nb) + a partial tile's slack is overrun only by crafted inputs (those spill).
__host__ __device__ __forceinline__ uint32_t slab_size(uint32_t f, uint32_t nb) {
    return (2 * ((f + nb - 1) / nb) + kSlabPad + 15) & ~15u;
}

struct PartWs {
    const Rec12* brec; // optimistic path: the region-ordered records (else null)
    uint32_t slab;     // optimistic path: 1 = fine records of (sub-bin f, region j) live in slab
                       // [slabs[f] + j slabs[kNFill + f], + slabs[kNFill + f]) (no count pass);
                       // 0 = counted cursors (hist)
    const uint32_t* slabs; // [2 kNFill] per sub-bin slab base and slab size (k_pf_order)
    uint32_t* spill_ctr;   // the spill list's record counter (shared with the coarse pass's overflow)
    uint64_t* keys;    // P1 output; P3 second-pass output (bucketed by region)
    uint64_t* akey;    // first-pass output (bucketed by coarse bin)
    uint32_t* aidx;
    uint32_t* acnt;    // weighted records' counts, coarse order (sparse: weighted positions only)
    uint8_t* areg;     // optimistic path: each coarse record's region within its bin (k_pf_count)
    uint32_t* bidx;    // second-pass output indices
    uint32_t* bcnt;    // weighted records' counts, region order (sparse)
    uint4* spill;      // records past a full sub-bin: {key lo, key hi, count, batch index}
    uint64_t spill_cap;
    uint32_t* seg_end; // optimistic path: end of each (sub-bin, region) segment written by the fine
                       // scatter (hist holds the starts); null on the exact paths (rstart ranges)
    const uint64_t* bkey;  // the region-bucketed keys the aggregate reads (keys or akey)
    uint32_t* hist;    // [kPartBlocks][bins] per-(block, bin) counts -> offsets
    uint32_t* rstart;  // [R + 1] region start in the bucketed arrays
    uint32_t* tot;     // [bins] scratch
    uint32_t R;        // regions
    uint32_t rbits;    // log2(R)
};

__device__ __forceinline__ uint32_t region_of(const Tbl& t, uint64_t key) {
    return (uint32_t)(slot_top(t, key) >> t.slice_log);
}

// The optimistic partition (k_pf_coarse -> k_pf_scatter -> k_pc_aggregate_slice<REC12>) carries each
// key as its slot hash h = key * kSlotMul (a bijection of the u64 keys: kSlotInv is the multiplier's
// inverse mod 2^64), so the passes after the coarse one take region and home slot from h by shifts
// instead of a 64-bit multiply per use; the aggregate turns h back into the key once per used slot
// when it writes the slice.  Spill records carry the key itself (k_spill_insert uses tbl_add).
constexpr uint64_t kSlotMul = 0x9E3779B97F4A7C15ull, kSlotInv = 0xF1DE83E19937733Dull;
static_assert(kSlotMul * kSlotInv == 1ull, "inverse of the slot hash multiplier");
constexpr uint64_t kEmptyH = kEmpty * kSlotMul;   // h of the EMPTY key (the sentinel's records)
__device__ __forceinline__ uint32_t region_of_h(const Tbl& t, uint64_t h) {
    return t.shift >= 64 ? 0u : (uint32_t)((h >> t.shift) >> t.slice_log);
}

// bin of a key for a pass: COARSE -> top kCoarseBits of the region id, else the region id
template <bool COARSE>
__device__ __forceinline__ uint32_t bin_of(const Tbl& t, const PartWs& w, uint64_t key) {
    const uint32_t r = region_of(t, key);
    if constexpr (COARSE) return w.rbits > kCoarseBits ? (r >> (w.rbits - kCoarseBits)) : r;
    return r;
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_pc_keys(Tbl t, PartWs w, uint32_t bins, const uint4* __restrict__ in,
                                               uint64_t stride16, uint64_t n, uint32_t cpr,
                                               unsigned long long* first_bad) {
    // one histogram copy per wave when they fit (bins <= 64 in the two-pass case): LDS atomics then
    // contend only inside a wave
    extern __shared__ uint32_t hist[];
    constexpr uint32_t kWaves = T / 64;
    const uint32_t copies = bins * kWaves <= kMaxRegions ? kWaves : 1u;
    uint32_t* my = hist + (copies > 1 ? (threadIdx.x >> 6) * bins : 0u);
    for (uint32_t i = threadIdx.x; i < bins * copies; i += T) hist[i] = 0;
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = min(n, lo + per);
    // one lane per read (U reads per lane per tile): both 16-B chunks of a read in the lane, so the
    // table-path carry, the key, its hash and the histogram atomic need no lane exchange and every
    // lane does useful work (SQ counters on the 2-lanes-per-read form: 62 % issue-stalled)
    constexpr uint32_t kReadsPerTile = T * U;
    uint4 nx[U][2];
    auto load_tile = [&](uint64_t t0) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t r = t0 + j * T + threadIdx.x;
            const bool ok = r < hi;
            nx[j][0] = ok ? ld_stream(&in[r * stride16]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
            nx[j][1] = (ok && cpr > 1) ? ld_stream(&in[r * stride16 + 1])
                                      : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
        }
    };
    if (lo < hi) load_tile(lo);
    for (uint64_t t0 = lo; t0 < hi; t0 += kReadsPerTile) {
        uint4 x[U][2];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            x[j][0] = nx[j][0];
            x[j][1] = nx[j][1];
        }
        if (t0 + kReadsPerTile < hi) load_tile(t0 + kReadsPerTile);
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t r = t0 + j * T + threadIdx.x;
            // L <= 32: table path for both chunks; the low chunk's alias carry goes into the high
            // half (for L = 16 the high chunk is "A" padding and the carry lands at bit 32, as the
            // reference's acc << 2 loop puts it)
            const Enc32 a = encode16(x[j][0].x, x[j][0].y, x[j][0].z, x[j][0].w, true);
            const Enc32 b = encode16(x[j][1].x, x[j][1].y, x[j][1].z, x[j][1].w, true);
            const bool live = r < hi;
            report_bad(live && (a.bad | b.bad) != 0u, r, first_bad);
            if (live) {
                const uint64_t key = (uint64_t)a.v | ((uint64_t)(b.v | a.cout) << 32);
                w.keys[r] = key;
                atomicAdd(&my[bin_of<true>(t, w, key)], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < bins; i += T) {
        uint32_t sum = 0;
        for (uint32_t c = 0; c < copies; ++c) sum += hist[c * bins + i];
        w.hist[(uint64_t)blockIdx.x * bins + i] = sum;
    }
}

// P1 for already-packed single-word keys (any L <= 32, any stride: the batch was packed into
// w.keys by ss_encode_fixed first): the same per-block histogram over the same block ranges.
template <int T>
__global__ __launch_bounds__(T) void k_pc_hist(Tbl t, PartWs w, uint32_t bins, uint64_t n) {
    extern __shared__ uint32_t hist[];
    constexpr uint32_t kWaves = T / 64;
    const uint32_t copies = bins * kWaves <= kMaxRegions ? kWaves : 1u;
    uint32_t* my = hist + (copies > 1 ? (threadIdx.x >> 6) * bins : 0u);
    for (uint32_t i = threadIdx.x; i < bins * copies; i += T) hist[i] = 0;
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = min(n, lo + per);
    for (uint64_t r = lo + threadIdx.x; r < hi; r += T) atomicAdd(&my[bin_of<true>(t, w, w.keys[r])], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < bins; i += T) {
        uint32_t sum = 0;
        for (uint32_t c = 0; c < copies; ++c) sum += hist[c * bins + i];
        w.hist[(uint64_t)blockIdx.x * bins + i] = sum;
    }
}

// per-block histogram of region ids over a coarse-bucketed key array (second pass).  The block's
// range spans few coarse buckets, so the histogram covers only that window of regions (as in
// k_pc_scatter_lds); a wider span counts straight into the global row.
template <int T>
__global__ __launch_bounds__(T) void k_pc_count(Tbl t, PartWs w, const uint64_t* __restrict__ src, uint64_t n) {
    constexpr uint32_t kWin = 1024;
    __shared__ uint32_t hist[kWin];
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = min(n, lo + per);
    uint32_t* row = w.hist + (uint64_t)blockIdx.x * w.R;
    for (uint32_t i = threadIdx.x; i < w.R; i += T) row[i] = 0;
    if (lo >= hi) return;
    const uint32_t shift = w.rbits > kCoarseBits ? (w.rbits - kCoarseBits) : 0;
    const uint32_t c0 = region_of(t, src[lo]) >> shift, c1 = region_of(t, src[hi - 1]) >> shift;
    const uint32_t rlo = c0 << shift, nb = (c1 - c0 + 1) << shift;
    if (nb > kWin) {
        __syncthreads();   // the row was zeroed by other threads
        for (uint64_t r = lo + threadIdx.x; r < hi; r += T) atomicAdd(&row[region_of(t, src[r])], 1u);
        return;
    }
    for (uint32_t i = threadIdx.x; i < nb; i += T) hist[i] = 0;
    __syncthreads();
    for (uint64_t r = lo + threadIdx.x; r < hi; r += T) atomicAdd(&hist[region_of(t, src[r]) - rlo], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += T) row[rlo + i] = hist[i];
}

// bin totals (thread per bin; coalesced over bins)
// bin totals: one block per bin, its threads over the kPartBlocks partition blocks' counts (a
// thread per bin looping over all blocks was a 1024-long serial chain: 40-65 us per call on the
// small per-length tables of a FASTQ file)
__global__ __launch_bounds__(256) void k_pc_tot(PartWs w, uint32_t bins) {
    __shared__ uint32_t red[4];
    const uint32_t r = blockIdx.x;
    uint32_t sum = 0;
    for (uint32_t b = threadIdx.x; b < kPartBlocks; b += 256) sum += w.hist[(uint64_t)b * bins + r];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) sum += (uint32_t)__shfl_xor((int)sum, off);
    if ((threadIdx.x & 63u) == 0) red[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) w.tot[r] = red[0] + red[1] + red[2] + red[3];
}

// exclusive scan of bin totals (one block of 1024) -> start[bins + 1]
__global__ __launch_bounds__(1024) void k_pc_scan(PartWs w, uint32_t bins, uint32_t* start,
                                                  const uint32_t* skip_if = nullptr) {
    __shared__ uint32_t sums[1024];
    if (skip_if && *skip_if) return;
    const uint32_t seg = (bins + 1023) / 1024;
    const uint32_t lo = threadIdx.x * seg, hi = min(bins, lo + seg);
    uint32_t local = 0;
    for (uint32_t i = lo; i < hi; ++i) local += w.tot[i];
    sums[threadIdx.x] = local;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = threadIdx.x >= off ? sums[threadIdx.x - off] : 0u;
        __syncthreads();
        sums[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = sums[threadIdx.x] - local;
    for (uint32_t i = lo; i < hi; ++i) {
        const uint32_t c = w.tot[i];   // read before the write: start may alias tot
        start[i] = run;
        run += c;
    }
    if (threadIdx.x == 1023) start[bins] = sums[1023];
}

// per-(block, bin) write offsets = bin start + counts of earlier blocks: one block per bin, a thread
// per partition block, block-wide exclusive scan
static_assert(kPartBlocks == 1024, "k_pc_offsets: one thread per partition block");
__global__ __launch_bounds__(1024) void k_pc_offsets(PartWs w, uint32_t bins, const uint32_t* start) {
    __shared__ uint32_t wtot[16];
    const uint32_t r = blockIdx.x, b = threadIdx.x, lane = b & 63u, wave = b >> 6;
    const uint64_t i = (uint64_t)b * bins + r;
    const uint32_t c = w.hist[i];
    uint32_t incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
        if (lane >= (uint32_t)off) incl += y;
    }
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
#pragma unroll
    for (uint32_t v = 0; v < 16; ++v) before += v < wave ? wtot[v] : 0u;
    w.hist[i] = start[r] + before + incl - c;
}

// LDS-staged scatter (both partition passes).  Per tile of kTile elements: local histogram of the
// block's active bins -> exclusive scan -> elements placed in LDS sorted by bin -> written out so
// consecutive lanes store consecutive positions of one bin's run (full-line stores), then the
// block's per-bin cursors advance.  Active bins: COARSE pass = the 64 coarse bins; fine pass =
// the regions of the (1-2) coarse buckets the block's range spans (range-sorted input), mapped to
// local bins region - lo_region; a block spanning more than kMaxLocalBins falls back to direct
// (unstaged) stores through the same cursors.
constexpr uint32_t kTile = 4096;      // elements per LDS-staged scatter tile
constexpr uint32_t kMaxLocalBins = 1024;

// exclusive scan of data[0..n) (n <= 1024) by a 512-thread block; returns the total
// exclusive scan of data[0, n) (n <= 2 T) by a block of T threads; wsum holds 2 T / 64 + 1 words
template <int T = 512>
__device__ __forceinline__ uint32_t block_scan(uint32_t* data, uint32_t n, uint32_t* wsum) {
    constexpr uint32_t NW = T / 64;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t i0 = 2 * tid, i1 = 2 * tid + 1;
    const uint32_t a = i0 < n ? data[i0] : 0u, b = i1 < n ? data[i1] : 0u;
    uint32_t v = a + b, incl = v;
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    if (tid < NW) {
        uint32_t run = 0;
        for (uint32_t w = 0; w < NW; ++w) {
            const uint32_t t = wsum[w];
            if (w == tid) wsum[NW + w] = run;
            run += t;
        }
        if (tid == 0) wsum[2 * NW] = run;
    }
    __syncthreads();
    const uint32_t excl = incl - v + wsum[NW + wave];
    if (i0 < n) data[i0] = excl;
    if (i1 < n) data[i1] = excl + a;
    const uint32_t total = wsum[2 * NW];
    __syncthreads();
    return total;
}

template <bool COARSE, bool HAS_IDX>
__global__ __launch_bounds__(512) void k_pc_scatter_lds(Tbl t, PartWs w, uint32_t bins,
                                                        const uint64_t* __restrict__ src,
                                                        const uint32_t* __restrict__ src_idx,
                                                        uint64_t* __restrict__ dst, uint32_t* __restrict__ dst_idx,
                                                        uint64_t n) {
    constexpr int T = 512;
    __shared__ uint32_t cursor[kMaxLocalBins];
    __shared__ uint32_t lstart[kMaxLocalBins];
    __shared__ uint32_t lcount[kMaxLocalBins];
    __shared__ uint64_t skey[kTile];
    __shared__ uint32_t sidx[kTile];
    __shared__ uint16_t sbin[kTile];
    __shared__ uint32_t wsum[17];
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = min(n, lo + per);
    if (lo >= hi) return;
    // active bin window of this block
    uint32_t bin_lo = 0, nb = bins;
    if constexpr (!COARSE) {
        const uint32_t shift = w.rbits > kCoarseBits ? (w.rbits - kCoarseBits) : 0;
        const uint32_t c0 = region_of(t, src[lo]) >> shift, c1 = region_of(t, src[hi - 1]) >> shift;
        bin_lo = c0 << shift;
        nb = (c1 - c0 + 1) << shift;
    }
    const bool staged = nb <= kMaxLocalBins;
    if (staged) {
        for (uint32_t i = threadIdx.x; i < nb; i += T) cursor[i] = w.hist[(uint64_t)blockIdx.x * bins + bin_lo + i];
    }
    __syncthreads();
    if (!staged) {   // rare (a block spanning many tiny coarse buckets): direct stores, global offsets
        for (uint64_t r = lo + threadIdx.x; r < hi; r += T) {
            const uint64_t key = src[r];
            const uint32_t b = bin_of<COARSE>(t, w, key);
            const uint32_t pos = atomicAdd(&w.hist[(uint64_t)blockIdx.x * bins + b], 1u);
            dst[pos] = key;
            dst_idx[pos] = HAS_IDX ? src_idx[r] : (uint32_t)r;
        }
        return;
    }
    // register double buffer: the next tile's keys / indices load while this tile is ranked,
    // scanned and written out
    uint64_t nkey[kTile / T];
    uint32_t nidx[kTile / T];
    auto load_tile = [&](uint64_t t0) {
        const uint32_t cnt = (uint32_t)min((uint64_t)kTile, hi - t0);
#pragma unroll
        for (int j = 0; j < (int)(kTile / T); ++j) {
            const uint32_t e = j * T + threadIdx.x;
            if (e < cnt) {
                nkey[j] = src[t0 + e];
                nidx[j] = HAS_IDX ? src_idx[t0 + e] : (uint32_t)(t0 + e);
            }
        }
    };
    load_tile(lo);
    for (uint64_t t0 = lo; t0 < hi; t0 += kTile) {
        const uint32_t cnt = (uint32_t)min((uint64_t)kTile, hi - t0);
        for (uint32_t i = threadIdx.x; i < nb; i += T) lcount[i] = 0;
        __syncthreads();
        uint64_t key[kTile / T];
        uint32_t idx[kTile / T], lb[kTile / T], rank[kTile / T];
#pragma unroll
        for (int j = 0; j < (int)(kTile / T); ++j) {
            key[j] = nkey[j];
            idx[j] = nidx[j];
        }
        if (t0 + kTile < hi) load_tile(t0 + kTile);
#pragma unroll
        for (int j = 0; j < (int)(kTile / T); ++j) {
            const uint32_t e = j * T + threadIdx.x;
            if (e < cnt) {
                lb[j] = bin_of<COARSE>(t, w, key[j]) - bin_lo;
                rank[j] = atomicAdd(&lcount[lb[j]], 1u);
            }
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nb; i += T) lstart[i] = lcount[i];
        __syncthreads();
        block_scan<T>(lstart, nb, wsum);
#pragma unroll
        for (int j = 0; j < (int)(kTile / T); ++j) {
            const uint32_t e = j * T + threadIdx.x;
            if (e < cnt) {
                const uint32_t sp = lstart[lb[j]] + rank[j];
                skey[sp] = key[j];
                sidx[sp] = idx[j];
                sbin[sp] = (uint16_t)lb[j];
            }
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < cnt; i += T) {
            const uint32_t b = sbin[i];
            const uint32_t gpos = cursor[b] + (i - lstart[b]);
            dst[gpos] = skey[i];
            dst_idx[gpos] = sidx[i];
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nb; i += T) cursor[i] += lcount[i];
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// Optimistic coarse partition (the C5 path for L 16 / 32, > 128 regions).  The exact passes above
// need a histogram of the whole batch before the coarse scatter (P1 writes every key, P3 reads
// them back).  Here the encode pass scatters directly: each 4096-read tile is ranked by coarse
// bin in LDS and reserves its runs with ONE atomicAdd per (tile, bin) on a fill counter.  Every bin
// is split into kFinePerBin sub-bins, one per fine-pass block; coarse block k appends to sub-bin
// k % kFinePerBin, so each counter takes 1/8 of the bin's atomics (the atomics on one address
// serialize: 128 shared counters cost ~0.57 ms of the pass at 125M reads, 8 x 128 cost the pass
// 1.54 -> 1.28 ms, profiles/r1/r1k/c5_coarse_probes.txt), while the 64 blocks that share a
// sub-bin still fill its lines back to back.  Sub-bin f = (bin, sub) owns slots [f * cap1,
// (f + 1) * cap1) of the coarse arrays (cap1 = 2.5 x the mean sub-bin load + 1024).  Order inside
// a sub-bin is arbitrary, which the aggregation does not care about (count = sum, first = min of
// the carried read index).
// Skew (counter.pyx:41-54 counts every duplicate; real read sets and Zipf pools repeat a few keys
// very often): a bin holding more than kHeavy reads of a tile (2x the mean of 32) is deduplicated in
// LDS before its reservation: every distinct key of the bin leaves the tile as ONE record, with its
// copy count (a weighted record, kWeighted) when it occurred more than once, and the minimum read
// index.  A hot key therefore costs one record per tile, and a bin that was not deduplicated holds at
// most 2x the mean per tile, which the 2.5x sub-bin capacity absorbs.  Records that still find their
// sub-bin full (crafted inputs: thousands of distinct keys in one bin) go to the spill list, which
// k_spill_insert counts into the table after the aggregate (exact; no whole-batch fallback).
// Fine pass: block f takes sub-bin f whole; all of its keys lie in the bin's 2^(rbits - 7)
// regions, so the histogram and the LDS staging use that window.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kCB = 1u << kCoarseBits;          // 128 coarse bins
// The fill counters take one atomicAdd per (4096-read tile, bin pair), ~2M device-scope atomics per
// 125M reads; spacing them apart measured no different from packing them.
constexpr uint32_t kFinePerBin = 8;                  // fine-pass blocks per coarse bin = sub-bins per bin
constexpr uint32_t kNFill = kCB * kFinePerBin;       // sub-bin fill counters
constexpr uint32_t kSpillCtr = kNFill;               // the spill list's record counter
constexpr uint32_t kFillWords = kNFill + 1;          // counters + the spill counter
// Sub-bins (2p, s) and (2p + 1, s) of a coarse bin pair share one 64-bit word (low / high half), so
// the coarse pass reserves both bins a wave-0 lane scans with ONE 64-bit atomic (a sub-bin's fill
// stays below 2^31: no carry into the high half).  fb = bin * kFinePerBin + sub.
__host__ __device__ __forceinline__ uint32_t fill_at(uint32_t fb) {
    const uint32_t bin = fb / kFinePerBin, sub = fb % kFinePerBin;
    return (((bin >> 1) * kFinePerBin + sub) << 1) | (bin & 1u);
}
// k_pf_coarse shape: 512 threads x 8 reads per 4096-read tile, capped at 128 VGPRs (4 waves per
// SIMD: two 72-KB-LDS blocks per CU, 16 waves).  Against 256 x 16 at 230 VGPRs (8 waves per CU):
// coarse 1.30 -> 1.19 ms uniform, 1.87 -> 1.40 ms Zipf 1.1 (its dedup phases are latency-bound);
// insert medians 2.87 -> 2.83 / 3.28 -> 2.80 ms.  1024 x 4: 1.38 / 1.86 ms.  Measured and not kept
// (DESIGN.md §4): the next tile's loads issued early, the reservation consumed after staging, the
// bin recomputed instead of staged, nontemporal record loads.
constexpr uint32_t kPfT = 512, kPfRPL = 8;   // k_pf_coarse: kPfT * kPfRPL-read tiles
constexpr uint32_t kHeavy = 64;              // reads of one bin in one tile above which the bin is deduplicated (2x the mean)

// sub-bin capacity of the optimistic partition for a batch of n reads (host and device agree)
__host__ __device__ __forceinline__ uint64_t pf_cap1(uint64_t n) {
    return ((5 * n / 2 + kNFill - 1) / kNFill + 1024 + 15) & ~15ull;   // x16: k_pf_count's dwordx4 loads
}

// 64-bit lane broadcast
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int lane) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, lane), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// Wave-level fold of lanes that share a key (hot keys fill whole waves of a skewed bucket): up to
// PEELS times, the active lanes whose key equals the key of the lowest active lane not yet folded
// into are folded into that lane (count summed, index min); the folded lanes turn inactive.  A peel
// costs one ballot + broadcast, and a 6-step sum / min only when at least two lanes match.  All 64
// lanes must call it (uniform control flow); returns with the surviving lanes active.  A peel whose
// key is unique in the wave ends the fold, or with kPastSingles passes over that lane.
template <int PEELS, bool kPastSingles = false>
__device__ __forceinline__ void wave_fold(bool& act, uint64_t key, uint32_t& cnt, uint32_t& idx) {
    const int lane = (int)(threadIdx.x & 63);
    bool led = false;
#pragma unroll
    for (int peel = 0; peel < PEELS; ++peel) {
        const uint64_t cand = __ballot(act && !led);
        if (!cand) break;
        const int leader = __ffsll((long long)cand) - 1;
        const uint64_t lk = shfl64(key, leader);
        const bool m = act && key == lk;
        const uint64_t mm = __ballot(m);
        if (__popcll(mm) < 2) {   // the lowest candidate's key is unique in the wave
            if (!kPastSingles) break;
            led = led || lane == leader;
            continue;
        }
        uint32_t cs = m ? cnt : 0u, mi = m ? idx : 0xFFFFFFFFu;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            cs += (uint32_t)__shfl_xor((int)cs, off);
            const uint32_t o = (uint32_t)__shfl_xor((int)mi, off);
            mi = o < mi ? o : mi;
        }
        if (m) {
            if (lane == leader) {
                cnt = cs;
                idx = mi;
                led = true;
            } else {
                act = false;
            }
        }
    }
}

// wave_fold peels in the coarse dedup and the spill insert.  Same-box A/B (125M reads, 3 rounds):
// a fine-dedup peel costs (Zipf scatter 0.90 -> 1.22 ms), aggregate peels cost (Zipf 3.59 -> 3.67 ms,
// uniform +0.03 ms: the fine dedup already bounds a region's copies of one key to ~1 per tile), so
// those have none.
constexpr int kCoarseFold = 1;   // 512 x 8 coarse tiles: 1 peel, Zipf coarse 1.40 -> 1.35 ms (2 peels: no better)
constexpr int kSpillFold = 8;    // Zipf 1.1 over 2^24: 278k spilled records, insert 0.30 -> 0.12 (4 peels) -> 0.09 ms (8)

// LDS dedup table of one tile: entry = (staged element + 1) | count << 16, 0 = free
__device__ __forceinline__ uint32_t dedup_home(uint64_t key, uint32_t log2n) {
    return (uint32_t)((key * 0xD6E8FEB86659FD93ull) >> (64 - log2n));
}

// KEYS: the keys come precomputed (in = n u64 keys, e.g. the drop-in engine's row fingerprints;
// stride16 / cpr / first_bad unused) instead of being encoded from 16 / 32-nt ASCII rows.
// G16 (32-nt rows, round 6): the tile is loaded in k_encode_g16's shape -- per step, lane l of a wave
// loads 16-B chunk (l & 1) of read (l >> 1) and of read 32 + (l >> 1), so each load instruction
// covers 1 KB of contiguous ASCII (the lane-per-read form loaded 16 B at a 32-B lane stride: every
// instruction touched 16 half-used lines, and the second instruction the same lines again); one DPP
// pair swap then hands the even lane read (l >> 1)'s high half and the odd lane read 32 + (l >> 1)'s
// low half (and its table-path carry), so every lane again holds one whole key.
// Staging (round 6): a tile element is its key (skey) and ONE meta word (tile offset | bin << 16 |
// kMetaDead), where the former kept the global read index and a bin byte apart (three random LDS
// stores per element, five LDS reads per record in the write-out: bin, the bin's start and base, key,
// index); a bin's start and reservation base are folded into one delta word (sdelta), so a record
// takes three LDS reads: meta, key, delta.
constexpr uint32_t kMetaDead = 0x80000000u;   // staged element folded into another (no record)
template <int T, int RPL, bool KEYS, bool G16>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(4))) void k_pf_coarse(
        Tbl t, PartWs w, const uint4* __restrict__ in, uint64_t stride16, uint64_t n, uint32_t cpr, uint64_t cap1,
        uint32_t* fill, unsigned long long* first_bad) {
    constexpr uint32_t TILE = T * RPL;
    constexpr uint32_t kHtLog = TILE == 4096 ? 12 : TILE == 2048 ? 11 : 13;
    static_assert((1u << kHtLog) == TILE, "tile must be 2048, 4096 or 8192 reads");
    static_assert(!(KEYS && G16), "G16 encodes ASCII rows");
    __shared__ uint32_t lcount[kCB], lstart[kCB], gbase[kCB], hcnt[kCB], sbase[kCB], sdelta[kCB];
    __shared__ uint8_t hflag[kCB];
    __shared__ uint32_t any_heavy;
    __shared__ uint64_t skey[TILE];
    __shared__ uint32_t smeta[TILE];
    __shared__ uint32_t ht[TILE];
    uint32_t* spill_ctr = fill + fill_at(kSpillCtr);
    const uint32_t shift = w.rbits - kCoarseBits;
    const uint64_t tiles = (n + TILE - 1) / TILE;
    const uint32_t sub = blockIdx.x % kFinePerBin;   // this block's sub-bin of every bin
    const uint32_t lane = threadIdx.x & 63u, wbase = threadIdx.x & ~63u;
    const bool odd = (lane & 1u) != 0;
    // tile offset of the read a lane holds at step j (G16: the lane-pair permutation of the wave's 64)
    // (el: the lane's step-0 offset, made opaque per tile below so that the compiler recomputes the
    // RPL offsets in each tile instead of keeping them all live across the tile loop)
    const uint32_t el0 = G16 ? wbase + ((lane & 1u) << 5) + (lane >> 1) : threadIdx.x;
    uint32_t el = el0;
    auto eoff = [&](int j) -> uint32_t { return (uint32_t)j * T + el; };
    uint4 nx[RPL][2];
    uint64_t nk[RPL];
    // branch-free loads (read index clamped to the last read; lanes past n are never live): the
    // compiler then waits for each chunk just before its encode instead of for all 2 * RPL loads
    const uint32_t hi16 = cpr > 1 ? 1u : 0u;    // L = 16: one chunk (the high half reads 'A's below)
    // G16: read A's tile-relative index at step 0 (read B = + 32); inside a tile the index math is
    // 32-bit from a per-tile base (the 64-bit clamp and multiply per load cost ~10 VALU each, ~1/8 of
    // the pass's VALU, and held 64-bit indices live through the encode)
    const uint32_t s16 = (uint32_t)stride16, relA0 = wbase + (lane >> 1);
    uint32_t relA = relA0;                      // (opaque per tile, as el)
    auto load_tile = [&](uint64_t tile) {
        const uint32_t offA = relA * s16 + (lane & 1u);     // in 16-B units
        const uint64_t tb = tile * TILE;
        const uint4* ub = in + tb * stride16;                                // the tile's rows (uniform)
        // a partial last tile clamps every offset to its last read's high chunk (lanes past n are
        // never live); a full tile's bound is no bound
        const uint32_t lim = tb + TILE <= n ? 0xFFFFFFFFu : (uint32_t)(n - 1 - tb) * s16 + 1u;
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            if constexpr (G16) {
                nx[j][0] = ld_stream(ub + min(offA + (uint32_t)j * T * s16, lim));
                nx[j][1] = ld_stream(ub + min(offA + ((uint32_t)j * T + 32u) * s16, lim));
            } else {
                const uint64_t r = min(tile * TILE + j * T + threadIdx.x, n - 1);
                if constexpr (KEYS) {
                    nk[j] = ((const uint64_t*)in)[r];
                } else {
                    nx[j][0] = ld_stream(&in[r * stride16]);
                    nx[j][1] = ld_stream(&in[r * stride16 + hi16]);
                }
            }
        }
    };
    // wave 0 lane, bins b0 = 2 lane and b0 + 1: reserve c0 / c1 slots of their sub-bins (b, sub) with
    // one 64-bit atomic on the pair's word (only the bins flagged in `mask`: bit 0 = b0, bit 1 =
    // b0 + 1); the part past cap1 reserves spill records (a second atomic, rare).  Sets the bins'
    // bases (gbase, and sdelta = base - start), and spill runs (sbase).
    auto reserve = [&](uint32_t b0, uint32_t c0, uint32_t c1, uint32_t mask) {
        const uint64_t add = ((mask & 1u) ? (uint64_t)c0 : 0ull) | ((mask & 2u) ? (uint64_t)c1 << 32 : 0ull);
        const uint64_t g2 = add ? atomicAdd((unsigned long long*)&fill[fill_at(b0 * kFinePerBin + sub)],
                                            (unsigned long long)add)
                                : 0ull;
#pragma unroll
        for (uint32_t k = 0; k < 2; ++k) {
            if (!(mask & (1u << k))) continue;
            const uint32_t g = (uint32_t)(g2 >> (32 * k)), c = k ? c1 : c0;
            gbase[b0 + k] = g;
            sdelta[b0 + k] = g - lstart[b0 + k];
            const uint64_t end = (uint64_t)g + c, from = max((uint64_t)g, cap1);
            sbase[b0 + k] = end > from ? atomicAdd(spill_ctr, (uint32_t)(end - from)) : 0u;
        }
    };
    static_assert(kCB == 128, "wave 0 scans two bins per lane");
    for (uint32_t i = threadIdx.x; i < kCB; i += T) lcount[i] = 0;
    __syncthreads();
    // three barriers per tile: (A) ranks counted, (B) wave 0 has scanned the bins, reserved the
    // tile's runs in the global bins and zeroed the counters for the next tile, (C) tile staged in
    // LDS.  The next tile's rank atomics only touch lcount (zeroed before B) and its staging waits
    // for its own barrier B, which every wave reaches only after this tile's write-out.  A tile with
    // a heavy bin adds three: (D) deduplicated, (E) survivors counted, (F) heavy bins reserved.
    for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        relA = relA0;
        el = el0;
        asm volatile("" : "+v"(relA), "+v"(el));
        load_tile(tile);
        uint64_t key[RPL];
        uint32_t br[RPL];     // bin << 16 | rank in the bin (one register per read)
        const uint64_t t0 = tile * TILE;
        const uint32_t cnt = (uint32_t)min((uint64_t)TILE, n - t0);
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const bool live = eoff(j) < cnt;
            if constexpr (KEYS) {
                key[j] = nk[j];
            } else if constexpr (G16) {
                // chunk (lane & 1) of read A = (lane >> 1) and of read B = 32 + (lane >> 1), table path
                const Enc32 a = encode16(nx[j][0].x, nx[j][0].y, nx[j][0].z, nx[j][0].w, true);
                const Enc32 b = encode16(nx[j][1].x, nx[j][1].y, nx[j][1].z, nx[j][1].w, true);
                const uint32_t recv = swap_pair(odd ? a.v : b.v);    // even: A's high half; odd: B's low half
                const uint32_t bc = swap_pair(b.cout);               // odd: the carry out of B's low half
                const uint32_t lo = odd ? recv : a.v;
                const uint32_t hi = odd ? (b.v | bc) : (recv | a.cout);
                const uint32_t ra = (uint32_t)j * T + relA;      // tile-relative
                report_bad(ra < cnt && a.bad != 0u, t0 + ra, first_bad);
                report_bad(ra + 32u < cnt && b.bad != 0u, t0 + ra + 32u, first_bad);
                key[j] = (uint64_t)lo | ((uint64_t)hi << 32);
            } else {
                const uint64_t r = t0 + j * T + threadIdx.x;
                // table path for both chunks (L <= 32); the low chunk's alias carry into the high half
                const Enc32 a = encode16(nx[j][0].x, nx[j][0].y, nx[j][0].z, nx[j][0].w, true);
                const uint4 h = hi16 ? nx[j][1] : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
                const Enc32 b = encode16(h.x, h.y, h.z, h.w, true);
                report_bad(live && (a.bad | b.bad) != 0u, r, first_bad);
                key[j] = (uint64_t)a.v | ((uint64_t)(b.v | a.cout) << 32);
            }
            key[j] *= kSlotMul;                                          // h from here on
            if (live) {
                const uint32_t b = region_of_h(t, key[j]) >> shift;
                br[j] = (b << 16) | atomicAdd(&lcount[b], 1u);
            }
        }
        __syncthreads();                                                  // (A)
        if (threadIdx.x < 64) {       // wave 0: scan, heavy flags, the reservation atomic of bins 2 lane, 2 lane + 1
            const uint32_t b0 = 2 * lane;
            const uint32_t c0 = lcount[b0], c1 = lcount[b0 + 1];
            uint32_t incl = c0 + c1;
            for (uint32_t off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(incl, off);
                if (lane >= off) incl += y;
            }
            const uint32_t excl = incl - c0 - c1;
            lstart[b0] = excl;
            lstart[b0 + 1] = excl + c0;
            const bool h0 = c0 > kHeavy, h1 = c1 > kHeavy;
            hflag[b0] = h0;
            hflag[b0 + 1] = h1;
            reserve(b0, c0, c1, (h0 ? 0u : 1u) | (h1 ? 0u : 2u));
            const uint64_t hv = __ballot(h0 || h1);
            if (lane == 0) any_heavy = hv != 0;
            lcount[b0] = 0;
            lcount[b0 + 1] = 0;
            hcnt[b0] = 0;
            hcnt[b0 + 1] = 0;
        }
        __syncthreads();                                                  // (B)
        const bool heavy_tile = any_heavy != 0;
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const uint32_t e = eoff(j);
            if (e < cnt) {
                const uint32_t sp = lstart[br[j] >> 16] + (br[j] & 0xFFFFu);
                skey[sp] = key[j];
                smeta[sp] = e | (br[j] & 0xFFFF0000u);
            }
        }
        if (heavy_tile)
            for (uint32_t i = threadIdx.x; i < TILE; i += T) ht[i] = 0;
        __syncthreads();                                                  // (C)
        if (heavy_tile) {
            // (D) every element of a heavy bin claims its key's entry or folds into the claimer's:
            // count += c in the entry, tile offset min into the claimer's meta, element marked dead.
            // Staged elements are bin-sorted, so a wave's lanes often share a hot key: those fold
            // in registers first (one LDS atomic per wave instead of 64 on one address).
            for (uint32_t i0 = 0; i0 < cnt; i0 += T) {
                const uint32_t i = i0 + threadIdx.x;
                const uint32_t meta = i < cnt ? smeta[i] : 0u, b = (meta >> 16) & (kCB - 1);
                bool act = i < cnt && hflag[b];
                const uint64_t k = act ? skey[i] : 0ull;
                uint32_t c = 1, mi = act ? (meta & 0xFFFFu) : 0xFFFFFFFFu;
                const bool was = act;
                wave_fold<kCoarseFold>(act, k, c, mi);
                if (was && !act) smeta[i] = meta | kMetaDead;             // folded into its wave leader
                if (!act) continue;
                smeta[i] = mi | (b << 16);
                uint32_t h = dedup_home(k, kHtLog);
                for (;;) {
                    uint32_t e = ht[h];
                    if (e == 0) {
                        e = atomicCAS(&ht[h], 0u, (i + 1) | (c << 16));
                        if (e == 0) break;
                    }
                    const uint32_t j = (e & 0xFFFFu) - 1;
                    if (skey[j] == k) {
                        atomicAdd(&ht[h], c << 16);
                        atomicMin(&smeta[j], mi | (b << 16));   // (same bin: the min is the offset's)
                        smeta[i] = kMetaDead;
                        break;
                    }
                    h = (h + 1) & (TILE - 1);
                }
            }
            __syncthreads();                                              // (D)
            for (uint32_t i = threadIdx.x; i < cnt; i += T) {
                const uint32_t meta = smeta[i], b = (meta >> 16) & (kCB - 1);
                if (!(meta & kMetaDead) && hflag[b]) atomicAdd(&hcnt[b], 1u);
            }
            __syncthreads();                                              // (E)
            if (threadIdx.x < 64) {
                const uint32_t b0 = 2 * threadIdx.x;
                reserve(b0, hcnt[b0], hcnt[b0 + 1], (hflag[b0] ? 1u : 0u) | (hflag[b0 + 1] ? 2u : 0u));
                hcnt[b0] = 0;     // now the heavy bins' write cursors
                hcnt[b0 + 1] = 0;
            }
            __syncthreads();                                              // (F)
        }
        for (uint32_t i = threadIdx.x; i < cnt; i += T) {
            const uint32_t meta = smeta[i];
            if (meta & kMetaDead) continue;                               // folded into its claimer
            const uint32_t b = (meta >> 16) & (kCB - 1);
            uint32_t c = 1;
            uint64_t pos;
            if (heavy_tile && hflag[b]) {
                pos = (uint64_t)gbase[b] + atomicAdd(&hcnt[b], 1u);
                uint32_t h = dedup_home(skey[i], kHtLog);
                while ((ht[h] & 0xFFFFu) != i + 1) h = (h + 1) & (TILE - 1);
                c = ht[h] >> 16;
            } else {
                pos = (uint32_t)(i + sdelta[b]);                          // base + (i - start)
            }
            const uint64_t k = skey[i];
            const uint32_t idx = (uint32_t)t0 + (meta & 0xFFFFu);
            if (pos < cap1) {
                const uint64_t at = (uint64_t)(b * kFinePerBin + sub) * cap1 + pos;
                Rec12 r;
                r.klo = (uint32_t)k;
                r.khi = (uint32_t)(k >> 32);
                r.idx = c > 1 ? (idx | kWeighted) : idx;
                ((Rec12*)w.akey)[at] = r;
                if (!w.slab) w.areg[at] = (uint8_t)(region_of_h(t, k) & ((1u << shift) - 1u));
                if (c > 1) w.acnt[at] = c;
            } else {
                const uint64_t sp = (uint64_t)sbase[b] + (pos - max((uint64_t)gbase[b], cap1));
                const uint64_t key = k * kSlotInv;                           // (the spill takes keys)
                if (sp < w.spill_cap)
                    w.spill[sp] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), c, idx);
                else
                    atomicOr(t.overflow, kOvfTable);
            }
        }
    }
}

// fine block fb = sub-bin fb (bin fb / kFinePerBin): slots [fb * cap1, fb * cap1 + fill)
__device__ __forceinline__ void fine_range(uint32_t fb, const uint32_t* fill, uint64_t cap1, uint32_t& bin,
                                           uint64_t& lo, uint64_t& hi) {
    bin = fb / kFinePerBin;
    lo = 0;
    hi = min((uint64_t)fill[fill_at(fb)], cap1);
}

// fine histogram: block fb counts the regions of its slice of coarse bin fb / 8 -> hist[fb][rpb]
template <int T>
__global__ __launch_bounds__(T) void k_pf_count(Tbl t, PartWs w, uint64_t cap1, const uint32_t* fill) {
    __shared__ uint32_t h[kMaxLocalBins];
    const uint32_t rpb = 1u << (w.rbits - kCoarseBits);
    uint32_t bin;
    uint64_t lo, hi;
    fine_range(blockIdx.x, fill, cap1, bin, lo, hi);
    for (uint32_t i = threadIdx.x; i < rpb; i += T) h[i] = 0;
    __syncthreads();
    // the coarse pass wrote each record's region-in-bin byte (1 B per record instead of the 8-B key)
    const uint4* src = (const uint4*)(w.areg + (uint64_t)blockIdx.x * cap1);
    const uint64_t n16 = (hi - lo + 15) / 16;
    // four dwordx4 per thread per step, loaded branch-free (clamped) before any is counted
    constexpr int kQ = 4;
    for (uint64_t q0 = threadIdx.x; q0 < n16; q0 += (uint64_t)kQ * T) {
        uint4 v[kQ];
#pragma unroll
        for (int u = 0; u < kQ; ++u) v[u] = src[min(q0 + (uint64_t)u * T, n16 - 1)];
#pragma unroll
        for (int u = 0; u < kQ; ++u) {
            const uint64_t q = q0 + (uint64_t)u * T;
            if (q >= n16) break;
            const uint32_t m = (uint32_t)min((uint64_t)16, hi - 16 * q);
            const uint32_t wd[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (uint32_t j = 0; j < 16; ++j) {
                const uint32_t r = (wd[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                if (j < m) atomicAdd(&h[r], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < rpb; i += T) w.hist[(uint64_t)blockIdx.x * rpb + i] = h[i];
}

// region totals over the bin's 8 fine blocks (thread per region) -> w.tot; then k_pc_scan (one
// block) -> rstart; then k_pf_offsets (thread per region) -> each fine block's write cursors
__global__ __launch_bounds__(256) void k_pf_tot(PartWs w) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= w.R) return;
    const uint32_t rpb = 1u << (w.rbits - kCoarseBits), bin = r / rpb, j = r % rpb;
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t sub = 0; sub < kFinePerBin; ++sub) tot += w.hist[(uint64_t)(bin * kFinePerBin + sub) * rpb + j];
    w.tot[r] = tot;
}

__global__ __launch_bounds__(256) void k_pf_offsets(PartWs w) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= w.R) return;
    const uint32_t rpb = 1u << (w.rbits - kCoarseBits), bin = r / rpb, j = r % rpb;
    uint32_t cur = w.rstart[r];
#pragma unroll
    for (uint32_t sub = 0; sub < kFinePerBin; ++sub) {
        const uint64_t idx = (uint64_t)(bin * kFinePerBin + sub) * rpb + j;
        const uint32_t c = w.hist[idx];
        w.hist[idx] = cur;
        cur += c;
    }
}

// Largest sub-bin first: order[k] = the sub-bin with the k-th largest fill (ties by index), so the
// fine scatter's blocks (dispatched in blockIdx order) start the long ones first and the pass does
// not end on a skewed sub-bin that started last.  One block: bitonic sort of (~fill, index) in LDS.
__global__ __launch_bounds__(512) void k_pf_order(const uint32_t* __restrict__ fill, uint64_t cap1,
                                                  uint32_t* __restrict__ order, uint32_t nb,
                                                  uint32_t* __restrict__ slabs) {
    static_assert(kNFill == 1024, "one 512-thread block sorts 1024 sub-bins");
    __shared__ uint64_t v[kNFill];
    __shared__ uint32_t base[kNFill];
    __shared__ uint32_t wsum[2 * (512 / 64) + 1];
    for (uint32_t i = threadIdx.x; i < kNFill; i += 512) {
        const uint32_t f = (uint32_t)min((uint64_t)fill[fill_at(i)], cap1);
        v[i] = ((uint64_t)~f << 32) | i;      // ascending = fill descending, then index
        if (slabs) base[i] = nb * slab_size(f, nb);
    }
    __syncthreads();
    if (slabs) {   // slab bases: sub-bins back to back in index order, each nb slabs of its size
        block_scan<512>(base, kNFill, wsum);
        for (uint32_t i = threadIdx.x; i < kNFill; i += 512) {
            slabs[i] = base[i];
            slabs[kNFill + i] = slab_size((uint32_t)~(v[i] >> 32), nb);
        }
        __syncthreads();
    }
    for (uint32_t k = 2; k <= kNFill; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            const uint32_t t = threadIdx.x;
            const uint32_t i = 2 * j * (t / j) + (t % j), l = i + j;   // the pair (i, l), i < l
            const bool up = (i & k) == 0;
            const uint64_t a = v[i], b = v[l];
            if ((a > b) == up) {
                v[i] = b;
                v[l] = a;
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < kNFill; i += 512) order[i] = (uint32_t)v[i];
}

// fine scatter: coarse bin slice -> (key, read index) grouped by region, LDS-staged like
// k_pc_scatter_lds (local bins = the coarse bin's regions).  A weighted record is staged with its
// position in the sub-bin instead of its read index; the write-out fetches its index and count.
// Region-level skew (a key too rare to make its coarse bin heavy can still hold a large share of its
// region: Zipf rank 13 is 0.7 % of all reads = 110x a region's mean): a region holding more than
// kHeavyFine records of a 4096-record tile is deduplicated like the coarse pass's heavy bins
// (unweighted records only; each distinct key leaves as one record, weighted when repeated).  The
// (sub-bin, region) segments then end before their reserved size; the end of each is written to
// w.seg_end and the aggregate reads only the written part.
constexpr uint32_t kHeavyFine = 2;    // x the mean records per region per tile
constexpr uint32_t kFsT = 1024, kFsTile = 8192;  // k_pf_scatter block and tile (512 x 4096: +4 % C5, same box)
template <int T, uint32_t kTile>
__global__ __launch_bounds__(T) void k_pf_scatter(Tbl t, PartWs w, uint64_t cap1, const uint32_t* fill,
                                                  const uint32_t* __restrict__ order) {
    constexpr uint32_t kHtLog = kTile == 2048 ? 11 : kTile == 4096 ? 12 : 13;
    static_assert(kTile == (1u << kHtLog), "fine tile = dedup table size");
    constexpr uint32_t kDead = 0xFFFFFFFFu;
    // <= 256 regions per coarse bin on this path (rbits - 7 <= 8)
    constexpr uint32_t kNB = 256;
    __shared__ uint32_t cursor[kNB];
    __shared__ uint32_t lstart[kNB];
    __shared__ uint32_t lcount[kNB];
    __shared__ uint32_t hcnt[kNB];
    __shared__ uint64_t skey[kTile];
    __shared__ uint32_t sidx[kTile];
    __shared__ uint32_t ht[kTile];
    __shared__ uint32_t wsum[2 * (T / 64) + 1];
    __shared__ uint32_t any_heavy;
    const uint32_t nb = 1u << (w.rbits - kCoarseBits);
    const uint32_t heavy_at = max(64u, kHeavyFine * (kTile / nb));
    uint32_t bin;
    uint64_t lo, hi;
    const uint32_t fb = order[blockIdx.x];     // this block's sub-bin
    fine_range(fb, fill, cap1, bin, lo, hi);
    const uint32_t r0 = bin * nb;
    const Rec12* srec = (const Rec12*)w.akey + (uint64_t)fb * cap1;
    const uint32_t* src_cnt = w.acnt + (uint64_t)fb * cap1;
    const uint32_t sbase = w.slab ? w.slabs[fb] : 0u, ssize = w.slab ? w.slabs[kNFill + fb] : 0u;
    for (uint32_t i = threadIdx.x; i < nb; i += T) {
        cursor[i] = w.slab ? sbase + i * ssize : w.hist[(uint64_t)fb * nb + i];
        if (w.slab) w.hist[(uint64_t)fb * nb + i] = sbase + i * ssize;   // the aggregate's segment start
    }
    __syncthreads();
    uint64_t nkey[kTile / T];
    uint32_t nidx[kTile / T];
    // Unconditional loads (index clamped to the sub-bin's last record; lanes past the tile are never
    // used) with the raw index word kept: no branch and no use of a loaded value between the loads,
    // so a tile's loads all go out back to back (a conditional load, or transforming the index right
    // after loading it, makes the compiler wait for each load before issuing the next).
    auto load_tile = [&](uint64_t t0) {
#pragma unroll
        for (int j = 0; j < (int)(kTile / T); ++j) {
            const Rec12 r = srec[min(t0 + j * T + threadIdx.x, hi - 1)];
            nkey[j] = ((uint64_t)r.khi << 32) | r.klo;
            nidx[j] = r.idx;
        }
    };
    if (lo < hi) load_tile(lo);
    for (uint64_t t0 = lo; t0 < hi; t0 += kTile) {
        const uint32_t cnt = (uint32_t)min((uint64_t)kTile, hi - t0);
        for (uint32_t i = threadIdx.x; i < nb; i += T) lcount[i] = 0;
        if (threadIdx.x == 0) any_heavy = 0;
        __syncthreads();
        uint64_t key[kTile / T];
        uint32_t idx[kTile / T], lb[kTile / T], rank[kTile / T];
#pragma unroll
        for (int j = 0; j < (int)(kTile / T); ++j) {
            key[j] = nkey[j];
            // a weighted coarse record is staged with its position in the sub-bin (its index and
            // count are fetched at the write-out)
            idx[j] = (nidx[j] & kWeighted) ? kWeighted | (uint32_t)(t0 + j * T + threadIdx.x) : nidx[j];
        }
        load_tile(t0 + kTile);
#pragma unroll
        for (int j = 0; j < (int)(kTile / T); ++j) {
            const uint32_t e = j * T + threadIdx.x;
            if (e < cnt) {
                lb[j] = region_of_h(t, key[j]) - r0;
                rank[j] = atomicAdd(&lcount[lb[j]], 1u);
            }
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nb; i += T) {
            lstart[i] = lcount[i];
            hcnt[i] = 0;
            if (lcount[i] > heavy_at) any_heavy = 1;
        }
        __syncthreads();
        block_scan<T>(lstart, nb, wsum);
        const bool heavy_tile = any_heavy != 0;
#pragma unroll
        for (int j = 0; j < (int)(kTile / T); ++j) {
            const uint32_t e = j * T + threadIdx.x;
            if (e < cnt) {
                const uint32_t sp = lstart[lb[j]] + rank[j];
                skey[sp] = key[j];
                sidx[sp] = idx[j];
            }
        }
        if (heavy_tile)
            for (uint32_t i = threadIdx.x; i < kTile; i += T) ht[i] = 0;
        __syncthreads();
        if (heavy_tile) {
            for (uint32_t i0 = 0; i0 < cnt; i0 += T) {
                const uint32_t i = i0 + threadIdx.x;
                const uint64_t k = i < cnt ? skey[i] : 0ull;
                const uint32_t x = i < cnt ? sidx[i] : kWeighted;
                const bool act = i < cnt && lcount[region_of_h(t, k) - r0] > heavy_at && !(x & kWeighted);
                if (!act) continue;
                uint32_t h = dedup_home(k, kHtLog);
                for (;;) {
                    uint32_t e = ht[h];
                    if (e == 0) {
                        e = atomicCAS(&ht[h], 0u, (i + 1) | (1u << 16));
                        if (e == 0) break;
                    }
                    const uint32_t j = (e & 0xFFFFu) - 1;
                    if (skey[j] == k) {
                        atomicAdd(&ht[h], 1u << 16);
                        atomicMin(&sidx[j], x);
                        sidx[i] = kDead;
                        break;
                    }
                    h = (h + 1) & (kTile - 1);
                }
            }
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < cnt; i += T) {
                const uint32_t b = region_of_h(t, skey[i]) - r0;
                if (lcount[b] > heavy_at && sidx[i] != kDead) atomicAdd(&hcnt[b], 1u);
            }
            for (uint32_t i = threadIdx.x; i < nb; i += T)
                if (lcount[i] > heavy_at) lstart[i] = 0;    // now the heavy region's write cursor
            __syncthreads();
        }
        // Wait for the next tile's loads here, before this tile's record stores are issued: vmcnt
        // counts loads and stores in issue order, and with a data-dependent number of stores in
        // between, the wait at the next tile's first use would also drain this tile's stores
#pragma unroll
        for (int j = 0; j < (int)(kTile / T); ++j) asm volatile("" ::"v"(nkey[j]), "v"(nidx[j]));
        for (uint32_t i = threadIdx.x; i < cnt; i += T) {
            const uint64_t k = skey[i];
            const uint32_t x = sidx[i];
            if (x == kDead) continue;
            const uint32_t b = region_of_h(t, k) - r0;
            uint32_t local, c = 1;
            if (heavy_tile && lcount[b] > heavy_at) {
                local = atomicAdd(&lstart[b], 1u);
                if (!(x & kWeighted)) {
                    uint32_t h = dedup_home(k, kHtLog);
                    while ((ht[h] & 0xFFFFu) != i + 1) h = (h + 1) & (kTile - 1);
                    c = ht[h] >> 16;
                }
            } else {
                local = i - lstart[b];
            }
            uint32_t xi = x;          // the read index (weighted flag kept) and the count
            if (x & kWeighted) {
                const uint32_t p = x & ~kWeighted;
                xi = srec[p].idx;
                c = src_cnt[p];
            } else if (c > 1) {
                xi = x | kWeighted;
            }
            const uint32_t gpos = cursor[b] + local;
            if (w.slab && gpos >= sbase + (b + 1) * ssize) {
                // the region's slab of this sub-bin is full: the record goes to the spill list
                // (counted by k_spill_insert after the aggregate)
                const uint64_t sp = atomicAdd(w.spill_ctr, 1u);
                const uint64_t key = k * kSlotInv;                           // (the spill takes keys)
                if (sp < w.spill_cap)
                    w.spill[sp] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), c, xi & ~kWeighted);
                else
                    atomicOr(t.overflow, kOvfTable);
                continue;
            }
            if (c > 1) w.bcnt[gpos] = c;
            Rec12 r;
            r.klo = (uint32_t)k;
            r.khi = (uint32_t)(k >> 32);
            r.idx = xi;
            ((Rec12*)w.keys)[gpos] = r;
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nb; i += T)
            cursor[i] += (heavy_tile && lcount[i] > heavy_at) ? hcnt[i] : lcount[i];
        __syncthreads();
    }
    for (uint32_t i = threadIdx.x; i < nb; i += T)
        w.seg_end[(uint64_t)fb * nb + i] = w.slab ? min(cursor[i], sbase + (i + 1) * ssize) : cursor[i];
}

// Spilled records (sub-bin full) into the table with the direct insert, after the aggregate; a slot
// claimed here is added to its region's occupancy (ss_counter_pack_ranges reads it).
__global__ __launch_bounds__(256) void k_spill_insert(Tbl t, PartWs w, const uint32_t* __restrict__ fill,
                                                      uint64_t base_index) {
    const uint64_t m = min((uint64_t)fill[fill_at(kSpillCtr)], w.spill_cap);
    // wave-uniform trip count (the folds below are wave operations)
    for (uint64_t i0 = (uint64_t)blockIdx.x * 256; i0 < m; i0 += (uint64_t)gridDim.x * 256) {
        const uint64_t i = i0 + threadIdx.x;
        const uint4 r = w.spill[min(i, m - 1)];
        const uint64_t k = ((uint64_t)r.y << 32) | r.x;
        // a full slab spills a run of one region's records, mostly copies of its heavy keys (one
        // weighted record per coarse tile): fold a wave's copies before the global atomics
        bool act = i < m;
        uint32_t c = r.z, idx = r.w;
        wave_fold<kSpillFold, true>(act, k, c, idx);
        if (act && tbl_add(t, k, c, base_index + idx) && t.occ && k != kEmpty) atomicAdd(&t.occ[region_of(t, k)], 1u);
    }
}


constexpr uint32_t kAggSliceT = 512;   // P4 threads per region (256 / 1024: slower)
constexpr int kAggP = 4;               // records per thread per aggregate step (loads in flight)


// P4, slice-direct form: the region's slice itself is the LDS hash table.  Keys are copied into LDS
// (16 KB for 2048 slots) next to two per-batch u32 arrays (count, first read index); every bucket
// element probes the slice from its home slot (a new key claims an EMPTY slot with one LDS CAS),
// then one LDS add and one LDS min.  The whole slice is written back coalesced (key, count, first
// combined with the slot's old values; one dwordx4 per slot).  32 KB of LDS per workgroup.
// Skewed regions: the fine scatter's dedup leaves at most ~one record per (tile, hot key), and
// weighted records carry their counts (one LDS add of c); folding lanes that share a key before the
// LDS atomics measured slower (see wave_fold).
// fresh: the table was reset and the reset is still pending (ss_counter_reset is lazy): the slice is
// taken as empty instead of loaded, and written back whole (empty slots as the 0xFF reset pattern),
// which replaces the table-sized reset memset and the slice read.
// Linear probe of an LDS slice (mask + 1 slots) for `key` from its home slot: the first slot
// holding the key, or the first free one, claimed with an LDS CAS (a slot another lane claimed
// for a different key first moves the probe on past it) -- the same slot sequential linear probing
// gives.  G slots are read per round (G independent LDS reads, one wait).
constexpr int kAggProbe = 2;   // probe rounds of 1 / 2 / 4 / 8 slots: aggregate 0.72 / 0.58 / 0.60 / 0.63 ms (U 2^24)
constexpr int kAggProbeS = 4;  // straggler rounds (aggregate, merge): 2 / 4 slots 0.52 / 0.49 ms U 2^24, 0.53 / 0.48 ms U 2^20
// One probe round of G slots from `off` (the rule above): true with `at` = the
// key's slot (found, or claimed by an LDS CAS) or S (the slice is full); false with off / done
// advanced past the round.  The aggregate and the owner merge give every record one round first,
// straight-line, and then walk each lane's unfinished records one after another (see there).
template <int G>
__device__ __forceinline__ bool lds_probe_round(unsigned long long* skey, uint32_t mask, uint64_t empty, uint64_t k,
                                                uint32_t& off, uint32_t& done, uint32_t& at) {
    const uint32_t S = mask + 1;
    unsigned long long cur[G];
#pragma unroll
    for (int g = 0; g < G; ++g) cur[g] = skey[(off + g) & mask];
    int hit = -1;
    bool free_at = false;
#pragma unroll
    for (int g = G - 1; g >= 0; --g) {
        if (cur[g] == k) {
            hit = g;
            free_at = false;
        } else if (cur[g] == empty) {
            hit = g;
            free_at = true;
        }
    }
    if (hit >= 0) {
        at = (off + (uint32_t)hit) & mask;
        if (!free_at) return true;
        const unsigned long long prev = atomicCAS(&skey[at], (unsigned long long)empty, (unsigned long long)k);
        if (prev == empty || prev == k) return true;
        off = (at + 1) & mask;                 // taken by another key: go on after it
        done += (uint32_t)hit + 1;
    } else {
        off = (off + G) & mask;
        done += G;
    }
    at = S;
    return done >= S;
}

// One block per region (a persistent grid walking the regions measured slower: aggregate 0.63 ->
// 0.87 ms, the loop form costs 58 -> 80 VGPRs).
template <int T, bool REC12>
__global__ __launch_bounds__(T) void k_pc_aggregate_slice(Tbl t, PartWs w, uint64_t base_index, bool fresh = false) {
    const uint32_t S = (uint32_t)t.slice_mask + 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long* skey = (unsigned long long*)smem;   // [S]
    uint32_t* bcnt = (uint32_t*)(skey + S);                   // [S] this batch's count
    uint32_t* bfst = bcnt + S;                                // [S] this batch's first read index
    __shared__ uint32_t sent[3];   // sentinel count, sentinel first, slice occupancy
    const uint32_t region = blockIdx.x;
    const uint64_t slice_base = (uint64_t)region << t.slice_log;
    // The region's segment table first, one vector load per lane (lanes 0-7 the segment starts,
    // 8-15 the ends; exact paths: lanes 0 / 1 the range), read back with readlane: ONE round trip,
    // issued before the LDS fill.  As scalar loads the compiler waited for each (start, end) pair in
    // turn, 8 dependent round trips per workgroup.
    static_assert(kFinePerBin <= 32, "segment table: two lanes per segment");
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t meta;
    if (w.seg_end) {
        const uint32_t rpb = 1u << (w.rbits - kCoarseBits);
        const uint32_t sg = lane % kFinePerBin;
        const uint64_t at = (uint64_t)((region / rpb) * kFinePerBin + sg) * rpb + region % rpb;
        meta = (lane < kFinePerBin ? w.hist : w.seg_end)[at];
    } else {
        meta = w.rstart[region + (lane & 1u)];
    }
    // REC12 (the optimistic partition): records, and the LDS slice, hold h = key * kSlotMul; the
    // sentinel key's h (kEmptyH) never enters the slice, so it marks the free slots there
    constexpr uint64_t kE = REC12 ? kEmptyH : kEmpty;
    // fresh: the fill does not wait on any load (one loop with a per-slot select waited for the
    // segment-table load in its first iteration)
    if (fresh) {
        for (uint32_t i = threadIdx.x; i < S; i += T) skey[i] = kE;
    } else {
        for (uint32_t i = threadIdx.x; i < S; i += T) {
            const uint64_t k = t.slots[slice_base + i].key;
            skey[i] = REC12 ? (k == kEmpty ? kEmptyH : k * kSlotMul) : k;
        }
    }
    for (uint32_t i = threadIdx.x; i < S; i += T) {
        bcnt[i] = 0;
        bfst[i] = 0xFFFFFFFFu;
    }
    if (threadIdx.x == 0) {
        sent[0] = 0;
        sent[1] = 0xFFFFFFFFu;
        sent[2] = 0;
    }
    constexpr int kP = kAggP;
    // the region's records: one range (exact paths) or its kFinePerBin fine-scatter segments,
    // walked as one flat index space (segment s covers flat [pre[s], pre[s + 1])) so every
    // iteration issues kP loads per thread whatever the segment lengths
    uint32_t seg0[kFinePerBin], pre[kFinePerBin + 1];
    pre[0] = 0;
    if (w.seg_end) {
#pragma unroll
        for (uint32_t sg = 0; sg < kFinePerBin; ++sg) {
            seg0[sg] = (uint32_t)__builtin_amdgcn_readlane((int)meta, (int)sg);
            pre[sg + 1] = pre[sg] + ((uint32_t)__builtin_amdgcn_readlane((int)meta, (int)(kFinePerBin + sg)) - seg0[sg]);
        }
    } else {
        seg0[0] = (uint32_t)__builtin_amdgcn_readlane((int)meta, 0);
        const uint32_t end = (uint32_t)__builtin_amdgcn_readlane((int)meta, 1);
#pragma unroll
        for (uint32_t sg = 0; sg < kFinePerBin; ++sg) pre[sg + 1] = end - seg0[0];
    }
    const uint32_t total = pre[kFinePerBin];
    auto flat_at = [&](uint32_t f) -> uint32_t {   // element index of flat position f < total
        uint32_t e = seg0[0] + f;
#pragma unroll
        for (uint32_t sg = 1; sg < kFinePerBin; ++sg)
            if (f >= pre[sg]) e = seg0[sg] + (f - pre[sg]);
        return e;
    };
    // software-pipelined: the next step's loads are in flight while this step's records are folded.
    // Every lane loads unconditionally (index clamped to the last record; lanes past the end are
    // masked by `valid` when folding) and the next step is always prefetched: with no branch around
    // a load the kP loads go out back to back, where a conditional load makes the compiler wait for
    // each one before the next (vmcnt(0) at every join).
    uint64_t nkey[kP];
    uint32_t nidx[kP], nel[kP];
    auto load_step = [&](uint32_t e0) {
#pragma unroll
        for (int q = 0; q < kP; ++q) {
            const uint32_t f = min(e0 + q * T + threadIdx.x, total - 1u);
            nel[q] = flat_at(f);
            if constexpr (REC12) {
                const Rec12 r = w.brec[nel[q]];
                nkey[q] = ((uint64_t)r.khi << 32) | r.klo;
                nidx[q] = r.idx;
            } else {
                nkey[q] = w.bkey[nel[q]];
                nidx[q] = w.bidx[nel[q]];
            }
        }
    };
    if (total) load_step(0);   // in flight across the barrier that publishes the LDS fill
    // a record's home slot in the slice (before the mask); REC12 records are h already
    auto home_of = [&](uint64_t k) -> uint64_t {
        return REC12 ? (t.shift >= 64 ? 0ull : k >> t.shift) : slot_top(t, k);
    };
    auto probe_round = [&](uint64_t k, uint32_t& off, uint32_t& done, uint32_t& at) -> bool {
        return lds_probe_round<kAggProbe>(skey, (uint32_t)t.slice_mask, kE, k, off, done, at);
    };
    auto probe_round_s = [&](uint64_t k, uint32_t& off, uint32_t& done, uint32_t& at) -> bool {   // stragglers
        return lds_probe_round<kAggProbeS>(skey, (uint32_t)t.slice_mask, kE, k, off, done, at);
    };
    auto commit = [&](uint32_t at, uint32_t c, uint32_t ix) {
        if (at == S) {
            atomicOr(t.overflow, kOvfTable);
        } else {
            atomicAdd(&bcnt[at], c);
            atomicMin(&bfst[at], ix);
        }
    };
    __syncthreads();
    for (uint32_t e0 = 0; e0 < total; e0 += kP * T) {
        uint64_t key[kP];
        uint32_t idx[kP], el[kP];
#pragma unroll
        for (int q = 0; q < kP; ++q) {
            key[q] = nkey[q];
            idx[q] = nidx[q];
            el[q] = nel[q];
        }
        // weighted records' counts (a conditional load) before the prefetch: waiting for them then
        // does not wait for the next step's loads as well (vmcnt counts in issue order)
        uint32_t cw[kP];
#pragma unroll
        for (int q = 0; q < kP; ++q) {
            const bool valid = e0 + q * T + threadIdx.x < total;
            cw[q] = (valid && (idx[q] & kWeighted)) ? w.bcnt[el[q]] : 1u;
        }
        load_step(e0 + kP * T);
        // Every record gets one probe round (kAggProbe slots) first, straight-line; the records still
        // probing after it (~1 in 7 at half load) are then walked by their own lane one after another,
        // so the wave runs its longest lane's remaining rounds in total, where a probe loop per record
        // ran the longest lane's rounds for each of the kP records in turn (~15 rounds per step
        // against ~9, and ~5 for the stragglers alone, by simulation of a 2048-slot slice at half load)
        uint32_t pend = 0, soff[kP];
#pragma unroll
        for (int q = 0; q < kP; ++q) {
            const bool valid = e0 + q * T + threadIdx.x < total;
            soff[q] = 0;
            if (valid && key[q] == kE) {
                atomicAdd(&sent[0], cw[q]);
                atomicMin(&sent[1], idx[q] & ~kWeighted);
            }
            if (!valid || key[q] == kE) continue;
            uint32_t off = (uint32_t)(home_of(key[q]) & t.slice_mask), done = 0, at;
            if (probe_round(key[q], off, done, at))
                commit(at, cw[q], idx[q] & ~kWeighted);
            else {
                pend |= 1u << q;
                soff[q] = off;
            }
        }
        if (__ballot(pend != 0)) {
            uint64_t k = 0;
            uint32_t off = 0, done = 0, c = 0, ix = 0;
            auto pick = [&]() {   // the lowest pending record becomes the lane's current one
#pragma unroll
                for (int q = kP - 1; q >= 0; --q)
                    if (pend & (1u << q)) {
                        k = key[q];
                        off = soff[q];
                        c = cw[q];
                        ix = idx[q] & ~kWeighted;
                    }
                done = (off - (uint32_t)home_of(k)) & (uint32_t)t.slice_mask;   // < S while probing
            };
            if (pend) pick();
            while (__ballot(pend != 0)) {
                uint32_t at;
                if (pend && probe_round_s(k, off, done, at)) {
                    commit(at, c, ix);
                    pend &= pend - 1u;
                    if (pend) pick();
                }
            }
        }
    }
    __syncthreads();
    uint32_t used = 0;
    uint4* sl = (uint4*)&t.slots[slice_base];
    for (uint32_t i = threadIdx.x; i < S; i += T) {
        const unsigned long long kh = skey[i];
        used += kh != kE ? 1u : 0u;
        const unsigned long long k = REC12 ? (kh != kE ? kh * kSlotInv : kEmpty) : kh;
        const uint32_t bc = bcnt[i];
        if (fresh) {   // every slot, one dwordx4 each (empty slots as the reset pattern)
            sl[i] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), ~bc,
                               bc ? (uint32_t)(base_index + bfst[i]) : kNoFirst);
        } else if (bc) {
            const uint4 old = sl[i];
            const uint32_t f = (uint32_t)(base_index + bfst[i]);
            sl[i] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), old.z - bc, f < old.w ? f : old.w);
        }
    }
    if (t.occ) {   // the slice's occupancy after this batch (ss_counter_pack_ranges)
        if (used) atomicAdd(&sent[2], used);
        __syncthreads();
        if (threadIdx.x == 0) t.occ[region] = sent[2];
    }
    if (threadIdx.x == 0 && sent[0]) {
        Slot* ss = &t.slots[t.mask + 1];
        atomicAdd(&ss->ncount, 0u - sent[0]);
        atomicMin(&ss->first, (uint32_t)(base_index + sent[1]));
    }
}

// ------------------------------------------------------------------------------------------------
// Owner-side merge of region-sorted runs (the multi-GPU counter's exchange step).
// Each source rank extracts the regions this rank owns in slot order (ss_counter_extract_ranges),
// so every received run is sorted by region.  k_run_bounds finds where each owned region starts
// in each run (thread per entry, a boundary writes the starts of the regions it crosses);
// k_merge_runs then gives every owned region one workgroup that loads the region's table slice
// into LDS (keys, counts, first), folds in the run segments of that region (LDS CAS claims new
// keys, LDS 64-bit adds / mins), and writes the slice back: no global atomics, no partition
// passes, and the owner keeps counting in its own table (non-owned regions are simply stale).
// The sentinel key ~0 (EMPTY) is always the last entry of the run that carries it.  Runs are given
// as (begin, end) index pairs into the received arrays, so the receiver's own part, which is
// already in its table, is simply left out.
// ------------------------------------------------------------------------------------------------
// Record accessors for the merge kernels: triples (three u64 arrays) or packed records.
struct TripleRecs {
    const uint64_t* keys;
    const uint64_t* counts;
    const uint64_t* first;
    __device__ __forceinline__ uint64_t key(uint64_t j) const { return keys[j]; }
    __device__ __forceinline__ void load(uint64_t j, uint32_t, uint64_t& k, unsigned long long& c,
                                         unsigned long long& f) const {
        k = keys[j];
        c = counts[j];
        f = first[j];
    }
};

struct PackedRecs {
    const uint4* rec;
    const uint64_t* run_base;   // per run: first_base of the source rank
    __device__ __forceinline__ uint64_t key(uint64_t j) const {
        const uint4 v = rec[j];
        return ((uint64_t)v.y << 32) | v.x;
    }
    __device__ __forceinline__ void load(uint64_t j, uint32_t run, uint64_t& k, unsigned long long& c,
                                         unsigned long long& f) const {
        const uint4 v = rec[j];
        k = ((uint64_t)v.y << 32) | v.x;
        c = v.z;
        f = run_base[run] + v.w;
    }
};

// record j's region relative to reg_lo (clamped to [0, nreg]); the sentinel sorts last
template <typename Recs>
__device__ __forceinline__ uint32_t run_rel(const Tbl& t, const Recs& recs, uint64_t j, uint32_t reg_lo, uint32_t nreg) {
    const uint64_t k = recs.key(j);
    if (k == kEmpty) return nreg;
    const uint32_t r = region_of(t, k);
    return r < reg_lo ? 0u : min(r - reg_lo, nreg);
}

template <typename Recs>
__global__ __launch_bounds__(256) void k_run_bounds(Tbl t, Recs recs,
                                                   const uint64_t* __restrict__ run_off, uint32_t n_runs,
                                                   uint32_t reg_lo, uint32_t nreg, uint32_t* __restrict__ bounds) {
    // run_off: (begin, end) pairs; entries outside every run (e.g. this rank's own part) are skipped
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t run = 0;
    while (run < n_runs && !(run_off[2 * run] <= i && i < run_off[2 * run + 1])) ++run;
    if (run == n_runs) return;
    const uint64_t beg = run_off[2 * run], end = run_off[2 * run + 1];
    auto rel = [&](uint64_t j) { return run_rel(t, recs, j, reg_lo, nreg); };
    const uint32_t r = rel(i);
    const uint32_t prev = i == beg ? 0u : rel(i - 1) + 1u;   // regions [prev, r] start at i
    uint32_t* b = bounds + (uint64_t)run * (nreg + 1);
    for (uint32_t q = (i == beg ? 0u : prev); q <= r; ++q) b[q] = (uint32_t)(i - beg);
    if (i + 1 == end)                                          // regions after the last entry: empty
        for (uint32_t q = r + 1; q <= nreg; ++q) b[q] = (uint32_t)(end - beg);
}

constexpr uint32_t kMergeT = 512;
constexpr uint32_t kMergeSearchRuns = 64;   // up to this many runs, each block finds its own bounds
constexpr int kMergeK = 4;                  // k_merge_runs: records in flight per thread

template <typename Recs>
__global__ __launch_bounds__(kMergeT) void k_merge_runs(Tbl t, Recs recs,
                                                       const uint64_t* __restrict__ run_off, uint32_t n_runs,
                                                       uint32_t reg_lo, uint32_t nreg,
                                                       const uint32_t* __restrict__ bounds) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t S = (uint32_t)t.slice_mask + 1;
    unsigned long long* skey = (unsigned long long*)smem;     // [S]
    uint32_t* scnt = (uint32_t*)(skey + S);                    // [S] counts (not complemented)
    uint32_t* sfst = scnt + S;                                 // [S]
    const uint32_t j = blockIdx.x;                             // owned region reg_lo + j
    const uint64_t base = (uint64_t)(reg_lo + j) << t.slice_log;
    uint4* sl = (uint4*)&t.slots[base];
    for (uint32_t q = threadIdx.x; q < S; q += kMergeT) {
        const uint4 v = sl[q];
        skey[q] = ((uint64_t)v.y << 32) | v.x;
        scnt[q] = ~v.z;
        sfst[q] = v.w;
    }
    // bounds == null: this region's segment of every run by a 64-ary search per (run, edge), one wave
    // each (4 dependent steps for a 2M-record run) -- no separate pass over every record
    __shared__ uint32_t s_lo[kMergeSearchRuns], s_hi[kMergeSearchRuns];
    if (!bounds) {
        // a 32-ary search per (run, edge), one half-wave each: the block's 16 half-waves take up to 16
        // searches at once (8 owners: all 14 in one round of ~5 dependent steps, where a wave per
        // search took two rounds of 4)
        const uint32_t hl = threadIdx.x & 31u, hsh = threadIdx.x & 32u;
        for (uint32_t q = threadIdx.x >> 5; q < 2 * n_runs; q += kMergeT / 32) {
            const uint32_t run = q >> 1, target = j + (q & 1u);
            const uint64_t beg = run_off[2 * run], end = run_off[2 * run + 1];
            uint64_t L = beg, H = end;     // the first record of region >= target lies in [L, H]
            while (H > L) {
                const uint64_t len = H - L;
                const uint64_t p = L + len * hl / 32;
                const bool below = run_rel(t, recs, p, reg_lo, nreg) < target;
                const uint32_t c = (uint32_t)__popcll((__ballot(below) >> hsh) & 0xFFFFFFFFull);
                if (c == 0) break;
                const uint64_t nx = c < 32 ? L + len * c / 32 : H;
                L = L + len * (c - 1) / 32 + 1;
                H = nx;
            }
            if (hl == 0) ((q & 1u) ? s_hi : s_lo)[run] = (uint32_t)(L - beg);
        }
    }
    __syncthreads();
    // the region's segments of up to kMergeSearchRuns runs folded as ONE flat index space (prefix of
    // their lengths in LDS): every thread keeps kMergeK records in flight, where run after run each
    // segment of ~1k records was one or two dependent load round trips of the whole block
    __shared__ uint32_t s_pre[kMergeSearchRuns + 1];
    __shared__ uint64_t s_at[kMergeSearchRuns];
    for (uint32_t g0 = 0; g0 < n_runs; g0 += kMergeSearchRuns) {
        const uint32_t nr = min(n_runs - g0, kMergeSearchRuns);
        if (threadIdx.x < 64) {           // wave 0: the group's segment starts and length prefix
            const uint32_t lane = threadIdx.x, run = g0 + lane;
            uint32_t len = 0;
            if (lane < nr) {
                const uint64_t r0 = run_off[2 * run];
                uint32_t lo = 0, hi = 0;
                if (run_off[2 * run + 1] != r0) {               // empty run: no bounds were written
                    const uint32_t* b = bounds + (uint64_t)run * (nreg + 1);
                    lo = bounds ? b[j] : s_lo[run];
                    hi = bounds ? b[j + 1] : s_hi[run];
                }
                len = hi - lo;
                s_at[lane] = r0 + lo;
            }
            uint32_t incl = len;
            for (uint32_t o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            if (lane < nr) s_pre[lane + 1] = incl;
            if (lane == 0) s_pre[0] = 0;
        }
        __syncthreads();
        const uint32_t tot = s_pre[nr];
        for (uint32_t e0 = 0; e0 < tot; e0 += kMergeT * kMergeK) {
            uint64_t key[kMergeK];
            unsigned long long c[kMergeK], f[kMergeK];
#pragma unroll
            for (int k = 0; k < kMergeK; ++k) {
                const uint32_t e = min(e0 + (uint32_t)k * kMergeT + threadIdx.x, tot - 1u);
                uint32_t lo = 0, hi = nr - 1;         // the run holding flat record e: s_pre[run] <= e
                while (lo < hi) {
                    const uint32_t mid = (lo + hi + 1) >> 1;
                    if (s_pre[mid] <= e) lo = mid;
                    else hi = mid - 1;
                }
                recs.load(s_at[lo] + (e - s_pre[lo]), g0 + lo, key[k], c[k], f[k]);
            }
            // one probe round per record, then each lane's unfinished records in turn (the aggregate's
            // form: the wave runs its longest lane's remaining rounds, not each record's longest probe)
            auto commit = [&](uint32_t at, unsigned long long cc, unsigned long long ff) {
                if (at == S) {
                    atomicOr(t.overflow, kOvfTable);
                    return;
                }
                if (ff > kMaxIndex) atomicOr(t.overflow, kOvfIndex);
                const uint32_t old = atomicAdd(&scnt[at], (uint32_t)cc);
                if ((cc >> 32) || old + (uint32_t)cc < old)     // a carry past 32 bits: rare
                    count_add_wide(t, base + at, old, (uint32_t)cc, cc & ~0xFFFFFFFFull);
                atomicMin(&sfst[at], (uint32_t)min((unsigned long long)kMaxIndex, ff));
            };
            const uint32_t mask = (uint32_t)t.slice_mask;
            uint32_t pend = 0, soff[kMergeK];
#pragma unroll
            for (int k = 0; k < kMergeK; ++k) {
                soff[k] = 0;
                if (e0 + (uint32_t)k * kMergeT + threadIdx.x >= tot) continue;
                uint32_t off = (uint32_t)(slot_top(t, key[k]) & mask), done = 0, at;
                if (lds_probe_round<kAggProbe>(skey, mask, kEmpty, key[k], off, done, at)) {
                    commit(at, c[k], f[k]);
                } else {
                    pend |= 1u << k;
                    soff[k] = off;
                }
            }
            if (__ballot(pend != 0)) {
                uint64_t kk = 0;
                unsigned long long cc = 0, ff = 0;
                uint32_t off = 0, done = 0;
                auto pick = [&]() {   // the lowest pending record becomes the lane's current one
#pragma unroll
                    for (int k = kMergeK - 1; k >= 0; --k)
                        if (pend & (1u << k)) {
                            kk = key[k];
                            cc = c[k];
                            ff = f[k];
                            off = soff[k];
                        }
                    done = (off - (uint32_t)slot_top(t, kk)) & mask;   // < S while probing
                };
                if (pend) pick();
                while (__ballot(pend != 0)) {
                    uint32_t at;
                    if (pend && lds_probe_round<kAggProbeS>(skey, mask, kEmpty, kk, off, done, at)) {
                        commit(at, cc, ff);
                        pend &= pend - 1u;
                        if (pend) pick();
                    }
                }
            }
        }
        __syncthreads();                  // s_pre / s_at of the next group
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < S; q += kMergeT) {
        const unsigned long long k = skey[q];
        sl[q] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), ~scnt[q], sfst[q]);
    }
}

// the sentinel key (~0 = "G" * 32) of each run: the last entry, if any
template <typename Recs>
__global__ void k_merge_sentinel(Tbl t, Recs recs, const uint64_t* run_off, uint32_t n_runs) {
    if (threadIdx.x != 0) return;
    for (uint32_t run = 0; run < n_runs; ++run) {
        const uint64_t beg = run_off[2 * run], end = run_off[2 * run + 1];
        if (end > beg && recs.key(end - 1) == kEmpty) {
            uint64_t k;
            unsigned long long c, f;
            recs.load(end - 1, run, k, c, f);
            Slot* sl = &t.slots[t.mask + 1];
            if (f > kMaxIndex) atomicOr(t.overflow, kOvfIndex);
            const uint32_t old = atomicAdd(&sl->ncount, 0u - (uint32_t)c);
            count_add_wide(t, t.mask + 1, ~old, (uint32_t)c, c & ~0xFFFFFFFFull);
            atomicMin(&sl->first, (uint32_t)min((unsigned long long)kMaxIndex, f));
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Packed exchange records (ss_counter_pack_ranges / ss_counter_merge_packed): 16 B per entry,
// {key u64, count u32 | (first - first_base) u32 << 32}, grouped by owner part and, inside a part,
// by table region (any order inside a region).  Two thirds of the (key, count, first) u64 triples
// extract_ranges produces, written straight into the all-to-all send buffer.
//   k_region_occ   (only when the aggregate's occupancy is stale) used slots per region
//   k_region_scan  one block: region offsets skipping the caller's own part, the sentinel slot at
//                  the end of its owner's segment, part counts
//   k_region_pack  one workgroup per region: slice -> records at the region's offset
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kPackT = 256;

__device__ __forceinline__ uint32_t part_of_region(uint64_t region, uint64_t R, uint32_t nparts) {
    return (uint32_t)(region * nparts / R);
}

__global__ __launch_bounds__(kPackT) void k_region_occ(Tbl t) {
    __shared__ uint32_t sum;
    if (threadIdx.x == 0) sum = 0;
    __syncthreads();
    const uint32_t S = (uint32_t)t.slice_mask + 1;
    const uint64_t base = (uint64_t)blockIdx.x << t.slice_log;
    uint32_t used = 0;
    for (uint32_t i = threadIdx.x; i < S; i += kPackT) used += t.slots[base + i].key != kEmpty ? 1u : 0u;
    if (used) atomicAdd(&sum, used);
    __syncthreads();
    if (threadIdx.x == 0) t.occ[blockIdx.x] = sum;
}

// roff[r] = first record of region r; roff[R] = the sentinel's position (or ~0), roff[R + 1] = total
__global__ __launch_bounds__(1024) void k_region_scan(Tbl t, uint32_t R, uint32_t nparts, int32_t skip,
                                                      unsigned long long* roff, unsigned long long* part_counts) {
    __shared__ unsigned long long sums[1024];
    __shared__ unsigned long long psum[kMaxParts];
    const uint32_t per = (R + 1023) / 1024;
    const uint32_t lo = min(R, threadIdx.x * per), hi = min(R, lo + per);
    for (uint32_t p = threadIdx.x; p < nparts; p += 1024) psum[p] = 0;
    unsigned long long local = 0;
    for (uint32_t r = lo; r < hi; ++r)
        if ((int32_t)part_of_region(r, R, nparts) != skip) local += t.occ[r];
    sums[threadIdx.x] = local;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const unsigned long long v = threadIdx.x >= off ? sums[threadIdx.x - off] : 0ull;
        __syncthreads();
        sums[threadIdx.x] += v;
        __syncthreads();
    }
    // the sentinel slot (key ~0 = "G" * 32) belongs to the owner of region_of(~0); it goes last in
    // that owner's segment, so every later part shifts by one
    const uint32_t sreg = region_of(t, kEmpty);
    const uint32_t sp = part_of_region(sreg, R, nparts);
    uint64_t skey;
    const bool sent = slot_used(t, t.mask + 1, skey) && (int32_t)sp != skip;
    unsigned long long run = sums[threadIdx.x] - local;
    for (uint32_t r = lo; r < hi; ++r) {
        const uint32_t p = part_of_region(r, R, nparts);
        const unsigned long long c = (int32_t)p != skip ? t.occ[r] : 0u;
        roff[r] = run + (sent && p > sp ? 1u : 0u);
        run += c;
        if (c) atomicAdd(&psum[p], c);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // sentinel position: the end of its owner's segment (segments are in part order)
        unsigned long long before = 0;
        for (uint32_t p = 0; p <= sp; ++p) before += psum[p];
        roff[R] = sent ? before : ~0ull;
        roff[R + 1] = sums[1023] + (sent ? 1u : 0u);
    }
    for (uint32_t p = threadIdx.x; p < nparts; p += 1024) part_counts[p] = psum[p] + (sent && p == sp ? 1u : 0u);
}

__global__ __launch_bounds__(kPackT) void k_region_pack(Tbl t, uint32_t R, uint32_t nparts, int32_t skip,
                                                        const unsigned long long* __restrict__ roff,
                                                        uint64_t first_base, uint4* __restrict__ rec, uint64_t cap,
                                                        unsigned long long* flags) {
    const uint32_t r = blockIdx.x;
    __shared__ unsigned long long cursor;
    if (r == 0 && threadIdx.x == 0 && roff[R] != ~0ull) {   // the sentinel record
        const Slot& sl = t.slots[t.mask + 1];
        const unsigned long long c = (uint32_t)~sl.ncount + (t.wide ? t.wide[t.mask + 1] : 0ull), f = sl.first - first_base;
        if (f >> 32 || sl.first < first_base || (c >> 32)) atomicOr(flags, kOvfField);   // (u32 record counts)
        if (roff[R] < cap)
            rec[roff[R]] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, (uint32_t)c, (uint32_t)f);
        else
            atomicOr(flags, kOvfExtract);
    }
    if ((int32_t)part_of_region(r, R, nparts) == skip) return;
    if (threadIdx.x == 0) cursor = roff[r];
    __syncthreads();
    const uint32_t S = (uint32_t)t.slice_mask + 1;
    const uint64_t base = (uint64_t)r << t.slice_log;
    constexpr int kU = 4;
    const uint4* slots = (const uint4*)&t.slots[base];
    for (uint32_t i0 = 0; i0 < S; i0 += kU * kPackT) {
        uint4 a[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t i = i0 + u * kPackT + threadIdx.x;
            a[u] = i < S ? slots[i] : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const bool used = !(a[u].x == 0xFFFFFFFFu && a[u].y == 0xFFFFFFFFu);
            const unsigned long long pos = wave_reserve(used, 0u, &cursor);
            if (!used) continue;
            const uint32_t c = ~a[u].z;
            // the 16-B record carries a u32 count: a count with a high part (wide) cannot cross
            if (a[u].w < first_base || (t.wide && t.wide[base + i0 + u * kPackT + threadIdx.x])) atomicOr(flags, kOvfField);
            if (pos < cap)
                rec[pos] = make_uint4(a[u].x, a[u].y, c, (uint32_t)(a[u].w - first_base));
            else
                atomicOr(flags, kOvfExtract);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Multi-word keys (33..1024 nt: W = ceil(L/32) words; ShortSeq192 / ShortSeqVar keys,
// short_seq_192.pyx:35-41 / short_seq_var.pyx:22-28: equal iff length and all words equal).
// The reads are packed first (ss_encode_fixed into ws_words), keyed by a 64-bit fingerprint of
// their words, and go through the same partition passes.  Equality is always decided on the full
// words: the LDS table claims a slot with ONE 64-bit CAS of (fingerprint high half | representative
// read index), so a thread that meets a claimed slot can compare words immediately (no waiting on
// another lane's second store); the global slice stores the full fingerprint plus the key words.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool words_eq(const uint64_t* a, const uint64_t* b, uint32_t W) {
    bool eq = true;
    for (uint32_t j = 0; j < W; ++j) eq &= a[j] == b[j];
    return eq;
}

// The same test for rows of a compile-time W1 words: each row read as the 16-B-aligned chunks
// holding it, ceil((8 W1 + 8) / 16) dwordx4 gathers instead of W1 dwordx2 (the aggregate's row
// gathers bound it on address processing, one cache line per lane per instruction).  An aligned
// chunk never leaves the page of the row bytes it holds.  EVEN: W1 even and the rows' base 16-B
// aligned, so every row starts a chunk.
template <int W1, bool EVEN>
__device__ __forceinline__ void row_chunks(const uint64_t* p, uint64_t (&v)[EVEN ? W1 : W1 + 2], bool& odd) {
    constexpr int NC = EVEN ? W1 / 2 : (W1 + 2) / 2;
    const uint4* c = (const uint4*)((uintptr_t)p & ~(uintptr_t)15);
    odd = !EVEN && ((uintptr_t)p & 8u);
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        const uint4 x = c[k];
        v[2 * k] = (uint64_t)x.y << 32 | x.x;
        v[2 * k + 1] = (uint64_t)x.w << 32 | x.z;
    }
}

template <int W1, bool EVEN>
__device__ __forceinline__ bool rows_eq(const uint64_t* a, const uint64_t* b) {
    uint64_t va[EVEN ? W1 : W1 + 2], vb[EVEN ? W1 : W1 + 2];
    bool oa, ob;
    row_chunks<W1, EVEN>(a, va, oa);
    row_chunks<W1, EVEN>(b, vb, ob);
    bool eq = true;
    // the odd rows' words by masks, not a select of the element (which the compiler turned into a
    // dynamically indexed array in scratch)
    const uint64_t ma = 0ull - (uint64_t)oa, mb = 0ull - (uint64_t)ob;
#pragma unroll
    for (int j = 0; j < W1; ++j) {
        if constexpr (EVEN) {
            eq &= va[j] == vb[j];
        } else {
            const uint64_t a = (va[j + 1] & ma) | (va[j] & ~ma), b = (vb[j + 1] & mb) | (vb[j] & ~mb);
            eq &= a == b;
        }
    }
    return eq;
}

// words_fp of a row of W1C words read as its aligned dwordx4 chunks (row_chunks)
template <int W1, bool EVEN>
__device__ __forceinline__ uint64_t row_fp(const uint64_t* p) {
    uint64_t v[EVEN ? W1 : W1 + 2];
    bool odd;
    row_chunks<W1, EVEN>(p, v, odd);
    const uint64_t m = 0ull - (uint64_t)odd;
    uint64_t h = fp_seed(W1);
#pragma unroll
    for (int j = 0; j < W1; ++j) {
        uint64_t x;
        if constexpr (EVEN) x = v[j];
        else x = (v[j + 1] & m) | (v[j] & ~m);
        h = fp_step(h, x);
    }
    return fp_final(h);
}

// W1C: rows of W1C words read as aligned chunks (row_fp), 0 for any width
template <int T, int W1C, bool EVEN>
__global__ __launch_bounds__(T) void k_mw_fp(Tbl t, PartWs w, uint32_t bins, const uint64_t* __restrict__ words,
                                             uint64_t n) {
    extern __shared__ uint32_t hist[];
    constexpr uint32_t kWaves = T / 64;
    const uint32_t copies = bins * kWaves <= kMaxRegions ? kWaves : 1u;
    uint32_t* my = hist + (copies > 1 ? (threadIdx.x >> 6) * bins : 0u);
    for (uint32_t i = threadIdx.x; i < bins * copies; i += T) hist[i] = 0;
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = min(n, lo + per);
    for (uint64_t r = lo + threadIdx.x; r < hi; r += T) {
        uint64_t fp;
        if constexpr (W1C > 0) fp = row_fp<W1C, EVEN>(words + r * W1C);
        else fp = words_fp(words + r * t.W, t.W);
        w.keys[r] = fp;
        atomicAdd(&my[bin_of<true>(t, w, fp)], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < bins; i += T) {
        uint32_t sum = 0;
        for (uint32_t c = 0; c < copies; ++c) sum += hist[c * bins + i];
        w.hist[(uint64_t)blockIdx.x * bins + i] = sum;
    }
}

constexpr uint32_t kMwT = 1024;
constexpr uint32_t kMwPerThread = (2u << kMwSliceLog) / kMwT;

// W1C: the rows' word count at compile time (row gathers as aligned dwordx4 chunks, rows_eq), 0 for
// any other count (a dwordx2 per word)
template <int T, int W1C, bool EVEN>
__global__ __launch_bounds__(T) void k_mw_aggregate(Tbl t, PartWs w, const uint64_t* __restrict__ words,
                                                    uint64_t base_index) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t S = (uint32_t)t.slice_mask + 1;
    const uint32_t LS = 2 * S;
    const uint32_t W = W1C ? (uint32_t)W1C : t.W;
    unsigned long long* lkey = (unsigned long long*)smem;                 // [LS] (fp_hi << 32 | rep)
    unsigned long long* skey = lkey + LS;                                 // [S] slice fingerprints
    uint32_t* lcnt = (uint32_t*)(skey + S);                               // [LS]
    uint32_t* lfst = lcnt + LS;                                           // [LS]
    const uint32_t region = blockIdx.x;
    const uint64_t slice_base = (uint64_t)region << t.slice_log;
    __shared__ int lds_full;   // an undersized table: the LDS hash ran full, the insert is void
    if (threadIdx.x == 0) lds_full = 0;
    for (uint32_t i = threadIdx.x; i < LS; i += T) {
        lkey[i] = kEmpty;
        lcnt[i] = 0;
        lfst[i] = 0xFFFFFFFFu;
    }
    for (uint32_t i = threadIdx.x; i < S; i += T) skey[i] = t.slots[slice_base + i].key;
    __syncthreads();
    const uint32_t b0 = w.rstart[region], b1 = w.rstart[region + 1];
    const uint32_t lds_shift = (t.shift >= 64 ? 64 : t.shift) - 1;
    for (uint32_t e = b0 + threadIdx.x; e < b1; e += T) {
        const uint64_t fp = w.bkey[e];
        const uint32_t idx = w.bidx[e];
        const uint64_t tag = (fp >> 32) << 32;
        if (*(volatile int*)&lds_full) break;   // overflow raised: the rest of the region need not probe
        uint32_t ls = (uint32_t)((fp * 0x9E3779B97F4A7C15ull) >> lds_shift) & (LS - 1);
        bool placed = false;
        for (uint32_t probe = 0; probe < LS; ++probe) {   // bounded: a region with > 2S distinct keys
            unsigned long long cur = lkey[ls];           // (an undersized table) raises the overflow word
            if (cur == kEmpty) {
                cur = atomicCAS(&lkey[ls], (unsigned long long)kEmpty, (unsigned long long)(tag | idx));
                if (cur == kEmpty) {   // claimed, this read is the representative
                    placed = true;
                    break;
                }
            }
            bool same = (cur & 0xFFFFFFFF00000000ull) == tag;
            if (same) {
                const uint64_t* ra = words + (cur & 0xFFFFFFFFull) * W;
                const uint64_t* rb = words + (uint64_t)idx * W;
                if constexpr (W1C > 0) same = rows_eq<W1C, EVEN>(ra, rb);
                else same = words_eq(ra, rb, W);
            }
            if (same) {
                placed = true;
                break;
            }
            ls = (ls + 1) & (LS - 1);
        }
        if (!placed) {
            atomicOr(t.overflow, kOvfTable);
            *(volatile int*)&lds_full = 1;
            continue;
        }
        atomicAdd(&lcnt[ls], 1u);
        atomicMin(&lfst[ls], idx);
    }
    __syncthreads();
    // phase 2a: distinct keys already in the slice (fingerprint + words match; the slice's key
    // words were written by earlier launches, so they are stable here).  skey is not modified.
    uint32_t slot[kMwPerThread];
    uint64_t fps[kMwPerThread];
#pragma unroll
    for (uint32_t j = 0; j < kMwPerThread; ++j) {
        const uint32_t ls = j * T + threadIdx.x;
        slot[j] = 0xFFFFFFFFu;
        fps[j] = kEmpty;
        if (ls >= LS) continue;
        const unsigned long long lk = lkey[ls];
        if (lk == kEmpty) continue;
        const uint64_t* kw = words + (lk & 0xFFFFFFFFull) * W;
        const uint64_t fp = words_fp(kw, W);
        fps[j] = fp;
        uint32_t off = (uint32_t)(slot_top(t, fp) & t.slice_mask);
        for (uint32_t probe = 0; probe < S; ++probe) {
            const unsigned long long cur = skey[off];
            if (cur == kEmpty) break;
            if (cur == fp && words_eq(t.keywords + (slice_base + off) * W, kw, W)) {
                slot[j] = off;
                break;
            }
            off = (off + 1) & (uint32_t)t.slice_mask;
        }
    }
    __syncthreads();
    // phase 2b: new keys claim free slice slots.  Every key that could match was resolved in 2a, and
    // the LDS entries are distinct keys, so a claimed slot is never a match: skip all non-empty slots.
    bool fresh[kMwPerThread];
#pragma unroll
    for (uint32_t j = 0; j < kMwPerThread; ++j) {
        fresh[j] = false;
        if (fps[j] == kEmpty || slot[j] != 0xFFFFFFFFu) continue;
        uint32_t off = (uint32_t)(slot_top(t, fps[j]) & t.slice_mask);
        for (uint32_t probe = 0; probe < S; ++probe) {
            if (skey[off] == kEmpty &&
                atomicCAS(&skey[off], (unsigned long long)kEmpty, (unsigned long long)fps[j]) == kEmpty) {
                slot[j] = off;
                fresh[j] = true;
                break;
            }
            off = (off + 1) & (uint32_t)t.slice_mask;
        }
        if (slot[j] == 0xFFFFFFFFu) atomicOr(t.overflow, kOvfTable);
    }
    // phase 3: slot read-modify-writes (the workgroup owns the slice) and key words of new slots
#pragma unroll
    for (uint32_t j = 0; j < kMwPerThread; ++j) {
        if (slot[j] == 0xFFFFFFFFu) continue;
        const uint32_t ls = j * T + threadIdx.x;
        Slot* sl = &t.slots[slice_base + slot[j]];
        const unsigned long long f = base_index + lfst[ls];
        if (fresh[j]) {
            const uint64_t* kw = words + (lkey[ls] & 0xFFFFFFFFull) * W;
            uint64_t* dst = t.keywords + (slice_base + slot[j]) * W;
            for (uint32_t q = 0; q < W; ++q) dst[q] = kw[q];
            sl->key = fps[j];
            sl->ncount = ~lcnt[ls];
            sl->first = (uint32_t)f;
        } else {
            sl->ncount -= lcnt[ls];
            if ((uint32_t)f < sl->first) sl->first = (uint32_t)f;
        }
    }
}

using MwAggFn = void (*)(Tbl, PartWs, const uint64_t*, uint64_t);
constexpr int kMwAggFns = 10;
// every k_mw_aggregate instance: rows of 2..7 words (keys of up to 192 nt, the ShortSeq192 class
// widths plus the length word) with dwordx4 row gathers, then the any-width form
constexpr MwAggFn kMwAgg[kMwAggFns] = {
    k_mw_aggregate<kMwT, 0, false>, k_mw_aggregate<kMwT, 2, true>,  k_mw_aggregate<kMwT, 2, false>,
    k_mw_aggregate<kMwT, 3, false>, k_mw_aggregate<kMwT, 4, true>,  k_mw_aggregate<kMwT, 4, false>,
    k_mw_aggregate<kMwT, 5, false>, k_mw_aggregate<kMwT, 6, true>,  k_mw_aggregate<kMwT, 6, false>,
    k_mw_aggregate<kMwT, 7, false>};

// index into kMwAgg / kMwFp of the instance for rows of W1 words at `rows`
inline int mw_variant(uint32_t W1, const uint64_t* rows) {
    const bool a16 = ((uintptr_t)rows & 15u) == 0;
    switch (W1) {
    case 2: return a16 ? 1 : 2;
    case 3: return 3;
    case 4: return a16 ? 4 : 5;
    case 5: return 6;
    case 6: return a16 ? 7 : 8;
    case 7: return 9;
    default: return 0;
    }
}

using MwFpFn = void (*)(Tbl, PartWs, uint32_t, const uint64_t*, uint64_t);
constexpr int kMwFpT = 512;
constexpr MwFpFn kMwFp[kMwAggFns] = {
    k_mw_fp<kMwFpT, 0, false>, k_mw_fp<kMwFpT, 2, true>,  k_mw_fp<kMwFpT, 2, false>, k_mw_fp<kMwFpT, 3, false>,
    k_mw_fp<kMwFpT, 4, true>,  k_mw_fp<kMwFpT, 4, false>, k_mw_fp<kMwFpT, 5, false>, k_mw_fp<kMwFpT, 6, true>,
    k_mw_fp<kMwFpT, 6, false>, k_mw_fp<kMwFpT, 7, false>};

// Merge of already-counted multi-word entries (distinct keys: e.g. the extraction of another
// table when a per-length table grows): phase 1 finds each entry's key among the slots that existed
// before the merge (the table is stable during the pass, so the key words are complete); phase 2
// gives the rest a fresh slot (a CAS on the fingerprint; a slot another entry claims is never this
// entry's key, the entries being distinct, so claimed slots are skipped without comparing words)
// and writes their key words, count and first index.  Found keys add count / min first.
__global__ __launch_bounds__(256) void k_mw_merge_find(Tbl t, const uint64_t* __restrict__ words, uint64_t m,
                                                       uint64_t* __restrict__ found) {
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (uint64_t)gridDim.x * 256) {
        const uint64_t* kw = words + e * t.W;
        const uint64_t fp = words_fp(kw, t.W);
        const uint64_t top = slot_top(t, fp), base = top & ~t.slice_mask;
        uint64_t off = top & t.slice_mask, at = kEmpty;
        for (uint64_t probe = 0; probe <= t.slice_mask; ++probe) {
            const uint64_t k = t.slots[base + off].key;
            if (k == kEmpty) break;
            if (k == fp && words_eq(t.keywords + (base + off) * t.W, kw, t.W)) {
                at = base + off;
                break;
            }
            off = (off + 1) & t.slice_mask;
        }
        found[e] = at;
    }
}

__global__ __launch_bounds__(256) void k_mw_merge_claim(Tbl t, const uint64_t* __restrict__ words,
                                                        const uint64_t* __restrict__ counts,
                                                        const uint64_t* __restrict__ first, uint64_t m,
                                                        const uint64_t* __restrict__ found) {
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (uint64_t)gridDim.x * 256) {
        const uint64_t* kw = words + e * t.W;
        const uint32_t c = (uint32_t)counts[e];
        const uint64_t chi = counts[e] & ~0xFFFFFFFFull;
        uint64_t f = first[e];
        if (f > kMaxIndex) {
            atomicOr(t.overflow, kOvfIndex);
            f = kMaxIndex;
        }
        uint64_t at = found[e];
        if (at == kEmpty) {
            const uint64_t fp = words_fp(kw, t.W);
            const uint64_t top = slot_top(t, fp), base = top & ~t.slice_mask;
            uint64_t off = top & t.slice_mask;
            for (uint64_t probe = 0; probe <= t.slice_mask; ++probe) {
                if (t.slots[base + off].key == kEmpty &&
                    atomicCAS(&t.slots[base + off].key, (unsigned long long)kEmpty, (unsigned long long)fp) == kEmpty) {
                    at = base + off;
                    break;
                }
                off = (off + 1) & t.slice_mask;
            }
            if (at == kEmpty) {
                atomicOr(t.overflow, kOvfTable);
                continue;
            }
            uint64_t* dst = t.keywords + at * t.W;
            for (uint32_t q = 0; q < t.W; ++q) dst[q] = kw[q];
            t.slots[at].ncount = ~c;
            t.slots[at].first = (uint32_t)f;
            count_add_wide(t, at, 0u, c, chi);
            continue;
        }
        const uint32_t old = atomicAdd(&t.slots[at].ncount, 0u - c);
        count_add_wide(t, at, ~old, c, chi);
        if (t.slots[at].first > (uint32_t)f) atomicMin(&t.slots[at].first, (uint32_t)f);
    }
}

// Per-call resets in one dispatch: up to four 8-B words set and a run of u32 words zeroed.  The
// streamed C5 step issued three stream write packets at ss_counter_reset, one for first_bad and a
// two-part fill of the sub-bin counters, ~80 us per step with the command processor's gaps between
// them (profiles/r3/r3e all-configs trace); as two of these launches they cost ~10 us.
struct PrepWords {
    unsigned long long* p[4];   // null: unused
    unsigned long long v[4];
    uint32_t* zero;             // [nzero] words set to 0 (or null)
    uint32_t nzero;
};
__global__ __launch_bounds__(256) void k_prep(PrepWords w) {
    if (threadIdx.x < 4 && w.p[threadIdx.x]) *w.p[threadIdx.x] = w.v[threadIdx.x];
    for (uint32_t i = threadIdx.x; i < w.nzero; i += 256) w.zero[i] = 0u;
}

hipError_t launch_prep(const PrepWords& w, hipStream_t s) {
    hipLaunchKernelGGL(k_prep, dim3(1), dim3(256), 0, s, w);
    return hipGetLastError();
}

Tbl tbl_of(const ss_counter* c) {
    Tbl t;
    t.slots = c->slots;
    t.wide = c->wide_live ? c->wide : nullptr;
    t.keywords = c->keywords;
    t.occ = c->occ;
    t.W = c->W;
    t.overflow = c->work;
    t.mask = c->cap - 1;
    t.slice_mask = (1ull << c->slice_log) - 1;
    t.shift = 64 - c->log2cap;
    t.slice_log = c->slice_log;
    return t;
}

// Perform a pending (lazy) reset of the slot array on `s` before anything reads the table.
int flush_reset(ss_counter* c, hipStream_t s) {
    if (!c->reset_pending) return SS_OK;
    c->reset_pending = false;
    return ss_check(hipMemsetAsync(c->slots, 0xFF, c->cap * sizeof(Slot), s), "ss_counter reset");
}

constexpr uint64_t kSinceUnknown = 1ull << 62;
unsigned grid_for(uint64_t items, uint64_t per_block, unsigned cap);   // ss_counter::since after a merge: spill before the next insert

// the wide count array allocated and, when it goes live, zeroed on `s`
int wide_on(ss_counter* c, hipStream_t s) {
    if (!c->wide && hipMalloc((void**)&c->wide, (c->cap + 1) * sizeof(uint64_t)) != hipSuccess) {
        ss_check(hipGetLastError(), "counter wide counts hipMalloc");
        c->wide = nullptr;
        return ss_fail(SS_ENOMEM, "counter wide counts: out of device memory");
    }
    if (c->wide_live) return SS_OK;
    c->wide_live = true;
    return ss_check(hipMemsetAsync(c->wide, 0, (c->cap + 1) * sizeof(uint64_t), s), "counter wide counts reset");
}

// Every slot's count into wide (the sentinel slot, present iff its count is nonzero, keeps 1): the
// slots restart below 2 and take another spill_at reads before the next spill.
__global__ __launch_bounds__(256) void k_spill_wide(Tbl t) {
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s <= t.mask + 1; s += (uint64_t)gridDim.x * 256) {
        const Slot sl = t.slots[s];
        const bool sent = s > t.mask;
        if (sent ? sl.ncount == 0xFFFFFFFFu : sl.key == kEmpty) continue;
        const uint32_t cnt = ~sl.ncount, keep = sent ? 1u : 0u;
        if (cnt <= keep) continue;
        t.wide[s] += cnt - keep;
        t.slots[s].ncount = ~keep;
    }
}

int spill_wide(ss_counter* c, hipStream_t s) {
    int rc = flush_reset(c, s);
    if (!rc) rc = wide_on(c, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_spill_wide, dim3(grid_for(c->cap + 1, 256, 256 * 16)), dim3(256), 0, s, tbl_of(c));
    c->since = 1;
    return ss_check(hipGetLastError(), "k_spill_wide");
}

// fold the oldest recorded timing set into the sums (waits for its last event)
void timer_fold_one(ss_counter* c) {
    const uint32_t k = (c->thead + ss_counter::kTimerRing - c->tpend) % ss_counter::kTimerRing;
    hipEvent_t* e = c->tev + (uint64_t)k * ss_counter::kPassEvents;
    (void)hipEventSynchronize(e[ss_counter::kPassEvents - 1]);
    for (uint32_t p = 0; p + 1 < ss_counter::kPassEvents; ++p) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e[p], e[p + 1]) == hipSuccess) c->tsum[p] += ms;
    }
    ++c->tn;
    --c->tpend;
}

// event p of this insert's timing set (null when timing is off)
hipEvent_t timer_event(ss_counter* c, uint32_t p) {
    if (!c->tev) return nullptr;
    if (p == 0 && c->tpend == ss_counter::kTimerRing) timer_fold_one(c);
    return c->tev[(uint64_t)c->thead * ss_counter::kPassEvents + p];
}

unsigned grid_for(uint64_t items, uint64_t per_block, unsigned cap) {
    uint64_t b = (items + per_block - 1) / per_block;
    if (b == 0) b = 1;
    if (cap && b > cap) b = cap;
    return (unsigned)b;
}

template <typename Recs>
int launch_merge(ss_counter* c, Recs recs, const uint64_t* d_run_offsets, uint32_t n_runs, uint64_t m,
                        uint32_t reg_lo, uint32_t nreg, uint32_t* d_bounds, hipStream_t s, const char* what) {
    int rc = flush_reset(c, s);
    if (rc) return rc;
    c->since = kSinceUnknown;   // (a carry past 32 bits goes to wide when live, else it is flagged)
    Tbl t = tbl_of(c);
    // few runs (the exchange's owners - 1): each region's block searches its segments itself;
    // otherwise one pass over every record writes the bounds (d_bounds)
    const bool search = n_runs <= kMergeSearchRuns;
    if (!search)
        hipLaunchKernelGGL((k_run_bounds<Recs>), dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, t, recs,
                           d_run_offsets, n_runs, reg_lo, nreg, d_bounds);
    if (nreg) {
        const size_t lds = ((size_t)1 << c->slice_log) * 16;
        hipLaunchKernelGGL((k_merge_runs<Recs>), dim3(nreg), dim3(kMergeT), lds, s, t, recs, d_run_offsets, n_runs,
                           reg_lo, nreg, search ? (const uint32_t*)nullptr : (const uint32_t*)d_bounds);
    }
    hipLaunchKernelGGL((k_merge_sentinel<Recs>), dim3(1), dim3(64), 0, s, t, recs, d_run_offsets, n_runs);
    return ss_check(hipGetLastError(), what);
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------------------------------------
// The drop-in engine's length classes counted by fingerprint (ss_classes_* in ss_internal.h).  The
// classes' rows (W1 = W + 1 words: the read's words and its length) are counted by their 64-bit
// fingerprint alone in one single-word scratch table `fpt` (ss_counter_insert_keys: the optimistic
// partitioned insert on 8-B keys, 12-B records, no row gathers), then
//   k_cls_verify: every row is compared with the first row of its fingerprint (the scratch entry's
//     first index is that row's place in the classes' combined row array): a difference means two
//     keys share a fingerprint and raises *flag (the engine then counts those classes again on the
//     exact multi-word path, whose aggregate decides equality on the words; the class tables are
//     untouched until the fold)
//   k_cls_fold_find / k_cls_fold_claim: unless *flag, every scratch entry -- a distinct key now --
//     goes into its class's table with ss_counter_merge_words' two phases, its words taken from its
//     first row.
// The row gathers this replaces (the multi-word aggregate read its own row and its representative's
// for every record: 1.9-3.3 ms of the f2 batch) become one compare per row against a row of ~1M
// distinct representatives that stay in the Infinity Cache.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kMaxClassesDesc = 32;
struct ClsDesc {
    Tbl tbl[kMaxClassesDesc];
    const uint64_t* rows[kMaxClassesDesc];
    uint64_t row0[kMaxClassesDesc + 1];     // combined row index of each class's first row; [ncls] = total
    uint64_t base[kMaxClassesDesc];         // the class table's first row index for this insert
    uint32_t W1[kMaxClassesDesc];
    uint32_t ncls;
};

__device__ __forceinline__ uint32_t cls_of(const ClsDesc& d, uint64_t g) {
    uint32_t c = 0;
    while (c + 1 < d.ncls && g >= d.row0[c + 1]) ++c;
    return c;
}

// the scratch slot holding key fp (kEmpty when absent)
__device__ __forceinline__ uint64_t find_slot(const Tbl& t, uint64_t fp) {
    const uint64_t top = slot_top(t, fp), base = top & ~t.slice_mask;
    uint64_t off = top & t.slice_mask;
    for (uint64_t probe = 0; probe <= t.slice_mask; ++probe) {
        const uint64_t k = t.slots[base + off].key;
        if (k == fp) return base + off;
        if (k == kEmpty) return kEmpty;
        off = (off + 1) & t.slice_mask;
    }
    return kEmpty;
}

__global__ __launch_bounds__(256) void k_cls_verify(Tbl f, ClsDesc d, const uint64_t* __restrict__ fps,
                                                    uint32_t* __restrict__ flag) {
    const uint64_t n = d.row0[d.ncls];
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < n; g += (uint64_t)gridDim.x * 256) {
        const uint32_t c = cls_of(d, g);
        const uint64_t sl = find_slot(f, fps[g]);
        bool bad = sl == kEmpty;
        if (!bad) {
            const uint64_t rep = f.slots[sl].first;
            if (rep != g) {
                bad = rep < d.row0[c] || rep >= d.row0[c + 1];
                if (!bad) {
                    const uint32_t W1 = d.W1[c];
                    const uint64_t* a = d.rows[c] + (g - d.row0[c]) * W1;
                    const uint64_t* b = d.rows[c] + (rep - d.row0[c]) * W1;
                    for (uint32_t j = 0; j < W1; ++j) bad |= a[j] != b[j];
                }
            }
        }
        if (__ballot(bad) && bad) atomicOr(flag, 1u);
    }
}

// The representatives beside the scratch slots (verify on rows of <= kRepW1 words): rep[s] = 64 B =
// {slot s's key, its first row's W1 words, .., its class in word 7} (kEmpty key: a free slot), so the
// check of a row is ONE 64-B read at its fingerprint's home slot (linear probing continues rarely)
// instead of a slot probe plus a gather of the representative's row.  The table of 2^21 slots is
// 128 MB: it stays in the Infinity Cache while the rows stream past.
constexpr uint32_t kRepW1 = 6;
__global__ __launch_bounds__(256) void k_cls_reps(Tbl f, ClsDesc d, uint64_t* __restrict__ rep) {
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s <= f.mask; s += (uint64_t)gridDim.x * 256) {
        const Slot sl = f.slots[s];
        uint64_t v[8] = {sl.key, 0, 0, 0, 0, 0, 0, ~0ull};
        if (sl.key != kEmpty) {
            const uint64_t g = sl.first;
            const uint32_t c = cls_of(d, g);
            const uint64_t* kw = d.rows[c] + (g - d.row0[c]) * d.W1[c];
            for (uint32_t j = 0; j < d.W1[c]; ++j) v[1 + j] = kw[j];
            v[7] = c;
        }
        uint4* dst = (uint4*)(rep + s * 8);
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k] = make_uint4((uint32_t)v[2 * k], (uint32_t)(v[2 * k] >> 32), (uint32_t)v[2 * k + 1],
                                                       (uint32_t)(v[2 * k + 1] >> 32));
    }
}

__global__ __launch_bounds__(256) void k_cls_verify_rep(Tbl f, ClsDesc d, const uint64_t* __restrict__ fps,
                                                        const uint64_t* __restrict__ rep, uint32_t* __restrict__ flag) {
    const uint64_t n = d.row0[d.ncls];
    const uint64_t G = (uint64_t)gridDim.x * 256;
    // two rows per lane per round: both rows' words and fingerprints, then both home slots'
    // representatives, in flight together (clamped, unconditional loads: a branch between them
    // serializes the round trips, and a lane's rounds are the kernel's critical path)
    for (uint64_t g0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; g0 < n; g0 += 2 * G) {
        uint32_t c[2], W1[2];
        uint64_t aw[2][kRepW1], fp[2], base[2], off[2];
        uint4 e[2][4];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint64_t g = min(g0 + k * G, n - 1);
            c[k] = cls_of(d, g);
            W1[k] = d.W1[c[k]];
            const uint64_t* a = d.rows[c[k]] + (g - d.row0[c[k]]) * W1[k];
#pragma unroll
            for (uint32_t j = 0; j < kRepW1; ++j) aw[k][j] = a[min(j, W1[k] - 1)];
            fp[k] = fps[g];
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint64_t top = slot_top(f, fp[k]);
            base[k] = top & ~f.slice_mask;
            off[k] = top & f.slice_mask;
            const uint4* p = (const uint4*)(rep + (base[k] + off[k]) * 8);
#pragma unroll
            for (int j = 0; j < 4; ++j) e[k][j] = p[j];
        }
        bool bad = false;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            bool b = true;
            for (uint64_t probe = 0; probe <= f.slice_mask; ++probe) {
                if (probe) {        // the home slot held another key: linear probing continues (rare)
                    off[k] = (off[k] + 1) & f.slice_mask;
                    const uint4* p = (const uint4*)(rep + (base[k] + off[k]) * 8);
#pragma unroll
                    for (int j = 0; j < 4; ++j) e[k][j] = p[j];
                }
                const uint64_t key = (uint64_t)e[k][0].y << 32 | e[k][0].x;
                if (key == fp[k]) {
                    const uint64_t rw[7] = {(uint64_t)e[k][0].w << 32 | e[k][0].z, (uint64_t)e[k][1].y << 32 | e[k][1].x,
                                            (uint64_t)e[k][1].w << 32 | e[k][1].z, (uint64_t)e[k][2].y << 32 | e[k][2].x,
                                            (uint64_t)e[k][2].w << 32 | e[k][2].z, (uint64_t)e[k][3].y << 32 | e[k][3].x,
                                            (uint64_t)e[k][3].w << 32 | e[k][3].z};
                    b = (uint32_t)rw[6] != c[k];
#pragma unroll
                    for (uint32_t j = 0; j < kRepW1; ++j) b |= j < W1[k] && aw[k][j] != rw[j];
                    break;
                }
                if (key == kEmpty) break;
            }
            bad |= b && g0 + k * G < n;
        }
        if (__ballot(bad) && bad) atomicOr(flag, 1u);
    }
}

// scratch slot s (an entry: key fp, ~count, first row g) -> its class and first row's words
__device__ __forceinline__ bool fold_entry(const Tbl& f, const ClsDesc& d, uint64_t s, uint64_t& fp, uint32_t& cnt,
                                           uint32_t& c, const uint64_t*& kw, uint64_t& first) {
    const Slot sl = f.slots[s];
    if (s > f.mask || sl.key == kEmpty) return false;
    fp = sl.key;
    cnt = ~sl.ncount;
    const uint64_t g = sl.first;
    c = cls_of(d, g);
    kw = d.rows[c] + (g - d.row0[c]) * d.W1[c];
    first = d.base[c] + (g - d.row0[c]);
    return true;
}

__global__ __launch_bounds__(256) void k_cls_fold_find(Tbl f, ClsDesc d, const uint32_t* __restrict__ flag,
                                                       uint64_t* __restrict__ found) {
    if (*flag) return;
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s <= f.mask; s += (uint64_t)gridDim.x * 256) {
        uint64_t fp, first;
        uint32_t cnt, c;
        const uint64_t* kw;
        uint64_t at = kEmpty;
        if (fold_entry(f, d, s, fp, cnt, c, kw, first)) {
            const Tbl& t = d.tbl[c];
            const uint64_t top = slot_top(t, fp), base = top & ~t.slice_mask;
            uint64_t off = top & t.slice_mask;
            for (uint64_t probe = 0; probe <= t.slice_mask; ++probe) {
                const uint64_t k = t.slots[base + off].key;
                if (k == kEmpty) break;
                if (k == fp && words_eq(t.keywords + (base + off) * t.W, kw, t.W)) {
                    at = base + off;
                    break;
                }
                off = (off + 1) & t.slice_mask;
            }
        }
        found[s] = at;
    }
}

__global__ __launch_bounds__(256) void k_cls_fold_claim(Tbl f, ClsDesc d, const uint32_t* __restrict__ flag,
                                                        const uint64_t* __restrict__ found) {
    if (*flag) return;
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s <= f.mask; s += (uint64_t)gridDim.x * 256) {
        uint64_t fp, first;
        uint32_t cnt, c;
        const uint64_t* kw;
        if (!fold_entry(f, d, s, fp, cnt, c, kw, first)) continue;
        const Tbl& t = d.tbl[c];
        if (first > kMaxIndex) {
            atomicOr(t.overflow, kOvfIndex);
            first = kMaxIndex;
        }
        uint64_t at = found[s];
        if (at == kEmpty) {
            const uint64_t top = slot_top(t, fp), base = top & ~t.slice_mask;
            uint64_t off = top & t.slice_mask;
            for (uint64_t probe = 0; probe <= t.slice_mask; ++probe) {
                if (t.slots[base + off].key == kEmpty &&
                    atomicCAS(&t.slots[base + off].key, (unsigned long long)kEmpty, (unsigned long long)fp) == kEmpty) {
                    at = base + off;
                    break;
                }
                off = (off + 1) & t.slice_mask;
            }
            if (at == kEmpty) {
                atomicOr(t.overflow, kOvfTable);
                continue;
            }
            uint64_t* dst = t.keywords + at * t.W;
            for (uint32_t q = 0; q < t.W; ++q) dst[q] = kw[q];
            t.slots[at].ncount = ~cnt;
            t.slots[at].first = (uint32_t)first;
            continue;
        }
        atomicAdd(&t.slots[at].ncount, 0u - cnt);
        if (t.slots[at].first > (uint32_t)first) atomicMin(&t.slots[at].first, (uint32_t)first);
    }
}

// ---- the same on read-order rows (k_encode_rows: read r's row at rows + r * S, S <= kRepW1 words:
// its W words, its length, zeros).  The scratch entry's first index is a read; the representative
// carries the row's S words and its class W (the index of its last nonzero word: the length; 0 for
// the zero row of a read that is no class read, an entry the fold skips).  A whole-row compare
// decides equality (the zero tail is part of every row), so verify needs no class lookups; the fold
// gives each new key its class table's next row (a wave-aggregated counter per class) and writes
// that row's read index into the class's row map.
struct FlatDesc {
    Tbl tbl[kRepW1];                // class W's table (W = 2 .. kRepW1 - 1; W1 = W + 1 <= S)
    uint64_t row0[kRepW1];          // its first row of this chunk (the row counter adds to it)
    uint64_t* rmap[kRepW1];         // its row map at row0
    uint64_t base;                  // global read index of the chunk's read 0
    uint32_t S;
};

// rep layout, 8 u64 per scratch slot: the row's words w0 .. w5 (zeros past S), the key, the class W --
// so the 16-B pieces of a representative line up with the row's own pieces (w0 w1 | w2 w3 | w4 w5) and
// with (key, W) last, one piece per lane of k_flat_verify's quads
// Two slots per step, every load branch-free (an empty slot's row loads are dropped), so a step waits
// for one slot round trip and one row round trip for both slots: the grid-stride loop walks ~32 slots
// per thread, and a used slot's row load depends on its slot
constexpr int kRepU = 2;
__global__ __launch_bounds__(256) void k_flat_reps(Tbl f, const uint64_t* __restrict__ rows, uint32_t S,
                                                   uint64_t* __restrict__ rep) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t s0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; s0 <= f.mask; s0 += kRepU * stride) {
        Slot sl[kRepU];
#pragma unroll
        for (int u = 0; u < kRepU; ++u) sl[u] = f.slots[min(s0 + u * stride, f.mask)];
        uint64_t v[kRepU][8];
#pragma unroll
        for (int u = 0; u < kRepU; ++u) {
            const bool used = sl[u].key != kEmpty;
            // (an empty slot reads the table's own first words: always there, whatever the rows hold)
            const uint64_t* row = used ? rows + (uint64_t)sl[u].first * S : (const uint64_t*)f.slots;
#pragma unroll
            for (uint32_t j = 0; j < kRepW1; ++j) v[u][j] = row[min(j, S - 1)];
        }
#pragma unroll
        for (int u = 0; u < kRepU; ++u) {
            const uint64_t s = s0 + u * stride;
            if (s > f.mask) continue;
            const bool used = sl[u].key != kEmpty;
            uint64_t w[8];
            w[6] = sl[u].key;
            w[7] = 0;
#pragma unroll
            for (uint32_t j = 0; j < kRepW1; ++j) {
                w[j] = (used && j < S) ? v[u][j] : 0ull;
                if (w[j]) w[7] = j;
            }
            uint4* dst = (uint4*)(rep + s * 8);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                dst[k] = make_uint4((uint32_t)w[2 * k], (uint32_t)(w[2 * k] >> 32), (uint32_t)w[2 * k + 1],
                                    (uint32_t)(w[2 * k + 1] >> 32));
        }
    }
}

// Every row against the representative of its fingerprint's slot, a quad of lanes per row: lane q
// (0..2) loads the row's 16-B piece q (words 2q, 2q + 1) and the representative's piece q, lane 3
// the representative's (key, W); the quad's four compares are AND-ed by two DPP quad permutes.  A
// wave-instruction thus loads 16 whole rows (768 contiguous bytes) and 16 whole 64-B
// representatives -- one cache line each -- where a lane per row issued six 8-B row loads and four
// 16-B representative loads, each of the latter touching 64 different lines.  kFlatQK rows per quad
// are in flight before any compare.  Every lane loads the row's fingerprint (the quad's four lanes
// read one address).  A key other than the fingerprint at the slot sends the quad on to the next
// slot (linear probing inside the slice); an empty slot or a word difference raises the flag.
constexpr int kFlatQK = 4;
__device__ __forceinline__ uint32_t quad_and(uint32_t v) {
    v &= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);    // quad_perm [1, 0, 3, 2]
    v &= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);    // quad_perm [2, 3, 0, 1]
    return v;
}

__global__ __launch_bounds__(256) void k_flat_verify(Tbl f, const uint64_t* __restrict__ rows, uint32_t S, uint64_t n,
                                                     const uint64_t* __restrict__ fps, const uint64_t* __restrict__ rep,
                                                     uint32_t* __restrict__ flag) {
    const uint32_t q = threadIdx.x & 3u;
    const uint64_t nq = (uint64_t)gridDim.x * 64u;
    const uint64_t quad = (uint64_t)blockIdx.x * 64u + (threadIdx.x >> 2);
    // this lane's words of a row: 2q, 2q + 1 (masked past S)
    const bool w0in = 2u * q < S, w1in = 2u * q + 1u < S;
    bool bad = false;
    for (uint64_t r0 = quad; r0 < n; r0 += kFlatQK * nq) {
        uint4 a[kFlatQK], e[kFlatQK];
        uint64_t fp[kFlatQK], at[kFlatQK];
#pragma unroll
        for (int k = 0; k < kFlatQK; ++k) {
            const uint64_t r = min(r0 + (uint64_t)k * nq, n - 1);
            a[k] = make_uint4(0u, 0u, 0u, 0u);
            if (w0in) a[k] = *(const uint4*)(rows + r * S + 2u * q);
            fp[k] = fps[r];
        }
#pragma unroll
        for (int k = 0; k < kFlatQK; ++k) {
            if (!w1in) a[k].z = a[k].w = 0u;
            if (!w0in) a[k].x = a[k].y = 0u;
            at[k] = slot_top(f, fp[k]);
            e[k] = *(const uint4*)(rep + at[k] * 8 + 2u * q);
        }
        // The kFlatQK rows probe in lockstep: each round decides every row still open and issues the
        // next slot's loads of all of them together, so a wave waits for one dependent round trip per
        // probe round of its longest row, where a probe loop per row waited for each row's displaced
        // quads in turn (most rounds have one: 16 quads per row, ~1 in 3 fingerprints off its home)
        uint32_t open = (1u << kFlatQK) - 1u;
        uint32_t probes[kFlatQK];
#pragma unroll
        for (int k = 0; k < kFlatQK; ++k) probes[k] = 0;
        for (;;) {
#pragma unroll
            for (int k = 0; k < kFlatQK; ++k) {
                if (!(open & (1u << k))) continue;     // (quad-uniform: the quad decides together)
                const bool live = r0 + (uint64_t)k * nq < n;
                const uint64_t key = (uint64_t)e[k].y << 32 | e[k].x;     // lane 3's piece: (key, W)
                const bool same = a[k].x == e[k].x && a[k].y == e[k].y && a[k].z == e[k].z && a[k].w == e[k].w;
                const uint32_t bits = (q < 3u ? (same ? 1u : 0u) | 6u
                                              : 1u | (key == fp[k] ? 2u : 0u) | (key != kEmpty ? 4u : 0u));
                const uint32_t all = quad_and(bits);
                if (all & 2u) {              // the fingerprint's slot: its words decide
                    bad |= live && !(all & 1u);
                    open &= ~(1u << k);
                } else if (!(all & 4u) || probes[k] == f.slice_mask) {
                    bad |= live;             // an empty slot: the fingerprint was never inserted
                    open &= ~(1u << k);
                }
            }
            if (!__ballot(open != 0u)) break;
#pragma unroll
            for (int k = 0; k < kFlatQK; ++k) {
                if (!(open & (1u << k))) continue;
                ++probes[k];
                at[k] = (at[k] & ~f.slice_mask) | ((at[k] + 1) & f.slice_mask);
                e[k] = *(const uint4*)(rep + at[k] * 8 + 2u * q);
            }
        }
    }
    if (__ballot(bad) && bad) atomicOr(flag, 1u);
}

// scratch slot s -> (fp, count, first read, class W, the rep's words); false for a free slot, the
// zero row's entry, or a class without a table
__device__ __forceinline__ bool flat_entry(const Tbl& f, const FlatDesc& d, const uint64_t* rep, uint64_t s,
                                           uint64_t& fp, uint32_t& cnt, uint32_t& W, const uint64_t*& kw,
                                           uint64_t& first) {
    if (s > f.mask) return false;
    const Slot sl = f.slots[s];
    if (sl.key == kEmpty) return false;
    W = (uint32_t)rep[s * 8 + 7];
    if (W < 2 || W + 1 > d.S || !d.tbl[W].slots) return false;
    fp = sl.key;
    cnt = ~sl.ncount;
    first = sl.first;
    kw = rep + s * 8;
    return true;
}

// find: the class table slot of each entry's key (kEmpty: a new key), and per block the new keys of
// each class (blkcnt[block * kRepW1 + W]); k_flat_fold_scan turns those into each block's first
// row per class; claim (the same grid, the same slots per block) gives each new key its block's
// next row (LDS counters) -- no contended global counters (one per class, wave-aggregated, took
// 3.1 ms on the f2 batch)
// EXTRACT (the class tables are known to be empty, ss_classes_flat_extract): every entry is new, no
// probe; found is not written
extern "C++" {      // (a template inside this file's extern "C" section)
// The extract's entry loads, all issued together: the slot and its whole 64-B representative (the
// words, the key, the class) do not depend on each other, so a grid-stride step waits one round
// trip instead of three (slot -> class -> words, as flat_entry does); kFlatXU slots per step are in
// flight.  Empty slots' representatives are read too (sequential 64-B rows: whole lines).
constexpr int kFlatXU = 2;
struct FlatLoad {
    uint4 sl;
    uint4 r[4];
};
__device__ __forceinline__ void flat_load(const Tbl& f, const uint64_t* rep, uint64_t s, FlatLoad& e) {
    const uint64_t sc = min(s, f.mask);                 // (past the table: decoded as no entry)
    e.sl = *(const uint4*)&f.slots[sc];
    const uint4* rp = (const uint4*)(rep + sc * 8);
#pragma unroll
    for (int k = 0; k < 4; ++k) e.r[k] = rp[k];
}
// flat_entry's rule on loaded values: the class W (rep word 7) and the slot's count and first read
__device__ __forceinline__ bool flat_decode(const Tbl& f, const FlatDesc& d, uint64_t s, const FlatLoad& e,
                                            uint32_t& cnt, uint32_t& W, uint64_t& first) {
    if (s > f.mask || (e.sl.x == 0xFFFFFFFFu && e.sl.y == 0xFFFFFFFFu)) return false;   // (kEmpty key)
    W = e.r[3].z;
    if (W < 2 || W + 1 > d.S || !d.tbl[W].slots) return false;
    cnt = ~e.sl.z;
    first = e.sl.w;
    return true;
}

template <bool EXTRACT>
__global__ __launch_bounds__(256) void k_flat_fold_find(Tbl f, FlatDesc d, const uint64_t* __restrict__ rep,
                                                        const uint32_t* __restrict__ flag, uint64_t* __restrict__ found,
                                                        uint32_t* __restrict__ blkcnt) {
    __shared__ uint32_t lc[kRepW1];
    if (threadIdx.x < kRepW1) lc[threadIdx.x] = 0;
    __syncthreads();
    // EXTRACT: the per-block count of k_flat_extract_claim's rows (the same slots per block); the
    // slot, then its class word -- the branch-free form of the claim (slot and whole representative
    // together) read 0.5 GB more here for the empty slots and measured 0.37 -> 0.43 ms at 2^24
    if (EXTRACT && !*flag) {
        for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s <= f.mask; s += (uint64_t)gridDim.x * 256) {
            uint64_t fp, first;
            uint32_t cnt, W;
            const uint64_t* kw;
            if (flat_entry(f, d, rep, s, fp, cnt, W, kw, first)) atomicAdd(&lc[W], 1u);
        }
    } else if (!*flag) {
        for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s <= f.mask; s += (uint64_t)gridDim.x * 256) {
            uint64_t fp, first, at = kEmpty;
            uint32_t cnt, W;
            const uint64_t* kw;
            if (flat_entry(f, d, rep, s, fp, cnt, W, kw, first)) {
                const Tbl& t = d.tbl[W];
                const uint64_t top = slot_top(t, fp), base = top & ~t.slice_mask;
                uint64_t off = top & t.slice_mask;
                for (uint64_t probe = 0; probe <= t.slice_mask; ++probe) {
                    const uint64_t k = t.slots[base + off].key;
                    if (k == kEmpty) break;
                    if (k == fp && words_eq(t.keywords + (base + off) * t.W, kw, t.W)) {
                        at = base + off;
                        break;
                    }
                    off = (off + 1) & t.slice_mask;
                }
                if (at == kEmpty) atomicAdd(&lc[W], 1u);
            }
            found[s] = at;
        }
    }
    __syncthreads();
    if (threadIdx.x < kRepW1) blkcnt[(uint64_t)blockIdx.x * kRepW1 + threadIdx.x] = lc[threadIdx.x];
}
}  // extern "C++"

// one block: blkcnt -> each block's first row per class (exclusive scan over the blocks, in place)
struct FlatTotals {
    uint64_t* p[kRepW1];            // class W's total (entries of the scratch of class W), null: not wanted
};

// (256 threads: the extract runs on the speculative finish's stream beside the verify, where a
// 1024-thread workgroup waited up to ~0.5 ms for one CU to free 16 wave slots)
__global__ __launch_bounds__(256) void k_flat_fold_scan(uint32_t* __restrict__ blkcnt, uint32_t nblk, FlatTotals tot) {
    __shared__ uint32_t carry[kRepW1];
    __shared__ uint32_t wsum[4][kRepW1];
    if (threadIdx.x < kRepW1) carry[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    for (uint32_t b0 = 0; b0 < nblk; b0 += 256) {
        const uint32_t b = b0 + threadIdx.x;
        uint32_t v[kRepW1], inc[kRepW1];
#pragma unroll
        for (uint32_t W = 0; W < kRepW1; ++W) {
            v[W] = b < nblk ? blkcnt[(uint64_t)b * kRepW1 + W] : 0u;
            inc[W] = v[W];
            for (uint32_t o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc[W], o);
                if (lane >= o) inc[W] += y;
            }
            if (lane == 63) wsum[wave][W] = inc[W];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t W = 0; W < kRepW1; ++W) {
            uint32_t before = carry[W];
            for (uint32_t u = 0; u < wave; ++u) before += wsum[u][W];
            if (b < nblk) blkcnt[(uint64_t)b * kRepW1 + W] = before + inc[W] - v[W];
        }
        __syncthreads();
        if (threadIdx.x < kRepW1)
            for (uint32_t u = 0; u < 4; ++u) carry[threadIdx.x] += wsum[u][threadIdx.x];
        __syncthreads();
    }
    if (threadIdx.x < kRepW1 && tot.p[threadIdx.x]) *tot.p[threadIdx.x] = carry[threadIdx.x];
}

__global__ __launch_bounds__(256) void k_flat_fold_claim(Tbl f, FlatDesc d, const uint64_t* __restrict__ rep,
                                                         const uint32_t* __restrict__ flag,
                                                         const uint64_t* __restrict__ found,
                                                         const uint32_t* __restrict__ blkoff) {
    __shared__ uint32_t lc[kRepW1];
    if (threadIdx.x < kRepW1) lc[threadIdx.x] = blkoff[(uint64_t)blockIdx.x * kRepW1 + threadIdx.x];
    __syncthreads();
    if (*flag) return;
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s <= f.mask; s += (uint64_t)gridDim.x * 256) {
        uint64_t fp, first;
        uint32_t cnt, W;
        const uint64_t* kw;
        if (!flat_entry(f, d, rep, s, fp, cnt, W, kw, first)) continue;
        const Tbl& t = d.tbl[W];
        const uint64_t at0 = found[s];
        if (at0 != kEmpty) {
            atomicAdd(&t.slots[at0].ncount, 0u - cnt);
            continue;
        }
        const uint32_t row = atomicAdd(&lc[W], 1u);     // LDS: this block's next row of class W
        d.rmap[W][row] = d.base + first;
        uint64_t trow = d.row0[W] + row;
        if (trow > kMaxIndex) {
            atomicOr(t.overflow, kOvfIndex);
            trow = kMaxIndex;
        }
        const uint64_t top = slot_top(t, fp), base = top & ~t.slice_mask;
        uint64_t off = top & t.slice_mask, at = kEmpty;
        for (uint64_t probe = 0; probe <= t.slice_mask; ++probe) {
            if (t.slots[base + off].key == kEmpty &&
                atomicCAS(&t.slots[base + off].key, (unsigned long long)kEmpty, (unsigned long long)fp) == kEmpty) {
                at = base + off;
                break;
            }
            off = (off + 1) & t.slice_mask;
        }
        if (at == kEmpty) {
            atomicOr(t.overflow, kOvfTable);
            continue;
        }
        uint64_t* dst = t.keywords + at * t.W;
        for (uint32_t q = 0; q < t.W; ++q) dst[q] = kw[q];
        t.slots[at].ncount = ~cnt;
        t.slots[at].first = (uint32_t)trow;
    }
}

// the scratch's entries of every class as dense per-class arrays in the fold's row order (the rows
// k_flat_fold_claim would give them in empty class tables): class W's entry at row gets its W + 1
// key words (the W words and the length: the class table's key layout), its count, first = row, and
// rmap[row] = base + its first read -- the layout ss_counter_extract_words gives the finish
struct FlatOut {
    uint64_t* words[kRepW1];
    uint64_t* counts[kRepW1];
    uint64_t* first[kRepW1];
    uint64_t* rmap[kRepW1];
    unsigned long long* ovf[kRepW1];
    uint64_t cap[kRepW1];
};

__global__ __launch_bounds__(256) void k_flat_extract_claim(Tbl f, FlatDesc d, FlatOut o, const uint64_t* __restrict__ rep,
                                                            const uint32_t* __restrict__ blkoff) {
    __shared__ uint32_t lc[kRepW1];
    if (threadIdx.x < kRepW1) lc[threadIdx.x] = blkoff[(uint64_t)blockIdx.x * kRepW1 + threadIdx.x];
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t s0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; s0 <= f.mask; s0 += kFlatXU * stride) {
        FlatLoad e[kFlatXU];
#pragma unroll
        for (int u = 0; u < kFlatXU; ++u) flat_load(f, rep, s0 + u * stride, e[u]);
#pragma unroll
        for (int u = 0; u < kFlatXU; ++u) {
            uint64_t first;
            uint32_t cnt, W;
            if (!flat_decode(f, d, s0 + u * stride, e[u], cnt, W, first)) continue;
            const uint32_t row = atomicAdd(&lc[W], 1u);     // LDS: this block's next row of class W
            if (row >= o.cap[W]) {
                atomicOr(o.ovf[W], (unsigned long long)kOvfTable);
                continue;
            }
            o.rmap[W][row] = d.base + first;
            o.counts[W][row] = cnt;
            o.first[W][row] = row;
            uint64_t* dst = o.words[W] + (uint64_t)row * (W + 1);
            const uint32_t wd[12] = {e[u].r[0].x, e[u].r[0].y, e[u].r[0].z, e[u].r[0].w, e[u].r[1].x, e[u].r[1].y,
                                     e[u].r[1].z, e[u].r[1].w, e[u].r[2].x, e[u].r[2].y, e[u].r[2].z, e[u].r[2].w};
#pragma unroll
            for (uint32_t q = 0; q < kRepW1; ++q)
                if (q <= W) dst[q] = (uint64_t)wd[2 * q] | ((uint64_t)wd[2 * q + 1] << 32);
        }
    }
}

int ss_counter_create(uint64_t capacity, ss_counter** out) {
    if (!out) return ss_fail(SS_EARG, "null out");
    if (capacity < 64) capacity = 64;
    uint32_t lg = 0;
    while ((1ull << lg) < capacity) ++lg;
    if (lg > 40) return ss_fail(SS_EARG, "capacity too large");
    ss_counter* c = new ss_counter();
    c->cap = 1ull << lg;
    c->log2cap = lg;
    c->slice_log = lg < kSliceLogMax ? lg : kSliceLogMax;
    hipError_t e = hipMalloc((void**)&c->slots, (c->cap + 1) * sizeof(Slot));
    if (e == hipSuccess)
        e = hipMalloc((void**)&c->work, (1 + (size_t)kMaxParts * kExtractBlocks) * sizeof(unsigned long long));
    const uint64_t R = c->cap >> c->slice_log;
    if (e == hipSuccess && R <= kMaxRegions) {   // region occupancy + pack scratch (ss_counter_pack_ranges)
        e = hipMalloc((void**)&c->occ, R * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMalloc((void**)&c->roff, (R + 2) * sizeof(unsigned long long));
        c->occ_R = R;
    }
    if (e != hipSuccess) {
        ss_counter_destroy(c);
        ss_check(e, "ss_counter_create hipMalloc");
        return SS_ENOMEM;
    }
    int rc = ss_counter_reset(c, nullptr);
    if (rc == SS_OK) rc = flush_reset(c, nullptr);
    if (rc == SS_OK) rc = ss_check(hipStreamSynchronize(nullptr), "ss_counter_create sync");
    if (rc) {
        ss_counter_destroy(c);
        return rc;
    }
    *out = c;
    return SS_OK;
}

int ss_counter_set_timing(ss_counter* c, int on) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (on && !c->tev) {
        c->tev = new hipEvent_t[(uint64_t)ss_counter::kTimerRing * ss_counter::kPassEvents]();
        for (uint32_t k = 0; k < ss_counter::kTimerRing * ss_counter::kPassEvents; ++k)
            if (hipEventCreate(&c->tev[k]) != hipSuccess) return ss_check(hipGetLastError(), "timing events");
    } else if (!on && c->tev) {
        while (c->tpend) timer_fold_one(c);
        for (uint32_t k = 0; k < ss_counter::kTimerRing * ss_counter::kPassEvents; ++k)
            if (c->tev[k]) (void)hipEventDestroy(c->tev[k]);
        delete[] c->tev;
        c->tev = nullptr;
    }
    return SS_OK;
}

int ss_counter_pass_times(ss_counter* c, double* h_ms, uint64_t* h_inserts) {
    if (!c || !h_ms || !h_inserts) return ss_fail(SS_EARG, "null argument");
    while (c->tpend) timer_fold_one(c);
    *h_inserts = c->tn;
    for (uint32_t p = 0; p + 1 < ss_counter::kPassEvents; ++p) {
        h_ms[p] = c->tn ? c->tsum[p] / (double)c->tn : 0.0;
        c->tsum[p] = 0.0;
    }
    c->tn = 0;
    return SS_OK;
}

int ss_counter_destroy(ss_counter* c) {
    if (!c) return SS_OK;
    (void)ss_counter_set_timing(c, 0);
    if (c->slots) (void)hipFree(c->slots);
    if (c->work) (void)hipFree(c->work);
    if (c->keywords) (void)hipFree(c->keywords);
    if (c->wide) (void)hipFree(c->wide);
    if (c->occ) (void)hipFree(c->occ);
    if (c->roff) (void)hipFree(c->roff);
    if (c->aux) (void)hipFree(c->aux);
    ss_counter_release(c);
    if (c->ws_hist) (void)hipFree(c->ws_hist);
    if (c->ws_rstart) (void)hipFree(c->ws_rstart);
    if (c->ws_segend) (void)hipFree(c->ws_segend);
    if (c->ws_order) (void)hipFree(c->ws_order);
    if (c->ws_tot) (void)hipFree(c->ws_tot);
    if (c->ws_fill) (void)hipFree(c->ws_fill);
    delete c;
    return SS_OK;
}

// the handle's scratch of at least `bytes` (grown by hipFree + hipMalloc: the free waits for the
// device, so earlier users on any stream are done with it; same-stream users are ordered anyway)
static int aux_scratch(ss_counter* c, size_t bytes, void** out) {
    if (c->aux_bytes < bytes) {
        if (c->aux) (void)hipFree(c->aux);
        c->aux = nullptr;
        c->aux_bytes = 0;
        const size_t want = std::max(bytes, (size_t)1 << 20);
        if (hipMalloc(&c->aux, want) != hipSuccess) {
            ss_check(hipGetLastError(), "counter scratch hipMalloc");
            return ss_fail(SS_ENOMEM, "counter scratch: out of device memory");
        }
        c->aux_bytes = want;
    }
    *out = c->aux;
    return SS_OK;
}

// 8-B device words set by a stream write packet (no fill-kernel dispatch; the streamed C5 step ran
// four fills before its first pass); hipMemsetAsync where the runtime refuses the packet
static hipError_t set_u64(uint64_t* p, bool ones, hipStream_t s) {
    if (hipStreamWriteValue64(s, p, ones ? ~0ull : 0ull, 0) == hipSuccess) return hipSuccess;
    (void)hipGetLastError();
    return hipMemsetAsync(p, ones ? 0xFF : 0, sizeof(uint64_t), s);
}

// the host half of a reset; the three device words it needs set go to p / v
int ss_counter_reset_host(ss_counter* c, unsigned long long** p, unsigned long long* v) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    c->L = -1;
    c->occ_src = 0;
    c->wide_live = false;       // (zeroed when it next goes live)
    c->since = 0;
    c->reset_pending = true;    // the slots [0, cap): flush_reset or a fresh aggregate
    unsigned long long* sent = (unsigned long long*)(c->slots + c->cap);     // the sentinel slot
    p[0] = sent;
    v[0] = ~0ull;
    p[1] = sent + 1;
    v[1] = ~0ull;
    p[2] = c->work;                                                          // overflow flags
    v[2] = 0ull;
    return SS_OK;
}

int ss_counter_reset(ss_counter* c, void* stream) {
    PrepWords w{};
    const int rc = ss_counter_reset_host(c, w.p, w.v);
    if (rc) return rc;
    return ss_check(launch_prep(w, (hipStream_t)stream), "ss_counter_reset");
}

// Several tables' reset words in one dispatch (the drop-in engine resets up to six tables between
// two kernels of a chunk; one launch each left ~5 us of command-processor gap between them)
struct PrepMany {
    unsigned long long* p[kPrepMany];
    unsigned long long v[kPrepMany];
    uint32_t n;
};
__global__ __launch_bounds__(64) void k_prep_many(PrepMany w) {
    if (threadIdx.x < w.n) *w.p[threadIdx.x] = w.v[threadIdx.x];
}

int ss_prep_words(unsigned long long* const* p, const unsigned long long* v, uint32_t n, void* stream) {
    if (n > kPrepMany) return ss_fail(SS_EARG, "ss_prep_words: too many words");
    if (!n) return SS_OK;
    PrepMany w{};
    for (uint32_t i = 0; i < n; ++i) {
        w.p[i] = p[i];
        w.v[i] = v[i];
    }
    w.n = n;
    hipLaunchKernelGGL(k_prep_many, dim3(1), dim3(64), 0, (hipStream_t)stream, w);
    return ss_check(hipGetLastError(), "ss_prep_words");
}

uint64_t ss_counter_capacity(const ss_counter* c) { return c ? c->cap : 0; }

static int fix_length(ss_counter* c, uint32_t L) {
    if (L > SS_MAX_NT) return ss_fail(SS_ETOO_LONG, "Sequences longer than 1024 bases are not supported.");
    if (c->L == kWordKeys) return ss_fail(SS_EARG, "the handle holds packed multi-word keys");
    if (c->L >= 0) {
        if ((uint32_t)c->L != L) return ss_fail(SS_EARG, "all keys of one counter handle must share one length");
        return SS_OK;
    }
    const uint32_t W = L <= 32 ? 1u : (L + 31) / 32;
    if (W > 1 && c->keywords_W != W) {   // key words of a multi-word table: [cap * W]
        if (c->keywords) (void)hipFree(c->keywords);
        c->keywords = nullptr;
        c->keywords_W = 0;
        if (hipMalloc((void**)&c->keywords, c->cap * W * sizeof(uint64_t)) != hipSuccess) {
            ss_check(hipGetLastError(), "counter key words hipMalloc");
            return ss_fail(SS_ENOMEM, "counter key words: out of device memory");
        }
        c->keywords_W = W;
    }
    c->W = W;
    c->L = (int32_t)L;
    return SS_OK;
}

int ss_counter_reserve(ss_counter* c, uint64_t max_reads) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    const uint64_t R = c->cap >> c->slice_log;
    if (R > kMaxRegions) return ss_fail(SS_EARG, "capacity too large for the partitioned insert");
    if (max_reads >= (1ull << 31)) return ss_fail(SS_EARG, "max_reads must be < 2^31 per insert");
    if (max_reads <= c->ws_reads) return SS_OK;
    ss_counter_release(c);
    // coarse arrays: room for the exact passes (max_reads) and for the optimistic partition's
    // 128 x 8 sub-bins of cap1 = 2.5 x the mean sub-bin load + 1024 slots (pf_cap1)
    const uint64_t cap1 = pf_cap1(max_reads);
    const uint64_t acap = kNFill * cap1 > max_reads ? kNFill * cap1 : max_reads;
    // fine-pass slabs (optimistic path, R > 128 regions): every (sub-bin, region of its bin) gets
    // slab_size(sub-bin fill) record slots (2 x its mean share + 256; k_pf_order lays them out once
    // the coarse fills are known), so the fine scatter needs no count pass; a slab that runs full
    // sends the rest to the spill list.  Only where the mean share is >= kSlabMinMean (the per-slab
    // slack would dominate small reservations) and the slots index in 32 bits.
    c->ws_slab = 0;
    c->ws_brecs = max_reads;
    if (R > (1u << kCoarseBits) && R <= (1u << (kCoarseBits + 8))) {
        const uint64_t nslab = (uint64_t)kNFill * (R >> kCoarseBits);
        const uint64_t mean = max_reads / nslab;
        // sum over sub-bins of nb x slab_size(fill, nb), fills summing to <= max_reads
        const uint64_t brecs = 2 * max_reads + nslab * (2 + kSlabPad + 15);
        if (mean >= kSlabMinMean && brecs < (1ull << 32)) {
            c->ws_slab = 1;
            c->ws_brecs = brecs > max_reads ? brecs : max_reads;
        }
    }
    const uint64_t brecs = c->ws_brecs;
    // ws_keys / ws_akey: 12-B records on the optimistic path, u64 keys on the exact paths
    hipError_t e = hipMalloc((void**)&c->ws_keys, brecs * sizeof(Rec12));
    if (e == hipSuccess) e = hipMalloc((void**)&c->ws_akey, acap * sizeof(Rec12));
    // coarse read indices of the exact paths (the optimistic path keeps them in the 12-B records)
    if (e == hipSuccess) e = hipMalloc((void**)&c->ws_aidx, max_reads * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void**)&c->ws_acnt, acap * sizeof(uint32_t));
    if (e == hipSuccess && !c->ws_slab) e = hipMalloc((void**)&c->ws_areg, acap);   // counted cursors only
    if (e == hipSuccess && !c->ws_fill) e = hipMalloc((void**)&c->ws_fill, kFillWords * sizeof(uint32_t));
    c->ws_cap1 = cap1;
    if (e == hipSuccess) e = hipMalloc((void**)&c->ws_bidx, max_reads * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void**)&c->ws_bcnt, brecs * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void**)&c->ws_spill, max_reads * sizeof(uint4));
    if (e == hipSuccess && !c->ws_hist) e = hipMalloc((void**)&c->ws_hist, (size_t)kPartBlocks * R * sizeof(uint32_t));
    if (e == hipSuccess && !c->ws_rstart) e = hipMalloc((void**)&c->ws_rstart, (R + 1) * sizeof(uint32_t));
    // one entry per (sub-bin, region of its bin): kNFill x (R / 128) = R x kFinePerBin
    if (e == hipSuccess && !c->ws_order) e = hipMalloc((void**)&c->ws_order, 3 * kNFill * sizeof(uint32_t));
    if (e == hipSuccess && !c->ws_segend) e = hipMalloc((void**)&c->ws_segend, R * kFinePerBin * sizeof(uint32_t));
    if (e == hipSuccess && !c->ws_tot) e = hipMalloc((void**)&c->ws_tot, (R + 1) * sizeof(uint32_t));
    if (e != hipSuccess) {
        ss_counter_release(c);
        ss_check(e, "ss_counter_reserve hipMalloc");
        return SS_ENOMEM;
    }
    c->ws_reads = max_reads;
    return SS_OK;
}

uint64_t ss_counter_reserved(const ss_counter* c) { return c ? c->ws_reads : 0; }

int ss_counter_release(ss_counter* c) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (c->ws_keys) (void)hipFree(c->ws_keys);
    if (c->ws_akey) (void)hipFree(c->ws_akey);
    if (c->ws_aidx) (void)hipFree(c->ws_aidx);
    if (c->ws_acnt) (void)hipFree(c->ws_acnt);
    if (c->ws_areg) (void)hipFree(c->ws_areg);
    if (c->ws_bidx) (void)hipFree(c->ws_bidx);
    if (c->ws_bcnt) (void)hipFree(c->ws_bcnt);
    if (c->ws_spill) (void)hipFree(c->ws_spill);
    if (c->ws_words) (void)hipFree(c->ws_words);
    c->ws_words = nullptr;
    c->ws_words_cap = 0;
    c->ws_keys = nullptr;
    c->ws_akey = nullptr;
    c->ws_aidx = nullptr;
    c->ws_acnt = nullptr;
    c->ws_areg = nullptr;
    c->ws_bidx = nullptr;
    c->ws_bcnt = nullptr;
    c->ws_spill = nullptr;
    c->ws_reads = 0;
    c->ws_slab = 0;
    c->ws_brecs = 0;
    return SS_OK;
}

// words_in: pre-packed multi-word rows (ss_counter_insert_words; d_ascii / L / stride / d_first_bad
// unused), else ASCII reads of length L
static int insert_impl(ss_counter* c, const uint8_t* d_ascii, uint64_t n, uint32_t L, uint64_t stride,
                       uint64_t base_index, uint64_t* d_first_bad, void* stream, const uint64_t* words_in,
                       const uint64_t* keys_in = nullptr) {
    hipStream_t s = (hipStream_t)stream;
    int rc = SS_OK;
    if (keys_in) {     // precomputed single-word keys: always partitioned
        if (c->W != 1) return ss_fail(SS_EARG, "precomputed keys need a single-word handle");
        if (n == 0) return SS_OK;
        if (n > c->ws_reads && (rc = ss_counter_reserve(c, n)) != SS_OK) return rc;
    }
    const uint32_t rb = c->log2cap - c->slice_log;
    // the optimistic coarse partition below (the C5 path) resets first_bad with its sub-bin counters
    const bool opt = !words_in && n > 0 && n <= c->ws_reads && rb > kCoarseBits && rb - kCoarseBits <= 8 &&
                     (keys_in || (d_ascii && (L == 16 || L == 32) && stride % 16 == 0 && (((uintptr_t)d_ascii) & 15) == 0));
    if (keys_in) {
        // nothing to encode, no first_bad
    } else if (!words_in) {
        if (!d_first_bad) return ss_fail(SS_EARG, "d_first_bad is required");
        if (stride < L) return ss_fail(SS_EARG, "stride < L");
        if ((rc = fix_length(c, L))) return rc;
        if (!opt) rc = ss_check(set_u64(d_first_bad, true, s), "reset first_bad");
        if (rc || n == 0) return rc;
        if (!d_ascii) return ss_fail(SS_EARG, "null buffer");
    } else if (n == 0) {
        return SS_OK;
    }
    if (base_index > kMaxIndex || n - 1 > kMaxIndex - base_index)
        return ss_fail(SS_EARG, "global read indices of a counter handle must stay below 2^32 - 1");
    // u64 counts: a slot's u32 could wrap within this insert -> every count into wide first
    // (not the drop-in engine's packed-word class tables: it spills their counts per row itself,
    // ss_counter_spill_counts, and its class kernels read the slot counts directly)
    if (c->L != kWordKeys && c->since + n > c->spill_at && (rc = spill_wide(c, s))) return rc;
    c->since += n;
    c->occ_src = 0;   // set again below by the paths whose aggregate records the region occupancy
    Tbl t = tbl_of(c);
    const bool multi = c->W > 1;
    const bool fast = !words_in && !keys_in && (L == 16 || L == 32) && stride % 16 == 0 && (((uintptr_t)d_ascii) & 15) == 0;
    const uint64_t* mw = words_in;          // the multi-word rows the partition passes read
    if (multi) {
        // multi-word keys: always partitioned; grow the workspace to this batch if needed
        if (n > c->ws_reads && (rc = ss_counter_reserve(c, n)) != SS_OK) return rc;
    }
    if (multi && !words_in) {
        const uint64_t need = c->ws_reads * c->W;
        if (c->ws_words_cap < need) {
            if (c->ws_words) (void)hipFree(c->ws_words);
            c->ws_words = nullptr;
            c->ws_words_cap = 0;
            if (hipMalloc((void**)&c->ws_words, need * sizeof(uint64_t)) != hipSuccess) {
                ss_check(hipGetLastError(), "counter word workspace hipMalloc");
                return ss_fail(SS_ENOMEM, "counter word workspace: out of device memory");
            }
            c->ws_words_cap = need;
        }
        rc = ss_encode_fixed_impl(d_ascii, n, L, stride, c->ws_words, c->W, d_first_bad, nullptr, nullptr, stream);
        if (rc) return rc;
        mw = c->ws_words;
    }
    // single-word keys of any other length / layout: pack into the key workspace first, then the
    // same partitioned passes (k_pc_hist replaces the fused encode of k_pc_keys)
    const bool packed_keys = !multi && !fast && n <= c->ws_reads;
    if (packed_keys && keys_in && !opt) {
        rc = ss_check(hipMemcpyAsync(c->ws_keys, keys_in, n * 8, hipMemcpyDeviceToDevice, s), "counter key copy");
        if (rc) return rc;
    } else if (packed_keys && !keys_in) {
        rc = ss_encode_fixed_impl(d_ascii, n, L, stride, c->ws_keys, 1, d_first_bad, nullptr, nullptr, stream);
        if (rc) return rc;
    }
    const bool part = multi || packed_keys || (fast && n <= c->ws_reads);
    // a pending reset: the single-word aggregate writes whole slices (fresh); other paths memset first
    bool fresh = false;
    if (part && !multi) {
        fresh = c->reset_pending;
        c->reset_pending = false;
    } else if ((rc = flush_reset(c, s)) != SS_OK) {
        return rc;
    }
    if (part) {
        PartWs w;
        w.keys = c->ws_keys;
        w.akey = c->ws_akey;
        w.aidx = c->ws_aidx;
        w.acnt = c->ws_acnt;
        w.areg = c->ws_areg;
        w.bidx = c->ws_bidx;
        w.bcnt = c->ws_bcnt;
        w.spill = c->ws_spill;
        w.spill_cap = c->ws_reads;
        w.seg_end = nullptr;
        w.hist = c->ws_hist;
        w.rstart = c->ws_rstart;
        w.tot = c->ws_tot;
        w.bkey = nullptr;
        w.brec = nullptr;
        w.slab = 0;
        w.slabs = nullptr;
        w.spill_ctr = nullptr;
        w.R = (uint32_t)(c->cap >> c->slice_log);
        w.rbits = c->log2cap - c->slice_log;
        const uint32_t S = 1u << c->slice_log;
        const size_t mw_lds = (size_t)2 * S * 16 + (size_t)S * 8;
        const bool two_pass = w.rbits > kCoarseBits;             // > 64 regions: coarse pass first
        const uint32_t bins1 = two_pass ? (1u << kCoarseBits) : w.R;
        constexpr int T1 = 512, U1 = 2, TS = 512, TF = 512;
        // dynamic LDS above the 64 KB default: opt in once per kernel (host-side attribute; a
        // function-local static is initialised once even with engines on several threads)
        static const hipError_t attrs = [] {
            const int agg_max = (int)(2 * (1u << kMwSliceLog) * 16 + (1u << kMwSliceLog) * 8 + 8);
            hipError_t ea = hipFuncSetAttribute((const void*)k_pc_keys<T1, U1>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, kMaxRegions * 4);
            if (ea == hipSuccess)
                ea = hipFuncSetAttribute((const void*)k_pc_hist<TF>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         kMaxRegions * 4);
            for (int f = 0; f < kMwAggFns && ea == hipSuccess; ++f)
                ea = hipFuncSetAttribute((const void*)kMwFp[f], hipFuncAttributeMaxDynamicSharedMemorySize,
                                         kMaxRegions * 4);
            for (int f = 0; f < kMwAggFns && ea == hipSuccess; ++f)
                ea = hipFuncSetAttribute((const void*)kMwAgg[f], hipFuncAttributeMaxDynamicSharedMemorySize, agg_max);

            return ea;
        }();
        if (attrs != hipSuccess) return ss_check(attrs, "hipFuncSetAttribute (dynamic LDS)");
        auto scan = [&](uint32_t bins, uint32_t* start) {
            hipLaunchKernelGGL(k_pc_tot, dim3(bins), dim3(256), 0, s, w, bins);
            hipLaunchKernelGGL(k_pc_scan, dim3(1), dim3(1024), 0, s, w, bins, start);
            hipLaunchKernelGGL(k_pc_offsets, dim3(bins), dim3(1024), 0, s, w, bins, (const uint32_t*)start);
        };
        if (!multi && (!packed_keys || (keys_in && opt)) && two_pass && w.rbits - kCoarseBits <= 8) {
            // optimistic coarse partition: encode + coarse scatter in one pass, fine pass by bin
            const uint64_t cap1 = c->ws_cap1;
            w.slab = (uint32_t)c->ws_slab;
            w.spill_ctr = c->ws_fill + fill_at(kSpillCtr);
            hipEvent_t tev[ss_counter::kPassEvents] = {};
            for (uint32_t p = 0; p < ss_counter::kPassEvents; ++p) tev[p] = timer_event(c, p);
            auto mark = [&](uint32_t p) {
                if (tev[p]) (void)hipEventRecord(tev[p], s);
            };
            mark(0);
            PrepWords pw{};
            pw.p[0] = (unsigned long long*)d_first_bad;
            pw.v[0] = ~0ull;
            pw.zero = c->ws_fill;
            pw.nzero = kFillWords;
            rc = ss_check(launch_prep(pw, s), "first_bad / fill reset");
            if (rc) return rc;
            // grid-stride over tiles: exactly the resident blocks (no second, partial round)
            static const int pf_grid = [] {
                int dev = 0, cus = 0, per = 0;
                (void)hipGetDevice(&dev);
                (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
                (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k_pf_coarse<kPfT, kPfRPL, false, true>, kPfT, 0);
                return (cus > 0 && per > 0) ? cus * per : (int)kPartBlocks;
            }();
            if (keys_in)
                hipLaunchKernelGGL((k_pf_coarse<kPfT, kPfRPL, true, false>), dim3(pf_grid), dim3(kPfT), 0, s, t, w,
                                   (const uint4*)keys_in, (uint64_t)0, n, 0u, cap1, c->ws_fill,
                                   (unsigned long long*)nullptr);
            else if (L == 32)     // 32-nt rows: coalesced lane-pair loads (G16)
                hipLaunchKernelGGL((k_pf_coarse<kPfT, kPfRPL, false, true>), dim3(pf_grid), dim3(kPfT), 0, s, t, w,
                                   (const uint4*)d_ascii, stride / 16, n, 2u, cap1, c->ws_fill,
                                   (unsigned long long*)d_first_bad);
            else
                hipLaunchKernelGGL((k_pf_coarse<kPfT, kPfRPL, false, false>), dim3(pf_grid), dim3(kPfT), 0, s, t, w,
                                   (const uint4*)d_ascii, stride / 16, n, L / 16, cap1, c->ws_fill,
                                   (unsigned long long*)d_first_bad);
            const unsigned fine_blocks = kCB * kFinePerBin;
            if (!w.slab) {   // counted cursors: region histogram per sub-bin, then the scans
                hipLaunchKernelGGL((k_pf_count<512>), dim3(fine_blocks), dim3(512), 0, s, t, w, cap1,
                                   (const uint32_t*)c->ws_fill);
                const unsigned rg = (w.R + 255) / 256;
                hipLaunchKernelGGL(k_pf_tot, dim3(rg), dim3(256), 0, s, w);
                hipLaunchKernelGGL(k_pc_scan, dim3(1), dim3(1024), 0, s, w, w.R, w.rstart, (const uint32_t*)nullptr);
                hipLaunchKernelGGL(k_pf_offsets, dim3(rg), dim3(256), 0, s, w);
            }
            w.seg_end = c->ws_segend;
            w.slabs = w.slab ? c->ws_order + kNFill : nullptr;
            mark(1);
            hipLaunchKernelGGL(k_pf_order, dim3(1), dim3(512), 0, s, (const uint32_t*)c->ws_fill, cap1, c->ws_order,
                               1u << (w.rbits - kCoarseBits), w.slab ? c->ws_order + kNFill : nullptr);
            mark(2);
            hipLaunchKernelGGL((k_pf_scatter<kFsT, kFsTile>), dim3(fine_blocks), dim3(kFsT), 0, s, t, w, cap1,
                               (const uint32_t*)c->ws_fill, (const uint32_t*)c->ws_order);
            mark(3);
            w.bkey = w.keys;
            w.brec = (const Rec12*)w.keys;
            hipLaunchKernelGGL((k_pc_aggregate_slice<kAggSliceT, true>), dim3(w.R), dim3(kAggSliceT),
                               ((size_t)1 << c->slice_log) * 16, s, t, w, base_index, fresh);
            mark(4);
            // records that found their sub-bin full (none unless many distinct keys pile into a bin)
            hipLaunchKernelGGL(k_spill_insert, dim3(1024), dim3(256), 0, s, t, w, (const uint32_t*)c->ws_fill,
                               base_index);
            mark(5);
            if (c->tev) {
                c->thead = (c->thead + 1) % ss_counter::kTimerRing;
                ++c->tpend;
            }
            c->occ_src = 1;
            return ss_check(hipGetLastError(), "optimistic partitioned insert");
        }
        if (multi) {
            const size_t fp_lds = (bins1 * (TF / 64) <= kMaxRegions ? bins1 * (TF / 64) : bins1) * 4;
            static_assert(TF == kMwFpT, "k_mw_fp instances");
            hipLaunchKernelGGL(kMwFp[mw_variant(t.W, mw)], dim3(kPartBlocks), dim3(TF), fp_lds, s, t, w, bins1, mw, n);
        } else if (packed_keys) {
            const size_t h_lds = (bins1 * (TF / 64) <= kMaxRegions ? bins1 * (TF / 64) : bins1) * 4;
            hipLaunchKernelGGL((k_pc_hist<TF>), dim3(kPartBlocks), dim3(TF), h_lds, s, t, w, bins1, n);
        } else {
            const size_t keys_lds = (bins1 * (T1 / 64) <= kMaxRegions ? bins1 * (T1 / 64) : bins1) * 4;
            hipLaunchKernelGGL((k_pc_keys<T1, U1>), dim3(kPartBlocks), dim3(T1), keys_lds, s, t, w, bins1,
                               (const uint4*)d_ascii, stride / 16, n, L / 16, (unsigned long long*)d_first_bad);
        }
        if (two_pass) {
            scan(bins1, w.tot + 0);   // coarse starts are not needed later; tot is reused as scratch
            hipLaunchKernelGGL((k_pc_scatter_lds<true, false>), dim3(kPartBlocks), dim3(512), 0, s, t, w, bins1,
                               (const uint64_t*)w.keys, (const uint32_t*)nullptr, w.akey, w.aidx, n);
            hipLaunchKernelGGL((k_pc_count<TS>), dim3(kPartBlocks), dim3(TS), 0, s, t, w, (const uint64_t*)w.akey, n);
            scan(w.R, w.rstart);
            hipLaunchKernelGGL((k_pc_scatter_lds<false, true>), dim3(kPartBlocks), dim3(512), 0, s, t, w, w.R,
                               (const uint64_t*)w.akey, (const uint32_t*)w.aidx, w.keys, w.bidx, n);
            w.bkey = w.keys;
        } else {
            scan(w.R, w.rstart);   // <= 64 regions: one pass, bins = regions (bin_of<true> == region)
            hipLaunchKernelGGL((k_pc_scatter_lds<true, false>), dim3(kPartBlocks), dim3(512), 0, s, t, w, w.R,
                               (const uint64_t*)w.keys, (const uint32_t*)nullptr, w.akey, w.bidx, n);
            w.bkey = w.akey;
        }
        if (multi)
            hipLaunchKernelGGL(kMwAgg[mw_variant(t.W, mw)], dim3(w.R), dim3(kMwT), mw_lds, s, t, w, mw, base_index);
        else
            hipLaunchKernelGGL((k_pc_aggregate_slice<kAggSliceT, false>), dim3(w.R), dim3(kAggSliceT),
                               ((size_t)1 << c->slice_log) * 16, s, t, w, base_index, fresh);
        if (!multi) c->occ_src = 1;
        return ss_check(hipGetLastError(), "partitioned insert");
    }
    if (fast) {
        constexpr int U = 4;
        const unsigned grid = grid_for(2 * n, (uint64_t)U * kThreads, 0);
        hipLaunchKernelGGL((k_count_g16<U>), dim3(grid), dim3(kThreads), 0, s, t, (const uint4*)d_ascii,
                           stride / 16, n, L / 16, base_index, (unsigned long long*)d_first_bad);
        return ss_check(hipGetLastError(), "k_count_g16");
    }
    const unsigned grid = grid_for(n, kThreads, 256 * 16);
    hipLaunchKernelGGL(k_count_gen, dim3(grid), dim3(kThreads), 0, s, t, d_ascii, stride, n, L, base_index,
                       (unsigned long long*)d_first_bad);
    return ss_check(hipGetLastError(), "k_count_gen");
}

int ss_counter_insert_fixed(ss_counter* c, const uint8_t* d_ascii, uint64_t n, uint32_t L,
                            uint64_t stride, uint64_t base_index, uint64_t* d_first_bad, void* stream) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (c->L == kWordKeys) return ss_fail(SS_EARG, "the handle holds packed multi-word keys (ss_counter_insert_words)");
    return insert_impl(c, d_ascii, n, L, stride, base_index, d_first_bad, stream, nullptr);
}

int ss_counter_set_words(ss_counter* c, uint32_t W) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (W < 2 || W > 64) return ss_fail(SS_EARG, "packed keys of 2..64 words");
    if (c->L == kWordKeys && c->W == W) return SS_OK;
    if (c->L != -1) return ss_fail(SS_EARG, "the handle already holds keys of another kind");
    if (c->keywords_W != W) {
        if (c->keywords) (void)hipFree(c->keywords);
        c->keywords = nullptr;
        c->keywords_W = 0;
        if (hipMalloc((void**)&c->keywords, c->cap * W * sizeof(uint64_t)) != hipSuccess) {
            ss_check(hipGetLastError(), "counter key words hipMalloc");
            return ss_fail(SS_ENOMEM, "counter key words: out of device memory");
        }
        c->keywords_W = W;
    }
    c->W = W;
    c->L = kWordKeys;
    return SS_OK;
}

int ss_counter_insert_words(ss_counter* c, const uint64_t* d_words, uint64_t n, uint64_t base_index, void* stream) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (c->L != kWordKeys) return ss_fail(SS_EARG, "ss_counter_set_words first");
    if (n && !d_words) return ss_fail(SS_EARG, "null buffer");
    return insert_impl(c, nullptr, n, 0, 0, base_index, nullptr, stream, d_words);
}

int ss_counter_insert_keys(ss_counter* c, const uint64_t* d_keys, uint64_t n, uint64_t base_index, void* stream) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (n && !d_keys) return ss_fail(SS_EARG, "null buffer");
    if (c->L < 0) {
        const int rc = fix_length(c, 32);
        if (rc) return rc;
    }
    return insert_impl(c, nullptr, n, 0, 0, base_index, nullptr, stream, nullptr, d_keys);
}

int ss_counter_merge(ss_counter* c, const uint64_t* d_keys, const uint32_t* d_lens,
                     const uint64_t* d_counts, const uint64_t* d_first, uint64_t m, void* stream) {
    (void)d_lens;   // every entry of a handle has the handle's length (checked by the caller)
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (m == 0) return SS_OK;
    if (!d_keys || !d_counts || !d_first) return ss_fail(SS_EARG, "null buffer");
    if (c->W > 1) return ss_fail(SS_EARG, "ss_counter_merge takes single-word keys (L <= 32)");
    const unsigned grid = grid_for(m, kThreads, 256 * 16);
    c->occ_src = 0;
    int rc = flush_reset(c, (hipStream_t)stream);
    if (!rc) rc = wide_on(c, (hipStream_t)stream);    // u64 counts come in: carries go to wide
    if (rc) return rc;
    c->since = kSinceUnknown;
    hipLaunchKernelGGL(k_merge, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, tbl_of(c), d_keys, d_counts,
                       d_first, m);
    return ss_check(hipGetLastError(), "k_merge");
}

int ss_counter_merge_words(ss_counter* c, const uint64_t* d_words, const uint64_t* d_counts,
                           const uint64_t* d_first, uint64_t m, void* stream) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (m == 0) return SS_OK;
    if (!d_words || !d_counts || !d_first) return ss_fail(SS_EARG, "null buffer");
    if (c->W < 2) return ss_fail(SS_EARG, "ss_counter_merge_words takes multi-word keys (L > 32): use ss_counter_merge");
    hipStream_t s = (hipStream_t)stream;
    int rc = flush_reset(c, s);
    if (!rc && c->L != kWordKeys) rc = wide_on(c, s);   // (the engine's class tables: see insert_impl)
    if (rc) return rc;
    c->since = kSinceUnknown;
    uint64_t* found = nullptr;
    if ((rc = aux_scratch(c, m * sizeof(uint64_t), (void**)&found))) return rc;
    const unsigned grid = grid_for(m, 256, 256 * 16);
    const Tbl t = tbl_of(c);
    hipLaunchKernelGGL(k_mw_merge_find, dim3(grid), dim3(256), 0, s, t, d_words, m, found);
    hipLaunchKernelGGL(k_mw_merge_claim, dim3(grid), dim3(256), 0, s, t, d_words, d_counts, d_first, m,
                       (const uint64_t*)found);
    return ss_check(hipGetLastError(), "ss_counter_merge_words");
}

int ss_counter_set_length(ss_counter* c, uint32_t L) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    return fix_length(c, L);
}

int ss_counter_length(const ss_counter* c) { return c ? c->L : -1; }

int ss_counter_size(ss_counter* c, uint64_t* d_size, void* stream) {
    if (!c || !d_size) return ss_fail(SS_EARG, "null argument");
    hipStream_t s = (hipStream_t)stream;
    int rc = flush_reset(c, s);
    if (!rc) rc = ss_check(hipMemsetAsync(d_size, 0, sizeof(uint64_t), s), "size memset");
    if (rc) return rc;
    const unsigned grid = grid_for(c->cap + 1, kThreads, 256 * 8);
    hipLaunchKernelGGL(k_size, dim3(grid), dim3(kThreads), 0, s, tbl_of(c), (unsigned long long*)d_size);
    return ss_check(hipGetLastError(), "k_size");
}

int ss_counter_overflow(ss_counter* c, uint64_t* d_flag, void* stream) {
    if (!c || !d_flag) return ss_fail(SS_EARG, "null argument");
    return ss_check(hipMemcpyAsync(d_flag, c->work, sizeof(uint64_t), hipMemcpyDeviceToDevice, (hipStream_t)stream),
                    "overflow copy");
}

static int extract_impl(ss_counter* c, uint32_t n_parts, uint64_t* d_keys, uint32_t* d_lens, uint64_t* d_words,
                        uint64_t* d_counts, uint64_t* d_first, uint64_t cap, uint64_t* d_part_counts,
                        void* stream, bool ranges = false) {
    if (n_parts == 0 || n_parts > kMaxParts) return ss_fail(SS_EARG, "n_parts must be in 1..64");
    if (!d_keys || !d_lens || !d_counts || !d_first || !d_part_counts) return ss_fail(SS_EARG, "null buffer");
    hipStream_t s = (hipStream_t)stream;
    int rc = flush_reset(c, s);
    if (rc) return rc;
    Tbl t = tbl_of(c);
    unsigned long long* bc = c->work + 1;
    hipLaunchKernelGGL(k_part_count, dim3(kExtractBlocks), dim3(kExtractT), 0, s, t, n_parts, bc, ranges);
    hipLaunchKernelGGL(k_part_offsets, dim3(1), dim3(1024), 0, s, n_parts, bc, (unsigned long long*)d_part_counts);
    hipLaunchKernelGGL(k_part_scatter, dim3(kExtractBlocks), dim3(kExtractT), 0, s, t, n_parts, c->L < 0 ? 0 : c->L,
                       (const unsigned long long*)bc, d_keys, d_lens, d_counts, d_first, cap, c->work, d_words,
                       ranges);
    return ss_check(hipGetLastError(), "ss_counter_extract");
}

int ss_counter_extract(ss_counter* c, uint32_t n_parts, uint64_t* d_keys, uint32_t* d_lens,
                       uint64_t* d_counts, uint64_t* d_first, uint64_t cap, uint64_t* d_part_counts,
                       void* stream) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (c->W > 1) return ss_fail(SS_EARG, "multi-word keys (L > 32): use ss_counter_extract_words");
    return extract_impl(c, n_parts, d_keys, d_lens, nullptr, d_counts, d_first, cap, d_part_counts, stream);
}

int ss_counter_geometry(const ss_counter* c, uint32_t* h_log2cap, uint32_t* h_slice_log) {
    if (!c || !h_log2cap || !h_slice_log) return ss_fail(SS_EARG, "null argument");
    *h_log2cap = c->log2cap;
    *h_slice_log = c->slice_log;
    return SS_OK;
}

int ss_counter_extract_ranges(ss_counter* c, uint32_t n_parts, uint64_t* d_keys, uint32_t* d_lens,
                              uint64_t* d_counts, uint64_t* d_first, uint64_t cap, uint64_t* d_part_counts,
                              void* stream) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (c->W > 1) return ss_fail(SS_EARG, "region-range extraction takes single-word keys (L <= 32)");
    return extract_impl(c, n_parts, d_keys, d_lens, nullptr, d_counts, d_first, cap, d_part_counts, stream, true);
}

int ss_counter_merge_runs(ss_counter* c, const uint64_t* d_keys, const uint64_t* d_counts, const uint64_t* d_first,
                          const uint64_t* d_run_offsets, uint32_t n_runs, uint64_t m, uint32_t part,
                          uint32_t n_parts, uint32_t L, uint32_t* d_bounds, void* stream) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (c->W > 1 || L > 32) return ss_fail(SS_EARG, "merge_runs takes single-word keys (L <= 32)");
    if (n_parts == 0 || part >= n_parts || n_runs == 0 || n_runs > kMaxParts) return ss_fail(SS_EARG, "bad part / runs");
    int rc = fix_length(c, L);
    if (rc) return rc;
    const uint64_t R = c->cap >> c->slice_log;
    const uint32_t reg_lo = (uint32_t)((part * R + n_parts - 1) / n_parts);
    const uint32_t reg_hi = (uint32_t)(((part + 1) * R + n_parts - 1) / n_parts);
    const uint32_t nreg = reg_hi - reg_lo;
    if (m == 0) return SS_OK;
    if (!d_keys || !d_counts || !d_first || !d_run_offsets || !d_bounds) return ss_fail(SS_EARG, "null buffer");
    hipStream_t s = (hipStream_t)stream;
    c->occ_src = 0;
    return launch_merge(c, TripleRecs{d_keys, d_counts, d_first}, d_run_offsets, n_runs, m, reg_lo, nreg, d_bounds, s,
                        "ss_counter_merge_runs");
}

int ss_counter_pack_ranges(ss_counter* c, uint32_t n_parts, int32_t skip_part, uint64_t first_base, void* d_rec,
                           uint64_t cap, uint64_t* d_part_counts, void* stream) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (c->W > 1) return ss_fail(SS_EARG, "pack_ranges takes single-word keys (L <= 32)");
    if (n_parts == 0 || n_parts > kMaxParts) return ss_fail(SS_EARG, "n_parts must be in 1..64");
    if (skip_part < -1 || skip_part >= (int32_t)n_parts) return ss_fail(SS_EARG, "skip_part out of range");
    if (!d_rec || !d_part_counts) return ss_fail(SS_EARG, "null buffer");
    if ((((uintptr_t)d_rec) & 15) != 0) return ss_fail(SS_EARG, "d_rec must be 16-byte aligned");
    if (!c->occ) return ss_fail(SS_EARG, "table too large for region packing");
    hipStream_t s = (hipStream_t)stream;
    int rc = flush_reset(c, s);
    if (rc) return rc;
    Tbl t = tbl_of(c);
    const uint32_t R = (uint32_t)c->occ_R;
    if (c->occ_src != 1) hipLaunchKernelGGL(k_region_occ, dim3(R), dim3(kPackT), 0, s, t);
    hipLaunchKernelGGL(k_region_scan, dim3(1), dim3(1024), 0, s, t, R, n_parts, skip_part, c->roff,
                       (unsigned long long*)d_part_counts);
    hipLaunchKernelGGL(k_region_pack, dim3(R), dim3(kPackT), 0, s, t, R, n_parts, skip_part,
                       (const unsigned long long*)c->roff, first_base, (uint4*)d_rec, cap, c->work);
    return ss_check(hipGetLastError(), "ss_counter_pack_ranges");
}

int ss_counter_merge_packed(ss_counter* c, const void* d_rec, const uint64_t* d_run_offsets,
                            const uint64_t* d_run_first_base, uint32_t n_runs, uint64_t m, uint32_t part,
                            uint32_t n_parts, uint32_t L, uint32_t* d_bounds, void* stream) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (c->W > 1 || L > 32) return ss_fail(SS_EARG, "merge_packed takes single-word keys (L <= 32)");
    if (n_parts == 0 || part >= n_parts || n_runs == 0 || n_runs > kMaxParts) return ss_fail(SS_EARG, "bad part / runs");
    int rc = fix_length(c, L);
    if (rc) return rc;
    const uint64_t R = c->cap >> c->slice_log;
    const uint32_t reg_lo = (uint32_t)((part * R + n_parts - 1) / n_parts);
    const uint32_t reg_hi = (uint32_t)(((part + 1) * R + n_parts - 1) / n_parts);
    if (m == 0) return SS_OK;
    if (!d_rec || !d_run_offsets || !d_run_first_base || !d_bounds) return ss_fail(SS_EARG, "null buffer");
    if ((((uintptr_t)d_rec) & 15) != 0) return ss_fail(SS_EARG, "d_rec must be 16-byte aligned");
    c->occ_src = 0;
    return launch_merge(c, PackedRecs{(const uint4*)d_rec, d_run_first_base}, d_run_offsets, n_runs, m, reg_lo,
                        reg_hi - reg_lo, d_bounds, (hipStream_t)stream, "ss_counter_merge_packed");
}

int ss_counter_words(const ss_counter* c) { return c ? (int)c->W : 0; }

int ss_counter_extract_words(ss_counter* c, uint32_t n_parts, uint64_t* d_fps, uint32_t* d_lens,
                             uint64_t* d_words, uint64_t* d_counts, uint64_t* d_first, uint64_t cap,
                             uint64_t* d_part_counts, void* stream) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (!d_words) return ss_fail(SS_EARG, "null buffer");
    return extract_impl(c, n_parts, d_fps, d_lens, d_words, d_counts, d_first, cap, d_part_counts, stream);
}

}  // extern "C"

// Counts moved out of the slots (the drop-in engine's spill, before a slot's u32 count could wrap):
// acc[first] += count for every entry (first = the entry's row), the slot's count set to 0 -- the
// sentinel slot (key ~0, present iff its count is nonzero) keeps 1 and spills count - 1.
__global__ __launch_bounds__(256) void k_spill_counts(Tbl t, uint64_t* __restrict__ acc) {
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s <= t.mask + 1; s += (uint64_t)gridDim.x * 256) {
        const Slot sl = t.slots[s];
        const bool sent = s > t.mask;
        if (sent ? sl.ncount == 0xFFFFFFFFu : sl.key == kEmpty) continue;
        const uint32_t cnt = ~sl.ncount, keep = sent ? 1u : 0u;
        if (cnt <= keep || sl.first == kMaxIndex) continue;
        acc[sl.first] += cnt - keep;
        t.slots[s].ncount = ~keep;
    }
}

int ss_counter_spill_counts(ss_counter* c, uint64_t* d_acc, void* stream) {
    if (!c || !d_acc) return ss_fail(SS_EARG, "null argument");
    hipStream_t s = (hipStream_t)stream;
    int rc = flush_reset(c, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_spill_counts, dim3(grid_for(c->cap + 1, 256, 256 * 16)), dim3(256), 0, s, tbl_of(c), d_acc);
    c->since = 1;
    return ss_check(hipGetLastError(), "k_spill_counts");
}

int ss_counter_set_spill_limit(ss_counter* c, uint64_t reads) {
    if (!c) return ss_fail(SS_EARG, "null counter");
    if (reads < 1 || reads > 0xFFFFFFFFull) return ss_fail(SS_EARG, "spill limit in 1 .. 2^32 - 1");
    c->spill_at = reads;
    return SS_OK;
}

// the scratch of the read-order path: rep[(cap + 1) * 8], found[cap + 1], then the per-block class
// counts / first rows (fpt's aux buffer: it outlives the call, a deferred fold or extract reads it)
static int flat_scratch(ss_counter* fpt, unsigned grid, uint64_t** rep, uint64_t** found, uint32_t** blk) {
    const uint64_t fwords = fpt->cap + 1 + ((uint64_t)grid * kRepW1 + 1) / 2;
    int rc = aux_scratch(fpt, ((fpt->cap + 1) * 8 + fwords) * sizeof(uint64_t), (void**)rep);
    if (rc) return rc;
    *found = *rep + (fpt->cap + 1) * 8;
    *blk = (uint32_t*)(*found + fpt->cap + 1);
    return SS_OK;
}

static int flat_desc(const ss_flat_class* cls, uint32_t S, uint64_t base, hipStream_t s, FlatDesc& d, bool flush = true) {
    d = FlatDesc{};
    d.S = S;
    d.base = base;
    for (uint32_t W = 2; W + 1 <= S; ++W) {
        ss_counter* t = cls[W].table;
        if (!t) continue;
        if (t->L != kWordKeys || t->W != W + 1) return ss_fail(SS_EARG, "class table: set_words(W + 1) first");
        if (!flush) {
            d.tbl[W] = tbl_of(t);
            d.row0[W] = cls[W].base;
            d.rmap[W] = cls[W].rmap;
            continue;
        }
        int rc = flush_reset(t, s);
        if (rc) return rc;
        t->occ_src = 0;
        d.tbl[W] = tbl_of(t);
        d.row0[W] = cls[W].base;
        d.rmap[W] = cls[W].rmap;
    }
    return SS_OK;
}

int ss_classes_flat_verify(ss_counter* fpt, const uint64_t* d_rows, uint32_t S, uint64_t n, const uint64_t* d_fps,
                           uint32_t* d_flag, void* stream, void* ev_reps) {
    if (!fpt || !d_flag || !d_rows || !d_fps) return ss_fail(SS_EARG, "null argument");
    if (S < 3 || S > kRepW1) return ss_fail(SS_EARG, "read-order rows of 3 to 6 words");
    if (n == 0) return SS_OK;
    hipStream_t s = (hipStream_t)stream;
    int rc = flush_reset(fpt, s);
    if (rc) return rc;
    const Tbl f = tbl_of(fpt);
    const unsigned grid = grid_for(fpt->cap, 256, 256 * 16);
    uint64_t *rep = nullptr, *found = nullptr;
    uint32_t* blk = nullptr;
    if ((rc = flat_scratch(fpt, grid, &rep, &found, &blk))) return rc;
    hipLaunchKernelGGL(k_flat_reps, dim3(grid), dim3(256), 0, s, f, d_rows, S, rep);
    if (ev_reps && (rc = ss_check(hipEventRecord((hipEvent_t)ev_reps, s), "class reps event"))) return rc;
    // one short block per 64 kFlatQK rows (no persistent grid): a kernel queued on another stream
    // beside the verify (the speculative finish) gets CU slots as the verify's blocks retire
    hipLaunchKernelGGL(k_flat_verify, dim3(grid_for(n, 64 * kFlatQK, 0)), dim3(256), 0, s, f, d_rows, S, n, d_fps,
                       (const uint64_t*)rep, d_flag);
    return ss_check(hipGetLastError(), "class verify (read-order rows)");
}

int ss_classes_flat_fold(ss_counter* fpt, uint32_t S, const ss_flat_class* cls, uint64_t base, const uint32_t* d_flag,
                         void* stream) {
    if (!fpt || !cls || !d_flag) return ss_fail(SS_EARG, "null argument");
    hipStream_t s = (hipStream_t)stream;
    FlatDesc d;
    int rc = flat_desc(cls, S, base, s, d);
    if (rc) return rc;
    const Tbl f = tbl_of(fpt);
    const unsigned grid = grid_for(fpt->cap, 256, 256 * 16);
    uint64_t *rep = nullptr, *found = nullptr;
    uint32_t* blk = nullptr;
    if ((rc = flat_scratch(fpt, grid, &rep, &found, &blk))) return rc;
    hipLaunchKernelGGL(k_flat_fold_find<false>, dim3(grid), dim3(256), 0, s, f, d, (const uint64_t*)rep, d_flag, found, blk);
    hipLaunchKernelGGL(k_flat_fold_scan, dim3(1), dim3(256), 0, s, blk, grid, FlatTotals{});
    hipLaunchKernelGGL(k_flat_fold_claim, dim3(grid), dim3(256), 0, s, f, d, (const uint64_t*)rep, d_flag,
                       (const uint64_t*)found, (const uint32_t*)blk);
    return ss_check(hipGetLastError(), "class fold (read-order rows)");
}

int ss_classes_flat_extract(ss_counter* fpt, uint32_t S, const ss_flat_class* cls, uint64_t base,
                            const ss_flat_out* out, const uint32_t* d_zero, void* stream) {
    if (!fpt || !cls || !out || !d_zero) return ss_fail(SS_EARG, "null argument");
    hipStream_t s = (hipStream_t)stream;
    FlatDesc d;
    int rc = flat_desc(cls, S, base, s, d, false);
    if (rc) return rc;
    FlatOut o{};
    FlatTotals tot{};
    for (uint32_t W = 2; W + 1 <= S; ++W) {
        if (!cls[W].table) continue;
        if (!out[W].words || !out[W].counts || !out[W].first || !out[W].total || !out[W].ovf)
            return ss_fail(SS_EARG, "flat extract: outputs of every class");
        if (cls[W].base) return ss_fail(SS_EARG, "flat extract: the class tables must hold no earlier rows");
        o.words[W] = out[W].words;
        o.counts[W] = out[W].counts;
        o.first[W] = out[W].first;
        o.rmap[W] = cls[W].rmap;
        o.ovf[W] = (unsigned long long*)out[W].ovf;
        o.cap[W] = out[W].cap;
        tot.p[W] = out[W].total;
    }
    const Tbl f = tbl_of(fpt);
    const unsigned grid = grid_for(fpt->cap, 256, 256 * 16);
    uint64_t *rep = nullptr, *found = nullptr;
    uint32_t* blk = nullptr;
    if ((rc = flat_scratch(fpt, grid, &rep, &found, &blk))) return rc;
    hipLaunchKernelGGL(k_flat_fold_find<true>, dim3(grid), dim3(256), 0, s, f, d, (const uint64_t*)rep, d_zero, found, blk);
    hipLaunchKernelGGL(k_flat_fold_scan, dim3(1), dim3(256), 0, s, blk, grid, tot);
    hipLaunchKernelGGL(k_flat_extract_claim, dim3(grid), dim3(256), 0, s, f, d, o, (const uint64_t*)rep,
                       (const uint32_t*)blk);
    return ss_check(hipGetLastError(), "class extract (read-order rows)");
}

int ss_classes_flat_verify_fold(ss_counter* fpt, const uint64_t* d_rows, uint32_t S, uint64_t n, const uint64_t* d_fps,
                                const ss_flat_class* cls, uint64_t base, uint32_t* d_flag,
                                void* stream) {
    if (!cls) return ss_fail(SS_EARG, "null argument");
    int rc = ss_classes_flat_verify(fpt, d_rows, S, n, d_fps, d_flag, stream, nullptr);
    if (!rc && n) rc = ss_classes_flat_fold(fpt, S, cls, base, d_flag, stream);
    return rc;
}

int ss_classes_verify_fold(ss_counter* fpt, const uint64_t* d_fps, const ss_class_rows* cls, uint32_t ncls,
                           uint32_t* d_flag, void* stream) {
    if (!fpt || !cls || !d_flag) return ss_fail(SS_EARG, "null argument");
    if (ncls == 0) return SS_OK;
    if (ncls > kMaxClassesDesc) return ss_fail(SS_EARG, "at most 32 length classes per insert");
    hipStream_t s = (hipStream_t)stream;
    ClsDesc d{};
    d.ncls = ncls;
    uint64_t row = 0;
    int rc = SS_OK;
    for (uint32_t k = 0; k < ncls; ++k) {
        ss_counter* t = cls[k].table;
        if (!t || t->L != kWordKeys || t->W != cls[k].W1) return ss_fail(SS_EARG, "class table: set_words(W1) first");
        if ((rc = flush_reset(t, s))) return rc;
        t->occ_src = 0;
        d.tbl[k] = tbl_of(t);
        d.rows[k] = cls[k].rows;
        d.row0[k] = row;
        d.base[k] = cls[k].base;
        d.W1[k] = cls[k].W1;
        row += cls[k].m;
    }
    d.row0[ncls] = row;
    if ((rc = flush_reset(fpt, s))) return rc;
    const Tbl f = tbl_of(fpt);
    uint32_t w1max = 0;
    for (uint32_t k = 0; k < ncls; ++k) w1max = std::max(w1max, cls[k].W1);
    // the scratch: rep[(cap + 1) * 8] (rows of <= kRepW1 words), then found[cap + 1]
    uint64_t* rep = nullptr;
    if ((rc = aux_scratch(fpt, (fpt->cap + 1) * 9 * sizeof(uint64_t), (void**)&rep))) return rc;
    uint64_t* found = rep + (fpt->cap + 1) * 8;
    if (w1max <= kRepW1) {
        hipLaunchKernelGGL(k_cls_reps, dim3(grid_for(fpt->cap, 256, 256 * 16)), dim3(256), 0, s, f, d, rep);
        hipLaunchKernelGGL(k_cls_verify_rep, dim3(grid_for(row, 256, 256 * 32)), dim3(256), 0, s, f, d, d_fps,
                           (const uint64_t*)rep, d_flag);
    } else {
        hipLaunchKernelGGL(k_cls_verify, dim3(grid_for(row, 256, 256 * 32)), dim3(256), 0, s, f, d, d_fps, d_flag);
    }
    const unsigned grid = grid_for(fpt->cap, 256, 256 * 16);
    hipLaunchKernelGGL(k_cls_fold_find, dim3(grid), dim3(256), 0, s, f, d, (const uint32_t*)d_flag, found);
    hipLaunchKernelGGL(k_cls_fold_claim, dim3(grid), dim3(256), 0, s, f, d, (const uint32_t*)d_flag,
                       (const uint64_t*)found);
    return ss_check(hipGetLastError(), "class verify / fold");
}

