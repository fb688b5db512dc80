// C ABI of the WharfMH walk engine (include/wharf_gpu.h): handle management,
// the graph / batch pipelines (rocPRIM sorts, selects and scans on the
// handle's stream) and the host side of every entry point.
#include <algorithm>
#include <cmath>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <charconv>
#include <unistd.h>
#include <chrono>
#include <stdexcept>
#include <string>
#include <vector>

#include "wharf_gpu.h"
#include "wharf_kernels.h"

using namespace wharf;

namespace {

thread_local std::string g_last_error;
// A droppable device cache of the handle in the current call (the reverse-slot index): a failed
// device allocation frees it and tries once more (guarded() installs the handle's reclaimer)
thread_local bool (*g_reclaim_fn)(void*) = nullptr;
thread_local void* g_reclaim_ctx = nullptr;

struct WharfError : std::runtime_error {
    int code;
    WharfError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess)                                                                       \
            throw WharfError(e_ == hipErrorOutOfMemory ? WHARF_E_NOMEM : WHARF_E_HIP,               \
                             std::string(#x) + ": " + hipGetErrorString(e_) + " (line " +           \
                             std::to_string(__LINE__) + ")");                                       \
    } while (0)

#define REQUIRE(cond, code, msg)                        \
    do {                                                \
        if (!(cond)) throw WharfError((code), (msg));   \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    // slack: growing buffers (the CSR double buffers of the batch merge) get
    // 1/16 headroom, so a stream of insert batches does not free and re-map
    // multi-GB buffers at every batch (measured: seconds per batch at 2.4 G edges)
    void ensure(size_t bytes, bool slack = false)
    {
        if (bytes <= cap && p) return;
        release();
        size_t b = std::max<size_t>(bytes, 256);
        if (slack) b += b / 16;
        hipError_t e = hipMalloc(&p, b);
        if (e == hipErrorOutOfMemory && g_reclaim_fn && g_reclaim_fn(g_reclaim_ctx)) {
            (void)hipGetLastError();
            e = hipMalloc(&p, b);
        }
        HIPCHK(e);
        cap = b;
    }
    // per-batch buffers: 1/4 headroom, so batches of varying size do not free and
    // re-allocate them every time (a hipMalloc costs the update ~0.1 ms)
    void ensure_grow(size_t bytes)
    {
        if (bytes <= cap && p) return;
        ensure(bytes + bytes / 4);
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

uint32_t bits_for(uint64_t x)   // bits needed to represent values < x
{
    uint32_t b = 0;
    while (b < 64 && (x - 1) >> b) b++;
    return b;
}

}  // namespace

struct wharf_handle {
    int device = 0;
    hipStream_t s = nullptr;
    hipEvent_t ev[6] = {};
    wharf_config cfg{};
    uint64_t n = 0, m = 0, lo = 0, hi = 0, n_loc = 0, W = 0;
    uint32_t sh_part = 0, sh_parts = 1, sh_bits = 0;   // block shard (wharf_set_shard_blocks); contiguous: 0, 1, 0

    ShardMap smap() const { return ShardMap{n, n_loc, lo, sh_part, sh_parts, sh_bits}; }
    // the local column of walk wid, if this handle owns it
    bool owned_li(uint64_t wid, uint64_t& li) const
    {
        const uint64_t r = wid / n, v = wid % n;
        if (r >= wpv || v < lo || v >= hi) return false;
        const uint64_t off = v - lo, q = off >> sh_bits;
        if (q % sh_parts != sh_part) return false;
        li = r * n_loc + (((q / sh_parts) << sh_bits) | (off & ((1ull << sh_bits) - 1)));
        return true;
    }
    uint32_t L = 0, wpv = 0;
    bool anchors = false, has_walks = false;
    bool walks_poisoned = false;               // a failed re-walk left the walks half updated (until generate)
    void check_walks() const
    {
        REQUIRE(!walks_poisoned, WHARF_E_STATE,
                "the walks are incomplete after a failed update (WHARF_E_STATE); call wharf_generate");
    }
    bool anchors_cold = true;                  // node2vec MH: no generation has filled the anchor cache yet
    uint32_t epoch = 0;
    // slack-row CSR: row v = slots [off[v], off[v] + deg[v]) of the pool (adj, erec), cap[v] reserved
    DevBuf off, adj, deg, cap, vrec, erec, row_epoch, ehash;
    DevBuf off2, adj2, erec2;                  // temporaries: contiguous CSR at creation, repack, export
    uint64_t pool_used = 0, pool_cap = 0;      // slots handed out / allocated
    uint64_t repacks = 0, grown = 0;           // pool repacks so far; slots handed to rows moved by the last batch
    uint64_t dead_slots = 0;                   // old places of moved rows (kGap) until a repack / compaction
    uint64_t ehash_mask = 0, ehash_used = 0;   // capacity - 1; occupied slots incl. tombstones
    DevBuf fdir, fpool, fplan;                 // node2vec MH: per-row neighbour filters (k_filter_*)
    DevBuf memo, srcidx;                       // deterministic re-walk: suffix table, source index
    uint64_t fpool_used = 0;                   // words handed out (rows that outgrew theirs leave gaps)
    DevBuf walks, aff, rtab, bitmap, counters, errflag;
    DevBuf tmp, k1, k2, flags, chg, cf, runstart, runs, count, pairs, sel, defer, rplan, pscan, scratch;
    DevBuf preoff;                             // node2vec MH: per-source degree prefix of the anchor pre-init
    DevBuf stab;                               // node2vec MH re-walk: start-state anchor table (k_rewalk_sorted)
    DevBuf sanc;                               // anchor carry: the sources' old anchor entries (k_save_rows)
    DevBuf rchunk;                             // per batch source: chunk counts, then their exclusive prefix (k_*_rows_c)
    bool symmetric = false;                    // every edge's reverse is an edge (anchor carry and rev need it)
    DevBuf rev, srev;                          // reverse-slot index (k_patch_rev, u32 per slot) and the sources' old entries
    bool rev_on = false, rev_valid = false;    // the index is kept / matches the pool (a repack invalidates it)
    bool rev_tried = false;                    // the lazy build (first generation) was considered
    static constexpr uint64_t kRevMinPool = 1ull << 28;   // slots: below, the in-edge scan is as fast
    DevBuf park, parkc;                        // node2vec MH re-walk passes: two parked-walker lists, their counts
    DevBuf bdesc;                              // node2vec MH block re-walk: per 256-walk block, its run of the list
    uint32_t st_park_passes = 0;               // passes of the last re-walk by passes (0: lock-step kernel)
    uint64_t start_bound = 0;                  // distinct re-walk start states of the next walk update, at most (0: unknown)
    wharf_stats st{};
    std::string err;

    // Host snapshot of the walk matrix for walk() / vertex_at_walk(): the
    // reference's corpus export calls walk(i) once per walk
    // (vertex-classification.cpp:145-148), which at one kernel + D2H + sync per
    // call is ~10^4 round trips per 10^4 walks.  Chunks of kSnapWalks walks are
    // gathered walk-major on the device and copied to pinned host memory once
    // kSnapFillAfter different walks of the chunk were read since the last
    // change; sparser reads (the affected walks of a small batch,
    // vertex-classification.cpp:171-176) read their own row from the device
    // instead of pulling a whole chunk.  Every change to the walks
    // (walks_version) invalidates both, and releases all but kSnapKeep chunks.
    static constexpr uint64_t kSnapWalks = 1ull << 16;
    static constexpr uint32_t kSnapFillAfter = 32;   // distinct walks of a chunk read before the chunk is taken
    static constexpr size_t kSnapKeep = 4;           // pinned chunks kept across a change of the walks
    struct Snap {
        uint64_t chunk = ~0ull;
        uint32_t* host = nullptr;
    };
    uint64_t walks_version = 0, snap_version = ~0ull;
    std::vector<Snap> snaps;
    std::vector<int64_t> snap_of;     // chunk -> slot in snaps, or -1
    std::vector<uint32_t> snap_reads; // chunk -> walks read from it one by one since the last change
    size_t snap_next = 0, snap_cap = 0;
    std::vector<uint32_t> one_row;    // the last walk read on its own (vertex_at_walk(i, p) for p = 0, 1, ...)
    uint64_t one_li = ~0ull, one_version = ~0ull;
    // The affected walks of the last update (the reference's incremental readout calls walk(i) for
    // exactly those, vertex-classification.cpp:171-176): when the update handed its ids to the host
    // and there are at most kStageMax, the first walk() of one of them stages all their rows with one
    // list gather and one copy.
    static constexpr uint64_t kStageMax = 1ull << 20;
    static constexpr uint64_t kStagePiece = 1ull << 16;   // rows per device gather of the stage (21 MB at L = 80)
    std::vector<uint32_t> last_aff;   // ascending global ids of the last update's affected walks
    uint64_t last_aff_version = ~0ull, stage_version = ~0ull;
    std::vector<uint64_t> stage_li;   // their local indices (ascending), and their rows
    std::vector<uint32_t> stage_rows;

    void walks_changed() { walks_version++; }

    // pinned chunks at most: 1/8 of the host's available memory, 4..256 chunks
    // (20 MB each at L = 80; 8 ranks on one node each take their own)
    size_t snap_max_chunks()
    {
        if (!snap_cap) {
            const uint64_t bytes = kSnapWalks * L * 4;
            const uint64_t avail = (uint64_t)sysconf(_SC_AVPHYS_PAGES) * (uint64_t)sysconf(_SC_PAGESIZE);
            snap_cap = (size_t)std::min<uint64_t>(256, std::max<uint64_t>(4, avail / 8 / std::max<uint64_t>(bytes, 1)));
        }
        return snap_cap;
    }

    // walk-major row (L entries) of owned walk li: from the snapshot, or read on its own
    const uint32_t* snap_row(uint64_t li)
    {
        const uint64_t nchunks = (W + kSnapWalks - 1) / kSnapWalks, c = li / kSnapWalks;
        if (snap_version != walks_version || snap_of.size() != nchunks) {
            // the snapshot is stale: drop it, and hand back all but a few pinned chunks
            while (snaps.size() > kSnapKeep) {
                if (snaps.back().host) (void)hipHostFree(snaps.back().host);
                snaps.pop_back();
            }
            snap_next = 0;
            snap_of.assign(nchunks, -1);
            snap_reads.assign(nchunks, 0);
            for (Snap& x : snaps) x.chunk = ~0ull;
            snap_version = walks_version;
        }
        if (snap_of[c] >= 0) return snaps[snap_of[c]].host + (li - c * kSnapWalks) * L;
        if (one_version == walks_version && one_li == li) return one_row.data();
        if (const uint32_t* r = staged_row(li)) return r;
        const char* fa = getenv("WHARF_WALK_FILL_AFTER");   // A/B (tools/walk_readout): 0 = round 3's rule
        const uint32_t fill_after = fa && *fa ? (uint32_t)atoi(fa) : kSnapFillAfter;
        if (snap_reads[c] < fill_after) {   // sparse so far: this row alone
            snap_reads[c]++;
            one_row.resize(L);
            sel.ensure(L * 4);
            launch_gather_rows(walks.as<uint32_t>(), W, L, nullptr, li, 1, sel.as<uint32_t>(), s);
            HIPCHK(hipMemcpyAsync(one_row.data(), sel.p, L * 4, hipMemcpyDeviceToHost, s));
            sync();
            one_li = li;
            one_version = walks_version;
            return one_row.data();
        }
        size_t slot;
        if (snaps.size() < snap_max_chunks()) {
            uint32_t* p = nullptr;
            HIPCHK(hipHostMalloc((void**)&p, kSnapWalks * L * 4, hipHostMallocDefault));
            snaps.push_back(Snap{~0ull, p});   // only once the allocation succeeded
            slot = snaps.size() - 1;
        } else {
            slot = snap_next;
            snap_next = (snap_next + 1) % snaps.size();
            if (snaps[slot].chunk != ~0ull) snap_of[snaps[slot].chunk] = -1;
            snaps[slot].chunk = ~0ull;
        }
        const uint64_t base = c * kSnapWalks, cnt = std::min(kSnapWalks, W - base);
        sel.ensure(kSnapWalks * L * 4);
        launch_gather_rows(walks.as<uint32_t>(), W, L, nullptr, base, cnt, sel.as<uint32_t>(), s);
        HIPCHK(hipMemcpyAsync(snaps[slot].host, sel.p, cnt * L * 4, hipMemcpyDeviceToHost, s));
        sync();
        snaps[slot].chunk = c;
        snap_of[c] = (int64_t)slot;
        return snaps[slot].host + (li - base) * L;
    }
    // the row of li from the affected-walk stage of the last update, or null
    const uint32_t* staged_row(uint64_t li)
    {
        if (last_aff_version != walks_version || last_aff.empty()) return nullptr;
        const char* ns = getenv("WHARF_WALK_NO_STAGE");   // A/B (tools/walk_readout)
        if (ns && atoi(ns)) return nullptr;
        if (stage_version != walks_version) {
            // stage only when li is one of them (a reader of other walks never pays for it)
            const uint64_t wid = smap().wid(li);
            if (!std::binary_search(last_aff.begin(), last_aff.end(), (uint32_t)wid)) return nullptr;
            const uint64_t k = last_aff.size();
            stage_li.resize(k);
            for (uint64_t i = 0; i < k; i++)
                if (!owned_li(last_aff[i], stage_li[i])) throw WharfError(WHARF_E_STATE, "affected walk not owned");
            count.ensure(k * 8);
            HIPCHK(hipMemcpyAsync(count.p, stage_li.data(), k * 8, hipMemcpyHostToDevice, s));
            stage_rows.resize(k * L);
            // through a bounded device buffer (k * L * 4 bytes is up to 1 GB at L = 255,
            // kept pinned in the handle afterwards): pieces of at most kStagePiece rows
            const uint64_t piece = std::min<uint64_t>(k, kStagePiece);
            sel.ensure(piece * L * 4);
            for (uint64_t f = 0; f < k; f += piece) {
                const uint64_t c = std::min(piece, k - f);
                launch_gather_rows(walks.as<uint32_t>(), W, L, count.as<uint64_t>() + f, 0, c, sel.as<uint32_t>(), s);
                HIPCHK(hipMemcpyAsync(stage_rows.data() + f * L, sel.p, c * L * 4, hipMemcpyDeviceToHost, s));
                sync();
            }
            stage_version = walks_version;
        }
        const auto it = std::lower_bound(stage_li.begin(), stage_li.end(), li);
        if (it == stage_li.end() || *it != li) return nullptr;
        return stage_rows.data() + (uint64_t)(it - stage_li.begin()) * L;
    }
    void free_snaps()
    {
        for (Snap& x : snaps)
            if (x.host) (void)hipHostFree(x.host);
        snaps.clear();
        snap_of.clear();
        snap_reads.clear();
        snap_next = 0;
        one_li = ~0ull;
        last_aff.clear();
        stage_li.clear();
        stage_rows.clear();
        last_aff_version = stage_version = ~0ull;
    }

    void sync() { HIPCHK(hipStreamSynchronize(s)); }
    uint64_t bitmap_words() const { return (((n + 31) / 32 + 1) + 3) & ~3ull; }   // the filters after it stay 16-B aligned

    template <class F> void rp(F&& f)   // run a rocPRIM call with the shared temp buffer
    {
        size_t bytes = 0;
        HIPCHK(f((void*)nullptr, bytes));
        tmp.ensure(bytes);
        bytes = tmp.cap;
        HIPCHK(f(tmp.p, bytes));
    }

    void sort_u64(uint64_t* in, uint64_t* out, uint64_t cnt, uint32_t end_bit)
    {
        rp([&](void* t, size_t& b) { return rocprim::radix_sort_keys(t, b, in, out, cnt, 0u, end_bit, s); });
    }

    // sorted unique keys of `cnt` keys in k1 -> k1 (count returned), self loops dropped if asked
    uint64_t unique_keys(uint64_t cnt, bool drop_loops, uint32_t end_bit)
    {
        if (cnt == 0) return 0;
        sort_u64(k1.as<uint64_t>(), k2.as<uint64_t>(), cnt, end_bit);
        flags.ensure(cnt);
        launch_unique_flags(k2.as<uint64_t>(), cnt, drop_loops, flags.as<uint8_t>(), s);
        count.ensure(16);
        uint64_t* in = k2.as<uint64_t>();
        uint64_t* out = k1.as<uint64_t>();
        uint8_t* fl = flags.as<uint8_t>();
        uint64_t* c = count.as<uint64_t>();
        rp([&](void* t, size_t& b) { return rocprim::select(t, b, in, fl, out, c, (size_t)cnt, s); });
        uint64_t res = 0;
        HIPCHK(hipMemcpyAsync(&res, c, 8, hipMemcpyDeviceToHost, s));
        sync();
        return res;
    }

    // slots the pool holds for `used` handed-out slots: 1/16 headroom (rows that
    // outgrow their slack move to its end) plus `extra`; none with
    // WHARF_POOL_NO_HEADROOM=1 (tests: every moved row repacks the pool)
    // (WHARF_POOL_HEADROOM=<slots>, tests: exactly that headroom)
    static uint64_t pool_capacity(uint64_t used, uint64_t extra)
    {
        const char* nh = getenv("WHARF_POOL_NO_HEADROOM");
        const char* hs = getenv("WHARF_POOL_HEADROOM");
        uint64_t head = nh && atoi(nh) ? 0 : std::max<uint64_t>(used >> 4, 1ull << 16);
        if (hs && *hs && !(nh && atoi(nh))) head = strtoull(hs, nullptr, 10);
        return used + head + extra;
    }
    // WHARF_NO_ROW_SLACK=1 (tests): rows get no slack, so every growing row moves
    static int row_slack()
    {
        const char* ns = getenv("WHARF_NO_ROW_SLACK");
        return ns && atoi(ns) ? 0 : 1;
    }

    // CSR from the sorted unique keys in k1: contiguous in off2/adj2, then laid
    // out as slack rows
    void csr_from_keys(uint64_t mm)
    {
        off2.ensure((n + 1) * 8);
        adj2.ensure(std::max<uint64_t>(mm, 1) * 4);
        launch_offsets_from_keys(k1.as<uint64_t>(), mm, n, off2.as<uint64_t>(), s);
        launch_low32(k1.as<uint64_t>(), mm, adj2.as<uint32_t>(), s);
        m = mm;
        layout_rows();
        off2.release();
        adj2.release();
    }

    // contiguous CSR (off2, adj2) -> slack rows (off, deg, cap, adj); the
    // capacities are scanned as u64 in off itself
    void layout_rows()
    {
        deg.ensure(std::max<uint64_t>(n, 1) * 4);
        cap.ensure(std::max<uint64_t>(n, 1) * 4);
        off.ensure((n + 1) * 8);
        DevBuf capw;
        capw.ensure((n + 1) * 8);
        launch_row_degrees(off2.as<uint64_t>(), n, deg.as<uint32_t>(), cap.as<uint32_t>(), capw.as<uint64_t>(),
                           row_slack(), s);
        scan_u64(capw.as<uint64_t>(), off.as<uint64_t>(), n + 1);
        HIPCHK(hipMemcpyAsync(&pool_used, off.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, s));
        sync();
        capw.release();
        pool_cap = pool_capacity(pool_used, 0);
        adj.release();
        adj.ensure(std::max<uint64_t>(pool_cap, 1) * 4);
        HIPCHK(hipMemsetAsync(adj.p, 0xFF, std::max<uint64_t>(pool_cap, 1) * 4, s));   // kGap
        launch_copy_rows(off2.as<uint64_t>(), deg.as<uint32_t>(), adj2.as<uint32_t>(), off.as<uint64_t>(), n,
                         adj.as<uint32_t>(), nullptr, nullptr, s);
    }

    // Device bytes still available (WHARF_REPACK_MEM_CAP=<bytes>, tests: as if only that much were free)
    static uint64_t free_bytes()
    {
        size_t f = 0, t = 0;
        HIPCHK(hipMemGetInfo(&f, &t));
        const char* c = getenv("WHARF_REPACK_MEM_CAP");
        return c ? std::min<uint64_t>(f, strtoull(c, nullptr, 10)) : (uint64_t)f;
    }

    // Room for `extra` more slots in the pool: a repack into a second pool with
    // fresh slack when the device can hold both pools, else the in-place
    // compaction (no second pool: dead slots squeezed out, capacities kept).
    // Neither changes what the handle computes, only where rows live.
    void make_room(uint64_t extra)
    {
        const uint64_t pc = pool_capacity(pool_used, extra);
        const uint64_t need = pc * 4 + rec_bytes(rec_fmt_for(pc), pc, rec_stride()) + 3 * (n + 1) * 8 + (256ull << 20);
        if (need <= free_bytes()) {
            try {
                repack(extra);
                return;
            } catch (const WharfError& e) {   // the second pool did not fit after all (fragmentation, a short
                if (e.code != WHARF_E_NOMEM) throw;   // estimate): repack() left the handle as it was
                (void)hipGetLastError();
            }
        }
        compact();
    }

    // Fresh slack for every row, in a new pool with room for `extra` more slots
    // (the pool ran out of headroom): rows, their anchor entries and records
    // move; the records are rebuilt (every row offset changed).  Nothing of the
    // handle changes until the new pool is complete: a failed allocation leaves
    // it as it was.
    void repack(uint64_t extra)
    {
        const uint64_t rs = rec_stride();
        DevBuf capw, cap2;
        try {
            capw.ensure((n + 1) * 8);
            cap2.ensure(std::max<uint64_t>(n, 1) * 4);
            launch_row_recap(deg.as<uint32_t>(), n, cap2.as<uint32_t>(), capw.as<uint64_t>(), row_slack(), s);
            off2.ensure((n + 1) * 8);
            scan_u64(capw.as<uint64_t>(), off2.as<uint64_t>(), n + 1);
            uint64_t used = 0;
            HIPCHK(hipMemcpyAsync(&used, off2.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, s));
            sync();
            capw.release();
            const uint64_t pc = pool_capacity(used, extra);
            adj2.ensure(std::max<uint64_t>(pc, 1) * 4);
            HIPCHK(hipMemsetAsync(adj2.p, 0xFF, std::max<uint64_t>(pc, 1) * 4, s));
            erec2.ensure(rec_bytes(rec_fmt_for(pc), pc, rs));   // (the records are rebuilt below)
            launch_copy_rows(off.as<uint64_t>(), deg.as<uint32_t>(), adj.as<uint32_t>(), off2.as<uint64_t>(), n,
                             adj2.as<uint32_t>(), anchors ? erec.as<uint64_t>() + 2 : nullptr,
                             anchors ? erec2.as<uint64_t>() + 2 : nullptr, s);
            HIPCHK(hipGetLastError());
            sync();
            std::swap(off, off2);
            std::swap(adj, adj2);
            std::swap(erec, erec2);
            std::swap(cap, cap2);
            pool_used = used;
            pool_cap = pc;
            rf = rec_fmt_for(pc);
        } catch (...) {
            capw.release();
            cap2.release();
            off2.release();
            adj2.release();
            erec2.release();
            throw;
        }
        cap2.release();
        off2.release();
        adj2.release();
        erec2.release();
        dead_slots = 0;
        launch_vrec(off.as<uint64_t>(), deg.as<uint32_t>(), n, row_epoch.as<uint32_t>(), vrec.as<ERec>(), s);
        launch_erec(adj.as<uint32_t>(), pool_used, vrec.as<ERec>(), erec.as<ERec>(), (uint32_t)rs, 1, rf, s);
        repacks++;
        rev_valid = false;   // every row moved: the reverse-slot index is rebuilt after the batch
    }

    // In-place compaction (k_compact_gather / k_compact_put): rows in slot
    // order keep their capacities and close up the dead slots moved rows left,
    // window by window through a staging buffer of at most half the free
    // memory.  Needs O(n) scratch instead of a second pool.
    void compact()
    {
        const uint64_t rs = rec_stride();
        DevBuf keys, vals, keys2, order, capw, snoff, sadj, sanc;
        try {
            keys.ensure(std::max<uint64_t>(n, 1) * 8);
            keys2.ensure(std::max<uint64_t>(n, 1) * 8);
            vals.ensure(std::max<uint64_t>(n, 1) * 4);
            order.ensure(std::max<uint64_t>(n, 1) * 4);
            launch_slot_order_keys(off.as<uint64_t>(), cap.as<uint32_t>(), n, keys.as<uint64_t>(), vals.as<uint32_t>(), s);
            uint64_t* ki = keys.as<uint64_t>();
            uint64_t* ko = keys2.as<uint64_t>();
            uint32_t* vi = vals.as<uint32_t>();
            uint32_t* vo = order.as<uint32_t>();
            const unsigned eb = std::max<uint32_t>(bits_for(pool_cap + 1), 1);
            rp([&](void* t, size_t& b) { return rocprim::radix_sort_pairs(t, b, ki, ko, vi, vo, (size_t)n, 0u, eb, s); });
            keys.release();
            keys2.release();
            vals.release();
            capw.ensure((n + 1) * 8);
            snoff.ensure((n + 1) * 8);
            launch_ordered_caps(order.as<uint32_t>(), cap.as<uint32_t>(), n, capw.as<uint64_t>(), s);
            scan_u64(capw.as<uint64_t>(), snoff.as<uint64_t>(), n + 1);
            capw.release();
            std::vector<uint64_t> hsn(n + 1);
            HIPCHK(hipMemcpyAsync(hsn.data(), snoff.p, (n + 1) * 8, hipMemcpyDeviceToHost, s));
            sync();
            const uint64_t used = hsn[n];
            const uint64_t per = 4 + (anchors ? 8 : 0);
            const uint64_t C = std::max<uint64_t>(std::min<uint64_t>(free_bytes() / 2 / per, used), std::min<uint64_t>(used, 1ull << 20));
            sadj.ensure(std::max<uint64_t>(C, 1) * 4);
            if (anchors) sanc.ensure(std::max<uint64_t>(C, 1) * 8);
            uint64_t* anc = anchors ? erec.as<uint64_t>() + 2 : nullptr;
            for (uint64_t D = 0; D < used; D += C) {
                const uint64_t cnt = std::min(C, used - D);
                HIPCHK(hipMemsetAsync(sadj.p, 0xFF, cnt * 4, s));   // slack slots: kGap
                if (anchors) HIPCHK(hipMemsetAsync(sanc.p, 0xFF, cnt * 8, s));
                // rows in slot order whose new places meet [D, D + cnt)
                const uint64_t r0 = (uint64_t)(std::upper_bound(hsn.begin(), hsn.begin() + n, D) - hsn.begin());
                const uint64_t r1 = (uint64_t)(std::lower_bound(hsn.begin(), hsn.begin() + n, D + cnt) - hsn.begin());
                launch_compact_gather(order.as<uint32_t>(), snoff.as<uint64_t>(), r0 ? r0 - 1 : 0, r1,
                                      off.as<uint64_t>(), deg.as<uint32_t>(), adj.as<uint32_t>(), anc, D, cnt,
                                      sadj.as<uint32_t>(), anchors ? sanc.as<uint64_t>() : nullptr, s);
                launch_compact_put(sadj.as<uint32_t>(), anchors ? sanc.as<uint64_t>() : nullptr, cnt, D,
                                   adj.as<uint32_t>(), anc, s);
            }
            if (pool_used > used) HIPCHK(hipMemsetAsync(adj.as<uint32_t>() + used, 0xFF, (pool_used - used) * 4, s));
            launch_scatter_offsets(order.as<uint32_t>(), snoff.as<uint64_t>(), n, off.as<uint64_t>(), s);
            HIPCHK(hipGetLastError());
            sync();
            pool_used = used;
        } catch (...) {
            for (DevBuf* b : {&keys, &vals, &keys2, &order, &capw, &snoff, &sadj, &sanc}) b->release();
            throw;
        }
        for (DevBuf* b : {&order, &snoff, &sadj, &sanc}) b->release();
        dead_slots = 0;
        launch_vrec(off.as<uint64_t>(), deg.as<uint32_t>(), n, row_epoch.as<uint32_t>(), vrec.as<ERec>(), s);
        launch_erec(adj.as<uint32_t>(), pool_used, vrec.as<ERec>(), erec.as<ERec>(), (uint32_t)rs, 1, rf, s);
        repacks++;
        rev_valid = false;   // every row moved: the reverse-slot index is rebuilt after the batch
    }

    void scan_u64(uint64_t* in, uint64_t* out, uint64_t cnt)
    {
        rp([&](void* t, size_t& b) {
            return rocprim::exclusive_scan(t, b, in, out, (uint64_t)0, (size_t)cnt, rocprim::plus<uint64_t>(), s);
        });
    }

    void finish_graph()
    {
        row_epoch.ensure(std::max<uint64_t>(n, 1) * 4);
        HIPCHK(hipMemsetAsync(row_epoch.p, 0, std::max<uint64_t>(n, 1) * 4, s));
        build_records();
        if (anchors) build_edge_hash();
        if (anchors) build_filters();
        bitmap.ensure((bitmap_words() + kFilterWords) * 4);   // exact bitmap, then the Bloom filter
        sync();
        rev_on = symmetric && rev_wanted(true);
        if (rev_on) build_rev();
    }

    // The reverse-slot index (k_patch_rev) on undirected graphs, unless WHARF_REV=0.  By
    // default at creation when its 4 B per pool slot leave room for the walk matrix of every
    // walk the handle may own and a margin (configs[3]: 10 GB next to a 56-GB graph and 107 GB
    // of walks), else at the first generation, once the walk matrix is allocated (an 8-GPU
    // rank's shard: configs[4]'s 16 GB beside its 226-GB graph and 27-GB walk shard)
    bool rev_wanted(bool at_creation) const
    {
        const char* e = getenv("WHARF_REV");   // 0 off, 1 on, 2 (tests) built at the first generation
        if (e && *e) return atoi(e) == 2 ? !at_creation : atoi(e) != 0;
        // a small pool is scanned faster than its sources' in-edges are patched one by one
        // (configs[2], 96 M slots: scan 0.155 ms, index 0.23 ms; configs[3], 2.6 G: 2.35 vs 0.9 ms)
        if (pool_cap < kRevMinPool) return false;
        const uint64_t walks_rest = at_creation ? (uint64_t)W * L * 4 : 0, margin = 12ull << 30;
        return std::max<uint64_t>(pool_cap, 1) * 4 + walks_rest + margin <= free_bytes();
    }

    // (a device without room for it just keeps the scan: the index is an optimisation)
    void build_rev()
    {
        try {
            rev.ensure(std::max<uint64_t>(pool_cap, 1) * 4);
        } catch (const WharfError& e) {
            if (e.code != WHARF_E_NOMEM) throw;
            (void)hipGetLastError();
            drop_rev();
            return;
        }
        HIPCHK(hipMemsetAsync(rev.p, 0xFF, std::max<uint64_t>(pool_cap, 1) * 4, s));   // kNoRidx
        unsigned long long* miss = errflag.as<unsigned long long>() + 4;
        HIPCHK(hipMemsetAsync(miss, 0, 8, s));
        launch_rev_build(off.as<uint64_t>(), deg.as<uint32_t>(), adj.as<uint32_t>(), n, pool_used, rev.as<uint32_t>(),
                         miss, s);
        unsigned long long v = 0;
        HIPCHK(hipMemcpyAsync(&v, miss, 8, hipMemcpyDeviceToHost, s));
        sync();
        rev_valid = v == 0;
        if (!rev_valid) drop_rev();   // not symmetric after all: the scan keeps the records
    }

    void drop_rev()
    {
        rev_on = rev_valid = false;
        rev.release();
        srev.release();
    }

    // a device allocation failed: free the reverse-slot index (true) unless an update holds it
    bool rev_pinned = false;
    bool reclaim()
    {
        if (!rev_on || rev_pinned || !rev.p) return false;
        (void)hipStreamSynchronize(s);
        drop_rev();
        rev_tried = true;   // not rebuilt lazily: the room is wanted elsewhere
        return true;
    }

    // the walk matrix is allocated on first use (and re-allocated by set_shard)
    void ensure_walks()
    {
        if (walks.p) return;
        walks.ensure(std::max<uint64_t>(W * L, 1) * 4);
        launch_fill_u32(walks.as<uint32_t>(), W * L, kSent, s);
        walks_changed();
        aff.ensure(std::max<uint64_t>(W, 1));
        has_walks = false;
    }

    // 16-B edge records, 32 B with the anchor entry (node2vec MH)
    uint64_t rec_stride() const { return anchors ? 2 : 1; }

    // The edge-record layout for a pool of pc slots: compact 8-B records (wharf_device.h RecFmt)
    // for a handle without anchors whose vertex ids and slot offsets leave at least
    // kMinCompactDegBits for the degree, else the 16-B layout.  WHARF_COMPACT_REC=0 (A/B, tests)
    // keeps the 16-B layout.
    RecFmt rf{0u, 0u, 0u};
    RecFmt rec_fmt_for(uint64_t pc) const
    {
        const char* e = getenv("WHARF_COMPACT_REC");
        if (anchors || (e && *e && atoi(e) == 0)) return RecFmt{0u, 0u, 0u};
        const uint32_t vb = std::max<uint32_t>(bits_for(std::max<uint64_t>(n, 2)), 1);
        uint32_t ob = std::max<uint32_t>(bits_for(std::max<uint64_t>(pc, 2)), 1);
        const char* mdb = getenv("WHARF_COMPACT_MIN_DEG_BITS");   // A/B: allow a narrower degree field
        const uint32_t min_db = mdb && *mdb ? (uint32_t)std::max(atoi(mdb), 1) : kMinCompactDegBits;
        if (vb + ob + min_db > 64) return RecFmt{0u, 0u, 0u};
        const char* db = getenv("WHARF_COMPACT_DEG_BITS");   // tests: a narrow degree field, so rows of
        if (db && *db) {                                     // degree >= 2^db - 1 take the escape
            const uint32_t d = std::min<uint32_t>(std::max<int>(atoi(db), 1), 32);
            if (vb + ob + d <= 64) ob = 64 - vb - d;
        }
        return RecFmt{1u, vb, ob};
    }
    static uint64_t rec_bytes(RecFmt f, uint64_t slots, uint64_t rs)
    {
        return std::max<uint64_t>(slots, 1) * (f.compact ? 8 : sizeof(ERec) * rs);
    }

    // vertex rows and per-slot edge records (one gather per walk step);
    // anchor entries start empty
    void build_records()
    {
        vrec.ensure(std::max<uint64_t>(n, 1) * sizeof(ERec));
        erec.release();
        rf = rec_fmt_for(pool_cap);
        erec.ensure(rec_bytes(rf, pool_cap, rec_stride()));
        launch_vrec(off.as<uint64_t>(), deg.as<uint32_t>(), n, row_epoch.as<uint32_t>(), vrec.as<ERec>(), s);
        launch_erec(adj.as<uint32_t>(), pool_used, vrec.as<ERec>(), erec.as<ERec>(), (uint32_t)rec_stride(), 0, rf, s);
    }

    void build_edge_hash()
    {
        uint64_t cap = 64;
        while (cap < 2 * m) cap <<= 1;   // load factor <= 1/2
        ehash.ensure(cap * 8);
        ehash_mask = cap - 1;
        ehash_used = m;
        launch_fill_u64(ehash.as<uint64_t>(), cap, kEmptyKey, s);
        launch_edge_hash_build(off.as<uint64_t>(), deg.as<uint32_t>(), n, adj.as<uint32_t>(), ehash.as<uint64_t>(),
                               ehash_mask, s);
    }

    // neighbour filters of every row: sizes, directory (exclusive scan), fill;
    // the pool keeps 1/4 headroom for rows that outgrow their words in batches
    void build_filters()
    {
        const char* off_env = getenv("WHARF_NO_NEIGHBOUR_FILTER");
        if (off_env && atoi(off_env)) { fdir.release(); fpool.release(); return; }
        DevBuf words;
        words.ensure((n + 1) * 8);
        fdir.ensure((n + 1) * 8);
        launch_filter_sizes(deg.as<uint32_t>(), n, words.as<uint64_t>(), s);
        uint64_t* in = words.as<uint64_t>();
        uint64_t* out = fdir.as<uint64_t>();
        rp([&](void* t, size_t& b) {
            return rocprim::exclusive_scan(t, b, in, out, (uint64_t)0, (size_t)(n + 1), rocprim::plus<uint64_t>(), s);
        });
        uint64_t total = 0;
        HIPCHK(hipMemcpyAsync(&total, fdir.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, s));
        sync();
        words.release();
        // WHARF_FILTER_NO_SLACK (tests): no headroom, so every row that outgrows its words re-builds all
        const char* ns = getenv("WHARF_FILTER_NO_SLACK");
        const uint64_t want = std::max<uint64_t>(ns && atoi(ns) ? total : total + total / 4, 1) * 4;
        if (fpool.cap > want + want / 2) fpool.release();   // do not keep a much larger pool
        fpool.ensure(want);
        fpool_used = total;
        HIPCHK(hipMemsetAsync(fpool.p, 0, total * 4, s));
        launch_filter_pack(deg.as<uint32_t>(), n, fdir.as<uint64_t>(), s);
        launch_filter_fill(off.as<uint64_t>(), deg.as<uint32_t>(), n, adj.as<uint32_t>(), fdir.as<uint64_t>(),
                           fpool.as<uint32_t>(), s);
    }

    // after a batch: rebuild the filters of the k batch sources from their new rows
    void update_filters(const RunInfo* runs_d, uint64_t k)
    {
        if (!fpool.p || !k) return;
        fplan.ensure_grow((k + 1) * 16);
        uint64_t* need = fplan.as<uint64_t>();
        uint64_t* gofs = need + k + 1;
        launch_filter_plan(runs_d, k, deg.as<uint32_t>(), fdir.as<uint64_t>(), need, s);
        rp([&](void* t, size_t& b) {
            return rocprim::exclusive_scan(t, b, need, gofs, (uint64_t)0, (size_t)(k + 1), rocprim::plus<uint64_t>(), s);
        });
        uint64_t grow = 0;
        HIPCHK(hipMemcpyAsync(&grow, gofs + k, 8, hipMemcpyDeviceToHost, s));
        sync();
        if (fpool_used + grow > fpool.cap / 4) {
            build_filters();   // out of headroom: re-size and re-fill every row (drops the gaps)
            return;
        }
        launch_filter_rows(runs_d, k, rchunk.as<uint32_t>() + (k + 1), off.as<uint64_t>(), deg.as<uint32_t>(),
                           adj.as<uint32_t>(), need, gofs, fpool_used,
                           fdir.as<uint64_t>(), fpool.as<uint32_t>(), s);
        fpool_used += grow;
    }

    WalkArgs walk_args()
    {
        ensure_walks();
        WalkArgs a{};
        a.vrec = vrec.as<ERec>();
        a.erec = erec.as<ERec>();
        a.rf = rf;
        a.deg = deg.as<uint32_t>();
        a.adj = adj.as<uint32_t>();
        a.anchor = anchors ? erec.as<uint64_t>() + 2 : nullptr;   // inside the 32-B records
        a.ehash = anchors ? ehash.as<uint64_t>() : nullptr;
        a.ehash_mask = ehash_mask;
        a.fdir = anchors && fpool.p ? fdir.as<uint64_t>() : nullptr;
        a.fpool = anchors && fpool.p ? fpool.as<uint32_t>() : nullptr;
        a.walks = walks.as<uint32_t>();
        a.rtab = rtab.as<uint64_t>();
        a.bitmap = bitmap.as<uint32_t>();
        a.bloom = bitmap.as<uint32_t>() + bitmap_words();
        a.aff = aff.as<uint8_t>();
        a.counters = counters.as<unsigned long long>();
        a.n = n; a.n_loc = n_loc; a.lo = lo; a.W = W; a.wpv = wpv;
        a.sh_part = sh_part; a.sh_parts = sh_parts; a.sh_bits = sh_bits;
        a.L = L; a.epoch = epoch;
        a.key0 = (uint32_t)cfg.seed; a.key1 = (uint32_t)(cfg.seed >> 32);
        a.inv_p = 1.0f / cfg.paramP;   // node2vec.h:81 `1 / this->paramP` in float
        a.inv_q = 1.0f / cfg.paramQ;
        a.model = cfg.model; a.init = cfg.sampler_init; a.det = cfg.deterministic;
        const char* ns = getenv("WHARF_NO_SURE_SKIP");   // A/B: initialise every uncached anchor a step meets
        a.no_sure = ns && atoi(ns) ? 1 : 0;
        const char* ls = getenv("WHARF_N2V_LANE_SORT");   // A/B and tests: 0 = list order
        a.lane_sort = ls && *ls ? (atoi(ls) != 0) : 1;
        // return-first inits (A/B path, WHARF_RET_FIRST=1; off by default: configs[4] shard re-walk
        // 17.8-18.2 -> 17.1-17.3 ms at wpv 1 but 67-78 -> 73-82 ms at wpv 10, configs[2] +0.7 %,
        // profiles/r03/retfirst) need the return to be the one heaviest class (p < 1, p < q) and
        // proposals that need has_edge at all (q != 1)
        a.err = errflag.as<unsigned long long>() + 5;   // re-walk list consumers (list_entry_ok)
        a.stage = 0;
        const char* rf = getenv("WHARF_RET_FIRST");
        a.ret_first = cfg.model == WHARF_NODE2VEC && !cfg.deterministic && cfg.sampler_init == WHARF_INIT_WEIGHT &&
                      !a.no_sure && a.inv_q != 1.0f && a.inv_p > fmaxf(1.0f, a.inv_q) && rf && *rf && atoi(rf) != 0;
        return a;
    }

    float elapsed(int a, int b)
    {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ev[a], ev[b]));
        return ms;
    }

    void read_counters()
    {
        unsigned long long c[8] = {};
        HIPCHK(hipMemcpyAsync(c, counters.p, 64, hipMemcpyDeviceToHost, s));
        sync();
        st.steps = c[0];
        st.accepts = c[1];
        st.last_anchor_inits = c[7];
        st.last_rewalk_passes = st_park_passes;
#ifdef WHARF_INIT_STATS
        fprintf(stderr, "[init-stats] epoch %u: steps %llu inits %llu distinct %llu deferred %llu sweep-lane-slots %llu "
                        "list-lane-slots %llu\n", epoch, c[0], c[3], c[4], c[2], c[5], c[6]);
        HIPCHK(hipMemsetAsync(counters.as<unsigned long long>() + 3, 0, 32, s));
#endif
    }
};

namespace {

void set_err(wharf_handle* h, const std::string& m)
{
    g_last_error = m;
    if (h) h->err = m;
}

template <class F>
int guarded(wharf_handle* h, F&& f)
{
    // the reverse-slot index is a cache: an allocation that fails for want of room drops it (the
    // in-edge scan takes over) and is retried, unless an update is using it at that moment
    struct Reclaim {
        Reclaim(wharf_handle* h)
        {
            g_reclaim_ctx = h;
            g_reclaim_fn = h ? +[](void* p) { return static_cast<wharf_handle*>(p)->reclaim(); } : nullptr;
        }
        ~Reclaim() { g_reclaim_fn = nullptr; g_reclaim_ctx = nullptr; }
    } reclaim(h);
    try {
        if (h) HIPCHK(hipSetDevice(h->device));
        f();
        return WHARF_OK;
    } catch (const WharfError& e) {
        set_err(h, e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_err(h, e.what());
        return WHARF_E_INVALID;
    }
}

void check_config(const wharf_config* c)
{
    REQUIRE(c, WHARF_E_INVALID, "config is null");
    REQUIRE(c->walks_per_vertex >= 1 && c->walks_per_vertex <= 255, WHARF_E_INVALID, "walks_per_vertex must be 1..255");
    REQUIRE(c->walk_length >= 2 && c->walk_length <= 255, WHARF_E_INVALID, "walk_length must be 2..255 (types::Position is u8)");
    REQUIRE(c->model == WHARF_DEEPWALK || c->model == WHARF_NODE2VEC, WHARF_E_INVALID, "Unrecognized random walking model");
    REQUIRE(c->sampler_init >= WHARF_INIT_RANDOM && c->sampler_init <= WHARF_INIT_WEIGHT, WHARF_E_INVALID,
            "Unrecognized sampler init strategy");
    REQUIRE(c->model != WHARF_NODE2VEC || (c->paramP > 0 && c->paramQ > 0), WHARF_E_INVALID, "paramP/paramQ must be > 0");
}

wharf_handle* new_handle(const wharf_config* cfg, uint64_t n, int device)
{
    check_config(cfg);
    REQUIRE(n >= 1 && n < 0xFFFFFFFEull, WHARF_E_INVALID, "n must be in [1, 2^32-2)");
    REQUIRE(n * (uint64_t)cfg->walks_per_vertex < (1ull << 32), WHARF_E_INVALID,
            "n * walks_per_vertex must be < 2^32 (types::WalkID is u32)");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    REQUIRE(device >= 0 && device < ndev, WHARF_E_INVALID, "no such HIP device " + std::to_string(device));
    HIPCHK(hipSetDevice(device));
    auto* h = new wharf_handle();
    h->device = device;
    h->cfg = *cfg;
    h->n = n;
    h->L = cfg->walk_length;
    h->wpv = cfg->walks_per_vertex;
    h->lo = cfg->shard_lo;
    h->hi = cfg->shard_hi ? cfg->shard_hi : n;
    if (h->lo > h->hi || h->hi > n) {
        delete h;
        throw WharfError(WHARF_E_INVALID, "shard range must satisfy shard_lo <= shard_hi <= n");
    }
    h->n_loc = h->hi - h->lo;
    h->W = h->n_loc * h->wpv;
    h->anchors = cfg->model == WHARF_NODE2VEC && !cfg->deterministic;
    HIPCHK(hipStreamCreateWithFlags(&h->s, hipStreamNonBlocking));
    for (auto& e : h->ev) HIPCHK(hipEventCreate(&e));
    // deterministic draw table: Random(r).lrand() for r < wpv (utility.h:157-206)
    std::vector<uint64_t> t((size_t)h->wpv * h->L);
    for (uint32_t r = 0; r < h->wpv; r++) {
        XoroHost x(r);
        for (uint32_t j = 0; j < h->L; j++) t[(size_t)r * h->L + j] = x.lrand();
    }
    h->rtab.ensure(t.size() * 8);
    HIPCHK(hipMemcpy(h->rtab.p, t.data(), t.size() * 8, hipMemcpyHostToDevice));
    h->counters.ensure(64);
    h->errflag.ensure(64);
    return h;
}

void free_handle(wharf_handle* h)
{
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->s) (void)hipStreamSynchronize(h->s);
    for (DevBuf* b : {&h->off, &h->adj, &h->deg, &h->cap, &h->vrec, &h->erec, &h->erec2, &h->ehash, &h->fdir, &h->fpool,
                      &h->fplan, &h->memo, &h->srcidx, &h->row_epoch, &h->off2, &h->adj2, &h->walks, &h->aff, &h->rtab,
                      &h->bitmap, &h->counters, &h->errflag, &h->tmp, &h->k1, &h->k2, &h->flags, &h->chg, &h->cf,
                      &h->runstart, &h->runs, &h->count, &h->pairs, &h->sel, &h->defer, &h->rplan, &h->pscan,
                      &h->scratch, &h->stab, &h->preoff, &h->park, &h->parkc, &h->bdesc, &h->sanc, &h->rchunk,
                      &h->rev, &h->srev})
        b->release();
    h->free_snaps();
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    if (h->s) (void)hipStreamDestroy(h->s);
    delete h;
}

// keys in h->k1 (cnt of them) -> canonical CSR
void build_graph_from_keys(wharf_handle* h, uint64_t cnt, bool drop_loops, bool symmetric_by_construction)
{
    const uint64_t mm = h->unique_keys(cnt, drop_loops, 32 + std::max<uint32_t>(bits_for(h->n), 1));
    h->symmetric = symmetric_by_construction;
    h->csr_from_keys(mm);   // (reads the keys, which stay for the symmetry check)
    // the same rule as rev_wanted(): the slack-row pool's capacity, not the edge count
    const char* rv = getenv("WHARF_REV");
    const bool rev_may = rv && *rv ? atoi(rv) != 0 : h->pool_cap >= wharf_handle::kRevMinPool;
    if (!symmetric_by_construction && (h->anchors || rev_may)) {   // (the anchor carry and the reverse index ask)
        unsigned long long* asym = h->errflag.as<unsigned long long>() + 3;
        HIPCHK(hipMemsetAsync(asym, 0, 8, h->s));
        launch_keys_symmetric(h->k1.as<uint64_t>(), mm, asym, h->s);
        unsigned long long v = 1;
        HIPCHK(hipMemcpyAsync(&v, asym, 8, hipMemcpyDeviceToHost, h->s));
        h->sync();
        h->symmetric = v == 0;
    }
    // the keys and sort temporaries are done with: free them before the records
    // (configs[4]: 2 x 29 GB of keys next to 131 GB of 32-B records)
    for (DevBuf* b : {&h->k1, &h->k2, &h->tmp, &h->flags}) b->release();
    h->finish_graph();
}

void rmat_keys(wharf_handle* h, uint64_t edges_number, uint64_t vertices_number, uint64_t seed, int directed,
               double a, double b, double c)
{
    REQUIRE(vertices_number >= 2, WHARF_E_INVALID, "vertices_number must be >= 2");
    REQUIRE(a + b + c <= 1.0, WHARF_E_INVALID, "in rMat: a + b + c add to more than 1");
    REQUIRE(edges_number < (1ull << 32), WHARF_E_INVALID, "edges_number must be < 2^32 (rMat<unsigned int>)");
    const uint32_t lg = bits_for(vertices_number);   // pbbs::log2_up
    RmatParams p;
    p.n = (uint32_t)(1ull << (lg - 1));              // utility.h:78
    p.a = a; p.ab = a + b; p.abc = a + b + c;
    p.h = hash32((uint32_t)hash64(0 + seed));        // pbbs::random(seed).ith_rand(0), rmat_util.h:244
    const uint64_t total = directed ? edges_number : 2 * edges_number;
    h->k1.ensure(std::max<uint64_t>(total, 1) * 8);
    h->k2.ensure(std::max<uint64_t>(total, 1) * 8);
    launch_rmat_keys(p, edges_number, directed, h->k1.as<uint64_t>(), h->s);
}

// node2vec MH re-walk by passes (k_rewalk_park): the walkers of
// k_rewalk_plan's list advance until they need an anchor that is not cached,
// the parked states' anchors are computed with full waves, and the next pass
// resumes them; a short list is finished with in-wave inits.  One sync per pass
// reads the parked count.
constexpr uint64_t kParkTail = 8192;   // parked walkers below which the last pass initialises in the wave

void park_passes(wharf_handle* h, const WalkArgs& a)
{
    hipStream_t s = h->s;
    uint64_t c2 = 0;
    HIPCHK(hipMemcpyAsync(&c2, a.counters + 2, 8, hipMemcpyDeviceToHost, s));
    h->sync();
    const uint64_t listn = c2 & kListMask;
    h->st_park_passes = 0;
    if (!listn) return;
    h->park.ensure(2 * listn * kParkRecBytes);
    h->parkc.ensure(16);
    unsigned long long* pc = h->parkc.as<unsigned long long>();
    char* P[2] = {h->park.as<char>(), h->park.as<char>() + listn * kParkRecBytes};
    HIPCHK(hipMemsetAsync(pc, 0, 16, s));
    launch_rewalk_park(a, 1, 1, nullptr, nullptr, P[0], pc, s);
    const char* te = getenv("WHARF_PARK_TAIL");   // tests: 0 = park until no walker is left
    const uint64_t tail = te ? strtoull(te, nullptr, 10) : kParkTail;
    uint32_t passes = 1;
    for (int cur = 0;; cur ^= 1) {
        uint64_t cnt = 0;
        HIPCHK(hipMemcpyAsync(&cnt, pc + cur, 8, hipMemcpyDeviceToHost, s));
        h->sync();
        if (!cnt) break;
        launch_park_init(a, P[cur], pc + cur, s);
        const bool last = cnt < tail;
        HIPCHK(hipMemsetAsync(pc + (cur ^ 1), 0, 8, s));
        launch_rewalk_park(a, 0, last ? 0 : 1, P[cur], pc + cur, P[cur ^ 1], pc + (cur ^ 1), s);
        passes++;
        if (last) break;
    }
    h->st_park_passes = passes;
}

// Rewalk points + suffix re-walk (wharfmh.h:519-537, batch_walk_update
// 733-923) of every owned walk that holds a vertex of the bitmap; h->runs
// holds the k sources (the deterministic suffix table is keyed by them), and
// ev[1] marks the start of the walk update.
void walk_update(wharf_handle* h, uint64_t k, uint32_t flags, uint32_t* affected_out, uint64_t* n_affected)
{
    hipStream_t s = h->s;
    if (h->has_walks && h->W) {
        HIPCHK(hipMemsetAsync(h->counters.p, 0, 24, s));
        HIPCHK(hipMemsetAsync(h->counters.as<unsigned long long>() + 7, 0, 8, s));
        h->st_park_passes = 0;
        // tests: WHARF_BLOOM_SATURATE=1 sets every bit of the walk kernels' source
        // filters, so every position is a positive and the exact checks decide
        const char* sat = getenv("WHARF_BLOOM_SATURATE");
        if (sat && atoi(sat)) HIPCHK(hipMemsetAsync(h->bitmap.as<uint32_t>() + h->bitmap_words(), 0xFF, kFilterWords * 4, s));
        WalkArgs a = h->walk_args();
        a.scan_only = (flags & WHARF_APPLY_WALK_UPDATES) ? 0 : 1;
        // chunked scans: non-temporal row loads when most walks are expected to re-walk.  The
        // share grows with k * L / n (RMAT batches: configs[2] 0.19 -> 81 % re-walk, NT loads
        // win; configs[3] 1/8 shard 0.024 -> 32 %, they lose 35 %); WHARF_NT_ROWS=0/1 forces it
        const char* ntr = getenv("WHARF_NT_ROWS");
        a.nt_rows = ntr ? (atoi(ntr) != 0) : ((double)k * h->L >= 0.08 * (double)std::max<uint64_t>(h->n, 1));
        // deterministic mode: suffixes walked once per (round, batch source) and copied
        // (k_det_suffix + k_rewalk_chunked<true>) while the table stays small; WHARF_NO_MEMO=1 (tests)
        // re-walks every suffix (k_rewalk_sweep)
        const uint64_t stride4 = (h->L + 3) & ~3ull;
        const char* no_memo = getenv("WHARF_NO_MEMO");
        if (a.det && !a.scan_only && k && !(no_memo && atoi(no_memo)) &&
            (uint64_t)h->wpv * k * stride4 * 4 <= (256ull << 20)) {
            h->srcidx.ensure(std::max<uint64_t>(h->n, 1) * 4);
            // kMemoPad words before and after the table: k_rewalk_chunked reads whole
            // chunks around a row (values outside the row are never written)
            h->memo.ensure(((uint64_t)h->wpv * k * stride4 + 2 * kMemoPad) * 4);
            // every non-source kNoSource: the copy settles a Bloom positive by its index alone
            // (WHARF_COPY_BITMAP=1, A/B: by the bitmap word, then the index)
            const char* cbm = getenv("WHARF_COPY_BITMAP");
            a.src_exact = !(cbm && atoi(cbm));
            if (a.src_exact) HIPCHK(hipMemsetAsync(h->srcidx.p, 0xFF, std::max<uint64_t>(h->n, 1) * 4, s));
            launch_src_index(h->runs.as<RunInfo>(), k, h->srcidx.as<uint32_t>(), s);
            a.memo = h->memo.as<uint32_t>() + kMemoPad;
            a.src_idx = h->srcidx.as<uint32_t>();
            a.runs = h->runs.as<RunInfo>();
            a.memo_k = k;
            a.memo_stride = (uint32_t)stride4;
        }
        if (a.model == kNode2Vec && !a.det) {   // k_rewalk_plan's compacted, sorted re-walk list
            h->defer.ensure(h->W * 8);
            a.defer = h->defer.as<uint64_t>();
            const char* rwm = getenv("WHARF_N2V_REWALK");   // =block: k_rewalk_block (row-staged stores)
            if (rwm && std::string(rwm) == "block" && !a.scan_only) {
                h->bdesc.ensure(((h->W + 255) / 256) * 8);
                a.bdesc = h->bdesc.as<uint64_t>();
            }
            const char* pg = getenv("WHARF_N2V_PLAN_GROUP");   // A/B: 1024-walk groups in the plan's list
            a.plan_group = !a.bdesc && pg && *pg && atoi(pg) != 0;
            const char* no_stab = getenv("WHARF_NO_START_TABLE");   // A/B and tests: binary search at every start
            if (!a.scan_only && k && !(no_stab && atoi(no_stab))) {
                // start states (x, prev): x a batch source, prev an in-neighbour of it, so at most
                // the sources' degrees (undirected) and the re-walking walks; twice that many
                // entries, four per 64-B bucket (a full neighbourhood falls back to the search)
                const uint64_t bound = std::min<uint64_t>(h->start_bound ? h->start_bound : h->W, h->W);
                uint64_t buckets = 64;
                while (buckets * 4 < 2 * bound && buckets < (1ull << 22)) buckets <<= 1;
                const char* tb = getenv("WHARF_START_TABLE_BUCKETS");   // tests: a tiny table (overflow fallback)
                if (tb && atoi(tb) > 0)
                    for (buckets = 1; buckets < (uint64_t)atoi(tb);) buckets <<= 1;
                h->stab.ensure(buckets * 64);
                HIPCHK(hipMemsetAsync(h->stab.p, 0xFF, buckets * 64, s));   // keys kStabEmpty, entries kAnchorNone64
                a.stab = h->stab.as<uint64_t>();
                a.stab_mask = buckets - 1;
            }
        }
        h->start_bound = 0;
        HIPCHK(hipEventRecord(h->ev[2], s));
        // Pre-init pays when this handle's walks enter nearly every state around the sources (the
        // same test as the cold-cache pass: >= 4 steps per slot; configs[2]: 39).  Its cost does not
        // shrink with the walk shard, so with few walks per slot (configs[4] 1/8 shard, wpv 1: 0.19)
        // the lazy inits are cheaper.  WHARF_NO_PREINIT=1 / 0 forces it off / on (A/B and tests).
        const char* no_pre = getenv("WHARF_NO_PREINIT");
        const bool dense = (uint64_t)h->W * (h->L - 1) >= 4 * h->pool_used;
        const bool preinit = no_pre && *no_pre ? atoi(no_pre) == 0 : dense;
        if (a.model == kNode2Vec && !a.det && a.anchor && !a.scan_only && k && preinit) {
            // the batch's invalidated anchors, computed ahead of the re-walk (k_anchor_preinit)
            h->preoff.ensure_grow((k + 1) * 16);
            uint64_t* degs = h->preoff.as<uint64_t>();
            uint64_t* preoff = degs + (k + 1);
            launch_source_degrees(h->runs.as<RunInfo>(), k, h->vrec.as<ERec>(), degs, s);
            h->scan_u64(degs, preoff, k + 1);
            WalkArgs pa = a;
            pa.runs = h->runs.as<RunInfo>();
            launch_anchor_preinit(pa, preoff, k, s);
        }
        // node2vec MH re-walk: the lock-step sorted kernel (k_rewalk_sorted); WHARF_N2V_REWALK=park
        // runs it by passes with batched anchor inits (k_rewalk_park: 2-3x slower on configs[4]'s
        // shard, whose re-walk is bound by the init loads themselves, profiles/r03/park_ab),
        // =flat lanes at their own pace
        const char* rw = getenv("WHARF_N2V_REWALK");
        a.park = a.model == kNode2Vec && !a.det && a.anchor && !a.scan_only && rw && std::string(rw) == "park";
        h->walks_changed();
        HIPCHK(hipMemsetAsync(a.err, 0, 8, s));
        // node2vec list order (tests): WHARF_N2V_LIST_ORDER=global sorts k_rewalk_plan's list by
        // rewalk point over all blocks (round 3's global sort, rebuilt on a full-width sort, below)
        // before the consumer;
        // WHARF_TEST_CORRUPT_LIST=1 plants one out-of-range entry, which the consumer must report
        // (WHARF_E_STATE) without touching memory through it
        const char* lord = getenv("WHARF_N2V_LIST_ORDER");
        const char* lbad = getenv("WHARF_TEST_CORRUPT_LIST");
        const bool n2v_list = a.model == kNode2Vec && !a.det && !a.scan_only && !a.bdesc;
        const bool gsort = n2v_list && !a.park && lord && std::string(lord) == "global";
        const bool corrupt = n2v_list && lbad && atoi(lbad) != 0;
        if (gsort || corrupt) {
            a.stage = 1;
            launch_walk(a, true, s);
            uint64_t c2 = 0;
            HIPCHK(hipMemcpyAsync(&c2, a.counters + 2, 8, hipMemcpyDeviceToHost, s));
            h->sync();
            const uint64_t cnt = c2 & kListMask;   // tickets << 40 | entries
            REQUIRE(cnt <= h->W, WHARF_E_STATE, "re-walk list longer than the walks");
            if (gsort && cnt > 1) {
                h->park.ensure(cnt * 8);
                uint64_t* in = h->defer.as<uint64_t>();
                uint64_t* out = h->park.as<uint64_t>();
                // all 64 bits: by point, then walk.  NOT bits [56, 64) alone: rocPRIM's radix_sort_keys
                // with begin_bit 56 returns a non-permutation for 3 k <= n <= 1 Mi keys in ROCm 7.2
                // (tools/sort_probe, profiles/r04/sort_probe) — round 3's global sort fed those
                // entries to k_rewalk_sorted, which dereferenced them
                h->rp([&](void* t, size_t& b) { return rocprim::radix_sort_keys(t, b, in, out, (size_t)cnt, 0u, 64u, s); });
                HIPCHK(hipMemcpyAsync(in, out, cnt * 8, hipMemcpyDeviceToDevice, s));
            }
            if (corrupt && cnt) {
                const uint64_t bad = (h->W + 12345) | (1ull << 56);
                HIPCHK(hipMemcpyAsync(h->defer.as<uint64_t>() + cnt / 2, &bad, 8, hipMemcpyHostToDevice, s));
                h->sync();
            }
            a.stage = 2;
        }
        launch_walk(a, true, s);
        HIPCHK(hipGetLastError());
        if (a.park) park_passes(h, a);
        HIPCHK(hipEventRecord(h->ev[3], s));
        // ascending affected walk ids: count per block, scan, write
        const unsigned nb = aff_blocks(h->W);
        h->sel.ensure((uint64_t)(nb + 1) * 8);
        uint32_t* bcount = h->sel.as<uint32_t>();
        uint32_t* boff = bcount + nb + 1;
        HIPCHK(hipMemsetAsync(bcount + nb, 0, 4, s));
        launch_aff_count(h->aff.as<uint8_t>(), h->W, bcount, s);
        h->rp([&](void* t, size_t& b) {
            return rocprim::exclusive_scan(t, b, bcount, boff, 0u, (size_t)nb + 1, rocprim::plus<uint32_t>(), s);
        });
        const bool on_device = affected_out && (flags & WHARF_AFFECTED_DEVICE);
        if (!on_device) h->pairs.ensure(h->W * 4);
        launch_aff_write(h->aff.as<uint8_t>(), h->W, boff, h->smap(),
                         on_device ? affected_out : h->pairs.as<uint32_t>(), s);
        uint32_t naff32 = 0;
        unsigned long long lerr = 0;
        HIPCHK(hipMemcpyAsync(&naff32, boff + nb, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&lerr, a.err, 8, hipMemcpyDeviceToHost, s));
        h->sync();
        // a skipped entry leaves the update's walks half re-walked: the walks are marked invalid, so
        // later reads and updates fail loudly until they are generated again
        if (lerr) h->walks_poisoned = true;
        REQUIRE(lerr == 0, WHARF_E_STATE,
                std::string("node2vec re-walk list: ") + ((lerr & 1) ? "an entry outside the walks" : "an entry outside its block") +
                    " was skipped; the walks of this update are incomplete");
        const uint64_t naff = naff32;
        if (affected_out && !on_device && naff) {
            HIPCHK(hipMemcpyAsync(affected_out, h->pairs.p, naff * 4, hipMemcpyDeviceToHost, s));
            h->sync();
        }
        // the ids for walk()'s affected-walk stage (host callers, at most kStageMax of them)
        h->last_aff.clear();
        h->last_aff_version = ~0ull;
        if (!on_device && naff && naff <= wharf_handle::kStageMax) {
            if (affected_out) {
                h->last_aff.assign(affected_out, affected_out + naff);
            } else {
                h->last_aff.resize(naff);
                HIPCHK(hipMemcpyAsync(h->last_aff.data(), h->pairs.p, naff * 4, hipMemcpyDeviceToHost, s));
                h->sync();
            }
            h->last_aff_version = h->walks_version;
        }
        h->st.affected = naff;
        if (n_affected) *n_affected = naff;
        h->read_counters();
        h->st.last_walk_kernel_ms = h->elapsed(2, 3);
        h->st.last_walk_update_ms = h->elapsed(1, 3);
    } else {
        h->sync();
    }
}

int do_update(wharf_handle* h, bool insert, uint64_t m, const uint32_t* pairs, uint32_t flags,
              uint32_t* affected_out, uint64_t* n_affected)
{
    return guarded(h, [&] {
        REQUIRE(h, WHARF_E_INVALID, "null handle");
        REQUIRE(m == 0 || pairs, WHARF_E_INVALID, "pairs is null");
        REQUIRE(m < (1ull << 31), WHARF_E_INVALID, "batch too large");
        h->check_walks();
        h->rev_pinned = false;
        auto t0 = std::chrono::steady_clock::now();
        h->st.affected = 0;
        h->st.batch_edges = 0;
        h->st.steps = h->st.accepts = h->st.last_anchor_inits = h->st.last_rewalk_passes = 0;
        h->st.last_graph_update_ms = h->st.last_walk_update_ms = h->st.last_walk_kernel_ms = 0;
        h->st.last_csr_move_ms = 0;
        h->st.last_moved_slots = 0;
        h->st.last_in_edge_mode = 0;
        if (n_affected) *n_affected = 0;
        if (m == 0) return;
        hipStream_t s = h->s;
        // 1. batch -> device keys, validated, sorted by (src, dst), deduplicated
        //    (wharfmh.h:450-470, 1056-1104)
        h->pairs.ensure_grow(m * 8);
        h->k1.ensure_grow(m * 8);
        h->k2.ensure_grow(m * 8);
        HIPCHK(hipMemcpyAsync(h->pairs.p, pairs, m * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemsetAsync(h->errflag.p, 0, 8, s));
        launch_pairs_to_keys(h->pairs.as<uint32_t>(), m, h->n, h->k1.as<uint64_t>(),
                             h->errflag.as<unsigned long long>(), s);
        HIPCHK(hipEventRecord(h->ev[0], s));
        const uint64_t mb = h->unique_keys(m, (flags & WHARF_REMOVE_DUPS) != 0, 32 + std::max<uint32_t>(bits_for(h->n), 1));
        unsigned long long errv = 0;
        HIPCHK(hipMemcpy(&errv, h->errflag.p, 8, hipMemcpyDeviceToHost));
        REQUIRE(errv == 0, WHARF_E_INVALID, "edge endpoint >= number_of_vertices()");
        h->st.batch_edges = mb;
        if (mb == 0) return;
        uint64_t* bkeys = h->k1.as<uint64_t>();

        // 2. source runs (pack_index, wharfmh.h:475-481)
        h->flags.ensure_grow(mb);
        launch_run_flags(bkeys, mb, h->flags.as<uint8_t>(), s);
        h->runstart.ensure_grow(mb * 4);
        {
            auto cnt_it = rocprim::counting_iterator<uint32_t>(0);
            uint8_t* fl = h->flags.as<uint8_t>();
            uint32_t* rsp = h->runstart.as<uint32_t>();
            uint64_t* c = h->count.as<uint64_t>();
            h->rp([&](void* t, size_t& b) { return rocprim::select(t, b, cnt_it, fl, rsp, c, (size_t)mb, s); });
        }
        // 3. which batch edges change their row (uniont / difference), exclusive scan
        h->chg.ensure_grow((mb + 1) * 4);
        h->cf.ensure_grow((mb + 1) * 4);
        HIPCHK(hipMemsetAsync(h->chg.as<uint32_t>() + mb, 0, 4, s));
        launch_batch_change(bkeys, mb, h->off.as<uint64_t>(), h->deg.as<uint32_t>(), h->adj.as<uint32_t>(), insert,
                            h->chg.as<uint32_t>(), s);
        {
            uint32_t* in = h->chg.as<uint32_t>();
            uint32_t* out = h->cf.as<uint32_t>();
            h->rp([&](void* t, size_t& b) {
                return rocprim::exclusive_scan(t, b, in, out, 0u, (size_t)(mb + 1), rocprim::plus<uint32_t>(), s);
            });
        }
        uint64_t k = 0;
        uint32_t total_chg = 0;
        unsigned long long batch_asym = 0;
        HIPCHK(hipMemcpyAsync(&k, h->count.p, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&total_chg, h->cf.as<uint32_t>() + mb, 4, hipMemcpyDeviceToHost, s));
        if ((h->anchors || h->rev_on) && h->symmetric) {   // a batch without every reverse edge leaves the graph directed
            unsigned long long* asym = h->errflag.as<unsigned long long>() + 3;
            HIPCHK(hipMemsetAsync(asym, 0, 8, s));
            launch_keys_symmetric(bkeys, mb, asym, s);
            HIPCHK(hipMemcpyAsync(&batch_asym, asym, 8, hipMemcpyDeviceToHost, s));
        }
        h->sync();

        // 4. the batch sources' rows (wharfmh.h:504-540, 652-690): merged in place
        //    or moved to the pool's end; their samplers are reset (row epoch)
        const uint64_t m_new = insert ? h->m + total_chg : h->m - total_chg;
        // row epochs live in 24 bits of the records (wharf_device.h make_rec) and
        // feed the Philox counters: refuse the batch that would wrap them.  The
        // epoch (and the sources' row epochs, k_commit_rows) advance only once
        // the batch can no longer fail: after the pool planning below.
        REQUIRE(h->epoch + 1 < (1u << kEpochBits), WHARF_E_INVALID, "update epoch limit (2^24 applied batches) reached");
        const uint32_t epoch = h->epoch + 1;
        h->runs.ensure_grow(k * sizeof(RunInfo));
        h->rplan.ensure_grow(k * sizeof(RowPlan));
        h->pscan.ensure_grow((k + 1) * 32);
        uint64_t* need = h->pscan.as<uint64_t>();
        uint64_t* save = need + (k + 1);
        uint64_t* relofs = save + (k + 1);
        uint64_t* sofs = relofs + (k + 1);
        unsigned long long* dead_d = h->errflag.as<unsigned long long>() + 1;
        const int slack = wharf_handle::row_slack();
        // the in-edge pass reads dead slots too: past a quarter of the pool, reclaim them
        if (h->dead_slots * 4 > h->pool_used) h->make_room(0);
        uint64_t grow = 0, saved = 0;
        unsigned long long dead = 0;
        for (int attempt = 0;; attempt++) {
            HIPCHK(hipMemsetAsync(h->bitmap.p, 0, (h->bitmap_words() + kFilterWords) * 4, s));
            HIPCHK(hipMemsetAsync(dead_d, 0, 8, s));
            launch_run_info(bkeys, h->runstart.as<uint32_t>(), k, mb, h->off.as<uint64_t>(), h->deg.as<uint32_t>(),
                            h->runs.as<RunInfo>(), h->bitmap.as<uint32_t>(), h->bitmap.as<uint32_t>() + h->bitmap_words(), s);
            launch_plan_rows(h->runs.as<RunInfo>(), k, h->cap.as<uint32_t>(), h->cf.as<uint32_t>(), insert, slack, need,
                             save, h->rplan.as<RowPlan>(), dead_d, s);
            h->scan_u64(need, relofs, k + 1);
            h->scan_u64(save, sofs, k + 1);
            HIPCHK(hipMemcpyAsync(&grow, relofs + k, 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(&saved, sofs + k, 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(&dead, dead_d, 8, hipMemcpyDeviceToHost, s));
            h->sync();
            if (h->pool_used + grow <= h->pool_cap) break;
            REQUIRE(attempt == 0, WHARF_E_NOMEM,
                    "slot pool exhausted: no device memory for a second pool and the in-place compaction left too "
                    "little room (used " + std::to_string(h->pool_used) + ", grow " + std::to_string(grow) +
                        ", capacity " + std::to_string(h->pool_cap) + "); the batch was not applied");
            // out of headroom: fresh slack everywhere (or dead slots squeezed out),
            // then plan again.  The fresh capacities can be smaller than the old
            // ones (rows that shrank keep theirs), so room is made for every
            // source moving with grown slack.
            const uint64_t all = saved + (insert ? total_chg : 0);
            h->make_room(all + all / 8 + 4 * k);
        }
        h->epoch = epoch;
        h->dead_slots += dead;
        if (batch_asym) h->symmetric = false;
        if (h->rev_on && !h->symmetric) h->drop_rev();
        // Anchor carry (node2vec MH on an undirected graph): the entries of the sources' rows travel
        // through the merge and only those whose anchor can change are reset (k_anchor_invalidate);
        // otherwise every entry of a rebuilt row starts empty.  WHARF_ANCHOR_CARRY=0 (A/B, tests).
        const char* acv = getenv("WHARF_ANCHOR_CARRY");
        const bool carry = h->anchors && h->symmetric && !(acv && *acv && atoi(acv) == 0);
        uint64_t* anc_base = h->anchors ? h->erec.as<uint64_t>() + 2 : nullptr;
        // every per-batch buffer is allocated before the reverse index is pinned: an allocation that
        // fails here can still reclaim the index (the batch then scans) instead of failing the batch
        if (carry) h->sanc.ensure_grow(std::max<uint64_t>(saved, 1) * 8);
        h->scratch.ensure_grow(std::max<uint64_t>(saved, 1) * 4);
        // source rows in chunks: counts of each run's longest range, exclusive prefix (k_run_chunks)
        h->rchunk.ensure_grow((k + 1) * 8);
        if (h->rev_on && h->rev_valid) h->srev.ensure_grow(std::max<uint64_t>(saved, 1) * 4);
        // reverse-slot index: carried through the merge and used for the in-edge records
        // unless a repack or compaction of this batch moved every row (then: scan, rebuild)
        // or the allocations above reclaimed it
        const bool use_rev = h->rev_on && h->rev_valid;
        h->rev_pinned = use_rev;   // from here to the in-edge pass the index must stay (no reclaim)
        h->grown = grow;
        h->start_bound = saved + (insert ? total_chg : 0);   // the sources' degrees after the update, at most
        const uint32_t rs = (uint32_t)h->rec_stride();
        uint32_t* rcnt = h->rchunk.as<uint32_t>();
        uint32_t* rpre = rcnt + (k + 1);
        launch_run_chunks(h->runs.as<RunInfo>(), h->rplan.as<RowPlan>(), k, rcnt, s);
        h->rp([&](void* t, size_t& b) {
            return rocprim::exclusive_scan(t, b, rcnt, rpre, 0u, (size_t)(k + 1), rocprim::plus<uint32_t>(), s);
        });
        launch_save_rows(h->runs.as<RunInfo>(), k, rpre, h->adj.as<uint32_t>(), sofs, h->scratch.as<uint32_t>(), anc_base,
                         carry ? h->sanc.as<uint64_t>() : nullptr, use_rev ? h->rev.as<uint32_t>() : nullptr,
                         use_rev ? h->srev.as<uint32_t>() : nullptr, s);
        launch_merge_rows(h->runs.as<RunInfo>(), k, rpre, bkeys, h->chg.as<uint32_t>(), h->cf.as<uint32_t>(),
                          h->scratch.as<uint32_t>(), sofs, relofs, h->pool_used, insert, h->rplan.as<RowPlan>(),
                          h->adj.as<uint32_t>(), carry ? h->sanc.as<uint64_t>() : nullptr, anc_base,
                          use_rev ? h->srev.as<uint32_t>() : nullptr, use_rev ? h->rev.as<uint32_t>() : nullptr, s);
        launch_commit_rows(h->runs.as<RunInfo>(), k, h->rplan.as<RowPlan>(), h->epoch, h->off.as<uint64_t>(),
                           h->deg.as<uint32_t>(), h->cap.as<uint32_t>(), h->vrec.as<ERec>(), h->row_epoch.as<uint32_t>(), s);
        h->pool_used += grow;
        h->m = m_new;
        // records: the source rows' slots (anchors reset), then every slot whose
        // target is a source (one streaming scan of the pool)
        launch_erec_rows(h->runs.as<RunInfo>(), k, rpre, h->off.as<uint64_t>(), h->deg.as<uint32_t>(), h->adj.as<uint32_t>(),
                         h->vrec.as<ERec>(), h->erec.as<ERec>(), rs, carry ? 1 : 0, h->rf, s);
        HIPCHK(hipEventRecord(h->ev[4], s));
        bool scan = !use_rev;
        if (use_rev) {   // the sources' in-edges from their own rows (k_patch_rev)
            unsigned long long* miss = h->errflag.as<unsigned long long>() + 4;
            HIPCHK(hipMemsetAsync(miss, 0, 8, s));
            launch_patch_rev(h->runs.as<RunInfo>(), k, rpre, h->off.as<uint64_t>(), h->deg.as<uint32_t>(),
                             h->adj.as<uint32_t>(), h->bitmap.as<uint32_t>(), h->vrec.as<ERec>(), h->erec.as<ERec>(), rs,
                             h->rf, h->rev.as<uint32_t>(), miss, s);
            unsigned long long v = 0;
            HIPCHK(hipMemcpyAsync(&v, miss, 8, hipMemcpyDeviceToHost, s));
            h->sync();
            if (v) {   // an edge without its reverse (1), or a stale carried entry (2, repaired before its
                       // write): neither can happen on a graph tracked as symmetric.  The index is not
                       // trusted again; the scan rewrites every in-edge record of the sources.
                h->drop_rev();
                h->st.rev_fallbacks++;
                scan = true;
            }
        }
        if (scan)
            launch_patch_in_edges(h->adj.as<uint32_t>(), h->pool_used, h->bitmap.as<uint32_t>(),
                                  h->bitmap.as<uint32_t>() + h->bitmap_words(), h->vrec.as<ERec>(), h->erec.as<ERec>(),
                                  rs, h->rf, s);
        HIPCHK(hipEventRecord(h->ev[5], s));
        h->rev_pinned = false;
        if (h->rev_on && !h->rev_valid) h->build_rev();   // after a repack / compaction in this batch
        h->st.last_moved_slots = scan ? h->pool_used : h->start_bound;   // (insert: exact; delete: an upper bound)
        h->st.last_in_edge_mode = scan ? 0 : 1;
        if (h->anchors) {
            // the edge set changes by the batch's changing edges only; rebuild when
            // inserts (and tombstones) push the load past 0.6
            if (insert && (h->ehash_used + total_chg) * 10 > (h->ehash_mask + 1) * 6) {
                h->build_edge_hash();
            } else {
                launch_edge_hash_update(bkeys, mb, h->chg.as<uint32_t>(), insert, h->ehash.as<uint64_t>(),
                                        h->ehash_mask, s);
                if (insert) h->ehash_used += total_chg;
            }
            h->update_filters(h->runs.as<RunInfo>(), k);
            // anchor carry: reset the carried entries a changed edge can affect (c's filter, new rows)
            if (carry)
                launch_anchor_invalidate(bkeys, mb, h->chg.as<uint32_t>(), h->off.as<uint64_t>(), h->deg.as<uint32_t>(),
                                         h->adj.as<uint32_t>(), anc_base, h->fpool.p ? h->fdir.as<uint64_t>() : nullptr,
                                         h->fpool.p ? h->fpool.as<uint32_t>() : nullptr, s);
        }
        HIPCHK(hipGetLastError());   // a failed launch of the CSR pipeline surfaces here
        HIPCHK(hipEventRecord(h->ev[1], s));

        // 5. rewalk points + suffix re-walk in one pass over the walk matrix
        //    (wharfmh.h:519-537 and batch_walk_update 733-923)
        walk_update(h, k, flags, affected_out, n_affected);
        h->st.last_graph_update_ms = h->elapsed(0, 1);
        h->st.last_csr_move_ms = h->elapsed(4, 5);
        h->st.last_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
}

}  // namespace

extern "C" {

void wharf_config_default(wharf_config* c)
{
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->walks_per_vertex = 10;              // globals.h:7
    c->walk_length = 80;                   // globals.h:10
    c->model = WHARF_NODE2VEC;             // globals.h:13 (the experiments pass -model deepwalk explicitly)
    c->paramP = 4.0f;                      // globals.h:16
    c->paramQ = 1.0f;                      // globals.h:19
    c->sampler_init = WHARF_INIT_WEIGHT;   // globals.h:22
    c->deterministic = 1;                  // globals.h:28
    c->seed = 0x5EED;
}

const char* wharf_last_error(const wharf_handle* h) { return h ? h->err.c_str() : g_last_error.c_str(); }
int wharf_abi_version(void) { return WHARF_ABI_VERSION; }

int wharf_device_count(int* count)
{
    return guarded(nullptr, [&] {
        REQUIRE(count, WHARF_E_INVALID, "count is null");
        HIPCHK(hipGetDeviceCount(count));
    });
}

int wharf_create(const wharf_config* cfg, uint64_t n, uint64_t m, const uint64_t* offsets, const uint32_t* targets,
                 int device, wharf_handle** out)
{
    wharf_handle* h = nullptr;
    int rc = guarded(nullptr, [&] {
        REQUIRE(out, WHARF_E_INVALID, "out is null");
        REQUIRE(offsets && (m == 0 || targets), WHARF_E_INVALID, "offsets/targets is null");
        for (uint64_t v = 0; v < n; v++)
            REQUIRE(offsets[v] <= (v + 1 < n ? offsets[v + 1] : m), WHARF_E_INVALID, "offsets must be non-decreasing and <= m");
        h = new_handle(cfg, n, device);
        std::vector<uint64_t> off(offsets, offsets + n);
        off.push_back(m);
        h->off2.ensure((n + 1) * 8);
        HIPCHK(hipMemcpyAsync(h->off2.p, off.data(), (n + 1) * 8, hipMemcpyHostToDevice, h->s));
        h->adj2.ensure(std::max<uint64_t>(m, 1) * 4);
        if (m) HIPCHK(hipMemcpyAsync(h->adj2.p, targets, m * 4, hipMemcpyHostToDevice, h->s));
        h->k1.ensure(std::max<uint64_t>(m, 1) * 8);
        h->k2.ensure(std::max<uint64_t>(m, 1) * 8);
        HIPCHK(hipMemsetAsync(h->errflag.p, 0, 8, h->s));
        launch_csr_to_keys(h->off2.as<uint64_t>(), n, h->adj2.as<uint32_t>(), h->k1.as<uint64_t>(),
                           h->errflag.as<unsigned long long>(), h->s);
        unsigned long long errv = 0;
        HIPCHK(hipMemcpyAsync(&errv, h->errflag.p, 8, hipMemcpyDeviceToHost, h->s));
        h->sync();
        REQUIRE(errv == 0, WHARF_E_INVALID, "edge target >= n");
        build_graph_from_keys(h, m, false, false);
        h->k1.release();
        h->k2.release();
        h->off2.release();
        h->adj2.release();
    });
    if (rc != WHARF_OK) {
        free_handle(h);
        return rc;
    }
    *out = h;
    return WHARF_OK;
}

int wharf_create_empty(const wharf_config* cfg, uint64_t n, int device, wharf_handle** out)
{
    static const uint64_t zero = 0;
    std::vector<uint64_t> off(n, 0);
    return wharf_create(cfg, n, 0, n ? off.data() : &zero, nullptr, device, out);
}

int wharf_create_rmat(const wharf_config* cfg, uint64_t n, uint64_t edges_number, uint64_t vertices_number,
                      uint64_t seed, double a, double b, double c, int device, wharf_handle** out)
{
    wharf_handle* h = nullptr;
    int rc = guarded(nullptr, [&] {
        REQUIRE(out, WHARF_E_INVALID, "out is null");
        REQUIRE(vertices_number >= 2, WHARF_E_INVALID, "vertices_number must be >= 2");
        REQUIRE((1ull << (bits_for(vertices_number) - 1)) <= n, WHARF_E_INVALID, "n smaller than the RMAT vertex range");
        h = new_handle(cfg, n, device);
        rmat_keys(h, edges_number, vertices_number, seed, /*directed=*/0, a, b, c);
        build_graph_from_keys(h, 2 * edges_number, /*drop self loops*/ true, /*symmetric: undirected samples*/ true);
        h->k1.release();
        h->k2.release();
        h->tmp.release();
        h->flags.release();
    });
    if (rc != WHARF_OK) {
        free_handle(h);
        return rc;
    }
    *out = h;
    return WHARF_OK;
}

int wharf_destroy(wharf_handle* h)
{
    free_handle(h);
    return WHARF_OK;
}

int wharf_destroy_index(wharf_handle* h)
{
    return guarded(h, [&] {
        REQUIRE(h, WHARF_E_INVALID, "null handle");
        h->ensure_walks();
        launch_fill_u32(h->walks.as<uint32_t>(), h->W * h->L, kSent, h->s);
        h->walks_changed();
        h->sync();
        h->has_walks = false;
        h->walks_poisoned = false;
    });
}

int wharf_release_caches(wharf_handle* h, uint64_t* freed_bytes)
{
    return guarded(h, [&] {
        REQUIRE(h, WHARF_E_INVALID, "null handle");
        const uint64_t held = h->rev.p ? (uint64_t)h->rev.cap + h->srev.cap : 0;
        const bool dropped = h->reclaim();   // (not rebuilt lazily afterwards: the room is wanted elsewhere)
        if (freed_bytes) *freed_bytes = dropped ? held : 0;
    });
}

// The line-count model behind the up-front init order (k_anchor_init_all / k_anchor_init_cur): 21
// uniform proposals over L 128-B lines touch L (1 - (1 - 1/L)^21) distinct lines.  Prev order pays
// that over cur's row (4 B per slot: 32 slots per line); cur order pays it over prev's neighbour
// filter (2^lg 32-bit words: 32 per line), plus prev's filter descriptor and the entry written at
// the reverse slot.  t[lg] = the fewest lines of cur's row at which cur order is cheaper.
// WHARF_INIT_CUR_BIAS (lines, A/B and tests) is added to the cur-order side.
static InitOrder init_order_table(const WalkArgs& a)
{
    auto distinct = [](double L) { return L <= 1.0 ? 1.0 : L * (1.0 - std::pow(1.0 - 1.0 / L, (double)kWeightProposals)); };
    const char* b = getenv("WHARF_INIT_CUR_BIAS");
    const double bias = b && *b ? atof(b) : 0.0;
    const bool use_f = a.fpool && a.inv_q != 1.0f;
    InitOrder ord;
    for (uint32_t lg = 0; lg < kInitOrderLg; lg++) {
        const double filt_lines = std::max(1.0, std::ldexp(1.0, (int)lg) / 32.0);
        const double cur_cost = 1.0 + (use_f ? 1.0 + distinct(filt_lines) : 0.0) + bias;
        uint64_t lo = 1, hi = 1;
        while (hi < (1ull << 32) && distinct((double)hi) <= cur_cost) hi <<= 1;
        if (distinct((double)hi) <= cur_cost) {
            ord.t[lg] = 0xFFFFFFFFu;   // never cheaper (D < 21 for every row)
            continue;
        }
        while (lo < hi) {   // the least L with distinct(L) > cur_cost
            const uint64_t mid = (lo + hi) / 2;
            if (distinct((double)mid) > cur_cost) hi = mid; else lo = mid + 1;
        }
        ord.t[lg] = (uint32_t)lo;
    }
    return ord;
}

int wharf_generate(wharf_handle* h)
{
    return guarded(h, [&] {
        REQUIRE(h, WHARF_E_INVALID, "null handle");
        auto t0 = std::chrono::steady_clock::now();
        HIPCHK(hipMemsetAsync(h->counters.p, 0, 16, h->s));
        HIPCHK(hipMemsetAsync(h->counters.as<unsigned long long>() + 7, 0, 8, h->s));
        h->st_park_passes = 0;
        WalkArgs a = h->walk_args();
        // the reverse-slot index, when it did not fit at creation beside every walk: now that the
        // walk matrix (of this handle's shard) is allocated (not timed with the generation)
        if (!h->rev_on && !h->rev_tried && h->symmetric && h->rev_wanted(false)) {
            h->rev_on = true;
            h->build_rev();
        }
        h->rev_tried = true;
        HIPCHK(hipEventRecord(h->ev[0], h->s));
        // node2vec MH with a cold anchor cache and at least as many steps as states
        // (slots): every anchor computed up front (k_anchor_init_all), timed with the
        // generation.  Round 4: the rule was 4 steps per slot; at configs[4]'s 1/8 shard
        // (1.6 per slot) the lazy generation leaves 1.1 G of 3.6 G states cold, and every
        // update's re-walk then runs into them: 88.5 M inits per batch, re-walk 65.5 ms,
        // against 9.4 M and 34.9 ms with all anchors computed (first generation 1.06 ->
        // 1.10 s; profiles/r04/preinit_all).  WHARF_PREINIT_ALL=1 / 0 forces it on / off.
        const char* no_pre = getenv("WHARF_NO_PREINIT");
        const char* pre_all = getenv("WHARF_PREINIT_ALL");
        const bool all_rule = pre_all && *pre_all ? atoi(pre_all) != 0 : (uint64_t)h->W * (h->L - 1) >= h->pool_used;
        if (a.model == kNode2Vec && !a.det && a.anchor && h->anchors_cold && h->pool_used && all_rule &&
            !(no_pre && atoi(no_pre))) {
            // the slot owners live in the walk matrix, which this generation overwrites next:
            // the rule (>= 1 step per slot) makes it the larger (W * L > pool_used); a 16-GB
            // allocation here (configs[4]) cost 0-1 s of page mapping, box to box
            size_t free_b = 0, total_b = 0;
            const bool in_walks = h->walks.cap >= h->pool_used * 4;
            if (!in_walks) HIPCHK(hipMemGetInfo(&free_b, &total_b));
            if (in_walks || h->pool_used * 4 + (1ull << 30) < free_b) {
                DevBuf owner;
                if (!in_walks) owner.ensure(h->pool_used * 4);
                uint32_t* ow = in_walks ? h->walks.as<uint32_t>() : owner.as<uint32_t>();
                HIPCHK(hipMemsetAsync(ow, 0, h->pool_used * 4, h->s));
                launch_slot_owner_fill(h->off.as<uint64_t>(), h->deg.as<uint32_t>(), h->n, ow, h->s);
                // round 5: the states of hub curs with small prevs in cur order (WHARF_INIT_BY_CUR=1: on;
                // WHARF_INIT_BY_CUR_Y / _X: the degree thresholds), on undirected graphs only
                const char* bc = getenv("WHARF_INIT_BY_CUR");
                const char* bcy = getenv("WHARF_INIT_BY_CUR_Y");
                const char* bcx = getenv("WHARF_INIT_BY_CUR_X");
                // (off by default: configs[4] first generation 1128 / 1141 ms with it, 1131 / 1107 ms without,
                // alternated on one box, profiles/r05/init_by_cur)
                const bool by_cur = h->symmetric && bc && *bc && atoi(bc) != 0;
                const uint32_t ty = by_cur ? (bcy && *bcy ? (uint32_t)atoi(bcy) : 256u) : 0u;
                const uint32_t tx = bcx && *bcx ? (uint32_t)atoi(bcx) : 256u;
                // round 6: with the reverse-slot index every state goes to the cheaper order
                // (init_order_table; WHARF_INIT_ORDER=0: all in prev order, or the round-5 rule above)
                const char* io = getenv("WHARF_INIT_ORDER");
                const bool hybrid = h->symmetric && h->rev_on && h->rev.p && !(io && *io && atoi(io) == 0);
                const char* rvf = getenv("WHARF_REV_VERIFY");
                launch_anchor_init_all(a, ow, h->pool_used, ty, tx, hybrid ? h->rev.as<uint32_t>() : nullptr,
                                       init_order_table(a), rvf && *rvf && atoi(rvf) != 0, h->s);
                HIPCHK(hipStreamSynchronize(h->s));   // before the owner buffer is released
                owner.release();
            }
        }
        h->anchors_cold = false;
        h->walks_changed();
        h->walks_poisoned = false;   // every walk is written anew
        launch_walk(a, false, h->s);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(h->ev[1], h->s));
        h->read_counters();
        h->has_walks = true;
        h->st.affected = 0;
        h->st.last_walk_kernel_ms = h->elapsed(0, 1);
        h->st.last_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
}

int wharf_insert_edges(wharf_handle* h, uint64_t m, const uint32_t* pairs, uint32_t flags, uint32_t* affected_out,
                       uint64_t* n_affected)
{
    return do_update(h, true, m, pairs, flags, affected_out, n_affected);
}

int wharf_delete_edges(wharf_handle* h, uint64_t m, const uint32_t* pairs, uint32_t flags, uint32_t* affected_out,
                       uint64_t* n_affected)
{
    return do_update(h, false, m, pairs, flags, affected_out, n_affected);
}

int wharf_batch_walk_update(wharf_handle* h, const uint32_t* sources, uint64_t k, uint32_t flags,
                            uint32_t* affected_out, uint64_t* n_affected)
{
    return guarded(h, [&] {
        REQUIRE(h, WHARF_E_INVALID, "null handle");
        REQUIRE(k == 0 || sources, WHARF_E_INVALID, "sources is null");
        h->check_walks();
        auto t0 = std::chrono::steady_clock::now();
        h->st.affected = 0;
        h->st.steps = h->st.accepts = h->st.last_anchor_inits = h->st.last_rewalk_passes = 0;
        h->st.batch_edges = 0;
        h->st.last_graph_update_ms = h->st.last_walk_update_ms = h->st.last_walk_kernel_ms = 0;
        h->st.last_csr_move_ms = 0;
        h->st.last_moved_slots = 0;
        if (n_affected) *n_affected = 0;
        // the vertex set of the MapOfChanges: sorted, deduplicated, validated
        std::vector<uint32_t> src(sources, sources + k);
        std::sort(src.begin(), src.end());
        src.erase(std::unique(src.begin(), src.end()), src.end());
        REQUIRE(src.empty() || src.back() < h->n, WHARF_E_INVALID, "source vertex >= number_of_vertices()");
        k = src.size();
        hipStream_t s = h->s;
        HIPCHK(hipMemsetAsync(h->bitmap.p, 0, (h->bitmap_words() + kFilterWords) * 4, s));
        if (k) {
            h->k1.ensure(k * 4);
            HIPCHK(hipMemcpyAsync(h->k1.p, src.data(), k * 4, hipMemcpyHostToDevice, s));
            h->runs.ensure(k * sizeof(RunInfo));
            launch_mark_sources(h->k1.as<uint32_t>(), k, h->runs.as<RunInfo>(), h->bitmap.as<uint32_t>(),
                                h->bitmap.as<uint32_t>() + h->bitmap_words(), s);
        }
        HIPCHK(hipEventRecord(h->ev[1], s));
        walk_update(h, k, flags | WHARF_APPLY_WALK_UPDATES, affected_out, n_affected);
        h->st.last_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
}

int wharf_number_of_vertices(const wharf_handle* h, uint64_t* n)
{
    if (!h || !n) return WHARF_E_INVALID;
    *n = h->n;
    return WHARF_OK;
}

int wharf_number_of_edges(const wharf_handle* h, uint64_t* m)
{
    if (!h || !m) return WHARF_E_INVALID;
    *m = h->m;
    return WHARF_OK;
}

int wharf_shard(const wharf_handle* h, uint64_t* lo, uint64_t* hi, uint64_t* walks)
{
    if (!h) return WHARF_E_INVALID;
    if (lo) *lo = h->lo;
    if (hi) *hi = h->hi;
    if (walks) *walks = h->W;
    return WHARF_OK;
}

int wharf_set_shard(wharf_handle* h, uint64_t lo, uint64_t hi)
{
    return guarded(h, [&] {
        REQUIRE(h, WHARF_E_INVALID, "null handle");
        if (hi == 0) hi = h->n;
        REQUIRE(lo <= hi && hi <= h->n, WHARF_E_INVALID, "shard range must satisfy lo <= hi <= n");
        h->sync();
        h->walks.release();
        h->walks_changed();
        h->free_snaps();
        h->aff.release();
        h->defer.release();
        h->park.release();
        h->bdesc.release();
        h->lo = lo;
        h->hi = hi;
        h->n_loc = hi - lo;
        h->sh_part = 0;
        h->sh_parts = 1;
        h->sh_bits = 0;
        h->W = h->n_loc * h->wpv;
        h->cfg.shard_lo = lo;
        h->cfg.shard_hi = hi;
        h->has_walks = false;
        h->walks_poisoned = false;   // a new walk matrix
    });
}

int wharf_set_shard_blocks(wharf_handle* h, uint32_t part, uint32_t parts, uint32_t block_bits)
{
    return guarded(h, [&] {
        REQUIRE(h, WHARF_E_INVALID, "null handle");
        REQUIRE(parts >= 1 && part < parts, WHARF_E_INVALID, "block shard: need part < parts");
        REQUIRE(block_bits >= 6 && block_bits < 32, WHARF_E_INVALID, "block shard: block_bits must be 6..31");
        REQUIRE((h->n * h->wpv) < (1ull << 32), WHARF_E_INVALID, "n * walks_per_vertex must be < 2^32");
        // owned vertices: the part's blocks of 2^bits, round-robin; only the graph's last block can be short
        const uint64_t B = 1ull << block_bits, nblocks = (h->n + B - 1) / B;
        uint64_t n_loc = 0;
        for (uint64_t q = part; q < nblocks; q += parts) n_loc += std::min(B, h->n - q * B);
        h->sync();
        h->walks.release();
        h->walks_changed();
        h->free_snaps();
        h->aff.release();
        h->defer.release();
        h->park.release();
        h->bdesc.release();
        h->lo = 0;
        h->hi = h->n;
        h->n_loc = n_loc;
        h->sh_part = part;
        h->sh_parts = parts;
        h->sh_bits = block_bits;
        h->W = n_loc * h->wpv;
        h->cfg.shard_lo = 0;
        h->cfg.shard_hi = 0;
        h->has_walks = false;
        h->walks_poisoned = false;   // a new walk matrix
    });
}

int wharf_shard_blocks(const wharf_handle* h, uint32_t* part, uint32_t* parts, uint32_t* block_bits)
{
    if (!h) return WHARF_E_INVALID;
    if (part) *part = h->sh_part;
    if (parts) *parts = h->sh_parts;
    if (block_bits) *block_bits = h->sh_bits;
    return WHARF_OK;
}

int wharf_get_graph(wharf_handle* h, uint64_t* offsets_out, uint32_t* targets_out)
{
    return guarded(h, [&] {
        REQUIRE(h && offsets_out, WHARF_E_INVALID, "null argument");
        // the slack rows, compacted: offsets = scan of the degrees, rows copied
        DevBuf coff, cadj;
        coff.ensure((h->n + 1) * 8);
        launch_deg_u64(h->deg.as<uint32_t>(), h->n, coff.as<uint64_t>(), h->s);
        h->scan_u64(coff.as<uint64_t>(), coff.as<uint64_t>(), h->n + 1);
        HIPCHK(hipMemcpyAsync(offsets_out, coff.p, (h->n + 1) * 8, hipMemcpyDeviceToHost, h->s));
        if (h->m && targets_out) {
            cadj.ensure(h->m * 4);
            launch_copy_rows(h->off.as<uint64_t>(), h->deg.as<uint32_t>(), h->adj.as<uint32_t>(), coff.as<uint64_t>(),
                             h->n, cadj.as<uint32_t>(), nullptr, nullptr, h->s);
            HIPCHK(hipMemcpyAsync(targets_out, cadj.p, h->m * 4, hipMemcpyDeviceToHost, h->s));
        }
        h->sync();
    });
}

// WHARF_WALK_NO_SNAPSHOT=1 (A/B, tools/walk_readout): walk() / vertex_at_walk() read the device per call
static bool no_snapshot()
{
    const char* e = getenv("WHARF_WALK_NO_SNAPSHOT");
    return e && atoi(e);
}

static uint64_t local_index(wharf_handle* h, uint64_t wid)
{
    h->check_walks();
    uint64_t li = 0;
    REQUIRE(h->owned_li(wid, li), WHARF_E_RANGE, "walk " + std::to_string(wid) + " is not owned by this handle");
    return li;
}

int wharf_walk(wharf_handle* h, uint64_t wid, uint32_t* out, uint32_t* len)
{
    return guarded(h, [&] {
        REQUIRE(h && out && len, WHARF_E_INVALID, "null argument");
        const uint64_t li = local_index(h, wid);
        h->ensure_walks();
        if (no_snapshot()) {   // A/B: one gather kernel, D2H and sync per call (round 2's path)
            h->sel.ensure(h->L * 4);
            launch_gather_rows(h->walks.as<uint32_t>(), h->W, h->L, nullptr, li, 1, h->sel.as<uint32_t>(), h->s);
            HIPCHK(hipMemcpyAsync(out, h->sel.p, h->L * 4, hipMemcpyDeviceToHost, h->s));
            h->sync();
        } else {
            std::memcpy(out, h->snap_row(li), h->L * 4);
        }
        uint32_t c = 0;
        while (c < h->L && out[c] != kSent) c++;
        *len = c;
    });
}

int wharf_walk_string(wharf_handle* h, uint64_t wid, char* buf, size_t cap, size_t* len)
{
    uint32_t v[256];   // walk_length <= 255 (types::Position is u8)
    uint32_t cnt = 0;
    int rc = wharf_walk(h, wid, v, &cnt);
    if (rc) return rc;
    char s[256 * 11 + 1];   // "v0 v1 ... " (wharfmh.h:375): <= 10 digits and a space per vertex
    char* e = s;
    for (uint32_t i = 0; i < cnt; i++) {
        e = std::to_chars(e, s + sizeof(s), v[i]).ptr;
        *e++ = ' ';
    }
    *e = 0;
    const size_t n = (size_t)(e - s);
    if (len) *len = n;
    if (buf) {
        if (cap < n + 1) {
            set_err(h, "buffer too small");
            return WHARF_E_INVALID;
        }
        std::memcpy(buf, s, n + 1);
    }
    return WHARF_OK;
}

int wharf_vertex_at_walk(wharf_handle* h, uint64_t wid, uint32_t position, uint32_t* vertex)
{
    return guarded(h, [&] {
        REQUIRE(h && vertex, WHARF_E_INVALID, "null argument");
        REQUIRE(position < h->L, WHARF_E_RANGE, "position >= walk_length");
        const uint64_t li = local_index(h, wid);
        h->ensure_walks();
        if (no_snapshot()) {
            HIPCHK(hipMemcpyAsync(vertex, h->walks.as<uint32_t>() + (uint64_t)position * h->W + li, 4,
                                  hipMemcpyDeviceToHost, h->s));
            h->sync();
        } else {
            *vertex = h->snap_row(li)[position];
        }
    });
}

static void export_walks_impl(wharf_handle* h, uint32_t* dst, int layout, hipMemcpyKind kind)
{
    REQUIRE(h && dst, WHARF_E_INVALID, "null argument");
    REQUIRE(layout == 0 || layout == 1, WHARF_E_INVALID, "layout must be 0 or 1");
    h->check_walks();
    const uint64_t bytes = h->W * h->L * 4;
    if (!bytes) return;
    h->ensure_walks();
    if (layout == 1) {
        HIPCHK(hipMemcpyAsync(dst, h->walks.p, bytes, kind, h->s));
    } else if (kind == hipMemcpyDeviceToDevice) {
        launch_transpose(h->walks.as<uint32_t>(), h->W, h->L, dst, h->s);
    } else {
        h->sel.ensure(bytes);
        launch_transpose(h->walks.as<uint32_t>(), h->W, h->L, h->sel.as<uint32_t>(), h->s);
        HIPCHK(hipMemcpyAsync(dst, h->sel.p, bytes, hipMemcpyDeviceToHost, h->s));
    }
    h->sync();
}

int wharf_export_walks(wharf_handle* h, uint32_t* dst, int layout)
{
    return guarded(h, [&] { export_walks_impl(h, dst, layout, hipMemcpyDeviceToHost); });
}

int wharf_export_walks_device(wharf_handle* h, uint32_t* dst, int layout)
{
    return guarded(h, [&] { export_walks_impl(h, dst, layout, hipMemcpyDeviceToDevice); });
}

// walk-major rows [first, first + count) of this handle's export order (the
// rows wharf_export_walks(layout 0) writes there), without the whole corpus:
// the bounded corpus gather (distributed.py) reads one chunk at a time
static void export_rows_impl(wharf_handle* h, uint64_t first, uint64_t count, uint32_t* dst, bool device)
{
    REQUIRE(h, WHARF_E_INVALID, "null handle");
    REQUIRE(first <= h->W && count <= h->W - first, WHARF_E_RANGE, "rows outside the handle's walks");
    h->check_walks();
    if (!count) return;
    REQUIRE(dst, WHARF_E_INVALID, "null argument");
    h->ensure_walks();
    if (device) {
        launch_gather_rows(h->walks.as<uint32_t>(), h->W, h->L, nullptr, first, count, dst, h->s);
    } else {
        const uint64_t chunk = 1ull << 20;   // staging bounded to 1 Mi rows
        for (uint64_t c0 = 0; c0 < count; c0 += chunk) {
            const uint64_t c = std::min(chunk, count - c0);
            h->sel.ensure(c * h->L * 4);
            launch_gather_rows(h->walks.as<uint32_t>(), h->W, h->L, nullptr, first + c0, c, h->sel.as<uint32_t>(), h->s);
            HIPCHK(hipMemcpyAsync(dst + c0 * h->L, h->sel.p, c * h->L * 4, hipMemcpyDeviceToHost, h->s));
            h->sync();
        }
    }
    HIPCHK(hipGetLastError());
    h->sync();
}

int wharf_export_walk_rows(wharf_handle* h, uint64_t first, uint64_t count, uint32_t* dst)
{
    return guarded(h, [&] { export_rows_impl(h, first, count, dst, false); });
}

int wharf_export_walk_rows_device(wharf_handle* h, uint64_t first, uint64_t count, uint32_t* dst_device)
{
    return guarded(h, [&] { export_rows_impl(h, first, count, dst_device, true); });
}

int wharf_write_corpus(wharf_handle* h, const char* path, const uint32_t* wids, uint64_t count, int append)
{
    return guarded(h, [&] {
        REQUIRE(h && path, WHARF_E_INVALID, "null argument");
        h->check_walks();
        h->ensure_walks();
        const uint64_t total = wids ? count : h->W;
        const uint64_t chunk = 1 << 20;
        std::vector<uint64_t> li;
        std::vector<uint32_t> rows;
        bool app = append != 0;
        if (total == 0 && !app) {
            int rc = wharf_format_corpus(nullptr, 0, h->L, path, 0);
            REQUIRE(rc == WHARF_OK, WHARF_E_INVALID, std::string("cannot write ") + path);
        }
        for (uint64_t c0 = 0; c0 < total; c0 += chunk) {
            const uint64_t c = std::min(chunk, total - c0);
            h->sel.ensure(c * h->L * 4);
            uint64_t* dlist = nullptr;
            if (wids) {
                li.resize(c);
                for (uint64_t i = 0; i < c; i++) li[i] = local_index(h, wids[c0 + i]);
                h->count.ensure(c * 8);
                HIPCHK(hipMemcpyAsync(h->count.p, li.data(), c * 8, hipMemcpyHostToDevice, h->s));
                dlist = h->count.as<uint64_t>();
            }
            launch_gather_rows(h->walks.as<uint32_t>(), h->W, h->L, dlist, c0, c, h->sel.as<uint32_t>(), h->s);
            rows.resize(c * h->L);
            HIPCHK(hipMemcpyAsync(rows.data(), h->sel.p, c * h->L * 4, hipMemcpyDeviceToHost, h->s));
            h->sync();
            int rc = wharf_format_corpus(rows.data(), c, h->L, path, app);
            REQUIRE(rc == WHARF_OK, WHARF_E_INVALID, std::string("cannot write ") + path);
            app = true;
        }
    });
}

int wharf_walk_ids(wharf_handle* h, uint32_t* ids)
{
    return guarded(h, [&] {
        REQUIRE(h && ids, WHARF_E_INVALID, "null argument");
        for (uint64_t li = 0; li < h->W; li++) {
            ids[li] = (uint32_t)h->smap().wid(li);
        }
    });
}

namespace {
// Builds the inverted index of this handle's walks for the vertices of
// [v0, v1), sorted by (vertex, key); returns the entry count.  Leaves the
// sorted keys (vertex - v0) << kb | key in k2 and their values in pairs.
uint64_t build_index(wharf_handle* h, int& kb, uint64_t v0, uint64_t v1)
{
    const uint64_t W = h->W;
    h->check_walks();
    h->ensure_walks();
    kb = (int)std::max<uint32_t>(bits_for(h->n * h->wpv * h->L), 1);
    const int vb = (int)std::max<uint32_t>(bits_for(v1 - v0), 1);
    REQUIRE(kb + vb <= 64, WHARF_E_INVALID, "index key does not fit 64 bits");
    h->sel.ensure((W + 1) * 8);
    h->count.ensure((W + 1) * 8);
    uint64_t* len = h->sel.as<uint64_t>();
    uint64_t* base = h->count.as<uint64_t>();
    HIPCHK(hipMemsetAsync(len + W, 0, 8, h->s));
    launch_walk_lengths(h->walks.as<uint32_t>(), W, h->L, (uint32_t)v0, (uint32_t)v1, len, h->s);
    h->rp([&](void* t, size_t& b) {
        return rocprim::exclusive_scan(t, b, len, base, (uint64_t)0, (size_t)(W + 1), rocprim::plus<uint64_t>(), h->s);
    });
    uint64_t E = 0;
    HIPCHK(hipMemcpyAsync(&E, base + W, 8, hipMemcpyDeviceToHost, h->s));
    h->sync();
    if (!E) return 0;
    h->k1.ensure(E * 8);
    h->k2.ensure(E * 8);
    h->flags.ensure(E * 4);
    h->pairs.ensure(E * 4);
    launch_index_entries(h->walks.as<uint32_t>(), W, h->L, h->smap(), kb, (uint32_t)v0, (uint32_t)v1, base,
                         h->k1.as<uint64_t>(), h->flags.as<uint32_t>(), h->s);
    uint64_t* ki = h->k1.as<uint64_t>();
    uint64_t* ko = h->k2.as<uint64_t>();
    uint32_t* vi = h->flags.as<uint32_t>();
    uint32_t* vo = h->pairs.as<uint32_t>();
    const unsigned eb = (unsigned)(kb + vb);
    h->rp([&](void* t, size_t& b) { return rocprim::radix_sort_pairs(t, b, ki, ko, vi, vo, (size_t)E, 0u, eb, h->s); });
    return E;
}

int index_size(wharf_handle* h, uint64_t v0, uint64_t v1, uint64_t* size)
{
    return guarded(h, [&] {
        REQUIRE(h && size, WHARF_E_INVALID, "null argument");
        REQUIRE(v0 <= v1 && v1 <= h->n, WHARF_E_INVALID, "vertex window out of range");
        h->ensure_walks();
        h->sel.ensure((h->W + 1) * 8);
        h->count.ensure((h->W + 1) * 8);
        uint64_t* len = h->sel.as<uint64_t>();
        uint64_t* base = h->count.as<uint64_t>();
        HIPCHK(hipMemsetAsync(len + h->W, 0, 8, h->s));
        launch_walk_lengths(h->walks.as<uint32_t>(), h->W, h->L, (uint32_t)v0, (uint32_t)v1, len, h->s);
        h->rp([&](void* t, size_t& b) {
            return rocprim::exclusive_scan(t, b, len, base, (uint64_t)0, (size_t)(h->W + 1), rocprim::plus<uint64_t>(), h->s);
        });
        HIPCHK(hipMemcpyAsync(size, base + h->W, 8, hipMemcpyDeviceToHost, h->s));
        h->sync();
    });
}

int export_index(wharf_handle* h, uint64_t v0, uint64_t v1, uint64_t* counts, uint64_t* keys, uint32_t* nexts)
{
    return guarded(h, [&] {
        REQUIRE(h && counts, WHARF_E_INVALID, "null argument");
        REQUIRE(v0 <= v1 && v1 <= h->n, WHARF_E_INVALID, "vertex window out of range");
        const uint64_t nv = v1 - v0;
        int kb = 0;
        const uint64_t E = nv ? build_index(h, kb, v0, v1) : 0;
        h->runs.ensure(std::max<uint64_t>(nv, 1) * 8);
        HIPCHK(hipMemsetAsync(h->runs.p, 0, std::max<uint64_t>(nv, 1) * 8, h->s));
        if (E) {
            REQUIRE(keys && nexts, WHARF_E_INVALID, "null argument");
            // k2 holds sorted ((vertex - v0) << kb | key); split into counts and keys (reuse k1)
            launch_index_split(h->k2.as<uint64_t>(), E, kb, h->runs.as<unsigned long long>(), h->k1.as<uint64_t>(), h->s);
            HIPCHK(hipMemcpyAsync(keys, h->k1.p, E * 8, hipMemcpyDeviceToHost, h->s));
            HIPCHK(hipMemcpyAsync(nexts, h->pairs.p, E * 4, hipMemcpyDeviceToHost, h->s));
        }
        if (nv) HIPCHK(hipMemcpyAsync(counts, h->runs.p, nv * 8, hipMemcpyDeviceToHost, h->s));
        h->sync();
    });
}
}  // namespace

int wharf_index_size(wharf_handle* h, uint64_t* size) { return index_size(h, 0, h ? h->n : 0, size); }

int wharf_index_size_range(wharf_handle* h, uint64_t v0, uint64_t v1, uint64_t* size)
{
    return index_size(h, v0, v1, size);
}

int wharf_export_index(wharf_handle* h, uint64_t* counts, uint64_t* keys, uint32_t* nexts)
{
    return export_index(h, 0, h ? h->n : 0, counts, keys, nexts);
}

int wharf_export_index_range(wharf_handle* h, uint64_t v0, uint64_t v1, uint64_t* counts, uint64_t* keys,
                             uint32_t* nexts)
{
    return export_index(h, v0, v1, counts, keys, nexts);
}

int wharf_export_index_paired(wharf_handle* h, uint64_t* counts, uint64_t* paired)
{
    return guarded(h, [&] {
        REQUIRE(h && counts, WHARF_E_INVALID, "null argument");
        int kb = 0;
        const uint64_t E = build_index(h, kb, 0, h->n);
        const uint64_t n = h->n;
        h->runs.ensure(n * 8);
        HIPCHK(hipMemsetAsync(h->runs.p, 0, n * 8, h->s));
        if (E) {
            REQUIRE(paired, WHARF_E_INVALID, "null argument");
            uint64_t* keys = h->k1.as<uint64_t>();
            uint64_t* z = h->k2.as<uint64_t>();
            launch_index_split(h->k2.as<uint64_t>(), E, kb, h->runs.as<unsigned long long>(), keys, h->s);
            launch_index_pair(keys, h->pairs.as<uint32_t>(), E, z, h->s);
            // per-vertex offsets, then each vertex's entries ascending (the C-tree
            // iteration order), in chunks of < 2^31 entries for rocPRIM's 32-bit sizes
            h->sel.ensure((n + 1) * 8);
            uint64_t* off = h->sel.as<uint64_t>();
            h->count.ensure((n + 1) * 8);
            uint64_t* cnt = h->count.as<uint64_t>();
            HIPCHK(hipMemcpyAsync(cnt, h->runs.p, n * 8, hipMemcpyDeviceToDevice, h->s));
            HIPCHK(hipMemsetAsync(cnt + n, 0, 8, h->s));
            h->rp([&](void* t, size_t& b) {
                return rocprim::exclusive_scan(t, b, cnt, off, (uint64_t)0, (size_t)(n + 1), rocprim::plus<uint64_t>(), h->s);
            });
            std::vector<uint64_t> hoff(n + 1);
            HIPCHK(hipMemcpyAsync(hoff.data(), off, (n + 1) * 8, hipMemcpyDeviceToHost, h->s));
            h->sync();
            const uint64_t kChunk = 1ull << 30;
            h->flags.ensure((n + 1) * 4);
            uint32_t* rel = h->flags.as<uint32_t>();
            for (uint64_t v0 = 0; v0 < n;) {
                uint64_t v1 = v0 + 1;   // at least one vertex per chunk
                uint64_t lo = v0 + 1, hi = n;
                while (lo <= hi) {   // largest v1 with hoff[v1] - hoff[v0] <= kChunk
                    const uint64_t mid = lo + (hi - lo) / 2;
                    if (hoff[mid] - hoff[v0] <= kChunk) { v1 = mid; lo = mid + 1; } else { hi = mid - 1; }
                }
                const uint64_t base = hoff[v0], size = hoff[v1] - base, segs = v1 - v0;
                REQUIRE(size < (1ull << 32), WHARF_E_INVALID, "a vertex holds >= 2^32 index entries");
                if (size) {
                    launch_rel_offsets(off, v0, segs, rel, h->s);
                    uint64_t* kin = z + base;
                    uint64_t* kout = keys + base;
                    h->rp([&](void* t, size_t& b) {
                        return rocprim::segmented_radix_sort_keys(t, b, kin, kout, (unsigned)size, (unsigned)segs, rel,
                                                                  rel + 1, 0u, 64u, h->s);
                    });
                }
                v0 = v1;
            }
            HIPCHK(hipMemcpyAsync(paired, keys, E * 8, hipMemcpyDeviceToHost, h->s));
        }
        HIPCHK(hipMemcpyAsync(counts, h->runs.p, n * 8, hipMemcpyDeviceToHost, h->s));
        h->sync();
    });
}

int wharf_memory_footprint(const wharf_handle* h, wharf_memory* out)
{
    if (!h || !out) return WHARF_E_INVALID;
    wharf_memory r{};
    r.n = h->n;
    r.m = h->m;
    r.csr_bytes = h->off.cap + h->adj.cap + h->deg.cap + h->cap.cap + h->rev.cap;
    r.records_bytes = h->vrec.cap + h->erec.cap;
    r.walks_bytes = h->walks.cap + h->aff.cap;
    const uint64_t anchor_part = h->anchors ? h->erec.cap / 2 : 0;   // bytes 16-31 of the 32-B records
    r.records_bytes -= anchor_part;
    r.samplers_bytes = anchor_part + h->row_epoch.cap;
    r.edge_hash_bytes = h->ehash.cap + h->fdir.cap + h->fpool.cap;
    r.update_buffers_bytes = h->off2.cap + h->adj2.cap + h->erec2.cap + h->scratch.cap + h->rplan.cap + h->pscan.cap +
                             h->sanc.cap + h->srev.cap;   // the anchor carry's / reverse index's saved entries
    r.scratch_bytes = h->tmp.cap + h->k1.cap + h->k2.cap + h->flags.cap + h->chg.cap + h->cf.cap + h->runstart.cap +
                      h->runs.cap + h->fplan.cap + h->memo.cap + h->srcidx.cap + h->count.cap + h->pairs.cap +
                      h->sel.cap + h->defer.cap + h->park.cap + h->parkc.cap + h->stab.cap + h->preoff.cap + h->rtab.cap + h->bitmap.cap + h->counters.cap +
                      h->errflag.cap + h->bdesc.cap + h->rchunk.cap;
    r.total_bytes = r.csr_bytes + r.records_bytes + r.walks_bytes + r.samplers_bytes + r.edge_hash_bytes +
                    r.update_buffers_bytes + r.scratch_bytes;
    *out = r;
    return WHARF_OK;
}

int wharf_get_stats(const wharf_handle* h, wharf_stats* out)
{
    if (!h || !out) return WHARF_E_INVALID;
    *out = h->st;
    out->n = h->n;
    out->m = h->m;
    out->walks = h->W;
    out->hbm_bytes_walks = h->W * h->L * 4;
    out->hbm_bytes_graph = (h->n + 1) * 8 + h->n * 8 + h->pool_cap * 4 + h->n * sizeof(ERec) +
                           wharf_handle::rec_bytes(h->rf, h->pool_cap, h->rec_stride());
    out->pool_slots = h->pool_used;
    out->pool_capacity = h->pool_cap;
    out->last_moved_row_slots = h->grown;
    out->repacks = h->repacks;
    out->dead_slots = h->dead_slots;
    return WHARF_OK;
}

int wharf_generate_batch_of_edges(int device, uint64_t edges_number, uint64_t vertices_number, uint64_t batch_seed,
                                  int self_loops, int directed, double a, double b, double c, uint32_t* out_pairs,
                                  uint64_t* count)
{
    wharf_config cfg;
    wharf_config_default(&cfg);
    wharf_handle* h = nullptr;
    int rc = guarded(nullptr, [&] {
        REQUIRE(out_pairs && count, WHARF_E_INVALID, "null argument");
        // a scratch handle on a single vertex (no walks) to own the stream and buffers
        cfg.walks_per_vertex = 1;
        cfg.walk_length = 2;
        h = new_handle(&cfg, 1, device);
        rmat_keys(h, edges_number, vertices_number, batch_seed, directed, a, b, c);
        const uint64_t total = directed ? edges_number : 2 * edges_number;
        const uint32_t nb = bits_for(vertices_number);
        const uint64_t k = h->unique_keys(total, !self_loops, 32 + std::max<uint32_t>(nb, 1));
        std::vector<uint64_t> keys(k);
        if (k) HIPCHK(hipMemcpy(keys.data(), h->k1.p, k * 8, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < k; i++) {
            out_pairs[2 * i] = (uint32_t)(keys[i] >> 32);
            out_pairs[2 * i + 1] = (uint32_t)keys[i];
        }
        *count = k;
    });
    free_handle(h);
    return rc;
}

int wharf_szudzik64(int device, int op, uint64_t count, uint64_t* x, uint64_t* y, uint64_t* z)
{
    return guarded(nullptr, [&] {
        REQUIRE(x && y && z && (op == 0 || op == 1), WHARF_E_INVALID, "bad argument");
        HIPCHK(hipSetDevice(device));
        if (!count) return;
        uint64_t* d = nullptr;
        HIPCHK(hipMalloc(&d, count * 24));
        try {
            HIPCHK(hipMemcpy(d, x, count * 8, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(d + count, y, count * 8, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(d + 2 * count, z, count * 8, hipMemcpyHostToDevice));
            launch_szudzik64(op, count, d, d + count, d + 2 * count, 0);
            HIPCHK(hipDeviceSynchronize());
            HIPCHK(hipMemcpy(x, d, count * 8, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(y, d + count, count * 8, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(z, d + 2 * count, count * 8, hipMemcpyDeviceToHost));
        } catch (...) {
            (void)hipFree(d);
            throw;
        }
        HIPCHK(hipFree(d));
    });
}

}  // extern "C"
