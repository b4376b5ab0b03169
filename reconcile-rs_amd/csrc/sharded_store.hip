// sharded_store.hip -- rh_sstore: one replica's map over several GPUs (include/rsos_hip.h).
//
// The north_star shards records by key range across the GPUs of one node.  A
// replica is one process holding one map (Inner<K, V>, /root/reference/src/replica.rs:68-74), so
// the in-process form of that partitioning is a list of column stores (rh_store), one per device,
// each owning a contiguous key range: shard s holds the keys in [split[s - 1], split[s]).  Every
// question of the Rsos<K> surface (rsos/src/rsos_trait.rs:39-90) and of a protocol round
// (rbsr/src/protocol.rs:212-317) decomposes over that partition with no device-to-device traffic:
//   - size, rank(z): sums -- rank(z) = (rows of the shards below z's) + rank in z's shard;
//   - aggregate(range): Aggregate's Add (rsos/src/aggregate.rs:79-89) of the shards' parts: the
//     shards wholly inside the range give their cached roots, at most two boundary shards are asked;
//   - select(r): the shard whose rank interval holds r;
//   - insert / delete: each row routed to its key's shard by the splitters;
//   - a protocol round: a run of segments inside one shard's key range is that shard's own round
//     (a segment's decisions, cut ranks and children depend on ranks only through differences
//     inside the segment, so the shard answers exactly what the whole map would); a segment that
//     straddles a boundary (at most one per boundary per round, the segments being key-ordered) is
//     resolved from its two boundary shards, decided on the host (round_decide.hpp) and cut by
//     selects and rank-range aggregates routed to the shards that hold them.
// Shards are driven concurrently by host threads (one per shard; each store has its own stream and
// lock), so per-shard device work overlaps.  Only the public rh_store_* entry points are used.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <numeric>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rsos_hip.h"
#include "internal.hpp"
#include "round_decide.hpp"

namespace rh {
int set_error(int code, const std::string &msg);  // rsos_hip_abi.hip: the calling thread's rh_last_error
bool debug_fail_point(const char *name);          // rh_debug_fail_point, armed on the calling thread
// rh_store_protocol_round in two halves (rsos_hip_abi.hip round_entry): a device round issued
// (*pending: the store stays locked) and completed later on the same thread
int store_round_issue(rh_store *s, int policy, uint64_t fan_out, const rh_segments *active, rh_segments *children,
                      rh_segments *enumerations, rh_round_outcome *outcome, bool *pending);
int store_round_complete(rh_store *s, rh_segments *children, rh_segments *enumerations, rh_round_outcome *outcome);
}

namespace {

// Runs one task per shard concurrently: the first on the calling thread, the others on the shards'
// own worker threads (which spin briefly, then sleep, between calls: a host-tier question is
// microseconds, a device one tens of microseconds).
class ShardPool {
  public:
    explicit ShardPool(int n) : slots_(n) {
        for (int i = 1; i < n; i++) slots_[i].th = std::thread([this, i] { loop(i); });
    }
    ~ShardPool() {
        for (size_t i = 1; i < slots_.size(); i++) {
            Slot &w = slots_[i];
            {
                std::lock_guard<std::mutex> g(w.mu);
                w.quit = true;
                w.state.store(1, std::memory_order_release);
            }
            w.cv.notify_one();
            w.th.join();
        }
    }
    // fn(s) for every shard s in `idx` (distinct, ascending); returns when all have finished.  An
    // exception thrown by fn -- on the calling thread or a worker -- is rethrown here, and only
    // after every posted task has finished (the tasks read the caller's stack).
    void run(const std::vector<int> &idx, const std::function<void(int)> &fn) {
        if (idx.empty()) return;
        if (idx.size() == 1) {
            fn(idx[0]);
            return;
        }
        for (size_t k = 1; k < idx.size(); k++) {
            Slot &w = slots_[idx[k]];
            {
                std::lock_guard<std::mutex> g(w.mu);
                w.fn = &fn;
                w.err = nullptr;
                w.state.store(1, std::memory_order_release);
            }
            w.cv.notify_one();
        }
        std::exception_ptr err;
        try {
            fn(idx[0]);
        } catch (...) {
            err = std::current_exception();
        }
        for (size_t k = 1; k < idx.size(); k++) {
            Slot &w = slots_[idx[k]];
            wait_for(w, 2);
            w.state.store(0, std::memory_order_relaxed);
            if (w.err && !err) err = w.err;
        }
        if (err) std::rethrow_exception(err);
    }

  private:
    struct Slot {
        std::thread th;
        std::mutex mu;
        std::condition_variable cv;
        std::atomic<int> state{0};  // 0 idle, 1 task posted, 2 done
        const std::function<void(int)> *fn = nullptr;
        std::exception_ptr err;  // what the task threw, handed back to run()
        bool quit = false;
    };
    std::vector<Slot> slots_;
    // spin this long before sleeping (RSOS_HIP_SSTORE_SPIN_US, default 50)
    static int64_t spin_us() {
        static const int64_t us = getenv("RSOS_HIP_SSTORE_SPIN_US") ? atoll(getenv("RSOS_HIP_SSTORE_SPIN_US")) : 50;
        return us;
    }
    static void wait_for(Slot &w, int want) {
        const auto t0 = std::chrono::steady_clock::now();
        while (w.state.load(std::memory_order_acquire) != want) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us())) {
                std::unique_lock<std::mutex> g(w.mu);
                w.cv.wait(g, [&] { return w.state.load(std::memory_order_acquire) == want; });
                return;
            }
        }
    }
    void loop(int i) {
        Slot &w = slots_[i];
        for (;;) {
            wait_for(w, 1);
            if (w.quit) return;
            try {
                (*w.fn)(i);
            } catch (...) {
                w.err = std::current_exception();
            }
            {
                std::lock_guard<std::mutex> g(w.mu);
                w.state.store(2, std::memory_order_release);
            }
            w.cv.notify_all();
        }
    }
};

int fail(int code, const std::string &msg) { return rh::set_error(code, msg); }

// a shard call's status, with its message (rh_last_error is per thread)
struct Status {
    int rc = RH_OK;
    std::string msg;
    void take(int r) {
        if (r != RH_OK && rc == RH_OK) {
            rc = r;
            const char *m = rh_last_error();
            msg = m ? m : "";
        }
    }
};

// the status of a task that threw (no exception crosses the C ABI)
void caught(Status &st) {
    try {
        throw;
    } catch (const std::bad_alloc &) {
        st.rc = RH_ERR_OOM;
        st.msg = "sharded store: host allocation failed";
    } catch (const std::exception &e) {
        st.rc = RH_ERR_STATE;
        st.msg = std::string("sharded store: internal error: ") + e.what();
    } catch (...) {
        st.rc = RH_ERR_STATE;
        st.msg = "sharded store: internal error";
    }
}

int key_row(const rh_schema &s) {
    switch (s.key_kind) {
    case RH_KEY_UNIT: return 0;
    case RH_KEY_U32: return 4;
    case RH_KEY_U64: return 8;
    default: return (int)s.key_len;
    }
}
int value_row(const rh_schema &s) {
    switch (s.value_kind) {
    case RH_VAL_UNIT: return 0;
    case RH_VAL_U32: return 4;
    case RH_VAL_U64: return 8;
    default: return (int)s.value_len;
    }
}

const rh_aggregate kZero{{0, 0, 0, 0}, 0};
void agg_add(rh_aggregate &a, const rh_aggregate &b) {
    rh_fp_add(a.fingerprint, b.fingerprint, a.fingerprint);
    a.size += b.size;
}

}  // namespace

struct rh_sstore {
    rh_schema schema{};
    int G = 0;
    size_t kl = 0;
    std::vector<rh_store *> shards;
    std::vector<uint8_t> split;     // G - 1 keys: shard s holds [split[s - 1], split[s])
    std::vector<uint64_t> sizes;    // rows per shard (valid while sizes_ok)
    std::vector<uint64_t> off;      // G + 1 prefix sums of sizes
    bool sizes_ok = false;
    // each shard's root (the aggregate of its whole key range), cached until the next write: a
    // key range spanning shards adds the roots of the shards inside it
    std::vector<rh_aggregate> roots;
    std::vector<uint8_t> root_ok;
    bool tier_on = false;  // the shards' host tiers (rh_sstore_set_host_tier): their questions are
                           // microseconds, asked on the calling thread
    uint64_t round_max = 128;  // ... and rounds of up to this many segments per shard go to them
    void changed() {
        sizes_ok = false;
        std::fill(root_ok.begin(), root_ok.end(), 0);
    }
    int root(int t, rh_aggregate *out) {
        if (!root_ok[t]) {
            if (int rc = rh_store_aggregate_keys(shards[t], 0, nullptr, 0, nullptr, &roots[t])) return rc;
            root_ok[t] = 1;
        }
        *out = roots[t];
        return RH_OK;
    }
    std::vector<uint8_t> dirty;     // shard has staged rows not yet applied
    std::mutex mu;                  // one call at a time: every answer is one snapshot of every shard
    ShardPool *pool = nullptr;
    // Set when a write failed after some shards had committed their part (a device or allocation
    // failure past the batch's checks): the shards then disagree with any one-store history, so
    // every call but a load (which replaces the contents) and destroy is refused until a load.
    std::string broken;
    int health() const {
        return broken.empty() ? RH_OK : rh::set_error(RH_ERR_STATE, "sharded store: " + broken + "; load to recover");
    }

    // ---- key order (the key type's Ord: numeric for u32 / u64 keys stored LE, bytewise else) ----
    int cmp(const uint8_t *a, const uint8_t *b) const {
        switch (schema.key_kind) {
        case RH_KEY_U64: {
            uint64_t x, y;
            memcpy(&x, a, 8);
            memcpy(&y, b, 8);
            return (x > y) - (x < y);
        }
        case RH_KEY_U32: {
            uint32_t x, y;
            memcpy(&x, a, 4);
            memcpy(&y, b, 4);
            return (x > y) - (x < y);
        }
        default: return kl ? memcmp(a, b, kl) : 0;
        }
    }
    const uint8_t *splitter(int j) const { return split.data() + (size_t)j * kl; }
    // the shard holding key z: the number of splitters <= z (bisect_right)
    int owner(const uint8_t *z) const {
        int lo = 0, hi = G - 1;
        while (lo < hi) {
            const int mid = (lo + hi) / 2;
            if (cmp(splitter(mid), z) <= 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    // the last shard that can hold a key below z: the number of splitters < z (bisect_left)
    int owner_below(const uint8_t *z) const {
        int lo = 0, hi = G - 1;
        while (lo < hi) {
            const int mid = (lo + hi) / 2;
            if (cmp(splitter(mid), z) < 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    // Until the first load, the key space is cut evenly: u32 / u64 keys at multiples of 2^32 / G
    // and 2^64 / G, byte keys by their leading 8 bytes read big-endian (their order), so that a map
    // filled by single inserts (just_insert_bulk, src/replica/write.rs:107-121) spreads over the
    // shards; a load re-cuts at equal counts.
    void even_splitters() {
        split.assign((size_t)(G - 1) * kl, 0);
        for (int j = 1; j < G; j++) {
            const unsigned __int128 v = ((unsigned __int128)1 << 64) * (unsigned)j / (unsigned)G;
            uint8_t *k = split.data() + (size_t)(j - 1) * kl;
            if (schema.key_kind == RH_KEY_U32) {
                const uint32_t x = (uint32_t)(v >> 32);
                memcpy(k, &x, 4);
            } else if (schema.key_kind == RH_KEY_U64) {
                const uint64_t x = (uint64_t)v;
                memcpy(k, &x, 8);
            } else {
                for (size_t b = 0; b < kl && b < 8; b++) k[b] = (uint8_t)((uint64_t)v >> (56 - 8 * b));
            }
        }
    }

    // ---- sizes (every read flushes the shards' staged rows first, concurrently) ----------------
    Status flush() {
        Status st;
        if (sizes_ok) return st;
        std::vector<uint64_t> got(G, 0);
        std::vector<Status> ss(G);
        std::vector<int> busy, idle;
        for (int s = 0; s < G; s++) (dirty[s] ? busy : idle).push_back(s);
        auto len = [&](int s) {
            try {
                ss[s].take(rh_store_len(shards[s], &got[s]));
            } catch (...) {
                caught(ss[s]);
            }
        };
        pool->run(busy, len);
        for (int s : idle) len(s);
        for (int s = 0; s < G; s++)
            if (ss[s].rc) {
                st.rc = ss[s].rc;
                st.msg = ss[s].msg;
                return st;
            }
        sizes = got;
        off.assign(G + 1, 0);
        for (int s = 0; s < G; s++) off[s + 1] = off[s] + sizes[s];
        std::fill(dirty.begin(), dirty.end(), 0);
        sizes_ok = true;
        return st;
    }
    uint64_t total() const { return off[G]; }
    // the shard holding global rank r (< total()): the last shard whose first rank is <= r
    int shard_of_rank(uint64_t r) const {
        return (int)(std::upper_bound(off.begin() + 1, off.begin() + G, r) - (off.begin() + 1));
    }
    // Shards on one device: their calls from concurrent threads contend for that device's queues
    // and the runtime's locks, while one thread issuing every shard's device work in turn serialises
    // the host side of it.  Measured with 4 and 8 shards on one GPU (profiles/r06_sstore_group_ab*:
    // 1 / 2 / 4 / 8 shards per thread, three boxes): at most 4 threads per device is best at both, so
    // a thread takes ceil(shards on its device / 4) of them.  RSOS_HIP_SSTORE_GROUP=<k>: k per thread.
    std::vector<int> dev;  // each shard's device
    bool shared_devices = false;
    static constexpr int THREADS_PER_DEVICE = 4;
    static int group_env() {
        static const int k = [] {
            const char *e = getenv("RSOS_HIP_SSTORE_GROUP");
            const int v = e ? atoi(e) : 0;
            return e ? (v < 1 ? 1 : v) : 0;  // 0: automatic
        }();
        return k;
    }
    int group_size(int device) const {
        if (group_env()) return group_env();
        const int on = (int)std::count(dev.begin(), dev.end(), device);
        return std::max(1, (on + THREADS_PER_DEVICE - 1) / THREADS_PER_DEVICE);
    }
    // the shards of idx in groups: a group is up to group_size() shards of one device, in idx order
    // (every shard its own group with group = false or when no device holds two); lead[i] names
    // group i by its first shard, grp[lead[i]] its members
    void grouping(const std::vector<int> &idx, bool group, std::vector<int> &lead,
                  std::vector<std::vector<int>> &grp) const {
        lead.clear();
        grp.assign(G, {});
        for (int s : idx) {
            const int k = group && shared_devices ? group_size(dev[s]) : 1;
            int l = -1;
            for (int t : lead)
                if (dev[t] == dev[s] && (int)grp[t].size() < k) l = t;
            if (l < 0) lead.push_back(l = s);
            grp[l].push_back(s);
        }
    }
    // run fn over shards concurrently and collect the first error (with its message).  group =
    // false: one thread per shard even on a shared device (host-only work: the host tiers'
    // answers, copies)
    int each(const std::vector<int> &idx, const std::function<int(int)> &fn, bool group = true) {
        std::vector<Status> ss(G);
        auto one = [&](int s) {
            try {
                ss[s].take(fn(s));
            } catch (...) {
                caught(ss[s]);
            }
        };
        std::vector<int> lead;
        std::vector<std::vector<int>> grp;
        grouping(idx, group, lead, grp);
        pool->run(lead, [&](int l) {
            for (int s : grp[l]) one(s);
        });
        for (int s : idx)
            if (ss[s].rc) return fail(ss[s].rc, ss[s].msg);
        return RH_OK;
    }
    // fn(group) per group of shards (grouping): a device's shards together, the groups concurrently
    int each_device(const std::vector<int> &idx, const std::function<int(const std::vector<int> &)> &fn,
                    bool group = true) {
        std::vector<int> lead;
        std::vector<std::vector<int>> grp;
        grouping(idx, group, lead, grp);
        return each(lead, [&](int l) { return fn(grp[l]); }, false);
    }
    std::vector<int> all() const {
        std::vector<int> v(G);
        for (int s = 0; s < G; s++) v[s] = s;
        return v;
    }

    // ---- rows routed to their shards ---------------------------------------------------------
    // per-shard copies of m host rows: rows[s] lists the input rows shard s takes, in input order
    struct Part {
        std::vector<uint8_t> keys, vals, tags, ops;
        std::vector<uint64_t> phys, node;
        std::vector<uint32_t> logical;
        size_t m = 0;
        rh_columns cols() const {
            auto p = [](const auto &v) { return v.empty() ? nullptr : v.data(); };
            return rh_columns{p(keys), reinterpret_cast<const uint64_t *>(p(phys)),
                              reinterpret_cast<const uint32_t *>(p(logical)),
                              reinterpret_cast<const uint64_t *>(p(node)), p(tags), p(vals)};
        }
    };
    void route(const uint8_t *keys, size_t m, std::vector<std::vector<uint32_t>> &rows) const {
        rows.assign(G, {});
        for (size_t i = 0; i < m; i++) rows[owner(keys + i * kl)].push_back((uint32_t)i);
    }
    void gather(const rh_columns &h, const uint8_t *ops, const std::vector<uint32_t> &rows, Part &p) const {
        const size_t m = rows.size(), vr = value_row(schema);
        const bool dated = schema.record_kind == RH_REC_DATED;
        p.m = m;
        auto pick = [&](auto &dst, const auto *src, size_t w) {
            using T = std::remove_cv_t<std::remove_pointer_t<decltype(src)>>;
            if (!src) return;
            dst.resize(m * w);
            for (size_t i = 0; i < m; i++) memcpy(&dst[i * w], reinterpret_cast<const T *>(src) + (size_t)rows[i] * w, w * sizeof(T));
        };
        pick(p.keys, static_cast<const uint8_t *>(h.keys), kl);
        pick(p.vals, static_cast<const uint8_t *>(h.values), vr);
        if (schema.record_kind != RH_REC_PLAIN) pick(p.tags, h.tags, 1);
        if (dated) {
            pick(p.phys, h.phys, 1);
            pick(p.node, h.node, 1);
            pick(p.logical, h.logical, 1);
        }
        pick(p.ops, ops, 1);
    }
    // whether m key rows hold a repeated key (strictly increasing input answers in one pass)
    bool has_duplicates(const uint8_t *keys, size_t m) const {
        bool sorted = true;
        for (size_t i = 1; i < m && sorted; i++) sorted = cmp(keys + (i - 1) * kl, keys + i * kl) < 0;
        if (sorted) return false;
        std::vector<uint32_t> ix(m);
        for (size_t i = 0; i < m; i++) ix[i] = (uint32_t)i;
        std::sort(ix.begin(), ix.end(), [&](uint32_t a, uint32_t b) { return cmp(keys + a * kl, keys + b * kl) < 0; });
        for (size_t i = 1; i < m; i++)
            if (cmp(keys + ix[i - 1] * kl, keys + ix[i] * kl) == 0) return true;
        return false;
    }

    // ---- rank-range pieces ------------------------------------------------------------------
    // the part of global rank range [lo, hi) in shard s, as shard-local ranks (empty: l == h)
    void piece(int s, uint64_t lo, uint64_t hi, uint64_t *l, uint64_t *h) const {
        const uint64_t a = std::clamp(lo, off[s], off[s + 1]), b = std::clamp(hi, off[s], off[s + 1]);
        *l = a - off[s];
        *h = std::max(a, b) - off[s];
    }
    // aggregates of q global rank ranges (clamped; inverted = ZERO), and m selects, in one call per
    // shard holding any of them (rh_store_split_segments)
    int split_ranks(size_t m, const uint64_t *sel, uint8_t *keys_out, size_t q, const uint64_t *lo,
                    const uint64_t *hi, rh_aggregate *out) {
        struct Job {
            std::vector<uint64_t> sel, lo, hi;
            std::vector<size_t> sel_at, agg_at;
            std::vector<uint8_t> keys;
            std::vector<rh_aggregate> aggs;
        };
        std::vector<Job> jobs(G);
        const uint64_t n = total();
        for (size_t i = 0; i < m; i++) {
            if (sel[i] >= n) return fail(RH_ERR_ARG, "select: rank out of range (r >= size)");
            const int s = shard_of_rank(sel[i]);
            jobs[s].sel.push_back(sel[i] - off[s]);
            jobs[s].sel_at.push_back(i);
        }
        for (size_t j = 0; j < q; j++) {
            out[j] = kZero;
            const uint64_t h = std::min(hi[j], n), l = std::min(lo[j], h);
            if (l == h) continue;
            for (int s = shard_of_rank(l); s < G && off[s] < h; s++) {
                uint64_t a, b;
                piece(s, l, h, &a, &b);
                if (a == b) continue;
                jobs[s].lo.push_back(a);
                jobs[s].hi.push_back(b);
                jobs[s].agg_at.push_back(j);
            }
        }
        std::vector<int> idx;
        for (int s = 0; s < G; s++)
            if (!jobs[s].sel.empty() || !jobs[s].lo.empty()) idx.push_back(s);
        int rc = each(idx, [&](int s) -> int {
            Job &J = jobs[s];
            J.keys.resize(J.sel.size() * kl + 1);
            J.aggs.resize(J.lo.size() + 1);
            return rh_store_split_segments(shards[s], J.sel.size(), J.sel.data(), J.keys.data(), J.lo.size(),
                                           J.lo.data(), J.hi.data(), J.aggs.data());
        });
        if (rc) return rc;
        for (int s : idx) {
            const Job &J = jobs[s];
            for (size_t i = 0; i < J.sel.size(); i++) memcpy(keys_out + J.sel_at[i] * kl, J.keys.data() + i * kl, kl);
            for (size_t i = 0; i < J.lo.size(); i++) agg_add(out[J.agg_at[i]], J.aggs[i]);
        }
        return RH_OK;
    }

    // ---- segments resolved over the shards ----------------------------------------------------
    // Segment j's keys lie in shards [a_j, b_j]: a_j holds its start bound (0 when unbounded), b_j
    // the keys just below its end bound (G - 1 when unbounded).  Its raw ranks come from those two
    // shards alone; its local aggregate adds the roots of the shards between them.  a_j > b_j is an
    // empty or inverted segment: its ranks still come from a_j and b_j, its aggregate is ZERO.
    void span(const uint8_t sk, const uint8_t *skey, const uint8_t ek, const uint8_t *ekey, int *a, int *b) const {
        *a = sk ? owner(skey) : 0;
        *b = ek ? owner_below(ekey) : G - 1;
    }
    int resolve_list(const std::vector<size_t> &J, const uint8_t *sk, const uint8_t *skeys, const uint8_t *ek,
                     const uint8_t *ekeys, uint64_t *raw_lo, uint64_t *raw_hi, rh_aggregate *local) {
        struct Job {
            std::vector<uint8_t> sk, ek, skeys, ekeys;
            std::vector<size_t> at;
            std::vector<uint8_t> side;  // 1: the start side, 2: the end side, 3: both
            std::vector<uint64_t> lo, hi;
            std::vector<rh_aggregate> aggs;
        };
        std::vector<Job> jobs(G);
        std::vector<int> A(J.size()), B(J.size());
        auto add = [&](int s, size_t t, int side) {
            const size_t j = J[t];
            Job &q = jobs[s];
            const bool st = side & 1, en = side & 2;
            q.sk.push_back(st ? sk[j] : 0);
            q.ek.push_back(en ? ek[j] : 0);
            const size_t o = q.skeys.size();
            q.skeys.resize(o + kl, 0);
            q.ekeys.resize(o + kl, 0);
            if (st && sk[j]) memcpy(q.skeys.data() + o, skeys + j * kl, kl);
            if (en && ek[j]) memcpy(q.ekeys.data() + o, ekeys + j * kl, kl);
            q.at.push_back(t);
            q.side.push_back((uint8_t)side);
        };
        for (size_t t = 0; t < J.size(); t++) {
            const size_t j = J[t];
            span(sk[j], sk[j] ? skeys + j * kl : nullptr, ek[j], ek[j] ? ekeys + j * kl : nullptr, &A[t], &B[t]);
            if (A[t] == B[t]) add(A[t], t, 3);
            else add(A[t], t, 1), add(B[t], t, 2);
        }
        std::vector<int> idx;
        for (int s = 0; s < G; s++)
            if (!jobs[s].at.empty()) idx.push_back(s);
        int rc = each(idx, [&](int s) -> int {
            Job &q = jobs[s];
            const size_t r = q.at.size();
            q.lo.resize(r), q.hi.resize(r), q.aggs.resize(r);
            return rh_store_resolve_segments(shards[s], r, q.sk.data(), q.skeys.data(), q.ek.data(), q.ekeys.data(),
                                             q.lo.data(), q.hi.data(), q.aggs.data());
        });
        if (rc) return rc;
        // the roots of the shards between a segment's two boundary shards
        std::vector<rh_aggregate> mid(G, kZero);
        for (size_t t = 0; t < J.size(); t++) {
            local[t] = kZero;
            for (int s = A[t] + 1; s < B[t]; s++)
                if ((rc = root(s, &mid[s]))) return rc;
        }
        for (int s : idx) {
            const Job &q = jobs[s];
            for (size_t i = 0; i < q.at.size(); i++) {
                const size_t t = q.at[i];
                if (q.side[i] & 1) raw_lo[t] = off[s] + q.lo[i];
                if (q.side[i] & 2) raw_hi[t] = off[s] + q.hi[i];
                if (A[t] <= B[t]) agg_add(local[t], q.aggs[i]);
            }
        }
        for (size_t t = 0; t < J.size(); t++)
            for (int s = A[t] + 1; s < B[t]; s++) agg_add(local[t], mid[s]);
        return RH_OK;
    }

    // ---- a protocol round --------------------------------------------------------------------
    // One piece of the round's output: the children and enumerations of a run of segments, either
    // owned (copied) or borrowed from a shard's own round output (valid until that shard's next call)
    struct Out {
        std::vector<uint8_t> csk, cek, cskeys, cekeys, esk, eek, eskeys, eekeys;
        std::vector<rh_aggregate> caggs;
        uint64_t cnt[5] = {0, 0, 0, 0, 0};  // skipped, enumerated, split, children, dropped
        bool borrowed = false;
        rh_segments bc{}, be{};
        void child(uint8_t s, const uint8_t *sk, uint8_t e, const uint8_t *ek, const rh_aggregate &a, size_t kl) {
            csk.push_back(s), cek.push_back(e);
            put(cskeys, s ? sk : nullptr, kl), put(cekeys, e ? ek : nullptr, kl);
            caggs.push_back(a);
        }
        void enumeration(uint8_t s, const uint8_t *sk, uint8_t e, const uint8_t *ek, size_t kl) {
            esk.push_back(s), eek.push_back(e);
            put(eskeys, s ? sk : nullptr, kl), put(eekeys, e ? ek : nullptr, kl);
        }
        static void put(std::vector<uint8_t> &v, const uint8_t *k, size_t kl) {
            const size_t o = v.size();
            v.resize(o + kl, 0);
            if (k) memcpy(v.data() + o, k, kl);
        }
        void count(const rh_round_outcome &o) {
            cnt[0] += o.skipped, cnt[1] += o.enumerated, cnt[2] += o.split, cnt[3] += o.children,
                cnt[4] += o.dropped_malformed;
        }
        // a shard's round, copied out of the shard's buffers (a shard asked more than once per round)
        void take(const rh_segments &c, const rh_segments &e, const rh_round_outcome &o, size_t kl) {
            auto app = [](std::vector<uint8_t> &v, const void *p, size_t bytes) {
                if (bytes) v.insert(v.end(), static_cast<const uint8_t *>(p), static_cast<const uint8_t *>(p) + bytes);
            };
            app(csk, c.start_kinds, c.n), app(cek, c.end_kinds, c.n);
            app(cskeys, c.start_keys, c.n * kl), app(cekeys, c.end_keys, c.n * kl);
            if (c.n) caggs.insert(caggs.end(), c.aggregates, c.aggregates + c.n);
            app(esk, e.start_kinds, e.n), app(eek, e.end_kinds, e.n);
            app(eskeys, e.start_keys, e.n * kl), app(eekeys, e.end_keys, e.n * kl);
            count(o);
        }
        // ... or left in place until the round is assembled (a shard asked once)
        void borrow(const rh_segments &c, const rh_segments &e, const rh_round_outcome &o) {
            borrowed = true;
            bc = c, be = e;
            count(o);
        }
        size_t nc() const { return borrowed ? bc.n : csk.size(); }
        size_t ne() const { return borrowed ? be.n : esk.size(); }
        // this piece's bytes into the round at children offset c, enumerations offset e
        void put_into(uint8_t *o, const rh::RoundLayout &L, uint64_t c, uint64_t e, size_t kl) const {
            auto cp = [](uint8_t *dst, const void *src, size_t bytes) {
                if (!bytes) return;
                if (src) memcpy(dst, src, bytes);
                else memset(dst, 0, bytes);
            };
            const size_t pc = nc(), pe = ne();
            if (pc) {
                cp(o + L.csk + c, borrowed ? (const void *)bc.start_kinds : csk.data(), pc);
                cp(o + L.cek + c, borrowed ? (const void *)bc.end_kinds : cek.data(), pc);
                cp(o + L.cskeys + c * kl, borrowed ? bc.start_keys : cskeys.data(), pc * kl);
                cp(o + L.cekeys + c * kl, borrowed ? bc.end_keys : cekeys.data(), pc * kl);
                cp(o + L.caggs + c * sizeof(rh_aggregate), borrowed ? (const void *)bc.aggregates : caggs.data(),
                   pc * sizeof(rh_aggregate));
            }
            if (pe) {
                cp(o + L.esk + e, borrowed ? (const void *)be.start_kinds : esk.data(), pe);
                cp(o + L.eek + e, borrowed ? (const void *)be.end_kinds : eek.data(), pe);
                cp(o + L.eskeys + e * kl, borrowed ? be.start_keys : eskeys.data(), pe * kl);
                cp(o + L.eekeys + e * kl, borrowed ? be.end_keys : eekeys.data(), pe * kl);
            }
        }
    };
    struct Run {
        int shard;  // -1: segments that straddle shard boundaries
        size_t j0, j1;
    };
    // The round's output buffer (round_layout()); grown, never zero-filled: every byte a caller
    // reads through the returned arrays is written by the assembly.  Page-locked: the peer's next
    // round reads it, and its shards copy their pieces of it to their devices -- from pageable
    // memory each such copy went through the runtime's staging buffers and stalled 8-17 ms now and
    // then under eight shards (profiles/r06_sstore8_stalls.txt).  Pageable if that allocation fails.
    struct RoundBuf {
        uint8_t *p = nullptr;
        size_t cap = 0;
        bool pinned = false;
        ~RoundBuf() { drop(); }
        void drop() {
            if (p && pinned) (void)hipHostFree(p);
            else delete[] p;
            p = nullptr, cap = 0, pinned = false;
        }
        uint8_t *room(size_t bytes) {
            if (bytes <= cap) return p;
            const size_t c = bytes + bytes / 4;
            drop();
            void *q = nullptr;
            if (hipHostMalloc(&q, c, hipHostMallocPortable) == hipSuccess && q) {
                p = static_cast<uint8_t *>(q), pinned = true;
            } else {
                (void)hipGetLastError();
                p = new uint8_t[c];  // std::bad_alloc: the round's caller reports RH_ERR_OOM
            }
            cap = c;
            return p;
        }
    } round_buf;
    uint8_t *round_room(size_t bytes) { return round_buf.room(bytes); }

    // ---- routing a round's segments to the shards --------------------------------------------
    // Generic: each segment's two boundary shards by binary search over the splitters -- O(r log G)
    // key comparisons, right for any input.
    void route_each(const rh_segments &in, std::vector<Run> &runs) const {
        const uint8_t *sk = in.start_kinds, *ek = in.end_kinds;
        const uint8_t *skeys = static_cast<const uint8_t *>(in.start_keys);
        const uint8_t *ekeys = static_cast<const uint8_t *>(in.end_keys);
        runs.clear();
        for (size_t j = 0; j < in.n; j++) {
            int a, b;
            span(sk[j], sk[j] ? skeys + j * kl : nullptr, ek[j], ek[j] ? ekeys + j * kl : nullptr, &a, &b);
            const int s = a == b ? a : -1;
            if (!runs.empty() && runs.back().shard == s && runs.back().j1 == j) runs.back().j1 = j + 1;
            else runs.push_back(Run{s, j, j + 1});
        }
    }
    // Key-ordered input (a round's children are in key order, rbsr/src/protocol.rs:299-317): when
    // the start bounds and the end bounds are each non-decreasing in j (Unbounded start = -inf,
    // Unbounded end = +inf), both boundary shards are non-decreasing in j, so each shard's run and
    // the straddling segments between them are found by 2 (G - 1) binary searches over the
    // segments -- O(G log r) comparisons.  The order itself is verified in O(r), split between the
    // shards' tasks (each checks its own run before asking its shard) and the caller (the
    // straddling runs); any violation falls back to route_each.
    bool pair_sorted(const uint8_t *sk, const uint8_t *skeys, const uint8_t *ek, const uint8_t *ekeys, size_t j) const {
        if (sk[j]) {
            if (sk[j - 1] && cmp(skeys + (j - 1) * kl, skeys + j * kl) > 0) return false;
        } else if (sk[j - 1]) {
            return false;
        }
        if (ek[j - 1]) {
            if (ek[j] && cmp(ekeys + (j - 1) * kl, ekeys + j * kl) > 0) return false;
        } else if (ek[j]) {
            return false;
        }
        return true;
    }
    // the pairs (j - 1, j) for j in [j0, j1) are ordered (pair_sorted's rule; integer keys
    // compared as integers in one tight loop: this check runs over every segment of a round on
    // the shard threads, ~1.6 ns a segment through cmp())
    template <class T>
    static bool pairs_sorted_int(const uint8_t *sk, const uint8_t *skeys, const uint8_t *ek, const uint8_t *ekeys,
                                 size_t j0, size_t j1) {
        bool ok = true;
        for (size_t j = j0; j < j1; j++) {
            T s0 = 0, s1 = 0, e0 = 0, e1 = 0;
            if (sk[j - 1]) memcpy(&s0, skeys + (j - 1) * sizeof(T), sizeof(T));
            if (sk[j]) memcpy(&s1, skeys + j * sizeof(T), sizeof(T));
            if (ek[j - 1]) memcpy(&e0, ekeys + (j - 1) * sizeof(T), sizeof(T));
            if (ek[j]) memcpy(&e1, ekeys + j * sizeof(T), sizeof(T));
            // starts: Unbounded (-inf) only before bounded ones; ends: bounded only before Unbounded (+inf)
            ok &= sk[j] ? (!sk[j - 1] || s0 <= s1) : !sk[j - 1];
            ok &= ek[j - 1] ? (!ek[j] || e0 <= e1) : !ek[j];
        }
        return ok;
    }
    bool pairs_sorted(const rh_segments &in, size_t j0, size_t j1) const {
        const uint8_t *sk = in.start_kinds, *ek = in.end_kinds;
        const uint8_t *skeys = static_cast<const uint8_t *>(in.start_keys);
        const uint8_t *ekeys = static_cast<const uint8_t *>(in.end_keys);
        j0 = std::max<size_t>(j0, 1);
        if (j0 >= j1) return true;
        static const uint8_t zkey[64] = {0};
        const uint8_t *sp = skeys ? skeys : zkey, *ep = ekeys ? ekeys : zkey;  // all-unbounded sides
        if (schema.key_kind == RH_KEY_U64 && skeys && ekeys) return pairs_sorted_int<uint64_t>(sk, sp, ek, ep, j0, j1);
        if (schema.key_kind == RH_KEY_U32 && skeys && ekeys) return pairs_sorted_int<uint32_t>(sk, sp, ek, ep, j0, j1);
        for (size_t j = j0; j < j1; j++)
            if (!pair_sorted(sk, skeys, ek, ekeys, j)) return false;
        return true;
    }
    bool route_sorted(const rh_segments &in, std::vector<Run> &runs) const {
        const size_t r = in.n;
        const uint8_t *sk = in.start_kinds, *ek = in.end_kinds;
        const uint8_t *skeys = static_cast<const uint8_t *>(in.start_keys);
        const uint8_t *ekeys = static_cast<const uint8_t *>(in.end_keys);
        auto first = [r](auto pred) {  // the first j in [0, r) with pred(j), else r (pred monotone)
            size_t lo = 0, hi = r;
            while (lo < hi) {
                const size_t mid = lo + (hi - lo) / 2;
                if (pred(mid)) hi = mid;
                else lo = mid + 1;
            }
            return lo;
        };
        // A[s]: the first segment whose start shard is >= s; B[s]: whose end shard is >= s
        std::vector<size_t> A(G + 1, 0), B(G + 1, 0);
        A[G] = B[G] = r;
        for (int t = 1; t < G; t++) {
            const uint8_t *sp = splitter(t - 1);
            A[t] = first([&](size_t j) { return sk[j] && cmp(sp, skeys + j * kl) <= 0; });
            B[t] = first([&](size_t j) { return !ek[j] || cmp(sp, ekeys + j * kl) < 0; });
        }
        runs.clear();
        size_t cur = 0;
        for (int t = 0; t < G; t++) {
            const size_t lo = std::max(A[t], B[t]), hi = std::min(A[t + 1], B[t + 1]);
            if (lo >= hi) continue;
            if (lo < cur) return false;  // not monotone after all
            if (cur < lo) runs.push_back(Run{-1, cur, lo});
            runs.push_back(Run{t, lo, hi});
            cur = hi;
        }
        if (cur < r) runs.push_back(Run{-1, cur, r});
        // the straddling runs' order is checked here; each shard's by its task
        for (const Run &R : runs)
            if (R.shard < 0 && !pairs_sorted(in, R.j0, R.j1)) return false;
        return true;
    }

    // RSOS_HIP_SSTORE_DBG=1: one line per protocol round on stderr -- segments, runs, straddling
    // segments, and the host times of its phases (us): routing, the straddling segments, the
    // shards' rounds (and the slowest shard's own call), the assembly
    static bool dbg() {
        static const bool on = getenv("RSOS_HIP_SSTORE_DBG") && atoi(getenv("RSOS_HIP_SSTORE_DBG")) > 0;
        return on;
    }
    static double now_us() {
        return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    // copying a round's pieces takes the shard threads past this many bytes
    static constexpr size_t PARALLEL_COPY_BYTES = 1 << 20;
    int protocol_round(int policy, uint64_t fan_out, const rh_segments &in, rh_segments *ch, rh_segments *en,
                       rh_round_outcome *oc) {
        const double t0 = dbg() ? now_us() : 0;
        std::vector<double> shard_us(dbg() ? G : 0, 0.0), verify_us(dbg() ? G : 0, 0.0);
        std::vector<Run> runs;
        bool fast = route_sorted(in, runs);
        if (!fast) route_each(in, runs);
        const double t1 = dbg() ? now_us() : 0;
        double t2 = t1, t3 = t1;
        std::vector<Out> outs;
        std::vector<std::vector<size_t>> mine;
        std::vector<int> idx;
        const uint8_t *sk = in.start_kinds, *ek = in.end_kinds;
        const uint8_t *skeys = static_cast<const uint8_t *>(in.start_keys);
        const uint8_t *ekeys = static_cast<const uint8_t *>(in.end_keys);
        for (int pass = 0; pass < 2; pass++) {
            outs.assign(runs.size(), Out{});
            mine.assign(G, {});
            std::vector<size_t> cross;
            for (size_t k = 0; k < runs.size(); k++) {
                if (runs[k].shard >= 0) mine[runs[k].shard].push_back(k);
                else
                    for (size_t j = runs[k].j0; j < runs[k].j1; j++) cross.push_back(j);
            }
            idx.clear();
            for (int s = 0; s < G; s++)
                if (!mine[s].empty()) idx.push_back(s);
            // the straddling segments first: their shard calls come before the shards' own rounds,
            // whose outputs then stay in place until the round is assembled
            int rc;
            if (!cross.empty() && (rc = cross_round(policy, fan_out, in, runs, cross, outs))) return rc;
            t2 = dbg() ? now_us() : 0;
            std::atomic<bool> unsorted{false};
            auto sub_of = [&](size_t k) {
                const Run &R = runs[k];
                const size_t j = R.j0;
                return rh_segments{const_cast<uint8_t *>(sk + j), skeys ? const_cast<uint8_t *>(skeys + j * kl) : nullptr,
                                   const_cast<uint8_t *>(ek + j), ekeys ? const_cast<uint8_t *>(ekeys + j * kl) : nullptr,
                                   in.aggregates + j, R.j1 - R.j0, R.j1 - R.j0};
            };
            // per device: every shard's round issued, then each completed -- the device runs one
            // shard's round while the host issues the next, and the host waits once per shard at
            // the end instead of between them
            // every shard's piece within its host tier's round size: host work only, one thread
            // per shard whatever the devices
            bool host_only = tier_on;
            for (int s : idx)
                for (size_t k : mine[s]) host_only = host_only && runs[k].j1 - runs[k].j0 <= round_max;
            rc = each_device(idx, [&](const std::vector<int> &gs) -> int {
                const double u0 = dbg() ? now_us() : 0;
                int first = RH_OK;
                std::string msg;
                auto keep = [&](int q) {
                    if (q && !first) first = q, msg = rh_last_error() ? rh_last_error() : "";
                };
                std::vector<std::pair<int, size_t>> pend;  // (shard, run) issued, to complete
                pend.reserve(gs.size());
                // every issued round completes, however this task ends: it holds its store's lock
                struct Drain {
                    std::vector<std::pair<int, size_t>> &pend;
                    rh_sstore *self;
                    ~Drain() {
                        for (const auto &p : pend) {
                            rh_segments c{}, e{};
                            rh_round_outcome o{};
                            (void)rh::store_round_complete(self->shards[p.first], &c, &e, &o);
                        }
                    }
                } drain{pend, this};
                for (int s : gs) {
                    if (first) break;
                    const double v0 = dbg() ? now_us() : 0;
                    if (fast && !pairs_sorted(in, runs[mine[s][0]].j0, runs[mine[s][0]].j1)) {
                        unsorted = true;
                        continue;
                    }
                    if (!verify_us.empty()) verify_us[s] = now_us() - v0;
                    if (mine[s].size() == 1) {
                        const size_t k = mine[s][0];
                        const rh_segments sub = sub_of(k);
                        rh_segments c{}, e{};
                        rh_round_outcome o{};
                        bool pending = false;
                        const int q = rh::store_round_issue(shards[s], policy, fan_out, &sub, &c, &e, &o, &pending);
                        keep(q);
                        if (!q && pending) pend.emplace_back(s, k);
                        else if (!q) outs[k].borrow(c, e, o);
                        continue;
                    }
                    for (size_t k : mine[s]) {  // a shard asked for several runs: one at a time, copied
                        const rh_segments sub = sub_of(k);
                        rh_segments c{}, e{};
                        rh_round_outcome o{};
                        const int q = rh_store_protocol_round(shards[s], policy, fan_out, &sub, &c, &e, &o);
                        keep(q);
                        if (q) break;
                        outs[k].take(c, e, o, kl);
                    }
                }
                while (!pend.empty()) {  // completed in issue order; the rest by `drain` if one throws
                    const auto p = pend.front();
                    pend.erase(pend.begin());
                    rh_segments c{}, e{};
                    rh_round_outcome o{};
                    const int q = rh::store_round_complete(shards[p.first], &c, &e, &o);
                    keep(q);
                    if (!q) outs[p.second].borrow(c, e, o);
                }
                if (!shard_us.empty())
                    for (int s : gs) shard_us[s] = now_us() - u0;
                return first ? rh::set_error(first, msg) : RH_OK;
            }, !host_only);
            if (rc) return rc;
            t3 = dbg() ? now_us() : 0;
            if (!unsorted) break;
            fast = false;  // the input was not key-ordered after all: route each segment
            route_each(in, runs);
        }
        // the pieces in segment order, in round_layout()
        uint64_t nc = 0, ne = 0, cnt[5] = {0, 0, 0, 0, 0};
        for (const Out &o : outs) {
            nc += o.nc(), ne += o.ne();
            for (int i = 0; i < 5; i++) cnt[i] += o.cnt[i];
        }
        if (oc) *oc = rh_round_outcome{cnt[0], cnt[1], cnt[2], cnt[3], cnt[4]};
        if (outs.size() == 1 && outs[0].borrowed) {  // one shard's round is the whole round: in place
            *ch = outs[0].bc;
            *en = outs[0].be;
            ch->cap = ch->n, en->cap = en->n;
            if (!ch->n) *ch = rh_segments{};
            if (!en->n) *en = rh_segments{};
        } else {
            const rh::RoundLayout L = rh::round_layout(nc, ne, kl);
            uint8_t *o = round_room(L.end);
            std::vector<uint64_t> at_c(outs.size()), at_e(outs.size());
            uint64_t c = 0, e = 0;
            for (size_t k = 0; k < outs.size(); k++) {
                at_c[k] = c, at_e[k] = e;
                c += outs[k].nc(), e += outs[k].ne();
            }
            memset(o, 0, 64);
            memcpy(o, cnt, sizeof cnt);
            if (L.end > PARALLEL_COPY_BYTES && idx.size() > 1) {
                // each shard's thread copies its own pieces (the straddling ones go with shard 0's task)
                int rc = each(idx, [&](int s) -> int {
                    for (size_t k : mine[s]) outs[k].put_into(o, L, at_c[k], at_e[k], kl);
                    if (s == idx[0])
                        for (size_t k = 0; k < runs.size(); k++)
                            if (runs[k].shard < 0) outs[k].put_into(o, L, at_c[k], at_e[k], kl);
                    return RH_OK;
                }, false);
                if (rc) return rc;
            } else {
                for (size_t k = 0; k < outs.size(); k++) outs[k].put_into(o, L, at_c[k], at_e[k], kl);
            }
            *ch = rh_segments{o + L.csk, o + L.cskeys, o + L.cek, o + L.cekeys, reinterpret_cast<rh_aggregate *>(o + L.caggs),
                              (size_t)nc, (size_t)nc};
            *en = rh_segments{o + L.esk, o + L.eskeys, o + L.eek, o + L.eekeys, nullptr, (size_t)ne, (size_t)ne};
        }
        if (dbg()) {
            const double t4 = now_us();
            size_t ncross = 0;
            for (const Run &R : runs)
                if (R.shard < 0) ncross += R.j1 - R.j0;
            fprintf(stderr,
                    "{\"sstore_round\": %zu, \"sorted\": %d, \"runs\": %zu, \"cross\": %zu, \"shards\": %zu, "
                    "\"route_us\": %.1f, \"cross_us\": %.1f, \"shards_us\": %.1f, \"slowest_shard_us\": %.1f, "
                    "\"assemble_us\": %.1f, \"verify_us_sum\": %.1f, \"children\": %llu}\n",
                    in.n, (int)fast, runs.size(), ncross, idx.size(), t1 - t0, t2 - t1, t3 - t2,
                    shard_us.empty() ? 0.0 : *std::max_element(shard_us.begin(), shard_us.end()), t4 - t3,
                    std::accumulate(verify_us.begin(), verify_us.end(), 0.0), (unsigned long long)nc);
        }
        return RH_OK;
    }
    // The segments that straddle a shard boundary: resolved from their boundary shards, decided on
    // the host (decide_segment), their SPLIT cuts selected and their children summed over the
    // shards holding them -- one call per shard for each of the two steps.
    int cross_round(int policy, uint64_t fan_out, const rh_segments &in, const std::vector<Run> &runs,
                    const std::vector<size_t> &J, std::vector<Out> &outs) {
        const uint8_t *sk = in.start_kinds, *ek = in.end_kinds;
        const uint8_t *skeys = static_cast<const uint8_t *>(in.start_keys);
        const uint8_t *ekeys = static_cast<const uint8_t *>(in.end_keys);
        static const uint8_t zkey[64] = {0};
        const uint8_t *skp = skeys ? skeys : zkey, *ekp = ekeys ? ekeys : zkey;
        const size_t nj = J.size();
        std::vector<uint64_t> lo(nj), hi(nj);
        std::vector<rh_aggregate> loc(nj);
        int rc = resolve_list(J, sk, skp, ek, ekp, lo.data(), hi.data(), loc.data());
        if (rc) return rc;
        const int sq = policy == RH_POLICY_SQRT_FAN_OUT;
        const uint64_t b = fan_out < 2 ? 2 : fan_out;
        std::vector<rh::SegDecision> d(nj);
        std::vector<uint64_t> sel, clo, chi;
        std::vector<size_t> first_sel(nj), first_child(nj);
        for (size_t t = 0; t < nj; t++) {
            d[t] = rh::decide_segment(lo[t], hi[t], loc[t], in.aggregates[J[t]], sq, b);
            first_sel[t] = sel.size(), first_child[t] = clo.size();
            if (d[t].kind != 2 || d[t].children < 2) continue;
            const uint64_t ncuts = d[t].children - 1;
            uint64_t x = lo[t];
            for (uint64_t k = 0; k <= ncuts; k++) {
                const uint64_t y = k == ncuts ? hi[t] : lo[t] + (k + 1) * d[t].stride;
                if (k != ncuts) sel.push_back(y);
                clo.push_back(x), chi.push_back(y);
                x = y;
            }
        }
        std::vector<uint8_t> cut(sel.size() * kl + 1);
        std::vector<rh_aggregate> caggs(clo.size() + 1);
        if ((!sel.empty() || !clo.empty()) &&
            (rc = split_ranks(sel.size(), sel.data(), cut.data(), clo.size(), clo.data(), chi.data(), caggs.data())))
            return rc;
        // each straddling segment's output goes to its run's piece, in segment order
        size_t t = 0;
        for (size_t k = 0; k < runs.size() && t < nj; k++) {
            if (runs[k].shard >= 0) continue;
            Out &o = outs[k];
            for (size_t j = runs[k].j0; j < runs[k].j1; j++, t++) {
                const rh::SegDecision &g = d[t];
                const uint8_t *s0 = sk[j] ? skp + j * kl : nullptr, *e0 = ek[j] ? ekp + j * kl : nullptr;
                o.cnt[g.kind == 3 ? 4 : g.kind]++;
                if (g.kind == 1) {
                    o.enumeration(sk[j], s0, ek[j], e0, kl);
                    if (g.children) o.child(sk[j], s0, ek[j], e0, kZero, kl);
                } else if (g.kind == 2) {
                    if (g.children < 2) {
                        o.child(sk[j], s0, ek[j], e0, loc[t], kl);
                    } else {
                        const uint64_t ncuts = g.children - 1;
                        const uint8_t *prev = nullptr;
                        for (uint64_t c = 0; c <= ncuts; c++) {
                            const uint8_t *key = c < ncuts ? cut.data() + (first_sel[t] + c) * kl : nullptr;
                            o.child(c ? 1 : sk[j], c ? prev : s0, c != ncuts ? 1 : ek[j], c != ncuts ? key : e0,
                                    caggs[first_child[t] + c], kl);
                            prev = key;
                        }
                    }
                }
                o.cnt[3] += g.children;
            }
        }
        return RH_OK;
    }
};

namespace {

int lock_sizes(rh_sstore *s, std::unique_lock<std::mutex> &g) {
    g = std::unique_lock<std::mutex>(s->mu);
    if (int rc = s->health()) return rc;
    Status st = s->flush();
    return st.rc ? fail(st.rc, st.msg) : RH_OK;
}

}  // namespace

extern "C" {

int rh_sstore_create(const int *devices, int n, const rh_schema *schema, rh_sstore **out) {
    if (!devices || n < 1 || n > 64 || !schema || !out) return fail(RH_ERR_ARG, "sstore: bad arguments");
    rh_sstore *s = new (std::nothrow) rh_sstore();
    if (!s) return fail(RH_ERR_OOM, "sstore: host allocation failed");
    s->schema = *schema;
    s->G = n;
    s->kl = (size_t)key_row(*schema);
    s->shards.assign(n, nullptr);
    s->dev.assign(devices, devices + n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < i; j++) s->shared_devices |= devices[i] == devices[j];
    for (int i = 0; i < n; i++) {
        const int rc = rh_store_create(devices[i], schema, &s->shards[i]);
        if (rc) {
            const std::string msg = rh_last_error();
            for (rh_store *t : s->shards) rh_store_destroy(t);
            delete s;
            return fail(rc, msg);
        }
    }
    s->sizes.assign(n, 0);
    s->off.assign(n + 1, 0);
    s->sizes_ok = true;
    s->dirty.assign(n, 0);
    s->roots.assign(n, kZero);
    s->root_ok.assign(n, 0);
    s->even_splitters();
    try {
        s->pool = new ShardPool(n);
    } catch (...) {
        for (rh_store *t : s->shards) rh_store_destroy(t);
        delete s;
        return fail(RH_ERR_OOM, "sstore: cannot start the shard threads");
    }
    *out = s;
    return RH_OK;
}

int rh_sstore_destroy(rh_sstore *s) {
    if (!s) return RH_OK;
    delete s->pool;
    for (rh_store *t : s->shards) rh_store_destroy(t);
    delete s;
    return RH_OK;
}

int rh_sstore_shard_count(rh_sstore *s) { return s ? s->G : fail(RH_ERR_ARG, "sstore is NULL"); }

int rh_sstore_shard(rh_sstore *s, int i, rh_store **out) {
    if (!s || !out || i < 0 || i >= s->G) return fail(RH_ERR_ARG, "sstore: bad shard index");
    *out = s->shards[i];
    return RH_OK;
}

int rh_sstore_splitters(rh_sstore *s, void *out) {
    if (!s || (s->G > 1 && !out)) return fail(RH_ERR_ARG, "NULL");
    std::lock_guard<std::mutex> g(s->mu);
    if (s->G > 1) memcpy(out, s->split.data(), s->split.size());
    return RH_OK;
}

int rh_sstore_set_splitters(rh_sstore *s, const void *keys) {
    if (!s || (s->G > 1 && !keys)) return fail(RH_ERR_ARG, "NULL");
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);
    if (rc) return rc;
    if (s->total() != 0) return fail(RH_ERR_STATE, "sstore: splitters can only be set on an empty map");
    const uint8_t *k = static_cast<const uint8_t *>(keys);
    for (int j = 1; j + 1 < s->G; j++)
        if (s->cmp(k + (j - 1) * s->kl, k + j * s->kl) > 0) return fail(RH_ERR_ARG, "sstore: splitters must not decrease");
    if (s->G > 1) s->split.assign(k, k + (size_t)(s->G - 1) * s->kl);
    return RH_OK;
}

int rh_sstore_load(rh_sstore *s, const rh_columns *h, size_t n) {
    if (!s || !h) return fail(RH_ERR_ARG, "NULL");
    if (n && s->kl && !h->keys) return fail(RH_ERR_ARG, "keys column is NULL");
    std::lock_guard<std::mutex> g(s->mu);
    const int G = s->G;
    const size_t kl = s->kl, vr = value_row(s->schema);
    const uint8_t *keys = static_cast<const uint8_t *>(h->keys);
    std::vector<uint64_t> cut(G + 1);
    for (int j = 0; j <= G; j++) cut[j] = (uint64_t)((unsigned __int128)n * (unsigned)j / (unsigned)G);
    // the keys must be strictly increasing across the cuts too (each shard checks its own rows)
    bool ok = true;
    for (int j = 1; j < G && ok; j++)
        if (cut[j] > 0 && cut[j] < n) ok = s->cmp(keys + (cut[j] - 1) * kl, keys + cut[j] * kl) < 0;
    auto part = [&](int j) {
        const uint64_t a = cut[j];
        const bool dated = s->schema.record_kind == RH_REC_DATED;
        auto at = [&](const void *p, size_t w) -> const void * {
            return p ? static_cast<const uint8_t *>(p) + a * w : nullptr;
        };
        return rh_columns{at(h->keys, kl), static_cast<const uint64_t *>(dated ? at(h->phys, 8) : nullptr),
                          static_cast<const uint32_t *>(dated ? at(h->logical, 4) : nullptr),
                          static_cast<const uint64_t *>(dated ? at(h->node, 8) : nullptr),
                          static_cast<const uint8_t *>(at(h->tags, 1)), at(h->values, vr)};
    };
    int rc = RH_OK;
    s->changed();
    s->broken.clear();
    std::fill(s->dirty.begin(), s->dirty.end(), 0);
    if (!ok) {
        rc = fail(RH_ERR_ARG, "keys must be strictly increasing (sorted, no duplicates)");
    } else {
        rc = s->each(s->all(), [&](int j) -> int {
            const rh_columns c = part(j);
            return rh_store_load(s->shards[j], &c, cut[j + 1] - cut[j]);
        });
    }
    if (rc) {  // the map is left empty, as a single store is after a failed load
        const std::string msg = rh_last_error();
        const rh_columns none{};
        for (int j = 0; j < G; j++) (void)rh_store_load(s->shards[j], &none, 0);
        s->even_splitters();
        s->sizes.assign(G, 0), s->off.assign(G + 1, 0), s->sizes_ok = true;
        return fail(rc, msg);
    }
    if (n) {
        s->split.resize((size_t)(G - 1) * kl);
        for (int j = 1; j < G; j++) memcpy(s->split.data() + (j - 1) * kl, keys + cut[j] * kl, kl);
    } else {
        s->even_splitters();
    }
    for (int j = 0; j < G; j++) s->sizes[j] = cut[j + 1] - cut[j];
    for (int j = 0; j <= G; j++) s->off[j] = cut[j];
    s->sizes_ok = true;
    return RH_OK;
}

int rh_sstore_stage(rh_sstore *s, const rh_columns *h, const uint8_t *ops, size_t m) {
    if (!s || !h || (m && !ops)) return fail(RH_ERR_ARG, "NULL");
    if (m == 0) return RH_OK;
    if (s->kl && !h->keys) return fail(RH_ERR_ARG, "keys column is NULL");
    std::lock_guard<std::mutex> g(s->mu);
    int rc;
    if ((rc = s->health())) return rc;
    const uint8_t *keys = static_cast<const uint8_t *>(h->keys);
    for (size_t i = 0; i < m; i++)
        if (ops[i] > 1) return fail(RH_ERR_ARG, "op must be 0 (insert) or 1 (delete)");
    if (m == 1 || s->G == 1) {  // the Rsos::insert path: one row, no copies
        const int t = s->G == 1 ? 0 : s->owner(keys);
        if ((rc = rh_store_stage(s->shards[t], h, ops, m))) return rc;
        s->dirty[t] = 1;
        s->changed();
        return RH_OK;
    }
    try {
        std::vector<std::vector<uint32_t>> rows;
        s->route(keys, m, rows);
        std::vector<rh_sstore::Part> parts(s->G);
        for (int t = 0; t < s->G; t++)  // every copy made before any shard takes a row
            if (!rows[t].empty()) s->gather(*h, ops, rows[t], parts[t]);
        int staged = 0;
        for (int t = 0; t < s->G; t++) {
            if (rows[t].empty()) continue;
            const rh_columns c = parts[t].cols();
            if ((rc = rh_store_stage(s->shards[t], &c, parts[t].ops.data(), parts[t].m))) {
                if (staged) s->broken = "a staged batch was refused by one shard after others had taken their rows";
                return rc;
            }
            staged++;
            s->dirty[t] = 1;
            s->changed();
        }
    } catch (const std::bad_alloc &) {
        return fail(RH_ERR_OOM, "stage: host allocation failed");
    }
    return RH_OK;
}

int rh_sstore_apply(rh_sstore *s, const rh_columns *h, const uint8_t *ops, size_t m, uint64_t *n_new, uint64_t *n_over,
                    uint64_t *n_del) {
    if (!s || !h || (m && !ops)) return fail(RH_ERR_ARG, "NULL");
    if (m && s->kl && !h->keys) return fail(RH_ERR_ARG, "keys column is NULL");
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);  // staged rows first: they were staged before this batch
    if (rc) return rc;
    // every check a shard's apply makes on the arguments, made here before any shard changes
    for (size_t i = 0; i < m; i++)
        if (ops[i] > 1) return fail(RH_ERR_ARG, "op must be 0 (insert) or 1 (delete)");
    if (m) {
        const rh_schema &sc = s->schema;
        if (sc.value_kind != RH_VAL_UNIT && !h->values) return fail(RH_ERR_ARG, "values column is NULL");
        if (sc.record_kind == RH_REC_DATED && (!h->phys || !h->logical || !h->node))
            return fail(RH_ERR_ARG, "DATED records need phys / logical / node columns");
    }
    uint64_t c[64][3] = {};
    try {
        std::vector<std::vector<uint32_t>> rows;
        s->route(static_cast<const uint8_t *>(h->keys), m, rows);
        std::vector<rh_sstore::Part> parts(s->G);
        std::vector<int> idx;
        for (int t = 0; t < s->G; t++)
            if (!rows[t].empty()) idx.push_back(t);
        std::vector<uint8_t> dup(s->G, 0);
        // every shard's rows gathered and checked first: a batch with a repeated key changes no shard
        if ((rc = s->each(idx, [&](int t) -> int {
                 s->gather(*h, ops, rows[t], parts[t]);
                 dup[t] = s->has_duplicates(parts[t].keys.data(), parts[t].m);
                 return RH_OK;
             })))
            return rc;
        for (int t : idx)
            if (dup[t]) return fail(RH_ERR_ARG, "duplicate key within one batch");
        for (int t : idx)  // the row cap, counting every row as new
            if (s->sizes[t] + parts[t].m >= (1ull << 31))
                return fail(RH_ERR_ARG, "store size limit (2^31 rows) exceeded in one shard: use more shards");
        s->changed();
        const bool inject = rh::debug_fail_point("sstore.apply_last_shard");
        rc = s->each(idx, [&](int t) -> int {
            if (inject && t == idx.back()) return rh::set_error(RH_ERR_OOM, "injected failure (sstore apply)");
            const rh_columns cols = parts[t].cols();
            return rh_store_apply(s->shards[t], &cols, parts[t].ops.data(), parts[t].m, &c[t][0], &c[t][1], &c[t][2]);
        });
        if (rc) {
            // past the checks above only a device or allocation failure remains; with more than one
            // shard written the others may have committed their part
            if (idx.size() > 1) s->broken = "an apply failed in one shard after others may have committed their rows";
            return rc;
        }
    } catch (const std::bad_alloc &) {
        return fail(RH_ERR_OOM, "apply: host allocation failed");
    }
    uint64_t tot[3] = {0, 0, 0};
    for (int t = 0; t < s->G; t++)
        for (int i = 0; i < 3; i++) tot[i] += c[t][i];
    if (n_new) *n_new = tot[0];
    if (n_over) *n_over = tot[1];
    if (n_del) *n_del = tot[2];
    return RH_OK;
}

int rh_sstore_len(rh_sstore *s, uint64_t *out) {
    if (!s || !out) return fail(RH_ERR_ARG, "NULL");
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);
    if (rc) return rc;
    *out = s->total();
    return RH_OK;
}

int rh_sstore_aggregates(rh_sstore *s, const uint64_t *lo, const uint64_t *hi, size_t r, rh_aggregate *out) {
    if (!s) return fail(RH_ERR_ARG, "sstore is NULL");
    if (r && (!lo || !hi || !out)) return fail(RH_ERR_ARG, "NULL buffer");
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);
    if (rc) return rc;
    try {
        return s->split_ranks(0, nullptr, nullptr, r, lo, hi, out);
    } catch (const std::bad_alloc &) {
        return fail(RH_ERR_OOM, "aggregates: host allocation failed");
    }
}

int rh_sstore_aggregate_keys(rh_sstore *s, int lo_kind, const void *lo_key, int hi_kind, const void *hi_key,
                             rh_aggregate *out) {
    if (!s || !out) return fail(RH_ERR_ARG, "NULL");
    if (lo_kind < 0 || lo_kind > 2 || hi_kind < 0 || hi_kind > 2) return fail(RH_ERR_ARG, "bad bound kind");
    if ((lo_kind && !lo_key) || (hi_kind && !hi_key)) return fail(RH_ERR_ARG, "bound key is NULL");
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);
    if (rc) return rc;
    const uint8_t *lk = static_cast<const uint8_t *>(lo_key), *hk = static_cast<const uint8_t *>(hi_key);
    // the shards the range can touch: from the one holding its lower bound to the one holding the
    // keys just below its upper bound (Included(k) reaches k's own shard)
    const int a = lo_kind ? s->owner(lk) : 0;
    const int b = !hi_kind ? s->G - 1 : hi_kind == 1 ? s->owner(hk) : s->owner_below(hk);
    *out = kZero;
    if (a > b) return RH_OK;  // an inverted or empty range: ZERO (rbsr/src/protocol.rs:230-232)
    if (a == b) return rh_store_aggregate_keys(s->shards[a], lo_kind, lo_key, hi_kind, hi_key, out);
    // the two edge shards (each asked one bound) and the cached roots of the shards between them;
    // host-tier edges on the calling thread (a thread handoff would cost more than the question)
    rh_aggregate part[2] = {kZero, kZero};
    auto edge = [&](int t) -> int {
        return t == a ? rh_store_aggregate_keys(s->shards[a], lo_kind, lo_key, 0, nullptr, &part[0])
                      : rh_store_aggregate_keys(s->shards[b], 0, nullptr, hi_kind, hi_key, &part[1]);
    };
    if (s->tier_on) {
        if ((rc = edge(a)) || (rc = edge(b))) return rc;
    } else if ((rc = s->each({a, b}, edge))) {
        return rc;
    }
    agg_add(*out, part[0]);
    for (int t = a + 1; t < b; t++) {
        rh_aggregate m;
        if ((rc = s->root(t, &m))) return rc;
        agg_add(*out, m);
    }
    agg_add(*out, part[1]);
    return RH_OK;
}

int rh_sstore_ranks(rh_sstore *s, const void *keys, size_t m, uint64_t *out) {
    if (!s || (m && (!keys || !out))) return fail(RH_ERR_ARG, "NULL");
    if (m == 0) return RH_OK;
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);
    if (rc) return rc;
    const uint8_t *k = static_cast<const uint8_t *>(keys);
    if (m == 1) {
        const int t = s->owner(k);
        uint64_t r = 0;
        if ((rc = rh_store_rank(s->shards[t], k, &r))) return rc;
        *out = s->off[t] + r;
        return RH_OK;
    }
    try {
        std::vector<std::vector<uint32_t>> rows;
        s->route(k, m, rows);
        std::vector<std::vector<uint8_t>> qk(s->G);
        std::vector<std::vector<uint64_t>> qr(s->G);
        std::vector<int> idx;
        for (int t = 0; t < s->G; t++)
            if (!rows[t].empty()) idx.push_back(t);
        rc = s->each(idx, [&](int t) -> int {
            qk[t].resize(rows[t].size() * s->kl + 1);
            for (size_t i = 0; i < rows[t].size(); i++) memcpy(&qk[t][i * s->kl], k + rows[t][i] * s->kl, s->kl);
            qr[t].resize(rows[t].size());
            return rh_store_ranks(s->shards[t], qk[t].data(), rows[t].size(), qr[t].data());
        });
        if (rc) return rc;
        for (int t : idx)
            for (size_t i = 0; i < rows[t].size(); i++) out[rows[t][i]] = s->off[t] + qr[t][i];
    } catch (const std::bad_alloc &) {
        return fail(RH_ERR_OOM, "ranks: host allocation failed");
    }
    return RH_OK;
}

int rh_sstore_rank(rh_sstore *s, const void *key, uint64_t *out) { return rh_sstore_ranks(s, key, 1, out); }

int rh_sstore_keys(rh_sstore *s, uint64_t lo, uint64_t hi, void *host_out) {
    if (!s) return fail(RH_ERR_ARG, "sstore is NULL");
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);
    if (rc) return rc;
    if (lo > hi || hi > s->total()) return fail(RH_ERR_ARG, "bad rank range");
    if (hi == lo) return RH_OK;
    if (!host_out) return fail(RH_ERR_ARG, "host_out NULL");
    std::vector<int> idx;
    for (int t = 0; t < s->G; t++)
        if (s->off[t] < hi && s->off[t + 1] > lo) idx.push_back(t);
    return s->each(idx, [&](int t) -> int {
        uint64_t a, b;
        s->piece(t, lo, hi, &a, &b);
        return rh_store_keys(s->shards[t], a, b, static_cast<uint8_t *>(host_out) + (s->off[t] + a - lo) * s->kl);
    });
}

int rh_sstore_select(rh_sstore *s, uint64_t r, void *key_out) {
    if (!s || !key_out) return fail(RH_ERR_ARG, "NULL");
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);
    if (rc) return rc;
    if (r >= s->total()) return fail(RH_ERR_ARG, "select: rank out of range (r >= size)");
    const int t = s->shard_of_rank(r);
    return rh_store_select(s->shards[t], r - s->off[t], key_out);
}

int rh_sstore_fingerprints(rh_sstore *s, uint64_t lo, uint64_t hi, uint8_t *host_out) {
    if (!s) return fail(RH_ERR_ARG, "sstore is NULL");
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);
    if (rc) return rc;
    if (lo > hi || hi > s->total()) return fail(RH_ERR_ARG, "bad rank range");
    if (hi == lo) return RH_OK;
    if (!host_out) return fail(RH_ERR_ARG, "host_out NULL");
    std::vector<int> idx;
    for (int t = 0; t < s->G; t++)
        if (s->off[t] < hi && s->off[t + 1] > lo) idx.push_back(t);
    return s->each(idx, [&](int t) -> int {
        uint64_t a, b;
        s->piece(t, lo, hi, &a, &b);
        return rh_store_fingerprints(s->shards[t], a, b, host_out + (s->off[t] + a - lo) * 32);
    });
}

int rh_sstore_resolve_segments(rh_sstore *s, size_t r, const uint8_t *start_kinds, const void *start_keys,
                               const uint8_t *end_kinds, const void *end_keys, uint64_t *raw_start, uint64_t *raw_end,
                               rh_aggregate *local) {
    if (!s) return fail(RH_ERR_ARG, "sstore is NULL");
    if (r == 0) return RH_OK;
    if (!start_kinds || !end_kinds || !raw_start || !raw_end || !local) return fail(RH_ERR_ARG, "NULL buffer");
    for (size_t j = 0; j < r; j++) {
        if (start_kinds[j] > 1 || end_kinds[j] > 1)
            return fail(RH_ERR_ARG, "segment bound kind must be 0 (Unbounded) or 1 (Included / Excluded)");
        if ((start_kinds[j] && !start_keys) || (end_kinds[j] && !end_keys)) return fail(RH_ERR_ARG, "bound key is NULL");
    }
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);
    if (rc) return rc;
    try {
        std::vector<uint8_t> zero(r * s->kl + 1, 0);
        const uint8_t *sk = start_keys ? static_cast<const uint8_t *>(start_keys) : zero.data();
        const uint8_t *ek = end_keys ? static_cast<const uint8_t *>(end_keys) : zero.data();
        std::vector<size_t> J(r);
        for (size_t j = 0; j < r; j++) J[j] = j;
        return s->resolve_list(J, start_kinds, sk, end_kinds, ek, raw_start, raw_end, local);
    } catch (const std::bad_alloc &) {
        return fail(RH_ERR_OOM, "resolve: host allocation failed");
    }
}

int rh_sstore_split_segments(rh_sstore *s, size_t m, const uint64_t *select_ranks, void *keys_out, size_t q,
                             const uint64_t *lo, const uint64_t *hi, rh_aggregate *out) {
    if (!s) return fail(RH_ERR_ARG, "sstore is NULL");
    if ((m && (!select_ranks || !keys_out)) || (q && (!lo || !hi || !out))) return fail(RH_ERR_ARG, "NULL buffer");
    if (m == 0 && q == 0) return RH_OK;
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);
    if (rc) return rc;
    try {
        return s->split_ranks(m, select_ranks, static_cast<uint8_t *>(keys_out), q, lo, hi, out);
    } catch (const std::bad_alloc &) {
        return fail(RH_ERR_OOM, "split: host allocation failed");
    }
}

int rh_sstore_protocol_round(rh_sstore *s, int policy, uint64_t fan_out, const rh_segments *active,
                             rh_segments *children, rh_segments *enumerations, rh_round_outcome *outcome) {
    if (!s || !active || !children || !enumerations) return fail(RH_ERR_ARG, "NULL");
    if (policy != RH_POLICY_FIXED_FAN_OUT && policy != RH_POLICY_SQRT_FAN_OUT) return fail(RH_ERR_ARG, "unknown policy");
    const size_t r = active->n;
    if (r && (!active->start_kinds || !active->end_kinds || !active->aggregates))
        return fail(RH_ERR_ARG, "active segments: NULL buffer");
    for (size_t j = 0; j < r; j++) {
        if (active->start_kinds[j] > 1 || active->end_kinds[j] > 1)
            return fail(RH_ERR_ARG, "segment bound kind must be 0 (Unbounded) or 1 (Included / Excluded)");
        if ((active->start_kinds[j] && !active->start_keys) || (active->end_kinds[j] && !active->end_keys))
            return fail(RH_ERR_ARG, "bound key is NULL");
    }
    *children = rh_segments{};
    *enumerations = rh_segments{};
    if (outcome) *outcome = rh_round_outcome{};
    if (r == 0) return RH_OK;
    std::unique_lock<std::mutex> g;
    int rc = lock_sizes(s, g);
    if (rc) return rc;
    try {
        rc = s->protocol_round(policy, fan_out, *active, children, enumerations, outcome);
    } catch (const std::bad_alloc &) {
        rc = fail(RH_ERR_OOM, "protocol round: host allocation failed");
    } catch (...) {  // nothing crosses the C ABI
        rc = fail(RH_ERR_STATE, "protocol round: internal error");
    }
    if (rc) {
        *children = rh_segments{};
        *enumerations = rh_segments{};
        if (outcome) *outcome = rh_round_outcome{};
    }
    return rc;
}

int rh_sstore_set_host_tier(rh_sstore *s, int enable, uint64_t round_max) {
    if (!s) return fail(RH_ERR_ARG, "sstore is NULL");
    std::lock_guard<std::mutex> g(s->mu);
    if (enable < 0 || enable > 1) return fail(RH_ERR_ARG, "bad host tier setting");
    const int rc = s->each(s->all(), [&](int t) -> int { return rh_store_set_host_tier(s->shards[t], enable, round_max); });
    s->tier_on = rc == RH_OK ? enable == 1 : false;
    s->round_max = round_max ? round_max : 128;
    return rc;
}

int rh_sstore_set_tier_policy(rh_sstore *s, int keep_fresh) {
    if (!s) return fail(RH_ERR_ARG, "sstore is NULL");
    std::lock_guard<std::mutex> g(s->mu);
    return s->each(s->all(), [&](int t) -> int { return rh_store_set_tier_policy(s->shards[t], keep_fresh); });
}

int rh_sstore_reserve(rh_sstore *s, uint64_t rows, uint64_t batch_rows) {
    if (!s) return fail(RH_ERR_ARG, "sstore is NULL");
    std::lock_guard<std::mutex> g(s->mu);
    const uint64_t per = (rows + s->G - 1) / s->G;
    return s->each(s->all(), [&](int t) -> int { return rh_store_reserve(s->shards[t], per + per / 8, batch_rows); });
}

int rh_sstore_compact(rh_sstore *s) {
    if (!s) return fail(RH_ERR_ARG, "sstore is NULL");
    std::lock_guard<std::mutex> g(s->mu);
    s->changed();
    return s->each(s->all(), [&](int t) -> int { return rh_store_compact(s->shards[t]); });
}

}  // extern "C"
