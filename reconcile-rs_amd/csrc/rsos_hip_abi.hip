// rsos_hip_abi.hip -- the C ABI of librsos_hip.so (include/rsos_hip.h): argument checking,
// schema dispatch, the end-to-end host helper, and the GPU-resident RSOS store.
//
// The store realises rsos::Rsos<K> (rsos/src/rsos_trait.rs:39-90) for fixed-width keys:
//   - records live in HBM in rank order (SoA columns), with per-record fingerprints and the
//     256-row block sums + 65536-row super-block sums -- the GPU form of the per-node
//     subtree Aggregate cache of FingerprintTreeMap (node.rs:54-91);
//   - the host keeps the key column for rank / select (rbsr's select returns &K, so keys
//     must be host-addressable) and answers them by binary search in the key's Ord;
//   - every call drains the store's stream before returning (one-snapshot-per-round,
//     rbsr/src/rsos_view.rs:36).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <memory>
#include <new>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rsos_hip.h"
#include "internal.hpp"
#include "host_tier.hpp"
#include "lift_kernels.hpp"
#include "small_batch.hpp"
#include "snapshot_kernels.hpp"
#include "store_kernels.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

// Failure injection for the error paths tests cannot otherwise reach (rh_debug_fail_point):
// the named point fails once, with RH_ERR_OOM, on this thread.
thread_local std::string g_fail_point;
bool fail_point(const char *name) {
    if (g_fail_point.empty() || g_fail_point != name) return false;
    g_fail_point.clear();
    return true;
}

// Foreground and background streams.  A question's kernels are one small workgroup each and
// latency-bound; the work a store does behind them (the host tier's refresh copies and prefix
// scans, the base's row prefix) launches grids of up to ~400 K workgroups that would fill every
// CU's slots and starve them (a 2.3 ms tiny round beside a refresh's 100 M-row prefix scan).  So
// background kernels run on streams with a CU mask without the last RSOS_HIP_BG_RESERVE (default
// 32) compute units, which stay free for the questions: with 32 (mask bits 224-255, CUs on every
// XCD) a no-wait drive beside a refresh took 0.38 ms against 2.5 ms unmasked; 8 (bits 248-255) did
// not help (profiles/r05_s19_nowait_ab.jsonl).  The store's own stream asks for the device's highest
// priority (RSOS_HIP_FORE_PRIORITY=0: not), which measured no difference on its own.  Either falls
// back to a plain stream where the runtime refuses it.  Copies stay on plain streams.
static hipError_t create_fore_stream(hipStream_t *st) {
    static const int prio = getenv("RSOS_HIP_FORE_PRIORITY") ? atoi(getenv("RSOS_HIP_FORE_PRIORITY")) : 1;
    int least = 0, greatest = 0;
    if (prio && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess && greatest != least &&
        hipStreamCreateWithPriority(st, hipStreamNonBlocking, greatest) == hipSuccess)
        return hipSuccess;
    (void)hipGetLastError();
    return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
}
static hipError_t create_back_stream(hipStream_t *st, int device) {
    static const int reserve = getenv("RSOS_HIP_BG_RESERVE") ? atoi(getenv("RSOS_HIP_BG_RESERVE")) : 32;
    int ncu = 0;
    if (reserve > 0 && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        ncu > 4 * reserve) {
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
        for (int c = 0; c < ncu - reserve; c++) mask[(size_t)c / 32] |= 1u << (c % 32);
        const hipError_t e = hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data());
        if (getenv("RSOS_HIP_STREAM_DBG")) {
            std::vector<uint32_t> got(mask.size(), 0u);
            if (e == hipSuccess) (void)hipExtStreamGetCUMask(*st, (uint32_t)got.size(), got.data());
            fprintf(stderr, "{\"back_stream\": {\"cus\": %d, \"reserve\": %d, \"created\": %d, \"mask_last_word\": \"%08x\"}}\n",
                    ncu, reserve, e == hipSuccess, got.empty() ? 0u : got.back());
        }
        if (e == hipSuccess) return hipSuccess;
    }
    (void)hipGetLastError();
    return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
}
// The background streams every store on a device shares, one per role (0: the tier refresh's
// kernels, 1: the row prefix), created once and kept for the process.  A CU mask is a property of
// a hardware queue, so each CU-masked stream takes a queue of its own: one pair per store made 20
// queues for 8 shards + their peers on one GPU, and device rounds stalled 8-20 ms behind the queue
// scheduler (profiles/r06_sstore8_stalls.txt).  The stores' work on them is ordered by events;
// sharing only serialises background work of different stores.  RSOS_HIP_SHARED_BG=0: per store.
static bool shared_back_streams() {
    static const bool on = !getenv("RSOS_HIP_SHARED_BG") || atoi(getenv("RSOS_HIP_SHARED_BG")) != 0;
    return on;
}
// Counted by the stores holding them: the last store of a device to let go destroys the stream, so
// none outlives its stores into the runtime's teardown (a profiler's tool had already finalised
// there and crashed on one left over).
struct BackStreams {
    std::mutex mu;
    std::vector<hipStream_t> made;  // [2 device + role]
    std::vector<int> users;
};
static BackStreams &back_streams() {
    static BackStreams *b = new BackStreams();  // never destroyed: stores may outlive static teardown
    return *b;
}
static hipError_t back_stream(int device, int role, hipStream_t *st) {
    if (!shared_back_streams()) return create_back_stream(st, device);
    BackStreams &b = back_streams();
    std::lock_guard<std::mutex> g(b.mu);
    const size_t k = 2 * (size_t)device + (size_t)role;
    if (b.made.size() <= k) b.made.resize(k + 1, nullptr), b.users.resize(k + 1, 0);
    if (!b.made[k]) {
        const hipError_t e = create_back_stream(&b.made[k], device);
        if (e != hipSuccess) {
            b.made[k] = nullptr;
            return e;
        }
    }
    b.users[k]++;
    *st = b.made[k];
    return hipSuccess;
}
// a store lets go of its background stream (its work on it has been waited for)
static void back_stream_put(int device, int role, hipStream_t st) {
    if (!st) return;
    if (!shared_back_streams()) {
        (void)hipStreamDestroy(st);
        return;
    }
    BackStreams &b = back_streams();
    std::lock_guard<std::mutex> g(b.mu);
    const size_t k = 2 * (size_t)device + (size_t)role;
    if (k < b.made.size() && b.made[k] == st && --b.users[k] == 0) {
        (void)hipStreamDestroy(st);
        b.made[k] = nullptr;
    }
}

// rh_debug_batch_timing: HIP events around every large batch's fused lift + search launch
std::atomic<int> g_time_batch{0};
std::mutex g_batch_mu;
double g_batch_us = 0;
uint64_t g_batch_n = 0;

#define RH_HIP(expr)                                                                           \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(e_ == hipErrorOutOfMemory ? RH_ERR_OOM : RH_ERR_HIP,                   \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                    \
    } while (0)

bool aligned16(const void *p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

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

int check_schema(const rh_schema *s) {
    if (!s) return fail(RH_ERR_ARG, "schema is NULL");
    if (s->key_kind < 0 || s->key_kind > 3) return fail(RH_ERR_ARG, "bad key_kind");
    if (s->value_kind < 0 || s->value_kind > 3) return fail(RH_ERR_ARG, "bad value_kind");
    if (s->record_kind < 0 || s->record_kind > 2) return fail(RH_ERR_ARG, "bad record_kind");
    if (s->reserved != 0) return fail(RH_ERR_ARG, "schema.reserved must be 0");
    if (s->key_kind == RH_KEY_U32 && s->key_len != 4) return fail(RH_ERR_ARG, "u32 key needs key_len 4");
    if (s->key_kind == RH_KEY_U64 && s->key_len != 8) return fail(RH_ERR_ARG, "u64 key needs key_len 8");
    if (s->value_kind == RH_VAL_U32 && s->value_len != 4) return fail(RH_ERR_ARG, "u32 value needs value_len 4");
    if (s->value_kind == RH_VAL_U64 && s->value_len != 8) return fail(RH_ERR_ARG, "u64 value needs value_len 8");
    return RH_OK;
}

rh::DevCols to_dev(const rh_columns &c) {
    rh::DevCols d;
    d.keys = static_cast<const uint8_t *>(c.keys);
    d.phys = c.phys;
    d.logical = c.logical;
    d.node = c.node;
    d.tags = c.tags;
    d.values = static_cast<const uint8_t *>(c.values);
    return d;
}

int check_cols(const rh_schema &s, const rh_columns *c, size_t n) {
    if (!c) return fail(RH_ERR_ARG, "columns is NULL");
    if (n == 0) return RH_OK;
    if (s.key_kind != RH_KEY_UNIT && !c->keys) return fail(RH_ERR_ARG, "keys column is NULL");
    if (s.value_kind != RH_VAL_UNIT && !c->values) return fail(RH_ERR_ARG, "values column is NULL");
    if (s.record_kind == RH_REC_DATED && (!c->phys || !c->logical || !c->node))
        return fail(RH_ERR_ARG, "DATED records need phys / logical / node columns");
    if (!aligned16(c->keys) || !aligned16(c->values) || !aligned16(c->phys) || !aligned16(c->node) ||
        !aligned16(c->logical))
        return fail(RH_ERR_ARG, "device columns must be 16-byte aligned");
    return RH_OK;
}

// dst_row (optional, single lift without block sums): record i's fingerprint to row dst_row[i]
int lift_dispatch(const rh_schema &s, const rh_columns &c, size_t n, uint8_t *fps, uint8_t *bs,
                  uint8_t *fps2, uint8_t *bs2, bool dual, hipStream_t st, const uint32_t *dst_row = nullptr,
                  const uint32_t *dst2 = nullptr) {
    bool supported = false;
    if (dst_row && (bs || dual)) return fail(RH_ERR_STATE, "lift to sorted rows: no block sums (internal error)");
    rh::DevCols dc = to_dev(c);
    dc.dst = dst_row;
    dc.dst2 = dst2;
    hipError_t e = rh::launch_lift_schema(s.key_kind, (int)s.key_len, s.value_kind, (int)s.value_len,
                                          s.record_kind, c.tags != nullptr, dual, dc, n, fps, bs,
                                          fps2, bs2, st, &supported);
    if (!supported)
        return fail(RH_ERR_UNSUPPORTED,
                    "no specialised lift kernel for this schema; canonical-encode on the host and "
                    "use rh_lift_encoded_async");
    if (e != hipSuccess) return fail(RH_ERR_HIP, std::string("lift launch: ") + hipGetErrorString(e));
    return RH_OK;
}

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;  // elements
    // Grows geometrically (x1.5): a run that gains a batch of rows per call (the delta run) is
    // reallocated O(log n) times, not every call -- hipFree drains the device, and one
    // realloc per batch cost ~0.6 ms of idle GPU per config5 batch.
    int ensure(size_t n) {
        if (n <= cap && p) return RH_OK;
        static const bool dbg = getenv("RSOS_HIP_ALLOC_DBG") != nullptr;  // every reallocation, to stderr
        if (dbg && p)
            fprintf(stderr, "rsos_hip: DevBuf<%zu B> %p grows %zu -> %zu elements (caller %p)\n", sizeof(T), (void *)this,
                    cap, n, __builtin_return_address(0));
        if (p) (void)hipFree(p);
        p = nullptr;
        const size_t grown = cap + cap / 2;
        cap = 0;
        size_t bytes = std::max<size_t>(std::max(n, grown), 1) * sizeof(T);
        bytes = (bytes + 255) & ~size_t(255);
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) return fail(RH_ERR_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
        cap = bytes / sizeof(T);
        return RH_OK;
    }
    // grow to n elements keeping the first `used` ones (ordered on `st`); geometric, as ensure():
    // an unreserved store's record heap gains a batch per call and must not copy itself each time
    int grow_keep(size_t n, size_t used, hipStream_t st) {
        if (n <= cap && p) return RH_OK;
        if (p) n = std::max(n, cap + cap / 2);
        T *q = nullptr;
        const size_t bytes = ((std::max<size_t>(n, 1) * sizeof(T)) + 255) & ~size_t(255);
        hipError_t e = hipMalloc(&q, bytes);
        if (e != hipSuccess) return fail(RH_ERR_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
        if (p && used) {
            e = hipMemcpyAsync(q, p, used * sizeof(T), hipMemcpyDeviceToDevice, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) {
                (void)hipFree(q);
                return fail(RH_ERR_HIP, std::string("grow: ") + hipGetErrorString(e));
            }
        }
        if (p) (void)hipFree(p);
        p = q;
        cap = bytes / sizeof(T);
        return RH_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace

namespace rh {
int set_error(int code, const std::string &msg) { return fail(code, msg); }
bool debug_fail_point(const char *name) { return fail_point(name); }
}  // namespace rh

// ---- dispatch table over the instantiated shapes (schemas.def) -------------------------------
namespace rh {
#define X(name, kk, kl, vk, vl)                                                                   \
    hipError_t launch_lift_##name(int rk, bool tags, bool dual, const DevCols &c, uint64_t n,    \
                                  uint8_t *fps, uint8_t *bsums, uint8_t *fps2, uint8_t *bsums2, \
                                  hipStream_t st);
#include "schemas.def"
#undef X

bool schema_instantiated(int kk, int kl, int vk, int vl) {
#define X(name, KK, KL, VK, VL) \
    if (kk == KK && kl == KL && vk == VK && vl == VL) return true;
#include "schemas.def"
#undef X
    return false;
}

hipError_t launch_lift_schema(int kk, int kl, int vk, int vl, int rk, bool tags, bool dual,
                              const DevCols &c, uint64_t n, uint8_t *fps, uint8_t *bsums,
                              uint8_t *fps2, uint8_t *bsums2, hipStream_t st, bool *supported) {
    *supported = true;
#define X(name, KK, KL, VK, VL)                                                                   \
    if (kk == KK && kl == KL && vk == VK && vl == VL)                                            \
        return launch_lift_##name(rk, tags, dual, c, n, fps, bsums, fps2, bsums2, st);
#include "schemas.def"
#undef X
    *supported = false;
    return hipSuccess;
}

#define X(name, kk, kl, vk, vl)                                                                               \
    hipError_t launch_lift_search_##name(int rk, bool tags, const DevCols &c, uint64_t n, uint8_t *fps,          \
                                         const uint8_t *q, const SearchJob &jb, const SearchJob &jd,             \
                                         const NextMinmax &nx, hipStream_t st, bool *supported, hipEvent_t ev0,  \
                                         hipEvent_t ev1);
#include "schemas.def"
#undef X

hipError_t launch_lift_search_schema(int kk, int kl, int vk, int vl, int rk, bool tags, const DevCols &c, uint64_t n,
                                     uint8_t *fps, const uint8_t *q, const SearchJob &jb, const SearchJob &jd,
                                     const NextMinmax &nx, hipStream_t st, bool *supported, hipEvent_t ev0,
                                     hipEvent_t ev1) {
#define X(name, KK, KL, VK, VL)                           \
    if (kk == KK && kl == KL && vk == VK && vl == VL)     \
        return launch_lift_search_##name(rk, tags, c, n, fps, q, jb, jd, nx, st, supported, ev0, ev1);
#include "schemas.def"
#undef X
    *supported = false;
    return hipSuccess;
}

#define X(name, kk, kl, vk, vl) \
    hipError_t launch_snap_lift_##name(int mode, const SnapLift &a, uint64_t lds, hipStream_t st, bool *supported);
#include "schemas.def"
#undef X

hipError_t launch_snap_lift_schema(int kk, int kl, int vk, int vl, int mode, const SnapLift &a, uint64_t lds,
                                   hipStream_t st, bool *supported) {
#define X(name, KK, KL, VK, VL) \
    if (kk == KK && kl == KL && vk == VK && vl == VL) return launch_snap_lift_##name(mode, a, lds, st, supported);
#include "schemas.def"
#undef X
    *supported = false;
    return hipSuccess;
}

#define X(name, kk, kl, vk, vl) \
    hipError_t launch_small_batch_##name(int rk, bool tags, const SmallBatch &a, hipStream_t st, bool *supported);
#include "schemas.def"
#undef X

hipError_t launch_small_batch_schema(int kk, int kl, int vk, int vl, int rk, bool tags, const SmallBatch &a,
                                     hipStream_t st, bool *supported) {
#define X(name, KK, KL, VK, VL) \
    if (kk == KK && kl == KL && vk == VK && vl == VL) return launch_small_batch_##name(rk, tags, a, st, supported);
#include "schemas.def"
#undef X
    *supported = false;
    return hipSuccess;
}
}  // namespace rh

// =================================================================================================
extern "C" {

int rh_abi_version(void) { return RH_ABI_VERSION; }

const char *rh_last_error(void) { return g_err.c_str(); }

int rh_schema_supported(const rh_schema *schema) {
    int rc = check_schema(schema);
    if (rc) return rc;
    const rh_schema &s = *schema;
    return rh::schema_instantiated(s.key_kind, (int)s.key_len, s.value_kind, (int)s.value_len) ? 1 : 0;
}

int64_t rh_schema_record_len(const rh_schema *schema, int tombstone) {
    int rc = check_schema(schema);
    if (rc) return rc;
    const rh_schema &s = *schema;
    int64_t key = s.key_kind == RH_KEY_BYTES ? 8 + (int64_t)s.key_len : key_row(s);
    int64_t stamp = s.record_kind == RH_REC_DATED ? 20 : 0;
    if (s.record_kind == RH_REC_PLAIN) tombstone = 0;
    int64_t tag = s.record_kind == RH_REC_PLAIN ? 0 : 4;
    int64_t val = tombstone ? 0 : (s.value_kind == RH_VAL_BYTES ? 8 + (int64_t)s.value_len : value_row(s));
    return key + stamp + tag + val;
}

size_t rh_num_blocks(size_t n) { return (n + RH_BLOCK - 1) / RH_BLOCK; }
size_t rh_num_superblocks(size_t n) { return (n + RH_SUPER - 1) / RH_SUPER; }

int rh_lift_records_async(const rh_schema *schema, const rh_columns *cols, size_t n, uint8_t *fps,
                          uint8_t *block_sums, void *stream) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if ((rc = check_cols(*schema, cols, n))) return rc;
    if (n && !fps) return fail(RH_ERR_ARG, "fps is NULL");
    if (!aligned16(fps) || !aligned16(block_sums)) return fail(RH_ERR_ARG, "outputs must be 16-byte aligned");
    return lift_dispatch(*schema, *cols, n, fps, block_sums, nullptr, nullptr, false,
                         static_cast<hipStream_t>(stream));
}

int rh_lift_dual_async(const rh_schema *schema, const rh_columns *cols, size_t n, uint8_t *fps_d,
                       uint8_t *bs_d, uint8_t *fps_p, uint8_t *bs_p, void *stream) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if (schema->record_kind != RH_REC_DATED) return fail(RH_ERR_ARG, "dual lift needs record_kind DATED");
    if ((rc = check_cols(*schema, cols, n))) return rc;
    if (n && (!fps_d || !fps_p)) return fail(RH_ERR_ARG, "fps outputs are NULL");
    if (!aligned16(fps_d) || !aligned16(fps_p) || !aligned16(bs_d) || !aligned16(bs_p))
        return fail(RH_ERR_ARG, "outputs must be 16-byte aligned");
    return lift_dispatch(*schema, *cols, n, fps_d, bs_d, fps_p, bs_p, true, static_cast<hipStream_t>(stream));
}

int rh_lift_encoded_async(const uint8_t *bytes, size_t bytes_len, const uint64_t *offsets, size_t n, uint8_t *fps,
                          uint8_t *block_sums, void *stream) {
    if (n == 0) return RH_OK;
    if (!offsets || !fps) return fail(RH_ERR_ARG, "offsets / fps is NULL");
    if (bytes_len && !bytes) return fail(RH_ERR_ARG, "bytes is NULL");
    if (bytes_len % 4) return fail(RH_ERR_ARG, "bytes_len must be a multiple of 4 (pad the buffer)");
    if (reinterpret_cast<uintptr_t>(bytes) % 4) return fail(RH_ERR_ARG, "bytes must be 4-byte aligned");
    if (!aligned16(fps) || !aligned16(block_sums)) return fail(RH_ERR_ARG, "outputs must be 16-byte aligned");
    // no host round trip: bytes_len bounds every read, whatever the offsets say
    RH_HIP(rh::launch_lift_encoded(bytes, offsets, n, bytes_len, fps, block_sums, static_cast<hipStream_t>(stream)));
    return RH_OK;
}

int rh_lift_fixed_async(const uint8_t *bytes, size_t bytes_len, size_t record_len, size_t n, uint8_t *fps,
                        uint8_t *block_sums, void *stream) {
    if (n == 0) return RH_OK;
    if (!fps) return fail(RH_ERR_ARG, "fps is NULL");
    if (bytes_len && !bytes) return fail(RH_ERR_ARG, "bytes is NULL");
    if (bytes_len % 4) return fail(RH_ERR_ARG, "bytes_len must be a multiple of 4 (pad the buffer)");
    if (reinterpret_cast<uintptr_t>(bytes) % 4) return fail(RH_ERR_ARG, "bytes must be 4-byte aligned");
    if (record_len && n > bytes_len / record_len) return fail(RH_ERR_ARG, "n * record_len exceeds bytes_len");
    if (!aligned16(fps) || !aligned16(block_sums)) return fail(RH_ERR_ARG, "outputs must be 16-byte aligned");
    RH_HIP(rh::launch_lift_fixed(bytes, record_len, n, bytes_len, fps, block_sums, static_cast<hipStream_t>(stream)));
    return RH_OK;
}

int rh_reduce_blocks_async(const uint8_t *in, size_t n_in, uint8_t *out, void *stream) {
    if (n_in && (!in || !out)) return fail(RH_ERR_ARG, "NULL buffer");
    if (!aligned16(in) || !aligned16(out)) return fail(RH_ERR_ARG, "buffers must be 16-byte aligned");
    RH_HIP(rh::launch_reduce(in, n_in, out, static_cast<hipStream_t>(stream)));
    return RH_OK;
}

int rh_range_aggregates_async(const uint8_t *fps, const uint8_t *bsums, const uint8_t *ssums, size_t n,
                              const uint64_t *lo, const uint64_t *hi, size_t r, rh_aggregate *out,
                              void *stream) {
    if (r == 0) return RH_OK;
    if (!lo || !hi || !out || (n && !fps)) return fail(RH_ERR_ARG, "NULL buffer");
    if (!aligned16(fps) || !aligned16(bsums) || !aligned16(ssums)) return fail(RH_ERR_ARG, "sums must be 16-byte aligned");
    if (ssums && !bsums) return fail(RH_ERR_ARG, "super-block sums need block sums");
    RH_HIP(rh::launch_range_query(fps, bsums, ssums, n, lo, hi, r, reinterpret_cast<uint64_t *>(out),
                                  static_cast<hipStream_t>(stream)));
    return RH_OK;
}

int rh_combine_aggregates_async(const rh_aggregate *in, size_t parts, size_t r, rh_aggregate *out, void *stream) {
    if (r == 0) return RH_OK;
    if (!in || !out) return fail(RH_ERR_ARG, "NULL buffer");
    RH_HIP(rh::launch_combine(reinterpret_cast<const uint64_t *>(in), parts, r, reinterpret_cast<uint64_t *>(out),
                              static_cast<hipStream_t>(stream)));
    return RH_OK;
}

void rh_fp_add(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
    unsigned __int128 carry = 0;
    for (int i = 0; i < 4; i++) {
        unsigned __int128 s = (unsigned __int128)a[i] + b[i] + carry;
        out[i] = (uint64_t)s;
        carry = s >> 64;
    }
}

void rh_fp_sub(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
    uint64_t borrow = 0;
    for (int i = 0; i < 4; i++) {
        uint64_t ai = a[i], bi = b[i];
        uint64_t d = ai - bi - borrow;
        borrow = (ai < bi) || (ai - bi < borrow);
        out[i] = d;
    }
}

}  // extern "C"

// =================================================================================================
// Device column set: owned copies of a batch's columns in HBM
namespace {

struct DevColumns {
    DevBuf<uint8_t> keys, values, tags;
    DevBuf<uint64_t> phys, node;
    DevBuf<uint32_t> logical;
    bool has_tags = false;

    int upload(const rh_schema &s, const rh_columns &h, size_t n, hipStream_t st) {
        int rc;
        const size_t kr = key_row(s), vr = value_row(s);
        if ((rc = keys.ensure(n * kr + 16))) return rc;
        if ((rc = values.ensure(n * vr + 16))) return rc;
        // a NULL host column (e.g. the values of a delete-only batch) is zero-filled
        auto put = [&](void *dst, const void *src, size_t bytes) -> hipError_t {
            if (!bytes) return hipSuccess;
            return src ? hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st) : hipMemsetAsync(dst, 0, bytes, st);
        };
        RH_HIP(put(keys.p, h.keys, n * kr));
        RH_HIP(put(values.p, h.values, n * vr));
        if (s.record_kind == RH_REC_DATED) {
            if ((rc = phys.ensure(n)) || (rc = node.ensure(n)) || (rc = logical.ensure(n))) return rc;
            RH_HIP(put(phys.p, h.phys, n * 8));
            RH_HIP(put(node.p, h.node, n * 8));
            RH_HIP(put(logical.p, h.logical, n * 4));
        }
        has_tags = h.tags != nullptr && s.record_kind != RH_REC_PLAIN;
        if (has_tags) {
            if ((rc = tags.ensure(n + 16))) return rc;
            if (n) RH_HIP(hipMemcpyAsync(tags.p, h.tags, n, hipMemcpyHostToDevice, st));
        }
        return RH_OK;
    }
    rh_columns view(const rh_schema &s) const {
        rh_columns c;
        c.keys = keys.p;
        c.values = values.p;
        c.phys = s.record_kind == RH_REC_DATED ? phys.p : nullptr;
        c.node = s.record_kind == RH_REC_DATED ? node.p : nullptr;
        c.logical = s.record_kind == RH_REC_DATED ? logical.p : nullptr;
        c.tags = has_tags ? tags.p : nullptr;
        return c;
    }
    void release() {
        keys.release(); values.release(); tags.release();
        phys.release(); node.release(); logical.release();
    }
};

}  // namespace

namespace {

// The host path as a pipeline, kept per device between calls: chunk k's columns go up on the
// copy-in stream while chunk k-1 is lifted and chunk k-2's fingerprints come down on the
// copy-out stream.  PCIe is full duplex, so a run costs about its host-to-device copy alone
// (pinned host buffers; pageable ones are staged by the runtime and serialise).
struct HostPipe {
    static constexpr int DEPTH = 3;
    hipStream_t in = nullptr, comp = nullptr, out = nullptr;
    DevColumns cols[DEPTH];
    DevBuf<uint8_t> fps[DEPTH];
    hipEvent_t up[DEPTH] = {}, down[DEPTH] = {}, lifted[DEPTH] = {};
    std::mutex mu;
    int init() {
        if (in) return RH_OK;
        RH_HIP(hipStreamCreateWithFlags(&in, hipStreamNonBlocking));
        RH_HIP(hipStreamCreateWithFlags(&comp, hipStreamNonBlocking));
        RH_HIP(hipStreamCreateWithFlags(&out, hipStreamNonBlocking));
        for (int b = 0; b < DEPTH; b++) {
            RH_HIP(hipEventCreateWithFlags(&up[b], hipEventDisableTiming));
            RH_HIP(hipEventCreateWithFlags(&lifted[b], hipEventDisableTiming));
            RH_HIP(hipEventCreateWithFlags(&down[b], hipEventDisableTiming));
        }
        return RH_OK;
    }
};

HostPipe &host_pipe(int device) {
    static std::mutex m;
    static std::vector<std::unique_ptr<HostPipe>> pipes;
    std::lock_guard<std::mutex> g(m);
    if ((int)pipes.size() <= device) pipes.resize(device + 1);
    if (!pipes[device]) pipes[device].reset(new HostPipe());
    return *pipes[device];
}

rh_columns host_rows(const rh_schema &s, const rh_columns &h, size_t at) {
    const size_t kr = key_row(s), vr = value_row(s);
    rh_columns c = h;
    if (c.keys) c.keys = static_cast<const uint8_t *>(c.keys) + at * kr;
    if (c.values) c.values = static_cast<const uint8_t *>(c.values) + at * vr;
    if (c.phys) c.phys += at;
    if (c.logical) c.logical += at;
    if (c.node) c.node += at;
    if (c.tags) c.tags += at;
    return c;
}

}  // namespace

extern "C" int rh_lift_host(int device, const rh_schema *schema, const rh_columns *h, size_t n, uint8_t *host_fps) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if (!h) return fail(RH_ERR_ARG, "columns is NULL");
    if (n == 0) return RH_OK;
    if (!host_fps) return fail(RH_ERR_ARG, "host_fps is NULL");
    RH_HIP(hipSetDevice(device));
    HostPipe &p = host_pipe(device);
    std::lock_guard<std::mutex> g(p.mu);
    if ((rc = p.init())) return rc;
    // ~128 MB of record columns per chunk
    const size_t rec = key_row(*schema) + value_row(*schema) + 21;
    const size_t chunk = std::max<size_t>(65536, (128u << 20) / rec);
    for (size_t k = 0, at = 0; at < n; k++, at += chunk) {
        const int b = (int)(k % HostPipe::DEPTH);
        const size_t c = std::min(chunk, n - at);
        // buffer set b is free once chunk k - DEPTH's fingerprints are down
        if (k >= (size_t)HostPipe::DEPTH) RH_HIP(hipStreamWaitEvent(p.in, p.down[b], 0));
        if ((rc = p.cols[b].upload(*schema, host_rows(*schema, *h, at), c, p.in)) || (rc = p.fps[b].ensure(chunk * 32)))
            return rc;
        RH_HIP(hipEventRecord(p.up[b], p.in));
        RH_HIP(hipStreamWaitEvent(p.comp, p.up[b], 0));
        if ((rc = lift_dispatch(*schema, p.cols[b].view(*schema), c, p.fps[b].p, nullptr, nullptr, nullptr, false,
                                p.comp)))
            return rc;
        RH_HIP(hipEventRecord(p.lifted[b], p.comp));
        RH_HIP(hipStreamWaitEvent(p.out, p.lifted[b], 0));
        RH_HIP(hipMemcpyAsync(host_fps + at * 32, p.fps[b].p, c * 32, hipMemcpyDeviceToHost, p.out));
        RH_HIP(hipEventRecord(p.down[b], p.out));
    }
    RH_HIP(hipStreamSynchronize(p.out));
    return RH_OK;
}

extern "C" int rh_host_alloc(size_t bytes, void **out) {
    if (!out) return fail(RH_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (!bytes) return RH_OK;
    RH_HIP(hipHostMalloc(out, bytes, hipHostMallocDefault));
    return RH_OK;
}

extern "C" int rh_host_free(void *p) {
    if (p) RH_HIP(hipHostFree(p));
    return RH_OK;
}

// =================================================================================================
// The GPU-resident store: an LSM of a sorted base run and a sorted signed-delta run (see
// store_kernels.hip).  Batches merge into the delta run in O(batch + delta); the delta run is
// merged into the base when it passes base / compact_div, and before any rank-order query
// (select, rank-range aggregates, key / fingerprint dumps).  Key-range aggregates and ranks
// are answered from base + delta without compaction.
// Page-locked host array with the part of std::vector's interface the protocol round uses:
// the round's copies in and out of HBM then run at PCIe speed without a staging copy.
template <class T>
struct PinnedVec {
    T *p = nullptr;
    size_t n = 0, cap = 0;
    // hipHostMallocMapped: the buffer also has a device address (hipHostGetDevicePointer), so a
    // kernel may read it or write it in place; the writes are visible to the host once the
    // stream has synchronised (the kernel's end-of-dispatch release), or after a system-scope
    // fence in the kernel (the small batch's sequence word)
    unsigned flags = hipHostMallocMapped | hipHostMallocPortable;
    void *dptr = nullptr;          // the device address of p, once looked up (store.dev_ptr)
    const void *dptr_of = nullptr;  // ... and the allocation it belongs to
    PinnedVec() = default;
    // extra allocation flags: hipHostMallocCoherent for a buffer the host polls while a kernel
    // writes it (a sequence word stored last), so the poll never depends on HIP_HOST_COHERENT
    explicit PinnedVec(unsigned extra) : flags(hipHostMallocMapped | hipHostMallocPortable | extra) {}
    PinnedVec(const PinnedVec &) = delete;
    PinnedVec &operator=(const PinnedVec &) = delete;
    ~PinnedVec() { release(); }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = cap = 0;
        dptr = nullptr;
    }
    void reserve(size_t want) {
        if (want <= cap) return;
        const size_t c = std::max<size_t>(std::max(want, cap + cap / 2), 64);
        T *q = nullptr;
        if (hipHostMalloc(reinterpret_cast<void **>(&q), c * sizeof(T), flags) != hipSuccess || !q)
            throw std::bad_alloc();
        if (n) memcpy(q, p, n * sizeof(T));
        if (p) (void)hipHostFree(p);
        p = q;
        cap = c;
        dptr = nullptr;  // a new allocation: its device address is looked up again
    }
    void resize(size_t m) { reserve(m); n = m; }
    void assign(size_t m, uint8_t byte) { resize(m); memset(p, byte, m * sizeof(T)); }
    void clear() { n = 0; }
    void push_back(const T &v) {
        if (n == cap) reserve(n + 1);
        p[n++] = v;
    }
    size_t size() const { return n; }
    size_t capacity() const { return cap; }
    bool empty() const { return n == 0; }
    T *data() { return p; }
    T &operator[](size_t i) { return p[i]; }
    const T &operator[](size_t i) const { return p[i]; }
};

// a PinnedVec's device address, type-erased (the copy list of rh_store::copy_down)
struct PinnedAny {
    void **dptr;
    const void **dptr_of;
    void *p;
    template <class T>
    PinnedAny(PinnedVec<T> &v) : dptr(&v.dptr), dptr_of(&v.dptr_of), p(v.p) {}
    int lookup(uint8_t **dev) const {  // 0 on success
        if (!*dptr || *dptr_of != p) {
            void *d = nullptr;
            if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d) {
                (void)hipGetLastError();
                return 1;
            }
            *dptr = d;
            *dptr_of = p;
        }
        *dev = static_cast<uint8_t *>(*dptr);
        return 0;
    }
};

struct rh_store {
    int device = 0;
    rh_schema schema{};
    hipStream_t stream = nullptr;
    std::mutex mu;  // serialises callers sharing one store (readers under a RwLock read guard)
    rh::StoreKeyOps *kops = nullptr;
    size_t kl = 0;
    // base run
    uint64_t nb = 0;
    int cb = 0;
    DevBuf<uint8_t> bkeys[2], bfps[2], bsums, ssums;
    DevBuf<uint64_t> bsmp, bsmp2;  // leading digits of every 256th (8th) key: sampled search
    DevBuf<uint32_t> btab;         // the base run's search table over bsmp2 (k_search_table)
    DevBuf<uint32_t> dtab;         // the delta run's, built before each batch's delta search
    DevBuf<uint64_t> dtabp;
    DevBuf<uint64_t> btabp;
    rh::SearchTable base_table() const { return rh::SearchTable{btab.p, btabp.p, rh::search_table_bits(nb)}; }
    DevBuf<uint64_t> dsmp[2], dsmp2[2];  // the same for each delta buffer (written by its merge)
    // delta run
    uint64_t nd = 0;
    int cd = 0;
    int64_t dtotal = 0;  // Σ count deltas
    DevBuf<uint8_t> dkeys[2], dbsums[2], dssums[2];
    DevBuf<uint32_t> dslot[2];  // the delta rows' record slots in dheap
    DevBuf<uint8_t> dheap;      // DeltaRecs, appended per batch (slots heap_len ..), emptied by compaction
    uint64_t heap_len = 0;
    DevBuf<int32_t> dblk[2];  // inclusive block prefix of the count deltas
    DevBuf<int16_t> dinb[2];  // each row's inclusive count prefix inside its 256-row block
    DevBuf<int32_t> dsblk[2];  // exclusive super-block prefix of the count deltas
    DevBuf<int32_t> dscnt;     // k_delta_finish's per-super-block count totals
    DevBuf<uint32_t> fin_ticket;
    DevBuf<uint64_t> mcnt;    // merge counters
    uint64_t compact_div = 6, compact_min = 65536, compactions = 0;  // 6: the measured optimum (profiles/r03_c5_divisor_sweep_64.txt)
    // the whole-map fingerprint = base total + delta contribution total, kept on the host after
    // every load / batch / compaction (the reference's root node Aggregate): aggregate(..) is O(1)
    uint64_t root_b[4] = {0, 0, 0, 0}, root_d[4] = {0, 0, 0, 0};
    DevBuf<uint64_t> tot;
    // batch scratch
    DevColumns staging;
    DevBuf<uint8_t> skeys, sfps, sops, hops, dops, cfps, cops;
    DevBuf<uint64_t> counts, results;
    DevBuf<uint32_t> flag;
    // query scratch
    DevBuf<uint64_t> q_lo, q_hi, q_dlo, q_dhi, q_merged;
    DevBuf<rh_aggregate> q_out, q_bout, q_dout;
    DevBuf<uint8_t> q_keys;
    DevBuf<uint32_t> q_rank, q_drank;
    DevBuf<uint8_t> snap;  // a host snapshot's bytes while it is decoded
    rh::Scratch scratch;

    uint64_t size() const { return (uint64_t)((int64_t)nb + dtotal); }
    // After a failed load: drain the stream (no copy into host state still in flight) and leave
    // the store empty, its size and root consistent
    void reset_empty() {
        (void)hipStreamSynchronize(stream);
        (void)hipGetLastError();
        nb = nd = 0;
        heap_len = 0;
        dtotal = 0;
        memset(root_b, 0, sizeof root_b);
        memset(root_d, 0, sizeof root_d);
        version++;
        base_epoch++;
    }
    // ---- the pending batch (rh_store_stage) --------------------------------------------------------
    // Single-record inserts and deletes (Rsos::insert / delete, FingerprintTreeMap::insert /
    // remove, mutate.rs:23-154) queue here on the host and reach the device as one batch
    // (rh_store_apply's path) before anything reads the store: the one-device-batch-per-round
    // shape of just_insert_bulk (src/replica/write.rs:107-121), never one device round trip per
    // record.  A key staged twice keeps its last operation -- the result of applying them in order.
    struct Pending {
        std::vector<uint8_t> keys, vals, tags, ops;
        std::vector<uint64_t> phys, node;
        std::vector<uint32_t> logical;
        size_t n = 0;
        void clear() {
            keys.clear(), vals.clear(), tags.clear(), ops.clear(), phys.clear(), node.clear(), logical.clear();
            n = 0;
        }
    } pend;
    int stage(const rh_columns &h, const uint8_t *ops, size_t m) {
        const size_t kr = kl, vr = value_row(schema);
        const bool dated = schema.record_kind == RH_REC_DATED;
        auto app = [](auto &v, const auto *src, size_t cnt) {
            if (src) v.insert(v.end(), src, src + cnt);
            else v.resize(v.size() + cnt);
        };
        app(pend.keys, static_cast<const uint8_t *>(h.keys), m * kr);
        app(pend.vals, static_cast<const uint8_t *>(h.values), m * vr);
        app(pend.tags, h.tags, m);
        app(pend.ops, ops, m);
        if (dated) {
            app(pend.phys, h.phys, m);
            app(pend.node, h.node, m);
            app(pend.logical, h.logical, m);
        }
        pend.n += m;
        return RH_OK;
    }
    int key_cmp(const uint8_t *a, const uint8_t *b) const {
        if (schema.key_kind == RH_KEY_U32 || schema.key_kind == RH_KEY_U64) {
            uint64_t x = 0, y = 0;
            memcpy(&x, a, kl);
            memcpy(&y, b, kl);
            return (x > y) - (x < y);
        }
        return memcmp(a, b, kl);
    }
    // One batch: the staged rows as they were staged, in one call -- the device sorts them (stably,
    // so the last operation staged for a key is the last of its run) and keeps the last row of each
    // repeated key: the result of applying them in order (just_insert_bulk,
    // src/replica/write.rs:107-121).  A batch of up to small_batch_max rows takes the one-workgroup
    // path (apply_small, reading the rows from page-locked host memory); larger ones go up in one
    // copy per column.  No host sort, no per-row host work.
    // A small batch commits on the host once k_small_batch's sequence word lands; the delta merge
    // behind it may still run.  Its completion is checked (an event) when the store is next
    // entered: a merge that failed leaves the host's bookkeeping ahead of the device, so the store
    // refuses every call with that error -- attributed to the batch -- until a load replaces the
    // contents.  Fail point "small_batch.merge" reports the next small batch's merge as failed.
    hipEvent_t small_ev = nullptr;
    bool small_pending = false, small_fault = false;
    std::string sticky;
    int health() {
        if (!sticky.empty()) return fail(RH_ERR_HIP, sticky);
        if (!small_pending) return RH_OK;
        const hipError_t e = small_fault ? hipErrorLaunchFailure : hipEventQuery(small_ev);
        if (e == hipErrorNotReady) return RH_OK;
        small_pending = false;
        if (e == hipSuccess) return RH_OK;
        small_fault = false;
        (void)hipGetLastError();
        sticky = std::string("a committed small batch's delta merge failed (") + hipGetErrorString(e) +
                 "): the store is inconsistent until its next load";
        return fail(RH_ERR_HIP, sticky);
    }
    void health_reset() {  // a load replaces the contents
        sticky.clear();
        small_pending = small_fault = false;
    }
    int flush() {
        if (int rc = health()) return rc;
        if (!pend.n) return RH_OK;
        const size_t m = pend.n;
        const bool dated = schema.record_kind == RH_REC_DATED;
        const rh_columns h{pend.keys.data(), dated ? pend.phys.data() : nullptr, dated ? pend.logical.data() : nullptr,
                           dated ? pend.node.data() : nullptr,
                           schema.record_kind == RH_REC_PLAIN ? nullptr : pend.tags.data(), pend.vals.data()};
        uint64_t c[3];
        const int rc = apply_host(h, pend.ops.data(), m, c, true);
        pend.clear();
        return rc;
    }
    // host columns: a small batch is packed into page-locked memory the device reads in place;
    // a large one is uploaded (one copy per column) and applied by the large-batch path
    int apply_host(const rh_columns &h, const uint8_t *ops, size_t m, uint64_t c[3], bool last_wins = false) {
        int rc;
        bool done = false;
        if (m && m <= small_limit()) {
            rh_columns d;
            const uint8_t *dops = nullptr;
            if ((rc = pack_small(h, ops, m, &d, &dops))) return rc;
            if ((rc = apply_small(d, dops, m, last_wins, c, &done))) return rc;
            if (done) return RH_OK;
        }
        if ((rc = staging.upload(schema, h, m, stream)) || (rc = hops.ensure(m + 64))) return rc;
        if (m) RH_HIP(hipMemcpyAsync(hops.p, ops, m, hipMemcpyHostToDevice, stream));
        return apply_device(staging.view(schema), hops.p, m, c, false, nullptr, nullptr, 0, nullptr, last_wins);
    }
    // ---- the small-batch path (small_batch.hpp) --------------------------------------------------
    // A/B switch: RSOS_HIP_SMALL_MAX=<rows> caps the small path (0: off), read when a store is created
    uint64_t small_env = getenv("RSOS_HIP_SMALL_MAX") ? strtoull(getenv("RSOS_HIP_SMALL_MAX"), nullptr, 10) : ~0ull;
    uint64_t small_limit() const {
        if (schema.key_kind == RH_KEY_UNIT) return 0;
        return std::min<uint64_t>(small_env, rh::small_batch_max((int)kl));
    }
    PinnedVec<uint8_t> sb_in;    // a small host batch, packed (the device reads it in place)
    PinnedVec<uint64_t> sb_res{hipHostMallocCoherent};  // the small path's result block (written by the device in place)
    // the device address of a mapped page-locked buffer: looked up once per allocation (the
    // buffer keeps it until it moves), not once per batch
    template <class T>
    int dev_ptr(PinnedVec<T> &v, T **dev) {
        if (!v.dptr || v.dptr_of != v.p) {
            void *d = nullptr;
            const hipError_t e = hipHostGetDevicePointer(&d, v.p, 0);
            if (e != hipSuccess || !d) {
                (void)hipGetLastError();
                return fail(RH_ERR_HIP, "page-locked buffer has no device address");
            }
            v.dptr = d;
            v.dptr_of = v.p;
        }
        *dev = static_cast<T *>(v.dptr);
        return RH_OK;
    }
    int pack_small(const rh_columns &h, const uint8_t *ops, size_t m, rh_columns *d, const uint8_t **dops) {
        const size_t kr = kl, vr = value_row(schema);
        const bool dated = schema.record_kind == RH_REC_DATED;
        const bool tags = h.tags && schema.record_kind != RH_REC_PLAIN;
        auto pad = [](size_t x) { return (x + 15) & ~size_t(15); };
        const size_t o_val = pad(m * kr), o_ph = o_val + pad(m * vr), o_nd = o_ph + (dated ? pad(m * 8) : 0),
                     o_lg = o_nd + (dated ? pad(m * 8) : 0), o_tg = o_lg + (dated ? pad(m * 4) : 0),
                     o_op = o_tg + (tags ? pad(m) : 0), end = o_op + pad(m);
        try {
            sb_in.resize(end + 16);
        } catch (const std::bad_alloc &) {
            return fail(RH_ERR_OOM, "small batch: page-locked allocation failed");
        }
        uint8_t *b = sb_in.data();
        auto put = [&](size_t off, const void *src, size_t bytes) {
            if (src) memcpy(b + off, src, bytes);
            else memset(b + off, 0, bytes);  // a NULL column (the values of a delete-only batch)
        };
        put(0, h.keys, m * kr);
        put(o_val, h.values, m * vr);
        if (dated) {
            put(o_ph, h.phys, m * 8);
            put(o_nd, h.node, m * 8);
            put(o_lg, h.logical, m * 4);
        }
        if (tags) put(o_tg, h.tags, m);
        put(o_op, ops, m);
        uint8_t *db;
        int rc = dev_ptr(sb_in, &db);
        if (rc) return rc;
        *d = rh_columns{db, dated ? reinterpret_cast<const uint64_t *>(db + o_ph) : nullptr,
                        dated ? reinterpret_cast<const uint32_t *>(db + o_lg) : nullptr,
                        dated ? reinterpret_cast<const uint64_t *>(db + o_nd) : nullptr, tags ? db + o_tg : nullptr,
                        db + o_val};
        *dops = db + o_op;
        return RH_OK;
    }
    // capacity of the delta run's other buffers for a batch of m rows into it (the largest run the
    // policy allows: threshold + one batch), and of the record heap
    int delta_capacity(size_t m) {
        int rc;
        const int nxt = 1 - cd;
        const uint64_t n_max = nd + m;
        const uint64_t thresh = std::max<uint64_t>(nb / compact_div, compact_min);
        const uint64_t plan = std::max<uint64_t>(n_max, std::min<uint64_t>(thresh, nb + nd) + m);
        if ((rc = dheap.grow_keep((heap_len + m) * sizeof(rh::DeltaRec) + 64, heap_len * sizeof(rh::DeltaRec), stream)))
            return rc;
        if ((rc = dkeys[nxt].ensure(plan * kl + 64)) || (rc = dslot[nxt].ensure(plan + 16)) ||
            (rc = dbsums[nxt].ensure(rh_num_blocks(plan) * 32 + 32)) ||
            (rc = dssums[nxt].ensure(rh_num_superblocks(plan) * 32 + 32)) ||
            (rc = dsblk[nxt].ensure(rh_num_superblocks(plan) + 16)) || (rc = dscnt.ensure(rh_num_superblocks(plan) + 16)) ||
            (rc = dblk[nxt].ensure(rh_num_blocks(plan) + 16)) || (rc = dinb[nxt].ensure(plan + 16)) ||
            (rc = dsmp[nxt].ensure(rh_num_blocks(plan) + 1)) || (rc = dsmp2[nxt].ensure(rh::sample2_entries(plan))) ||
            (rc = dsmp[cd].ensure(1)) || (rc = dsmp2[cd].ensure(1)) || (rc = mcnt.ensure(8)))
            return rc;
        return RH_OK;
    }
    // A batch of m <= small_limit() rows in two launches (the one-workgroup front, then the delta
    // merge) and no copy command: the columns may live in device memory or in mapped page-locked
    // host memory; the result block and the host tier's fold rows are written into mapped
    // page-locked memory.  *done = false: the shape has no small path (the caller takes the large one).
    int apply_small(const rh_columns &c, const uint8_t *ops, size_t m, bool last_wins, uint64_t out[3], bool *done) {
        int rc;
        *done = false;
        out[0] = out[1] = out[2] = 0;
        if (m == 0 || m > small_limit()) return RH_OK;
        if (nb + nd + m >= (1ull << 31)) return fail(RH_ERR_ARG, "store size limit (2^31 rows) exceeded: use rh_sstore_* for a larger map");
        if ((rc = pre_batch())) return rc;
        snap_ok = run_copy_allowed(m);
        int fmode = fold_mode(m);
        bool want = fold_rows_wanted(fmode);
        if (want && !fold_room(m)) fmode = 0, want = false, rf_log_ok = false;  // the tier goes stale
        if ((rc = skeys.ensure(m * kl + 64)) || (rc = delta_capacity(m))) return rc;
        uint32_t *upos = scratch.u32(3, m + 1), *usrc = scratch.u32(4, m + 1), *rlist = scratch.u32(5, m + 1);
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        uint64_t *res = nullptr;
        uint8_t *fk = nullptr, *fr = nullptr, *fd = nullptr, *ff = nullptr, *fo = nullptr;
        try {
            sb_res.resize(16);
        } catch (const std::bad_alloc &) {
            return fail(RH_ERR_OOM, "small batch: page-locked allocation failed");
        }
        if ((rc = dev_ptr(sb_res, &res))) return rc;
        if (want && ((rc = dev_ptr(fold_keys, &fk)) || (rc = dev_ptr(fold_recs, &fr)) || (rc = dev_ptr(fold_ops, &fd)) ||
                     (rc = dev_ptr(fold_fps, &ff)) || (rc = dev_ptr(fold_sops, &fo))))
            return rc;
        const int nxt = 1 - cd;
        rh::SmallBatch a{};
        a.c = to_dev(c);
        a.ops = ops;
        a.m = (uint32_t)m;
        a.last_wins = last_wins ? 1 : 0;
        a.jb = rh::SearchJob{bkeys[cb].p, nb, bsmp.p, bsmp2.p, base_table(), nullptr, nullptr};
        a.jd = rh::SearchJob{dkeys[cd].p, nd, dsmp[cd].p, dsmp2[cd].p, rh::SearchTable{}, nullptr, nullptr};
        if (!a.jb.smp2 || nb == 0) a.jb.tb = rh::SearchTable{};
        a.base_fps = bfps[cb].p;
        a.dslot = dslot[cd].p;
        a.heap = dheap.p;
        a.heap_base = (uint32_t)heap_len;
        a.skeys = skeys.p;
        a.upos = upos, a.usrc = usrc, a.rlist = rlist;
        a.mcnt = mcnt.p;
        a.res = res;
        if (fail_point("small_batch.stale_seq")) sb_res.data()[13] = small_seq + 1;  // a test's stale word
        a.seq = ++small_seq;
        disarm(sb_res.data() + 13);
        a.fkeys = fk, a.frecs = fr, a.fdrop = fd, a.ffps = ff, a.fops = fo;
        bool supported = false;
        hipError_t e = rh::launch_small_batch_schema(schema.key_kind, (int)schema.key_len, schema.value_kind,
                                                     (int)schema.value_len, schema.record_kind, c.tags != nullptr, a,
                                                     stream, &supported);
        if (e != hipSuccess) return fail(RH_ERR_HIP, std::string("small batch launch: ") + hipGetErrorString(e));
        if (!supported) return RH_OK;
        const uint64_t version0 = version;
        version++;  // from here on the batch may commit
        RH_HIP(rh::launch_delta_merge(schema.key_kind, (int)kl, dkeys[cd].p, dslot[cd].p, nd, skeys.p, m, upos, usrc, rlist,
                                      mcnt.p, dkeys[nxt].p, dslot[nxt].p, rh_num_blocks(nd + m), dsmp[nxt].p,
                                      dsmp2[nxt].p, dheap.p, heap_len, stream));
        if (!small_ev) RH_HIP(hipEventCreateWithFlags(&small_ev, hipEventDisableTiming));
        RH_HIP(hipEventRecord(small_ev, stream));
        small_pending = true;
        if (fail_point("small_batch.merge")) small_fault = true;
        if ((rc = wait_small(a.seq))) return rc;
        const uint64_t *h = sb_res.data();
        if (h[6] & 1) {  // nothing committed
            version = version0;
            return fail(RH_ERR_ARG, "duplicate key within one batch");
        }
        const uint64_t kept = h[12];
        int64_t dcnt;
        memcpy(&dcnt, &h[7], 8);
        out[0] = h[0], out[1] = h[1], out[2] = h[2];
        cd = nxt;
        nd = nd + h[3] - h[5];
        heap_len += kept;
        dtotal += dcnt;
        rh_fp_add(root_d, &h[8], root_d);  // mod 2^256
        dsums_ok = false;
        small_batches++;
        *done = true;
        fold_batch(fmode, kept, want);
        const uint64_t thresh_now = std::max<uint64_t>(nb / compact_div, compact_min);
        if (nd > thresh_now || heap_len > thresh_now) {
            if ((rc = compact())) return rc;
        }
        return post_batch();
    }
    uint64_t small_batches = 0, large_batches = 0, small_seq = 0;
    // The small path's wait: k_small_batch writes its sequence word into the mapped result block
    // after every host-visible result (a system-scope fence first), and the host polls it.  The
    // merge behind it need not have finished -- it writes only device buffers, which every later
    // command on the stream is ordered after -- so a small batch returns without the merge's time
    // and the stream's completion signal.  A stream that fails or drains without the word is an error.
    int wait_small(uint64_t seq) { return wait_word(sb_res.data() + 13, seq); }
    // A sequence word is cleared before every launch that stores it: the buffer holding it may hold
    // anything the same sequence number could match -- a larger round's header copied over it (the
    // round output buffer), or an earlier owner's words (page-locked memory is reused by the runtime
    // after a store is destroyed) -- and a match would return the previous answer still in place.
    // (The kernel that last wrote it has been waited for: nothing else writes it meanwhile.)
    // (RSOS_HIP_SEQ_DISARM=0 skips it: the regression test's control run)
    static void disarm(uint64_t *w) {
        static const bool on = !getenv("RSOS_HIP_SEQ_DISARM") || atoi(getenv("RSOS_HIP_SEQ_DISARM")) != 0;
        if (on) __atomic_store_n(w, 0ull, __ATOMIC_RELEASE);
    }
    // Poll a word a kernel stores last (after a system-scope fence) into mapped page-locked memory
    int wait_word(const uint64_t *w, uint64_t seq) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spin = 1;; spin++) {
            if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == seq) return RH_OK;
            if ((spin & 63) == 0) {
                const hipError_t e = hipStreamQuery(stream);
                if (e == hipSuccess) {
                    if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == seq) return RH_OK;
                    return fail(RH_ERR_HIP, "the stream finished without the kernel's result word");
                }
                if (e != hipErrorNotReady) return fail(RH_ERR_HIP, std::string("hipStreamQuery: ") + hipGetErrorString(e));
                if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
                    RH_HIP(hipStreamSynchronize(stream));
                    if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == seq) return RH_OK;
                    return fail(RH_ERR_HIP, "the stream finished without the kernel's result word");
                }
            }
        }
    }
    // ---- the host tier (host_tier.hpp) ---------------------------------------------------------
    // The tier answers from (its copy of a base run) + (its delta tree: every batch since).  It is
    // fresh while tier_version == version.  A batch of up to tree_limit() rows keeps it fresh by
    // folding the batch's signed deltas into the tree (fold_batch, O(batch log)).  Anything the
    // tree cannot absorb cheaply -- a load, a larger batch, a tree grown past tree_limit() --
    // starts a refresh in the background (start_refresh): the device compacts (so its base run is
    // the whole map), forms the prefix sums and the search samples, and a copy stream brings keys,
    // prefix sums and samples down into the tier's spare page-locked set.  Meanwhile:
    //   - if the tier is still fresh (a tree past its limit), it keeps answering, the batches
    //     applied meanwhile fold into it and are logged for the new copy; the copy is swapped in
    //     (finish_refresh: the log replayed into a new tree) by the next write;
    //   - if it is stale (a load, a large batch), questions are answered by the device (the delta
    //     run is empty right after the refresh's compaction), and writes go on without waiting:
    //     logged for the copy, or, too large to log, leaving the tier stale when the copy lands,
    //     for the next write to refresh again (one refresh per copy time under a stream of large
    //     batches, never one per batch).
    // So no question pays the O(n) copy (rsos/src/fingerprint_tree_map/query.rs:25-76 never does)
    // and no write waits for one; writes pay the compaction.  A wait remains only where a copy's
    // source would be overwritten: a second compaction during one copy, a load, a reservation.
    uint64_t version = 0;       // bumped by every change of contents (load, batch, failed load)
    uint64_t base_epoch = 0;    // bumped whenever the device's base run changes (load, compaction)
    bool tier_on = false;
    uint64_t tier_version = ~0ull, tier_round_max = 128;
    uint64_t tier_epoch = ~0ull;  // the device base the tier's copy is (while they agree, the
                                  // device's DeltaRecs are relative to the tier's base too)
    uint64_t tier_refreshes = 0, tier_folds = 0, tier_waits = 0;
    rh::HostTier tier;
    struct TierSet {  // a base copy: keys in rank order, exclusive prefix sums, every 64th key's digit
        PinnedVec<uint8_t> keys;
        PinnedVec<uint64_t> prefix, samp;
        void release() { keys.release(), prefix.release(), samp.release(); }
    };
    TierSet tsets[2];
    int tact = 0;  // the set the tier reads
    DevBuf<uint8_t> tier_dpre, tier_spre, tier_bpre;
    DevBuf<uint64_t> tier_dsmp;
    std::vector<uint8_t> tier_out;  // the last host round, in round_layout()
    // A/B switch and test hook: RSOS_HIP_TIER_TREE=<entries> sets the tree limit (read at creation)
    uint64_t tree_env = getenv("RSOS_HIP_TIER_TREE") ? strtoull(getenv("RSOS_HIP_TIER_TREE"), nullptr, 10) : 0;
    // the largest delta tree the tier keeps, and the largest batch it folds: a tree of this size
    // still answers a question in about a microsecond (host_delta.hpp)
    uint64_t tree_limit() const {
        if (tree_env) return tree_env;
        return std::max<uint64_t>(1ull << 16, std::min<uint64_t>(tier.nb / 8, 1ull << 18));
    }
    // the refresh in flight (one at a time): its copy into tsets[rf_set] lands at rf_ev on cstream
    bool rf_on = false, refresh_wanted = false;
    int rf_set = 1, rf_cb = 0;  // rf_cb: the base buffer the copy reads
    uint64_t stale_questions = 0;  // questions the device answered since the last batch
    uint64_t rf_version = 0, rf_epoch = 0, rf_nb = 0;
    hipStream_t cstream = nullptr, kstream = nullptr;  // the refresh's copies; its kernels
    // the workgroups of a refresh's row prefix scan that runs beside the store's questions
    // (RSOS_HIP_TIER_SYNC=0; 0: one per 256 rows).  At 10^8 rows, 1,024: no-wait drive p50 0.94 ms,
    // write p50 8.1 ms; all: 1.03 / 7.4; 256: 0.78 / 12.3 (profiles/r05_s22_nowait_wgs.jsonl)
    uint32_t bg_prefix_wgs = getenv("RSOS_HIP_BG_PREFIX_WGS") ? (uint32_t)atoi(getenv("RSOS_HIP_BG_PREFIX_WGS")) : 1024;
    hipEvent_t rf_ready = nullptr, rf_ev = nullptr, rf_kdone = nullptr;
    // the batches applied while the copy is in flight, as mode-1 rows against its base (which is
    // the device's base until the next compaction, and no compaction runs while a copy is in
    // flight): replayed into the new copy's tree when it is swapped in
    struct LogBatch {
        size_t off, m;
    };
    std::vector<LogBatch> rf_log;
    std::vector<uint8_t> rf_keys, rf_recs, rf_drop;
    bool rf_log_ok = true;
    uint64_t rf_log_version = 0;
    // a batch's rows as the folds read them, in key order: keys, the device's DeltaRecs and drop
    // flags (against the device's base), the fingerprints and ops (against the tier's own base)
    // (coherent: the small path writes them in place before the sequence word the host polls)
    PinnedVec<uint8_t> fold_keys{hipHostMallocCoherent}, fold_recs{hipHostMallocCoherent},
        fold_ops{hipHostMallocCoherent}, fold_fps{hipHostMallocCoherent}, fold_sops{hipHostMallocCoherent};
    bool tier_fresh() const { return tier_on && tier_version == version; }
    // Device -> host copies into the tier's page-locked (mapped) buffers: one kernel whose 16-byte
    // stores cross PCIe at ~52 GB/s (launch_copy_to_host), where copy commands move ~30 GB/s
    // (profiles/r05_s1_interleave_trace_summary.txt); RSOS_HIP_COPY_KERNEL=0 keeps the copy commands.
    struct Down {
        void *host;
        PinnedAny pin;
        const void *dev;
        size_t bytes;
    };
    int copy_kernel = getenv("RSOS_HIP_COPY_KERNEL") ? atoi(getenv("RSOS_HIP_COPY_KERNEL")) : 1;
    // kernel = false: copy commands (a background copy under "writes never wait": a copy kernel
    // would hold CUs beside the batches and questions that run meanwhile)
    int copy_down(const Down *d, int n, hipStream_t st, bool kernel_ok = true) {
        rh::CopyJobs j{};
        bool kernel = copy_kernel != 0 && kernel_ok;
        for (int k = 0; k < n && kernel; k++) {
            uint8_t *dp = nullptr;
            if (d[k].pin.lookup(&dp)) kernel = false;
            j.src[k] = static_cast<const uint8_t *>(d[k].dev), j.dst[k] = dp, j.bytes[k] = d[k].bytes;
        }
        if (kernel) {
            j.n = n;
            RH_HIP(rh::launch_copy_to_host(j, st));
            return RH_OK;
        }
        for (int k = 0; k < n; k++)
            if (d[k].bytes) RH_HIP(hipMemcpyAsync(d[k].host, d[k].dev, d[k].bytes, hipMemcpyDeviceToHost, st));
        return RH_OK;
    }
    // A few result bytes into page-locked memory by a one-workgroup kernel, not a copy command: a
    // background copy on the copy engines (a no-wait run refresh) would hold it back
    template <class T>
    int down_small(PinnedVec<T> &v, const void *dev, size_t bytes) {
        const Down d{v.data(), v, dev, bytes};
        return copy_down(&d, 1, stream);
    }
    // A refresh's device buffers, sized for the base buffers' capacity (reserve() calls it too): a
    // base grown by compactions reallocates nothing here -- a hipFree waits for every copy in
    // flight, the other store's too (no-wait drives of 40-175 ms before, profiles/r05_nowait_cycles.txt)
    int refresh_room() {
        int rc;
        const uint64_t c = std::max<uint64_t>(nb, base_cap_rows()), cbk = rh_num_blocks(c), cs = rh_num_superblocks(c);
        if ((rc = tier_dpre.ensure((c + 1) * 32 + 64)) || (rc = tier_spre.ensure((cs + 1) * 32 + 64)) ||
            (rc = tier_bpre.ensure((cbk + 1) * 32 + 64)) || (rc = tier_dsmp.ensure((c + 63) / 64 + (c + 4095) / 4096 + 8)))
            return rc;
        return RH_OK;
    }
    // Start a refresh of the host tier: compact, the prefix sums and samples on the device, and
    // their copy down on the copy stream into the spare set.  Returns at once (no wait).
    int start_refresh() {
        int rc;
        if (!tier_on) return RH_OK;
        if (rf_on) {  // one copy at a time: the next one starts once it has landed
            refresh_wanted = true;
            return RH_OK;
        }
        if ((rc = compact())) return rc;
        if ((rc = refresh_streams())) return rc;
        const uint64_t n = nb, nsmp = (n + 63) / 64, nsmp2 = (n + 4095) / 4096;  // samp2: host_tier.hpp
        if ((rc = refresh_room())) return rc;
        const int spare = 1 - tact;
        TierSet &S = tsets[spare];
        try {  // headroom, once the set must grow anyway: a growing map re-pins rarely
            S.keys.clear(), S.prefix.clear(), S.samp.clear();  // the old contents are not kept
            if (S.keys.capacity() < n * kl + 64 || S.prefix.capacity() < (n + 1) * 4 + 8 ||
                S.samp.capacity() < nsmp + nsmp2 + 8) {
                S.keys.reserve((n + n / 4) * kl + 64);
                S.prefix.reserve((n + n / 4 + 1) * 4 + 8);
                S.samp.reserve((n + n / 4) / 64 + (n + n / 4) / 4096 + 16);
            }
            S.keys.resize(n * kl + 64);
            S.prefix.resize((n + 1) * 4 + 8);
            S.samp.resize(nsmp + nsmp2 + 8);
        } catch (const std::bad_alloc &) {
            return tier_oom();
        }
        // the prefix scan and the samples run on the copy stream too, behind the compaction: the
        // store's own stream goes on at once (a question answered by the device meanwhile is not
        // queued behind ~1-2 ms of scans at 10^8 rows); the next compaction, which rewrites the
        // base's block sums they read, waits for them (rf_kdone)
        RH_HIP(hipEventRecord(rf_ready, stream));
        RH_HIP(hipStreamWaitEvent(kstream, rf_ready, 0));
        if (n) {
            RH_HIP(rh::launch_prefix(bfps[cb].p, n, bsums.p, ssums.p, tier_spre.p, tier_bpre.p, tier_dpre.p, kstream,
                                     tier_sync_writes ? 0u : bg_prefix_wgs));
            RH_HIP(kops->sample_stride(bkeys[cb].p, n, 64, tier_dsmp.p, kstream));
            RH_HIP(kops->sample_stride(bkeys[cb].p, n, 4096, tier_dsmp.p + nsmp, kstream));
        }
        RH_HIP(hipEventRecord(rf_kdone, kstream));
        // by kernel stores (on kstream) when the write or load that starts the refresh waits for it
        // (the default policy); by the copy engines (on cstream) when it runs behind the store's work
        hipStream_t down = tier_sync_writes ? kstream : cstream;
        if (down == cstream) RH_HIP(hipStreamWaitEvent(cstream, rf_kdone, 0));
        if (n) {
            const Down d[3] = {{S.keys.data(), S.keys, bkeys[cb].p, n * kl},
                               {S.prefix.data(), S.prefix, tier_dpre.p, (n + 1) * 32},
                               {S.samp.data(), S.samp, tier_dsmp.p, (nsmp + nsmp2) * 8}};
            if ((rc = copy_down(d, 3, down, tier_sync_writes))) return rc;
        } else {
            memset(S.prefix.data(), 0, 32);
        }
        RH_HIP(hipEventRecord(rf_ev, down));
        rf_on = true;
        refresh_wanted = false;
        rf_set = spare;
        rf_cb = cb;
        rf_version = rf_log_version = version;
        rf_epoch = base_epoch;
        rf_nb = n;
        rf_log.clear();
        rf_keys.clear(), rf_recs.clear(), rf_drop.clear();
        rf_log_ok = true;
        return RH_OK;
    }
    // The copy has landed: the new set becomes the tier's, the logged batches folded into its tree.
    void finish_refresh() {
        rf_on = false;
        if (rf_run) {  // a run copy: the tier takes it if nothing was written since it started
            rf_run = false;
            rf_tset = -1;
            if (rf_version == version && rf_epoch == tier_epoch) {
                ract = 1 - ract;
                tier.set_run(trh[ract].run(rf_run_n));
                tier_version = version;
                tier_runs++;
                tier_refreshes++;
                run_discards = 0;
            } else {
                refresh_wanted = true;
                run_discards++;
            }
            return;
        }
        if (!(rf_log_ok && rf_log_version == version) && tier_fresh()) {
            // the copy cannot be brought up to date but the tier still is (a tree past its limit):
            // keep the tier, drop the copy, and let the next write start another
            refresh_wanted = true;
            rf_log.clear();
            rf_keys = std::vector<uint8_t>(), rf_recs = std::vector<uint8_t>(), rf_drop = std::vector<uint8_t>();
            return;
        }
        tact = rf_set;
        TierSet &S = tsets[tact];
        tier.build((uint32_t)kl, schema.key_kind, rf_nb, S.keys.data(), S.prefix.data(), S.samp.data(),
                   S.samp.data() + (rf_nb + 63) / 64);
        tier_epoch = rf_epoch;
        tier_refreshes++;
        bool ok = rf_log_ok && rf_log_version == version;
        std::vector<rh::DeltaTree::Rec> rows;
        try {
            for (const LogBatch &b : rf_log) {
                rows.resize(b.m);
                for (size_t j = 0; j < b.m; j++) {
                    const size_t i = b.off + j;
                    rec_row(rf_keys.data() + i * kl, reinterpret_cast<const rh::DeltaRec *>(rf_recs.data()) + i, &rows[j]);
                }
                tier.fold(rows.data(), rf_drop.data() + b.off, b.m);
            }
        } catch (const std::bad_alloc &) {
            ok = false;
        }
        tier_version = ok ? version : ~0ull;
        if (!ok) refresh_wanted = true;
        rf_log.clear();
        rf_keys = std::vector<uint8_t>(), rf_recs = std::vector<uint8_t>(), rf_drop = std::vector<uint8_t>();
    }
    // Has the copy landed?  wait: block until it has.  Then swap it in.
    int poll_refresh(bool wait) {
        if (!rf_on) return RH_OK;
        const hipError_t e = wait ? hipEventSynchronize(rf_ev) : hipEventQuery(rf_ev);
        if (e == hipErrorNotReady) return RH_OK;
        if (e != hipSuccess) {
            rf_on = false;
            tier_version = ~0ull;
            return fail(RH_ERR_HIP, std::string("host tier copy: ") + hipGetErrorString(e));
        }
        if (wait) tier_waits++;
        finish_refresh();
        return RH_OK;
    }
    // Before anything writes what an in-flight copy reads (a compaction, a load, a reservation),
    // or before a batch while the tier is stale: let the copy land and swap it in.
    int settle() { return rf_on ? poll_refresh(true) : RH_OK; }
    // Two policies for a refresh that a write starts (RSOS_HIP_TIER_SYNC, read when a store is
    // created):
    //   1 (the default): writes keep the tier fresh -- a stale tier's copy in flight is waited for
    //     before a batch, a refresh a batch or a load starts is waited for by it (post_batch,
    //     load_finish), so no question is ever answered by the device; a write that outgrows the
    //     tree pays the compaction and the whole copy (~0.1 s per 10^8 rows);
    //   0: writes never wait -- a landed copy is swapped in (its log replayed), a copy in flight is
    //     not waited for (the batch is logged for it, or breaks its log and the tier stays stale),
    //     and questions meanwhile go to the device.
    bool tier_sync_writes = !(getenv("RSOS_HIP_TIER_SYNC") && atoi(getenv("RSOS_HIP_TIER_SYNC")) == 0);
    int pre_batch() { return poll_refresh(tier_sync_writes && rf_on && !tier_fresh()); }
    // After a batch (committed, folded, logged): start the refresh the tier needs, unless one is
    // in flight -- so under a stream of large batches the refreshes (a compaction and a copy
    // each) run back to back, one per copy time, not one per batch, and no write waits for one.
    // The batch has committed by now: a tier that cannot be brought up to date for want of host
    // memory is left stale (questions go to the device; the next write tries again) -- reporting
    // it would make the caller think the batch failed.  Device errors still propagate.
    int post_batch() {
        tier_host_oom = false;
        const int rc = tier_stale_on_host_oom(post_batch_tier());
        if (rc == RH_OK) prefetch_run_columns();
        return rc;
    }
    // When the next question is the device's (tier off, or stale until a copy lands), the delta
    // run's columns for this version are formed now, queued behind the batch on the store's
    // stream, instead of by that question (a drive's first round paid them: a long run's five
    // launches over the whole run, both stores) -- if questions read them after the previous
    // batch (a stream of batches with no questions between, config5, never pays for them).  A
    // failure is left for the question to meet again.  RSOS_HIP_RUN_PREFETCH=0: at the question.
    int run_prefetch = getenv("RSOS_HIP_RUN_PREFETCH") ? atoi(getenv("RSOS_HIP_RUN_PREFETCH")) : 1;
    bool run_cols_asked = false;  // a question read the run's columns since the last batch
    void prefetch_run_columns() {
        const bool asked = run_cols_asked;
        run_cols_asked = false;
        if (!run_prefetch || !asked || nd == 0 || (tier_on && tier_fresh())) return;
        const std::string keep = g_err;
        if (run_columns(false) != RH_OK) {
            trun_ver = trun_pre_ver = ~0ull;
            g_err = keep;
            (void)hipGetLastError();
        }
    }
    // A failure to pin host memory for the tier leaves the tier stale (questions go to the device;
    // the next write tries again) and is not the caller's error: the write or load has committed.
    // Device allocation failures (e.g. the compaction a refresh starts) still propagate.
    bool tier_host_oom = false;
    int tier_oom(const char *what = "host tier: page-locked allocation failed") {
        tier_host_oom = true;
        tier_version = ~0ull;
        return fail(RH_ERR_OOM, what);
    }
    int tier_stale_on_host_oom(int rc) {
        if (rc == RH_ERR_OOM && tier_host_oom) {
            tier_host_oom = false;
            tier_version = ~0ull;
            g_err.clear();  // reported as success: no stale message for the caller to read
            return RH_OK;
        }
        return rc;
    }
    int post_batch_tier() {
        if (!tier_on) return RH_OK;
        stale_questions = 0;
        int rc;
        if (tier_sync_writes) {
            if (rf_on && !tier_fresh() && (rc = settle())) return rc;
            const bool snap = snap_ok;
            snap_ok = false;
            // a copy of the delta run serves while the tier's base is still the device's and the
            // run is at most a quarter of the base (past that the base is refreshed)
            const bool run_ok = !rf_on && tier_epoch == base_epoch && nd <= tier.nb / 4 + (1u << 16);
            if (snap && !tier_fresh() && run_ok) return tier_run_snapshot();  // a batch too large to fold
            if (!tier_fresh() && !rf_on) {
                if ((rc = start_refresh())) return rc;
                return settle();
            }
            if (tier_fresh() && tier.dt.size() > tree_limit() && run_ok) return tier_run_snapshot();  // the tree full
        }
        if (rf_on) return RH_OK;
        if (!tier_fresh() || refresh_wanted || tier.dt.size() > tree_limit()) return refresh_now();
        return RH_OK;
    }
    // A question to a stale tier with no copy in flight starts one only when that costs the
    // question nothing (the delta run is empty: no compaction), or after enough questions since
    // the last batch to pay for the compaction it waits behind -- otherwise the next batch does.
    static constexpr uint64_t STALE_QUESTIONS = 256;
    bool question_may_refresh() { return nd == 0 || ++stale_questions >= STALE_QUESTIONS; }
    // ---- the tier's run copy (host_tier.hpp HostTier::Run) --------------------------------------
    // With writes keeping the tier fresh, a batch too large for the tree would cost a compaction
    // and a copy of the whole base (~0.1 s per 10^8 rows).  While the tier's base is still the
    // device's (no compaction since its copy), the device's delta run is exactly every change
    // since: its DeltaRecs, as columns with prefix sums, are copied down instead -- O(delta run),
    // <= n / compact_div rows -- and the tier answers from base + run copy.  The next small batch
    // (or a compaction, or a run copy past a quarter of the base) refreshes the base instead.
    struct RunDev {  // the delta run's columns on the device (run_columns), one version's
        DevBuf<uint8_t> c, fl, bs, ss, spre, bpre, pre;
        DevBuf<uint32_t> cnt, cntp, br;
        DevBuf<uint64_t> smp, gs;
        void release() {
            c.release(), fl.release(), bs.release(), ss.release(), spre.release(), bpre.release(), pre.release();
            cnt.release(), cntp.release(), br.release(), smp.release(), gs.release();
        }
    };
    // two sets: run_columns fills trs[tcur]; while a no-wait run copy reads one (rf_tset), the
    // next version's columns go to the other, so neither the copy nor the questions wait
    RunDev trs[2];
    int tcur = 0;
    struct RunHost {  // a run copy's page-locked columns
        PinnedVec<uint8_t> keys, fl;
        PinnedVec<uint64_t> pre, smp, gs;
        PinnedVec<uint32_t> cntp, br;
        void release() { keys.release(), fl.release(), pre.release(), smp.release(), gs.release(), cntp.release(), br.release(); }
        // room for a run of n1 entries (headroom: the run grows batch by batch)
        void fit(uint64_t n1, uint32_t kl) {
            auto f = [](auto &v, size_t want) {
                if (v.capacity() < want) {
                    v.clear();
                    v.reserve(want + want / 2);
                }
                v.resize(want);
            };
            const uint64_t ns = (n1 + 63) / 64, ns2 = (n1 + 4095) / 4096;
            f(keys, n1 * kl + 64), f(pre, (n1 + 1) * 4 + 8), f(cntp, n1 + 16), f(fl, n1 + 16), f(br, n1 + 16);
            f(smp, ns + ns2 + 8), f(gs, ns + 8);
        }
        rh::HostTier::Run run(uint64_t n1) {
            rh::HostTier::Run r;
            r.n = n1;
            r.keys = keys.data();
            r.prefix = pre.data();
            r.cntp = reinterpret_cast<const int32_t *>(cntp.data());
            r.flags = fl.data();
            r.brank = br.data();
            r.samp = smp.data();
            r.samp2 = smp.data() + (n1 + 63) / 64;
            r.gsamp = gs.data();
            return r;
        }
    };
    // trh[ract]: the run copy the tier reads; trh[1 - ract]: the one a no-wait run refresh fills
    RunHost trh[2];
    int ract = 0;
    uint64_t tier_runs = 0;
    bool snap_ok = false;  // set before a batch: a run copy may replace the refresh it causes
    // with a run copy held, batches fold into the tree as deltas against base + run (mode 2: a
    // host search of the run per row); one larger than this takes a new run copy instead
    static constexpr size_t RUN_FOLD_MAX = 4096;
    bool run_copy_allowed(size_t m) const {
        return tier_sync_writes && tier_fresh() && tier_epoch == base_epoch &&
               (m > tree_limit() || (tier.has_run() && m > RUN_FOLD_MAX));
    }
    // The delta run as columns (k_tier_run: contributions with their block and super-block sums,
    // the count deltas' exclusive prefix sums, flags, base ranks, select's index G(64 k)), formed
    // on the device once per version of the contents: device reads over base + run use them in
    // place (rh::RoundRun), the run copy adds the contributions' prefix sums and takes them down.
    // trun_ver: the version they hold.
    uint64_t trun_ver = ~0ull, trun_pre_ver = ~0ull;  // the version trs[tcur].pre holds
    // the run's row prefix (run_columns forms it for a short run; a long run's on demand)
    int run_row_prefix() {
        int rc;
        if ((rc = run_columns())) return rc;
        if (trun_pre_ver == version) return RH_OK;
        RH_HIP(rh::launch_row_prefix(trs[tcur].c.p, nd, trs[tcur].bpre.p, trs[tcur].pre.p, stream));
        trun_pre_ver = version;
        return RH_OK;
    }
    // A/B switch: RSOS_HIP_RUNCOL_FUSED=0 forms a short run's columns in the eight launches too
    int run_cols_fused = getenv("RSOS_HIP_RUNCOL_FUSED") ? atoi(getenv("RSOS_HIP_RUNCOL_FUSED")) : 1;
    int run_prep_wait = getenv("RSOS_HIP_RUN_PREP_WAIT") ? atoi(getenv("RSOS_HIP_RUN_PREP_WAIT")) : 1;
    int run_columns(bool question = true) {
        int rc;
        const uint64_t n1 = nd;
        run_cols_asked = run_cols_asked || question;
        if (trun_ver == version && trs[tcur].gs.p) return RH_OK;
        if (rf_on && rf_run && rf_tset == tcur) tcur = 1 - tcur;  // a run copy reads this set
        trun_ver = trun_pre_ver = ~0ull;
        // sized for the longest run the delta run's buffers are planned for (compaction threshold +
        // a batch), not this one: a run growing batch by batch would otherwise reallocate here, and
        // the hipFree waits for everything in flight -- a background refresh copy included (no-wait
        // drives of 40-175 ms, profiles/r05f_interleave.jsonl)
        const uint64_t nc = std::max<uint64_t>(n1, dslot[cd].cap > 16 ? dslot[cd].cap - 16 : 0);
        const uint64_t nbk = rh_num_blocks(n1);
        {
            const uint64_t cbk = rh_num_blocks(nc), csb = rh_num_superblocks(nc), cs = (nc + 63) / 64;
            if ((rc = trs[tcur].c.ensure(nc * 32 + 64)) || (rc = trs[tcur].cnt.ensure(nc + 16)) || (rc = trs[tcur].fl.ensure(nc + 16)) ||
                (rc = trs[tcur].br.ensure(nc + 16)) || (rc = trs[tcur].bs.ensure(cbk * 32 + 32)) ||
                (rc = trs[tcur].ss.ensure(csb * 32 + 32)) || (rc = trs[tcur].cntp.ensure(nc + 16)) || (rc = trs[tcur].gs.ensure(cs + 8)))
                return rc;
            if ((rc = trs[tcur].spre.ensure((csb + 1) * 32 + 64)) || (rc = trs[tcur].bpre.ensure((cbk + 1) * 32 + 64)) ||
                (rc = trs[tcur].pre.ensure((nc + 1) * 32 + 64)))
                return rc;
        }
        if (n1 <= rh::RUNCOL_SMALL && run_cols_fused) {  // a short run: every column in one launch
            const rh::RunCols o{trs[tcur].c.p,  trs[tcur].cnt.p,  trs[tcur].fl.p,   trs[tcur].br.p,   trs[tcur].pre.p, trs[tcur].bs.p,
                                trs[tcur].ss.p, trs[tcur].spre.p, trs[tcur].bpre.p, trs[tcur].cntp.p, trs[tcur].gs.p};
            RH_HIP(rh::launch_run_columns_small(dslot[cd].p, dheap.p, n1, o, stream));
            trun_ver = trun_pre_ver = version;
            return RH_OK;
        }
        // a long run: the columns with their block sums in one pass, the block prefix; its row prefix
        // (another read and write of 32 B an entry: ~0.1 ms at 10^7 entries, more than the rounds
        // of one reconciliation save with it) only for the tier's run copy (run_row_prefix)
        RH_HIP(rh::launch_tier_run(dslot[cd].p, dheap.p, n1, trs[tcur].c.p, trs[tcur].cnt.p, trs[tcur].fl.p, trs[tcur].br.p, stream,
                                   trs[tcur].bs.p));
        RH_HIP(rh::launch_reduce(trs[tcur].bs.p, nbk, trs[tcur].ss.p, stream));
        RH_HIP(rh::launch_block_prefix(n1, trs[tcur].bs.p, trs[tcur].ss.p, trs[tcur].spre.p, trs[tcur].bpre.p, stream));
        RH_HIP(rh::launch_exclusive_scan_u32(trs[tcur].cnt.p, trs[tcur].cntp.p, n1 + 1, scratch, stream));
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        RH_HIP(rh::launch_tier_gsamp(trs[tcur].br.p, trs[tcur].cntp.p, trs[tcur].fl.p, n1, trs[tcur].gs.p, stream));
        trun_ver = version;
        return RH_OK;
    }
    int tier_run_snapshot() {
        int rc;
        if (fail_point("tier.run_copy")) return tier_oom("injected failure (tier run copy)");
        const uint64_t n1 = nd;
        if (n1 == 0) {  // nothing since the base copy: the base alone is the map
            tier.set_run(rh::HostTier::Run{});
            tier_version = version;
            return RH_OK;
        }
        const uint64_t ns = (n1 + 63) / 64, ns2 = (n1 + 4095) / 4096;
        // the contributions' row prefix: the host walks it (HostTier::Run::prefix)
        // (the samples sized like run_columns' buffers: for the longest run planned)
        const uint64_t nc = std::max<uint64_t>(n1, dslot[cd].cap > 16 ? dslot[cd].cap - 16 : 0);
        if ((rc = run_row_prefix()) || (rc = trs[tcur].smp.ensure((nc + 63) / 64 + (nc + 4095) / 4096 + 8))) return rc;
        RH_HIP(kops->sample_stride(dkeys[cd].p, n1, 64, trs[tcur].smp.p, stream));
        RH_HIP(kops->sample_stride(dkeys[cd].p, n1, 4096, trs[tcur].smp.p + ns, stream));
        RunHost &H = trh[ract];  // rewritten in place: the writer holds the lock, no question reads it
        try {
            H.fit(n1, (uint32_t)kl);
        } catch (const std::bad_alloc &) {
            tier_version = ~0ull;
            return tier_oom();
        }
        {
            const Down d[7] = {{H.keys.data(), H.keys, dkeys[cd].p, n1 * kl},
                               {H.pre.data(), H.pre, trs[tcur].pre.p, (n1 + 1) * 32},
                               {H.cntp.data(), H.cntp, trs[tcur].cntp.p, (n1 + 1) * 4},
                               {H.fl.data(), H.fl, trs[tcur].fl.p, n1},
                               {H.br.data(), H.br, trs[tcur].br.p, n1 * 4},
                               {H.smp.data(), H.smp, trs[tcur].smp.p, (ns + ns2) * 8},
                               {H.gs.data(), H.gs, trs[tcur].gs.p, ns * 8}};
            if ((rc = copy_down(d, 7, stream))) return rc;
        }
        if ((rc = sync())) {
            tier_version = ~0ull;
            return rc;
        }
        tier.set_run(H.run(n1));
        tier_version = version;
        tier_runs++;
        tier_refreshes++;  // a copy from the device, as a refresh is (rh_store_tier_stats)
        return RH_OK;
    }
    // ---- the no-wait run refresh ----------------------------------------------------------------
    // With writes never waiting (RSOS_HIP_TIER_SYNC=0) and the tier's base still the device's, a
    // stale tier is refreshed by a copy of the delta run alone -- O(run), no compaction (a base
    // refresh compacts first: ~3 ms per 10^8-row store) -- into the spare run set on the copy
    // engines.  It lands only if nothing was written meanwhile (it is never replayed: the next
    // write takes another).  The copy reads one of the two device column sets (the next version's
    // columns go to the other: run_columns) and a staged copy of the run's keys.
    bool rf_run = false;  // the refresh in flight is a run copy
    uint64_t rf_run_n = 0;
    // Run copies discarded in a row because a write landed during each: writes arriving faster
    // than one O(run) copy would keep the tier stale for as long as they last.  After
    // RUN_DISCARD_MAX of them the next refresh is a base refresh, into which the batches applied
    // while it is in flight are logged and replayed, so it lands under a steady write stream.
    static constexpr int RUN_DISCARD_MAX = 2;
    int run_discards = 0;
    uint64_t run_fallbacks = 0;  // base refreshes taken for that reason (RSOS_HIP_ROUND_DBG / tests)
    int rf_tset = -1;               // the column set it reads
    DevBuf<uint8_t> trun_keys;      // ... and the run's keys, staged
    bool run_refresh_ok() const {
        return tier_on && !tier_sync_writes && !rf_on && tier_epoch == base_epoch && nd > 0 &&
               nd <= tier.nb / 4 + (1u << 16);
    }
    int refresh_streams() {
        if (cstream) return RH_OK;
        // the copies on a plain stream (the copy engines); the scans and samples, and kernel
        // copies, on a CU-masked one (create_back_stream): a copy issued on a CU-masked stream
        // held the next write's uploads behind it (write p50 7 -> 100 ms, 10^8 rows)
        RH_HIP(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
        RH_HIP(back_stream(device, 0, &kstream));
        RH_HIP(hipEventCreateWithFlags(&rf_ready, hipEventDisableTiming));
        RH_HIP(hipEventCreateWithFlags(&rf_ev, hipEventDisableTiming));
        RH_HIP(hipEventCreateWithFlags(&rf_kdone, hipEventDisableTiming));
        return RH_OK;
    }
    int start_run_refresh() {
        int rc;
        if ((rc = refresh_streams())) return rc;
        const uint64_t n1 = nd, ns = (n1 + 63) / 64, ns2 = (n1 + 4095) / 4096;
        const uint64_t nc = std::max<uint64_t>(n1, dslot[cd].cap > 16 ? dslot[cd].cap - 16 : 0);
        if ((rc = run_row_prefix())) return rc;
        RunDev &T = trs[tcur];
        if ((rc = T.smp.ensure((nc + 63) / 64 + (nc + 4095) / 4096 + 8)) || (rc = trun_keys.ensure(nc * kl + 64))) return rc;
        RH_HIP(kops->sample_stride(dkeys[cd].p, n1, 64, T.smp.p, stream));
        RH_HIP(kops->sample_stride(dkeys[cd].p, n1, 4096, T.smp.p + ns, stream));
        {  // the keys staged in HBM (the batch after next rewrites dkeys[cd]; a wait for the copy
           // there held small writes 45 ms)
            rh::CopyJobs j{};
            j.src[0] = dkeys[cd].p, j.dst[0] = trun_keys.p, j.bytes[0] = n1 * kl, j.n = 1;
            RH_HIP(rh::launch_copy_to_host(j, stream, 2048));
        }
        RunHost &H = trh[1 - ract];
        try {
            H.fit(n1, (uint32_t)kl);
        } catch (const std::bad_alloc &) {
            return tier_oom();
        }
        // on the copy engines (a copy kernel beside the store's work slowed its questions to
        // milliseconds, profiles/r05_nowait_run_refresh.txt); the store's own small result copies
        // are kernel stores (down_small), so they do not queue behind it
        RH_HIP(hipEventRecord(rf_ready, stream));
        RH_HIP(hipStreamWaitEvent(cstream, rf_ready, 0));
        const Down d[7] = {{H.keys.data(), H.keys, trun_keys.p, n1 * kl},
                           {H.pre.data(), H.pre, T.pre.p, (n1 + 1) * 32},
                           {H.cntp.data(), H.cntp, T.cntp.p, (n1 + 1) * 4},
                           {H.fl.data(), H.fl, T.fl.p, n1},
                           {H.br.data(), H.br, T.br.p, n1 * 4},
                           {H.smp.data(), H.smp, T.smp.p, (ns + ns2) * 8},
                           {H.gs.data(), H.gs, T.gs.p, ns * 8}};
        if ((rc = copy_down(d, 7, cstream, false))) return rc;
        RH_HIP(hipEventRecord(rf_ev, cstream));
        // the write waits for the columns and row prefix it queued (~0.4 ms at 10^7 run rows), not
        // for the copy: the drive that follows reads them at once instead of queueing behind them
        // (RSOS_HIP_RUN_PREP_WAIT=0: return at once)
        if (run_prep_wait) RH_HIP(hipEventSynchronize(rf_ready));
        rf_on = rf_run = true;
        rf_tset = tcur;
        refresh_wanted = false;
        rf_version = version;
        rf_epoch = base_epoch;
        rf_run_n = n1;
        rf_log.clear();
        rf_log_ok = false;
        return RH_OK;
    }
    // the refresh a stale tier takes: a run copy when that is enough, else the base's
    // a question's refresh (tier_ready) is only ever a run copy: no question compacts
    bool run_refresh_next() const { return run_refresh_ok() && run_discards < RUN_DISCARD_MAX; }
    int refresh_now() {
        if (run_refresh_next()) return start_run_refresh();
        if (run_refresh_ok()) run_fallbacks++;
        run_discards = 0;
        return start_refresh();
    }
    // How a batch of m rows reaches the tier (decided before the batch, under the lock):
    //   0: it does not (tier off or stale, or the batch is larger than the tree takes: the tier
    //      goes stale and a refresh follows the batch),
    //   1: from the device's DeltaRecs (the tier's base is the device's: contribs relative to it),
    //   2: from the batch's sorted fingerprints and ops, the deltas formed against the tier's own
    //      base on the host (the device compacted since the tier's copy was taken).
    int fold_mode(size_t m) const {
        if (!tier_fresh() || m > tree_limit()) return 0;
        if (tier.has_run()) return m <= RUN_FOLD_MAX ? 2 : 0;  // deltas against base + run copy
        return tier_epoch == base_epoch ? 1 : 2;
    }
    // whether the batch's rows must come down at all (a fold, or a refresh in flight to log for)
    bool fold_rows_wanted(int fmode) const { return fmode != 0 || (rf_on && !rf_run); }
    // page-locked room for a batch's fold rows (a failure leaves the tier stale, never fails the batch)
    bool fold_room(size_t m) {
        try {
            fold_keys.resize(m * kl + 8);
            fold_recs.resize(m * sizeof(rh::DeltaRec) + 8);
            fold_ops.resize(m + 8);
            fold_fps.resize(m * 32 + 8);
            fold_sops.resize(m + 8);
        } catch (const std::bad_alloc &) {
            return false;
        }
        return true;
    }
    // enqueue the copies the folds read (behind the batch's merge, before its result copy)
    int fold_copies(const uint8_t *sorted_keys, const uint8_t *sorted_fps, const uint8_t *sorted_ops,
                    const uint8_t *recs, const uint8_t *drop, size_t m) {
        RH_HIP(hipMemcpyAsync(fold_keys.data(), sorted_keys, m * kl, hipMemcpyDeviceToHost, stream));
        RH_HIP(hipMemcpyAsync(fold_recs.data(), recs, m * sizeof(rh::DeltaRec), hipMemcpyDeviceToHost, stream));
        RH_HIP(hipMemcpyAsync(fold_ops.data(), drop, m, hipMemcpyDeviceToHost, stream));
        RH_HIP(hipMemcpyAsync(fold_fps.data(), sorted_fps, m * 32, hipMemcpyDeviceToHost, stream));
        RH_HIP(hipMemcpyAsync(fold_sops.data(), sorted_ops, m, hipMemcpyDeviceToHost, stream));
        return RH_OK;
    }
    // a mode-1 row: the device's DeltaRec of a key
    static void rec_row(const uint8_t *key, const rh::DeltaRec *d, rh::DeltaTree::Rec *r) {
        r->key = key;
        memcpy(r->fp, d->contrib, 32);
        const bool in_b = d->flags & rh::DeltaRec::IN_BASE, live = d->flags & rh::DeltaRec::LIVE;
        r->cnt = (int8_t)((live ? 1 : 0) - (in_b ? 1 : 0));
        r->live = live;
    }
    // After the batch committed (the copies have landed): the batch's rows into the tier's delta
    // tree, in key order -- the same rule as k_delta_build: an upsert's entry is (cur - base,
    // 1 - in_base, live), a delete of a base key (-base, -1, dead), a delete of any other key drops
    // its entry.  Keeps the tier fresh.  With a refresh in flight the rows are also logged for it.
    std::vector<rh::DeltaTree::Rec> fold_rows;
    std::vector<uint8_t> fold_drop;
    void fold_batch(int mode, size_t m, bool copied) {
        if (rf_on && !rf_run) {  // the log for the copy in flight (mode-1 rows against its base)
            if (!copied || rf_keys.size() / kl + m > 2 * tree_limit()) {
                rf_log_ok = false;
            } else if (rf_log_ok) {
                try {
                    rf_log.push_back(LogBatch{rf_keys.size() / kl, m});
                    rf_keys.insert(rf_keys.end(), fold_keys.data(), fold_keys.data() + m * kl);
                    rf_recs.insert(rf_recs.end(), fold_recs.data(), fold_recs.data() + m * sizeof(rh::DeltaRec));
                    rf_drop.insert(rf_drop.end(), fold_ops.data(), fold_ops.data() + m);
                    rf_log_version = version;
                } catch (const std::bad_alloc &) {
                    rf_log_ok = false;
                }
            }
        }
        if (!mode || !copied) return;
        rh::HostTier &t = tier;
        try {
            fold_rows.resize(m);
            fold_drop.resize(m);
        } catch (const std::bad_alloc &) {
            return;  // stays stale
        }
        const uint8_t *K = fold_keys.data();
        for (size_t j = 0; j < m; j++) {
            rh::DeltaTree::Rec &r = fold_rows[j];
            if (mode == 1) {
                rec_row(K + j * kl, reinterpret_cast<const rh::DeltaRec *>(fold_recs.data()) + j, &r);
                fold_drop[j] = fold_ops[j] != 0;
            } else {
                uint64_t cur[4];
                memcpy(cur, fold_fps.data() + 32 * j, 32);
                fold_drop[j] = t.entry_vs_base(K + j * kl, fold_sops[j] ? nullptr : cur, &r);
            }
        }
        t.fold(fold_rows.data(), fold_drop.data(), m);
        tier_version = version;
        tier_folds++;
    }
    // Wait for the stream by polling it: the batch path ends in one short wait for a 96-byte
    // result, where an interrupt-driven wake-up costs tens of microseconds per batch.  Long
    // waits (a compaction, a large load) fall back to the blocking call after ~1 ms.
    int sync() {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t e = hipStreamQuery(stream);
            if (e == hipSuccess) return RH_OK;
            if (e != hipErrorNotReady) return fail(RH_ERR_HIP, std::string("hipStreamQuery: ") + hipGetErrorString(e));
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(1)) break;
        }
        RH_HIP(hipStreamSynchronize(stream));
        return RH_OK;
    }
    // root_dst: where the base total lands (pinned memory keeps the copy asynchronous)
    int resum_base(bool have_block_sums = false, uint64_t *root_dst = nullptr, bool have_samples = false) {
        int rc;
        const size_t nbk = rh_num_blocks(nb), ns = rh_num_superblocks(nb);
        if ((rc = bsums.ensure(nbk * 32 + 32)) || (rc = ssums.ensure(ns * 32 + 32)) || (rc = tot.ensure(4)) ||
            (rc = bsmp.ensure(nbk + 1)) || (rc = bsmp2.ensure(rh::sample2_entries(nb))))
            return rc;
        if (nb) {
            if (!have_samples) RH_HIP(kops->sample(bkeys[cb].p, nb, bsmp.p, bsmp2.p, stream));
            if ((rc = btab.ensure((1ull << rh::search_table_bits(nb)) + 2)) || (rc = btabp.ensure(3))) return rc;
            RH_HIP(rh::launch_search_table(bsmp2.p, nb, btab.p, btabp.p, stream));
            if (!have_block_sums) RH_HIP(rh::launch_reduce(bfps[cb].p, nb, bsums.p, stream));
            RH_HIP(rh::launch_reduce(bsums.p, nbk, ssums.p, stream));
            RH_HIP(rh::launch_total(ssums.p, ns, tot.p, stream));
            RH_HIP(hipMemcpyAsync(root_dst ? root_dst : root_b, tot.p, 32, hipMemcpyDeviceToHost, stream));  // the caller syncs
        } else {
            memset(root_dst ? root_dst : root_b, 0, sizeof root_b);
        }
        return RH_OK;
    }
    // After a merge into delta buffer `buf` (sized for n_max rows; the merge wrote its block
    // sums and block count totals, zero past the true row count, which only the device knows):
    // the inclusive block prefix of the count deltas (its last entry -> *total), the super-block
    // sums, and the contribution total -> fp_total.  No host round trip.
    rh::CntPrefix cnt_prefix(int buf) const { return rh::CntPrefix{dsblk[buf].p, dblk[buf].p, dinb[buf].p}; }
    // The delta run's block sums and count prefixes are formed on the first question that needs
    // them after a batch (a key-range aggregate, a rank); the batch path keeps the run's count
    // and contribution totals itself (k_delta_build / k_delta_parts), so the root stays O(1).
    bool dsums_ok = true;
    DevBuf<uint64_t> fin_out;  // finish_delta_async's totals when only the sums are wanted
    int ensure_delta_sums() {
        int rc;
        if (nd == 0 || dsums_ok) return RH_OK;
        if ((rc = fin_out.ensure(8))) return rc;
        RH_HIP(rh::launch_delta_sums(dslot[cd].p, dheap.p, nd, dbsums[cd].p, dblk[cd].p, dinb[cd].p, stream));
        if ((rc = finish_delta_async(cd, nd, reinterpret_cast<int32_t *>(fin_out.p), fin_out.p + 4))) return rc;
        dsums_ok = true;
        return RH_OK;
    }
    int finish_delta_async(int buf, uint64_t n_max, int32_t *total, uint64_t *fp_total) {
        int rc;
        const size_t nbk = rh_num_blocks(n_max), ns = rh_num_superblocks(n_max) + 1;
        if ((rc = dsblk[buf].ensure(ns)) || (rc = dscnt.ensure(ns)) || (rc = dssums[buf].ensure(ns * 32))) return rc;
        if (!fin_ticket.p) {
            if ((rc = fin_ticket.ensure(1))) return rc;
            RH_HIP(hipMemsetAsync(fin_ticket.p, 0, 4, stream));
        }
        RH_HIP(rh::launch_delta_finish(dbsums[buf].p, dblk[buf].p, nbk, dssums[buf].p, dscnt.p, dsblk[buf].p,
                                       fin_ticket.p, total, fp_total, stream));
        return RH_OK;
    }
    // Replace the contents with m records.  Sorted, duplicate-free input is required unless
    // last_wins, which sorts on the device and keeps the last record of each repeated key --
    // the result of inserting the records one by one (just_insert_bulk, src/replica/write.rs:107-121).
    // sort m (key, fp, op) rows into key order (sops receives the ops); *flags & 1: duplicate
    // keys.  One sync: the MSD-only pass, then the full sort only if it reported a tie.
    int sort_keys(const uint8_t *keys, const uint8_t *fps, const uint8_t *ops, uint64_t m, uint8_t *okeys,
                  uint8_t *ofps, uint32_t *flags) {
        int rc;
        if ((rc = sops.ensure(m + 64)) || (rc = flag.ensure(4))) return rc;
        for (int full = 0; full < 2; full++) {
            RH_HIP(kops->sort_batch(keys, fps, ops, m, scratch, okeys, ofps, sops.p, flag.p, full == 1, stream));
            if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
            RH_HIP(hipMemcpyAsync(flags, flag.p, 4, hipMemcpyDeviceToHost, stream));
            if ((rc = sync())) return rc;
            if (!(*flags & 6)) return RH_OK;  // 2: leading-digit tie, 4: skewed buckets
        }
        return RH_OK;
    }
    static constexpr uint64_t DTAB_MIN = 1ull << 16;  // delta rows from which the delta search uses a table
    hipEvent_t dep = nullptr;  // orders the store's stream after a producer stream
    int after(void *producer) {
        if (!dep) RH_HIP(hipEventCreateWithFlags(&dep, hipEventDisableTiming));
        RH_HIP(hipEventRecord(dep, static_cast<hipStream_t>(producer)));
        RH_HIP(hipStreamWaitEvent(stream, dep, 0));
        return RH_OK;
    }
    // lifted: bfps[cb] and bsums already hold the records' fingerprints and block sums (the
    // snapshot reload's dual lift wrote them, sized exactly as below)
    int load_device(const rh_columns &c, size_t m, bool last_wins = false, bool lifted = false) {
        int rc = load_begin(c, m, lifted);
        return rc ? rc : load_finish(m, last_wins);
    }
    // the load in two halves, so that two stores loading the same columns (a snapshot reload)
    // overlap on their streams: begin enqueues the copy, the sortedness check and the sums;
    // finish waits, and re-orders the rows if the keys were not sorted
    PinnedVec<uint32_t> load_flag;
    int load_begin(const rh_columns &c, size_t m, bool lifted) {
        int rc = load_prep(m);
        if (rc) return rc;
        if (m) {
            RH_HIP(hipMemcpyAsync(bkeys[cb].p, c.keys, m * kl, hipMemcpyDeviceToDevice, stream));
            if (!lifted &&
                (rc = lift_dispatch(schema, c, m, bfps[cb].p, bsums.p, nullptr, nullptr, false, stream)))
                return rc;
            RH_HIP(hipMemsetAsync(flag.p, 0, 4, stream));
            RH_HIP(kops->check_sorted(bkeys[cb].p, m, flag.p, stream));
        }
        return load_sums(m, flag.p);
    }
    // a load's first part: an empty run with room for m base rows, whose keys, fingerprints and
    // block sums the caller then writes into bkeys[cb], bfps[cb] and bsums
    int load_prep(size_t m) {
        int rc;
        if ((rc = drain_prefix_build())) return rc;  // it reads bfps[cb], rewritten here
        // ranks are 32-bit on the device (searches, the protocol round): refuse what they cannot hold
        if (m >= (1ull << 31)) return fail(RH_ERR_ARG, "store size limit (2^31 rows) exceeded: use rh_sstore_* for a larger map");
        if ((rc = settle())) return rc;  // a tier copy in flight reads the base run
        health_reset();
        version++;
        base_epoch++;
        base_loaded = true;
        if ((rc = bkeys[cb].ensure(m * kl + 64)) || (rc = bfps[cb].ensure(m * 32 + 64)) || (rc = flag.ensure(4)) ||
            (rc = counts.ensure(4)))
            return rc;
        nd = 0;
        heap_len = 0;
        dtotal = 0;
        nb = 0;
        memset(root_d, 0, sizeof root_d);
        // the lift writes the block sums as it goes; they stand unless the keys turn out to be
        // unsorted (then the rows are re-ordered and everything is re-summed)
        return bsums.ensure(rh_num_blocks(m) * 32 + 32);
    }
    // the second part, once the m rows are in place (enqueued behind them on this stream):
    // super sums, samples and the root; *unsorted (device) -> the host copy load_finish checks
    int load_sums(size_t m, const uint32_t *unsorted, bool have_samples = false) {
        nb = m;
        load_flag.assign(10, 0);  // [0] unsorted flag, [2..9] the base total (8-byte aligned)
        uint64_t *root_pin = reinterpret_cast<uint64_t *>(load_flag.data() + 2);
        int rc = resum_base(true, root_pin, have_samples);
        if (rc) return rc;
        if (m) RH_HIP(hipMemcpyAsync(load_flag.data(), unsorted, 4, hipMemcpyDeviceToHost, stream));
        return RH_OK;
    }
    PinnedVec<uint64_t> snap_words;  // a fused snapshot reload's result words (snapshot_locate)
    PinnedVec<uint64_t> snap_hdr;    // a device snapshot's 16-byte header, read back during the walk
    hipEvent_t hdr_ev = nullptr;
    // A load whose rows are written before it is known to succeed (the fused snapshot reload):
    // the rows go to the spare base buffers, and the store changes only at load_commit -- a
    // corrupt file leaves it as it was, as Replica::load_snapshot does (src/snapshot.rs:76-98)
    DevBuf<uint8_t> sbsums, sssums;
    DevBuf<uint64_t> sbsmp, sbsmp2, sbtabp, stot;
    DevBuf<uint32_t> sbtab;
    int load_target(size_t m) {
        if (m >= (1ull << 31)) return fail(RH_ERR_ARG, "store size limit (2^31 rows) exceeded: use rh_sstore_* for a larger map");
        const int nxt = 1 - cb;
        int rc;
        if ((rc = drain_prefix_build())) return rc;  // one from two bases ago may read bfps[nxt]
        if ((rc = settle())) return rc;  // a tier copy in flight reads the base run
        // load_commit swaps the spare set in: it gets at least the active set's capacity, so that
        // rows reserved by rh_store_reserve stay reserved across a reload (no reallocation, and
        // no device-draining hipFree, at the next compaction)
        auto at_least = [](size_t need, size_t cap) { return std::max(need, cap); };
        if ((rc = bkeys[nxt].ensure(at_least(m * kl + 64, bkeys[cb].cap))) ||
            (rc = bfps[nxt].ensure(at_least(m * 32 + 64, bfps[cb].cap))) ||
            (rc = sbsums.ensure(at_least(rh_num_blocks(m) * 32 + 32, bsums.cap))) ||
            (rc = sssums.ensure(at_least(rh_num_superblocks(m) * 32 + 32, ssums.cap))) ||
            (rc = sbsmp.ensure(at_least(rh_num_blocks(m) + 1, bsmp.cap))) ||
            (rc = sbsmp2.ensure(at_least(rh::sample2_entries(m), bsmp2.cap))) ||
            (rc = sbtab.ensure(at_least((1ull << rh::search_table_bits(m)) + 2, btab.cap))) || (rc = sbtabp.ensure(3)) ||
            (rc = stot.ensure(4)) || (rc = flag.ensure(4)) || (rc = counts.ensure(4)))
            return rc;
        return RH_OK;
    }
    // behind the target's rows, block sums and samples (on st): its super sums, search table and
    // total, and the total and *unsorted into the pinned load_flag -- all in the spare buffers
    int load_stage_sums(size_t m, const uint32_t *unsorted, hipStream_t st) {
        const size_t nbk = rh_num_blocks(m), ns = rh_num_superblocks(m);
        load_flag.assign(10, 0);  // [0] unsorted flag, [2..9] the base total (8-byte aligned)
        RH_HIP(rh::launch_search_table(sbsmp2.p, m, sbtab.p, sbtabp.p, st));
        RH_HIP(rh::launch_reduce(sbsums.p, nbk, sssums.p, st));
        RH_HIP(rh::launch_total(sssums.p, ns, stot.p, st));
        RH_HIP(hipMemcpyAsync(load_flag.data() + 2, stot.p, 32, hipMemcpyDeviceToHost, st));
        RH_HIP(hipMemcpyAsync(load_flag.data(), unsorted, 4, hipMemcpyDeviceToHost, st));
        return RH_OK;
    }
    // the target becomes the base run (host state only: load_finish then takes the root and
    // checks the order flag)
    void load_commit(size_t m) {
        health_reset();
        auto swap_buf = [](auto &x, auto &y) {
            std::swap(x.p, y.p);
            std::swap(x.cap, y.cap);
        };
        cb = 1 - cb;
        swap_buf(bsums, sbsums);
        swap_buf(ssums, sssums);
        swap_buf(bsmp, sbsmp);
        swap_buf(bsmp2, sbsmp2);
        swap_buf(btab, sbtab);
        swap_buf(btabp, sbtabp);
        version++;
        base_epoch++;
        base_loaded = true;
        nd = 0;
        heap_len = 0;
        dtotal = 0;
        memset(root_d, 0, sizeof root_d);
        nb = m;
    }
    // page-locked host tier capacity for `rows` rows ahead of the refresh that fills it: pinning
    // fresh pages is most of a first refresh (11-13 ms at 10^6 rows against ~1 ms of copying)
    // A buffer the tier reads that moves (a larger reservation re-pins and copies) leaves the tier
    // stale: its pointers are re-taken by the next refresh, never read after the move.
    int tier_reserve(uint64_t rows) {
        if (!tier_on) return RH_OK;
        const void *k0 = tsets[tact].keys.p, *p0 = tsets[tact].prefix.p, *s0 = tsets[tact].samp.p;
        // the set the tier reads now; the spare set is pinned by the first refresh that copies into
        // it (start_refresh: a failure there leaves the tier stale, never fails the caller), so
        // enabling the tier or reserving pins (key_len + 32) B per row, not twice that
        try {
            TierSet &S = tsets[tact];
            S.keys.clear(), S.prefix.clear(), S.samp.clear();  // a move leaves the tier stale: nothing to keep
            S.keys.reserve(rows * kl + 64);
            S.prefix.reserve((rows + 1) * 4 + 8);
            S.samp.reserve(rows / 64 + rows / 4096 + 16);
        } catch (const std::bad_alloc &) {
            tier_version = ~0ull;
            return tier_oom();
        }
        // a base copy that moved is gone: the next refresh copies the base again (not a run copy)
        if (tsets[tact].keys.p != k0 || tsets[tact].prefix.p != p0 || tsets[tact].samp.p != s0)
            tier_version = ~0ull, tier_epoch = ~0ull;
        // the run copy's page-locked columns, for the largest run the policy copies (a quarter of
        // the base): pinned here, with the base's, not by the write whose run first outgrows them
        // (both sets under "writes never wait": the spare is filled while the tier reads the other)
        {
            const uint64_t rr = rows / 4 + (1u << 16);
            RunHost &H = trh[ract];
            const void *before[7] = {H.keys.p, H.pre.p, H.cntp.p, H.fl.p, H.br.p, H.smp.p, H.gs.p};
            try {
                auto room = [](auto &v, size_t want) {
                    if (v.capacity() < want) {
                        v.clear();
                        v.reserve(want);
                    }
                };
                for (int k = 0; k < (tier_sync_writes ? 1 : 2); k++) {
                    RunHost &R = trh[k == 0 ? ract : 1 - ract];
                    room(R.keys, rr * kl + 64);
                    room(R.pre, (rr + 1) * 4 + 8);
                    room(R.cntp, rr + 16);
                    room(R.fl, rr + 16);
                    room(R.br, rr + 16);
                    room(R.smp, rr / 64 + rr / 4096 + 16);
                    room(R.gs, rr / 64 + 16);
                }
            } catch (const std::bad_alloc &) {
                tier_version = ~0ull;
                return tier_oom();
            }
            const void *after[7] = {H.keys.p, H.pre.p, H.cntp.p, H.fl.p, H.br.p, H.smp.p, H.gs.p};
            if (tier.has_run() && memcmp(before, after, sizeof before)) tier_version = ~0ull;  // a held run moved
        }
        return RH_OK;
    }
    int load_finish(size_t m, bool last_wins) {
        int rc = load_finish_rows(m, last_wins);
        if (rc) return rc;
        tier_host_oom = false;
        rc = tier_reserve(nb + nb / 4);
        if (!rc) rc = start_refresh();  // the tier copies the new base in the background
        if (!rc && tier_sync_writes) rc = settle();  // ... and, with writes keeping it fresh, the load waits
        return tier_stale_on_host_oom(rc);
    }
    int load_finish_rows(size_t m, bool last_wins) {
        int rc;
        if ((rc = sync())) return rc;
        memcpy(root_b, load_flag.data() + 2, sizeof root_b);
        const uint32_t bad = load_flag[0];
        if (!bad) return RH_OK;
        nb = 0;  // an error below leaves the store empty
        memset(root_b, 0, sizeof root_b);
        uint64_t kept = m;
        {
            if (!last_wins) return fail(RH_ERR_ARG, "keys must be strictly increasing (sorted, no duplicates)");
            const int nxt = 1 - cb;
            if ((rc = bkeys[nxt].ensure(m * kl + 64)) || (rc = bfps[nxt].ensure(m * 32 + 64)) || (rc = sops.ensure(m + 64)))
                return rc;
            uint32_t flags = 0;
            if ((rc = sort_keys(bkeys[cb].p, bfps[cb].p, nullptr, m, bkeys[nxt].p, bfps[nxt].p, &flags))) return rc;
            if (flags & 1) {  // stable sort: within a run of equal keys the last record is last
                RH_HIP(kops->dedup_last(bkeys[nxt].p, bfps[nxt].p, m, scratch, bkeys[cb].p, bfps[cb].p, counts.p,
                                        stream));
                if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
                RH_HIP(hipMemcpyAsync(&kept, counts.p, 8, hipMemcpyDeviceToHost, stream));
                if ((rc = sync())) return rc;
            } else {
                cb = nxt;
            }
        }
        nb = kept;
        if ((rc = resum_base())) return rc;
        return sync();
    }
    int compact() {  // merge the delta run into the base run
        int rc;
        if (nd == 0) return RH_OK;
        if ((rc = drain_prefix_build())) return rc;  // one from two bases ago may read bfps[1 - cb]
        // a tier copy in flight reads bkeys[rf_cb]; the merge writes the other base buffer, so one
        // compaction runs beside the copy (whose log then breaks: later batches' records are
        // relative to the new base), and a second one, which would write the buffer being copied,
        // waits for it
        if (rf_on && !rf_run) {
            if (1 - cb == rf_cb) {
                if ((rc = settle())) return rc;
            } else {
                rf_log_ok = false;
                // the merge rewrites the base's block sums, which the copy's prefix scan reads
                RH_HIP(hipStreamWaitEvent(stream, rf_kdone, 0));
            }
        }
        if ((rc = cfps.ensure(nd * 32 + 64)) || (rc = cops.ensure(nd + 64))) return rc;
        const int nxt = 1 - cb;
        const uint64_t nbk = rh_num_blocks(nb + nd);
        if ((rc = bkeys[nxt].ensure((nb + nd) * kl + 64)) || (rc = bfps[nxt].ensure((nb + nd) * 32 + 64)) ||
            (rc = bsums.ensure(nbk * 32 + 32)) || (rc = mcnt.ensure(8)) || (rc = bsmp.ensure(nbk + 1)) ||
            (rc = bsmp2.ensure(rh::sample2_entries(nb + nd))))
            return rc;
        // every delta key's base slot is in its DeltaRec (brank): the merge needs no search; the
        // merged base, its block sums and its search samples in one pass
        RH_HIP(rh::launch_compact(schema.key_kind, (int)kl, bkeys[cb].p, bfps[cb].p, nb, dkeys[cd].p, dslot[cd].p, dheap.p, nd,
                                  scratch, cfps.p, cops.p, bkeys[nxt].p, bfps[nxt].p, bsums.p, nbk, mcnt.p, bsmp.p, bsmp2.p,
                                  stream));
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        try {
            res_host.resize(12);
        } catch (const std::bad_alloc &) {
            return fail(RH_ERR_OOM, "pinned result buffer");
        }
        // the merged size is known on the host (size() = base rows + the delta run's count total),
        // so the sums and the search table are enqueued behind the merge without a round trip; the
        // merge's own counts (pinned, asynchronous) are checked against it after the one sync
        uint64_t *c = res_host.data();
        if ((rc = down_small(res_host, mcnt.p, 24))) return rc;
        const uint64_t want = size(), nb_old = nb;
        base_epoch++;  // same contents, a new base: the tier's copy stays valid, not the device's deltas
        base_loaded = false;
        cb = nxt;
        nb = want;
        nd = 0;
        heap_len = 0;
        dtotal = 0;
        memset(root_d, 0, sizeof root_d);
        compactions++;
        if ((rc = resum_base(true, nullptr, true))) return rc;
        if ((rc = sync())) return rc;
        if (nb_old + c[0] - c[2] != want) return fail(RH_ERR_STATE, "compaction size mismatch (internal error)");
        return RH_OK;
    }
    // Capacity for `rows` resident rows taking batches of up to `batch` rows: both base buffers
    // for a compaction's output, both delta buffers for the largest run the policy allows, the
    // batch buffers and the merge / compaction scratch.  Growing any of these later frees the
    // old buffer, and hipFree waits for the whole device.
    int reserve(uint64_t rows, uint64_t batch) {
        int rc;
        if ((rc = settle())) return rc;   // a tier copy in flight reads the base run it may move
        if ((rc = compact())) return rc;  // the delta run is empty: its buffers hold nothing
        const uint64_t thresh = std::max<uint64_t>(rows / compact_div, compact_min);
        const uint64_t plan = thresh + batch, base = rows + plan;
        for (int k = 0; k < 2; k++) {
            if (k == cb) {
                if ((rc = bkeys[k].grow_keep(base * kl + 64, nb * kl, stream)) ||
                    (rc = bfps[k].grow_keep(base * 32 + 64, nb * 32, stream)))
                    return rc;
            } else if ((rc = bkeys[k].ensure(base * kl + 64)) || (rc = bfps[k].ensure(base * 32 + 64))) {
                return rc;
            }
            if ((rc = dkeys[k].ensure(plan * kl + 64)) || (rc = dslot[k].ensure(plan + 16)) ||
                (rc = dbsums[k].ensure(rh_num_blocks(plan) * 32 + 32)) ||
                (rc = dssums[k].ensure(rh_num_superblocks(plan) * 32 + 32)) ||
                (rc = dsblk[k].ensure(rh_num_superblocks(plan) + 16)) || (rc = dscnt.ensure(rh_num_superblocks(plan) + 16)) ||
                (rc = dblk[k].ensure(rh_num_blocks(plan) + 16)) || (rc = dinb[k].ensure(plan + 16)))
                return rc;
        }
        if ((rc = bsums.ensure(rh_num_blocks(base) * 32 + 32)) || (rc = ssums.ensure(rh_num_superblocks(base) * 32 + 32)) ||
            (rc = bsmp.ensure(rh_num_blocks(base) + 1)) || (rc = bsmp2.ensure(rh::sample2_entries(base))) ||
            (rc = btab.ensure((1ull << rh::search_table_bits(base)) + 2)) || (rc = btabp.ensure(3)) ||
            (rc = dtab.ensure((1ull << rh::search_table_bits(plan, false)) + 2)) || (rc = dtabp.ensure(3)) ||
            (rc = dsmp[0].ensure(rh_num_blocks(plan) + 1)) || (rc = dsmp[1].ensure(rh_num_blocks(plan) + 1)) ||
            (rc = dsmp2[0].ensure(rh::sample2_entries(plan))) || (rc = dsmp2[1].ensure(rh::sample2_entries(plan))) ||
            (rc = cfps.ensure(plan * 32 + 64)) ||
            (rc = cops.ensure(plan + 64)) || (rc = skeys.ensure(batch * kl + 64)) ||
            (rc = sfps.ensure(batch * 32 + 64)) || (rc = sops.ensure(std::max(batch, base) + 64)) ||
            (rc = dheap.ensure(plan * sizeof(rh::DeltaRec) + 64)) || (rc = dops.ensure(batch + 64)) ||
            (rc = mcnt.ensure(8)) || (rc = results.ensure(12)) || (rc = flag.ensure(4)) || (rc = counts.ensure(4)))
            return rc;
        RH_HIP(rh::reserve_merge_scratch(scratch, plan, batch, base));
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        if (tier_on && (rc = refresh_room())) return rc;
        // the row prefix's stream now, not at a later question (creating a queue takes ms)
        if (row_prefix == 1 && !pstream) {
            RH_HIP(back_stream(device, 1, &pstream));
            RH_HIP(hipEventCreateWithFlags(&pre_ev, hipEventDisableTiming));
            RH_HIP(hipEventCreateWithFlags(&pre_base_ev, hipEventDisableTiming));
        }
        tier_host_oom = false;
        // the tier's page-locked room: a failure leaves the tier stale, not the device reservation failed
        if ((rc = tier_stale_on_host_oom(tier_reserve(rows)))) return rc;
        // bsums / ssums / samples may have moved: derive them again from the kept fingerprints
        if ((rc = resum_base())) return rc;
        if ((rc = sync())) return rc;
        // a tier whose page-locked sets moved is stale: with writes keeping it fresh, the
        // reservation (a setup call) copies it again now, not the next question's device path
        if (tier_on && tier_sync_writes && !tier_fresh() && !rf_on && (rc = tier_stale_on_host_oom(start_refresh())))
            return rc;
        return tier_sync_writes ? settle() : RH_OK;
    }
    hipEvent_t res_ev = nullptr;  // apply_device_many: the result copy of the batch in flight
    int sync_event(hipEvent_t ev) {  // sync() for one event: poll ~1 ms, then block
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t e = hipEventQuery(ev);
            if (e == hipSuccess) return RH_OK;
            if (e != hipErrorNotReady) return fail(RH_ERR_HIP, std::string("hipEventQuery: ") + hipGetErrorString(e));
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(1)) break;
        }
        RH_HIP(hipEventSynchronize(ev));
        return RH_OK;
    }
    // k batches in order, each exactly as apply_device would apply it; batch i + 1 is sorted
    // while the host waits for batch i's result, so the device does not idle between
    // batches.  On an error, batches before the failing one stay applied, the failing one and
    // those after it are not.
    int apply_device_many(const rh_columns *cs, const uint8_t *const *ops, const size_t *ms, size_t k, uint64_t *out) {
        int rc;
        size_t mmax = 0;
        for (size_t i = 0; i < k; i++) {
            mmax = std::max(mmax, ms[i]);
            out[3 * i] = out[3 * i + 1] = out[3 * i + 2] = 0;
        }
        // every batch's buffers at the largest size first: growing one later frees it (a device drain)
        if ((rc = batch_buffers(mmax))) return rc;
        bool prepared = false;
        for (size_t i = 0; i < k; i++) {
            const bool pipe = ms[i] > 0 && i + 1 < k && ms[i + 1] > 0;
            bool next_prepared = false;
            rc = apply_device(cs[i], ops ? ops[i] : nullptr, ms[i], out + 3 * i, prepared, pipe ? &cs[i + 1] : nullptr,
                              pipe && ops ? ops[i + 1] : nullptr, pipe ? ms[i + 1] : 0, &next_prepared);
            if (rc) return rc;
            prepared = next_prepared;
        }
        return RH_OK;
    }
    // the batch buffers for batches of up to m rows (sorted keys / fingerprints / ops, the sort's
    // positions, the per-key search results)
    int batch_buffers(size_t m) {
        int rc;
        if ((rc = skeys.ensure(m * kl + 64)) || (rc = sfps.ensure(m * 32 + 64)) || (rc = sops.ensure(m + 64)) ||
            (rc = dops.ensure(m + 64)) || (rc = flag.ensure(4)) || (rc = counts.ensure(4)) || (rc = results.ensure(12)))
            return rc;
        (void)scratch.u32(7, m), (void)scratch.u32(9, m), (void)scratch.u32(10, m), (void)scratch.i32(0, m);
        (void)scratch.u8(2, m), (void)scratch.u8(3, m);
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        return RH_OK;
    }
    // Step 1 of a batch: the key sort (sorted keys / ops into skeys / sops, each input row's sorted
    // row into the position scratch, the sort's flags into the result block).  Queued only; needs
    // batch_buffers(m).  The lift comes after it (step 2), writing each fingerprint straight to
    // its sorted row of sfps, so the sort gathers no fingerprints.
    // pre: the keys' digit min / max partials are in the pre-minmax slot (queued by the previous
    // batch's k_lift_search, pre_minmax)
    // The bucket sort's positions come in two levels (store_kernels.hpp sort_batch): scratch u32(7)
    // holds each input row's slot and sort_s2o each slot's sorted row; the full sort writes the sorted
    // rows into u32(7) directly (sort_s2o = nullptr).
    uint32_t *sort_s2o = nullptr;
    int prepare_batch(const rh_columns &c, const uint8_t *ops, size_t m, bool full, bool pre = false) {
        uint32_t *pos = scratch.u32(7, m);
        const bool two = !full && m <= rh::SORT_BUCKET_MAX;
        uint32_t *s2o = two ? reinterpret_cast<uint32_t *>(scratch.i32(0, m)) : nullptr;
        const uint32_t npart = (uint32_t)((m + rh::MINMAX_TILE - 1) / rh::MINMAX_TILE);
        const uint64_t *part = pre ? scratch.u64(3, 2ull * npart) : nullptr;
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        sort_s2o = s2o;
        uint32_t *r_flags = reinterpret_cast<uint32_t *>(results.p + 6);
        RH_HIP(kops->sort_batch(static_cast<const uint8_t *>(c.keys), nullptr, ops, m, scratch, skeys.p, nullptr, sops.p,
                                r_flags, full, stream, pos, part, npart, s2o));
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        return RH_OK;
    }
    // Steps 2-3: the lift into the sorted rows and the searches of the sorted keys in the base and
    // delta runs, as one fused launch (lift_search.hpp) -- or, for a shape without one, the lift
    // and the two search kernels.
    // next (nullable): the next batch, whose keys' digit min / max the fused launch also forms
    // (*pre_minmax = whether it did: its sort then skips that pass)
    int lift_and_search(const rh_columns &c, size_t m, const rh::SearchJob &jb, const rh::SearchJob &jd,
                        const rh_columns *next = nullptr, size_t next_m = 0, bool *pre_minmax = nullptr) {
        if (pre_minmax) *pre_minmax = false;
        const uint32_t *pos = scratch.u32(7, m);
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        if (fused_lift_search) {
            rh::DevCols dc = to_dev(c);
            dc.dst = pos;
            dc.dst2 = sort_s2o;
            rh::NextMinmax nx{};
            if (next && next_m && next_m <= rh::SORT_BUCKET_MAX && pre_minmax) {
                nx.keys = static_cast<const uint8_t *>(next->keys);
                nx.m = next_m;
                nx.part = scratch.u64(3, 2 * ((next_m + rh::MINMAX_TILE - 1) / rh::MINMAX_TILE));
                if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
            }
            bool supported = false;
            const bool timed = g_time_batch.load() != 0;
            if (timed && !ls_ev[0]) {
                RH_HIP(hipEventCreate(&ls_ev[0]));
                RH_HIP(hipEventCreate(&ls_ev[1]));
            }
            // timed: the launch stamps the events itself (hipExtLaunchKernel), so timing it adds
            // no marker packets -- and no ~6 us gaps -- around the kernel
            const hipError_t e =
                rh::launch_lift_search_schema(schema.key_kind, (int)schema.key_len, schema.value_kind, (int)schema.value_len,
                                              schema.record_kind, c.tags != nullptr, dc, m, sfps.p, skeys.p, jb, jd, nx,
                                              stream, &supported, timed ? ls_ev[0] : nullptr, timed ? ls_ev[1] : nullptr);
            if (timed && supported && e == hipSuccess) ls_pending = true;
            if (e != hipSuccess) return fail(RH_ERR_HIP, std::string("lift + search launch: ") + hipGetErrorString(e));
            if (supported) {
                if (pre_minmax) *pre_minmax = nx.keys != nullptr;
                return RH_OK;
            }
        }
        int rc;
        if ((rc = lift_dispatch(schema, c, m, sfps.p, nullptr, nullptr, nullptr, false, stream, pos, sort_s2o)))
            return rc;
        RH_HIP(kops->search_sampled(jb.keys, jb.n, jb.smp, jb.smp2, skeys.p, m, jb.rank, jb.present, stream, jb.tb));
        RH_HIP(kops->search_sampled(jd.keys, jd.n, jd.smp, jd.smp2, skeys.p, m, jd.rank, jd.present, stream, jd.tb));
        return RH_OK;
    }
    hipEvent_t ls_ev[2] = {nullptr, nullptr};  // rh_debug_batch_timing: around the fused launch
    bool ls_pending = false;
    void take_batch_timing() {  // after the batch's wait: the launch's time into the global sum
        if (!ls_pending) return;
        ls_pending = false;
        float ms = 0;
        if (hipEventElapsedTime(&ms, ls_ev[0], ls_ev[1]) != hipSuccess) {
            (void)hipGetLastError();
            return;
        }
        std::lock_guard<std::mutex> g(g_batch_mu);
        g_batch_us += 1000.0 * ms;
        g_batch_n++;
    }
    // A/B switch: RSOS_HIP_PRE_MINMAX=0 = the next batch's sort runs its own min / max pass
    bool pre_minmax_on = !(getenv("RSOS_HIP_PRE_MINMAX") && *getenv("RSOS_HIP_PRE_MINMAX") == '0');
    // A/B switch: RSOS_HIP_UNFUSED set (non-empty) = separate lift / search launches
    bool fused_lift_search = !(getenv("RSOS_HIP_UNFUSED") && *getenv("RSOS_HIP_UNFUSED"));
    PinnedVec<uint64_t> res_host;  // the batch's 96-byte result block
    // prepared: step 1 of this batch was queued by the previous call (apply_device_many).
    // next: a batch whose step 1 is queued once this batch's kernels are -- the device runs them
    // while the host waits for this batch's result (an event on the result copy, not the stream);
    // *next_prepared says whether they were (a re-sort of this batch overwrites them).
    // last_wins: repeated keys keep their last row (the staged batch); otherwise they reject the batch
    int apply_device(const rh_columns &c, const uint8_t *ops, size_t m, uint64_t out[3], bool prepared = false,
                     const rh_columns *next = nullptr, const uint8_t *next_ops = nullptr, size_t next_m = 0,
                     bool *next_prepared = nullptr, bool last_wins = false) {
        int rc;
        out[0] = out[1] = out[2] = 0;
        if (next_prepared) *next_prepared = false;
        if (m == 0) return RH_OK;
        if (nb + nd + m >= (1ull << 31)) return fail(RH_ERR_ARG, "store size limit (2^31 rows) exceeded: use rh_sstore_* for a larger map");
        // keeping the last row of a repeated key needs the sort to order ties by input row, which
        // the batch sort does only when it carries the rows' indices (it does with ops)
        if (last_wins && !ops) return fail(RH_ERR_ARG, "last-wins batch without its op column");
        if ((rc = pre_batch())) return rc;
        if (!prepared && !next && m <= small_limit()) {  // the small-batch path: two launches
            bool done = false;
            if ((rc = apply_small(c, ops, m, last_wins, out, &done))) return rc;
            if (done) return RH_OK;
        }
        snap_ok = run_copy_allowed(m);
        int fmode = fold_mode(m);  // how this batch reaches a fresh host tier
        bool want = fold_rows_wanted(fmode);
        if (want && !fold_room(m)) fmode = 0, want = false, rf_log_ok = false;  // the tier goes stale
        const uint64_t version0 = version;
        version++;  // a rejected batch leaves the contents as they were; the tier refreshes anyway
        if ((rc = batch_buffers(m))) return rc;
        // 1. key sort (queued by the previous call when prepared)
        if (!prepared && (rc = prepare_batch(c, ops, m, false))) return rc;
        // 2-5 run without a host round trip: everything is written to the delta run's *other*
        // buffers, and one sync at the end brings back the flags and counts.  A duplicate key
        // then leaves the store exactly as it was (nothing is committed); a tie on the leading
        // key digit re-runs the steps with the full sort.
        const int nxt = 1 - cd;
        const uint64_t n_max = nd + m;
        uint32_t *rank_b = scratch.u32(9, m), *rank_d = scratch.u32(10, m);
        uint8_t *present_b = scratch.u8(2, m), *present_d = scratch.u8(3, m);
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        // capacity for the largest delta run the policy allows (threshold + one batch), so the
        // run grows without reallocations (a hipFree drains the device)
        const uint64_t thresh = std::max<uint64_t>(nb / compact_div, compact_min);
        const uint64_t plan = std::max<uint64_t>(n_max, std::min<uint64_t>(thresh, nb + nd) + m);
        // the heap keeps its records (the live delta rows point into it) when it grows
        if ((rc = dheap.grow_keep((heap_len + m) * sizeof(rh::DeltaRec) + 64, heap_len * sizeof(rh::DeltaRec), stream)))
            return rc;
        if ((rc = dkeys[nxt].ensure(plan * kl + 64)) || (rc = dslot[nxt].ensure(plan + 16)) ||
            (rc = dbsums[nxt].ensure(rh_num_blocks(plan) * 32 + 32)) ||
            (rc = dssums[nxt].ensure(rh_num_superblocks(plan) * 32 + 32)) ||
            (rc = dsblk[nxt].ensure(rh_num_superblocks(plan) + 16)) || (rc = dscnt.ensure(rh_num_superblocks(plan) + 16)) ||
            (rc = dblk[nxt].ensure(rh_num_blocks(plan) + 16)) || (rc = dinb[nxt].ensure(plan + 16)) ||
            (rc = dsmp[nxt].ensure(rh_num_blocks(plan) + 1)) || (rc = dsmp2[nxt].ensure(rh::sample2_entries(plan))) ||
            (rc = dsmp[cd].ensure(1)) || (rc = dsmp2[cd].ensure(1)) || (rc = mcnt.ensure(8)))
            return rc;
        // one 96-byte result block, one D2H copy: [0..2] batch counts, [3..5] merge counts,
        // [6] sort flags, [7] the change of the delta run's count total (int64), [8..11] the change
        // of its contribution total
        uint64_t *r_counts = results.p, *r_merge = results.p + 3;
        int64_t *r_dcnt = reinterpret_cast<int64_t *>(results.p + 7);
        // pinned: the copy stays asynchronous and sync() polls for it (a pageable destination
        // makes the runtime stage the copy and block in an interrupt-driven wait)
        try {
            res_host.resize(12);
        } catch (const std::bad_alloc &) {
            return fail(RH_ERR_OOM, "pinned result buffer");
        }
        uint64_t *host = res_host.data();
        uint32_t flags = 0;
        int next_rc = RH_OK;
        bool pre = false;  // the next batch's digit min / max formed by this batch's fused launch
        for (int full = 0; full < 2; full++) {
            // 1 again with the full sort (the bucket sort's order was not final)
            if (full == 1 && (rc = prepare_batch(c, ops, m, true))) return rc;
            // 2-3. the lift, and where each key is now (base and delta runs).  A delta run of more
            // than a few blocks is searched through a table over its stride-8 samples (one
            // L2-resident table line instead of a binary search of the stride-256 samples); the
            // table is built here, where the run's row count is known on the host
            rh::SearchTable dt{};
            if (nd >= DTAB_MIN) {
                if ((rc = dtab.ensure((1ull << rh::search_table_bits(nd, false)) + 2)) || (rc = dtabp.ensure(3))) return rc;
                if (full == 0) RH_HIP(rh::launch_search_table(dsmp2[cd].p, nd, dtab.p, dtabp.p, stream, false));
                dt = rh::SearchTable{dtab.p, dtabp.p, rh::search_table_bits(nd, false)};
            }
            rh::SearchJob jb{bkeys[cb].p, nb, bsmp.p, bsmp2.p, base_table(), rank_b, present_b};
            rh::SearchJob jd{dkeys[cd].p, nd, dsmp[cd].p, dsmp2[cd].p, dt, rank_d, present_d};
            if (!jb.smp2 || nb == 0) jb.tb = rh::SearchTable{};
            if (!jd.smp2 || nd == 0) jd.tb = rh::SearchTable{};
            // (the first pass also forms the next batch's digit min / max for its sort)
            const bool want_pre = full == 0 && next && next_m && pre_minmax_on;
            if ((rc = lift_and_search(c, m, jb, jd, want_pre ? next : nullptr, next_m, want_pre ? &pre : nullptr)))
                return rc;
            // 4. the batch's delta records and counts, merged into the delta run's other buffer
            //    (one pass: the merged run, its block sums, count prefixes and search samples)
            RH_HIP(rh::launch_delta_apply(schema.key_kind, (int)kl, sfps.p, sops.p, m, rank_b, present_b, bfps[cb].p,
                                          rank_d, present_d, dkeys[cd].p, dslot[cd].p, nd, dheap.p, heap_len, skeys.p,
                                          dops.p, r_counts, scratch, dkeys[nxt].p, dslot[nxt].p, dbsums[nxt].p, dblk[nxt].p,
                                          dinb[nxt].p, rh_num_blocks(n_max), mcnt.p, r_merge, dsmp[nxt].p,
                                          dsmp2[nxt].p, results.p + 8, r_dcnt, stream));
            if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
            // the batch's rows for the host tier's fold and a refresh's log
            if (want && (rc = fold_copies(skeys.p, sfps.p, sops.p, dheap.p + heap_len * sizeof(rh::DeltaRec), dops.p, m)))
                return rc;
            // 5. the one round trip
            if ((rc = down_small(res_host, results.p, 96))) return rc;
            if (full == 0 && next && next_m) {
                if (!res_ev) RH_HIP(hipEventCreateWithFlags(&res_ev, hipEventDisableTiming));
                RH_HIP(hipEventRecord(res_ev, stream));
                // a failure to queue the next batch is reported after this batch commits (the
                // batches before the failing one stay applied), never instead of it
                next_rc = batch_buffers(next_m);
                if (!next_rc) next_rc = prepare_batch(*next, next_ops, next_m, false, pre);
                if ((rc = next_rc ? sync() : sync_event(res_ev))) return rc;
                if (next_prepared) *next_prepared = !next_rc;
            } else if ((rc = sync())) {
                return rc;
            }
            memcpy(&flags, &host[6], 4);
            take_batch_timing();
            if (!(flags & 6)) break;  // 2: leading-digit tie, 4: skewed buckets
            if (next_prepared) *next_prepared = false;  // the re-sort overwrites the next batch's step 1
        }
        int64_t dcnt;
        memcpy(&dcnt, &host[7], 8);
        const uint64_t c2[3] = {host[3], host[4], host[5]};
        out[0] = host[0];
        out[1] = host[1];
        out[2] = host[2];
        if (flags & 1) {
            out[0] = out[1] = out[2] = 0;
            if (!last_wins || next) return fail(RH_ERR_ARG, "duplicate key within one batch");
            // nothing was committed: reduce the batch to the last row of each key (the sort's
            // positions and sorted keys are still in place) and apply that
            version = version0;
            if (next_prepared) *next_prepared = false;
            return apply_last_rows(c, ops, m, out);
        }
        cd = nxt;
        nd = nd + c2[0] - c2[2];
        heap_len += m;
        large_batches++;
        dtotal += dcnt;
        rh_fp_add(root_d, &host[8], root_d);  // mod 2^256
        dsums_ok = false;
        fold_batch(fmode, m, want);
        // the heap also holds records no row points to any more (overwritten or dropped keys)
        const uint64_t thresh_now = std::max<uint64_t>(nb / compact_div, compact_min);
        if (nd > thresh_now || heap_len > thresh_now) {
            if ((rc = compact())) return rc;
        }
        if ((rc = post_batch())) return rc;
        return next_rc ? next_rc : RH_OK;
    }
    // A batch with repeated keys, after its sort (scratch u32(7): each input row's sorted row; skeys:
    // the stable sort): the last row of each key, in input order, into the second column set, then
    // applied as a batch without repeats.
    DevColumns lastcols;
    DevBuf<uint8_t> lastops;
    int apply_last_rows(const rh_columns &c, const uint8_t *ops, size_t m, uint64_t out[3]) {
        int rc;
        const uint32_t *pos = scratch.u32(7, m);
        uint32_t *keep = scratch.u32(11, m + 1), *dst = scratch.u32(12, m + 1);
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        RH_HIP(kops->keep_last_rows(skeys.p, pos, sort_s2o, m, keep, stream));
        RH_HIP(rh::launch_exclusive_scan_u32(keep, dst, m + 1, scratch, stream));
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        try {
            res_host.resize(12);
        } catch (const std::bad_alloc &) {
            return fail(RH_ERR_OOM, "pinned result buffer");
        }
        RH_HIP(hipMemcpyAsync(res_host.data(), dst + m, 4, hipMemcpyDeviceToHost, stream));
        if ((rc = sync())) return rc;
        uint32_t kept;
        memcpy(&kept, res_host.data(), 4);
        const size_t kr = kl, vr = value_row(schema);
        const bool dated = schema.record_kind == RH_REC_DATED, tags = c.tags != nullptr;
        if ((rc = lastcols.keys.ensure(kept * kr + 16)) || (rc = lastcols.values.ensure(kept * vr + 16)) ||
            (rc = lastops.ensure(kept + 64)))
            return rc;
        if (dated && ((rc = lastcols.phys.ensure(kept + 1)) || (rc = lastcols.node.ensure(kept + 1)) ||
                      (rc = lastcols.logical.ensure(kept + 1))))
            return rc;
        if (tags && (rc = lastcols.tags.ensure(kept + 16))) return rc;
        lastcols.has_tags = tags;
        auto cp = [&](const void *src, uint32_t row, void *o) -> hipError_t {
            return rh::launch_compact_rows(static_cast<const uint8_t *>(src), row, keep, dst, m, static_cast<uint8_t *>(o),
                                           stream);
        };
        RH_HIP(cp(c.keys, (uint32_t)kr, lastcols.keys.p));
        RH_HIP(cp(c.values, (uint32_t)vr, lastcols.values.p));
        if (dated) {
            RH_HIP(cp(c.phys, 8, lastcols.phys.p));
            RH_HIP(cp(c.node, 8, lastcols.node.p));
            RH_HIP(cp(c.logical, 4, lastcols.logical.p));
        }
        if (tags) RH_HIP(cp(c.tags, 1, lastcols.tags.p));
        if (ops) RH_HIP(cp(ops, 1, lastops.p));
        else RH_HIP(hipMemsetAsync(lastops.p, 0, kept, stream));
        if (!c.values && kept) RH_HIP(hipMemsetAsync(lastcols.values.p, 0, kept * vr, stream));
        return apply_device(lastcols.view(schema), lastops.p, kept, out);
    }
    // Reads while a delta run is pending go to base + run as they stand (no O(n) compaction on a
    // read): the run's columns (run_columns) and the base run, as the device kernels take them
    int view_of(rh::RoundRun *run, rh::RoundIn *in) {
        int rc;
        if ((rc = run_columns())) return rc;
        if ((rc = ensure_base_prefix())) return rc;
        *run = rh::RoundRun{nd,
                            dkeys[cd].p,
                            trs[tcur].c.p,
                            trs[tcur].bs.p,
                            trs[tcur].ss.p,
                            reinterpret_cast<const int32_t *>(trs[tcur].cntp.p),
                            trs[tcur].fl.p,
                            trs[tcur].br.p,
                            trs[tcur].gs.p,
                            nb,
                            trs[tcur].bpre.p,
                            trun_pre_ver == version ? trs[tcur].pre.p : nullptr};
        *in = base_in();
        return RH_OK;
    }
    // The base run's exclusive prefixes, formed once per base (after a load or a compaction) on the
    // first question that sums over it on the device: over its block sums (bpre_b[k] = Σ blocks
    // [0, k), ~n / 256 entries, on the store's stream: any range sum is head and tail rows plus one
    // difference) and, when the device has the room (32 B a row: 3.2 GB at 10^8 rows), over its
    // rows (pre_b[i] = Σ fps [0, i): any range sum is one difference, two loads).  The row prefix
    // reads and writes 64 B a row (~1.2 ms at 10^8 rows), so it is formed at a loaded base's first
    // question, or once a compacted base has served max(16, n / 2^20) device questions, beside them
    // on a stream of its own (pstream), and
    // used from the first question after it has landed (pre_ev); until then the block prefix
    // serves.  A base that changes every few questions (large batches with compactions between
    // drives) never forms it.  RSOS_HIP_ROW_PREFIX=0: block prefix only;
    // 2: the row prefix in order on the store's stream, used from the first question (tests).
    DevBuf<uint8_t> bpre_b, spre_b, pre_b;
    uint64_t bpre_epoch = ~0ull, pre_epoch = ~0ull;
    bool pre_b_ok = false, pre_pending = false;
    hipStream_t pstream = nullptr;
    hipEvent_t pre_ev = nullptr, pre_base_ev = nullptr;
    int row_prefix = getenv("RSOS_HIP_ROW_PREFIX") ? atoi(getenv("RSOS_HIP_ROW_PREFIX")) : 1;
    // before anything rewrites a base buffer or pre_b: the build in flight reads them (host wait;
    // the build is long done in the common case)
    int drain_prefix_build() {
        if (!pre_pending) return RH_OK;
        RH_HIP(hipEventSynchronize(pre_ev));
        pre_pending = false;
        pre_b_ok = pre_epoch == base_epoch;
        return RH_OK;
    }
    uint64_t epoch_questions = 0;  // device questions over the current base so far
    bool base_loaded = true;       // the current base came from a load (false: a compaction)
    // the rows either base buffer holds (a compaction switches between them; they grow separately)
    uint64_t base_cap_rows() const { return std::max(bfps[0].cap, bfps[1].cap) / 32; }
    int ensure_base_prefix() {
        int rc;
        if (bpre_epoch != base_epoch || !bpre_b.p) {
            // sized for the base buffer's capacity (a reserved store's base grows by compactions
            // without reallocating; a hipFree here would wait for a tier copy in flight: no-wait
            // drives of ~175 ms, profiles/r05_nowait_long_calls.txt)
            const uint64_t cap_rows = std::max<uint64_t>(nb, base_cap_rows());
            const uint64_t nbk = rh_num_blocks(cap_rows), ns = rh_num_superblocks(cap_rows);
            if (pre_pending) RH_HIP(hipStreamWaitEvent(stream, pre_ev, 0));  // it reads bpre_b
            if ((rc = bpre_b.ensure((nbk + 1) * 32 + 64)) || (rc = spre_b.ensure((ns + 1) * 32 + 64))) return rc;
            pre_b_ok = false;
            if (nb) RH_HIP(rh::launch_block_prefix(nb, bsums.p, ssums.p, spre_b.p, bpre_b.p, stream));
            else RH_HIP(hipMemsetAsync(bpre_b.p, 0, 32, stream));
            bpre_epoch = base_epoch;
            epoch_questions = 0;
            // pre_b sized like the base buffer, allocated at a base's first question (a large
            // hipMalloc is tens of ms: not inside a later drive), reallocated only when the base
            // buffer was (no extra device-draining hipFree)
            if (row_prefix && nb && pre_b.cap < (nb + 1) * 32 + 64) {
                const size_t need = (std::max<size_t>(nb, base_cap_rows()) + 1) * 32 + 64;
                if ((rc = drain_prefix_build())) return rc;
                pre_b.release();
                size_t free_b = 0, total_b = 0;  // room for it, with 1 GiB to spare, or go without
                if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b >= need + (1ull << 30)) {
                    const std::string keep = g_err;  // a refused allocation is not the caller's error
                    if (pre_b.ensure(need) != RH_OK) g_err = keep;
                }
            }
            if (row_prefix == 1 && pre_b.p && !pstream) {  // its stream too (a queue: milliseconds)
                RH_HIP(back_stream(device, 1, &pstream));
                RH_HIP(hipEventCreateWithFlags(&pre_ev, hipEventDisableTiming));
                RH_HIP(hipEventCreateWithFlags(&pre_base_ev, hipEventDisableTiming));
            }
        }
        // the row prefix once the base has served enough questions to pay for it: ~1.2 ms at 10^8
        // rows against a few us saved a question; a base rewritten every drive never forms it
        // (a loaded base is formed at its first question: loads are rare, compactions are not)
        const uint64_t want_q = base_loaded ? 0 : std::max<uint64_t>(16, nb >> 20);
        if (!row_prefix || !nb || pre_epoch == base_epoch || (row_prefix != 2 && ++epoch_questions <= want_q))
            return RH_OK;
        pre_epoch = base_epoch;  // tried once per base
        if (pre_b.cap < (nb + 1) * 32 + 64 || (row_prefix != 2 && !pstream)) return RH_OK;  // no room for it
        if (row_prefix == 2) {  // in order on the store's stream, used at once (the tests' switch)
            RH_HIP(rh::launch_row_prefix(bfps[cb].p, nb, bpre_b.p, pre_b.p, stream));
            pre_b_ok = true;
            return RH_OK;
        }
        RH_HIP(hipEventRecord(pre_base_ev, stream));  // the base and its block prefix are in place
        RH_HIP(hipStreamWaitEvent(pstream, pre_base_ev, 0));
        RH_HIP(rh::launch_row_prefix(bfps[cb].p, nb, bpre_b.p, pre_b.p, pstream));
        RH_HIP(hipEventRecord(pre_ev, pstream));
        pre_pending = true;
        return RH_OK;
    }
    // the base run as the round and query kernels read it (no segments)
    rh::RoundIn base_in() {
        rh::RoundIn b{nullptr, nullptr, nullptr, nullptr, nullptr, bkeys[cb].p, bfps[cb].p, bsums.p, ssums.p, bpre_b.p};
        if (pre_pending && hipEventQuery(pre_ev) == hipSuccess) {  // the row prefix has landed
            pre_pending = false;
            pre_b_ok = pre_epoch == base_epoch;
        }
        b.pre = pre_b_ok && pre_epoch == base_epoch ? pre_b.p : nullptr;
        return b;
    }
    // the run ranks of m keys (lower bounds among the delta run's keys)
    hipError_t search_run(const uint8_t *keys, size_t m, uint32_t *out) {
        return kops->search_sampled(dkeys[cd].p, nd, dsmp[cd].p, dsmp2[cd].p, keys, m, out, nullptr, stream,
                                    rh::SearchTable{});
    }
    static constexpr uint64_t KEYS_VIEW_MAX = 1ull << 22;  // larger key dumps compact, then copy
    // the keys of ranks [lo, hi) over base + run (hi - lo <= KEYS_VIEW_MAX)
    int keys_view(uint64_t lo, uint64_t hi, void *host_out) {
        int rc;
        rh::RoundRun run;
        rh::RoundIn din;
        if ((rc = view_of(&run, &din)) || (rc = q_keys.ensure((hi - lo) * kl + 64))) return rc;
        RH_HIP(rh::launch_select_view(run, bkeys[cb].p, (uint32_t)kl, nullptr, lo, hi - lo, q_keys.p, stream));
        RH_HIP(hipMemcpyAsync(host_out, q_keys.p, (hi - lo) * kl, hipMemcpyDeviceToHost, stream));
        return sync();
    }
    int query(const uint64_t *lo, const uint64_t *hi, size_t r, rh_aggregate *out) {  // rank ranges
        int rc;
        if (r == 0) return RH_OK;
        if ((rc = q_lo.ensure(r)) || (rc = q_hi.ensure(r)) || (rc = q_out.ensure(r))) return rc;
        RH_HIP(hipMemcpyAsync(q_lo.p, lo, r * 8, hipMemcpyHostToDevice, stream));
        RH_HIP(hipMemcpyAsync(q_hi.p, hi, r * 8, hipMemcpyHostToDevice, stream));
        if (nd) {  // over base + run: select the bounds, sum between their places
            rh::RoundRun run;
            rh::RoundIn din;
            if ((rc = view_of(&run, &din))) return rc;
            RH_HIP(rh::launch_range_query_view(din, run, (uint32_t)kl, size(), q_lo.p, q_hi.p, r,
                                               reinterpret_cast<uint64_t *>(q_out.p), stream));
        } else {
            RH_HIP(rh::launch_range_query(bfps[cb].p, bsums.p, ssums.p, nb, q_lo.p, q_hi.p, r,
                                          reinterpret_cast<uint64_t *>(q_out.p), stream));
        }
        RH_HIP(hipMemcpyAsync(out, q_out.p, r * sizeof(rh_aggregate), hipMemcpyDeviceToHost, stream));
        return sync();
    }
    int aggregate_keys(int lo_kind, const void *lo_key, int hi_kind, const void *hi_key, rh_aggregate *out) {
        int rc;
        if (!lo_kind && !hi_kind) {  // `..`: the cached root
            rh_fp_add(root_b, root_d, out->fingerprint);
            out->size = size();
            return RH_OK;
        }
        if (query_fused) {
            uint8_t k2[64] = {0};
            if (lo_kind) memcpy(k2, lo_key, kl);
            if (hi_kind) memcpy(k2 + kl, hi_key, kl);
            return query_tiny(2, k2, 2 * kl, 1, lo_kind, hi_kind, out, sizeof(rh_aggregate));
        }
        if ((rc = q_keys.ensure(2 * kl + 64)) || (rc = q_lo.ensure(1)) || (rc = q_hi.ensure(1)) ||
            (rc = q_dlo.ensure(1)) || (rc = q_dhi.ensure(1)) || (rc = q_out.ensure(1)) || (rc = q_bout.ensure(1)) ||
            (rc = q_dout.ensure(1)))
            return rc;
        if (lo_kind) RH_HIP(hipMemcpyAsync(q_keys.p, lo_key, kl, hipMemcpyHostToDevice, stream));
        if (hi_kind) RH_HIP(hipMemcpyAsync(q_keys.p + kl, hi_key, kl, hipMemcpyHostToDevice, stream));
        RH_HIP(kops->bounds(bkeys[cb].p, nb, q_keys.p, lo_kind, q_keys.p + kl, hi_kind, q_lo.p, q_hi.p, stream));
        rh_aggregate *res = nd ? q_bout.p : q_out.p;
        RH_HIP(rh::launch_range_query(bfps[cb].p, bsums.p, ssums.p, nb, q_lo.p, q_hi.p, 1,
                                      reinterpret_cast<uint64_t *>(res), stream));
        if (nd) {
            if ((rc = ensure_delta_sums())) return rc;
            RH_HIP(kops->bounds(dkeys[cd].p, nd, q_keys.p, lo_kind, q_keys.p + kl, hi_kind, q_dlo.p, q_dhi.p, stream));
            RH_HIP(rh::launch_range_query(dheap.p, dbsums[cd].p, dssums[cd].p, nd, q_dlo.p, q_dhi.p, 1,
                                          reinterpret_cast<uint64_t *>(q_dout.p), stream, sizeof(rh::DeltaRec),
                                          dslot[cd].p));
            RH_HIP(rh::launch_agg_merge(reinterpret_cast<uint64_t *>(q_bout.p), reinterpret_cast<uint64_t *>(q_dout.p),
                                        q_dlo.p, q_dhi.p, cnt_prefix(cd), reinterpret_cast<uint64_t *>(q_out.p), stream));
        }
        RH_HIP(hipMemcpyAsync(out, q_out.p, sizeof(rh_aggregate), hipMemcpyDeviceToHost, stream));
        return sync();
    }
    // ---- the small questions in one launch (round_tiny.hpp k_query_tiny) ----------------------
    // ranks of up to QUERY_TINY keys, selects of up to QUERY_TINY ranks, one key-range aggregate,
    // over base + delta run as they stand: the input and the answer in mapped page-locked memory,
    // the host polling the sequence word the kernel stores last.  A/B: RSOS_HIP_QUERY_FUSED=0.
    PinnedVec<uint8_t> qt_buf{hipHostMallocCoherent};
    uint64_t qt_seq = 0;
    int query_fused = getenv("RSOS_HIP_QUERY_FUSED") ? atoi(getenv("RSOS_HIP_QUERY_FUSED")) : 1;
    int query_tiny(int mode, const void *in, size_t in_bytes, uint64_t m, int lo_kind, int hi_kind, void *out,
                   size_t out_bytes) {
        int rc;
        rh::RoundRun run{};
        if (nd) {
            rh::RoundIn unused;
            if ((rc = view_of(&run, &unused))) return rc;
        }
        run.nb = nb;
        constexpr size_t o_out = 0, o_seq = 4096;  // output: at most QUERY_TINY 32-byte keys
        try {
            qt_buf.resize(o_seq + 64);
        } catch (const std::bad_alloc &) {
            return fail(RH_ERR_OOM, "query: page-locked allocation failed");
        }
        uint8_t *d;
        if ((rc = dev_ptr(qt_buf, &d))) return rc;
        rh::QueryTiny q{};
        if (in_bytes > sizeof q.in) return fail(RH_ERR_ARG, "query: question larger than the tiny query's");
        memcpy(q.in, in, in_bytes);
        q.mode = mode, q.m = m, q.lo_kind = lo_kind, q.hi_kind = hi_kind;
        if ((rc = ensure_base_prefix())) return rc;
        q.base = base_in();
        q.run = run;
        q.bsmp = bsmp.p, q.bsmp2 = bsmp2.p, q.btab = (!bsmp2.p || nb == 0) ? rh::SearchTable{} : base_table();
        q.dsmp = nd ? dsmp[cd].p : nullptr, q.dsmp2 = nd ? dsmp2[cd].p : nullptr;
        if (fail_point("query.stale_seq")) *reinterpret_cast<uint64_t *>(qt_buf.data() + o_seq) = qt_seq + 1;
        q.out = d + o_out, q.seq_word = reinterpret_cast<uint64_t *>(d + o_seq), q.seq = ++qt_seq;
        disarm(reinterpret_cast<uint64_t *>(qt_buf.data() + o_seq));
        RH_HIP(kops->query_tiny(q, stream));
        if ((rc = wait_word(reinterpret_cast<const uint64_t *>(qt_buf.data() + o_seq), q.seq))) return rc;
        memcpy(out, qt_buf.data() + o_out, out_bytes);
        return RH_OK;
    }
    int ranks(const void *keys, size_t m, uint64_t *out) {
        int rc;
        if (query_fused && m <= rh::QUERY_TINY) return query_tiny(0, keys, m * kl, m, 0, 0, out, m * 8);
        if ((rc = q_keys.ensure(m * kl + 64)) || (rc = q_rank.ensure(m)) || (rc = q_drank.ensure(m)) ||
            (rc = q_merged.ensure(m)))
            return rc;
        RH_HIP(hipMemcpyAsync(q_keys.p, keys, m * kl, hipMemcpyHostToDevice, stream));
        RH_HIP(kops->search_sampled(bkeys[cb].p, nb, bsmp.p, bsmp2.p, q_keys.p, m, q_rank.p, nullptr, stream,
                                    base_table()));
        if (nd) RH_HIP(kops->search(dkeys[cd].p, nd, q_keys.p, m, q_drank.p, nullptr, stream));
        if ((rc = ensure_delta_sums())) return rc;  // the count prefix
        RH_HIP(rh::launch_rank_merge(q_rank.p, nd ? q_drank.p : nullptr, cnt_prefix(cd), m, q_merged.p, stream));
        RH_HIP(hipMemcpyAsync(out, q_merged.p, m * 8, hipMemcpyDeviceToHost, stream));
        return sync();
    }
    // rbsr protocol round, step 1 (protocol.rs:225-255): every segment's local aggregate and
    // raw rank bounds, against the compacted base run (select needs rank order anyway).
    // The two steps move their inputs in one host-to-device copy and their results out in one
    // device-to-host copy, through page-locked staging: a round trip is then 1 + kernels + 1
    // queue operations.
    PinnedVec<uint8_t> stage_in, stage_out, stage_out2;  // step 2's results land beside step 1's
    DevBuf<uint8_t> q_in, q_res;
    static size_t pad8(size_t x) { return (x + 7) & ~size_t(7); }
    static size_t pad16(size_t x) { return (x + 15) & ~size_t(15); }
    // step 1, results in stage_out: lo[r] u64, hi[r] u64, aggregates[r]
    int resolve_staged(size_t r, const uint8_t *sk, const uint8_t *skeys, const uint8_t *ek, const uint8_t *ekeys,
                       const uint64_t **lo, const uint64_t **hi, const rh_aggregate **aggs) {
        int rc;
        const size_t kb = pad8(2 * r * kl), in_bytes = kb + pad8(2 * r), out_bytes = 16 * r + r * sizeof(rh_aggregate);
        if ((rc = q_in.ensure(in_bytes + 64)) || (rc = q_res.ensure(out_bytes + 64)) || (rc = q_rank.ensure(2 * r)) ||
            (nd && (rc = q_drank.ensure(2 * r))))
            return rc;
        stage_in.resize(in_bytes);
        stage_out.resize(out_bytes);
        uint8_t *h = stage_in.data();
        for (size_t j = 0; j < r; j++) {  // row 2j: start key, 2j + 1: end key (unbounded: zeros)
            if (sk[j]) memcpy(h + 2 * j * kl, skeys + j * kl, kl); else memset(h + 2 * j * kl, 0, kl);
            if (ek[j]) memcpy(h + (2 * j + 1) * kl, ekeys + j * kl, kl); else memset(h + (2 * j + 1) * kl, 0, kl);
        }
        memcpy(h + kb, sk, r);
        memcpy(h + kb + r, ek, r);
        RH_HIP(hipMemcpyAsync(q_in.p, h, in_bytes, hipMemcpyHostToDevice, stream));
        uint64_t *d_lo = reinterpret_cast<uint64_t *>(q_res.p), *d_hi = d_lo + r, *d_agg = d_hi + r;
        if (nb)
            RH_HIP(kops->search_sampled(bkeys[cb].p, nb, bsmp.p, bsmp2.p, q_in.p, 2 * r, q_rank.p, nullptr, stream,
                                        base_table()));
        else RH_HIP(hipMemsetAsync(q_rank.p, 0, 2 * r * 4, stream));
        if (nd) {  // ranks in the run as well; view ranks and sums over base + run
            rh::RoundRun run;
            rh::RoundIn din;
            if ((rc = view_of(&run, &din))) return rc;
            RH_HIP(search_run(q_in.p, 2 * r, q_drank.p));
            RH_HIP(rh::launch_resolve_view(q_rank.p, q_drank.p, q_in.p + kb, q_in.p + kb + r, din, run, r, d_lo, d_hi,
                                           d_agg, stream));
        } else {
            RH_HIP(rh::launch_resolve_bounds(q_rank.p, q_in.p + kb, q_in.p + kb + r, r, nb, d_lo, d_hi, stream));
            // an inverted segment (hi < lo) is clamped to the empty range: ZERO
            RH_HIP(rh::launch_range_query(bfps[cb].p, bsums.p, ssums.p, nb, d_lo, d_hi, r, d_agg, stream));
        }
        RH_HIP(hipMemcpyAsync(stage_out.data(), q_res.p, out_bytes, hipMemcpyDeviceToHost, stream));
        if ((rc = sync())) return rc;
        *lo = reinterpret_cast<const uint64_t *>(stage_out.data());
        *hi = *lo + r;
        *aggs = reinterpret_cast<const rh_aggregate *>(*hi + r);
        return RH_OK;
    }
    int resolve(size_t r, const uint8_t *sk, const uint8_t *skeys, const uint8_t *ek, const uint8_t *ekeys,
                uint64_t *raw_lo, uint64_t *raw_hi, rh_aggregate *out) {
        const uint64_t *lo, *hi;
        const rh_aggregate *aggs;
        int rc = resolve_staged(r, sk, skeys, ek, ekeys, &lo, &hi, &aggs);
        if (rc) return rc;
        memcpy(raw_lo, lo, r * 8);
        memcpy(raw_hi, hi, r * 8);
        memcpy(out, aggs, r * sizeof(rh_aggregate));
        return RH_OK;
    }
    // step 2 (protocol.rs:288-313): the select() cuts of every SPLIT and the children's
    // aggregates; results in stage_out: keys[m] (padded to 8 B), aggregates[q]
    int split_staged(size_t m, const uint64_t *sel, size_t q, const uint64_t *lo, const uint64_t *hi,
                     const uint8_t **keys, const rh_aggregate **aggs) {
        int rc;
        const uint64_t nv = size();
        for (size_t i = 0; i < m; i++)
            if (sel[i] >= nv) return fail(RH_ERR_ARG, "select: rank out of range (r >= size)");
        const size_t in_bytes = 8 * (m + 2 * q), kb = pad8(m * kl), out_bytes = kb + q * sizeof(rh_aggregate);
        if ((rc = q_in.ensure(in_bytes + 64)) || (rc = q_res.ensure(out_bytes + 64))) return rc;
        stage_in.resize(in_bytes);
        stage_out2.resize(out_bytes);
        uint64_t *h = reinterpret_cast<uint64_t *>(stage_in.data());
        memcpy(h, sel, m * 8);
        memcpy(h + m, lo, q * 8);
        memcpy(h + m + q, hi, q * 8);
        RH_HIP(hipMemcpyAsync(q_in.p, h, in_bytes, hipMemcpyHostToDevice, stream));
        const uint64_t *d_sel = reinterpret_cast<const uint64_t *>(q_in.p), *d_lo = d_sel + m, *d_hi = d_lo + q;
        if (nd) {  // select and sums over base + run
            rh::RoundRun run;
            rh::RoundIn din;
            if ((rc = view_of(&run, &din))) return rc;
            RH_HIP(rh::launch_select_view(run, bkeys[cb].p, (uint32_t)kl, d_sel, 0, m, q_res.p, stream));
            RH_HIP(rh::launch_range_query_view(din, run, (uint32_t)kl, nv, d_lo, d_hi, q,
                                               reinterpret_cast<uint64_t *>(q_res.p + kb), stream));
        } else {
            if (m) RH_HIP(rh::launch_gather_keys(bkeys[cb].p, (uint32_t)kl, d_sel, m, q_res.p, stream));
            if (q)
                RH_HIP(rh::launch_range_query(bfps[cb].p, bsums.p, ssums.p, nb, d_lo, d_hi, q,
                                              reinterpret_cast<uint64_t *>(q_res.p + kb), stream));
        }
        RH_HIP(hipMemcpyAsync(stage_out2.data(), q_res.p, out_bytes, hipMemcpyDeviceToHost, stream));
        if ((rc = sync())) return rc;
        *keys = stage_out2.data();
        *aggs = reinterpret_cast<const rh_aggregate *>(stage_out2.data() + kb);
        return RH_OK;
    }
    int split(size_t m, const uint64_t *sel, uint8_t *keys_out, size_t q, const uint64_t *lo, const uint64_t *hi,
              rh_aggregate *out) {
        const uint8_t *keys;
        const rh_aggregate *aggs;
        int rc = split_staged(m, sel, q, lo, hi, &keys, &aggs);
        if (rc) return rc;
        if (m) memcpy(keys_out, keys, m * kl);
        if (q) memcpy(out, aggs, q * sizeof(rh_aggregate));
        return RH_OK;
    }
    // A whole protocol round (protocol_round_with_policy, protocol.rs:212-317) for the policies
    // that decide on the span alone, in one device round trip, over the base run and any pending
    // delta run (k_round_*_view: no compaction): the bounds' ranks, local aggregates, decisions,
    // children (cut keys and aggregates) and enumerations are formed on the device, in
    // round_layout().  Tiny rounds read their segments from and write the round into mapped
    // page-locked memory (no copy command); larger ones go up in one copy (a peer's round handed
    // over in place) and are emitted straight into mapped memory sized for the worst case (up to
    // kDirectMax; past it, the header comes down first so the copy is exact).
    DevBuf<uint8_t> r_in, r_kind, r_out;
    DevBuf<uint64_t> r_seg, r_part;
    // A/B switch: RSOS_HIP_ROUND_PLAN3=0 plans a large round with k_round_plan and library scans
    int plan3 = getenv("RSOS_HIP_ROUND_PLAN3") ? atoi(getenv("RSOS_HIP_ROUND_PLAN3")) : 1;
    PinnedVec<uint8_t> pr_out{hipHostMallocCoherent};  // a round's output (polled: round_tiny's sequence word)
    static constexpr size_t kRoundSmall = 256 << 10;  // below this, one speculative copy each way
    static constexpr size_t kDirectMax = 256ull << 20;  // mapped output sized for the worst case up to this
    int round_copyout = getenv("RSOS_HIP_ROUND_COPYOUT") ? atoi(getenv("RSOS_HIP_ROUND_COPYOUT")) : 2;
    int round_copyin = getenv("RSOS_HIP_ROUND_COPYIN") ? atoi(getenv("RSOS_HIP_ROUND_COPYIN")) : 0;
    // A device round in two halves: round_issue queues its copies and launches, round_complete
    // waits for it and points the outputs at it.  Several stores on one device issue their rounds
    // back to back and then wait (rh::store_round_issue, the sharded store), so their host gaps and
    // device work overlap; protocol_round is the two in turn.
    struct RoundPending {
        bool on = false, tiny = false, view = false, zero_copy = false, direct = false;
        uint64_t seq = 0, cap = 0;
        size_t r = 0, worst = 0;
        rh::RoundIn din{};
        rh::RoundRun run{};
        rh::RoundSegs g{};
        uint64_t *place = nullptr;
        double h0 = 0, hv = 0, hs = 0, h1 = 0, h2 = 0, l0 = 0, l1 = 0, c0 = 0;
    } rp;
    int protocol_round(int policy, uint64_t param, const rh_segments &in, rh_segments *ch, rh_segments *en,
                       rh_round_outcome *oc) {
        const int rc = round_issue(policy, param, in, ch, en, oc);
        if (rc || !rp.on) return rc;
        return round_complete(ch, en, oc);
    }
    int round_issue(int policy, uint64_t param, const rh_segments &in, rh_segments *ch, rh_segments *en,
                    rh_round_outcome *oc) {
        int rc;
        const size_t r = in.n;
        const double h0 = round_dbg ? now_us() : 0;
        rp.on = false;
        if (oc) *oc = rh_round_outcome{};
        *ch = rh_segments{};
        *en = rh_segments{};
        if (r == 0) return RH_OK;
        // a pending delta run stays where it is: the round reads base + run through the run's
        // columns (no O(n) compaction on a read)
        const bool view = nd != 0;
        rh::RoundRun run{};
        if (view) {
            rh::RoundIn unused;
            if ((rc = view_of(&run, &unused))) return rc;
        }
        const double hv = round_dbg ? now_us() : 0;
        const uint64_t n = size();                 // live keys of base + run
        const uint64_t b = param < 2 ? 2 : param;  // FanOut::new
        // device input: start kinds, end kinds, start keys then end keys (searched as one run of
        // 2r queries), remote aggregates
        const size_t o_ek = pad16(r), o_sk = o_ek + pad16(r), o_ekeys = o_sk + r * kl,
                     o_rem = pad16(o_ekeys + r * kl), in_bytes = o_rem + r * sizeof(rh_aggregate);
        uint64_t cap = r * std::min<uint64_t>(b, 16);
        if ((rc = r_in.ensure(in_bytes + 64)) || (rc = r_kind.ensure(r)) || (rc = r_seg.ensure(18 * r)) ||
            (rc = q_rank.ensure(2 * r)) || (view && (rc = q_drank.ensure(2 * r))) ||
            (rc = r_out.ensure(rh::round_layout(cap, r, kl).end)))
            return rc;
        const struct { const void *src; size_t off, bytes; } parts[5] = {
            {in.start_kinds, 0, r}, {in.end_kinds, o_ek, r}, {in.start_keys, o_sk, r * kl},
            {in.end_keys, o_ekeys, r * kl}, {in.aggregates, o_rem, r * sizeof(rh_aggregate)}};
        // tiny rounds read their segments from, and write the round into, page-locked host memory
        // (mapped into the device's address space): no copy command either way
        const size_t worst = rh::round_layout(cap, r, kl).end;
        bool zero_copy = r <= rh::round_tiny_max() && in_bytes <= kRoundSmall && worst <= kRoundSmall;
        const uint8_t *in_p = r_in.p;
        uint8_t *out_p = r_out.p;
        if (in_bytes <= kRoundSmall) {
            stage_in.resize(in_bytes);
            for (const auto &p : parts)
                if (p.src) memcpy(stage_in.data() + p.off, p.src, p.bytes);
            if (zero_copy) {
                pr_out.resize(worst);
                uint8_t *di = nullptr, *dout = nullptr;
                // both buffers are allocated mapped; if the runtime still gives no device address,
                // take the copy path below instead (dev_ptr looks each one up once per allocation)
                if (dev_ptr(stage_in, &di) || dev_ptr(pr_out, &dout)) {
                    zero_copy = false;
                } else {
                    in_p = di;
                    out_p = dout;
                }
            }
            if (!zero_copy) {
                RH_HIP(hipMemcpyAsync(r_in.p, stage_in.data(), in_bytes, hipMemcpyHostToDevice, stream));
            }
        } else {
            // the peer store's children, handed over in place (round_layout), already sit in this
            // input layout whenever a row of keys is a whole number of 16-byte units: one copy
            const uint8_t *base = reinterpret_cast<const uint8_t *>(in.start_kinds);
            const bool contiguous = base && in.end_kinds && in.start_keys && in.end_keys && in.aggregates &&
                                    reinterpret_cast<const uint8_t *>(in.end_kinds) == base + o_ek &&
                                    static_cast<const uint8_t *>(in.start_keys) == base + o_sk &&
                                    static_cast<const uint8_t *>(in.end_keys) == base + o_ekeys &&
                                    reinterpret_cast<const uint8_t *>(in.aggregates) == base + o_rem;
            // the peer's round, read in place by a kernel (RSOS_HIP_ROUND_COPYIN=1): 206-219 against
            // the copy engine's 213-214 M segments/s, no gain (profiles/r05_rbsr_copyin_ab.jsonl)
            void *dsrc = nullptr;
            if (contiguous && round_copyin && hipHostGetDevicePointer(&dsrc, const_cast<uint8_t *>(base), 0) == hipSuccess &&
                dsrc) {
                rh::CopyJobs j{};
                j.src[0] = static_cast<const uint8_t *>(dsrc), j.dst[0] = r_in.p, j.bytes[0] = in_bytes, j.n = 1;
                RH_HIP(rh::launch_copy_to_host(j, stream));
            } else if (contiguous) {
                (void)hipGetLastError();
                RH_HIP(hipMemcpyAsync(r_in.p, base, in_bytes, hipMemcpyHostToDevice, stream));
            } else {
                for (const auto &p : parts)  // keys of an all-unbounded side may be NULL (never read)
                    if (p.src) RH_HIP(hipMemcpyAsync(r_in.p + p.off, p.src, p.bytes, hipMemcpyHostToDevice, stream));
            }
        }
        const double hs = round_dbg ? now_us() : 0;
        const uint8_t *d_sk = in_p, *d_ek = in_p + o_ek, *d_skeys = in_p + o_sk, *d_ekeys = in_p + o_ekeys;
        const uint64_t *d_rem = reinterpret_cast<const uint64_t *>(in_p + o_rem);
        uint64_t *lo = r_seg.p, *hi = lo + r, *loc = hi + r, *st = loc + 5 * r, *si = st + r, *ei = si + r,
                 *nch = ei + r, *choff = nch + r, *nen = choff + r, *enoff = nen + r, *place = enoff + r;
        const rh::RoundSegs g{r_kind.p, lo, hi, loc, st, si, ei, nch, choff, nen, enoff};
        if ((rc = ensure_base_prefix())) return rc;
        rh::RoundIn din = base_in();
        din.sk = d_sk, din.ek = d_ek, din.skeys = d_skeys, din.ekeys = d_ekeys, din.remote = d_rem;
        uint64_t *hdr = reinterpret_cast<uint64_t *>(r_out.p);
        const int sq = policy == RH_POLICY_SQRT_FAN_OUT;
        uint64_t h[5];
        if (zero_copy && round_fused && kl <= rh::ROUND_TINY_KL && r <= rh::ROUND_TINY_SEGS) {
            // a tiny round whole in one launch (round_tiny.hpp): the bound keys' searches in both
            // runs, the bounds, decisions and emission, the per-segment arrays in LDS; the host
            // waits for the sequence word the kernel stores last into the mapped output
            rh::RoundTiny t{};
            memcpy(t.isk, stage_in.data(), r);
            memcpy(t.iek, stage_in.data() + o_ek, r);
            memcpy(t.ikeys, stage_in.data() + o_sk, 2 * r * kl);  // start keys then end keys
            memcpy(t.irem, stage_in.data() + o_rem, r * sizeof(rh_aggregate));
            t.in = din;
            t.run = run;
            t.run.nb = nb;
            t.bsmp = bsmp.p, t.bsmp2 = bsmp2.p, t.btab = (!bsmp2.p || nb == 0) ? rh::SearchTable{} : base_table();
            t.dsmp = view ? dsmp[cd].p : nullptr, t.dsmp2 = view ? dsmp2[cd].p : nullptr;
            t.g = g, t.gplace = place, t.r = r, t.n = n, t.sqrt_policy = sq, t.b = b, t.cap = cap, t.out = out_p;
            if (fail_point("round.stale_seq")) reinterpret_cast<uint64_t *>(pr_out.data())[7] = round_seq + 1;
            t.seq = ++round_seq;
            disarm(reinterpret_cast<uint64_t *>(pr_out.data()) + 7);
            if (round_dbg == 1) {  // 2: the host's times only (no copy of the clocks after each round)
                if ((rc = dbg_clk.ensure(8))) return rc;
                t.dbg = dbg_clk.p;
            }
            const double h1 = round_dbg ? now_us() : 0;
            RH_HIP(kops->round_tiny(t, stream));
            const double h2 = round_dbg ? now_us() : 0;
            rp.tiny = true, rp.seq = t.seq, rp.h1 = h1, rp.h2 = h2;
            rp.cap = cap, rp.r = r, rp.view = view, rp.din = din, rp.run = run, rp.g = g, rp.place = place;
            rp.h0 = h0, rp.hv = hv, rp.hs = hs;
            rp.on = true;
            return RH_OK;
        }
        const double l0 = round_dbg ? now_us() : 0;
        if ((rc = round_launch(r, b, n, sq, cap, worst, zero_copy, out_p, view, din, run, g, place, hdr, d_skeys, d_rem)))
            return rc;
        rp.tiny = false, rp.cap = cap, rp.r = r, rp.worst = worst, rp.zero_copy = zero_copy, rp.direct = rq_direct;
        rp.view = view, rp.din = din, rp.run = run, rp.g = g, rp.place = place;
        rp.h0 = h0, rp.hv = hv, rp.hs = hs, rp.l0 = l0, rp.l1 = round_dbg ? now_us() : 0;
        rp.on = true;
        return RH_OK;
    }
    int round_complete(rh_segments *ch, rh_segments *en, rh_round_outcome *oc) {
        int rc;
        rp.on = false;
        uint64_t h[5];
        const size_t r = rp.r;
        const uint64_t cap = rp.cap;
        if (rp.tiny) {
            const double h0 = rp.h0, hv = rp.hv, hs = rp.hs, h1 = rp.h1, h2 = rp.h2;
            if ((rc = wait_word(reinterpret_cast<const uint64_t *>(pr_out.data()) + 7, rp.seq))) return rc;
            const double h3 = round_dbg ? now_us() : 0;
            memcpy(h, pr_out.data(), sizeof h);
            rc = round_finish(h, cap, r, rp.view, rp.din, rp.run, rp.g, rp.place, false, ch, en, oc);
            if (round_dbg) {  // phase times of this round (10 ns ticks), summed until the store is destroyed
                const double h4 = now_us();
                if (round_dbg == 1) {
                    uint64_t c[8];
                    RH_HIP(hipMemcpy(c, dbg_clk.p, sizeof c, hipMemcpyDeviceToHost));
                    for (int k = 0; k < 6; k++) dbg_sum[k] += (double)(c[k + 1] - c[k]) * 0.01;
                }
                dbg_host[0] += h1 - h0, dbg_host[1] += h2 - h1, dbg_host[2] += h3 - h2, dbg_host[3] += h4 - h3;
                dbg_prep[0] += hv - h0, dbg_prep[1] += hs - hv, dbg_prep[2] += h1 - hs;
                if (h0 - dbg_last < 100) dbg_host[4] += h0 - dbg_last, dbg_host_n++;  // the caller's own time
                                                                                        // between rounds of a drive
                dbg_last = now_us();
                dbg_rounds++;
            }
            return rc;
        }
        rp.c0 = round_dbg ? now_us() : 0;
        const double h0 = rp.h0, l0 = rp.l0, l1 = rp.l1;
        const bool zero_copy = rp.zero_copy, direct = rp.direct;
        const size_t worst = rp.worst;
        if ((rc = sync())) return rc;
        memcpy(h, pr_out.data(), sizeof h);
        if (round_dbg == 3) {  // any multi-launch round over 1 ms, phase by phase (us)
            const double l2 = now_us();
            if (l2 - h0 > 1000)
                fprintf(stderr,
                        "{\"slow_round_us\": {\"r\": %zu, \"total\": %.1f, \"view\": %.1f, \"stage\": %.1f, "
                        "\"args\": %.1f, \"launches\": %.1f, \"issue_to_complete\": %.1f, \"wait\": %.1f}}\n",
                        r, l2 - h0, rp.hv - h0, rp.hs - rp.hv, l0 - rp.hs, l1 - l0, rp.c0 - l1, l2 - rp.c0);
        }
        if ((zero_copy || direct) && round_dbg && r > 1024) {  // the large rounds' host times: prep, launches, wait
            const double l2 = now_us();
            dbg_large[0] += l0 - h0, dbg_large[1] += l1 - l0, dbg_large[2] += l2 - l1;
            if (dbg_large_last > 0 && h0 - dbg_large_last < 5000) dbg_large[3] += h0 - dbg_large_last;
            dbg_large_n++;
        }
        rc = round_finish(h, cap, r, rp.view, rp.din, rp.run, rp.g, rp.place, worst > kRoundSmall && !direct, ch, en, oc);
        if (round_dbg) dbg_large_last = now_us();
        return rc;
    }
    bool rq_direct = false;  // round_launch: the round goes straight to mapped memory
    // a round's device work after its input is staged (the multi-launch path), up to the copy of
    // its header (or the whole small round) to the host: queued, not waited for
    int round_launch(size_t r, uint64_t b, uint64_t n, int sq, uint64_t cap, size_t worst, bool zero_copy,
                     uint8_t *out_p, bool view, const rh::RoundIn &din, const rh::RoundRun &run,
                     const rh::RoundSegs &g, uint64_t *place, uint64_t *hdr, const uint8_t *d_skeys,
                     const uint64_t *d_rem) {
        int rc;
        uint64_t *nch = g.nch, *choff = g.choff, *nen = g.nen, *enoff = g.enoff;
        const double l0 = round_dbg ? now_us() : 0;
        if (nb)
            RH_HIP(kops->search_sampled(bkeys[cb].p, nb, bsmp.p, bsmp2.p, d_skeys, 2 * r, q_rank.p, nullptr, stream,
                                        base_table()));
        else RH_HIP(hipMemsetAsync(q_rank.p, 0, 2 * r * 4, stream));
        // a larger round reaches the host through mapped memory sized for the worst case, with one
        // wait and no header round trip first: emitted there directly, the header copied after it
        // by a kernel (RSOS_HIP_ROUND_COPYOUT=2, the default), or emitted into device memory and
        // copied out whole by that kernel (1); 0: a header copy, then the round's bytes.  Writes
        // over PCIe from the emit itself overlap its sums: 2.515-2.551 ms per reconciliation
        // against 2.61-2.62 (1) and 2.64-2.65 (0) (profiles/r04_s18_rbsr_copyout_ab.jsonl)
        bool direct = false;
        uint8_t *dout = nullptr;
        if (!zero_copy && worst > kRoundSmall && worst <= kDirectMax && round_copyout) {
            pr_out.resize(worst);
            direct = !dev_ptr(pr_out, &dout);
        }
        uint8_t *eo = direct && round_copyout == 2 ? dout : r_out.p;  // where emit writes
        // emit reads the header `hd` that the plan wrote and writes the round into `o`
        auto emit = [&](uint64_t c, const uint64_t *hd, uint8_t *o) {
            return view ? rh::launch_round_emit_view(hd, c, r, (uint32_t)kl, din, run, g, place, o, stream)
                        : rh::launch_round_emit(hd, c, r, (uint32_t)kl, din, g, o, stream);
        };
        if (view) RH_HIP(search_run(d_skeys, 2 * r, q_drank.p));  // the bound keys' ranks in the run too
        if (r <= rh::round_tiny_max()) {
            if (view)
                RH_HIP(rh::launch_round_small_view(q_rank.p, q_drank.p, din, run, g, place, r, n, sq, b, cap,
                                                   (uint32_t)kl, out_p, stream));
            else RH_HIP(rh::launch_round_small(q_rank.p, din, g, r, n, sq, b, cap, (uint32_t)kl, out_p, stream));
        } else if (r <= rh::round_small_max()) {
            if (view) RH_HIP(rh::launch_round_bounds_view(q_rank.p, q_drank.p, din, run, g, place, r, stream));
            else RH_HIP(rh::launch_round_bounds(q_rank.p, din, g, r, n, stream));
            RH_HIP(rh::launch_round_plan_scan(din, g, r, n, sq, b, out_p, stream));
            RH_HIP(emit(cap, reinterpret_cast<const uint64_t *>(out_p), zero_copy ? out_p : eo));
        } else {
            if (view) RH_HIP(rh::launch_round_bounds_view(q_rank.p, q_drank.p, din, run, g, place, r, stream));
            else RH_HIP(rh::launch_round_bounds(q_rank.p, din, g, r, n, stream));
            const double lb = round_dbg ? now_us() : 0;
            if (plan3) {  // three launches
                if ((rc = r_part.ensure(5 * ((r + 255) / 256) + 8))) return rc;
                RH_HIP(rh::launch_round_plan3(g, d_rem, r, n, sq, b, r_part.p, hdr, stream));
            } else {
                RH_HIP(hipMemsetAsync(hdr, 0, 64, stream));
                RH_HIP(rh::launch_round_plan(g, d_rem, r, n, sq, b, hdr, stream));
            }
            const double lc = round_dbg ? now_us() : 0;
            if (!plan3) {
                RH_HIP(rh::launch_exclusive_scan_u64(nch, choff, r, scratch, stream));
                RH_HIP(rh::launch_exclusive_scan_u64(nen, enoff, r, scratch, stream));
            }
            const double ld = round_dbg ? now_us() : 0;
            RH_HIP(emit(cap, hdr, eo));
            if (round_dbg) dbg_large_l[0] += lb - l0, dbg_large_l[1] += lc - lb, dbg_large_l[2] += ld - lc, dbg_large_l[3] += now_us() - ld;
        }
        if (direct)  // the round (or, emitted in place, its header alone)
            RH_HIP(rh::launch_round_copy_out(hdr, cap, (uint32_t)kl, r_out.p, dout, round_copyout == 2 ? 64 : worst,
                                             stream));
        rq_direct = direct;
        if (!zero_copy && !direct) {  // the round (small) or its header comes down behind the work
            const size_t bytes = worst <= kRoundSmall ? worst : 64;
            pr_out.resize(bytes);
            RH_HIP(hipMemcpyAsync(pr_out.data(), r_out.p, bytes, hipMemcpyDeviceToHost, stream));
        }
        return RH_OK;
    }
    // the round's header is in h (and pr_out): emit again if its children outnumber cap (a wide
    // fan-out; the per-segment arrays are in g / place), copy the rest down if it is still on the
    // device, and point the outputs at pr_out
    int round_finish(const uint64_t h[5], uint64_t cap, size_t r, bool view, const rh::RoundIn &din,
                     const rh::RoundRun &run, const rh::RoundSegs &g, const uint64_t *place, bool copy_rest,
                     rh_segments *ch, rh_segments *en, rh_round_outcome *oc) {
        int rc;
        const uint64_t nc = h[3], ne = h[1];
        const rh::RoundLayout L = rh::round_layout(nc, ne, kl);
        const bool regrow = nc > cap;
        if (regrow) {  // more children than the first guess (a wide fan-out): emit again
            cap = nc;
            if ((rc = r_out.ensure(L.end))) return rc;  // r_out may have moved: restore its header
            pr_out.resize(L.end);
            uint64_t *hdr = reinterpret_cast<uint64_t *>(r_out.p);
            RH_HIP(hipMemcpyAsync(hdr, pr_out.data(), 64, hipMemcpyHostToDevice, stream));
            RH_HIP(view ? rh::launch_round_emit_view(hdr, cap, r, (uint32_t)kl, din, run, g, place, r_out.p, stream)
                        : rh::launch_round_emit(hdr, cap, r, (uint32_t)kl, din, g, r_out.p, stream));
        }
        if (regrow || copy_rest) {
            pr_out.resize(L.end);
            RH_HIP(hipMemcpyAsync(pr_out.data() + 64, r_out.p + 64, L.end - 64, hipMemcpyDeviceToHost, stream));
            if ((rc = sync())) return rc;
        }
        if (oc) *oc = rh_round_outcome{h[0], h[1], h[2], h[3], h[4]};
        uint8_t *o = pr_out.data();
        *ch = rh_segments{o + L.csk, o + L.cskeys, o + L.cek, o + L.cekeys,
                          reinterpret_cast<rh_aggregate *>(o + L.caggs), (size_t)nc, (size_t)nc};
        *en = rh_segments{o + L.esk, o + L.eskeys, o + L.eek, o + L.eekeys, nullptr, (size_t)ne, (size_t)ne};
        return RH_OK;
    }
    // A/B switch: RSOS_HIP_ROUND_FUSED=0 keeps tiny rounds on the two searches + k_round_small(_view)
    int round_fused = getenv("RSOS_HIP_ROUND_FUSED") ? atoi(getenv("RSOS_HIP_ROUND_FUSED")) : 1;
    uint64_t round_seq = 0;
    // RSOS_HIP_ROUND_DBG=1: k_round_tiny's phase clocks and the host's times per round, averaged to
    // stderr when the store is destroyed; 2: the host's times only (no clock copy per round); 3: as
    // 2, plus a line for every multi-launch round that took over 1 ms
    int round_dbg = getenv("RSOS_HIP_ROUND_DBG") ? atoi(getenv("RSOS_HIP_ROUND_DBG")) : 0;
    DevBuf<uint64_t> dbg_clk;
    double dbg_sum[6] = {0, 0, 0, 0, 0, 0};
    double dbg_host[5] = {0, 0, 0, 0, 0}, dbg_last = 0;  // host: prep, launch, wait, finish, caller
    uint64_t dbg_host_n = 0;
    double dbg_prep[3] = {0, 0, 0};  // prep: the view, the staging, the launch record
    double dbg_large[4] = {0, 0, 0, 0}, dbg_large_last = 0;  // rounds of > 1,024 segments
    double dbg_large_l[4] = {0, 0, 0, 0};  // their launches: searches + bounds, plan, scans, emit
    uint64_t dbg_large_n = 0;
    uint64_t dbg_rounds = 0;
    static double now_us() {
        return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    void release() {
        if (round_dbg == 1 && dbg_rounds)
            fprintf(stderr,
                    "{\"k_round_tiny_phases_us\": {\"rounds\": %llu, \"input\": %.2f, \"searches\": %.2f, "
                    "\"bounds\": %.2f, \"decide\": %.2f, \"emit\": %.2f, \"fence\": %.2f}}\n",
                    (unsigned long long)dbg_rounds, dbg_sum[0] / dbg_rounds, dbg_sum[1] / dbg_rounds,
                    dbg_sum[2] / dbg_rounds, dbg_sum[3] / dbg_rounds, dbg_sum[4] / dbg_rounds, dbg_sum[5] / dbg_rounds);
        if (round_dbg && dbg_large_n)
            fprintf(stderr,
                    "{\"large_round_host_us\": {\"rounds\": %llu, \"prep\": %.2f, \"launches\": %.2f, \"wait\": %.2f, "
                    "\"caller_between_rounds\": %.2f, \"searches_bounds\": %.2f, \"plan\": %.2f, \"scans\": %.2f, "
                    "\"emit\": %.2f}}\n",
                    (unsigned long long)dbg_large_n, dbg_large[0] / dbg_large_n, dbg_large[1] / dbg_large_n,
                    dbg_large[2] / dbg_large_n, dbg_large[3] / dbg_large_n, dbg_large_l[0] / dbg_large_n,
                    dbg_large_l[1] / dbg_large_n, dbg_large_l[2] / dbg_large_n, dbg_large_l[3] / dbg_large_n);
        if (round_dbg && dbg_rounds > 1)
            fprintf(stderr,
                    "{\"round_host_us\": {\"prep\": %.2f, \"launch\": %.2f, \"wait\": %.2f, \"finish\": %.2f, "
                    "\"caller_between_rounds\": %.2f, \"prep_view\": %.2f, \"prep_stage\": %.2f, \"prep_args\": %.2f}}\n",
                    dbg_host[0] / dbg_rounds, dbg_host[1] / dbg_rounds, dbg_host[2] / dbg_rounds, dbg_host[3] / dbg_rounds,
                    dbg_host_n ? dbg_host[4] / dbg_host_n : 0.0, dbg_prep[0] / dbg_rounds, dbg_prep[1] / dbg_rounds,
                    dbg_prep[2] / dbg_rounds);
        (void)hipStreamSynchronize(stream);
        if (cstream) (void)hipStreamSynchronize(cstream);
        if (kstream) (void)hipStreamSynchronize(kstream);
        for (int k = 0; k < 2; k++) {
            bkeys[k].release(); bfps[k].release(); dkeys[k].release(); dslot[k].release();
        }
        bsums.release(); ssums.release(); tot.release(); bsmp.release(); bsmp2.release(); btab.release(); btabp.release(); dtab.release(); dtabp.release(); dsmp[0].release(); dsmp[1].release(); dsmp2[0].release(); dsmp2[1].release(); dscnt.release(); fin_ticket.release(); mcnt.release();
        for (int k = 0; k < 2; k++) {
            dbsums[k].release(); dssums[k].release(); dblk[k].release(); dinb[k].release(); dsblk[k].release();
        }
        staging.release();
        skeys.release(); sfps.release(); sops.release(); hops.release(); dheap.release(); heap_len = 0;
        dops.release(); cfps.release(); cops.release(); counts.release(); flag.release();
        results.release();
        q_lo.release(); q_hi.release(); q_dlo.release(); q_dhi.release(); q_merged.release();
        q_out.release(); q_bout.release(); q_dout.release(); q_keys.release(); q_rank.release(); q_drank.release();
        q_in.release(); q_res.release();
        stage_in.release(); stage_out.release(); stage_out2.release(); load_flag.release();
        r_in.release(); r_kind.release(); r_out.release(); r_seg.release(); r_part.release(); pr_out.release();
        trs[0].release(); trs[1].release(); trun_keys.release();
        tsets[0].release(); tsets[1].release(); tier_dpre.release(); tier_spre.release(); tier_bpre.release(); tier_dsmp.release();
        if (cstream) (void)hipStreamDestroy(cstream);
        back_stream_put(device, 0, kstream);
        if (rf_ready) (void)hipEventDestroy(rf_ready);
        if (rf_ev) (void)hipEventDestroy(rf_ev);
        if (rf_kdone) (void)hipEventDestroy(rf_kdone);
        cstream = kstream = nullptr, rf_ready = rf_ev = rf_kdone = nullptr, rf_on = false;
        snap.release();
        if (pstream) {
            (void)hipStreamSynchronize(pstream);
            back_stream_put(device, 1, pstream);
            (void)hipEventDestroy(pre_ev);
            (void)hipEventDestroy(pre_base_ev);
            pstream = nullptr, pre_ev = pre_base_ev = nullptr;
        }
        pre_pending = pre_b_ok = false;
        bpre_b.release(); spre_b.release(); pre_b.release(); dbg_clk.release();
        sbsums.release(); sssums.release(); sbsmp.release(); sbsmp2.release(); sbtab.release(); sbtabp.release();
        stot.release(); snap_words.release(); snap_hdr.release();
        scratch.release();
        if (dep) (void)hipEventDestroy(dep);
        if (hdr_ev) (void)hipEventDestroy(hdr_ev);
        dep = nullptr;
        if (res_ev) (void)hipEventDestroy(res_ev);
        res_ev = nullptr;
        if (small_ev) (void)hipEventDestroy(small_ev);
        small_ev = nullptr;
        for (auto &e : ls_ev)
            if (e) (void)hipEventDestroy(e), e = nullptr;
    }
};

// Every call that reads or replaces the store first takes its lock; readers then flush the pending
// batch (rh_store_stage) so that they see every staged record
#define RH_LOCK_NOFLUSH(s)                          \
    std::lock_guard<std::mutex> guard_((s)->mu);    \
    RH_HIP(hipSetDevice((s)->device))
#define RH_LOCK(s)                                  \
    RH_LOCK_NOFLUSH(s);                             \
    do {                                            \
        const int frc_ = (s)->flush();              \
        if (frc_) return frc_;                      \
    } while (0)

static int flush_locked(rh_store *s) {
    if (int rc = s->health()) return rc;
    if (!s->pend.n) return RH_OK;
    RH_HIP(hipSetDevice(s->device));
    return s->flush();
}

static int round_entry(rh_store *s, int policy, uint64_t fan_out, const rh_segments *active, rh_segments *children,
                       rh_segments *enumerations, rh_round_outcome *outcome, bool *pending);

// Under the store's lock: 1 if the host tier answers (refreshing it first if the store changed
// since; only then is the device touched), 0 if the tier is off, < 0 on error
static int tier_ready(rh_store *s) {
    const int frc = flush_locked(s);
    if (frc) return frc;
    if (!s->tier_on) return 0;
    if (s->tier_fresh()) return 1;  // the common case: no device call at all
    RH_HIP(hipSetDevice(s->device));
    int rc;
    // a stale tier takes a landed copy now (a fresh one takes it at the next write: no log replay
    // on a question)
    if (s->rf_on && !s->tier_fresh() && (rc = s->poll_refresh(false))) return rc;
    if (s->tier_fresh()) return 1;
    // stale: the device answers; a refresh is under way (or starts here when that is cheap)
    // (a run copy costs no compaction: always, unless copies keep being discarded; a base copy
    // when question_may_refresh says so)
    if (!s->rf_on && (s->run_refresh_next() || s->question_may_refresh()) && (rc = s->refresh_now())) return rc;
    return 0;
}

extern "C" {

int rh_store_create(int device, const rh_schema *schema, rh_store **out) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if (!out) return fail(RH_ERR_ARG, "out is NULL");
    if (rh_schema_supported(schema) != 1)
        return fail(RH_ERR_UNSUPPORTED, "store needs a schema with a specialised lift kernel");
    rh::StoreKeyOps *kops = rh::store_key_ops(schema->key_kind, key_row(*schema));
    if (!kops) return fail(RH_ERR_UNSUPPORTED, "store keys must be u32, u64 or 8/16/32-byte arrays");
    RH_HIP(hipSetDevice(device));
    rh_store *s = new rh_store();
    s->device = device;
    s->schema = *schema;
    s->kops = kops;
    s->kl = key_row(*schema);
    hipError_t e = create_fore_stream(&s->stream);
    if (e != hipSuccess) {
        delete s;
        return fail(RH_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    s->scratch.stream = s->stream;
    *out = s;
    return RH_OK;
}

int rh_store_destroy(rh_store *s) {
    if (!s) return RH_OK;
    (void)hipSetDevice(s->device);
    s->release();
    (void)hipStreamDestroy(s->stream);
    delete s;
    return RH_OK;
}

int rh_store_load(rh_store *s, const rh_columns *h, size_t n) {
    // the row cap first: it is a property of the arguments (include/rsos_hip.h, "Row cap")
    if (n >= (1ull << 31)) return fail(RH_ERR_ARG, "store size limit (2^31 rows) exceeded: use rh_sstore_* for a larger map");
    if (!s || !h) return fail(RH_ERR_ARG, "NULL");
    RH_LOCK_NOFLUSH(s);
    s->pend.clear();  // a load replaces the contents: staged rows before it are superseded
    int rc;
    if ((rc = s->staging.upload(s->schema, *h, n, s->stream))) return rc;
    return s->load_device(s->staging.view(s->schema), n);
}

int rh_store_load_device(rh_store *s, const rh_columns *dev_cols, size_t n, void *after_stream) {
    if (n >= (1ull << 31)) return fail(RH_ERR_ARG, "store size limit (2^31 rows) exceeded: use rh_sstore_* for a larger map");
    if (!s) return fail(RH_ERR_ARG, "NULL");
    int rc = check_cols(s->schema, dev_cols, n);
    if (rc) return rc;
    RH_LOCK_NOFLUSH(s);
    s->pend.clear();
    if ((rc = s->after(after_stream))) return rc;
    return s->load_device(*dev_cols, n);
}

int rh_store_len(rh_store *s, uint64_t *out) {
    if (!s || !out) return fail(RH_ERR_ARG, "NULL");
    std::lock_guard<std::mutex> g(s->mu);
    const int rc = flush_locked(s);
    if (rc) return rc;
    *out = s->size();
    return RH_OK;
}

int rh_store_aggregates(rh_store *s, const uint64_t *lo, const uint64_t *hi, size_t r, rh_aggregate *out) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    if (r && (!lo || !hi || !out)) return fail(RH_ERR_ARG, "NULL buffer");
    {
        std::lock_guard<std::mutex> g(s->mu);
        const int t = tier_ready(s);
        if (t < 0) return t;
        if (t) {
            for (size_t j = 0; j < r; j++) s->tier.agg(lo[j], hi[j], out + j);
            return RH_OK;
        }
    }
    RH_LOCK(s);
    return s->query(lo, hi, r, out);
}

int rh_store_aggregate(rh_store *s, uint64_t lo, uint64_t hi, rh_aggregate *out) {
    return rh_store_aggregates(s, &lo, &hi, 1, out);
}

int rh_store_ranks(rh_store *s, const void *keys, size_t m, uint64_t *out) {
    if (!s || (m && (!keys || !out))) return fail(RH_ERR_ARG, "NULL");
    if (m == 0) return RH_OK;
    {
        std::lock_guard<std::mutex> g(s->mu);
        const int t = tier_ready(s);
        if (t < 0) return t;
        if (t) {
            const uint8_t *k = static_cast<const uint8_t *>(keys);
            for (size_t j = 0; j < m; j++) out[j] = s->tier.rank(k + j * s->kl);
            return RH_OK;
        }
    }
    RH_LOCK(s);
    return s->ranks(keys, m, out);
}

int rh_store_rank(rh_store *s, const void *key, uint64_t *out) { return rh_store_ranks(s, key, 1, out); }

int rh_store_keys(rh_store *s, uint64_t lo, uint64_t hi, void *host_out) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    std::lock_guard<std::mutex> guard_(s->mu);
    int rc;
    // the staged rows first: the range is checked against the size they leave
    if ((rc = flush_locked(s))) return rc;
    if (lo > hi || hi > s->size()) return fail(RH_ERR_ARG, "bad rank range");
    if (hi == lo) return RH_OK;
    if (!host_out) return fail(RH_ERR_ARG, "host_out NULL");
    if ((rc = tier_ready(s)) < 0) return rc;
    if (rc) {
        s->tier.copy_keys(lo, hi, static_cast<uint8_t *>(host_out));
        return RH_OK;
    }
    RH_HIP(hipSetDevice(s->device));
    if (s->query_fused && hi - lo <= rh::QUERY_TINY) {  // select and short dumps: one launch
        uint64_t rk[rh::QUERY_TINY];
        for (uint64_t i = lo; i < hi; i++) rk[i - lo] = i;
        return s->query_tiny(1, rk, (hi - lo) * 8, hi - lo, 0, 0, host_out, (hi - lo) * s->kl);
    }
    if (s->nd && hi - lo <= rh_store::KEYS_VIEW_MAX) return s->keys_view(lo, hi, host_out);
    if ((rc = s->compact())) return rc;
    RH_HIP(hipMemcpyAsync(host_out, s->bkeys[s->cb].p + lo * s->kl, (hi - lo) * s->kl, hipMemcpyDeviceToHost,
                          s->stream));
    return s->sync();
}

int rh_store_select(rh_store *s, uint64_t r, void *key_out) {
    if (!s || !key_out) return fail(RH_ERR_ARG, "NULL");
    if (r == UINT64_MAX) return fail(RH_ERR_ARG, "select: rank out of range (r >= size)");
    const int rc = rh_store_keys(s, r, r + 1, key_out);
    if (rc == RH_ERR_ARG) return fail(RH_ERR_ARG, "select: rank out of range (r >= size)");
    return rc;
}

int rh_store_aggregate_keys(rh_store *s, int lo_kind, const void *lo_key, int hi_kind, const void *hi_key,
                            rh_aggregate *out) {
    if (!s || !out) return fail(RH_ERR_ARG, "NULL");
    if (lo_kind < 0 || lo_kind > 2 || hi_kind < 0 || hi_kind > 2) return fail(RH_ERR_ARG, "bad bound kind");
    if ((lo_kind && !lo_key) || (hi_kind && !hi_key)) return fail(RH_ERR_ARG, "bound key is NULL");
    {
        std::lock_guard<std::mutex> g(s->mu);
        const int t = tier_ready(s);
        if (t < 0) return t;
        if (t) {
            const rh::HostTier &t = s->tier;
            t.agg(t.bound(lo_kind, static_cast<const uint8_t *>(lo_key), true),
                  t.bound(hi_kind, static_cast<const uint8_t *>(hi_key), false), out);  // inverted -> ZERO
            return RH_OK;
        }
    }
    RH_LOCK(s);
    return s->aggregate_keys(lo_kind, lo_key, hi_kind, hi_key, out);
}

int rh_store_resolve_segments(rh_store *s, size_t r, const uint8_t *start_kinds, const void *start_keys,
                              const uint8_t *end_kinds, const void *end_keys, uint64_t *raw_start,
                              uint64_t *raw_end, rh_aggregate *local) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    if (r == 0) return RH_OK;
    if (!start_kinds || !end_kinds || !raw_start || !raw_end || !local) return fail(RH_ERR_ARG, "NULL buffer");
    for (size_t j = 0; j < r; j++) {
        if (start_kinds[j] > 1 || end_kinds[j] > 1)
            return fail(RH_ERR_ARG, "segment bound kind must be 0 (Unbounded) or 1 (Included / Excluded)");
        if ((start_kinds[j] && !start_keys) || (end_kinds[j] && !end_keys)) return fail(RH_ERR_ARG, "bound key is NULL");
    }
    if (s->tier_on && r <= s->tier_round_max) {
        std::lock_guard<std::mutex> g(s->mu);
        const int t = tier_ready(s);
        if (t < 0) return t;
        if (t) {
            const uint8_t *sk = static_cast<const uint8_t *>(start_keys), *ek = static_cast<const uint8_t *>(end_keys);
            const rh::HostTier &t = s->tier;
            for (size_t j = 0; j < r; j++) {
                const rh::HostTier::Cur a = start_kinds[j] ? t.lt(sk + j * s->kl) : t.begin();
                const rh::HostTier::Cur b = end_kinds[j] ? t.lt(ek + j * s->kl) : t.end();
                raw_start[j] = a.r;
                raw_end[j] = b.r;
                t.agg(a, b, local + j);  // inverted -> ZERO
            }
            return RH_OK;
        }
    }
    RH_LOCK(s);
    try {
        return s->resolve(r, start_kinds, static_cast<const uint8_t *>(start_keys), end_kinds,
                          static_cast<const uint8_t *>(end_keys), raw_start, raw_end, local);
    } catch (const std::bad_alloc &) {
        return fail(RH_ERR_OOM, "resolve: host allocation failed");
    }
}

int rh_store_split_segments(rh_store *s, size_t m, const uint64_t *select_ranks, void *keys_out, size_t q,
                            const uint64_t *lo, const uint64_t *hi, rh_aggregate *out) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    if ((m && (!select_ranks || !keys_out)) || (q && (!lo || !hi || !out))) return fail(RH_ERR_ARG, "NULL buffer");
    if (m == 0 && q == 0) return RH_OK;
    if (s->tier_on && m + q <= 16 * s->tier_round_max) {
        std::lock_guard<std::mutex> g(s->mu);
        const int t = tier_ready(s);
        if (t < 0) return t;
        if (t) {
            for (size_t i = 0; i < m; i++)
                if (select_ranks[i] >= s->tier.n) return fail(RH_ERR_ARG, "select: rank out of range (r >= size)");
            for (size_t i = 0; i < m; i++)
                memcpy(static_cast<uint8_t *>(keys_out) + i * s->kl, s->tier.at(select_ranks[i]).k, s->kl);
            for (size_t i = 0; i < q; i++) s->tier.agg(lo[i], hi[i], out + i);
            return RH_OK;
        }
    }
    RH_LOCK(s);
    try {  // no exception crosses the C ABI
        return s->split(m, select_ranks, static_cast<uint8_t *>(keys_out), q, lo, hi, out);
    } catch (const std::bad_alloc &) {
        return fail(RH_ERR_OOM, "split: host allocation failed");
    }
}

int rh_store_protocol_round(rh_store *s, int policy, uint64_t fan_out, const rh_segments *active,
                            rh_segments *children, rh_segments *enumerations, rh_round_outcome *outcome) {
    return round_entry(s, policy, fan_out, active, children, enumerations, outcome, nullptr);
}

}  // extern "C"

// rh_store_protocol_round; with `pending` non-NULL a device round is only issued: *pending = true,
// the store stays locked, and rh::store_round_complete finishes it (on the same thread)
static int round_entry(rh_store *s, int policy, uint64_t fan_out, const rh_segments *active, rh_segments *children,
                       rh_segments *enumerations, rh_round_outcome *outcome, bool *pending) {
    if (pending) *pending = false;
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
    if (s->tier_on && r <= s->tier_round_max) {  // small rounds on the host tier
        std::lock_guard<std::mutex> g(s->mu);
        try {
            const int t = tier_ready(s);
            if (t < 0) return t;
            if (t) {
                uint64_t h[5];
                s->tier.round(policy == RH_POLICY_SQRT_FAN_OUT, fan_out < 2 ? 2 : fan_out, *active, s->tier_out, h);
                const uint64_t nc = h[3], ne = h[1];
                const rh::RoundLayout L = rh::round_layout(nc, ne, s->kl);
                uint8_t *o = s->tier_out.data();
                if (outcome) *outcome = rh_round_outcome{h[0], h[1], h[2], h[3], h[4]};
                *children = rh_segments{o + L.csk, o + L.cskeys, o + L.cek, o + L.cekeys,
                                        reinterpret_cast<rh_aggregate *>(o + L.caggs), (size_t)nc, (size_t)nc};
                *enumerations = rh_segments{o + L.esk, o + L.eskeys, o + L.eek, o + L.eekeys, nullptr, (size_t)ne,
                                            (size_t)ne};
                return RH_OK;
            }
        } catch (const std::bad_alloc &) {
            *children = rh_segments{};
            *enumerations = rh_segments{};
            return fail(RH_ERR_OOM, "protocol round: host allocation failed");
        }
    }
    if (pending) {
        std::unique_lock<std::mutex> g(s->mu);
        RH_HIP(hipSetDevice(s->device));
        int rc = s->flush();
        if (rc) return rc;
        try {
            rc = s->round_issue(policy, fan_out, *active, children, enumerations, outcome);
        } catch (const std::bad_alloc &) {
            s->rp.on = false;
            *children = rh_segments{};
            *enumerations = rh_segments{};
            return fail(RH_ERR_OOM, "protocol round: host allocation failed");
        }
        if (rc || !s->rp.on) return rc;
        g.release();  // held until rh::store_round_complete
        *pending = true;
        return RH_OK;
    }
    RH_LOCK(s);
    try {  // no exception crosses the C ABI
        return s->protocol_round(policy, fan_out, *active, children, enumerations, outcome);
    } catch (const std::bad_alloc &) {
        *children = rh_segments{};
        *enumerations = rh_segments{};
        return fail(RH_ERR_OOM, "protocol round: host allocation failed");
    }
}

namespace rh {
int store_round_issue(rh_store *s, int policy, uint64_t fan_out, const rh_segments *active, rh_segments *children,
                      rh_segments *enumerations, rh_round_outcome *outcome, bool *pending) {
    return round_entry(s, policy, fan_out, active, children, enumerations, outcome, pending);
}
int store_round_complete(rh_store *s, rh_segments *children, rh_segments *enumerations, rh_round_outcome *outcome) {
    std::unique_lock<std::mutex> g(s->mu, std::adopt_lock);  // taken by store_round_issue
    try {
        const int rc = s->round_complete(children, enumerations, outcome);
        if (rc) *children = rh_segments{}, *enumerations = rh_segments{};
        return rc;
    } catch (const std::bad_alloc &) {
        *children = rh_segments{};
        *enumerations = rh_segments{};
        return fail(RH_ERR_OOM, "protocol round: host allocation failed");
    }
}
}  // namespace rh

extern "C" {

int rh_store_fingerprints(rh_store *s, uint64_t lo, uint64_t hi, uint8_t *host_out) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    RH_LOCK(s);
    int rc;
    if (lo > hi || hi > s->size()) return fail(RH_ERR_ARG, "bad rank range");
    if (hi > lo && !host_out) return fail(RH_ERR_ARG, "host_out NULL");
    if ((rc = s->compact())) return rc;
    if (hi > lo)
        RH_HIP(hipMemcpyAsync(host_out, s->bfps[s->cb].p + lo * 32, (hi - lo) * 32, hipMemcpyDeviceToHost, s->stream));
    return s->sync();
}

int rh_store_compact(rh_store *s) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    RH_LOCK(s);
    return s->compact();
}

int rh_store_stats(rh_store *s, uint64_t *base_rows, uint64_t *delta_rows, uint64_t *compactions) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    std::lock_guard<std::mutex> g(s->mu);
    const int rc = flush_locked(s);
    if (rc) return rc;
    if (base_rows) *base_rows = s->nb;
    if (delta_rows) *delta_rows = s->nd;
    if (compactions) *compactions = s->compactions;
    return RH_OK;
}

int rh_store_batch_stats(rh_store *s, uint64_t *small_batches, uint64_t *large_batches) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    std::lock_guard<std::mutex> g(s->mu);
    const int rc = flush_locked(s);
    if (rc) return rc;
    if (small_batches) *small_batches = s->small_batches;
    if (large_batches) *large_batches = s->large_batches;
    return RH_OK;
}

int rh_store_tier_stats(rh_store *s, uint64_t *base_rows, uint64_t *delta_entries, uint64_t *refreshes,
                        uint64_t *folds) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    std::lock_guard<std::mutex> g(s->mu);
    const int rc = flush_locked(s);
    if (rc) return rc;
    const bool fresh = s->tier_fresh();
    if (base_rows) *base_rows = fresh ? s->tier.nb : 0;
    if (delta_entries) *delta_entries = fresh ? s->tier.dt.size() + s->tier.run.n : 0;
    if (refreshes) *refreshes = s->tier_refreshes;
    if (folds) *folds = s->tier_folds;
    return RH_OK;
}

int rh_store_tier_sync(rh_store *s) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    std::lock_guard<std::mutex> g(s->mu);
    int rc;
    if ((rc = flush_locked(s))) return rc;
    if (!s->tier_on) return RH_OK;
    RH_HIP(hipSetDevice(s->device));
    if (!s->tier_fresh() && !s->rf_on && (rc = s->refresh_now())) return rc;
    if ((rc = s->settle())) return rc;
    if (!s->tier_fresh() && (rc = s->refresh_now()) == RH_OK) rc = s->settle();
    return rc;
}

int rh_store_set_tier_policy(rh_store *s, int keep_fresh) {
    if (!s || keep_fresh < 0 || keep_fresh > 1) return fail(RH_ERR_ARG, "bad tier policy");
    std::lock_guard<std::mutex> g(s->mu);
    RH_HIP(hipSetDevice(s->device));
    int rc;
    if ((rc = s->settle())) return rc;
    s->tier_sync_writes = keep_fresh == 1;
    return RH_OK;
}

int rh_store_reserve(rh_store *s, uint64_t rows, uint64_t batch_rows) {
    if (rows >= (1ull << 31) || batch_rows >= (1ull << 31))
        return fail(RH_ERR_ARG, "store size limit (2^31 rows) exceeded: use rh_sstore_* for a larger map");
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    RH_LOCK(s);
    return s->reserve(rows, batch_rows);
}

int rh_store_stage(rh_store *s, const rh_columns *h, const uint8_t *ops, size_t m) {
    if (!s || !h || (m && !ops)) return fail(RH_ERR_ARG, "NULL");
    if (m == 0) return RH_OK;
    const rh_schema &sc = s->schema;
    if (sc.key_kind != RH_KEY_UNIT && !h->keys) return fail(RH_ERR_ARG, "keys column is NULL");
    for (size_t i = 0; i < m; i++)
        if (ops[i] > 1) return fail(RH_ERR_ARG, "op must be 0 (insert) or 1 (delete)");
    std::lock_guard<std::mutex> g(s->mu);
    if (s->pend.n + m >= (1ull << 31)) return fail(RH_ERR_ARG, "pending batch limit (2^31 rows) exceeded");
    try {
        return s->stage(*h, ops, m);
    } catch (const std::bad_alloc &) {
        return fail(RH_ERR_OOM, "stage: host allocation failed");
    }
}

int rh_store_set_host_tier(rh_store *s, int enable, uint64_t round_max) {
    if (!s || enable < 0 || enable > 1) return fail(RH_ERR_ARG, "bad host tier setting");
    std::lock_guard<std::mutex> g(s->mu);
    RH_HIP(hipSetDevice(s->device));
    int rc;
    if ((rc = s->settle())) return rc;
    const bool was_on = s->tier_on;
    s->tier_on = enable == 1;
    s->tier_round_max = round_max ? round_max : 128;
    if (s->tier_on) {
        if ((rc = s->tier_reserve(s->nb + s->nd + (s->nb + s->nd) / 4))) return rc;
        if (!was_on) {  // the first copy, in the background (an empty store's: at its load or first question)
            s->tier_version = ~0ull;
            if ((rc = flush_locked(s))) return rc;
            if (s->nb + s->nd > 0 && (rc = s->start_refresh())) return rc;
            // with writes keeping the tier fresh, enabling it waits for its first copy too: no
            // question after this call is answered by the device
            if (s->tier_sync_writes && (rc = s->settle())) return rc;
        }
    }
    if (!s->tier_on) {  // give the host memory back
        s->tier_version = ~0ull;
        s->tier.reset();
        s->tier_epoch = ~0ull;  // no base copy held
        s->tsets[0].release(), s->tsets[1].release();
        s->trh[0].release(), s->trh[1].release();
        s->tier_out = std::vector<uint8_t>();
        s->tier_dpre.release(), s->tier_spre.release(), s->tier_bpre.release(), s->tier_dsmp.release();
    }
    return RH_OK;
}

int rh_store_set_compaction(rh_store *s, uint64_t divisor, uint64_t min_rows) {
    if (!s || divisor == 0) return fail(RH_ERR_ARG, "bad compaction policy");
    s->compact_div = divisor;
    s->compact_min = min_rows;
    return RH_OK;
}

int rh_store_apply(rh_store *s, const rh_columns *h, const uint8_t *ops, size_t m, uint64_t *n_new,
                   uint64_t *n_over, uint64_t *n_del) {
    if (!s || !h || (m && !ops)) return fail(RH_ERR_ARG, "NULL");
    RH_LOCK(s);
    int rc;
    uint64_t c[3];
    if ((rc = s->apply_host(*h, ops, m, c))) return rc;
    if (n_new) *n_new = c[0];
    if (n_over) *n_over = c[1];
    if (n_del) *n_del = c[2];
    return RH_OK;
}

int rh_store_apply_device(rh_store *s, const rh_columns *dev_cols, const uint8_t *dev_ops, size_t m,
                          uint64_t *n_new, uint64_t *n_over, uint64_t *n_del, void *after_stream) {
    if (!s) return fail(RH_ERR_ARG, "NULL");
    int rc = check_cols(s->schema, dev_cols, m);
    if (rc) return rc;
    RH_LOCK(s);
    if ((rc = s->after(after_stream))) return rc;
    uint64_t c[3];
    if ((rc = s->apply_device(*dev_cols, dev_ops, m, c))) return rc;
    if (n_new) *n_new = c[0];
    if (n_over) *n_over = c[1];
    if (n_del) *n_del = c[2];
    return RH_OK;
}

int rh_store_apply_device_many(rh_store *s, const rh_columns *dev_cols, const uint8_t *const *dev_ops,
                               const size_t *n, size_t k, uint64_t *counts, void *after_stream) {
    if (!s || (k && (!dev_cols || !n))) return fail(RH_ERR_ARG, "NULL");
    int rc;
    for (size_t i = 0; i < k; i++)
        if ((rc = check_cols(s->schema, &dev_cols[i], n[i]))) return rc;
    RH_LOCK(s);
    if ((rc = s->after(after_stream))) return rc;
    std::vector<uint64_t> c(3 * k + 3);
    rc = s->apply_device_many(dev_cols, dev_ops, n, k, c.data());
    if (counts) memcpy(counts, c.data(), 3 * k * sizeof(uint64_t));
    return rc;
}

}  // extern "C"

// =================================================================================================
// Snapshot reload (src/snapshot.rs:30-58; reload = just_insert_bulk, src/replicated_map/persistence.rs:143)
namespace {

int snapshot_header(const uint8_t *h, size_t len, uint64_t *n) {
    // the checks and messages of decode_snapshot, src/snapshot.rs:60-98
    if (len < 8)
        return fail(RH_ERR_DATA, "snapshot is " + std::to_string(len) +
                                     " bytes, shorter than the 8-byte format header (truncated, or a "
                                     "pre-Entry/State snapshot without the versioned header)");
    if (memcmp(h, "RCNL", 4) != 0) {
        char m[64];
        snprintf(m, sizeof m, "[%02x, %02x, %02x, %02x]", h[0], h[1], h[2], h[3]);
        return fail(RH_ERR_DATA, std::string("snapshot magic ") + m +
                                     " does not match [52, 43, 4e, 4c]; the file is not a reconcile snapshot, "
                                     "or predates the versioned format");
    }
    uint32_t version;
    memcpy(&version, h + 4, 4);
    if (version != 1)
        return fail(RH_ERR_DATA, "snapshot format version " + std::to_string(version) +
                                     " is not supported by this build (expected 1); it was written by a "
                                     "different reconcile version and must be migrated or discarded");
    if (len < 16) return fail(RH_ERR_DATA, "snapshot body is truncated (io error: unexpected end of file)");
    memcpy(n, h + 8, 8);
    return RH_OK;
}

uint32_t gcd32(uint32_t a, uint32_t b) {
    while (b) {
        const uint32_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}

// the entry layout of a file of len bytes (what the walk needs); snapshot_format adds the checks
// against the header's entry count
int snapshot_layout(const rh_schema &s, int key_form, size_t len, rh::SnapFmt *f) {
    if (key_form != RH_FORM_ARRAY && key_form != RH_FORM_VEC) return fail(RH_ERR_ARG, "bad key_form");
    if (key_form == RH_FORM_VEC && s.key_kind != RH_KEY_BYTES) return fail(RH_ERR_ARG, "RH_FORM_VEC needs byte keys");
    f->key_pre = key_form == RH_FORM_VEC ? 8 : 0;
    f->key_len = key_row(s);
    f->val_pre = s.value_kind == RH_VAL_BYTES ? 8 : 0;
    f->val_len = value_row(s);
    if (f->key_len % 4 || f->val_len % 4)
        return fail(RH_ERR_UNSUPPORTED, "snapshot decode needs key and value lengths that are multiples of 4");
    f->lt = f->key_pre + f->key_len + 20 + 4;  // key, Timestamp (u64 + u32 + u64), State variant
    f->lp = f->lt + f->val_pre + f->val_len;
    f->g = gcd32(f->lt, f->lp);
    f->phases = f->lp / f->g;
    // ~16 entries per segment, and a run of segments + one entry must fit the 32 KiB LDS stage
    f->seg = (uint64_t)f->g * ((16ull * f->lp + f->g - 1) / f->g);
    if (f->seg + f->lp + 48 > 32768) f->seg = (uint64_t)f->g * ((32768ull - f->lp - 48) / f->g);
    if (f->lp + 48 > 32768 || f->seg < f->g || f->phases > 256)
        return fail(RH_ERR_UNSUPPORTED, "snapshot entries too long for the device decoder");
    f->len = len;
    f->base = 16;
    return RH_OK;
}

int snapshot_format(const rh_schema &s, int key_form, size_t len, uint64_t n, rh::SnapFmt *f) {
    int rc = snapshot_layout(s, key_form, len, f);
    if (rc) return rc;
    if (n >= (1ull << 31)) return fail(RH_ERR_UNSUPPORTED, "snapshot has more than 2^31 entries");
    if (n > (len - 16) / f->lt)
        return fail(RH_ERR_DATA, "snapshot entry count " + std::to_string(n) + " exceeds what its " +
                                     std::to_string(len) + " bytes can hold (io error: unexpected end of file)");
    return RH_OK;
}

int snapshot_decode_into(const rh_schema &s, int key_form, const uint8_t *dev, size_t len, uint64_t n,
                         const rh_columns &o, rh::Scratch &scr, hipStream_t st, rh_snapshot_info *info) {
    rh::SnapFmt f;
    int rc = snapshot_format(s, key_form, len, n, &f);
    if (rc) return rc;
    rh::SnapResult res;
    int corrupt = 0;
    RH_HIP(rh::snapshot_decode(f, dev, n, (uint8_t *)o.keys, (uint64_t *)o.phys, (uint32_t *)o.logical,
                               (uint64_t *)o.node, (uint8_t *)o.tags, (uint8_t *)o.values, scr, st, &res, &corrupt));
    if (scr.err) return fail(RH_ERR_OOM, "scratch allocation failed");
    if (corrupt)
        return fail(RH_ERR_DATA, "snapshot entries are corrupt: " + std::to_string(res.parsed) + " of " +
                                     std::to_string(n) + " entries parse (bad State variant, Vec length or "
                                     "end of file)");
    info->entries = n;
    info->tombstones = res.tombstones;
    info->entries_end = res.entries_end;
    info->keys = n;
    return RH_OK;
}

// The reload through the fused pass (snap_lift.hpp): locate the entries, then lift and load them
// straight from the file into the stores' spare base buffers; one wait, then the stores commit
// (a corrupt file leaves both as they were).  The caller holds both stores' locks and n > 0.
// rh_debug_reload_timing: HIP events around the locate stage and the fused pass
std::atomic<int> g_time_reload{0};
std::mutex g_reload_mu;
double g_reload_us[2] = {0, 0};

int snapshot_reload_fused(rh_store *dated, rh_store *proj, int mode, const rh::SnapFmt &f, const uint8_t *dev,
                          uint64_t n, uint32_t nsmax, uint64_t lds, rh_snapshot_info *info, rh::SnapTables &t,
                          bool walked) {
    rh_store *a = dated ? dated : proj;
    int rc;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    struct EvGuard {
        hipEvent_t *e;
        ~EvGuard() {
            for (int k = 0; k < 3; k++)
                if (e[k]) (void)hipEventDestroy(e[k]);
        }
    } ev_guard{ev};
    if (g_time_reload.load()) {
        for (auto &e : ev) RH_HIP(hipEventCreate(&e));
        RH_HIP(hipEventRecord(ev[0], a->stream));
    }
    for (rh_store *x : {dated, proj})
        if (x && (rc = x->load_target(n))) return rc;
    if (walked) RH_HIP(rh::snapshot_place(f, n, true, a->scratch, a->stream, &t, a->flag.p));
    else RH_HIP(rh::snapshot_locate(f, dev, n, true, a->scratch, a->stream, &t, a->flag.p));
    const uint64_t nblk = (n + 255) / 256;
    uint32_t *part = static_cast<uint32_t *>(a->scratch.get(98, nblk * 4));
    if (a->scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
    if (ev[1]) RH_HIP(hipEventRecord(ev[1], a->stream));
    rh::SnapLift L;
    L.blob = dev;
    L.f = f;
    L.n = n;
    L.nseg = t.nseg;
    L.start = t.start;
    L.segq = t.segq;
    L.basev = t.basev;
    L.nsmax = nsmax;
    L.keys = a->bkeys[1 - a->cb].p;
    L.fps = a->bfps[1 - a->cb].p;
    L.bsums = a->sbsums.p;
    L.smp = a->sbsmp.p;
    L.smp2 = a->sbsmp2.p;
    if (mode == 2) {
        L.keys2 = proj->bkeys[1 - proj->cb].p;
        L.fps2 = proj->bfps[1 - proj->cb].p;
        L.bsums2 = proj->sbsums.p;
        L.smp_2 = proj->sbsmp.p;
        L.smp2_2 = proj->sbsmp2.p;
    }
    L.words = t.words;
    L.tomb_part = part;
    L.unsorted = a->flag.p;
    const rh_schema &s = a->schema;
    bool sup = false;
    RH_HIP(rh::launch_snap_lift_schema(s.key_kind, (int)s.key_len, s.value_kind, (int)s.value_len, mode, L, lds,
                                       a->stream, &sup));
    if (!sup) return fail(RH_ERR_STATE, "fused snapshot pass unavailable (internal error)");
    if (ev[2]) RH_HIP(hipEventRecord(ev[2], a->stream));
    RH_HIP(rh::snapshot_sum_tombstones(part, nblk, t.words, a->stream));
    try {
        a->snap_words.assign(4, 0);
    } catch (const std::bad_alloc &) {
        return fail(RH_ERR_OOM, "pinned result buffer");
    }
    RH_HIP(hipMemcpyAsync(a->snap_words.data(), t.words, 32, hipMemcpyDeviceToHost, a->stream));
    // both stores' super sums, search tables and totals into their spare buffers, on their own
    // streams, before the one wait
    if (mode == 2 && (rc = proj->after(a->stream))) return rc;
    for (rh_store *x : {dated, proj})
        if (x && (rc = x->load_stage_sums(n, a->flag.p, x->stream))) return rc;
    if ((rc = a->sync())) return rc;
    // the projection store's staged copy of the unsorted flag (a->flag) must land before the dated
    // store's re-sort in load_finish reuses that flag word for its sort flags
    if (mode == 2 && (rc = proj->sync())) return rc;
    if (ev[2]) {
        float ms[2] = {0, 0};
        RH_HIP(hipEventElapsedTime(&ms[0], ev[0], ev[1]));
        RH_HIP(hipEventElapsedTime(&ms[1], ev[1], ev[2]));
        std::lock_guard<std::mutex> g(g_reload_mu);
        g_reload_us[0] = 1e3 * ms[0];
        g_reload_us[1] = 1e3 * ms[1];
    }
    const uint64_t *w = a->snap_words.data();
    if (w[3] < n || w[1])
        return fail(RH_ERR_DATA, "snapshot entries are corrupt: " + std::to_string(std::min<uint64_t>(w[3], n)) +
                                     " of " + std::to_string(n) +
                                     " entries parse (bad State variant, Vec length or end of file)");
    rh_snapshot_info inf{};
    inf.entries = n;
    inf.tombstones = w[2];
    inf.entries_end = w[0];
    // the stores change from here on.  A failure in either half of either store leaves BOTH
    // stores empty (streams drained): never a new size beside an old root, nor one store
    // replaced and the other not
    for (rh_store *x : {dated, proj}) {
        if (!x) continue;
        if (x == proj && fail_point("snapshot.load_begin")) rc = fail(RH_ERR_OOM, "injected failure (load_begin)");
        else x->load_commit(n);
        if (rc) break;
    }
    for (rh_store *x : {dated, proj}) {
        if (rc) break;
        if (!x) continue;
        if (x == dated && fail_point("snapshot.load_finish")) rc = fail(RH_ERR_OOM, "injected failure (load_finish)");
        else rc = x->load_finish(n, true);
        inf.keys = x->nb;
    }
    if (rc) {
        const std::string msg = g_err;
        for (rh_store *x : {dated, proj})
            if (x) x->reset_empty();
        return fail(rc, msg);
    }
    if (info) *info = inf;
    return RH_OK;
}

}  // namespace

extern "C" {

int rh_snapshot_header(const void *bytes, size_t len, uint64_t *entries) {
    if ((!bytes && len) || !entries) return fail(RH_ERR_ARG, "NULL");
    return snapshot_header(static_cast<const uint8_t *>(bytes), len, entries);
}

int rh_snapshot_decode_device(const rh_schema *schema, int key_form, const void *dev_bytes, size_t len,
                              const rh_columns *o, size_t cap, rh_snapshot_info *info, void *stream) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if ((!dev_bytes && len) || !o) return fail(RH_ERR_ARG, "NULL");
    if (!aligned16(dev_bytes)) return fail(RH_ERR_ARG, "snapshot bytes must be 16-byte aligned");
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint8_t h[16] = {0};
    const size_t hl = std::min<size_t>(len, 16);
    if (hl) RH_HIP(hipMemcpyAsync(h, dev_bytes, hl, hipMemcpyDeviceToHost, st));
    RH_HIP(hipStreamSynchronize(st));
    uint64_t n = 0;
    if ((rc = snapshot_header(h, len, &n))) return rc;
    if (n > cap) return fail(RH_ERR_ARG, "snapshot has " + std::to_string(n) + " entries, more than cap");
    if (n && ((key_row(*schema) && !o->keys) || (value_row(*schema) && !o->values) || !o->phys || !o->logical ||
              !o->node || !o->tags))
        return fail(RH_ERR_ARG, "output columns are NULL");
    if (!aligned16(o->keys) || !aligned16(o->values) || !aligned16(o->phys) || !aligned16(o->node) ||
        !aligned16(o->logical))
        return fail(RH_ERR_ARG, "device columns must be 16-byte aligned");
    // the decode tables are kept per device between calls (the call is synchronous, so the
    // next call may reuse them on any stream)
    static std::mutex scr_mu;
    static std::vector<rh::Scratch> scr_by_dev;
    int dev = 0;
    RH_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> g(scr_mu);
    if ((int)scr_by_dev.size() <= dev) scr_by_dev.resize(dev + 1);
    rh::Scratch &scr = scr_by_dev[dev];
    scr.stream = st;
    scr.err = hipSuccess;
    rh_snapshot_info inf{};
    rc = snapshot_decode_into(*schema, key_form, static_cast<const uint8_t *>(dev_bytes), len, n, *o, scr, st, &inf);
    if (!rc && info) *info = inf;
    return rc;
}

int rh_store_load_snapshot(rh_store *dated, rh_store *proj, int key_form, const void *bytes, size_t len,
                           int on_device, rh_snapshot_info *info, void *after_stream) {
    if (!dated && !proj) return fail(RH_ERR_ARG, "no store given");
    if (!bytes && len) return fail(RH_ERR_ARG, "bytes is NULL");
    if (dated && dated->schema.record_kind != RH_REC_DATED) return fail(RH_ERR_ARG, "dated store must be DATED");
    if (proj && proj->schema.record_kind != RH_REC_PROJECTION)
        return fail(RH_ERR_ARG, "projection store must be PROJECTION");
    if (dated && proj &&
        (dated->schema.key_kind != proj->schema.key_kind || dated->schema.key_len != proj->schema.key_len ||
         dated->schema.value_kind != proj->schema.value_kind || dated->schema.value_len != proj->schema.value_len ||
         dated->device != proj->device))
        return fail(RH_ERR_ARG, "dated and projection stores differ in key / value kind or device");
    rh_store *a = dated ? dated : proj;
    std::unique_lock<std::mutex> la(a->mu, std::defer_lock), lb;
    if (dated && proj) {
        lb = std::unique_lock<std::mutex>(proj->mu, std::defer_lock);
        std::lock(la, lb);
    } else {
        la.lock();
    }
    RH_HIP(hipSetDevice(a->device));
    for (rh_store *x : {dated, proj})  // a reload replaces the contents: staged rows are superseded
        if (x) x->pend.clear();
    int rc;
    uint8_t h[16] = {0};
    const size_t hl = std::min<size_t>(len, 16);
    rh_schema ds = a->schema;
    ds.record_kind = RH_REC_DATED;
    const int mode = dated && proj ? 2 : dated ? 0 : 1;
    rh::SnapTables t;
    bool walked = false;
    if (on_device) {
        if (!aligned16(bytes)) return fail(RH_ERR_ARG, "snapshot bytes must be 16-byte aligned");
        if ((rc = a->after(after_stream))) return rc;
        try {
            a->snap_hdr.assign(2, 0);
        } catch (const std::bad_alloc &) {
            return fail(RH_ERR_OOM, "pinned header buffer");
        }
        if (hl) RH_HIP(hipMemcpyAsync(a->snap_hdr.data(), bytes, hl, hipMemcpyDeviceToHost, a->stream));
        if (!a->hdr_ev) RH_HIP(hipEventCreateWithFlags(&a->hdr_ev, hipEventDisableTiming));
        RH_HIP(hipEventRecord(a->hdr_ev, a->stream));
        // the walk needs the file length, not the entry count: for a shape with the fused pass it
        // starts now, behind the header's copy, and the header is read back while it runs
        rh::SnapFmt fl;
        uint32_t nsm = 0;
        bool sup = false;
        if (hl == 16 && snapshot_layout(ds, key_form, len, &fl) == RH_OK && rh::snap_lift_lds_bytes(fl, &nsm)) {
            RH_HIP(rh::launch_snap_lift_schema(ds.key_kind, (int)ds.key_len, ds.value_kind, (int)ds.value_len, mode,
                                               rh::SnapLift{}, 0, a->stream, &sup));
            if (sup) {
                RH_HIP(rh::snapshot_walk(fl, static_cast<const uint8_t *>(bytes), a->scratch, a->stream, &t));
                if (a->scratch.err) {
                    (void)hipStreamSynchronize(a->stream);
                    return fail(RH_ERR_OOM, "scratch allocation failed");
                }
                walked = true;
            }
        }
        g_err.clear();  // a layout the walk could not take is reported below, after the header
        RH_HIP(hipEventSynchronize(a->hdr_ev));
        memcpy(h, a->snap_hdr.data(), hl);
    } else if (hl) {
        memcpy(h, bytes, hl);
    }
    // a started walk reads the caller's bytes: every early return below waits for it first
    struct WalkGuard {
        rh_store *a;
        bool *on;
        ~WalkGuard() {
            if (*on) (void)hipStreamSynchronize(a->stream);
        }
    } walk_guard{a, &walked};
    uint64_t n = 0;
    if ((rc = snapshot_header(h, len, &n))) return rc;
    rh::SnapFmt f;
    if ((rc = snapshot_format(ds, key_form, len, n, &f))) return rc;
    const uint8_t *dev = static_cast<const uint8_t *>(bytes);
    if (!on_device) {
        if ((rc = a->snap.ensure(len + 16))) return rc;
        RH_HIP(hipMemcpyAsync(a->snap.p, bytes, len, hipMemcpyHostToDevice, a->stream));
        dev = a->snap.p;
    }
    {  // the fused pass, where the shape has one (records up to 192 B)
        uint32_t nsmax = 0;
        const uint64_t lds = n ? rh::snap_lift_lds_bytes(f, &nsmax) : 0;
        bool fused = false;
        if (lds)
            RH_HIP(rh::launch_snap_lift_schema(ds.key_kind, (int)ds.key_len, ds.value_kind, (int)ds.value_len, mode,
                                               rh::SnapLift{}, lds, a->stream, &fused));
        if (fused) {
            rc = snapshot_reload_fused(dated, proj, mode, f, dev, n, nsmax, lds, info, t, walked);
            if (!on_device) a->snap.release();
            return rc;
        }
    }
    DevColumns &stg = a->staging;
    const size_t kr = key_row(ds), vr = value_row(ds);
    if ((rc = stg.keys.ensure(n * kr + 16)) || (rc = stg.values.ensure(n * vr + 16)) || (rc = stg.phys.ensure(n + 1)) ||
        (rc = stg.node.ensure(n + 1)) || (rc = stg.logical.ensure(n + 1)) || (rc = stg.tags.ensure(n + 16)))
        return rc;
    stg.has_tags = true;
    const rh_columns cols = stg.view(ds);
    rh_snapshot_info inf{};
    rc = snapshot_decode_into(ds, key_form, dev, len, n, cols, a->scratch, a->stream, &inf);
    if (!on_device) a->snap.release();
    if (rc) return rc;
    // both stores: Replica::map_insert's two lifts in one read of the columns (the dual kernel
    // writes straight into each store's fingerprint and block-sum buffers)
    const bool dual = dated && proj && n;
    if (dual) {
        for (rh_store *x : {dated, proj})
            if ((rc = x->bfps[x->cb].ensure(n * 32 + 64)) || (rc = x->bsums.ensure(rh_num_blocks(n) * 32 + 32)))
                return rc;
        if ((rc = lift_dispatch(ds, cols, n, dated->bfps[dated->cb].p, dated->bsums.p, proj->bfps[proj->cb].p,
                                proj->bsums.p, true, a->stream)))
            return rc;
        if ((rc = proj->after(a->stream))) return rc;
    }
    // both stores' loads overlap on their own streams.  A failure in either half of either store
    // leaves BOTH stores empty (streams drained): never a new size beside an old root, nor one
    // store replaced and the other not
    for (rh_store *x : {dated, proj}) {
        if (!x) continue;
        if (x == proj && fail_point("snapshot.load_begin")) rc = fail(RH_ERR_OOM, "injected failure (load_begin)");
        else rc = x->load_begin(cols, n, dual);
        if (rc) break;
    }
    for (rh_store *x : {dated, proj}) {
        if (rc) break;
        if (!x) continue;
        if (x == dated && fail_point("snapshot.load_finish")) rc = fail(RH_ERR_OOM, "injected failure (load_finish)");
        else rc = x->load_finish(n, true);
        inf.keys = x->nb;
    }
    if (rc) {
        const std::string msg = g_err;
        for (rh_store *x : {dated, proj})
            if (x) x->reset_empty();
        return fail(rc, msg);
    }
    if (info) *info = inf;
    return RH_OK;
}

int rh_debug_reload_timing(int on) {
    g_time_reload.store(on ? 1 : 0);
    return RH_OK;
}

int rh_debug_last_reload_us(double *locate_us, double *lift_us) {
    if (!locate_us || !lift_us) return fail(RH_ERR_ARG, "NULL");
    std::lock_guard<std::mutex> g(g_reload_mu);
    *locate_us = g_reload_us[0];
    *lift_us = g_reload_us[1];
    return RH_OK;
}

int rh_debug_batch_timing(int on) {
    std::lock_guard<std::mutex> g(g_batch_mu);
    g_time_batch.store(on ? 1 : 0);
    if (on) g_batch_us = 0, g_batch_n = 0;
    return RH_OK;
}

int rh_debug_batch_kernel_us(double *lift_search_us, uint64_t *launches) {
    if (!lift_search_us || !launches) return fail(RH_ERR_ARG, "NULL");
    std::lock_guard<std::mutex> g(g_batch_mu);
    *lift_search_us = g_batch_us;
    *launches = g_batch_n;
    return RH_OK;
}

int rh_debug_fail_point(const char *name) {
    g_fail_point = name ? name : "";
    return RH_OK;
}

}  // extern "C"

// =================================================================================================
// The encoded store: Rsos<K> for any serde K / V (String, Vec<u8>, structs, ...).  The device holds
// the per-record fingerprints in rank order with their block / super-block sums; the records'
// canonical bytes (rsos::encoding::encode_to_vec of k, then of v -- lift is BLAKE3 of their
// concatenation, rsos/src/fingerprint.rs:270-275) are hashed on ingest by the generic encoded-lift
// kernels and not kept.  Keys never cross the ABI: their order is the caller's (the key type's Ord,
// which for String / Vec<u8> is not the order of their length-prefixed encodings), so the caller
// keeps the keys and addresses rows by rank -- exactly what select / enumerate need anyway
// (rsos_trait.rs:66-80).  A batch is a list of rank-addressed operations; the device rebuilds the
// rank order from the old rows and the batch's lifted rows in one pass (launch_seg_copy).
struct rh_estore {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    uint64_t n = 0;
    int cur = 0;
    DevBuf<uint8_t> fps[2], bsums, ssums, lfps, bytes;
    DevBuf<uint64_t> offs, segs, tot, q_lo, q_hi;
    DevBuf<rh_aggregate> q_out;
    uint64_t root[4] = {0, 0, 0, 0};
    // host tier: the exclusive prefix sums of the fingerprints (the same as the store's)
    bool tier_on = false;
    uint64_t version = 0, tier_version = ~0ull;
    rh::HostTier tier;
    PinnedVec<uint64_t> tier_prefix;
    DevBuf<uint8_t> tier_dpre, tier_spre, tier_bpre;

    int sync() {
        RH_HIP(hipStreamSynchronize(stream));
        return RH_OK;
    }
    // upload m records' bytes (host) and lift them into lfps (+ block sums into `bs`, nullable)
    int lift_host(const uint8_t *b, const uint64_t *o, size_t m, uint8_t *out, uint8_t *bs) {
        int rc;
        if (!m) return RH_OK;
        bool fixed = true;  // every record the same length: the fixed-length kernels, no offsets
        for (size_t i = 0; i < m; i++) {
            if (o[i + 1] < o[i]) return fail(RH_ERR_ARG, "record offsets must not decrease");
            fixed = fixed && o[i + 1] - o[i] == o[1] - o[0];
        }
        const uint64_t len = o[m] - o[0], padded = ((len + 3) & ~3ull) + 64;
        if ((rc = bytes.ensure(padded)) || (rc = offs.ensure(m + 1))) return rc;
        RH_HIP(hipMemsetAsync(bytes.p + (len & ~3ull), 0, padded - (len & ~3ull), stream));
        if (len) RH_HIP(hipMemcpyAsync(bytes.p, b + o[0], len, hipMemcpyHostToDevice, stream));
        if (fixed) {  // e.g. a batch of Entry<Timestamp, Vec<u8>> whose values all have one length
            RH_HIP(rh::launch_lift_fixed(bytes.p, o[1] - o[0], m, padded - 64, out, bs, stream));
            return RH_OK;
        }
        if (o[0] == 0) {
            RH_HIP(hipMemcpyAsync(offs.p, o, (m + 1) * 8, hipMemcpyHostToDevice, stream));
        } else {  // rebase to the uploaded span
            std::vector<uint64_t> r(m + 1);
            for (size_t i = 0; i <= m; i++) r[i] = o[i] - o[0];
            RH_HIP(hipMemcpyAsync(offs.p, r.data(), (m + 1) * 8, hipMemcpyHostToDevice, stream));
            RH_HIP(hipStreamSynchronize(stream));  // r dies here
        }
        RH_HIP(rh::launch_lift_encoded(bytes.p, offs.p, m, padded - 64, out, bs, stream));
        return RH_OK;
    }
    // block sums (if not already written), super-block sums and the root of fps[cur]
    int resum(bool have_bsums) {
        int rc;
        const size_t nbk = rh_num_blocks(n), ns = rh_num_superblocks(n);
        if ((rc = bsums.ensure(nbk * 32 + 32)) || (rc = ssums.ensure(ns * 32 + 32)) || (rc = tot.ensure(4))) return rc;
        if (n) {
            if (!have_bsums) RH_HIP(rh::launch_reduce(fps[cur].p, n, bsums.p, stream));
            RH_HIP(rh::launch_reduce(bsums.p, nbk, ssums.p, stream));
            RH_HIP(rh::launch_total(ssums.p, ns, tot.p, stream));
            RH_HIP(hipMemcpyAsync(root, tot.p, 32, hipMemcpyDeviceToHost, stream));
        } else {
            memset(root, 0, sizeof root);
        }
        return sync();
    }
    int tier_refresh() {
        int rc;
        const uint64_t nbk = rh_num_blocks(n), ns = rh_num_superblocks(n);
        if ((rc = tier_dpre.ensure((n + 1) * 32 + 64)) || (rc = tier_spre.ensure((ns + 1) * 32 + 64)) ||
            (rc = tier_bpre.ensure((nbk + 1) * 32 + 64)))
            return rc;
        try {
            tier_prefix.resize((n + 1) * 4 + 8);
        } catch (const std::bad_alloc &) {
            return fail(RH_ERR_OOM, "host tier: page-locked allocation failed");
        }
        if (n) {
            RH_HIP(rh::launch_prefix(fps[cur].p, n, bsums.p, ssums.p, tier_spre.p, tier_bpre.p, tier_dpre.p, stream));
            RH_HIP(hipMemcpyAsync(tier_prefix.data(), tier_dpre.p, (n + 1) * 32, hipMemcpyDeviceToHost, stream));
            if ((rc = sync())) return rc;
        } else {
            memset(tier_prefix.data(), 0, 32);
        }
        tier.build(0, RH_KEY_BYTES, n, nullptr, tier_prefix.data());
        tier_version = version;
        return RH_OK;
    }
    void release() {
        (void)hipStreamSynchronize(stream);
        for (int k = 0; k < 2; k++) fps[k].release();
        bsums.release(); ssums.release(); lfps.release(); bytes.release(); offs.release(); segs.release();
        tot.release(); q_lo.release(); q_hi.release(); q_out.release();
        tier_prefix.release(); tier_dpre.release(); tier_spre.release(); tier_bpre.release();
    }
};

extern "C" {

int rh_estore_create(int device, rh_estore **out) {
    if (!out) return fail(RH_ERR_ARG, "out is NULL");
    RH_HIP(hipSetDevice(device));
    rh_estore *s = new rh_estore();
    s->device = device;
    const hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete s;
        return fail(RH_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    *out = s;
    return RH_OK;
}

int rh_estore_destroy(rh_estore *s) {
    if (!s) return RH_OK;
    (void)hipSetDevice(s->device);
    s->release();
    (void)hipStreamDestroy(s->stream);
    delete s;
    return RH_OK;
}

int rh_estore_load(rh_estore *s, const uint8_t *bytes, const uint64_t *offsets, size_t n) {
    if (!s || (n && (!bytes || !offsets))) return fail(RH_ERR_ARG, "NULL");
    if (n >= (1ull << 31)) return fail(RH_ERR_ARG, "store size limit (2^31 rows) exceeded: use rh_sstore_* for a larger map");
    std::lock_guard<std::mutex> g(s->mu);
    RH_HIP(hipSetDevice(s->device));
    int rc;
    s->version++;
    if ((rc = s->fps[s->cur].ensure(n * 32 + 64)) || (rc = s->bsums.ensure(rh_num_blocks(n) * 32 + 32))) return rc;
    s->n = 0;
    if ((rc = s->lift_host(bytes, offsets, n, s->fps[s->cur].p, s->bsums.p))) return rc;
    s->n = n;
    return s->resum(true);
}

int rh_estore_apply(rh_estore *s, const uint64_t *pos, const uint8_t *kinds, size_t m, const uint8_t *bytes,
                    const uint64_t *offsets, size_t nrec) {
    if (!s || (m && (!pos || !kinds)) || (nrec && (!bytes || !offsets))) return fail(RH_ERR_ARG, "NULL");
    std::lock_guard<std::mutex> g(s->mu);
    const uint64_t n = s->n;
    // the output as segments of old rows and of the batch's records, in the new rank order
    std::vector<uint64_t> start, src;
    uint64_t at = 0, old = 0, rec = 0, last = 0;
    int64_t last_kind = -1;
    auto emit = [&](uint64_t from, uint64_t len, bool is_new) {
        if (!len) return;
        const uint64_t sv = from | (is_new ? (1ull << 63) : 0);
        if (!start.empty()) {  // extend the previous run when it continues
            const uint64_t pv = src.back(), plen = at - start.back();
            if ((pv >> 63) == (sv >> 63) && (pv & ~(1ull << 63)) + plen == from) {
                at += len;
                return;
            }
        }
        start.push_back(at);
        src.push_back(sv);
        at += len;
    };
    try {
        for (size_t i = 0; i < m; i++) {
            const uint64_t p = pos[i];
            const int k = kinds[i];
            if (k > 2) return fail(RH_ERR_ARG, "op kind must be 0 (insert), 1 (overwrite) or 2 (delete)");
            if (i && (p < last || (p == last && (last_kind != 0 || k < last_kind))))
                return fail(RH_ERR_ARG, "ops must be sorted by position, inserts first, at most one overwrite / delete per row");
            if (k == 0 ? p > n : p >= n) return fail(RH_ERR_ARG, "op position out of range");
            if (p > old) {
                emit(old, p - old, false);
                old = p;
            }
            if (k != 2) {
                if (rec >= nrec) return fail(RH_ERR_ARG, "fewer records than insert / overwrite ops");
                emit(rec++, 1, true);
            }
            if (k != 0) old = p + 1;
            last = p;
            last_kind = k;
        }
        if (rec != nrec) return fail(RH_ERR_ARG, "more records than insert / overwrite ops");
        emit(old, n - old, false);
    } catch (const std::bad_alloc &) {
        return fail(RH_ERR_OOM, "apply: host allocation failed");
    }
    const uint64_t n_out = at;
    if (n_out >= (1ull << 31)) return fail(RH_ERR_ARG, "store size limit (2^31 rows) exceeded: use rh_sstore_* for a larger map");
    RH_HIP(hipSetDevice(s->device));
    int rc;
    const int nxt = 1 - s->cur;
    const size_t ns = start.size();
    if ((rc = s->lfps.ensure(nrec * 32 + 64)) || (rc = s->fps[nxt].ensure(n_out * 32 + 64)) ||
        (rc = s->segs.ensure(2 * ns + 2)))
        return rc;
    s->version++;
    if ((rc = s->lift_host(bytes, offsets, nrec, s->lfps.p, nullptr))) return rc;
    if (ns) {
        std::vector<uint64_t> h(2 * ns);
        std::copy(start.begin(), start.end(), h.begin());
        std::copy(src.begin(), src.end(), h.begin() + ns);
        RH_HIP(hipMemcpyAsync(s->segs.p, h.data(), 2 * ns * 8, hipMemcpyHostToDevice, s->stream));
        RH_HIP(rh::launch_seg_copy(s->fps[s->cur].p, s->lfps.p, s->segs.p, s->segs.p + ns, ns, n_out, s->fps[nxt].p,
                                   s->stream));
        RH_HIP(hipStreamSynchronize(s->stream));  // h dies here
    }
    s->cur = nxt;
    s->n = n_out;
    return s->resum(false);
}

int rh_estore_len(rh_estore *s, uint64_t *out) {
    if (!s || !out) return fail(RH_ERR_ARG, "NULL");
    std::lock_guard<std::mutex> g(s->mu);
    *out = s->n;
    return RH_OK;
}

int rh_estore_aggregates(rh_estore *s, const uint64_t *lo, const uint64_t *hi, size_t r, rh_aggregate *out) {
    if (!s || (r && (!lo || !hi || !out))) return fail(RH_ERR_ARG, "NULL");
    if (!r) return RH_OK;
    std::lock_guard<std::mutex> g(s->mu);
    int rc;
    if (s->tier_on) {
        if (s->tier_version != s->version) {
            RH_HIP(hipSetDevice(s->device));
            if ((rc = s->tier_refresh())) return rc;
        }
        for (size_t j = 0; j < r; j++) s->tier.agg(lo[j], hi[j], out + j);
        return RH_OK;
    }
    RH_HIP(hipSetDevice(s->device));
    if ((rc = s->q_lo.ensure(r)) || (rc = s->q_hi.ensure(r)) || (rc = s->q_out.ensure(r))) return rc;
    RH_HIP(hipMemcpyAsync(s->q_lo.p, lo, r * 8, hipMemcpyHostToDevice, s->stream));
    RH_HIP(hipMemcpyAsync(s->q_hi.p, hi, r * 8, hipMemcpyHostToDevice, s->stream));
    RH_HIP(rh::launch_range_query(s->fps[s->cur].p, s->bsums.p, s->ssums.p, s->n, s->q_lo.p, s->q_hi.p, r,
                                  reinterpret_cast<uint64_t *>(s->q_out.p), s->stream));
    RH_HIP(hipMemcpyAsync(out, s->q_out.p, r * sizeof(rh_aggregate), hipMemcpyDeviceToHost, s->stream));
    return s->sync();
}

int rh_estore_root(rh_estore *s, rh_aggregate *out) {
    if (!s || !out) return fail(RH_ERR_ARG, "NULL");
    std::lock_guard<std::mutex> g(s->mu);
    memcpy(out->fingerprint, s->root, 32);
    out->size = s->n;
    return RH_OK;
}

int rh_estore_fingerprints(rh_estore *s, uint64_t lo, uint64_t hi, uint8_t *host_out) {
    if (!s) return fail(RH_ERR_ARG, "NULL");
    std::lock_guard<std::mutex> g(s->mu);
    if (lo > hi || hi > s->n) return fail(RH_ERR_ARG, "bad rank range");
    if (hi == lo) return RH_OK;
    if (!host_out) return fail(RH_ERR_ARG, "host_out NULL");
    RH_HIP(hipSetDevice(s->device));
    RH_HIP(hipMemcpyAsync(host_out, s->fps[s->cur].p + lo * 32, (hi - lo) * 32, hipMemcpyDeviceToHost, s->stream));
    return s->sync();
}

int rh_estore_set_host_tier(rh_estore *s, int enable) {
    if (!s || enable < 0 || enable > 1) return fail(RH_ERR_ARG, "bad host tier setting");
    std::lock_guard<std::mutex> g(s->mu);
    s->tier_on = enable == 1;
    if (!s->tier_on) {
        s->tier_version = ~0ull;
        s->tier.reset();
        s->tier_prefix.release();
    }
    return RH_OK;
}

}  // extern "C"
