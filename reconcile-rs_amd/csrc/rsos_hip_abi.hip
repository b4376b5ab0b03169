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
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rsos_hip.h"
#include "internal.hpp"
#include "lift_kernels.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

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

int lift_dispatch(const rh_schema &s, const rh_columns &c, size_t n, uint8_t *fps, uint8_t *bs,
                  uint8_t *fps2, uint8_t *bs2, bool dual, hipStream_t st) {
    bool supported = false;
    hipError_t e = rh::launch_lift_schema(s.key_kind, (int)s.key_len, s.value_kind, (int)s.value_len,
                                          s.record_kind, c.tags != nullptr, dual, to_dev(c), n, fps, bs,
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
    int ensure(size_t n) {
        if (n <= cap && p) return RH_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
        bytes = (bytes + 255) & ~size_t(255);
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) return fail(RH_ERR_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
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

int rh_lift_encoded_async(const uint8_t *bytes, const uint64_t *offsets, size_t n, uint8_t *fps,
                          uint8_t *block_sums, void *stream) {
    if (n == 0) return RH_OK;
    if (!offsets || !fps) return fail(RH_ERR_ARG, "offsets / fps is NULL");
    if (!aligned16(fps) || !aligned16(block_sums)) return fail(RH_ERR_ARG, "outputs must be 16-byte aligned");
    // the kernel needs the total byte count as its read limit: read offsets[n] (8 bytes)
    uint64_t total = 0;
    hipStream_t st = static_cast<hipStream_t>(stream);
    RH_HIP(hipMemcpyAsync(&total, offsets + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    RH_HIP(hipStreamSynchronize(st));
    if (total && !bytes) return fail(RH_ERR_ARG, "bytes is NULL");
    const uint64_t limit = (total + 3) & ~3ull;
    RH_HIP(rh::launch_lift_encoded(bytes, offsets, n, limit, fps, block_sums, st));
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
        if (n && kr) RH_HIP(hipMemcpyAsync(keys.p, h.keys, n * kr, hipMemcpyHostToDevice, st));
        if (n && vr) RH_HIP(hipMemcpyAsync(values.p, h.values, n * vr, hipMemcpyHostToDevice, st));
        if (s.record_kind == RH_REC_DATED) {
            if ((rc = phys.ensure(n)) || (rc = node.ensure(n)) || (rc = logical.ensure(n))) return rc;
            if (n) {
                RH_HIP(hipMemcpyAsync(phys.p, h.phys, n * 8, hipMemcpyHostToDevice, st));
                RH_HIP(hipMemcpyAsync(node.p, h.node, n * 8, hipMemcpyHostToDevice, st));
                RH_HIP(hipMemcpyAsync(logical.p, h.logical, n * 4, hipMemcpyHostToDevice, st));
            }
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

extern "C" int rh_lift_host(int device, const rh_schema *schema, const rh_columns *h, size_t n, uint8_t *host_fps) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if (!h) return fail(RH_ERR_ARG, "columns is NULL");
    if (n == 0) return RH_OK;
    if (!host_fps) return fail(RH_ERR_ARG, "host_fps is NULL");
    RH_HIP(hipSetDevice(device));
    hipStream_t st;
    RH_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    DevColumns dc;
    DevBuf<uint8_t> fps;
    rc = dc.upload(*schema, *h, n, st);
    if (!rc) rc = fps.ensure(n * 32);
    if (!rc) {
        rh_columns v = dc.view(*schema);
        rc = lift_dispatch(*schema, v, n, fps.p, nullptr, nullptr, nullptr, false, st);
    }
    if (!rc) {
        hipError_t e = hipMemcpyAsync(host_fps, fps.p, n * 32, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = fail(RH_ERR_HIP, std::string("rh_lift_host: ") + hipGetErrorString(e));
    }
    (void)hipStreamSynchronize(st);
    dc.release();
    fps.release();
    (void)hipStreamDestroy(st);
    return rc;
}

// =================================================================================================
// The GPU-resident store
struct rh_store {
    int device = 0;
    rh_schema schema{};
    hipStream_t stream = nullptr;
    std::mutex mu;  // serialises callers sharing one store (readers under a RwLock read guard)
    size_t n = 0;
    size_t krow = 0, vrow = 0;
    // host mirror (rank order): key column for rank/select, full columns for rebuilds
    std::vector<uint8_t> h_keys, h_values, h_tags;
    std::vector<uint64_t> h_phys, h_node;
    std::vector<uint32_t> h_logical;
    bool has_tags = false;
    // device
    DevColumns cols;
    DevBuf<uint8_t> fps, bsums, ssums;
    DevBuf<uint64_t> q_lo, q_hi;
    DevBuf<rh_aggregate> q_out;

    int cmp_keys(const uint8_t *a, const uint8_t *b) const {
        switch (schema.key_kind) {
        case RH_KEY_U32: { uint32_t x, y; memcpy(&x, a, 4); memcpy(&y, b, 4); return (x > y) - (x < y); }
        case RH_KEY_U64: { uint64_t x, y; memcpy(&x, a, 8); memcpy(&y, b, 8); return (x > y) - (x < y); }
        case RH_KEY_UNIT: return 0;
        default: return memcmp(a, b, krow);
        }
    }
    // number of keys strictly below key (query.rs:93-121)
    size_t rank_of(const uint8_t *key) const {
        size_t lo = 0, hi = n;
        while (lo < hi) {
            size_t mid = (lo + hi) / 2;
            if (cmp_keys(&h_keys[mid * krow], key) < 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    int rebuild() {
        int rc;
        rh_columns h;
        h.keys = h_keys.data();
        h.values = h_values.data();
        h.phys = h_phys.data();
        h.node = h_node.data();
        h.logical = h_logical.data();
        h.tags = has_tags ? h_tags.data() : nullptr;
        if ((rc = cols.upload(schema, h, n, stream))) return rc;
        const size_t nb = rh_num_blocks(n), ns = rh_num_superblocks(n);
        if ((rc = fps.ensure(n * 32 + 32)) || (rc = bsums.ensure(nb * 32 + 32)) || (rc = ssums.ensure(ns * 32 + 32)))
            return rc;
        if (n) {
            rh_columns v = cols.view(schema);
            if ((rc = lift_dispatch(schema, v, n, fps.p, bsums.p, nullptr, nullptr, false, stream))) return rc;
            RH_HIP(rh::launch_reduce(bsums.p, nb, ssums.p, stream));
        }
        RH_HIP(hipStreamSynchronize(stream));
        return RH_OK;
    }
    int query(const uint64_t *lo, const uint64_t *hi, size_t r, rh_aggregate *out) {
        int rc;
        if (r == 0) return RH_OK;
        if ((rc = q_lo.ensure(r)) || (rc = q_hi.ensure(r)) || (rc = q_out.ensure(r))) return rc;
        RH_HIP(hipMemcpyAsync(q_lo.p, lo, r * 8, hipMemcpyHostToDevice, stream));
        RH_HIP(hipMemcpyAsync(q_hi.p, hi, r * 8, hipMemcpyHostToDevice, stream));
        RH_HIP(rh::launch_range_query(fps.p, bsums.p, ssums.p, n, q_lo.p, q_hi.p, r,
                                      reinterpret_cast<uint64_t *>(q_out.p), stream));
        RH_HIP(hipMemcpyAsync(out, q_out.p, r * sizeof(rh_aggregate), hipMemcpyDeviceToHost, stream));
        RH_HIP(hipStreamSynchronize(stream));
        return RH_OK;
    }
};

extern "C" {

int rh_store_create(int device, const rh_schema *schema, rh_store **out) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if (!out) return fail(RH_ERR_ARG, "out is NULL");
    if (rh_schema_supported(schema) != 1)
        return fail(RH_ERR_UNSUPPORTED, "store needs a schema with a specialised lift kernel");
    RH_HIP(hipSetDevice(device));
    rh_store *s = new rh_store();
    s->device = device;
    s->schema = *schema;
    s->krow = key_row(*schema);
    s->vrow = value_row(*schema);
    hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete s;
        return fail(RH_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    *out = s;
    return RH_OK;
}

int rh_store_destroy(rh_store *s) {
    if (!s) return RH_OK;
    (void)hipSetDevice(s->device);
    (void)hipStreamSynchronize(s->stream);
    s->cols.release();
    s->fps.release();
    s->bsums.release();
    s->ssums.release();
    s->q_lo.release();
    s->q_hi.release();
    s->q_out.release();
    (void)hipStreamDestroy(s->stream);
    delete s;
    return RH_OK;
}

int rh_store_load(rh_store *s, const rh_columns *h, size_t n) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    if (!h) return fail(RH_ERR_ARG, "columns is NULL");
    std::lock_guard<std::mutex> g(s->mu);
    RH_HIP(hipSetDevice(s->device));
    const rh_schema &sc = s->schema;
    if (n) {
        if (s->krow && !h->keys) return fail(RH_ERR_ARG, "keys NULL");
        if (s->vrow && !h->values) return fail(RH_ERR_ARG, "values NULL");
        if (sc.record_kind == RH_REC_DATED && (!h->phys || !h->node || !h->logical))
            return fail(RH_ERR_ARG, "DATED needs stamp columns");
    }
    const uint8_t *k = static_cast<const uint8_t *>(h->keys);
    for (size_t i = 1; i < n; i++)
        if (s->cmp_keys(k + (i - 1) * s->krow, k + i * s->krow) >= 0)
            return fail(RH_ERR_ARG, "keys must be strictly increasing (sorted, no duplicates)");
    s->n = n;
    s->h_keys.assign(k, k + n * s->krow);
    const uint8_t *v = static_cast<const uint8_t *>(h->values);
    s->h_values.assign(v, v + n * s->vrow);
    if (sc.record_kind == RH_REC_DATED) {
        s->h_phys.assign(h->phys, h->phys + n);
        s->h_node.assign(h->node, h->node + n);
        s->h_logical.assign(h->logical, h->logical + n);
    }
    s->has_tags = h->tags != nullptr && sc.record_kind != RH_REC_PLAIN;
    if (s->has_tags) s->h_tags.assign(h->tags, h->tags + n);
    else s->h_tags.clear();
    return s->rebuild();
}

int rh_store_len(const rh_store *s, uint64_t *out) {
    if (!s || !out) return fail(RH_ERR_ARG, "NULL");
    *out = s->n;
    return RH_OK;
}

int rh_store_aggregates(rh_store *s, const uint64_t *lo, const uint64_t *hi, size_t r, rh_aggregate *out) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    if (r && (!lo || !hi || !out)) return fail(RH_ERR_ARG, "NULL buffer");
    std::lock_guard<std::mutex> g(s->mu);
    RH_HIP(hipSetDevice(s->device));
    return s->query(lo, hi, r, out);
}

int rh_store_aggregate(rh_store *s, uint64_t lo, uint64_t hi, rh_aggregate *out) {
    return rh_store_aggregates(s, &lo, &hi, 1, out);
}

int rh_store_rank(const rh_store *s, const void *key, uint64_t *out) {
    if (!s || !key || !out) return fail(RH_ERR_ARG, "NULL");
    *out = s->rank_of(static_cast<const uint8_t *>(key));
    return RH_OK;
}

int rh_store_select(const rh_store *s, uint64_t r, void *key_out) {
    if (!s || !key_out) return fail(RH_ERR_ARG, "NULL");
    if (r >= s->n) return fail(RH_ERR_ARG, "select: rank out of range (r >= size)");
    memcpy(key_out, &s->h_keys[r * s->krow], s->krow);
    return RH_OK;
}

// Bound -> rank: Included(k) lower = rank(k); Excluded(k) lower = rank(k) + [k present];
// Included(k) upper = rank(k) + [k present]; Excluded(k) upper = rank(k).
static size_t bound_rank(const rh_store *s, int kind, const uint8_t *key, bool lower) {
    if (kind == 0) return lower ? 0 : s->n;
    size_t r = s->rank_of(key);
    bool present = r < s->n && s->cmp_keys(&s->h_keys[r * s->krow], key) == 0;
    bool incl = kind == 1;
    if (lower) return (!incl && present) ? r + 1 : r;
    return (incl && present) ? r + 1 : r;
}

int rh_store_aggregate_keys(rh_store *s, int lo_kind, const void *lo_key, int hi_kind, const void *hi_key,
                            rh_aggregate *out) {
    if (!s || !out) return fail(RH_ERR_ARG, "NULL");
    if (lo_kind < 0 || lo_kind > 2 || hi_kind < 0 || hi_kind > 2) return fail(RH_ERR_ARG, "bad bound kind");
    if ((lo_kind && !lo_key) || (hi_kind && !hi_key)) return fail(RH_ERR_ARG, "bound key is NULL");
    uint64_t lo = bound_rank(s, lo_kind, static_cast<const uint8_t *>(lo_key), true);
    uint64_t hi = bound_rank(s, hi_kind, static_cast<const uint8_t *>(hi_key), false);
    if (hi < lo) hi = lo;  // inverted range -> ZERO (rbsr/src/protocol.rs:230-232)
    return rh_store_aggregates(s, &lo, &hi, 1, out);
}

int rh_store_fingerprints(rh_store *s, uint64_t lo, uint64_t hi, uint8_t *host_out) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    if (lo > hi || hi > s->n) return fail(RH_ERR_ARG, "bad rank range");
    if (hi > lo && !host_out) return fail(RH_ERR_ARG, "host_out NULL");
    std::lock_guard<std::mutex> g(s->mu);
    RH_HIP(hipSetDevice(s->device));
    if (hi > lo) {
        RH_HIP(hipMemcpyAsync(host_out, s->fps.p + lo * 32, (hi - lo) * 32, hipMemcpyDeviceToHost, s->stream));
        RH_HIP(hipStreamSynchronize(s->stream));
    }
    return RH_OK;
}

// Batched insert / overwrite / delete.  Host merge of the sorted batch into the rank-ordered
// mirror, then a device rebuild (re-lift + re-sum).  Semantics follow FingerprintTreeMap::insert
// (overwrite = new fp replaces old: the `new - old` delta of mutate.rs:31-41) and ::remove
// (mutate.rs:93-154): the resulting aggregates equal a fold of lift over the final contents.
int rh_store_apply(rh_store *s, const rh_columns *h, const uint8_t *ops, size_t m, uint64_t *n_new,
                   uint64_t *n_over, uint64_t *n_del) {
    if (!s || !h || (m && !ops)) return fail(RH_ERR_ARG, "NULL");
    std::lock_guard<std::mutex> g(s->mu);
    RH_HIP(hipSetDevice(s->device));
    const rh_schema &sc = s->schema;
    const size_t kr = s->krow, vr = s->vrow;
    const uint8_t *bk = static_cast<const uint8_t *>(h->keys);
    const uint8_t *bv = static_cast<const uint8_t *>(h->values);
    bool any_insert = false;
    for (size_t i = 0; i < m; i++) any_insert |= ops[i] == 0;
    if (m && !bk) return fail(RH_ERR_ARG, "keys NULL");
    if (any_insert && vr && !bv) return fail(RH_ERR_ARG, "values NULL");
    if (any_insert && sc.record_kind == RH_REC_DATED && (!h->phys || !h->node || !h->logical))
        return fail(RH_ERR_ARG, "DATED needs stamp columns");
    // order the batch by key
    std::vector<size_t> order(m);
    for (size_t i = 0; i < m; i++) order[i] = i;
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return s->cmp_keys(bk + a * kr, bk + b * kr) < 0; });
    for (size_t i = 1; i < m; i++)
        if (s->cmp_keys(bk + order[i - 1] * kr, bk + order[i] * kr) == 0)
            return fail(RH_ERR_ARG, "duplicate key within one batch");
    const bool tags_out = s->has_tags || (h->tags != nullptr && sc.record_kind != RH_REC_PLAIN);
    std::vector<uint8_t> nk, nv, nt;
    std::vector<uint64_t> np, nn;
    std::vector<uint32_t> nl;
    nk.reserve((s->n + m) * kr);
    nv.reserve((s->n + m) * vr);
    const bool dated = sc.record_kind == RH_REC_DATED;
    uint64_t c_new = 0, c_over = 0, c_del = 0;
    auto push_old = [&](size_t i) {
        nk.insert(nk.end(), &s->h_keys[i * kr], &s->h_keys[i * kr] + kr);
        nv.insert(nv.end(), s->h_values.data() + i * vr, s->h_values.data() + (i + 1) * vr);
        if (dated) { np.push_back(s->h_phys[i]); nn.push_back(s->h_node[i]); nl.push_back(s->h_logical[i]); }
        if (tags_out) nt.push_back(s->has_tags ? s->h_tags[i] : 0);
    };
    auto push_new = [&](size_t j) {
        nk.insert(nk.end(), bk + j * kr, bk + (j + 1) * kr);
        if (vr) nv.insert(nv.end(), bv + j * vr, bv + (j + 1) * vr);
        if (dated) { np.push_back(h->phys[j]); nn.push_back(h->node[j]); nl.push_back(h->logical[j]); }
        if (tags_out) nt.push_back(h->tags ? h->tags[j] : 0);
    };
    size_t i = 0;
    for (size_t t = 0; t < m; t++) {
        const size_t j = order[t];
        const uint8_t *key = bk + j * kr;
        while (i < s->n && s->cmp_keys(&s->h_keys[i * kr], key) < 0) push_old(i++);
        const bool present = i < s->n && s->cmp_keys(&s->h_keys[i * kr], key) == 0;
        if (ops[j] == 0) {
            push_new(j);
            if (present) { c_over++; i++; } else c_new++;
        } else {
            if (present) { c_del++; i++; }
        }
    }
    while (i < s->n) push_old(i++);
    s->n = nk.size() / (kr ? kr : 1);
    if (!kr) s->n = nv.size() / (vr ? vr : 1);
    s->h_keys.swap(nk);
    s->h_values.swap(nv);
    s->h_phys.swap(np);
    s->h_node.swap(nn);
    s->h_logical.swap(nl);
    s->h_tags.swap(nt);
    s->has_tags = tags_out;
    if (n_new) *n_new = c_new;
    if (n_over) *n_over = c_over;
    if (n_del) *n_del = c_del;
    return s->rebuild();
}

}  // extern "C"
