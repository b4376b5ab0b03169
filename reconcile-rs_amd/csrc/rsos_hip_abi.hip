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
#include "store_kernels.hpp"

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
// The GPU-resident store: keys + fingerprints + block / super-block sums in HBM, rank order.
struct rh_store {
    int device = 0;
    rh_schema schema{};
    hipStream_t stream = nullptr;
    std::mutex mu;  // serialises callers sharing one store (readers under a RwLock read guard)
    rh::StoreKeyOps *kops = nullptr;
    size_t kl = 0;
    uint64_t n = 0;
    int cur = 0;
    DevBuf<uint8_t> keys[2], fps[2];  // double-buffered: a batch merges from one into the other
    DevBuf<uint8_t> bsums, ssums;
    DevColumns staging;               // host batches land here
    DevBuf<uint8_t> bfps, skeys, sfps, sops, hops;
    DevBuf<uint64_t> q_lo, q_hi, counts;
    DevBuf<rh_aggregate> q_out;
    DevBuf<uint8_t> q_keys;
    DevBuf<uint32_t> flag, q_rank;
    rh::Scratch scratch;

    int sync() {
        RH_HIP(hipStreamSynchronize(stream));
        return RH_OK;
    }
    int resum() {  // block + super-block sums of the current contents
        int rc;
        const size_t nb = rh_num_blocks(n), ns = rh_num_superblocks(n);
        if ((rc = bsums.ensure(nb * 32 + 32)) || (rc = ssums.ensure(ns * 32 + 32))) return rc;
        if (n) {
            RH_HIP(rh::launch_reduce(fps[cur].p, n, bsums.p, stream));
            RH_HIP(rh::launch_reduce(bsums.p, nb, ssums.p, stream));
        }
        return RH_OK;
    }
    int load_device(const rh_columns &c, size_t m) {
        int rc;
        const int nxt = cur;  // contents are replaced in place
        if ((rc = keys[nxt].ensure(m * kl + 64)) || (rc = fps[nxt].ensure(m * 32 + 64)) || (rc = flag.ensure(4))) return rc;
        if (m) {
            RH_HIP(hipMemcpyAsync(keys[nxt].p, c.keys, m * kl, hipMemcpyDeviceToDevice, stream));
            if ((rc = lift_dispatch(schema, c, m, fps[nxt].p, nullptr, nullptr, nullptr, false, stream))) return rc;
            RH_HIP(hipMemsetAsync(flag.p, 0, 4, stream));
            RH_HIP(kops->check_sorted(keys[nxt].p, m, flag.p, stream));
        }
        uint32_t bad = 0;
        if (m) RH_HIP(hipMemcpyAsync(&bad, flag.p, 4, hipMemcpyDeviceToHost, stream));
        if ((rc = sync())) return rc;
        if (bad) {
            n = 0;
            return fail(RH_ERR_ARG, "keys must be strictly increasing (sorted, no duplicates)");
        }
        n = m;
        if ((rc = resum())) return rc;
        return sync();
    }
    int apply_device(const rh_columns &c, const uint8_t *ops, size_t m, uint64_t out[3]) {
        int rc;
        out[0] = out[1] = out[2] = 0;
        if (m == 0) return RH_OK;
        if (n + m >= (1ull << 31)) return fail(RH_ERR_ARG, "store size limit (2^31 rows) exceeded");
        if ((rc = bfps.ensure(m * 32 + 64)) || (rc = skeys.ensure(m * kl + 64)) || (rc = sfps.ensure(m * 32 + 64)) ||
            (rc = sops.ensure(m + 64)) || (rc = flag.ensure(4)) || (rc = counts.ensure(4)))
            return rc;
        // 1. lift the batch (deletes are lifted too and ignored: their value columns may be garbage
        //    but are never read past their own rows)
        if ((rc = lift_dispatch(schema, c, m, bfps.p, nullptr, nullptr, nullptr, false, stream))) return rc;
        // 2. key order + duplicate check
        RH_HIP(hipMemsetAsync(flag.p, 0, 4, stream));
        RH_HIP(kops->sort_batch(static_cast<const uint8_t *>(c.keys), bfps.p, ops, m, scratch, skeys.p, sfps.p,
                                sops.p, flag.p, stream));
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        uint32_t dup = 0;
        RH_HIP(hipMemcpyAsync(&dup, flag.p, 4, hipMemcpyDeviceToHost, stream));
        if ((rc = sync())) return rc;
        if (dup) return fail(RH_ERR_ARG, "duplicate key within one batch");
        // 3. merge into the other buffer, then swap
        const int nxt = 1 - cur;
        if ((rc = keys[nxt].ensure((n + m) * kl + 64)) || (rc = fps[nxt].ensure((n + m) * 32 + 64))) return rc;
        RH_HIP(kops->merge(keys[cur].p, fps[cur].p, n, skeys.p, sfps.p, sops.p, m, scratch, keys[nxt].p, fps[nxt].p,
                           counts.p, stream));
        if (scratch.err) return fail(RH_ERR_OOM, "scratch allocation failed");
        RH_HIP(hipMemcpyAsync(out, counts.p, 24, hipMemcpyDeviceToHost, stream));
        if ((rc = sync())) return rc;
        cur = nxt;
        n = n + out[0] - out[2];
        if ((rc = resum())) return rc;
        return sync();
    }
    int query(const uint64_t *lo, const uint64_t *hi, size_t r, rh_aggregate *out) {
        int rc;
        if (r == 0) return RH_OK;
        if ((rc = q_lo.ensure(r)) || (rc = q_hi.ensure(r)) || (rc = q_out.ensure(r))) return rc;
        RH_HIP(hipMemcpyAsync(q_lo.p, lo, r * 8, hipMemcpyHostToDevice, stream));
        RH_HIP(hipMemcpyAsync(q_hi.p, hi, r * 8, hipMemcpyHostToDevice, stream));
        RH_HIP(rh::launch_range_query(fps[cur].p, bsums.p, ssums.p, n, q_lo.p, q_hi.p, r,
                                      reinterpret_cast<uint64_t *>(q_out.p), stream));
        RH_HIP(hipMemcpyAsync(out, q_out.p, r * sizeof(rh_aggregate), hipMemcpyDeviceToHost, stream));
        return sync();
    }
    void release() {
        (void)hipStreamSynchronize(stream);
        for (int k = 0; k < 2; k++) { keys[k].release(); fps[k].release(); }
        bsums.release(); ssums.release(); staging.release();
        bfps.release(); skeys.release(); sfps.release(); sops.release(); hops.release();
        q_lo.release(); q_hi.release(); counts.release(); q_out.release(); q_keys.release();
        flag.release(); q_rank.release();
        scratch.release();
    }
};

#define RH_LOCK(s)                                  \
    std::lock_guard<std::mutex> guard_((s)->mu);    \
    RH_HIP(hipSetDevice((s)->device))

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
    hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
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
    if (!s || !h) return fail(RH_ERR_ARG, "NULL");
    RH_LOCK(s);
    int rc;
    if ((rc = s->staging.upload(s->schema, *h, n, s->stream))) return rc;
    return s->load_device(s->staging.view(s->schema), n);
}

int rh_store_load_device(rh_store *s, const rh_columns *dev_cols, size_t n) {
    if (!s) return fail(RH_ERR_ARG, "NULL");
    int rc = check_cols(s->schema, dev_cols, n);
    if (rc) return rc;
    RH_LOCK(s);
    return s->load_device(*dev_cols, n);
}

int rh_store_len(const rh_store *s, uint64_t *out) {
    if (!s || !out) return fail(RH_ERR_ARG, "NULL");
    *out = s->n;
    return RH_OK;
}

int rh_store_aggregates(rh_store *s, const uint64_t *lo, const uint64_t *hi, size_t r, rh_aggregate *out) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    if (r && (!lo || !hi || !out)) return fail(RH_ERR_ARG, "NULL buffer");
    RH_LOCK(s);
    return s->query(lo, hi, r, out);
}

int rh_store_aggregate(rh_store *s, uint64_t lo, uint64_t hi, rh_aggregate *out) {
    return rh_store_aggregates(s, &lo, &hi, 1, out);
}

int rh_store_ranks(rh_store *s, const void *keys, size_t m, uint64_t *out) {
    if (!s || (m && (!keys || !out))) return fail(RH_ERR_ARG, "NULL");
    if (m == 0) return RH_OK;
    RH_LOCK(s);
    int rc;
    if ((rc = s->q_keys.ensure(m * s->kl + 64)) || (rc = s->q_rank.ensure(m))) return rc;
    RH_HIP(hipMemcpyAsync(s->q_keys.p, keys, m * s->kl, hipMemcpyHostToDevice, s->stream));
    RH_HIP(s->kops->search(s->keys[s->cur].p, s->n, s->q_keys.p, m, s->q_rank.p, nullptr, s->stream));
    std::vector<uint32_t> r32(m);
    RH_HIP(hipMemcpyAsync(r32.data(), s->q_rank.p, m * 4, hipMemcpyDeviceToHost, s->stream));
    if ((rc = s->sync())) return rc;
    for (size_t j = 0; j < m; j++) out[j] = r32[j];
    return RH_OK;
}

int rh_store_rank(rh_store *s, const void *key, uint64_t *out) { return rh_store_ranks(s, key, 1, out); }

int rh_store_keys(rh_store *s, uint64_t lo, uint64_t hi, void *host_out) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    if (lo > hi || hi > s->n) return fail(RH_ERR_ARG, "bad rank range");
    if (hi == lo) return RH_OK;
    if (!host_out) return fail(RH_ERR_ARG, "host_out NULL");
    RH_LOCK(s);
    RH_HIP(hipMemcpyAsync(host_out, s->keys[s->cur].p + lo * s->kl, (hi - lo) * s->kl, hipMemcpyDeviceToHost,
                          s->stream));
    return s->sync();
}

int rh_store_select(rh_store *s, uint64_t r, void *key_out) {
    if (!s || !key_out) return fail(RH_ERR_ARG, "NULL");
    if (r >= s->n) return fail(RH_ERR_ARG, "select: rank out of range (r >= size)");
    return rh_store_keys(s, r, r + 1, key_out);
}

int rh_store_aggregate_keys(rh_store *s, int lo_kind, const void *lo_key, int hi_kind, const void *hi_key,
                            rh_aggregate *out) {
    if (!s || !out) return fail(RH_ERR_ARG, "NULL");
    if (lo_kind < 0 || lo_kind > 2 || hi_kind < 0 || hi_kind > 2) return fail(RH_ERR_ARG, "bad bound kind");
    if ((lo_kind && !lo_key) || (hi_kind && !hi_key)) return fail(RH_ERR_ARG, "bound key is NULL");
    RH_LOCK(s);
    int rc;
    if ((rc = s->q_keys.ensure(2 * s->kl + 64)) || (rc = s->q_lo.ensure(1)) || (rc = s->q_hi.ensure(1)) ||
        (rc = s->q_out.ensure(1)))
        return rc;
    if (lo_kind) RH_HIP(hipMemcpyAsync(s->q_keys.p, lo_key, s->kl, hipMemcpyHostToDevice, s->stream));
    if (hi_kind) RH_HIP(hipMemcpyAsync(s->q_keys.p + s->kl, hi_key, s->kl, hipMemcpyHostToDevice, s->stream));
    RH_HIP(s->kops->bounds(s->keys[s->cur].p, s->n, s->q_keys.p, lo_kind, s->q_keys.p + s->kl, hi_kind, s->q_lo.p,
                           s->q_hi.p, s->stream));
    RH_HIP(rh::launch_range_query(s->fps[s->cur].p, s->bsums.p, s->ssums.p, s->n, s->q_lo.p, s->q_hi.p, 1,
                                  reinterpret_cast<uint64_t *>(s->q_out.p), s->stream));
    RH_HIP(hipMemcpyAsync(out, s->q_out.p, sizeof(rh_aggregate), hipMemcpyDeviceToHost, s->stream));
    return s->sync();
}

int rh_store_fingerprints(rh_store *s, uint64_t lo, uint64_t hi, uint8_t *host_out) {
    if (!s) return fail(RH_ERR_ARG, "store is NULL");
    if (lo > hi || hi > s->n) return fail(RH_ERR_ARG, "bad rank range");
    if (hi > lo && !host_out) return fail(RH_ERR_ARG, "host_out NULL");
    RH_LOCK(s);
    if (hi > lo)
        RH_HIP(hipMemcpyAsync(host_out, s->fps[s->cur].p + lo * 32, (hi - lo) * 32, hipMemcpyDeviceToHost, s->stream));
    return s->sync();
}

int rh_store_apply(rh_store *s, const rh_columns *h, const uint8_t *ops, size_t m, uint64_t *n_new,
                   uint64_t *n_over, uint64_t *n_del) {
    if (!s || !h || (m && !ops)) return fail(RH_ERR_ARG, "NULL");
    RH_LOCK(s);
    int rc;
    if ((rc = s->staging.upload(s->schema, *h, m, s->stream)) || (rc = s->hops.ensure(m + 64))) return rc;
    if (m) RH_HIP(hipMemcpyAsync(s->hops.p, ops, m, hipMemcpyHostToDevice, s->stream));
    uint64_t c[3];
    if ((rc = s->apply_device(s->staging.view(s->schema), s->hops.p, m, c))) return rc;
    if (n_new) *n_new = c[0];
    if (n_over) *n_over = c[1];
    if (n_del) *n_del = c[2];
    return RH_OK;
}

int rh_store_apply_device(rh_store *s, const rh_columns *dev_cols, const uint8_t *dev_ops, size_t m,
                          uint64_t *n_new, uint64_t *n_over, uint64_t *n_del) {
    if (!s) return fail(RH_ERR_ARG, "NULL");
    int rc = check_cols(s->schema, dev_cols, m);
    if (rc) return rc;
    RH_LOCK(s);
    uint64_t c[3];
    if ((rc = s->apply_device(*dev_cols, dev_ops, m, c))) return rc;
    if (n_new) *n_new = c[0];
    if (n_over) *n_over = c[1];
    if (n_del) *n_del = c[2];
    return RH_OK;
}

}  // extern "C"
