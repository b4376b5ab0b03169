// wire_codec.cpp -- RangeAggregate<K> on the wire: the bytes rbsr's protocol round exchanges.
//
// RangeAggregate { range: KeyRange(StartBound, EndBound), aggregate: Aggregate }
// (rbsr/src/protocol.rs:47-88) serialised by the gossip codec, bincode 1.3.3 DefaultOptions
// (gossip/src/bincode.rs:65-70): varint integers, little-endian, no struct framing.  The varint
// (bincode's VarintEncoding) is: v < 251 -> one byte; else a marker 251 / 252 / 253 followed by
// v as u16 / u32 / u64 LE (254 = u128, which no field here uses).  u8 is a raw byte, so
// Fingerprint's [u8; 32] (rsos/src/fingerprint.rs:74-83) is 32 raw bytes.  Pinned by the
// golden vector of tests/wire_format.rs:37-62 (tests/test_wire.py).
#include <cstdint>
#include <cstring>
#include <string>

#include "../../include/rsos_hip.h"

namespace rh {
int set_error(int code, const std::string &msg);  // rsos_hip_abi.hip
}

namespace {

struct Writer {
    uint8_t *out;
    size_t cap, pos = 0;
    void byte(uint8_t b) {
        if (out && pos < cap) out[pos] = b;
        pos++;
    }
    void le(uint64_t v, int n) {
        for (int i = 0; i < n; i++) byte((uint8_t)(v >> (8 * i)));
    }
    void varint(uint64_t v) {
        if (v < 251) byte((uint8_t)v);
        else if (v <= 0xffff) { byte(251); le(v, 2); }
        else if (v <= 0xffffffffull) { byte(252); le(v, 4); }
        else { byte(253); le(v, 8); }
    }
    void raw(const uint8_t *p, size_t n) {
        for (size_t i = 0; i < n; i++) byte(p[i]);
    }
};

enum Rd { RD_OK = 0, RD_EOF = 1, RD_BAD = 2 };

struct Reader {
    const uint8_t *in;
    size_t len, pos = 0;
    std::string why;
    Rd le(uint64_t *v, int n) {
        if (len - pos < (size_t)n) return RD_EOF;
        uint64_t x = 0;
        for (int i = 0; i < n; i++) x |= (uint64_t)in[pos + i] << (8 * i);
        pos += n;
        *v = x;
        return RD_OK;
    }
    Rd varint(uint64_t *v, uint64_t max, const char *what) {
        uint64_t m;
        Rd r = le(&m, 1);
        if (r) return r;
        if (m < 251) *v = m;
        else if (m == 251) { if ((r = le(v, 2))) return r; }
        else if (m == 252) { if ((r = le(v, 4))) return r; }
        else if (m == 253) { if ((r = le(v, 8))) return r; }
        else {
            why = std::string(what) + ": invalid varint marker " + std::to_string(m) + " (u128 range)";
            return RD_BAD;
        }
        if (*v > max) {
            why = std::string(what) + ": varint " + std::to_string(*v) + " out of range";
            return RD_BAD;
        }
        return RD_OK;
    }
    Rd raw(uint8_t *dst, size_t n) {
        if (len - pos < n) return RD_EOF;
        memcpy(dst, in + pos, n);
        pos += n;
        return RD_OK;
    }
};

struct KeyCodec {
    int kind, form;
    size_t kl;
    void put(Writer &w, const uint8_t *k) const {
        if (kind == RH_KEY_U32) { uint32_t v; memcpy(&v, k, 4); w.varint(v); }
        else if (kind == RH_KEY_U64) { uint64_t v; memcpy(&v, k, 8); w.varint(v); }
        else {
            if (form == RH_FORM_VEC) w.varint(kl);
            w.raw(k, kl);
        }
    }
    Rd get(Reader &r, uint8_t *k) const {
        uint64_t v;
        Rd s;
        if (kind == RH_KEY_U32) {
            if ((s = r.varint(&v, 0xffffffffull, "u32 key"))) return s;
            uint32_t x = (uint32_t)v;
            memcpy(k, &x, 4);
            return RD_OK;
        }
        if (kind == RH_KEY_U64) {
            if ((s = r.varint(&v, ~0ull, "u64 key"))) return s;
            memcpy(k, &v, 8);
            return RD_OK;
        }
        if (form == RH_FORM_VEC) {
            if ((s = r.varint(&v, ~0ull, "key length"))) return s;
            if (v != kl) {
                r.why = "key length " + std::to_string(v) + " != schema key_len " + std::to_string(kl);
                return RD_BAD;
            }
        }
        return r.raw(k, kl);
    }
};

int key_codec(const rh_schema *s, int form, KeyCodec *kc) {
    if (!s) return rh::set_error(RH_ERR_ARG, "schema is NULL");
    if (form != RH_FORM_ARRAY && form != RH_FORM_VEC) return rh::set_error(RH_ERR_ARG, "bad key_form");
    if (s->key_kind == RH_KEY_U32 && s->key_len == 4 && form == RH_FORM_ARRAY) *kc = {RH_KEY_U32, form, 4};
    else if (s->key_kind == RH_KEY_U64 && s->key_len == 8 && form == RH_FORM_ARRAY) *kc = {RH_KEY_U64, form, 8};
    else if (s->key_kind == RH_KEY_BYTES && s->key_len > 0) *kc = {RH_KEY_BYTES, form, s->key_len};
    else return rh::set_error(RH_ERR_ARG, "wire keys must be u32, u64 or byte strings (RH_FORM_VEC only for bytes)");
    return RH_OK;
}

}  // namespace

extern "C" {

int rh_wire_encode_range_aggregates(const rh_schema *schema, int key_form, int msg_tag, const uint8_t *start_kinds,
                                    const void *start_keys, const uint8_t *end_kinds, const void *end_keys,
                                    const rh_aggregate *aggs, size_t r, uint8_t *out, size_t cap, size_t *out_len) {
    KeyCodec kc;
    int rc = key_codec(schema, key_form, &kc);
    if (rc) return rc;
    if (!out_len) return rh::set_error(RH_ERR_ARG, "out_len is NULL");
    if (r && (!start_kinds || !end_kinds || !aggs)) return rh::set_error(RH_ERR_ARG, "NULL input");
    if (msg_tag < -1) return rh::set_error(RH_ERR_ARG, "bad msg_tag");
    const uint8_t *sk = static_cast<const uint8_t *>(start_keys), *ek = static_cast<const uint8_t *>(end_keys);
    Writer w{out, cap};
    for (size_t i = 0; i < r; i++) {
        if (start_kinds[i] > 1 || end_kinds[i] > 1)
            return rh::set_error(RH_ERR_ARG, "bound kinds are 0 (Unbounded) or 1 (start Included / end Excluded)");
        if ((start_kinds[i] && !sk) || (end_kinds[i] && !ek)) return rh::set_error(RH_ERR_ARG, "bound keys are NULL");
        if (msg_tag >= 0) w.varint((uint64_t)msg_tag);
        w.varint(start_kinds[i]);
        if (start_kinds[i]) kc.put(w, sk + i * kc.kl);
        w.varint(end_kinds[i]);
        if (end_kinds[i]) kc.put(w, ek + i * kc.kl);
        for (int l = 0; l < 4; l++) w.le(aggs[i].fingerprint[l], 8);
        w.varint(aggs[i].size);
    }
    *out_len = w.pos;
    if (out && w.pos > cap)
        return rh::set_error(RH_ERR_ARG, "output buffer too small: need " + std::to_string(w.pos) + " bytes");
    return RH_OK;
}

int rh_wire_decode_range_aggregates(const rh_schema *schema, int key_form, int msg_tag, const uint8_t *in, size_t len,
                                    size_t r_cap, uint8_t *start_kinds, void *start_keys, uint8_t *end_kinds,
                                    void *end_keys, rh_aggregate *aggs, size_t *r_out, size_t *consumed) {
    KeyCodec kc;
    int rc = key_codec(schema, key_form, &kc);
    if (rc) return rc;
    if (!r_out || !consumed) return rh::set_error(RH_ERR_ARG, "r_out / consumed is NULL");
    if (len && !in) return rh::set_error(RH_ERR_ARG, "input is NULL");
    if (r_cap && (!start_kinds || !start_keys || !end_kinds || !end_keys || !aggs))
        return rh::set_error(RH_ERR_ARG, "NULL output");
    if (msg_tag < -1) return rh::set_error(RH_ERR_ARG, "bad msg_tag");
    uint8_t *sk = static_cast<uint8_t *>(start_keys), *ek = static_cast<uint8_t *>(end_keys);
    Reader rd{in, len};
    size_t n = 0, done = 0;
    Rd st = RD_OK;
    while (n < r_cap) {
        uint64_t v;
        // one item; an end of input anywhere in it is a clean end of the stream
        // (gossip/src/bincode.rs:86-95), so the partial item is dropped
        if (msg_tag >= 0) {
            if ((st = rd.varint(&v, 0xffffffffull, "message tag"))) break;
            if (v != (uint64_t)msg_tag) {
                rd.why = "message tag " + std::to_string(v) + " is not " + std::to_string(msg_tag);
                st = RD_BAD;
                break;
            }
        }
        if ((st = rd.varint(&v, 0xffffffffull, "start bound tag"))) break;
        if (v > 1) {
            rd.why = "invalid start bound variant " + std::to_string(v) + " (expected 0 <= i < 2)";
            st = RD_BAD;
            break;
        }
        start_kinds[n] = (uint8_t)v;
        memset(sk + n * kc.kl, 0, kc.kl);
        if (v && (st = kc.get(rd, sk + n * kc.kl))) break;
        if ((st = rd.varint(&v, 0xffffffffull, "end bound tag"))) break;
        if (v > 1) {
            rd.why = "invalid end bound variant " + std::to_string(v) + " (expected 0 <= i < 2)";
            st = RD_BAD;
            break;
        }
        end_kinds[n] = (uint8_t)v;
        memset(ek + n * kc.kl, 0, kc.kl);
        if (v && (st = kc.get(rd, ek + n * kc.kl))) break;
        uint64_t limb[4];
        for (int l = 0; l < 4 && !st; l++) st = rd.le(&limb[l], 8);
        if (st) break;
        if ((st = rd.varint(&v, ~0ull, "aggregate size"))) break;
        memcpy(aggs[n].fingerprint, limb, 32);
        aggs[n].size = v;
        n++;
        done = rd.pos;
    }
    *r_out = n;
    *consumed = done;
    if (st == RD_BAD) return rh::set_error(RH_ERR_DATA, "RangeAggregate item " + std::to_string(n) + ": " + rd.why);
    return RH_OK;
}

}  // extern "C"
