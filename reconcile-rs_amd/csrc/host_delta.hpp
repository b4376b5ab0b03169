// host_delta.hpp -- the host tier's mirror of the store's delta run: an order-statistic B+ tree of
// signed deltas, so that a batch changes the host tier in O(batch * log n), never O(n).
//
// The device store keeps a base run and a delta run of DeltaRecs (store_kernels.hpp): for a key k
// the batches since the last compaction changed, contrib = cur_fp - base_fp (mod 2^256) and the
// count delta live - in_base in {-1, 0, +1}.  Every question then composes base and delta -- rank
// = rank_B + Σ count deltas below, aggregate = base prefix + Σ contribs below -- exactly the
// signed deltas FingerprintTreeMap composes into its cached subtree aggregates on insert and
// remove (rsos/src/fingerprint_tree_map/mutate.rs:31-41, :57, :93-154).  This tree holds the same
// entries on the host, in key order, with per-subtree sums of both, so the prefix of either at
// any key or position is one root-to-leaf walk: O(log n), the reference's own query cost
// (query.rs:25-121).  An entry is never (not in base, not live): deleting a key the base does not
// hold drops its entry, as the device merge does.
//
// No rebalancing on erase (the tree is rebuilt from scratch at every base refresh, and erasures --
// dropped insertions -- are rare); leaves may run underfull or empty, which every walk tolerates.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/rsos_hip.h"

namespace rh {

// 256-bit LE limbs, mod 2^256 (the Fingerprint group, rsos/src/fingerprint.rs:145-173)
inline void fp4_add(uint64_t *a, const uint64_t *b) {
    unsigned __int128 c = 0;
    for (int q = 0; q < 4; q++) {
        c += (unsigned __int128)a[q] + b[q];
        a[q] = (uint64_t)c;
        c >>= 64;
    }
}
inline void fp4_sub(uint64_t *a, const uint64_t *b) {
    unsigned char borrow = 0;
    for (int q = 0; q < 4; q++) {
        const uint64_t x = a[q], y = b[q];
        a[q] = x - y - borrow;
        borrow = (x < y) || (x == y && borrow);
    }
}

// The key type's Ord: u32 / u64 numerically (LE in memory), byte arrays by memcmp
struct KeyOrder {
    uint32_t kl = 0;
    int kk = RH_KEY_BYTES;
    // an order-preserving u64 of a key's leading bytes
    uint64_t digit(const uint8_t *k) const {
        if (kk == RH_KEY_U32) {
            uint32_t v;
            memcpy(&v, k, 4);
            return v;
        }
        uint64_t v;
        memcpy(&v, k, 8);
        return kk == RH_KEY_U64 ? v : __builtin_bswap64(v);
    }
    int cmp(const uint8_t *a, const uint8_t *b) const {
        const uint64_t x = digit(a), y = digit(b);
        if (x != y) return x < y ? -1 : 1;
        return kk == RH_KEY_BYTES && kl > 8 ? memcmp(a + 8, b + 8, kl - 8) : 0;
    }
};

class DeltaTree {
    struct Leaf;
    struct Node;

public:
    static constexpr int LF = 64;    // entries per leaf
    static constexpr int NF = 64;    // children per inner node
    static constexpr int KMAX = 32;  // longest key (the store's 32-byte arrays)
    static constexpr int FILL = 48;  // entries / children per node of a bulk build (3/4 full)

    struct Pos {              // a key's place among the entries
        uint64_t idx = 0;     // entries with key < z
        int64_t cnt = 0;      // Σ count deltas of those
        bool found = false;   // an entry with key == z exists ...
        int8_t fcnt = 0;      // ... with this count delta
        uint8_t flive = 0;    // ... and this live flag
    };
    struct Rec {              // one entry, as the fold hands it over
        const uint8_t *key;
        uint64_t fp[4];
        int8_t cnt;
        uint8_t live;
    };

    DeltaTree() = default;
    DeltaTree(const DeltaTree &) = delete;
    DeltaTree &operator=(const DeltaTree &) = delete;
    ~DeltaTree() { clear(); }

    void set_order(KeyOrder o) {
        clear();
        ko = o;
    }
    void clear() {
        free_sub(root, height);
        root = nullptr;
        height = 0;
        total_size = 0;
        total_cnt = 0;
        memset(total_fp, 0, sizeof total_fp);
        first_leaf = nullptr;
    }
    uint64_t size() const { return total_size; }
    int64_t cnt_total() const { return total_cnt; }
    const uint64_t *fp_total() const { return total_fp; }

    // entries with key < z, their count-delta sum, and z's own entry if any
    Pos lt(const uint8_t *z) const {
        Pos p;
        if (!root) return p;
        const void *cur = root;
        for (int h = height; h > 0; h--) {
            const Node *nd = static_cast<const Node *>(cur);
            const int c = route(nd, z);
            for (int i = 0; i < c; i++) p.idx += nd->size[i], p.cnt += nd->cnt[i];
            cur = nd->ch[c];
        }
        const Leaf *l = static_cast<const Leaf *>(cur);
        const int pos = leaf_lower(l, z);
        for (int i = 0; i < pos; i++) p.cnt += l->cnt[i];
        p.idx += pos;
        if (pos < l->n && ko.cmp(l->keys + pos * ko.kl, z) == 0) {
            p.found = true;
            p.fcnt = l->cnt[pos];
            p.flive = l->live[pos];
        }
        return p;
    }
    // Σ contribs of entries [0, idx)
    void fp_prefix(uint64_t idx, uint64_t out[4]) const {
        memset(out, 0, 32);
        if (!root) return;
        if (idx >= total_size) {
            memcpy(out, total_fp, 32);
            return;
        }
        const void *cur = root;
        for (int h = height; h > 0; h--) {
            const Node *nd = static_cast<const Node *>(cur);
            int c = 0;
            while (idx >= nd->size[c]) idx -= nd->size[c], fp4_add(out, nd->fp[c]), c++;
            cur = nd->ch[c];
        }
        const Leaf *l = static_cast<const Leaf *>(cur);
        for (uint64_t i = 0; i < idx; i++) fp4_add(out, l->fp[i]);
    }
    // entry idx (< size())
    const uint8_t *key_at(uint64_t idx, int8_t *cnt = nullptr, uint8_t *live = nullptr) const {
        const Leaf *l = leaf_at(&idx);
        if (cnt) *cnt = l->cnt[idx];
        if (live) *live = l->live[idx];
        return l->keys + idx * ko.kl;
    }
    // in-order walk from entry idx: while (it.l) { ... it.advance(); }
    struct Iter {
        const Leaf *l = nullptr;
        int i = 0;
        uint32_t kl = 0;
        const uint8_t *key() const { return l->keys + i * kl; }
        uint8_t live() const { return l->live[i]; }
        int8_t cnt() const { return l->cnt[i]; }
        void advance() {
            if (++i < l->n) return;
            i = 0;
            for (l = l->next; l && l->n == 0; l = l->next) {
            }
        }
    };
    Iter iter(uint64_t idx) const {
        Iter it;
        it.kl = ko.kl;
        if (idx >= total_size) return it;
        it.l = leaf_at(&idx);
        it.i = (int)idx;
        return it;
    }

    // insert or replace the entry of r.key
    void upsert(const Rec &r) {
        if (!root) {
            root = new_leaf();
            first_leaf = static_cast<Leaf *>(root);
        }
        if (height == 0 ? static_cast<Leaf *>(root)->n == LF : static_cast<Node *>(root)->n == NF) grow_root();
        Node *path[16];
        int pc[16], depth = 0;
        void *cur = root;
        for (int h = height; h > 0; h--) {
            Node *nd = static_cast<Node *>(cur);
            int c = route(nd, r.key);
            const bool full = h == 1 ? static_cast<Leaf *>(nd->ch[c])->n == LF : static_cast<Node *>(nd->ch[c])->n == NF;
            if (full) {
                split_child(nd, c, h == 1);
                c = route(nd, r.key);
            }
            path[depth] = nd, pc[depth] = c, depth++;
            cur = nd->ch[c];
        }
        Leaf *l = static_cast<Leaf *>(cur);
        const int pos = leaf_lower(l, r.key);
        uint64_t dfp[4];
        int64_t dcnt;
        int dsize;
        if (pos < l->n && ko.cmp(l->keys + pos * ko.kl, r.key) == 0) {  // replace: apply new - old
            memcpy(dfp, r.fp, 32);
            fp4_sub(dfp, l->fp[pos]);
            dcnt = (int64_t)r.cnt - l->cnt[pos];
            dsize = 0;
        } else {
            const int tail = l->n - pos;
            memmove(l->keys + (pos + 1) * ko.kl, l->keys + pos * ko.kl, (size_t)tail * ko.kl);
            memmove(l->fp[pos + 1], l->fp[pos], (size_t)tail * 32);
            memmove(l->cnt + pos + 1, l->cnt + pos, (size_t)tail);
            memmove(l->live + pos + 1, l->live + pos, (size_t)tail);
            memcpy(l->keys + pos * ko.kl, r.key, ko.kl);
            l->n++;
            memcpy(dfp, r.fp, 32);
            dcnt = r.cnt;
            dsize = 1;
        }
        memcpy(l->fp[pos], r.fp, 32);
        l->cnt[pos] = r.cnt;
        l->live[pos] = r.live;
        for (int i = 0; i < depth; i++) {
            Node *nd = path[i];
            nd->size[pc[i]] += dsize;
            nd->cnt[pc[i]] += dcnt;
            fp4_add(nd->fp[pc[i]], dfp);
        }
        total_size += dsize;
        total_cnt += dcnt;
        fp4_add(total_fp, dfp);
    }
    // remove key's entry if any
    void erase(const uint8_t *key) {
        if (!root) return;
        Node *path[16];
        int pc[16], depth = 0;
        void *cur = root;
        for (int h = height; h > 0; h--) {
            Node *nd = static_cast<Node *>(cur);
            const int c = route(nd, key);
            path[depth] = nd, pc[depth] = c, depth++;
            cur = nd->ch[c];
        }
        Leaf *l = static_cast<Leaf *>(cur);
        const int pos = leaf_lower(l, key);
        if (pos >= l->n || ko.cmp(l->keys + pos * ko.kl, key) != 0) return;
        uint64_t fp[4];
        memcpy(fp, l->fp[pos], 32);
        const int64_t cnt = l->cnt[pos];
        const int tail = l->n - pos - 1;
        memmove(l->keys + pos * ko.kl, l->keys + (pos + 1) * ko.kl, (size_t)tail * ko.kl);
        memmove(l->fp[pos], l->fp[pos + 1], (size_t)tail * 32);
        memmove(l->cnt + pos, l->cnt + pos + 1, (size_t)tail);
        memmove(l->live + pos, l->live + pos + 1, (size_t)tail);
        l->n--;
        for (int i = 0; i < depth; i++) {
            Node *nd = path[i];
            nd->size[pc[i]] -= 1;
            nd->cnt[pc[i]] -= cnt;
            fp4_sub(nd->fp[pc[i]], fp);
        }
        total_size -= 1;
        total_cnt -= cnt;
        fp4_sub(total_fp, fp);
    }

    // Apply m sorted, distinct keys' new states (drop[j]: remove key j's entry) in one pass over the
    // whole tree: what a large batch costs less as, O(size + m) sequential work instead of
    // O(m log size) walks.
    void merge_rebuild(const Rec *recs, const uint8_t *drop, size_t m) {
        std::vector<uint8_t> keys;
        std::vector<uint64_t> fps;
        std::vector<int8_t> cnts;
        std::vector<uint8_t> lives;
        const size_t cap = total_size + m;
        keys.reserve(cap * ko.kl);
        fps.reserve(cap * 4);
        cnts.reserve(cap);
        lives.reserve(cap);
        auto put = [&](const uint8_t *k, const uint64_t *fp, int8_t c, uint8_t lv) {
            keys.insert(keys.end(), k, k + ko.kl);
            fps.insert(fps.end(), fp, fp + 4);
            cnts.push_back(c);
            lives.push_back(lv);
        };
        Iter it = iter(0);
        size_t j = 0;
        while (it.l || j < m) {
            int c;
            if (!it.l) c = 1;
            else if (j >= m) c = -1;
            else c = ko.cmp(it.key(), recs[j].key);
            if (c < 0) {
                put(it.key(), it.l->fp[it.i], it.cnt(), it.live());
                it.advance();
            } else {
                if (!drop[j]) put(recs[j].key, recs[j].fp, recs[j].cnt, recs[j].live);
                if (c == 0) it.advance();
                j++;
            }
        }
        clear();
        build(keys.data(), fps.data(), cnts.data(), lives.data(), cnts.size());
    }

    // bulk load of n sorted, distinct entries
    void build(const uint8_t *keys, const uint64_t *fps, const int8_t *cnts, const uint8_t *lives, size_t n) {
        clear();
        if (n == 0) return;
        struct Sum {
            uint64_t size;
            int64_t cnt;
            uint64_t fp[4];
        };
        std::vector<void *> level;
        std::vector<Sum> sums;
        Leaf *prev = nullptr;
        for (size_t i = 0; i < n; i += FILL) {
            Leaf *l = new_leaf();
            const int k = (int)std::min<size_t>(FILL, n - i);
            memcpy(l->keys, keys + i * ko.kl, (size_t)k * ko.kl);
            memcpy(l->fp, fps + 4 * i, (size_t)k * 32);
            memcpy(l->cnt, cnts + i, (size_t)k);
            memcpy(l->live, lives + i, (size_t)k);
            l->n = k;
            Sum s{(uint64_t)k, 0, {0, 0, 0, 0}};
            for (int q = 0; q < k; q++) s.cnt += l->cnt[q], fp4_add(s.fp, l->fp[q]);
            if (prev) prev->next = l;
            else first_leaf = l;
            prev = l;
            level.push_back(l);
            sums.push_back(s);
            total_size += s.size;
            total_cnt += s.cnt;
            fp4_add(total_fp, s.fp);
        }
        int h = 0;
        while (level.size() > 1) {
            std::vector<void *> up;
            std::vector<Sum> upsums;
            for (size_t i = 0; i < level.size(); i += FILL) {
                Node *nd = new_node();
                const int k = (int)std::min<size_t>(FILL, level.size() - i);
                Sum s{0, 0, {0, 0, 0, 0}};
                for (int q = 0; q < k; q++) {
                    nd->ch[q] = level[i + q];
                    nd->size[q] = sums[i + q].size;
                    nd->cnt[q] = sums[i + q].cnt;
                    memcpy(nd->fp[q], sums[i + q].fp, 32);
                    memcpy(nd->sep + q * ko.kl, first_key(level[i + q], h), ko.kl);
                    s.size += nd->size[q], s.cnt += nd->cnt[q], fp4_add(s.fp, nd->fp[q]);
                }
                nd->n = k;
                up.push_back(nd);
                upsums.push_back(s);
            }
            level.swap(up);
            sums.swap(upsums);
            h++;
        }
        root = level[0];
        height = h;
    }

private:
    // Key storage is sized by the store's key length (LF * kl bytes after the fixed part), not by
    // the longest key: ~57 B per entry at the bulk fill for 8- and 16-byte keys.
    struct Leaf {
        int n = 0;
        Leaf *next = nullptr;
        uint64_t fp[LF][4];
        int8_t cnt[LF];
        uint8_t live[LF];
        uint8_t keys[];  // LF * kl bytes
    };
    struct Node {
        int n = 0;
        void *ch[NF];
        uint64_t size[NF];
        int64_t cnt[NF];
        uint64_t fp[NF][4];
        uint8_t sep[];  // NF * kl bytes: sep[c] <= every key of child c (c >= 1), > every key of child c - 1
    };
    Leaf *new_leaf() const { return new (::operator new(sizeof(Leaf) + (size_t)LF * ko.kl)) Leaf(); }
    Node *new_node() const { return new (::operator new(sizeof(Node) + (size_t)NF * ko.kl)) Node(); }
    static void del_leaf(Leaf *l) {
        l->~Leaf();
        ::operator delete(l);
    }
    static void del_node(Node *nd) {
        nd->~Node();
        ::operator delete(nd);
    }
    KeyOrder ko{};
    void *root = nullptr;
    int height = 0;  // inner levels above the leaves
    Leaf *first_leaf = nullptr;
    uint64_t total_size = 0;
    int64_t total_cnt = 0;
    uint64_t total_fp[4] = {0, 0, 0, 0};

    void free_sub(void *p, int h) {
        if (!p) return;
        if (h == 0) {
            del_leaf(static_cast<Leaf *>(p));
            return;
        }
        Node *nd = static_cast<Node *>(p);
        for (int i = 0; i < nd->n; i++) free_sub(nd->ch[i], h - 1);
        del_node(nd);
    }
    // child of nd that holds z: the number of separators sep[1..n) that are <= z
    int route(const Node *nd, const uint8_t *z) const {
        int lo = 1, hi = nd->n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (ko.cmp(nd->sep + mid * ko.kl, z) <= 0) lo = mid + 1;
            else hi = mid;
        }
        return lo - 1;
    }
    int leaf_lower(const Leaf *l, const uint8_t *z) const {
        int lo = 0, hi = l->n;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (ko.cmp(l->keys + mid * ko.kl, z) < 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    const Leaf *leaf_at(uint64_t *idx) const {
        const void *cur = root;
        for (int h = height; h > 0; h--) {
            const Node *nd = static_cast<const Node *>(cur);
            int c = 0;
            while (*idx >= nd->size[c]) *idx -= nd->size[c], c++;
            cur = nd->ch[c];
        }
        return static_cast<const Leaf *>(cur);
    }
    const uint8_t *first_key(const void *p, int h) const {
        if (h == 0) return static_cast<const Leaf *>(p)->keys;
        return static_cast<const Node *>(p)->sep;
    }
    void grow_root() {
        Node *r = new_node();
        r->n = 1;
        r->ch[0] = root;
        r->size[0] = total_size;
        r->cnt[0] = total_cnt;
        memcpy(r->fp[0], total_fp, 32);
        memcpy(r->sep, first_key(root, height), ko.kl);
        root = r;
        height++;
        split_child(r, 0, height == 1);
    }
    // split nd's full child c in halves; the upper half becomes child c + 1
    void split_child(Node *nd, int c, bool leaf) {
        uint64_t ysize = 0;
        int64_t ycnt = 0;
        uint64_t yfp[4] = {0, 0, 0, 0};
        void *y;
        const uint8_t *ysep;
        if (leaf) {
            Leaf *x = static_cast<Leaf *>(nd->ch[c]);
            Leaf *l = new_leaf();
            const int mid = x->n / 2, k = x->n - mid;
            memcpy(l->keys, x->keys + mid * ko.kl, (size_t)k * ko.kl);
            memcpy(l->fp, x->fp[mid], (size_t)k * 32);
            memcpy(l->cnt, x->cnt + mid, (size_t)k);
            memcpy(l->live, x->live + mid, (size_t)k);
            l->n = k;
            x->n = mid;
            l->next = x->next;
            x->next = l;
            for (int q = 0; q < k; q++) ycnt += l->cnt[q], fp4_add(yfp, l->fp[q]);
            ysize = (uint64_t)k;
            y = l;
            ysep = l->keys;
        } else {
            Node *x = static_cast<Node *>(nd->ch[c]);
            Node *r = new_node();
            const int mid = x->n / 2, k = x->n - mid;
            memcpy(r->ch, x->ch + mid, (size_t)k * sizeof(void *));
            memcpy(r->sep, x->sep + mid * ko.kl, (size_t)k * ko.kl);
            memcpy(r->size, x->size + mid, (size_t)k * 8);
            memcpy(r->cnt, x->cnt + mid, (size_t)k * 8);
            memcpy(r->fp, x->fp[mid], (size_t)k * 32);
            r->n = k;
            x->n = mid;
            for (int q = 0; q < k; q++) ysize += r->size[q], ycnt += r->cnt[q], fp4_add(yfp, r->fp[q]);
            y = r;
            ysep = r->sep;
        }
        const int tail = nd->n - c - 1;
        memmove(nd->ch + c + 2, nd->ch + c + 1, (size_t)tail * sizeof(void *));
        memmove(nd->sep + (c + 2) * ko.kl, nd->sep + (c + 1) * ko.kl, (size_t)tail * ko.kl);
        memmove(nd->size + c + 2, nd->size + c + 1, (size_t)tail * 8);
        memmove(nd->cnt + c + 2, nd->cnt + c + 1, (size_t)tail * 8);
        memmove(nd->fp[c + 2], nd->fp[c + 1], (size_t)tail * 32);
        nd->ch[c + 1] = y;
        memcpy(nd->sep + (c + 1) * ko.kl, ysep, ko.kl);
        nd->size[c + 1] = ysize;
        nd->cnt[c + 1] = ycnt;
        memcpy(nd->fp[c + 1], yfp, 32);
        nd->size[c] -= ysize;
        nd->cnt[c] -= ycnt;
        fp4_sub(nd->fp[c], yfp);
        nd->n++;
    }
};

}  // namespace rh
